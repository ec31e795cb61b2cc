"""Per-kernel LDS bank-conflict share from a rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
SQ_INSTS_LDS csv: cycles lost to conflicts / LDS-active cycles, per kernel (summed over dispatches),
sorted by conflict cycles.  usage: python tools/pmc_lds_conflicts.py <counter_collection.csv>"""
import collections
import csv
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Kernel_Name"][:90]][r["Counter_Name"]] += float(r["Counter_Value"])
rows = sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_LDS_BANK_CONFLICT", 0))
print(f"{'kernel':90s} {'conflict cyc':>14s} {'LDS active':>14s} {'share':>7s} {'LDS insts':>12s}")
for k, v in rows[:30]:
    c, a = v.get("SQ_LDS_BANK_CONFLICT", 0), v.get("SQ_ACTIVE_INST_LDS", 0)
    print(f"{k:90s} {c:14.4g} {a:14.4g} {c / a if a else 0:7.3f} {v.get('SQ_INSTS_LDS', 0):12.4g}")
