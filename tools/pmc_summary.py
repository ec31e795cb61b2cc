"""Sum rocprofv3 --pmc counters (csv output) per kernel-name substring, averaged over dispatches.
usage: python tools/pmc_summary.py <counter_collection.csv> <kernel substring>"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
sub = sys.argv[2]
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
for r in rows:
    if sub in r["Kernel_Name"]:
        agg[r["Counter_Name"]] += float(r["Counter_Value"])
        disp[r["Counter_Name"]].add(r["Dispatch_Id"])
for k in sorted(agg):
    print(f"{k:32s} {agg[k] / len(disp[k]):14.4g}   ({len(disp[k])} dispatches)")
