"""Per-kernel effective clock from a rocprofv3 --pmc GRBM_GUI_ACTIVE counter_collection.csv:
GRBM_GUI_ACTIVE (summed over the 8 XCDs) / 8 / (end - start).  usage: clock_summary.py <csv>"""
import csv
import collections
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    if r.get("Counter_Name") != "GRBM_GUI_ACTIVE":
        continue
    dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    name = r["Kernel_Name"][:90]
    agg[(name, r.get("Grid_Size", ""))].append((float(r["Counter_Value"]) / 8 / dur / 1e9, dur * 1e6))
for (name, g), v in agg.items():
    v = v[1:] if len(v) > 2 else v
    print(f"{name:90s} n={len(v):2d} clock {sum(c for c, _ in v) / len(v):.3f} GHz  dur {sum(d for _, d in v) / len(v):8.1f} us")
