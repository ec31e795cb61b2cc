"""Launch-by-launch list of one steady-state bench step of a rocprofv3 kernel trace (the step = the
interval between the n-th and n+1-th launches of a marker kernel): start offset, gap before, duration,
grid size, name; optional substring filter.  usage: step_list.py <kernel_trace.csv> [n] [filter]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
flt = sys.argv[3] if len(sys.argv) > 3 else ""
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [int(r["Start_Timestamp"]) for r in rows if "bert_embed" in r["Kernel_Name"]]
t0, t1 = marks[n], marks[n + 1]
prev = None
gk = [k for k in rows[0] if k.startswith("Grid_Size")] or [k for k in rows[0] if "Grid" in k]
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if not (t0 <= s < t1):
        continue
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    prev = e
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    if flt and flt not in name:
        continue
    grid = "x".join(r[k] for k in gk)
    print(f"{(s - t0) / 1e3:9.1f} us  gap {gap:7.1f}  dur {(e - s) / 1e3:7.1f}  grid {grid:>14s}  {name[:80]}")
