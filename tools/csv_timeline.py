"""Per-launch timeline (start gap, duration) of the last N kernels of a rocprofv3 kernel_trace.csv.
usage: python tools/csv_timeline.py <kernel_trace.csv> [N]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)[-n:]
prev = None
for s, e, name in ev:
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"gap {gap:8.2f} us  dur {(e - s) / 1e3:8.2f} us  {name.replace('(anonymous namespace)::', '')[:100]}")
    prev = e
