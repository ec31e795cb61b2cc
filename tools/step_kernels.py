"""Per-kernel time inside one steady-state bench step of a rocprofv3 kernel trace: the step is the
interval between two consecutive launches of a marker kernel (default bert_embed; the n-th and
n+1-th).  usage: step_kernels.py <kernel_trace.csv> [n] [marker]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
marker = sys.argv[3] if len(sys.argv) > 3 else "bert_embed"
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
marks = [int(r["Start_Timestamp"]) for r in rows if marker in r["Kernel_Name"]]
t0, t1 = marks[n], marks[n + 1]
agg = collections.defaultdict(lambda: [0, 0.0])
busy = 0.0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if s >= t0 and s < t1:
        k = r["Kernel_Name"][:100]
        agg[k][0] += 1
        agg[k][1] += (e - s) / 1e3
        busy += (e - s) / 1e3
print(f"step {n}: wall {(t1 - t0) / 1e6:.2f} ms, kernel sum {busy / 1e3:.2f} ms")
for k, (c, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{us / 1e3:8.3f} ms {c:4d}x {us / c:8.1f} us  {k}")
