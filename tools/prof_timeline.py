"""Per-launch timeline (start gap, duration) of the last N kernels in a rocprofv3 --kernel-trace db.
usage: python tools/prof_timeline.py <results.db> [N]"""
import sqlite3
import sys

c = sqlite3.connect(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = c.execute("select name, start, end from kernels order by start").fetchall()[-n:]
prev = None
for name, s, e in rows:
    gap = (s - prev) / 1e3 if prev is not None else 0.0
    print(f"gap {gap:8.2f} us  dur {(e - s) / 1e3:8.2f} us  {name.replace('(anonymous namespace)::', '')[:90]}")
    prev = e
