"""Summarise rocprofv3 --kernel-trace --stats csv output (<prefix>_kernel_stats.csv) into a per-kernel
table: calls, avg/min/max us, total ms, share.
usage: python tools/prof_csv_summary.py <kernel_stats.csv> [out.txt]"""
import csv
import sys


def summary(path, width=88):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows) or 1.0
    out = [f"{'kernel':<{width}} {'calls':>6} {'avg_us':>9} {'min_us':>9} {'max_us':>9} {'total_ms':>9} {'pct':>6}"]
    for r in rows:
        name = r["Name"].replace("(anonymous namespace)::", "").replace("unsigned short", "u16")[:width]
        out.append(f"{name:<{width}} {int(r['Calls']):>6} {float(r['AverageNs']) / 1e3:>9.2f} "
                   f"{float(r['MinNs']) / 1e3:>9.2f} {float(r['MaxNs']) / 1e3:>9.2f} "
                   f"{float(r['TotalDurationNs']) / 1e6:>9.3f} {100 * float(r['TotalDurationNs']) / tot:>5.1f}%")
    return "\n".join(out)


if __name__ == "__main__":
    s = summary(sys.argv[1])
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(s + "\n")
    print(s)
