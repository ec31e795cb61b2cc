"""Summarise a rocprofv3 --kernel-trace database (rocpd sqlite) into a per-kernel stats table.
usage: python tools/prof_summary.py <results.db> [out.txt]"""
import sqlite3
import sys


def summary(db, by_grid=False):
    c = sqlite3.connect(db)
    grp = "name, grid_x" if by_grid else "name"
    rows = c.execute("select name, count(*), avg(duration), min(duration), max(duration), sum(duration), "
                     "max(vgpr_count), max(accum_vgpr_count), max(lds_size), max(grid_x), max(workgroup_x) "
                     f"from kernels group by {grp} order by sum(duration) desc").fetchall()
    tot = sum(r[5] for r in rows) or 1
    out = [f"{'kernel':<70} {'calls':>6} {'avg_us':>10} {'min_us':>10} {'max_us':>10} {'total_ms':>10} {'pct':>6}  vgpr agpr lds grid wg"]
    for r in rows:
        name = r[0].replace("(anonymous namespace)::", "")
        name = name[:70]
        out.append(f"{name:<70} {r[1]:>6} {r[2]/1e3:>10.2f} {r[3]/1e3:>10.2f} {r[4]/1e3:>10.2f} {r[5]/1e6:>10.3f} "
                   f"{100*r[5]/tot:>5.1f}%  {r[6]} {r[7]} {r[8]} {r[9]} {r[10]}")
    return "\n".join(out)


if __name__ == "__main__":
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    s = summary(args[0], by_grid="--by-grid" in sys.argv)
    print(s)
    if len(args) > 1:
        open(args[1], "w").write(s + "\n")
