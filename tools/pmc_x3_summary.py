"""Label the dispatches of tools/pmc_x3.py runs (PLAN order: one warm-up dispatch per op, then REPS each) and
summarise per label: kernel time (the --kernel-trace pass), HBM bytes (FETCH_SIZE x2 gfx950 correction +
WRITE_SIZE, MI355X_MICROARCH.md HBM section), MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs /
(GRBM_GUI_ACTIVE / 8), the clock GRBM_GUI_ACTIVE / 8 / duration, and the wave-cycle buckets (SQ_WAIT_ANY =
parked on s_waitcnt / barrier, SQ_WAIT_INST_ANY = issue stalls) as fractions of SQ_WAVE_CYCLES.
usage: python tools/pmc_x3_summary.py <out.json> <tag> <kernel_trace.csv> <counter_collection.csv>..."""
import collections
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_x3 import PLAN, REPS  # noqa: E402


def label(rows_by_id):
    """{dispatch id: kernel name} -> {dispatch id: label} following PLAN (warm-up pass, then REPS)."""
    ids = sorted(rows_by_id)
    seq = [(n, s, 1) for n, s, _, _ in PLAN] + [(n, s, REPS) for n, s, _, _ in PLAN]
    out, pos = {}, 0
    for i, (name, sub, cnt) in enumerate(seq):
        got = 0
        while got < cnt:
            if pos >= len(ids):
                raise SystemExit(f"ran out of dispatches at {name}")
            d = ids[pos]
            pos += 1
            if sub in rows_by_id[d]:
                if i >= len(PLAN):
                    out[d] = name
                got += 1
    return out


def main():
    out, tag, trace = sys.argv[1], sys.argv[2], sys.argv[3]
    tr = {int(r["Dispatch_Id"]): r for r in csv.DictReader(open(trace))}
    lab = label({d: r["Kernel_Name"] for d, r in tr.items()})
    dur = collections.defaultdict(list)
    for d, name in lab.items():
        dur[name].append((int(tr[d]["End_Timestamp"]) - int(tr[d]["Start_Timestamp"])) / 1e3)
    cnt = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in sys.argv[4:]:
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        names = {}
        for r in csv.DictReader(open(path)):
            d = int(r["Dispatch_Id"])
            per[d][r["Counter_Name"]] += float(r["Counter_Value"])
            names[d] = r["Kernel_Name"]
        lp = label(names)
        for d, name in lp.items():
            for k, v in per[d].items():
                cnt[name][k].append(v)
    res = {}
    for name, sub, _, (kind, work) in PLAN:
        c = {k: sum(v) / len(v) for k, v in cnt[name].items()}
        t = sum(dur[name]) / len(dur[name])
        e = {"kernel": sub, "dispatches": len(dur[name]), "duration_us": round(t, 2)}
        if kind == "mfma":
            e["bf16_mfma_tflop"] = work / 1e12
            e["achieved_pflops"] = round(work / t / 1e9, 4)
            e["frac_of_2p5pf"] = round(work / t / 1e9 / 2.5, 4)
        else:
            e["algorithmic_bytes"] = work
            e["achieved_tbps"] = round(work / t / 1e6, 3)
        if "FETCH_SIZE" in c:
            e["fetch_bytes"] = 2.0 * c["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in c:
            e["write_bytes"] = c["WRITE_SIZE"] * 1024
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            e["hbm_bytes"] = e["fetch_bytes"] + e["write_bytes"]
            e["hbm_tbps"] = round(e["hbm_bytes"] / t / 1e6, 3)
        if "GRBM_GUI_ACTIVE" in c:
            clk = c["GRBM_GUI_ACTIVE"] / 8
            e["clock_ghz"] = round(clk / t / 1e3, 3)
            if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                e["mfma_busy"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / clk, 4)
        if "SQ_WAVE_CYCLES" in c:
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS"):
                if k in c:
                    e[k.lower() + "_frac"] = round(c[k] / c["SQ_WAVE_CYCLES"], 4)
        e["counters"] = {k: v for k, v in sorted(c.items())}
        res[name] = e
        print(f"{name:14s} {t:8.1f} us  " + "  ".join(f"{k}={v}" for k, v in e.items()
                                                    if k not in ("counters", "kernel")), flush=True)
    json.dump({"source": f"{tag}: tools/pmc_x3.py under rocprofv3 (--kernel-trace pass + one --pmc pass per "
                         "counter group), tools/pmc_x3_summary.py", "kernels": res}, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
