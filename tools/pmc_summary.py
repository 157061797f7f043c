"""Summarise rocprofv3 output for one kernel: average duration from a kernel-trace stats CSV
and per-dispatch PMC counters (FETCH_SIZE / WRITE_SIZE / TCC hit rate) from counter passes.

FETCH_SIZE is doubled for wide reads per MI355X_MICROARCH.md (HBM section): on gfx950 it
reports half the bytes of 16-B/lane reads.  Both raw and corrected values are printed.

    python tools/pmc_summary.py --kernel match_fast_kernel --dir gpurun_out/<tag>
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def rows(pattern):
    for p in sorted(glob.glob(pattern, recursive=True)):
        with open(p, newline="") as f:
            yield from csv.DictReader(f)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--kernel", default="match_fast_kernel")
    ap.add_argument("--skip", type=int, default=1, help="drop the first N dispatches (warmup)")
    args = ap.parse_args()
    out = {"kernel": args.kernel}
    for r in rows(os.path.join(args.dir, "**", "*kernel_stats.csv")):
        if args.kernel in r["Name"]:
            out["avg_ns"] = float(r["AverageNs"])
            out["calls"] = int(r["Calls"])
    # Launches that do no work (a call the engine reruns: e.g. the walk order's buffer-growth
    # rerun, whose first fast kernel exits at once) would dilute the averages: per-launch
    # numbers keep launches above 1 % of the median duration / counter total.
    durs = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            for r in rows(os.path.join(args.dir, "**", "*kernel_trace.csv")) if args.kernel in r["Kernel_Name"]]
    if durs:
        med = sorted(durs)[len(durs) // 2]
        full = [d for d in durs if d >= 0.01 * med]
        out["avg_ns"] = sum(full) / len(full)
        out["calls"] = len(full)
        out["calls_dropped_empty"] = len(durs) - len(full)
    per = defaultdict(lambda: defaultdict(float))  # (pass, dispatch) -> counter -> value
    for p in sorted(glob.glob(os.path.join(args.dir, "**", "*counter_collection.csv"), recursive=True)):
        with open(p, newline="") as f:
            for r in csv.DictReader(f):
                if args.kernel not in r.get("Kernel_Name", ""):
                    continue
                per[(p, int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    acc = defaultdict(list)
    by_pass = defaultdict(list)
    for (p, d), cs in sorted(per.items()):
        by_pass[p].append(cs)
    for p, lst in by_pass.items():
        tot = sorted(sum(cs.values()) for cs in lst)
        med = tot[len(tot) // 2] if tot else 0
        lst = [cs for cs in lst if sum(cs.values()) >= 0.01 * med]
        for cs in lst[args.skip:] or lst:
            for k, v in cs.items():
                acc[k].append(v)
    avg = {k: sum(v) / len(v) for k, v in acc.items()}
    out["counters_avg_per_dispatch"] = avg
    if "FETCH_SIZE" in avg:  # KiB in rocprofv3's derived metric
        out["fetch_bytes_raw"] = avg["FETCH_SIZE"] * 1024
        out["fetch_bytes_corrected_x2"] = 2 * avg["FETCH_SIZE"] * 1024
    if "WRITE_SIZE" in avg:
        out["write_bytes"] = avg["WRITE_SIZE"] * 1024
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        t = avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"]
        out["l2_hit_rate"] = avg["TCC_HIT_sum"] / t if t else None
    if "fetch_bytes_corrected_x2" in out and "write_bytes" in out:
        out["traffic_bytes"] = out["fetch_bytes_corrected_x2"] + out["write_bytes"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
