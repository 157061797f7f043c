"""Write profiles/pmc_match_fast.json (the `traffic` bench.py reports) from one
tools/gpu_round.sh output directory: the match kernel's PMC passes plus the FETCH_SIZE
calibration on tools/gather_bench.hip's random 16-B gathers.

Calibration (MI355X_MICROARCH.md: "other access widths are uncalibrated: calibrate on a known
byte count in your own access pattern"): on a 1 GiB table every random 16-B read misses L2
once, and FETCH_SIZE / TCC_MISS comes out at 64 B — one 64-B request per miss, the same
request shape (TCC_EA0_RDREQ ~= TCC_MISS, no 32-B requests) the match kernel shows.  So for
this kernel HBM read bytes = FETCH_SIZE as reported (not x2, the streaming-read rule).

    python tools/update_traffic.py gpurun_out/<tag> [--workload D --cal-dir gpurun_out/<B tag>]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def calibration(d):
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "cal", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    big = [c for c in per.values() if c.get("TCC_MISS_sum", 0) > 1e7]  # the 1 GiB table
    if not big:
        return None
    ratio = sum(1024.0 * c["FETCH_SIZE"] / c["TCC_MISS_sum"] for c in big) / len(big)
    return {"fetch_bytes_per_l2_miss": round(ratio, 2), "dispatches": len(big),
            "pattern": "tools/gather_bench.hip indep_kernel: random 16-B reads of a 1 GiB table"}


WORKLOADS = {
    "B": ("B: 10M filters, 1M-topic batch (bench.py defaults)", "pmc_match_fast.json"),
    "D": ("D: 1M adversarial filters, 1M-topic batch (bench.py --workload D)", "pmc_match_fast_D.json"),
    "C1": ("C1: config C's 100M-filter table on one GPU, 1M-topic batch (bench.py --n-filters 100000000 "
           "--vocab-scale 4)", "pmc_match_fast_C1.json"),
}


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("dir", help="gpurun_out/<tag> holding pmc_summary.json")
    ap.add_argument("--workload", default="B", choices=sorted(WORKLOADS))
    ap.add_argument("--cal-dir", default=None, help="directory holding the calibration run (default: dir)")
    ap.add_argument("--copied-to", default=None, help="where pmc_summary.json is kept under profiles/")
    args = ap.parse_args()
    d = args.dir
    s = json.load(open(os.path.join(d, "pmc_summary.json")))
    c = s["counters_avg_per_dispatch"]
    cal = calibration(args.cal_dir or d)
    per_miss = cal["fetch_bytes_per_l2_miss"] if cal else None
    fetch = s["fetch_bytes_raw"]
    name, fname = WORKLOADS[args.workload]
    src = os.path.relpath(os.path.join(d, "pmc_summary.json"), ROOT) + " (rocprofv3 --pmc passes)"
    if args.copied_to:
        src += "; copied to " + args.copied_to
    out = {
        "kernel": s["kernel"],
        "workload": name,
        "batch_topics": 1000000,
        "fetch_bytes_raw_per_launch": fetch,
        "write_bytes_per_launch": s["write_bytes"],
        "traffic_bytes_per_launch": fetch + s["write_bytes"],
        "traffic_rule": "FETCH_SIZE + WRITE_SIZE; FETCH_SIZE calibrated on random 16-B gathers "
                        "(%s B per L2 miss, one 64-B request per miss; not the x2 streaming rule)" % per_miss,
        "calibration": cal,
        "l2_hit_rate": s["l2_hit_rate"],
        "l2_misses_per_launch": c["TCC_MISS_sum"],
        "l2_requests_per_launch": c["TCC_HIT_sum"] + c["TCC_MISS_sum"],
        "avg_kernel_ns": s.get("avg_ns"),
        "source": src,
    }
    with open(os.path.join(ROOT, "profiles", fname), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
