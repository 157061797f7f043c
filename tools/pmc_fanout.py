"""Write profiles/pmc_fanout_E.json (the fan-out call's `traffic` in bench.py --workload E) from
rocprofv3 --pmc passes over the fan-out kernels.  Per kernel: counters summed over its
dispatches, divided by the number of fan-out calls (one fanout_write_kernel dispatch per call).
FETCH_SIZE is doubled: calibrated with tools/gather_bench.hip `cal` (a 1 GiB buffer read once
with 4-B lanes and once with 16-B lanes reports 0.5 GiB either way, profiles/r3_fetch_calibration.txt;
MI355X_MICROARCH.md's HBM section states it for 16-B lanes); WRITE_SIZE as reported (1 GiB
written with 4-B lanes reports 1.0 GiB).

    python tools/pmc_fanout.py gpurun_out/<tag> --strategy hash_clientid
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def read_passes(d):
    per = defaultdict(lambda: defaultdict(float))   # kernel -> counter -> sum
    calls = defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].split("<")[0]
            k = k.replace("emqx::", "")
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            calls[(k, os.path.dirname(f))].add(int(r["Dispatch_Id"]))
    n_calls = defaultdict(int)
    for (k, dd), ids in calls.items():
        n_calls[(k, dd)] = len(ids)
    return per, calls


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--strategy", default="hash_clientid")
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--fetch-scale", type=float, default=2.0)
    args = ap.parse_args()
    out_k = {}
    counters = defaultdict(dict)
    for pd in sorted(glob.glob(os.path.join(args.dir, "pmc*"))):
        if not os.path.isdir(pd):
            continue
        per, calls = read_passes(pd)
        writes = [len(v) for (k, _), v in calls.items() if k.endswith("fanout_write_kernel")]
        nc = max(sum(writes), 1)
        for k, cs in per.items():
            for c, v in cs.items():
                counters[k][c] = v / nc
    total_fetch = sum(cs.get("FETCH_SIZE", 0.0) for cs in counters.values()) * 1024 * args.fetch_scale
    total_write = sum(cs.get("WRITE_SIZE", 0.0) for cs in counters.values()) * 1024
    for k, cs in counters.items():
        out_k[k] = {"fetch_bytes": round(cs.get("FETCH_SIZE", 0.0) * 1024 * args.fetch_scale),
                    "write_bytes": round(cs.get("WRITE_SIZE", 0.0) * 1024),
                    **{c: round(v, 1) for c, v in cs.items() if c not in ("FETCH_SIZE", "WRITE_SIZE")}}
    res = {"workload": "E: match + fan-out, 10M subscriptions, 1M-topic batch (bench.py --workload E)",
           "strategy": args.strategy, "batch_topics": args.batch,
           "traffic_bytes_per_call": round(total_fetch + total_write),
           "traffic_rule": "FETCH_SIZE x %.0f (streaming 4-B / 16-B reads, calibrated: "
                           "profiles/r3_fetch_calibration.txt) + WRITE_SIZE, summed over the fan-out kernels per "
                           "call; the random 16-B record reads count 64 B per miss at x1 (round 1's calibration), so "
                           "doubling them bounds the traffic from above" % args.fetch_scale,
           "per_kernel_bytes": out_k,
           "source": os.path.relpath(args.dir, ROOT) + " (rocprofv3 --pmc passes)"}
    with open(os.path.join(ROOT, "profiles", "pmc_fanout_E.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
