"""HBM traffic of one retained-lookup call (config R) from rocprofv3 --pmc passes: FETCH_SIZE
and WRITE_SIZE summed over every retain_* dispatch (walk, spill rounds, count, write), divided
by the number of walk dispatches (one per call).  FETCH_SIZE is taken raw: the walk is random
16-B gathers, for which tools/gather_bench.hip calibrated 64 B per L2 miss.

    python tools/pmc_retain.py --dir gpurun_out/<tag> --retained 864333 --filters 100000
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--out", default=None)
    ap.add_argument("--filters", type=int, required=True)
    ap.add_argument("--retained", type=int, required=True)
    args = ap.parse_args()
    res = {}
    for counter in ("FETCH_SIZE", "WRITE_SIZE"):
        tot, walks, per_kernel = 0.0, set(), defaultdict(float)
        for p in sorted(glob.glob(os.path.join(args.dir, "**", "*counter_collection.csv"), recursive=True)):
            with open(p, newline="") as f:
                for r in csv.DictReader(f):
                    name = r.get("Kernel_Name", "")
                    if "retain_" not in name or r["Counter_Name"] != counter:
                        continue
                    v = float(r["Counter_Value"]) * 1024  # KiB
                    tot += v
                    per_kernel[name.split("(")[0]] += v
                    if "retain_walk_kernel" in name or "retain_walk_queue_kernel" in name:
                        walks.add((p, r["Dispatch_Id"]))
        if walks:
            res[counter] = {"bytes_per_call": tot / len(walks), "calls": len(walks),
                            "per_kernel_per_call": {k: v / len(walks) for k, v in per_kernel.items()}}
    out = {"workload": "R", "filters_per_call": args.filters, "retained_topics": args.retained,
           "counters": res,
           "traffic_bytes_per_call": sum(c["bytes_per_call"] for c in res.values()) if len(res) == 2 else None,
           "traffic_rule": "FETCH_SIZE raw (64 B per L2 miss on random 16-B gathers) + WRITE_SIZE, all retain_* kernels of a call",
           "source": args.dir}
    s = json.dumps(out, indent=1)
    print(s)
    if args.out:
        with open(args.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
