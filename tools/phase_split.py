"""Split match_fast_kernel's L2 traffic by phase (config B): the diagnostic kernel runs five
calls with the walk skipped after phase A (tokenize + intern; emqx_set_tuning "diag_stop"),
then five whole calls.  Run it under one `rocprofv3 --pmc ...` pass per counter group; the
`--summarise DIR` form reads those passes back: the first five diag dispatches are phase A,
the next five the whole kernel, and phase B is the difference.

    rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d OUT/p1 -o p -- python3 tools/phase_split.py
    python tools/phase_split.py --summarise OUT
"""
import argparse
import csv
import glob
import json
import os
import sys
import time
from collections import defaultdict

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CALLS = 5


def run(a):
    import torch
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine
    dev = torch.device("cuda", 0)
    t0 = time.time()
    wl = W.config_b(n_filters=a.n_filters, n_topics=a.batch, seed=2)
    e = Engine(0)
    e.insert_packed(*wl.filters)
    e.commit()
    print(f"table ready {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    n = wl.n_topics
    tb = torch.from_numpy(wl.topics[0]).to(dev)
    to = torch.from_numpy(wl.topics[1].view(np.int64)).to(dev)
    cap = 64 * n
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ids = torch.empty(cap, dtype=torch.int32, device=dev)

    def call():
        e.match_device(tb.data_ptr(), to.data_ptr(), n, off.data_ptr(), ids.data_ptr(), cap)
        return e.stats()["last_kernel_ms"]

    for _ in range(3):
        call()
    e.set_tuning("diag", 1)
    e.set_tuning("diag_stop", 1)
    a_ms = [call() for _ in range(CALLS)]
    e.set_tuning("diag_stop", 0)
    full_ms = [call() for _ in range(CALLS)]
    e.set_tuning("diag", 0)
    print(json.dumps({"phase_a_ms": round(float(np.median(a_ms)), 4),
                      "diag_full_ms": round(float(np.median(full_ms)), 4), "batch": n}), flush=True)


def summarise(d):
    per = defaultdict(lambda: defaultdict(float))  # dispatch -> counter -> value
    for p in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        with open(p, newline="") as f:
            for r in csv.DictReader(f):
                k = r.get("Kernel_Name", "")
                if "match_fast_kernel" in k and "true>" in k:
                    per[(p, int(r["Dispatch_Id"]))][r["Counter_Name"]] += float(r["Counter_Value"])
    by_pass = defaultdict(list)
    for (p, dsp), cs in sorted(per.items()):
        by_pass[p].append(cs)
    res = {"phase_a": defaultdict(float), "whole": defaultdict(float)}
    for p, lst in by_pass.items():
        if len(lst) < 2 * CALLS:
            continue
        for part, sl in (("phase_a", lst[:CALLS]), ("whole", lst[CALLS:2 * CALLS])):
            for cs in sl:
                for c, v in cs.items():
                    res[part][c] += v / CALLS
    out = {k: dict(v) for k, v in res.items()}
    out["phase_b"] = {c: out["whole"][c] - out["phase_a"].get(c, 0.0) for c in out["whole"]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-filters", type=int, default=10_000_000)
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--summarise")
    a = ap.parse_args()
    if a.summarise:
        summarise(a.summarise)
    else:
        run(a)
