"""Pinned host batches in flight, for a rocprofv3 timeline: four 250K-topic
batches of config B's 1M batch on the 10M table, submitted together, five times.  Run under
  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d <dir> -- python3 tools/host_trace.py
then `python tools/host_trace.py --analyze <dir>` reports how much of the H2D copy time overlaps
kernels and how much the batches overlap each other."""
import argparse
import glob
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(cache):
    import torch  # noqa: F401
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine, HostBatch
    if cache and os.path.exists(cache + ".0.npz"):
        z = np.load(cache + ".0.npz")
        filters, topics = (z["fb"], z["fo"]), (z["tb"], z["to"])
    else:
        wl = W.config_b()
        filters, topics = wl.filters, wl.topics
    e = Engine(0)
    e.insert_packed(*filters)
    e.commit()
    n = len(topics[1]) - 1
    hbs = []
    for k in range(4):
        part = W.take(topics, np.arange(n * k // 4, n * (k + 1) // 4))
        hb = HostBatch(e, cap_topics=len(part[1]), cap_bytes=int(part[1][-1]) + 64, cap_ids=1 << 23)
        hb.pack(*part)
        hbs.append(hb)
    for _ in range(6):
        for hb in hbs:
            hb.submit(0)
        for hb in hbs:
            hb.wait(copy=False)
    print("done", sum(int(hb.s.n_out) for hb in hbs))


def analyze(d):
    """Steady state of the host-batch phase (from the 2nd csr_to_host_kernel on): how much of
    the span has an H2D copy running, a kernel running, both at once, and two batches'
    kernels at once."""
    import csv

    def load(pat):
        rows = []
        for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
            with open(f) as fh:
                rows += list(csv.DictReader(fh))
        return rows
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Stream_Id"])
          for r in load("*kernel_trace.csv")]
    cs = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Direction"]) for r in load("*memory_copy_trace.csv")]
    c2h = sorted(a for a, _, n, _ in ks if "csr_to_host" in n)
    if len(c2h) < 8:
        print({"kernels": len(ks), "copies": len(cs), "note": "no host-batch phase found"})
        return
    w0, w1 = c2h[1], max(b for _, b, n, _ in ks if "csr_to_host" in n)
    ks = [(max(a, w0), min(b, w1), n, s) for a, b, n, s in ks if b > w0 and a < w1]
    cs = [(max(a, w0), min(b, w1), n) for a, b, n in cs if b > w0 and a < w1 and "HOST_TO_DEVICE" in n]
    # sweep: count active kernels (per stream) and copies over time
    ev = []
    for a, b, _, st in ks:
        ev += [(a, 0, 1, st), (b, 0, -1, st)]
    for a, b, _ in cs:
        ev += [(a, 1, 1, None), (b, 1, -1, None)]
    ev.sort(key=lambda x: (x[0], -x[2]))
    act = {}
    ncopy = 0
    t_prev = w0
    tk = tc = tboth = tkk = 0
    for t, kind, dlt, st in ev:
        dt = t - t_prev
        nk = sum(1 for v in act.values() if v > 0)
        tk += dt if nk else 0
        tc += dt if ncopy else 0
        tboth += dt if (nk and ncopy) else 0
        tkk += dt if nk >= 2 else 0
        t_prev = t
        if kind == 0:
            act[st] = act.get(st, 0) + dlt
        else:
            ncopy += dlt
    span = w1 - w0
    names = {}
    for a, b, nme, _ in ks:
        k = nme.split("(")[0].replace("void ", "")[:40]
        names[k] = names.get(k, 0) + (b - a)
    print(json.dumps({"window_us": round(span / 1e3, 1), "kernel_active_frac": round(tk / span, 3),
                      "h2d_active_frac": round(tc / span, 3), "h2d_and_kernel_frac": round(tboth / span, 3),
                      "two_batches_kernels_frac": round(tkk / span, 3),
                      "kernel_us_by_name": {k: round(v / 1e3, 1) for k, v in sorted(names.items(), key=lambda x: -x[1])[:6]}}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyze", default=None)
    ap.add_argument("--cache", default="/tmp/wlB")
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
    else:
        run(a.cache)
