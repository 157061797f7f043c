"""Pinned host batches in flight, for a rocprofv3 timeline: four 250K-topic
batches of config B's 1M batch on the 10M table, submitted together, five times.  Run under
  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d <dir> -- python3 tools/host_trace.py
then `python tools/host_trace.py --analyze <dir>` reports how much of the H2D copy time overlaps
kernels and how much the batches overlap each other."""
import argparse
import glob
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
    import csv
    def load(pat):
        rows = []
        for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
            with open(f) as fh:
                rows += list(csv.DictReader(fh))
        return rows
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in load("*kernel_trace.csv")]
    cs = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", "")) for r in load("*memory_copy_trace.csv")]
    ks.sort()
    cs.sort()
    if not ks or not cs:
        print({"kernels": len(ks), "copies": len(cs)})
        return

    def union(iv):
        out = []
        for a, b in sorted(iv):
            if out and a <= out[-1][1]:
                out[-1][1] = max(out[-1][1], b)
            else:
                out.append([a, b])
        return out

    ku = union([(a, b) for a, b, _ in ks])
    def overlap(a, b):
        t = 0
        for x, y in ku:
            t += max(0, min(b, y) - max(a, x))
        return t
    h2d = [(a, b) for a, b, dr in cs if "HOST_TO_DEVICE" in dr.upper() or "H2D" in dr.upper()]
    tot = sum(b - a for a, b in h2d)
    ov = sum(overlap(a, b) for a, b in h2d)
    span = max(b for _, b, _ in ks) - min(a for a, _, _ in ks)
    kbusy = sum(b - a for a, b in ku)
    names = {}
    for a, b, nme in ks:
        k = nme.split("(")[0][:60]
        names[k] = names.get(k, 0) + (b - a)
    print({"h2d_copies": len(h2d), "h2d_ns": tot, "h2d_ns_overlapping_kernels": ov,
           "h2d_overlap_frac": round(ov / max(tot, 1), 3), "kernel_busy_frac_of_span": round(kbusy / max(span, 1), 3),
           "kernel_ns_by_name": dict(sorted(names.items(), key=lambda x: -x[1])[:8])})


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--analyze", default=None)
    ap.add_argument("--cache", default="/tmp/wlB")
    a = ap.parse_args()
    if a.analyze:
        analyze(a.analyze)
    else:
        run(a.cache)
