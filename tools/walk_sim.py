"""CPU model of match_fast_kernel's L2 traffic on config B (emqx_htrie_walk_sim): builds the
table on the host (the engine's builder, no device), replays the kernel's walk of a topic batch
tile by tile against per-XCD LRU L2 models, and prints the misses per topic split by item level
and node kind.  Calibrated against the PMC passes (profiles/r3_v11_phase_split_B.json: 28.4 M
L2 misses per 1M-topic launch in the walk, 1.0 M in phase A), it prices layout ideas before
they are built.

    python tools/walk_sim.py [--n-filters 10000000] [--batch 1000000] [--resident 768]
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = ["topics", "tiles", "items", "loads", "l2_accesses", "l2_misses", "vocab_loads", "vocab_misses",
         "items_both_probes", "both_probes_split_lines", "chain_items", "chain_misses"] + \
        ["misses_l%d" % i for i in range(8)] + ["items_l%d" % i for i in range(8)] + \
        ["wide_items", "wide_misses", "steps", "plus_misses", "literal_misses", "emits", "plus_loads", "ph_loads",
         "wide_loads"] + ["hits_l%d" % i for i in range(8)] + ["spine_items", "spine_literal_misses"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-filters", type=int, default=10_000_000)
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--xcds", type=int, default=8)
    ap.add_argument("--l2-mb", type=float, default=2.0, help="effective L2 per XCD (2: calibrated to the PMC passes)")
    ap.add_argument("--line", type=int, default=64)
    ap.add_argument("--ways", type=int, default=16)
    ap.add_argument("--resident", type=int, default=768, help="tiles resident per XCD (24 waves/CU x 32 CUs)")
    ap.add_argument("--a-ticks", type=int, default=10, help="walk steps a tile's phase A lasts")
    ap.add_argument("--slab", type=int, default=1, help="1: slab writes allocate in L2")
    ap.add_argument("--whatif", type=int, default=0, help="bit 0: '+' copy in every line of a node array")
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--cache", default="/tmp/wlB_sim.npz")
    a = ap.parse_args()
    from emqx_amd import _lib
    from emqx_amd import workloads as W
    L = _lib.lib()
    t0 = time.time()
    if a.cache and os.path.exists(a.cache):
        z = np.load(a.cache)
        fb, fo, tb, to = z["fb"], z["fo"], z["tb"], z["to"]
    else:
        wl = W.config_b(n_filters=a.n_filters, n_topics=a.batch, seed=2)
        fb, fo = wl.filters
        tb, to = wl.topics
        if a.cache:
            np.savez(a.cache, fb=fb, fo=fo, tb=tb, to=to)
    print(f"workload {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    h = ctypes.c_void_p()
    assert L.emqx_htrie_create(0, a.threads, ctypes.byref(h)) == 0
    nf = len(fo) - 1
    ids = np.zeros(nf, np.uint32)
    fo = np.ascontiguousarray(fo, dtype=np.uint64)
    assert L.emqx_htrie_insert(h, fb.ctypes.data, fo.ctypes.data, nf, ids.ctypes.data) == 0
    st = np.zeros(8, np.uint64)
    assert L.emqx_htrie_commit(h, 1, st.ctypes.data) == 0
    print(f"table built {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    params = np.array([a.xcds, int(a.l2_mb * (1 << 20)), a.line, a.ways, a.resident, a.a_ticks, a.slab, a.whatif], np.uint64)
    out = np.zeros(len(NAMES), np.uint64)
    to = np.ascontiguousarray(to, dtype=np.uint64)
    n = len(to) - 1
    assert L.emqx_htrie_walk_sim(h, tb.ctypes.data, to.ctypes.data, n, params.ctypes.data, out.ctypes.data,
                                 len(NAMES)) == 0
    L.emqx_htrie_destroy(h)
    r = dict(zip(NAMES, (int(x) for x in out)))
    per = {k: round(v / n, 3) for k, v in r.items() if k not in ("topics", "tiles")}
    print(json.dumps({"params": vars(a), "sim_s": round(time.time() - t0, 1), "per_topic": per, "totals": r}))


if __name__ == "__main__":
    main()
