"""Per-tile timeline of match_fast_kernel on config B (diagnostic build path: emqx_set_tuning
"diag" + "timeline", emqx_diag_timeline): when each wave's tile starts, ends its phase A
(tokenize + intern) and ends its walk, and on which CU.  Summarises the occupancy profile —
how much of the kernel runs with the chip short of resident waves (the launch ramp and the
tail) — and the spread of tile durations.  One JSON line to stdout.

    python tools/timeline.py [--n-filters 10000000] [--batch 1000000]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-filters", type=int, default=10_000_000)
    ap.add_argument("--batch", type=int, default=1_000_000)
    ap.add_argument("--variant", type=int, default=-1)
    a = ap.parse_args()
    import torch
    from emqx_amd import _lib
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine
    dev = torch.device("cuda", 0)
    t0 = time.time()
    wl = W.config_b(n_filters=a.n_filters, n_topics=a.batch, seed=2)
    e = Engine(0)
    e.insert_packed(*wl.filters)
    e.commit()
    if a.variant >= 0:
        e.set_tuning("fast_variant", a.variant)
    print(f"table ready {time.time() - t0:.1f}s", file=sys.stderr)
    n = wl.n_topics
    tb = torch.from_numpy(wl.topics[0]).to(dev)
    to = torch.from_numpy(wl.topics[1].view(np.int64)).to(dev)
    cap = 64 * n
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ids = torch.empty(cap, dtype=torch.int32, device=dev)

    def call():
        return e.match_device(tb.data_ptr(), to.data_ptr(), n, off.data_ptr(), ids.data_ptr(), cap)

    for _ in range(3):
        call()
    plain_ms = []
    for _ in range(5):
        call()
        plain_ms.append(e.stats()["last_kernel_ms"])
    ntiles = (n + 63) // 64
    e.set_tuning("timeline", ntiles)
    e.set_tuning("diag", 1)
    call()
    diag_ms = e.stats()["last_kernel_ms"]
    e.set_tuning("diag", 0)
    buf = np.zeros((ntiles, 4), dtype=np.uint32)
    got = ctypes.c_uint64(0)
    _lib.check(_lib.lib().emqx_diag_timeline(e._h, buf.ctypes.data, ntiles, ctypes.byref(got)), "emqx_diag_timeline")
    e.set_tuning("timeline", 0)
    start = (buf[:, 0].astype(np.uint64) | (buf[:, 1].astype(np.uint64) << np.uint64(32))).astype(np.int64)
    a_ticks = (buf[:, 2] & 0xFFFFF).astype(np.int64)
    cu = (buf[:, 2] >> 20).astype(np.int64)
    dur = buf[:, 3].astype(np.int64)
    t_begin = start.min()
    s = (start - t_begin) * 10.0 / 1e3  # us (100 MHz ticks)
    d = dur * 10.0 / 1e3
    end = s + d
    span = float(end.max())
    # resident tiles over time, 2-us buckets
    nb = int(np.ceil(span / 2.0)) + 1
    delta = np.zeros(nb + 1)
    np.add.at(delta, np.floor(s / 2.0).astype(np.int64), 1)
    np.add.at(delta, np.floor(end / 2.0).astype(np.int64), -1)
    active = np.cumsum(delta)[:nb]
    peak = float(np.percentile(active, 95))
    low = active < 0.8 * peak
    res = {
        "workload": f"config B: {wl.n_filters} filters, {n}-topic batch, one call",
        "kernel_ms_plain": round(float(np.median(plain_ms)), 4), "kernel_ms_diag_call": round(diag_ms, 4),
        "timeline_span_us": round(span, 1), "tiles": int(ntiles),
        "tile_us": {"p10": round(float(np.percentile(d, 10)), 1), "p50": round(float(np.percentile(d, 50)), 1),
                    "p90": round(float(np.percentile(d, 90)), 1), "max": round(float(d.max()), 1)},
        "phase_a_share_of_tile_time": round(float(a_ticks.sum() / max(dur.sum(), 1)), 4),
        "resident_tiles": {"p95": peak, "mean": round(float(active.mean()), 1)},
        "time_below_80pct_resident_frac": round(float(low.mean()), 4),
        "tile_time_while_below_80pct_frac": round(float(active[low].sum() / max(active.sum(), 1)), 4),
        "last_start_us": round(float(s.max()), 1),
        "tiles_per_cu": {"min": int(np.bincount(cu).min()), "max": int(np.bincount(cu).max()),
                         "cus": int(np.count_nonzero(np.bincount(cu)))},
        "occupancy_profile_10us": [round(float(x), 1) for x in active[::5][:200]],
    }
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
