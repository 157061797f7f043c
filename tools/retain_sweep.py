"""Retained-walk tuning sweep on config R in one process (experiments only): the store is built
once, then each setting runs `--calls` calls; prints median call / walk ms, pieces shared and
whether the per-filter counts and id sums equal the first setting's.

  python tools/retain_sweep.py 'balance=0' 'balance=1,queue_wait=2048' ...
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from emqx_amd import workloads as W
    from emqx_amd.engine import pack
    from emqx_amd.retainer import RetainIndex
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    calls = 12
    check = "--nocheck" not in sys.argv
    for a in sys.argv[1:]:
        if a.startswith("--calls="):
            calls = int(a.split("=")[1])
    dev = torch.device("cuda:0")
    retained, nf = 1_000_000, 100_000
    topics_wl = W.config_b(n_filters=retained // 10, n_topics=int(retained * 1.15), seed=41)
    names = list(dict.fromkeys(W.unpack(topics_wl.topics)))[:retained]
    filt_wl = W.config_b(n_filters=nf, n_topics=1000, seed=42)
    rng = np.random.default_rng(5)
    now = 1_000_000
    expiry = np.where(rng.random(len(names)) < 0.1, now - 500 + rng.integers(0, 1000, len(names)), 0).astype(np.int64)
    idx = RetainIndex(0)
    tb, to = pack(names)
    idx.store_packed(tb, to, expiry)
    idx.commit()
    fb, fo = filt_wl.filters
    d_fb = torch.from_numpy(fb.copy()).to(dev)
    d_fo = torch.from_numpy(fo.view(np.int64).copy()).to(dev)
    d_off = torch.empty(nf + 1, dtype=torch.int64, device=dev)
    cap = 1 << 24
    d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
    ref = None
    for spec in args:
        kv = dict(x.split("=") for x in spec.split(",") if x)
        for k, v in kv.items():
            idx.set_tuning(k, int(v))
        cms, wms = [], []
        t0 = time.perf_counter()
        for _ in range(calls):
            n = idx.match_device(d_fb.data_ptr(), d_fo.data_ptr(), nf, now, d_off.data_ptr(), d_ids.data_ptr(), cap)
            st = idx.stats()
            cms.append(st["last_match_ms"])
            wms.append(st["last_walk_ms"])
        wall = (time.perf_counter() - t0) / calls * 1e3
        off = d_off.cpu().numpy()
        ids = d_ids[:n].cpu().numpy().view(np.uint32).astype(np.uint64)
        cs = np.concatenate([np.zeros(1, np.uint64), np.cumsum(ids, dtype=np.uint64)])
        sig = (np.diff(off), cs[off[1:]] - cs[off[:-1]])
        same = True
        if ref is None:
            ref = sig
        else:
            same = bool(np.array_equal(ref[0], sig[0]) and np.array_equal(ref[1], sig[1]))
        print(json.dumps({"spec": spec, "call_ms": round(float(np.median(cms)), 4),
                          "walk_ms": round(float(np.median(wms)), 4), "wall_ms": round(wall, 4),
                          "pieces": int(st["last_spilled"]), "shares": int(st.get("last_shares", 0)),
                          "rounds": int(st["last_spill_rounds"]), "aborts": int(st.get("queue_aborts", 0)),
                          "same": same}), flush=True)
        if check and not same:
            raise SystemExit("results differ")


if __name__ == "__main__":
    main()
