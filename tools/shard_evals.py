"""Per-rank capacity and walk work of the filter-sharded layout (emqx_amd/dist.py),
computed with the oracle's evals (SURVEY §8 d: node visits of the canonical level trie, the
quantity the engine's walk count equals) on config C's generator (config B's, vocab x4,
seed 3) at a reduced filter count, for G = 1, 2, 4, 8:

* two key spaces (round 3): engine A of rank r holds the root-wildcard filters and the space-L
  filters placed on r, engine B the space-P filters placed on r; a topic walks engine A of its
  L rank and engine B of its P rank (shard_plan / shard_place / topic_requests);
* the round-2 layout (first two levels hashed, wildcard-keyed filters replicated), for
  comparison: filters on the busiest rank.

Prints one JSON line per G.  Usage: python tools/shard_evals.py [--filters 2000000] [--topics 100000]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--filters", type=int, default=2_000_000)
    ap.add_argument("--topics", type=int, default=100_000)
    a = ap.parse_args()
    from emqx_amd import dist as D
    from emqx_amd import workloads as W
    from oracle import cpp as C
    import torch
    wl = W.config_b(n_filters=a.filters, n_topics=a.topics, seed=3, vocab_scale=4)
    n = wl.n_topics
    o = C.CppOracle(True)
    o.add_packed(*wl.filters)
    base = o.evals_packed(*wl.topics).astype(np.float64)
    del o
    tt = (torch.from_numpy(wl.topics[0]), torch.from_numpy(wl.topics[1].astype(np.int64)))
    for G in (1, 2, 4, 8):
        plan = D.shard_plan(wl.filters, G)
        first, span, eng = D.shard_place(wl.filters, G, plan)
        req = D.topic_requests(*tt, G, plan).numpy()
        held, ev, visits = [], [], []
        for r in range(G):
            engines = D.shard_engines(wl.filters, r, G, plan)
            held.append(sum(len(g) for _, g in engines))
            e_r, v_r = 0.0, 0
            for e, (packed, gids) in enumerate(engines):
                mine = np.nonzero(req[:, e] == 2 * r + e)[0]
                v_r += int(mine.size)
                if mine.size and len(gids):
                    o = C.CppOracle(True)
                    o.add_packed(*packed)
                    e_r += float(o.evals_packed(*W.take(wl.topics, mine)).sum())
                    del o
            ev.append(e_r)
            visits.append(v_r)
        own2 = D.shard_owner(wl.filters, G)
        r2 = max(np.count_nonzero((own2 == r) | (own2 == D.SHARD_ALL)) for r in range(G))
        print(json.dumps({
            "G": G, "filters": wl.n_filters, "topics": n, "evals_per_topic_single_table": round(base.mean(), 2),
            "two_key_spaces": {"filters_on_busiest_rank_frac": round(max(held) / wl.n_filters, 4),
                               "target_1_5_over_G": round(1.5 / G, 4),
                               "filters_stored_total_x": round(sum(held) / wl.n_filters, 3),
                               "plan_keys": int(len(plan)),
                               "max_rank_evals_per_batch_topic": round(max(ev) / n, 3),
                               "mean_rank_evals_per_batch_topic": round(float(np.mean(ev)) / n, 3),
                               "requests_per_topic": round(float(np.count_nonzero(req >= 0)) / n, 3),
                               "max_rank_requests_frac": round(max(visits) / n, 4)},
            "round2_two_level_hash": {"filters_on_busiest_rank_frac": round(r2 / wl.n_filters, 4)}}), flush=True)


if __name__ == "__main__":
    main()
