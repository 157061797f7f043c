"""Per-rank walk work of the filter-sharded layouts, computed by the oracle's
evals (SURVEY §8 d: node visits of the canonical level trie, the quantity the engine's walk
count equals) on config C's generator (config B's, vocab x4, seed 3) at a reduced filter
count, for G = 1, 2, 4, 8:

* first-level sharding (emqx_amd/dist.py): rank r holds the filters whose first level hashes
  to r plus every root-wildcard filter, and matches only the topics it owns;
* round-1's layout (filter i on rank i mod G): every rank walks every topic.

Prints one JSON line per G: evals per batch topic on the busiest rank, the mean rank, and
topics per rank.  Usage: python tools/shard_evals.py [--filters 2000000] [--topics 100000]"""
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
    for G in (1, 2, 4, 8):
        own_f = D.shard_owner(wl.filters, G)
        own_t = D.topic_owner(torch.from_numpy(wl.topics[0]), torch.from_numpy(wl.topics[1].astype(np.int64)),
                              G).numpy()
        new_ev, new_n, rr_ev = [], [], []
        for r in range(G):
            shard = W.take(wl.filters, np.nonzero((own_f == r) | (own_f == D.SHARD_ALL))[0])
            o = C.CppOracle(True)
            o.add_packed(*shard)
            mine = np.nonzero(own_t == r)[0]
            new_ev.append(float(o.evals_packed(*W.take(wl.topics, mine)).sum()) if mine.size else 0.0)
            new_n.append(int(mine.size))
            del o
            o = C.CppOracle(True)
            o.add_packed(*W.take(wl.filters, np.arange(r, wl.n_filters, G)))
            rr_ev.append(float(o.evals_packed(*wl.topics).sum()))
            del o
        print(json.dumps({
            "G": G, "filters": wl.n_filters, "topics": n, "evals_per_topic_single_table": round(base.mean(), 2),
            "first_level_sharding": {"max_rank_evals_per_batch_topic": round(max(new_ev) / n, 3),
                                     "mean_rank_evals_per_batch_topic": round(float(np.mean(new_ev)) / n, 3),
                                     "topics_per_rank_max_frac": round(max(new_n) / n, 4),
                                     "filters_on_busiest_rank_frac": round(float(max(
                                         np.count_nonzero((own_f == r) | (own_f == D.SHARD_ALL)) for r in range(G))
                                         / wl.n_filters), 4)},
            "round1_mod_G": {"max_rank_evals_per_batch_topic": round(max(rr_ev) / n, 3)}}), flush=True)


if __name__ == "__main__":
    main()
