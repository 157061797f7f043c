"""Diagnostic for the one-launch small-batch path on the '#'-rich table of
tests/test_gpu_small_batch.py: fresh engines, the same batch matched with small_batch on, then
again on the same engine with it off, then with it on again; prints which topics differ from the
oracle in each pass (table state vs. path)."""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch  # noqa: F401
    from emqx_amd.engine import Engine
    from oracle import emqx_ref as R
    from test_gpu_small_batch import _deep_topic_batch
    filters, topics = _deep_topic_batch()
    exp = [R.brute_force_routes(filters, t) for t in topics]
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    if len(sys.argv) > 2:  # the test module's earlier tests first: a 150K-filter engine, host batches
        import numpy as np
        from emqx_amd import workloads as W
        from test_gpu_small_batch import _host_batch
        wl = W.config_b(n_filters=150_000, n_topics=4096, seed=41)
        t = Engine()
        t.insert_packed(*wl.filters)
        t.commit()
        modes = {"s1": (1,), "s0": (0,), "both": (1, 0)}[sys.argv[2]]
        sizes = (1, 3, 17, 48, 64, 65, 200, 511, 1024, 1025) if len(sys.argv) < 4 else tuple(map(int, sys.argv[3].split(",")))
        for n in sizes:
            for small in modes:
                t.set_tuning("small_batch", small)
                _host_batch(t, W.take(wl.topics, np.arange(100, 100 + n)), 0)
        t.set_tuning("small_batch", 1)
        if os.environ.get("DIAG_CLOSE"):
            t.close()
        print("prefix done", flush=True)
    for r in range(runs):
        e = Engine()
        e.insert(filters)
        e.commit()
        line = []
        for small in (1, 0, 1, 1):
            e.set_tuning("small_batch", small)
            got = e.match(topics, mode=0)
            bad = [(i, len(g), len(x)) for i, (g, x) in enumerate(zip(got, exp)) if g != x]
            line.append((small, bad[:3]))
        st = e.stats()
        print(r, line, {k: st[k] for k in ("last_evals", "last_deferred", "n_words", "n_slots")}, flush=True)
        print("  a/b/c ->", e.match([b"a/b/c"], mode=0), "expect", [R.brute_force_routes(filters, b"a/b/c")], flush=True)
        print("  lookup +/+/c/# ->", e.lookup(b"+/+/c/#"), "index", filters.index(b"+/+/c/#"), flush=True)
        print("  stats", st, flush=True)
        e.close()


if __name__ == "__main__":
    main()
