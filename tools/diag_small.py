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
        e.close()


if __name__ == "__main__":
    main()
