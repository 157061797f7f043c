"""oracle/pruned.py (the oracle restated on the filters that can match a topic slice, used for
config C's 100M table in bench.py --sharded and tests/test_gpu_c100m.py): the same answers as
the oracle over the whole table, on config C's generator at a size the CPU test can afford."""

import numpy as np

from emqx_amd import workloads as W
from oracle import cpp as C
from oracle import pruned


import pytest


@pytest.mark.parametrize("pairs", [False, True])
def test_pruned_slice_equals_full_table(pairs):
    wl = W.config_b(n_filters=300_000, n_topics=4000, seed=3, vocab_scale=4)
    k = 1500
    sl = W.take(wl.topics, np.arange(k))
    off, ids, cand = pruned.slice_csr(wl.filters, wl.fcodes, sl, wl.tcodes[:k], threads=4, pairs=pairs)
    assert 0 < len(cand) < wl.n_filters  # it does narrow
    if pairs:
        assert len(cand) < len(pruned.candidates(wl.fcodes, wl.tcodes[:k]))
    o = C.CppOracle(True)
    o.add_packed(*wl.filters)
    o.freeze()
    off2, ids2, _ = o.match_csr(*sl, threads=4)
    assert int(off[-1]) == int(off2[-1]) > 0
    assert C.csr_mismatches(off, ids, off2, ids2).size == 0


def test_candidates_keep_every_matching_filter():
    # a filter with a literal that appears in no topic at its level is dropped; '+', '#' and
    # absent levels never are
    P, H, A = pruned.PLUS_CODE, pruned.HASH_CODE, pruned.ABSENT
    f = np.array([[1, 2, A], [1, 3, A], [P, 2, A], [H, A, A], [5, P, H]], dtype=np.int32)
    t = np.array([[1, 2, 7], [4, 2, A]], dtype=np.int32)
    assert pruned.candidates(f, t).tolist() == [0, 2, 3]
    # pairs: (1, 2) occurs in a topic, (5, +) has a wildcard, (1, 3) does not occur
    f2 = np.array([[1, 2, A], [4, 7, A], [1, P, H], [4, 2, A]], dtype=np.int32)
    t2 = np.array([[1, 2, 7], [4, 2, A], [1, 7, A]], dtype=np.int32)
    assert pruned.candidates(f2, t2).tolist() == [0, 1, 2, 3]
    assert pruned.candidates(f2, t2, pairs=True).tolist() == [0, 2, 3]
