"""The committed config-C golden vectors (tests/golden/c100m_slice.npz, made by
tests/golden/make_c100m.py) are well formed: a CSR over the slice with every topic's ids sorted,
unique and below the table size, and fingerprints for the generated table and batch."""

import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "c100m_slice.npz")


def test_c100m_golden_is_a_sorted_csr():
    g = np.load(GOLDEN)
    k, n = int(g["slice"]), int(g["n_filters"])
    off, ids = g["off"].astype(np.int64), g["ids"].astype(np.int64)
    assert k >= 10_000 and n == 100_000_000 and int(g["vocab_scale"]) == 4 and int(g["seed"]) == 3
    assert off.shape == (k + 1,) and off[0] == 0 and np.all(np.diff(off) >= 0) and off[-1] == ids.size
    assert ids.size > 10 * k and ids.max() < n
    d = np.diff(ids)
    starts = np.zeros(ids.size, dtype=bool)
    starts[off[:-1][np.diff(off) > 0]] = True
    assert np.all(d[~starts[1:]] > 0)  # strictly increasing inside each topic
    assert g["table_fp"].shape == (2,) and g["batch_fp"].shape == (2,)
