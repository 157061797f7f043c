"""Writes tests/golden/c100m_slice.npz: the oracle's answers for the first SLICE topics of config
C's 1M-topic batch over config C's whole 100M-filter table (BASELINE configs[2]: generator B at
100M filters, vocab x4, seed 3; emqx_amd/workloads.py config_b) — the golden vectors of
tests/test_gpu_c100m.py.

The oracle is oracle/trie_oracle.cpp (the emqx_trie compact DFS + match_routes/1 union,
apps/emqx/src/emqx_trie.erl:315-334, apps/emqx/src/emqx_router.erl:128-133) restated on the
filters that can match the slice (oracle/pruned.py with pair narrowing, exact for the slice and
checked against the full-table oracle in tests/test_pruned_oracle.py).  The file also holds a
fingerprint of the generated table and batch (xxh3-64 of the packed bytes and offsets), so the
GPU test knows it generated the same inputs before it compares ids.

Run:  python tests/golden/make_c100m.py   (~5 min and ~30 GB of host memory here; deterministic)
"""

import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

N_FILTERS = 100_000_000
N_TOPICS = 1_000_000  # the C1 bench batch; the slice is its first SLICE topics
SEED, VOCAB_SCALE = 3, 4
SLICE = 12_000
OUT = os.path.join(ROOT, "tests", "golden", "c100m_slice.npz")


def fingerprint(packed) -> np.ndarray:
    """xxh3-64 of a packed list's bytes and of its offsets (u64)."""
    import xxhash
    buf, offs = packed
    return np.array([xxhash.xxh3_64_intdigest(np.ascontiguousarray(buf).data),
                     xxhash.xxh3_64_intdigest(np.ascontiguousarray(np.asarray(offs, np.uint64)).data)],
                    dtype=np.uint64)


def main():
    from emqx_amd import workloads as W
    from oracle import pruned
    t0 = time.time()
    wl = W.config_b(n_filters=N_FILTERS, n_topics=N_TOPICS, seed=SEED, vocab_scale=VOCAB_SCALE)
    print("generated in %.0f s" % (time.time() - t0), flush=True)
    sl = W.take(wl.topics, np.arange(SLICE))
    t0 = time.time()
    off, ids, cand = pruned.slice_csr(wl.filters, wl.fcodes, sl, wl.tcodes[:SLICE], threads=8, pairs=True)
    print("oracle over %d candidate filters in %.0f s: %d ids" % (len(cand), time.time() - t0, int(off[-1])),
          flush=True)
    np.savez_compressed(OUT, n_filters=N_FILTERS, n_topics=N_TOPICS, seed=SEED, vocab_scale=VOCAB_SCALE,
                        slice=SLICE, table_fp=fingerprint(wl.filters), batch_fp=fingerprint(sl),
                        candidates=len(cand), off=off.astype(np.uint64), ids=ids.astype(np.uint32))
    print("wrote", OUT, os.path.getsize(OUT), "bytes")


if __name__ == "__main__":
    main()
