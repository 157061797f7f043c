"""Oracle answers for a topic slice of a table too large to restate whole in a test: the C++
oracle (oracle/trie_oracle.cpp, the emqx_trie DFS + match_routes/1 union) over only the filters
that can match some topic of the slice.  TEST INFRASTRUCTURE (tests/, bench.py parity legs).

The narrowing is exact for the slice: a filter matches a topic only if every literal level of
the filter before its '#' equals the topic's word at that level (emqx_topic:match/2,
apps/emqx/src/emqx_topic.erl:68-87), so a filter whose literal word at some level appears at
that level in no topic of the slice matches none of them, and dropping it changes no answer.
With pairs=True a filter whose literal words at two consecutive levels lv, lv + 1 appear
together at those levels in no topic of the slice is dropped too (the same argument on the pair:
a matching topic carries both words there).
The test is on the generator's level codes (emqx_amd/workloads.py config_b: codes of one level
index one vocabulary, so equal codes are equal words); levels whose topic vocabulary differs
from the filter's (config B's level 8) are not used to narrow.
"""

from __future__ import annotations

import numpy as np

PLUS_CODE, HASH_CODE, ABSENT = -1, -2, -3


def candidates(fcodes: np.ndarray, tcodes: np.ndarray, levels: int = 8, chunk: int = 1 << 22,
               pairs: bool = False) -> np.ndarray:
    """Indices of the filters (rows of fcodes) that may match some topic (row of tcodes)."""
    L = min(levels, fcodes.shape[1], tcodes.shape[1])
    sets = []
    for lv in range(L):
        w = tcodes[:, lv]
        sets.append(np.unique(w[w >= 0]))
    psets = []
    if pairs:
        for lv in range(L - 1):
            a, b = tcodes[:, lv].astype(np.int64), tcodes[:, lv + 1].astype(np.int64)
            both = (a >= 0) & (b >= 0)
            psets.append(np.unique((a[both] << 32) | b[both]))

    def one(c0):
        f = fcodes[c0:c0 + chunk]
        ok = np.ones(f.shape[0], dtype=bool)
        for lv, words in enumerate(sets):
            col = f[:, lv]
            lit = col >= 0
            ok &= ~lit | np.isin(col, words)
        for lv, keys in enumerate(psets):
            a, b = f[:, lv].astype(np.int64), f[:, lv + 1].astype(np.int64)
            both = ok & (a >= 0) & (b >= 0)
            ok[both] = np.isin((a[both] << 32) | b[both], keys)
        return np.nonzero(ok)[0] + c0
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(8) as ex:
        keep = list(ex.map(one, range(0, fcodes.shape[0], chunk)))
    return np.concatenate(keep) if keep else np.zeros(0, np.int64)


def slice_csr(filters, fcodes, topics, tcodes, mode: int = 0, threads: int = 1, pairs: bool = False):
    """(offsets, ids, candidates) of the oracle for `topics` (packed) over the full table
    `filters` (packed, ids = row numbers), restated on the candidate filters only."""
    from emqx_amd.workloads import take
    from . import cpp as C
    cand = candidates(fcodes, tcodes, pairs=pairs)
    o = C.CppOracle(True, trie_all=(mode == C.MODE_TRIE))
    oid = o.add_packed(*take(filters, cand))
    o.freeze()
    off, ids, _ = o.match_csr(*topics, mode=mode, threads=threads)
    # oracle ids -> table row numbers (monotone: per-topic order stays sorted)
    glob = np.zeros(int(oid.max(initial=0)) + 1, dtype=np.int64)
    glob[oid.astype(np.int64)] = cand
    return off, glob[ids.astype(np.int64)].astype(np.uint32), cand
