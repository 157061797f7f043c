"""ctypes wrapper of oracle/trie_oracle.cpp — TEST INFRASTRUCTURE ONLY.

Used by tests/ (parity checker) and bench.py's cpu_baseline leg.  Build with
``make -C oracle`` (done by ``__graft_entry__.build()``).
"""

from __future__ import annotations

import ctypes
import os
from typing import Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = os.path.join(_HERE, "_build", "liboracle.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB):
            raise RuntimeError("oracle not built: run `make -C oracle`")
        L = ctypes.CDLL(_LIB)
        vp, u64p, u32p, u8p = ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p
        L.orc_create.restype = vp
        L.orc_create.argtypes = [ctypes.c_int, ctypes.c_int]
        L.orc_destroy.argtypes = [vp]
        L.orc_add.argtypes = [vp, u8p, u64p, ctypes.c_uint64, u32p]
        L.orc_delete.argtypes = [vp, u8p, u64p, ctypes.c_uint64]
        L.orc_freeze.argtypes = [vp]
        L.orc_num_keys.restype = ctypes.c_uint64
        L.orc_num_keys.argtypes = [vp]
        L.orc_match.restype = ctypes.c_uint64
        L.orc_match.argtypes = [vp, u8p, u64p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int,
                                u32p, u32p, ctypes.c_uint32]
        L.orc_evals.argtypes = [vp, u8p, u64p, ctypes.c_uint64, u64p]
        L.orc_match_csr.restype = vp
        L.orc_match_csr.argtypes = [vp, u8p, u64p, ctypes.c_uint64, ctypes.c_int, ctypes.c_int, u64p, u64p]
        L.orc_csr_copy.argtypes = [vp, u32p]
        L.orc_csr_free.argtypes = [vp]
        L.orr_create.restype = vp
        L.orr_create.argtypes = [u8p, u64p, ctypes.c_uint64, vp]
        L.orr_destroy.argtypes = [vp]
        L.orr_select.argtypes = [vp, u8p, u64p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_int, u32p, u64p]
        L.orf_create.restype = vp
        L.orf_create.argtypes = [u32p, u32p, u32p, ctypes.c_uint64]
        L.orf_destroy.argtypes = [vp]
        L.orf_publish.restype = ctypes.c_uint64
        L.orf_publish.argtypes = [vp, u64p, u32p, ctypes.c_uint64, u32p, ctypes.c_int, u32p, u64p]
        L.orf_checksum.argtypes = [u64p, u32p, u32p, ctypes.c_uint64, u64p]
        L.orf_publish_list.argtypes = [vp, u64p, u32p, ctypes.c_uint64, u32p, ctypes.c_int, u64p, u32p, u32p]
        L.orf_publish_list_rr.argtypes = [vp, u64p, u32p, ctypes.c_uint64, u32p, u64p, u32p, u32p]
        L.orf_rr_reset.argtypes = [vp]
        L.orf_churn.restype = ctypes.c_uint64
        L.orf_churn.argtypes = [vp, u32p, u32p, u32p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int]
        L.orc_topic_match.restype = ctypes.c_int
        L.orc_topic_match.argtypes = [u8p, ctypes.c_uint64, u8p, ctypes.c_uint64]
        _lib = L
    return _lib


def pack(strs: Sequence[bytes]):
    """bytes list -> (uint8 buffer, uint64 offsets[n+1])."""
    offs = np.zeros(len(strs) + 1, dtype=np.uint64)
    if strs:
        offs[1:] = np.cumsum([len(s) for s in strs], dtype=np.uint64)
    buf = np.frombuffer(b"".join(strs), dtype=np.uint8) if strs else np.zeros(1, np.uint8)
    if buf.size == 0:
        buf = np.zeros(1, np.uint8)
    return np.ascontiguousarray(buf), offs


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


MODE_ROUTES = 0
MODE_TRIE = 1


class CppOracle:
    """compact: broker.perf.trie_compaction; trie_all: insert exact filters into the
    trie too (emqx_trie_SUITE style) instead of the router's wildcard-only trie."""

    def __init__(self, compact: bool = True, trie_all: bool = False):
        self.h = lib().orc_create(int(compact), int(trie_all))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_destroy(self.h)
            self.h = None

    def add_packed(self, buf, offs):
        n = len(offs) - 1
        ids = np.zeros(max(n, 1), dtype=np.uint32)
        lib().orc_add(self.h, _p(buf), _p(offs), n, _p(ids))
        return ids[:n]

    def add(self, filters: Sequence[bytes]):
        return self.add_packed(*pack(list(filters)))

    def delete(self, filters: Sequence[bytes]):
        buf, offs = pack(list(filters))
        lib().orc_delete(self.h, _p(buf), _p(offs), len(filters))

    def freeze(self):
        lib().orc_freeze(self.h)

    def num_keys(self) -> int:
        return int(lib().orc_num_keys(self.h))

    def match_packed(self, buf, offs, mode=MODE_ROUTES, threads=1, stride=64, want_ids=True):
        n = len(offs) - 1
        counts = np.zeros(max(n, 1), dtype=np.uint32)
        ids = np.zeros(max(n * stride, 1), dtype=np.uint32) if want_ids else None
        lookups = lib().orc_match(self.h, _p(buf), _p(offs), n, mode, threads, _p(counts),
                                  _p(ids) if want_ids else None, stride)
        return counts[:n], (ids[: n * stride].reshape(n, stride) if want_ids else None), int(lookups)

    def match_csr(self, buf, offs, mode=MODE_ROUTES, threads=1):
        """(offsets uint64 (n+1,), ids uint32 (offsets[n],) sorted per topic, total lookups)."""
        n = len(offs) - 1
        off = np.zeros(n + 1, dtype=np.uint64)
        lk = np.zeros(1, dtype=np.uint64)
        r = lib().orc_match_csr(self.h, _p(buf), _p(offs), n, mode, threads, _p(off), _p(lk))
        try:
            ids = np.zeros(max(int(off[-1]), 1), dtype=np.uint32)
            lib().orc_csr_copy(r, _p(ids))
        finally:
            lib().orc_csr_free(r)
        return off, ids[: int(off[-1])], int(lk[0])

    def match_lists(self, topics: Sequence[bytes], mode=MODE_ROUTES, threads=1, stride=256):
        buf, offs = pack(list(topics))
        counts, ids, _ = self.match_packed(buf, offs, mode, threads, stride)
        if counts.size and int(counts.max(initial=0)) > stride:
            return self.match_lists(topics, mode, threads, int(counts.max()) + 1)
        return [ids[i, : counts[i]].tolist() for i in range(len(topics))]

    def evals_packed(self, buf, offs):
        n = len(offs) - 1
        out = np.zeros(max(n, 1), dtype=np.uint64)
        lib().orc_evals(self.h, _p(buf), _p(offs), n, _p(out))
        return out[:n]


class FanoutOracle:
    """oracle/fanout_oracle.cpp: route/aggre/do_dispatch + the hash $share picks, per topic a
    delivery count and an order-free checksum of its deliveries."""

    def __init__(self, sub_filter, sub_id, sub_group):
        self._a = [np.ascontiguousarray(np.asarray(x, dtype=np.uint32)) for x in (sub_filter, sub_id, sub_group)]
        self.h = lib().orf_create(_p(self._a[0]), _p(self._a[1]), _p(self._a[2]), len(self._a[0]))

    def __del__(self):
        if getattr(self, "h", None):
            lib().orf_destroy(self.h)
            self.h = None

    def publish(self, moff, mids, keys, threads=1):
        moff = np.ascontiguousarray(np.asarray(moff, dtype=np.uint64))
        mids = np.ascontiguousarray(np.asarray(mids, dtype=np.uint32))
        keys = np.ascontiguousarray(np.asarray(keys, dtype=np.uint32))
        n = len(moff) - 1
        counts = np.zeros(max(n, 1), np.uint32)
        sums = np.zeros(max(n, 1), np.uint64)
        total = lib().orf_publish(self.h, _p(moff), _p(mids) if mids.size else None, n, _p(keys), threads,
                                  _p(counts), _p(sums))
        return counts[:n], sums[:n], int(total)

    def publish_list(self, moff, mids, keys, threads=1, round_robin=False):
        """Deliveries listed: (offsets[n+1], subscribers, filters | SHARED_BIT), route order per
        topic (oracle/fanout_oracle.cpp orf_publish_list; round_robin: orf_publish_list_rr, the
        counter seeded 0, state kept over calls until ``rr_reset``)."""
        counts, _, total = self.publish(moff, mids, keys, threads)
        moff = np.ascontiguousarray(np.asarray(moff, dtype=np.uint64))
        mids = np.ascontiguousarray(np.asarray(mids, dtype=np.uint32))
        keys = np.ascontiguousarray(np.asarray(keys, dtype=np.uint32))
        n = len(moff) - 1
        off = np.zeros(n + 1, np.uint64)
        off[1:] = np.cumsum(counts, dtype=np.uint64)
        subs = np.zeros(max(total, 1), np.uint32)
        fils = np.zeros(max(total, 1), np.uint32)
        if round_robin:
            lib().orf_publish_list_rr(self.h, _p(moff), _p(mids) if mids.size else None, n, _p(keys), _p(off),
                                      _p(subs), _p(fils))
        else:
            lib().orf_publish_list(self.h, _p(moff), _p(mids) if mids.size else None, n, _p(keys), threads, _p(off),
                                   _p(subs), _p(fils))
        return off, subs[:total], fils[:total]

    def rr_reset(self):
        """Forgets every publisher's round_robin state (orf_rr_reset)."""
        lib().orf_rr_reset(self.h)

    def churn(self, sub_filter, sub_id, sub_group, add, threads=1) -> int:
        """Subscribe (add) / unsubscribe operations as the reference's ETS bags take them
        (oracle/fanout_oracle.cpp orf_churn); returns the ops that changed the table."""
        a = [np.ascontiguousarray(np.asarray(x, dtype=np.uint32)) for x in (sub_filter, sub_id, sub_group)]
        ad = np.ascontiguousarray(np.asarray(add, dtype=np.uint8))
        return int(lib().orf_churn(self.h, _p(a[0]), _p(a[1]), _p(a[2]), ad.ctypes.data_as(ctypes.c_void_p), len(ad),
                                   threads))


def delivery_checksums(off, subs, fils):
    """fanout_oracle.cpp's per-topic checksum of a delivery CSR (e.g. the GPU's)."""
    off = np.ascontiguousarray(np.asarray(off, dtype=np.uint64))
    subs = np.ascontiguousarray(np.asarray(subs, dtype=np.uint32))
    fils = np.ascontiguousarray(np.asarray(fils, dtype=np.uint32))
    n = len(off) - 1
    sums = np.zeros(max(n, 1), np.uint64)
    lib().orf_checksum(_p(off), _p(subs) if subs.size else None, _p(fils) if fils.size else None, n, _p(sums))
    return sums[:n]


def topic_match(name: bytes, filt: bytes) -> bool:
    nb = np.frombuffer(name or b"\0", np.uint8)
    fb = np.frombuffer(filt or b"\0", np.uint8)
    return bool(lib().orc_topic_match(_p(nb), len(name), _p(fb), len(filt)))


class RetainScan:
    """oracle/retain_oracle.cpp: the reference's retained lookup as it runs (full-table
    match-spec select per wildcard filter, key read per plain one)."""

    def __init__(self, buf, offs, expiry=None):
        self._exp = None if expiry is None else np.ascontiguousarray(np.asarray(expiry, dtype=np.int64))
        self.h = lib().orr_create(_p(buf), _p(offs), len(offs) - 1, _p(self._exp) if self._exp is not None else None)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orr_destroy(self.h)
            self.h = None

    def select_packed(self, buf, offs, now: int, threads: int = 1):
        n = len(offs) - 1
        counts = np.zeros(max(n, 1), dtype=np.uint32)
        sums = np.zeros(max(n, 1), dtype=np.uint64)
        lib().orr_select(self.h, _p(buf), _p(offs), n, now, threads, _p(counts), _p(sums))
        return counts[:n], sums[:n]


def pair_csr_mismatches(off_g, a_g, b_g, off_o, a_o, b_o):
    """Topics whose (a, b) pair multisets differ between two CSRs (vectorised: pairs sorted
    within each topic, then compared element-wise)."""
    off_g = np.asarray(off_g, dtype=np.int64)
    off_o = np.asarray(off_o, dtype=np.int64)
    n = len(off_g) - 1
    cnt_g, cnt_o = np.diff(off_g), np.diff(off_o)
    bad = np.nonzero(cnt_g != cnt_o)[0]
    if bad.size or not n:
        return bad

    def canon(off, a, b):
        t = np.repeat(np.arange(n, dtype=np.int64), np.diff(off))
        key = (np.asarray(a, dtype=np.uint64) << np.uint64(32)) | np.asarray(b, dtype=np.uint64)
        o = np.lexsort((key, t))
        return key[o], t[o]

    kg, tg = canon(off_g, a_g, b_g)
    ko, _ = canon(off_o, a_o, b_o)
    return np.unique(tg[kg != ko])


def csr_mismatches(off_g, ids_g, off_o, ids_o):
    """Topics whose GPU match set differs from the oracle's (sorted filter-id
    sets per topic).  off_*: (n+1,) offsets, ids_*: the CSR ids; the oracle's ids are sorted
    per topic already, the GPU's are in any order.  Returns the sorted mismatching topic
    indices (empty array = bit-exact)."""
    off_g = np.asarray(off_g).astype(np.int64)
    off_o = np.asarray(off_o).astype(np.int64)
    n = len(off_o) - 1
    cg, co = np.diff(off_g), np.diff(off_o)
    bad = cg != co
    same = ~bad
    if int(off_g[-1] - off_g[0]) and same.any():
        ids_g = np.asarray(ids_g)[off_g[0]:off_g[-1]].astype(np.uint32).astype(np.int64)
        tg = np.repeat(np.arange(n, dtype=np.int64), cg)
        kg = np.sort((tg << 32) | ids_g)
        keep_g = same[kg >> 32]
        ids_o = np.asarray(ids_o)[: off_o[-1]].astype(np.uint32).astype(np.int64)
        to_ = np.repeat(np.arange(n, dtype=np.int64), co)
        ko = (to_ << 32) | ids_o
        ko = ko[same[to_]]
        kg = kg[keep_g]
        diff = kg != ko
        if diff.any():
            bad[np.unique(kg[diff] >> 32)] = True
    return np.nonzero(bad)[0]
