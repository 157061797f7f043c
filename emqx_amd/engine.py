"""Python handle on one device engine (a committed level-trie snapshot on one MI355X).

Thin wrapper over the C ABI: packing, capacity retries and CSR -> list conversion.  All
matching runs in the HIP kernels of ``emqx_amd/csrc/match_kernels.hip``.
"""

from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import MODE_ROUTES, MODE_TRIE, MODE_TRIE_WILDCARD, EngineError, check

__all__ = ["Engine", "HostBatch", "pack", "MODE_ROUTES", "MODE_TRIE", "MODE_TRIE_WILDCARD", "EngineError"]


def pack(items: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    """bytes items -> (uint8 buffer, uint64 offsets[n+1])."""
    n = len(items)
    offs = np.zeros(n + 1, dtype=np.uint64)
    if n:
        offs[1:] = np.cumsum(np.fromiter((len(s) for s in items), dtype=np.uint64, count=n))
    joined = b"".join(items)
    buf = np.frombuffer(joined, dtype=np.uint8) if joined else np.zeros(1, dtype=np.uint8)
    return np.ascontiguousarray(buf), offs


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class Engine:
    """One device table.  ``device=-1`` uses the current HIP device."""

    def __init__(self, device: int = -1):
        L = _lib.lib()
        h = ctypes.c_void_p()
        opts = _lib.EngineOpts(device, 0)
        check(L.emqx_engine_create(ctypes.byref(opts), ctypes.byref(h)), "emqx_engine_create")
        self._h = h
        self._cap_hint = 1 << 16

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().emqx_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---- mutations ---------------------------------------------------------------
    def insert_packed(self, buf: np.ndarray, offs: np.ndarray) -> np.ndarray:
        n = len(offs) - 1
        ids = np.zeros(max(n, 1), dtype=np.uint32)
        check(_lib.lib().emqx_insert_filters(self._h, _ptr(buf), _ptr(offs), n, _ptr(ids)),
              "emqx_insert_filters")
        return ids[:n]

    def insert_packed_ext(self, buf: np.ndarray, offs: np.ndarray, ext_ids: np.ndarray) -> np.ndarray:
        """Insert filters whose matches report ``ext_ids`` (e.g. global ids of a shard)."""
        n = len(offs) - 1
        ext = np.ascontiguousarray(np.asarray(ext_ids, dtype=np.uint32))
        assert ext.size == n
        ids = np.zeros(max(n, 1), dtype=np.uint32)
        check(_lib.lib().emqx_insert_filters_ext(self._h, _ptr(buf), _ptr(offs), n, _ptr(ext), _ptr(ids)),
              "emqx_insert_filters_ext")
        return ids[:n]

    def insert(self, filters: Sequence[bytes]) -> np.ndarray:
        return self.insert_packed(*pack(list(filters)))

    def delete(self, ids) -> None:
        a = np.ascontiguousarray(np.asarray(ids, dtype=np.uint32).reshape(-1))
        check(_lib.lib().emqx_delete_filters(self._h, _ptr(a), a.size), "emqx_delete_filters")

    def lookup(self, filt: bytes) -> Optional[int]:
        b = np.frombuffer(filt or b"\0", dtype=np.uint8)
        out = ctypes.c_uint32()
        rc = _lib.lib().emqx_lookup_filter(self._h, _ptr(b), len(filt), ctypes.byref(out))
        if rc == _lib.EMQX_ENOTFOUND:
            return None
        check(rc, "emqx_lookup_filter")
        return int(out.value)

    def name(self, fid: int) -> bytes:
        n = ctypes.c_uint64()
        check(_lib.lib().emqx_filter_name(self._h, fid, None, 0, ctypes.byref(n)), "emqx_filter_name")
        buf = ctypes.create_string_buffer(max(n.value, 1))
        check(_lib.lib().emqx_filter_name(self._h, fid, buf, n.value, ctypes.byref(n)), "emqx_filter_name")
        return buf.raw[: n.value]

    def set_tuning(self, key: str, value: int) -> None:
        check(_lib.lib().emqx_set_tuning(self._h, key.encode(), int(value)), "emqx_set_tuning")

    DIAG_NAMES = ("steps", "items", "lit_probes", "lit_hits", "lit_extra_loads", "plus_probes",
                  "plus_hits", "emits", "spills", "ticks_a", "ticks_b", "waves",
                  "lvl0", "lvl1", "lvl2", "lvl3", "lvl4", "lvl5", "lvl6", "lvl7+", "small_arrays", "wide_arrays")

    def diag(self, reset: bool = True) -> dict:
        out = np.zeros(32, dtype=np.uint64)
        check(_lib.lib().emqx_diag_read(self._h, _ptr(out), 32, int(reset)), "emqx_diag_read")
        return {k: int(out[i]) for i, k in enumerate(self.DIAG_NAMES)}

    def commit(self) -> None:
        check(_lib.lib().emqx_commit(self._h), "emqx_commit")

    COMMIT_STATS = ("kind", "relocations", "in_place", "patches", "new_slots", "spare_used", "spare_cap",
                    "garbage", "host_us", "extents", "vocab_slots", "upload_us")

    def commit_stats(self) -> dict:
        """Details of the last commit (emqx_commit_stats)."""
        out = np.zeros(len(self.COMMIT_STATS), dtype=np.uint64)
        check(_lib.lib().emqx_commit_stats(self._h, _ptr(out), len(out)), "emqx_commit_stats")
        return {k: int(out[i]) for i, k in enumerate(self.COMMIT_STATS)}

    def stats(self) -> dict:
        s = _lib.Stats()
        check(_lib.lib().emqx_stats_get(self._h, ctypes.byref(s)), "emqx_stats_get")
        return s.as_dict()

    # ---- matching ------------------------------------------------------------------
    def match_packed(self, buf: np.ndarray, offs: np.ndarray, mode: int = MODE_ROUTES):
        """-> (offsets[n+1] uint64, ids uint32) CSR."""
        n = len(offs) - 1
        out_off = np.zeros(n + 1, dtype=np.uint64)
        cap = self._cap_hint
        while True:
            ids = np.zeros(max(cap, 1), dtype=np.uint32)
            total = ctypes.c_uint64()
            rc = _lib.lib().emqx_match_batch(self._h, mode, _ptr(buf), _ptr(offs), n, _ptr(out_off),
                                              _ptr(ids), cap, ctypes.byref(total))
            if rc == _lib.EMQX_EOVERFLOW:
                cap = int(total.value) + 1
                self._cap_hint = max(self._cap_hint, cap)
                continue
            check(rc, "emqx_match_batch")
            return out_off, ids[: int(total.value)]

    def match(self, topics: Sequence[bytes], mode: int = MODE_ROUTES) -> List[List[int]]:
        """Per-topic lists of matching filter ids (sorted)."""
        off, ids = self.match_packed(*pack(list(topics)), mode=mode)
        return [sorted(ids[off[i]:off[i + 1]].tolist()) for i in range(len(topics))]

    def match_device(self, d_bytes_ptr: int, d_offs_ptr: int, n: int, d_out_off_ptr: int,
                     d_out_ids_ptr: int, cap: int, mode: int = MODE_ROUTES, stream: int = 0) -> int:
        """Device-resident batch (raw HIP pointers, e.g. ``tensor.data_ptr()``).  Returns the
        number of ids written; raises EngineError(EMQX_EOVERFLOW) with ``.needed`` set when
        ``cap`` is too small."""
        total = ctypes.c_uint64()
        rc = _lib.lib().emqx_match_batch_device(
            self._h, mode, ctypes.c_void_p(d_bytes_ptr), ctypes.c_void_p(d_offs_ptr), n,
            ctypes.c_void_p(d_out_off_ptr), ctypes.c_void_p(d_out_ids_ptr), cap, ctypes.byref(total),
            ctypes.c_void_p(stream) if stream else None)
        if rc == _lib.EMQX_EOVERFLOW:
            err = EngineError(rc, "emqx_match_batch_device")
            err.needed = int(total.value)
            raise err
        check(rc, "emqx_match_batch_device")
        return int(total.value)

    SUMMARY_WORDS = 8  # flags, total, evals, max stack, deferred, need_slab, deep_fill, error

    def match_device_async(self, d_bytes_ptr: int, d_offs_ptr: int, n: int, d_out_off_ptr: int,
                           d_out_ids_ptr: int, cap: int, d_summary_ptr: int, mode: int = MODE_ROUTES,
                           stream: int = 0) -> None:
        """Enqueue a device-resident batch and return at once; ``d_summary_ptr`` (8 uint64,
        device or pinned memory) receives the call summary when the stream reaches it:
        word 0 == 0 means the output is complete (see include/emqx_match.h)."""
        check(_lib.lib().emqx_match_batch_device_async(
            self._h, mode, ctypes.c_void_p(d_bytes_ptr), ctypes.c_void_p(d_offs_ptr), n,
            ctypes.c_void_p(d_out_off_ptr), ctypes.c_void_p(d_out_ids_ptr), cap, ctypes.c_void_p(d_summary_ptr),
            ctypes.c_void_p(stream) if stream else None), "emqx_match_batch_device_async")


class HostBatch:
    """A pinned host batch (emqx_host_batch_*): topics are packed straight into page-locked
    buffers the engine owns, and results come back into page-locked buffers — the NIF's
    "pinned batch buffers".  Several may be in flight at once: submit() returns at once,
    wait() blocks for this batch only."""

    def __init__(self, engine: "Engine", cap_topics: int = 1 << 16, cap_bytes: int = 4 << 20,
                 cap_ids: int = 1 << 21):
        self._engine = engine
        p = ctypes.POINTER(_lib.HostBatchStruct)()
        check(_lib.lib().emqx_host_batch_create(engine._h, cap_topics, cap_bytes, cap_ids, ctypes.byref(p)),
              "emqx_host_batch_create")
        self._p = p

    @property
    def s(self):
        return self._p.contents

    def close(self):
        if getattr(self, "_p", None):
            _lib.lib().emqx_host_batch_destroy(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def pack(self, buf: np.ndarray, offs: np.ndarray):
        """Copies a packed batch (offsets rebased to 0) into the pinned inputs."""
        n = len(offs) - 1
        o = np.asarray(offs, dtype=np.uint64)
        nb = int(o[-1] - o[0]) if n else 0
        s = self.s
        if n > s.cap_topics or nb > s.cap_bytes:
            check(_lib.lib().emqx_host_batch_reserve(self._p, max(n, s.cap_topics), max(nb, s.cap_bytes), s.cap_ids),
                  "emqx_host_batch_reserve")
            s = self.s
        if nb:
            ctypes.memmove(s.topic_bytes, np.ascontiguousarray(buf[int(o[0]):int(o[-1])]).ctypes.data, nb)
        dst = np.ctypeslib.as_array(s.topic_offsets, shape=(n + 1,))
        dst[:] = o - o[0]
        s.n = n

    def submit(self, mode: int = MODE_ROUTES):
        self._mode_last = mode
        check(_lib.lib().emqx_host_batch_submit(self._p, mode), "emqx_host_batch_submit")

    def wait(self, copy: bool = True):
        """-> (offsets uint64 (n+1,), ids uint32): views of the pinned outputs (copy=False) or
        copies.  Grows the id buffer and reruns once on EMQX_EOVERFLOW."""
        rc = _lib.lib().emqx_host_batch_wait(self._p)
        if rc == _lib.EMQX_EOVERFLOW:
            s = self.s
            check(_lib.lib().emqx_host_batch_reserve(self._p, s.cap_topics, s.cap_bytes, s.n_out + 1024),
                  "emqx_host_batch_reserve")
            rc = _lib.lib().emqx_host_batch_submit(self._p, self._mode_last)
            if rc == 0:
                rc = _lib.lib().emqx_host_batch_wait(self._p)
        check(rc, "emqx_host_batch_wait")
        s = self.s
        off = np.ctypeslib.as_array(s.out_offsets, shape=(s.n + 1,))
        ids = np.ctypeslib.as_array(s.out_ids, shape=(max(s.n_out, 1),))[: s.n_out]
        return (off.copy(), ids.copy()) if copy else (off, ids)
