"""Retained-message lookup on the device: the ``emqx_retainer_mnesia`` storage
callbacks (apps/emqx_retainer/src/emqx_retainer_mnesia.erl) over the C ABI of
include/emqx_retain.h.

:class:`RetainIndex` is the thin ABI wrapper (topic store + committed device snapshot +
batched filter lookup).  :class:`MnesiaRetainer` mirrors the backend module: it keeps the
messages on the host keyed by topic id, as the ``?TAB`` record keeps ``msg`` beside its token
key, and asks the index which topics a subscription filter selects:

  store_retained/2   -> RetainIndex.store (table-full rule of :74-98)
  read_message/2     -> exact id lookup, ``expiry == 0 or expiry >= now`` (:199-208)
  match_messages/3   -> RetainIndex.match, sorted by timestamp (sort_retained/1), cursor
                        batches of max_read_number (:146-158, :182-196)
  delete_message/2   -> exact delete, or match_delete_messages/1 for a wildcard (:117-128)
  clear_expired/1, page_read/4, clean/1, size/1
  dispatch/4         -> emqx_retainer.erl:119-131 (plain -> read, wildcard -> match)

Mutations are published by one commit the next time a lookup needs them.
"""

from __future__ import annotations

import ctypes
import threading
import time
from typing import Dict, List, NamedTuple, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import EMQX_ENOTFOUND, EMQX_EOVERFLOW, EngineError, check
from .engine import _ptr, pack


class Message(NamedTuple):
    """The fields of #message{} the retainer reads (apps/emqx/include/emqx.hrl)."""
    topic: bytes
    payload: bytes
    timestamp: int = 0        # ms
    expiry_time: int = 0      # ms, 0 = never (emqx_retainer:get_expiry_time/1)


def now_ms() -> int:
    return int(time.time() * 1000)


class RetainIndex:
    def __init__(self, device: int = -1):
        h = ctypes.c_void_p()
        check(_lib.lib().emqx_retain_create(device, ctypes.byref(h)), "emqx_retain_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().emqx_retain_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def store_packed(self, buf: np.ndarray, offs: np.ndarray, expiry: Optional[np.ndarray] = None) -> np.ndarray:
        n = len(offs) - 1
        ids = np.zeros(max(n, 1), dtype=np.uint32)
        exp = None if expiry is None else np.ascontiguousarray(np.asarray(expiry, dtype=np.int64))
        check(_lib.lib().emqx_retain_store(self._h, _ptr(buf), _ptr(offs), n, _ptr(exp), _ptr(ids)),
              "emqx_retain_store")
        return ids[:n]

    def store(self, topics: Sequence[bytes], expiry: Optional[Sequence[int]] = None) -> np.ndarray:
        return self.store_packed(*pack(list(topics)), None if expiry is None else np.asarray(expiry, np.int64))

    def delete(self, ids) -> None:
        a = np.ascontiguousarray(np.asarray(ids, dtype=np.uint32).reshape(-1))
        check(_lib.lib().emqx_retain_delete(self._h, _ptr(a), a.size), "emqx_retain_delete")

    def lookup(self, topic: bytes) -> Optional[int]:
        out = ctypes.c_uint32()
        rc = _lib.lib().emqx_retain_lookup(self._h, topic, len(topic), ctypes.byref(out))
        if rc == EMQX_ENOTFOUND:
            return None
        check(rc, "emqx_retain_lookup")
        return int(out.value)

    def topic(self, tid: int) -> bytes:
        n = ctypes.c_uint64()
        check(_lib.lib().emqx_retain_topic(self._h, tid, None, 0, ctypes.byref(n)), "emqx_retain_topic")
        buf = ctypes.create_string_buffer(max(int(n.value), 1))
        check(_lib.lib().emqx_retain_topic(self._h, tid, buf, n.value, ctypes.byref(n)), "emqx_retain_topic")
        return buf.raw[: n.value]

    def expired(self, now: int) -> np.ndarray:
        n = ctypes.c_uint64()
        rc = _lib.lib().emqx_retain_expired(self._h, now, None, 0, ctypes.byref(n))
        if rc not in (0, EMQX_EOVERFLOW):
            check(rc, "emqx_retain_expired")
        ids = np.zeros(max(int(n.value), 1), dtype=np.uint32)
        check(_lib.lib().emqx_retain_expired(self._h, now, _ptr(ids), ids.size, ctypes.byref(n)), "emqx_retain_expired")
        return ids[: n.value]

    def commit(self) -> None:
        check(_lib.lib().emqx_retain_commit(self._h), "emqx_retain_commit")

    def set_tuning(self, key: str, value: int) -> None:
        """emqx_retain_set_tuning: "tile", "step_budget", "spill_budget", "spill_per_wave", "spill_rounds"."""
        check(_lib.lib().emqx_retain_set_tuning(self._h, key.encode(), int(value)), "emqx_retain_set_tuning")

    def stats(self) -> dict:
        st = _lib.RetainStats()
        check(_lib.lib().emqx_retain_stats_get(self._h, ctypes.byref(st)), "emqx_retain_stats_get")
        return st.as_dict()

    def match_packed(self, buf: np.ndarray, offs: np.ndarray, now: int,
                     match_spec: bool = False) -> Tuple[np.ndarray, np.ndarray]:
        """dispatch/4's topic ids for every filter: CSR (offsets[n+1] u64, ids u32).  match_spec:
        match_messages/3 / page_read/4 semantics instead (the strict expiry guard for every
        filter, emqx_retain_match_spec_batch)."""
        fn = _lib.lib().emqx_retain_match_spec_batch if match_spec else _lib.lib().emqx_retain_match_batch
        n = len(offs) - 1
        off = np.zeros(n + 1, dtype=np.uint64)
        cap = max(4 * n, 1024)
        while True:
            ids = np.zeros(cap, dtype=np.uint32)
            got = ctypes.c_uint64()
            rc = fn(self._h, _ptr(buf), _ptr(offs), n, now, _ptr(off), _ptr(ids), cap, ctypes.byref(got))
            if rc == EMQX_EOVERFLOW:
                cap = int(got.value) + 16
                continue
            check(rc, "emqx_retain_match_batch")
            return off, ids[: got.value]

    def match(self, filters: Sequence[bytes], now: int, match_spec: bool = False) -> List[List[int]]:
        off, ids = self.match_packed(*pack(list(filters)), now, match_spec)
        return [sorted(int(x) for x in ids[off[i]:off[i + 1]]) for i in range(len(filters))]

    def match_device(self, d_bytes: int, d_offs: int, n: int, now: int, d_out_off: int, d_out_ids: int, cap: int,
                     stream: int = 0) -> int:
        got = ctypes.c_uint64()
        rc = _lib.lib().emqx_retain_match_batch_device(self._h, d_bytes, d_offs, n, now, d_out_off, d_out_ids, cap,
                                                       ctypes.byref(got), ctypes.c_void_p(stream))
        if rc == EMQX_EOVERFLOW:
            err = EngineError(rc, "emqx_retain_match_batch_device")
            err.needed = int(got.value)
            raise err
        check(rc, "emqx_retain_match_batch_device")
        return int(got.value)


class MnesiaRetainer:
    """emqx_retainer_mnesia on the device index (see the module docstring)."""

    def __init__(self, device: int = -1, max_retained_messages: int = 0, max_read_number: int = 0):
        self.index = RetainIndex(device)
        self.max_retained_messages = max_retained_messages
        self.max_read_number = max_read_number
        self._msgs: Dict[int, Message] = {}
        self._dirty = False
        self._lock = threading.Lock()

    def _sync(self) -> None:
        if self._dirty:
            with self._lock:
                if self._dirty:
                    self.index.commit()
                    self._dirty = False

    # emqx_retainer_mnesia.erl:74-98
    def store_retained(self, msg: Message) -> bool:
        with self._lock:
            if self.is_table_full() and self.index.lookup(msg.topic) is None:
                return False  # mnesia:abort(table_is_full), logged by the reference
            tid = int(self.index.store([msg.topic], [msg.expiry_time])[0])
            self._msgs[tid] = msg
            self._dirty = True
            return True

    def is_table_full(self) -> bool:
        return self.max_retained_messages > 0 and self.size() >= self.max_retained_messages

    def size(self) -> int:
        return len(self._msgs)

    # emqx_retainer_mnesia.erl:199-208
    def read_message(self, topic: bytes, now: Optional[int] = None) -> List[Message]:
        now = now_ms() if now is None else now
        tid = self.index.lookup(topic)
        m = self._msgs.get(tid) if tid is not None else None
        if m is None or not (m.expiry_time == 0 or m.expiry_time >= now):
            return []
        return [m]

    def _sorted(self, ids) -> List[Message]:
        ms = [self._msgs[int(i)] for i in ids if int(i) in self._msgs]
        ms.sort(key=lambda m: m.timestamp)  # sort_retained/1: stable by timestamp
        return ms

    # emqx_retainer_mnesia.erl:146-158 (+ start_batch_read/2, batch_read_messages/2)
    def match_messages(self, filt: bytes, cursor=None, now: Optional[int] = None):
        if cursor is None:
            self._sync()
            # make_match_spec/1: the strict guard Et > Now, plain filters included
            ms = self._sorted(self.index.match([filt], now_ms() if now is None else now, match_spec=True)[0])
            if self.max_read_number == 0:
                return ms, None
            cursor = ms
        k = self.max_read_number
        batch, rest = cursor[:k], cursor[k:]
        return batch, (rest if len(batch) == k else None)

    def match_messages_batch(self, filters: Sequence[bytes], now: Optional[int] = None) -> List[List[Message]]:
        """One device call for many subscriptions (a subscribe storm)."""
        self._sync()
        return [self._sorted(ids) for ids in self.index.match(filters, now_ms() if now is None else now,
                                                              match_spec=True)]

    # emqx_retainer_mnesia.erl:117-128, 217-223
    def delete_message(self, topic: bytes) -> None:
        from .topic import wildcard
        if wildcard(topic):
            self._sync()
            ids = self.index.match([topic], -1)[0]
        else:
            tid = self.index.lookup(topic)
            ids = [] if tid is None else [tid]
        with self._lock:
            if ids:
                self.index.delete(ids)
                for i in ids:
                    self._msgs.pop(int(i), None)
                self._dirty = True

    # emqx_retainer_mnesia.erl:106-115
    def clear_expired(self, now: Optional[int] = None) -> None:
        with self._lock:
            ids = self.index.expired(now_ms() if now is None else now)
            if ids.size:
                self.index.delete(ids)
                for i in ids:
                    self._msgs.pop(int(i), None)
                self._dirty = True

    # emqx_retainer_mnesia.erl:133-144
    def page_read(self, topic: Optional[bytes], page: int, limit: int, now: Optional[int] = None) -> List[Message]:
        self._sync()
        if topic is None:
            ms = self._sorted(list(self._msgs))
            t = now_ms() if now is None else now
            ms = [m for m in ms if m.expiry_time == 0 or m.expiry_time > t]
        else:
            ms = self._sorted(self.index.match([topic], now_ms() if now is None else now, match_spec=True)[0])
        start = (page - 1) * limit if page > 1 else 0
        return ms[start:start + limit]

    def clean(self) -> None:
        with self._lock:
            ids = list(self._msgs)
            if ids:
                self.index.delete(ids)
            self._msgs.clear()
            self._dirty = True

    # emqx_retainer.erl:90-107: retained publish stores, an empty retained payload deletes
    def on_message_publish(self, msg: Message, retain: bool = True) -> None:
        if not retain:
            return
        if msg.payload == b"":
            self.delete_message(msg.topic)
        else:
            self.store_retained(msg)

    # emqx_retainer.erl:119-131
    def dispatch(self, filt: bytes, now: Optional[int] = None) -> List[Message]:
        from .topic import wildcard
        if not wildcard(filt):
            return self.read_message(filt, now)
        out, cursor = self.match_messages(filt, None, now)
        while cursor is not None:
            more, cursor = self.match_messages(filt, cursor, now)
            out.extend(more)
        return out
