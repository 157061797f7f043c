"""Synchronous per-topic matching over the cross-caller batcher (emqx_batcher_* in the C ABI).

This mirrors what the Erlang NIF does for ``emqx_router:match_routes/1``: every caller submits
one topic and blocks until its ids arrive, while the batcher's worker thread turns the
concurrent submissions into one device batch.  (In the NIF the callback enif_send()s the ids
to the waiting Erlang process; here it sets a threading.Event.)
"""

from __future__ import annotations

import ctypes
import itertools
import threading
from typing import Dict, List

from . import _lib
from ._lib import MODE_ROUTES, check
from .engine import Engine


class Batcher:
    def __init__(self, engine: Engine, mode: int = MODE_ROUTES, max_batch: int = 4096, max_wait_us: int = 200):
        self._engine = engine  # keep the engine alive for the batcher's lifetime
        self._pending: Dict[int, list] = {}
        self._lock = threading.Lock()
        self._ids = itertools.count(1)
        self._cb = _lib.BATCH_CB(self._on_result)
        h = ctypes.c_void_p()
        check(_lib.lib().emqx_batcher_create(engine._h, mode, max_batch, max_wait_us, self._cb, ctypes.byref(h)),
              "emqx_batcher_create")
        self._h = h

    def _on_result(self, ctx, status, ids, n):
        key = int(ctx or 0)
        with self._lock:
            slot = self._pending.pop(key)
        slot[1] = status
        slot[2] = [ids[i] for i in range(n)] if status == 0 else []
        slot[0].set()

    def match(self, topic: bytes) -> List[int]:
        """Blocks until this topic's filter ids come back from its batch."""
        key = next(self._ids)
        slot = [threading.Event(), None, None]
        with self._lock:
            self._pending[key] = slot
        buf = ctypes.create_string_buffer(topic, len(topic)) if topic else None
        rc = _lib.lib().emqx_batcher_submit(self._h, buf, len(topic), ctypes.c_void_p(key))
        if rc != 0:
            with self._lock:
                self._pending.pop(key, None)
            check(rc, "emqx_batcher_submit")
        slot[0].wait()
        check(slot[1], "batched match")
        return slot[2]

    def stats(self):
        b, t = ctypes.c_uint64(), ctypes.c_uint64()
        check(_lib.lib().emqx_batcher_stats(self._h, ctypes.byref(b), ctypes.byref(t)), "emqx_batcher_stats")
        return {"batches": b.value, "topics": t.value}

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().emqx_batcher_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
