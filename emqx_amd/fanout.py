"""Publish fan-out on the device: ``emqx_broker`` subscribe/publish and ``emqx_shared_sub`` picks.

Mirrors the broker-side API around the route lookup (apps/emqx/src/emqx_broker.erl:113-214,
apps/emqx/src/emqx_shared_sub.erl:98-126):

* ``SubTable`` — the subscription table of one device (C ABI ``emqx_subtab_*``): filter id ->
  plain subscribers and ``$share`` groups (members in subscription order).
* ``Broker`` — ``subscribe/3``, ``unsubscribe/1`` and ``publish/1`` over a ``Router`` and a
  ``SubTable``.  ``publish_batch`` runs match + fan-out for a whole batch in one device call
  (``emqx_publish_batch``); the result per topic is the list of deliveries
  ``(filter, subscriber, shared)`` that ``emqx_broker:route/2`` would dispatch.

* ``PubBatcher`` — the cross-caller publish batcher (``emqx_pub_batcher_*``): single-message
  submissions from many threads coalesced into pinned device batches, as the NIF's
  ``publish_async/4`` does for many publisher processes.

Subscriber and group handles are the caller's (any hashable); they are mapped to uint32 ids
here, as the NIF maps pids and group names.  Per-message keys: the hash strategies take
``erlang:phash2(ClientId)`` (``hash_clientid``) or ``erlang:phash2(Topic)`` (``hash_topic``),
computed by the caller (the NIF does it in Erlang; phash2 is not restated here);
``round_robin`` and ``sticky`` take the *publisher* of the message, whose process dictionary
holds that state in the reference (emqx_shared_sub.erl:234-247,279-285).
"""

from __future__ import annotations

import ctypes
import threading
from typing import Dict, Hashable, List, Optional, Sequence, Tuple

import numpy as np

from . import _lib
from ._lib import (FANOUT_RETRY_BIT, FANOUT_SHARED_BIT, NO_GROUP, PICK_FRESH, PICK_NONE, PICK_RETRY, PUB_CB,
                   SHARE_HASH_CLIENTID, SHARE_HASH_TOPIC, SHARE_RANDOM, SHARE_ROUND_ROBIN, SHARE_STICKY, EngineError,
                   check)
from .engine import pack
from .router import Router

__all__ = ["SubTable", "Broker", "PubBatcher", "STRATEGIES", "FANOUT_SHARED_BIT", "FANOUT_RETRY_BIT", "NO_GROUP",
           "PICK_KINDS"]

# emqx_shared_sub:do_pick/6 result types (EMQX_PICK_*): false, {fresh, Sub}, {retry, Sub}
PICK_KINDS = {PICK_NONE: None, PICK_FRESH: "fresh", PICK_RETRY: "retry"}

# broker.shared_subscription_strategy values (emqx_shared_sub.erl:60-65); 'hash' = hash_clientid
STRATEGIES = {"random": SHARE_RANDOM, "round_robin": SHARE_ROUND_ROBIN, "sticky": SHARE_STICKY,
              "hash": SHARE_HASH_CLIENTID, "hash_clientid": SHARE_HASH_CLIENTID, "hash_topic": SHARE_HASH_TOPIC}


def _u32(a) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(a, dtype=np.uint32))


def _p(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def _strategy(s) -> int:
    return STRATEGIES[s] if isinstance(s, str) else int(s)


class SubTable:
    """One device subscription table (``emqx_subtab``)."""

    def __init__(self, device: int = -1):
        h = ctypes.c_void_p()
        check(_lib.lib().emqx_subtab_create(device, ctypes.byref(h)), "emqx_subtab_create")
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            _lib.lib().emqx_subtab_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def add(self, filter_ids, sub_ids, group_ids=None) -> None:
        f, s = _u32(filter_ids), _u32(sub_ids)
        g = None if group_ids is None else _u32(group_ids)
        check(_lib.lib().emqx_subtab_add(self._h, _p(f), _p(s), _p(g), len(f)), "emqx_subtab_add")

    def remove(self, filter_ids, sub_ids, group_ids=None) -> None:
        f, s = _u32(filter_ids), _u32(sub_ids)
        g = None if group_ids is None else _u32(group_ids)
        check(_lib.lib().emqx_subtab_remove(self._h, _p(f), _p(s), _p(g), len(f)), "emqx_subtab_remove")

    def commit(self) -> None:
        check(_lib.lib().emqx_subtab_commit(self._h), "emqx_subtab_commit")

    def commit_wait(self) -> int:
        """emqx_subtab_commit_wait: the last commit's device-half status (raw rc)."""
        return int(_lib.lib().emqx_subtab_commit_wait(self._h))

    def set_tuning(self, key: str, value: int) -> None:
        """emqx_subtab_set_tuning (fault injection for tests)."""
        check(_lib.lib().emqx_subtab_set_tuning(self._h, key.encode(), int(value)), "emqx_subtab_set_tuning")

    def stats(self) -> dict:
        c = np.zeros(4, dtype=np.uint64)
        check(_lib.lib().emqx_subtab_stats(self._h, _p(c)), "emqx_subtab_stats")
        return {"plain": int(c[0]), "shared_members": int(c[1]), "groups": int(c[2]), "device_bytes": int(c[3])}

    COMMIT_STATS = ("kind", "commits", "full_commits", "words", "records", "moves", "garbage", "host_us", "total_us")

    def commit_stats(self) -> dict:
        """emqx_subtab_commit_stats: what the commits wrote (kind 0 = full, 1 = incremental)."""
        c = np.zeros(len(self.COMMIT_STATS), dtype=np.uint64)
        check(_lib.lib().emqx_subtab_commit_stats(self._h, _p(c), len(c)), "emqx_subtab_commit_stats")
        return {k: int(v) for k, v in zip(self.COMMIT_STATS, c)}

    def forget_publishers(self, publishers) -> None:
        """Drops the round_robin / sticky state of these publishers (their processes ended)."""
        p = _u32(publishers)
        check(_lib.lib().emqx_subtab_forget_publishers(self._h, _p(p), len(p)), "emqx_subtab_forget_publishers")

    def set_alive(self, sub_ids, alive: bool) -> None:
        """emqx_subtab_set_alive: subscriber processes up / down (published by the next commit)."""
        s = _u32(sub_ids)
        check(_lib.lib().emqx_subtab_set_alive(self._h, _p(s), len(s), 1 if alive else 0), "emqx_subtab_set_alive")

    def repick(self, strategy, filter_ids, group_ids, keys, failed_lists) -> Tuple[np.ndarray, np.ndarray]:
        """emqx_share_repick: dispatch/4's retries, request i with FailedSubs = failed_lists[i];
        returns (subs, kinds) with kinds EMQX_PICK_NONE / _FRESH / _RETRY."""
        f, g = _u32(filter_ids), _u32(group_ids)
        n = len(f)
        k = None if keys is None else _u32(keys)
        off = np.zeros(n + 1, dtype=np.uint64)
        off[1:] = np.cumsum([len(x) for x in failed_lists]) if n else []
        flat = _u32([x for lst in failed_lists for x in lst]) if n and off[-1] else np.zeros(1, np.uint32)
        subs = np.zeros(max(n, 1), dtype=np.uint32)
        kinds = np.zeros(max(n, 1), dtype=np.uint32)
        check(_lib.lib().emqx_share_repick(self._h, _strategy(strategy), n, _p(f), _p(g), _p(k), _p(off), _p(flat),
                                           _p(subs), _p(kinds)), "emqx_share_repick")
        return subs[:n], kinds[:n]

    def fanout_device(self, strategy, d_moff: int, d_mids: int, n: int, d_keys: Optional[int], d_out_off: int,
                      d_out_subs: int, d_out_filters: Optional[int], cap: int, stream: Optional[int] = None) -> int:
        """Device-pointer fan-out (pointers as ints, e.g. ``tensor.data_ptr()``); returns the
        number of deliveries.  Raises ``EngineError`` (EOVERFLOW carries the needed capacity)."""
        n_out = ctypes.c_uint64(0)
        rc = _lib.lib().emqx_fanout_batch_device(
            self._h, _strategy(strategy), ctypes.c_void_p(d_moff), ctypes.c_void_p(d_mids), n,
            ctypes.c_void_p(d_keys) if d_keys else None, ctypes.c_void_p(d_out_off), ctypes.c_void_p(d_out_subs),
            ctypes.c_void_p(d_out_filters) if d_out_filters else None, cap, ctypes.byref(n_out),
            ctypes.c_void_p(stream) if stream else None)
        if rc == _lib.EMQX_EOVERFLOW:
            err = EngineError(rc, "emqx_fanout_batch_device")
            err.needed = int(n_out.value)
            raise err
        check(rc, "emqx_fanout_batch_device")
        return int(n_out.value)

    SUMMARY_WORDS = 4  # {flags (bit 0: overflow), deliveries, match entries, 0}

    def fanout_device_async(self, strategy, d_moff: int, d_mids: int, n: int, match_cap: int,
                            d_keys: Optional[int], d_out_off: int, d_out_subs: int, d_out_filters: Optional[int],
                            cap: int, d_summary: int, stream: Optional[int] = None) -> None:
        """Enqueue the fan-out on ``stream`` without host synchronisation
        (emqx_fanout_batch_device_async); the result counts land in ``d_summary``."""
        check(_lib.lib().emqx_fanout_batch_device_async(
            self._h, _strategy(strategy), ctypes.c_void_p(d_moff), ctypes.c_void_p(d_mids), n, match_cap,
            ctypes.c_void_p(d_keys) if d_keys else None, ctypes.c_void_p(d_out_off), ctypes.c_void_p(d_out_subs),
            ctypes.c_void_p(d_out_filters) if d_out_filters else None, cap, ctypes.c_void_p(d_summary),
            ctypes.c_void_p(stream) if stream else None), "emqx_fanout_batch_device_async")


def publish_packed(engine, subtab: SubTable, strategy, buf: np.ndarray, offs: np.ndarray,
                   keys: Optional[np.ndarray] = None, cap_hint: int = 1 << 16):
    """``emqx_publish_batch`` on packed topics: (out_offsets[n+1], subs, filters) where
    ``filters`` carry FANOUT_SHARED_BIT for $share picks."""
    n = len(offs) - 1
    out_off = np.zeros(n + 1, dtype=np.uint64)
    k = None if keys is None else _u32(keys)
    cap = max(cap_hint, 1)
    for _ in range(3):
        subs = np.zeros(cap, dtype=np.uint32)
        fils = np.zeros(cap, dtype=np.uint32)
        n_out = ctypes.c_uint64(0)
        rc = _lib.lib().emqx_publish_batch(engine._h, subtab.handle, _strategy(strategy), _p(buf), _p(offs), n,
                                           _p(k), _p(out_off), _p(subs), _p(fils), cap, ctypes.byref(n_out))
        if rc == _lib.EMQX_EOVERFLOW:
            cap = int(n_out.value) + 1
            continue
        check(rc, "emqx_publish_batch")
        t = int(n_out.value)
        return out_off, subs[:t], fils[:t]
    raise EngineError(_lib.EMQX_EOVERFLOW, "emqx_publish_batch")


class Broker:
    """emqx_broker + emqx_shared_sub of one node, on one device."""

    def __init__(self, device: int = -1, node: object = "emqx@127.0.0.1", strategy="round_robin"):
        self.router = Router(device, node)
        self.subs = SubTable(device)
        self.strategy = _strategy(strategy)
        self._sub_ids: Dict[Hashable, int] = {}
        self._subs_by_id: List[Hashable] = []
        self._group_ids: Dict[Hashable, int] = {}
        self._members: Dict[Tuple[bytes, Hashable], set] = {}
        self._plain: Dict[bytes, set] = {}
        self._dirty = False
        self._lock = threading.Lock()

    def _sid(self, sub) -> int:
        i = self._sub_ids.get(sub)
        if i is None:
            i = self._sub_ids[sub] = len(self._subs_by_id)
            self._subs_by_id.append(sub)
        return i

    def _gid(self, group) -> int:
        return self._group_ids.setdefault(group, len(self._group_ids))

    # emqx_broker.erl:124-163 / emqx_shared_sub.erl:300-307
    def subscribe(self, topic: bytes, sub, share=None) -> None:
        with self._lock:
            if share is None:
                s = self._plain.setdefault(topic, set())
                if sub in s:
                    return
                s.add(sub)
                self.router.add_route(topic)
            else:
                m = self._members.setdefault((topic, share), set())
                if sub in m:
                    return
                m.add(sub)
                self.router.add_route(topic, (share, self.router.node))
            fid = self.router.engine.lookup(topic)
            self.subs.add([fid], [self._sid(sub)], None if share is None else [self._gid(share)])
            self._dirty = True

    # emqx_broker.erl:169-195 / emqx_shared_sub.erl:309-314
    def unsubscribe(self, topic: bytes, sub, share=None) -> None:
        with self._lock:
            fid = self.router.engine.lookup(topic)
            if fid is None:
                return
            if share is None:
                s = self._plain.get(topic, set())
                if sub not in s:
                    return
                s.discard(sub)
                self.subs.remove([fid], [self._sid(sub)])
                if not s:
                    self.router.delete_route(topic)
            else:
                m = self._members.get((topic, share), set())
                if sub not in m:
                    return
                m.discard(sub)
                self.subs.remove([fid], [self._sid(sub)], [self._gid(share)])
                if not m:
                    self.router.delete_route(topic, (share, self.router.node))
            self._dirty = True

    def _sync(self):
        if self._dirty:
            self.router._sync()
            self.subs.commit()
            self._dirty = False

    def publish_batch(self, topics: Sequence[bytes], keys: Optional[Sequence[int]] = None, strategy=None,
                      with_retry: bool = False):
        """Deliveries per topic: [(filter, subscriber, shared)] as emqx_broker:publish/1 routes them
        on this node (``with_retry``: (filter, subscriber, shared, retry), retry = a do_pick/6
        {retry, Sub} pick, sent without an ack request)."""
        self._sync()
        st = self.strategy if strategy is None else _strategy(strategy)
        buf, offs = pack(list(topics))
        out_off, subs, fils = publish_packed(self.router.engine, self.subs, st, buf, offs,
                                             None if keys is None else np.asarray(keys, dtype=np.uint32))
        names = self.router._names
        res = []
        for i in range(len(topics)):
            row = []
            for s, f in zip(subs[out_off[i]:out_off[i + 1]], fils[out_off[i]:out_off[i + 1]]):
                shared = bool(int(f) & FANOUT_SHARED_BIT)
                fid = int(f) & ~(FANOUT_SHARED_BIT | FANOUT_RETRY_BIT)
                d = (names[fid], self._subs_by_id[int(s)], shared)
                row.append(d + (bool(int(f) & FANOUT_RETRY_BIT),) if with_retry else d)
            res.append(row)
        return res

    def publish(self, topic: bytes, key: int = 0):
        return self.publish_batch([topic], [key])[0]

    def down(self, sub) -> None:
        """The subscriber's process went down (is_alive_sub/1 false); its subscriptions stay
        until cleaned up, as between the 'DOWN' and cleanup_down/1 in the reference."""
        with self._lock:
            self.subs.set_alive([self._sid(sub)], False)
            self._dirty = True

    def repick(self, topic: bytes, share, key: int, failed, strategy=None):
        """emqx_shared_sub:dispatch/4's next pick after deliveries to ``failed`` failed:
        (type, sub) with type "fresh" / "retry", or False when the group has no member."""
        self._sync()
        st = self.strategy if strategy is None else _strategy(strategy)
        fid = self.router.engine.lookup(topic)
        gid = self._group_ids.get(share)
        if fid is None or gid is None:
            return False
        subs, kinds = self.subs.repick(st, [fid], [gid], [key], [[self._sid(x) for x in failed]])
        kind = PICK_KINDS[int(kinds[0])]
        return False if kind is None else (kind, self._subs_by_id[int(subs[0])])


class PubBatcher:
    """emqx_pub_batcher over an engine and a subscription table: ``submit`` one message (topic,
    key) with a callback ``fn(status, subs, filters)`` (numpy copies), called from the batcher's
    completion thread.  ``try_submit`` returns False instead of waiting when every pinned
    buffer is busy (EMQX_EBUSY)."""

    def __init__(self, engine, subtab: SubTable, strategy, max_batch: int = 4096, max_wait_us: int = 200):
        self._fns: Dict[int, object] = {}
        self._next = 1
        self._mu = threading.Lock()

        def on_done(ctx, status, subs, fils, n):
            with self._mu:
                fn = self._fns.pop(int(ctx or 0), None)
            if fn is None:
                return
            if status == 0 and n:
                s = np.ctypeslib.as_array(subs, shape=(n,)).copy()
                f = np.ctypeslib.as_array(fils, shape=(n,)).copy()
            else:
                s = f = np.zeros(0, np.uint32)
            fn(status, s, f)

        self._cb = PUB_CB(on_done)  # kept alive with the batcher
        h = ctypes.c_void_p()
        check(_lib.lib().emqx_pub_batcher_create(engine._h, subtab.handle, _strategy(strategy), max_batch, max_wait_us,
                                                 self._cb, ctypes.byref(h)), "emqx_pub_batcher_create")
        self._h = h

    def _register(self, fn) -> int:
        with self._mu:
            k = self._next
            self._next += 1
            self._fns[k] = fn
        return k

    def submit(self, topic: bytes, key: int, fn) -> None:
        k = self._register(fn)
        rc = _lib.lib().emqx_pub_batcher_submit(self._h, topic, len(topic), key & 0xFFFFFFFF, ctypes.c_void_p(k))
        if rc != 0:
            with self._mu:
                self._fns.pop(k, None)
        check(rc, "emqx_pub_batcher_submit")

    def try_submit(self, topic: bytes, key: int, fn) -> bool:
        k = self._register(fn)
        rc = _lib.lib().emqx_pub_batcher_try_submit(self._h, topic, len(topic), key & 0xFFFFFFFF, ctypes.c_void_p(k))
        if rc != 0:
            with self._mu:
                self._fns.pop(k, None)
        if rc == _lib.EMQX_EBUSY:
            return False
        check(rc, "emqx_pub_batcher_try_submit")
        return True

    def stats(self) -> dict:
        c = np.zeros(6, dtype=np.uint64)
        check(_lib.lib().emqx_pub_batcher_stats_ext(self._h, _p(c), 6), "emqx_pub_batcher_stats_ext")
        return {"batches": int(c[0]), "messages": int(c[1]), "max_inflight": int(c[2])}

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.lib().emqx_pub_batcher_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
