"""Loader for the engine's C ABI (include/emqx_match.h -> emqx_amd/_build/libemqxmatch.so).

The library is built in-tree (``make -C emqx_amd/csrc`` / ``__graft_entry__.build()``).
There is no fallback: if the library is missing this raises, and every match call runs
on the HIP device or fails with ``EngineError``.
"""

from __future__ import annotations

import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
# EMQX_LIB: an alternative build of the same library (experiments: `make retain-prof`)
LIB_PATH = os.environ.get("EMQX_LIB") or os.path.join(HERE, "_build", "libemqxmatch.so")

EMQX_OK = 0
EMQX_EINVAL = -1
EMQX_ENOMEM = -2
EMQX_EDEVICE = -3
EMQX_EOVERFLOW = -4
EMQX_ENOTFOUND = -5
EMQX_ETOODEEP = -6
EMQX_EBUSY = -7

MODE_ROUTES = 0
MODE_TRIE = 1
MODE_TRIE_WILDCARD = 2

# Every symbol include/emqx_match.h declares (checked by tests/test_abi_cpu.py).
EXPORTS = (
    "emqx_engine_create", "emqx_engine_destroy", "emqx_insert_filters", "emqx_insert_filters_ext",
    "emqx_delete_filters",
    "emqx_lookup_filter", "emqx_filter_name", "emqx_commit", "emqx_match_batch",
    "emqx_match_batch_device", "emqx_match_batch_device_async", "emqx_stats_get", "emqx_topic_match", "emqx_topic_wildcard",
    "emqx_set_tuning", "emqx_diag_read", "emqx_diag_timeline", "emqx_build_check", "emqx_batcher_create",
    "emqx_batcher_submit", "emqx_batcher_destroy", "emqx_batcher_stats", "emqx_batcher_stats_ext",
    "emqx_batcher_submit_many", "emqx_batcher_try_submit", "emqx_strerror", "emqx_version",
    "emqx_subtab_create", "emqx_subtab_destroy", "emqx_subtab_add", "emqx_subtab_remove", "emqx_subtab_commit",
    "emqx_subtab_commit_wait", "emqx_subtab_stats", "emqx_subtab_commit_stats", "emqx_subtab_forget_publishers", "emqx_subtab_set_alive",
    "emqx_subtab_set_tuning",
    "emqx_share_repick", "emqx_coalescer_create", "emqx_coalescer_insert_filters", "emqx_coalescer_delete_filters",
    "emqx_coalescer_subscribe", "emqx_coalescer_subscribe_many", "emqx_coalescer_set_alive", "emqx_coalescer_flush", "emqx_coalescer_destroy",
    "emqx_coalescer_stats",
    "emqx_fanout_batch_device", "emqx_fanout_batch_device_async", "emqx_publish_batch",
    "emqx_pub_batch_create", "emqx_pub_batch_destroy", "emqx_pub_batch_reserve", "emqx_pub_batch_submit",
    "emqx_pub_batch_wait", "emqx_pub_batch_query",
    "emqx_pub_batcher_create", "emqx_pub_batcher_submit", "emqx_pub_batcher_try_submit",
    "emqx_pub_batcher_submit_many", "emqx_pub_batcher_destroy", "emqx_pub_batcher_stats_ext",
    "emqx_host_batch_create", "emqx_host_batch_destroy", "emqx_host_batch_reserve", "emqx_host_batch_submit",
    "emqx_host_batch_wait", "emqx_host_batch_query",
    "emqx_commit_stats", "emqx_shard_owner", "emqx_shard_owner_device",
    "emqx_shard_plan", "emqx_shard_place", "emqx_shard_route", "emqx_shard_route_device", "emqx_permute_scratch_bytes", "emqx_batch_permute_device", "emqx_owner_sort_scratch_bytes",
    "emqx_owner_sort_device", "emqx_shard_step_create", "emqx_shard_step_destroy", "emqx_shard_send_cap",
    "emqx_shard_step_send", "emqx_shard_step_recv", "emqx_shard_step_answer", "emqx_shard_step_merge",
    "emqx_shard_step_send_fixed", "emqx_shard_step_recv_fixed", "emqx_shard_step_answer_fixed",
    "emqx_shard_step_merge_fixed",
    "emqx_csr_unpermute_device", "emqx_htrie_create", "emqx_htrie_destroy", "emqx_htrie_insert", "emqx_htrie_delete",
    "emqx_htrie_commit", "emqx_htrie_match", "emqx_htrie_check", "emqx_htrie_walk_sim",
)
# Every symbol include/emqx_retain.h declares (retained-message index).
RETAIN_EXPORTS = (
    "emqx_retain_create", "emqx_retain_destroy", "emqx_retain_store", "emqx_retain_delete",
    "emqx_retain_lookup", "emqx_retain_topic", "emqx_retain_expired", "emqx_retain_commit",
    "emqx_retain_match_batch", "emqx_retain_match_batch_device", "emqx_retain_stats_get",
    "emqx_retain_match_spec_batch", "emqx_retain_set_tuning",
)

NO_GROUP = 0xFFFFFFFF
SHARD_NONE = 0xFFFFFFFF
FANOUT_SHARED_BIT = 0x80000000
FANOUT_RETRY_BIT = 0x40000000
PICK_NONE, PICK_FRESH, PICK_RETRY = 0, 1, 2
SHARE_RANDOM, SHARE_ROUND_ROBIN, SHARE_STICKY, SHARE_HASH_CLIENTID, SHARE_HASH_TOPIC = 0, 1, 2, 3, 4


class EngineError(RuntimeError):
    def __init__(self, code: int, what: str = ""):
        self.code = code
        msg = lib().emqx_strerror(code).decode(errors="replace")
        super().__init__(f"{what}: {msg} ({code})" if what else f"{msg} ({code})")


class EngineOpts(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("flags", ctypes.c_uint32)]


class Stats(ctypes.Structure):
    _fields_ = [
        ("size", ctypes.c_uint64),
        ("n_filters", ctypes.c_uint64), ("n_ids", ctypes.c_uint64), ("n_nodes", ctypes.c_uint64),
        ("n_slots", ctypes.c_uint64), ("n_words", ctypes.c_uint64), ("table_bytes", ctypes.c_uint64),
        ("epoch", ctypes.c_uint64), ("last_evals", ctypes.c_uint64), ("last_deferred", ctypes.c_uint64),
        ("last_max_stack", ctypes.c_uint64),
        ("last_build_ms", ctypes.c_double), ("last_match_ms", ctypes.c_double),
        ("last_kernel_ms", ctypes.c_double),
        ("delta_filters", ctypes.c_uint64), ("last_commit_kind", ctypes.c_uint64),
        ("max_depth", ctypes.c_uint64), ("last_ordered", ctypes.c_uint64), ("last_order_ms", ctypes.c_double),
    ]

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.size = ctypes.sizeof(self)

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "size"}


class RetainStats(ctypes.Structure):
    _fields_ = [
        ("size", ctypes.c_uint64),
        ("n_ids", ctypes.c_uint64), ("n_live", ctypes.c_uint64), ("n_nodes", ctypes.c_uint64),
        ("n_words", ctypes.c_uint64), ("table_bytes", ctypes.c_uint64), ("epoch", ctypes.c_uint64),
        ("last_ranges", ctypes.c_uint64), ("last_visits", ctypes.c_uint64), ("last_total", ctypes.c_uint64),
        ("last_build_ms", ctypes.c_double), ("last_match_ms", ctypes.c_double), ("last_walk_ms", ctypes.c_double),
        ("last_spill_rounds", ctypes.c_uint64), ("last_spilled", ctypes.c_uint64),
        ("last_spill_full", ctypes.c_uint64),
        ("last_shares", ctypes.c_uint64),
        ("queue_aborts", ctypes.c_uint64),
    ]

    def __init__(self, *a, **kw):
        super().__init__(*a, **kw)
        self.size = ctypes.sizeof(self)

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "size"}


class HostBatchStruct(ctypes.Structure):
    """struct emqx_host_batch (include/emqx_match.h): pinned buffers of one host batch."""
    _fields_ = [
        ("topic_bytes", ctypes.POINTER(ctypes.c_uint8)), ("topic_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("cap_topics", ctypes.c_uint64), ("cap_bytes", ctypes.c_uint64), ("n", ctypes.c_uint64),
        ("out_offsets", ctypes.POINTER(ctypes.c_uint64)), ("out_ids", ctypes.POINTER(ctypes.c_uint32)),
        ("cap_ids", ctypes.c_uint64), ("n_out", ctypes.c_uint64), ("priv", ctypes.c_void_p),
    ]


class PubBatchStruct(ctypes.Structure):
    """struct emqx_pub_batch (include/emqx_match.h): pinned buffers of one publish batch."""
    _fields_ = [
        ("topic_bytes", ctypes.POINTER(ctypes.c_uint8)), ("topic_offsets", ctypes.POINTER(ctypes.c_uint64)),
        ("keys", ctypes.POINTER(ctypes.c_uint32)),
        ("cap_topics", ctypes.c_uint64), ("cap_bytes", ctypes.c_uint64), ("n", ctypes.c_uint64),
        ("out_offsets", ctypes.POINTER(ctypes.c_uint64)), ("out_subs", ctypes.POINTER(ctypes.c_uint32)),
        ("out_filters", ctypes.POINTER(ctypes.c_uint32)),
        ("cap_out", ctypes.c_uint64), ("n_out", ctypes.c_uint64), ("priv", ctypes.c_void_p),
    ]


BATCH_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint64)
DONE_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int)
PUB_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_uint32),
                          ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint64)

_lib = None


def lib():
    """Loads libemqxmatch.so (once).  If torch is already imported its HIP runtime
    (same soname) is reused, so device pointers from torch tensors are valid here."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not built; run `make -C emqx_amd/csrc` or __graft_entry__.build()")
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    sig = {
        "emqx_engine_create": (i32, [ctypes.POINTER(EngineOpts), ctypes.POINTER(vp)]),
        "emqx_engine_destroy": (i32, [vp]),
        "emqx_insert_filters": (i32, [vp, vp, vp, u64, vp]),
        "emqx_insert_filters_ext": (i32, [vp, vp, vp, u64, vp, vp]),
        "emqx_delete_filters": (i32, [vp, vp, u64]),
        "emqx_lookup_filter": (i32, [vp, vp, u64, ctypes.POINTER(u32)]),
        "emqx_filter_name": (i32, [vp, u32, vp, u64, ctypes.POINTER(u64)]),
        "emqx_commit": (i32, [vp]),
        "emqx_match_batch": (i32, [vp, u32, vp, vp, u64, vp, vp, u64, ctypes.POINTER(u64)]),
        "emqx_match_batch_device": (i32, [vp, u32, vp, vp, u64, vp, vp, u64, ctypes.POINTER(u64), vp]),
        "emqx_match_batch_device_async": (i32, [vp, u32, vp, vp, u64, vp, vp, u64, vp, vp]),
        "emqx_stats_get": (i32, [vp, ctypes.POINTER(Stats)]),
        "emqx_topic_match": (i32, [vp, u64, vp, u64]),
        "emqx_topic_wildcard": (i32, [vp, u64]),
        "emqx_set_tuning": (i32, [vp, ctypes.c_char_p, ctypes.c_int64]),
        "emqx_diag_read": (i32, [vp, vp, u32, i32]),
        "emqx_diag_timeline": (i32, [vp, vp, u64, ctypes.POINTER(u64)]),
        "emqx_build_check": (i32, [vp, vp, u64, vp, ctypes.c_char_p, u64]),
        "emqx_batcher_create": (i32, [vp, u32, u32, u32, BATCH_CB, ctypes.POINTER(vp)]),
        "emqx_batcher_submit": (i32, [vp, vp, u64, vp]),
        "emqx_batcher_destroy": (i32, [vp]),
        "emqx_batcher_stats": (i32, [vp, ctypes.POINTER(u64), ctypes.POINTER(u64)]),
        "emqx_batcher_stats_ext": (i32, [vp, vp, u32]),
        "emqx_batcher_submit_many": (i32, [vp, vp, vp, u64, vp]),
        "emqx_batcher_try_submit": (i32, [vp, vp, u64, vp]),
        "emqx_subtab_create": (i32, [ctypes.c_int32, ctypes.POINTER(vp)]),
        "emqx_subtab_destroy": (i32, [vp]),
        "emqx_subtab_add": (i32, [vp, vp, vp, vp, u64]),
        "emqx_subtab_remove": (i32, [vp, vp, vp, vp, u64]),
        "emqx_subtab_commit": (i32, [vp]),
        "emqx_subtab_commit_wait": (i32, [vp]),
        "emqx_subtab_set_tuning": (i32, [vp, ctypes.c_char_p, ctypes.c_int64]),
        "emqx_subtab_stats": (i32, [vp, vp]),
        "emqx_subtab_commit_stats": (i32, [vp, vp, u32]),
        "emqx_subtab_forget_publishers": (i32, [vp, vp, u64]),
        "emqx_subtab_set_alive": (i32, [vp, vp, u64, i32]),
        "emqx_share_repick": (i32, [vp, u32, u64, vp, vp, vp, vp, vp, vp, vp]),
        "emqx_coalescer_create": (i32, [vp, vp, u32, DONE_CB, ctypes.POINTER(vp)]),
        "emqx_coalescer_insert_filters": (i32, [vp, vp, vp, u64, vp, vp]),
        "emqx_coalescer_delete_filters": (i32, [vp, vp, u64, vp]),
        "emqx_coalescer_subscribe": (i32, [vp, vp, vp, vp, u64, i32, vp]),
        "emqx_coalescer_subscribe_many": (i32, [vp, vp, vp, vp, vp, u64, vp]),
        "emqx_coalescer_set_alive": (i32, [vp, vp, u64, i32, vp]),
        "emqx_coalescer_flush": (i32, [vp]),
        "emqx_coalescer_destroy": (i32, [vp]),
        "emqx_coalescer_stats": (i32, [vp, vp, u32]),
        "emqx_pub_batch_create": (i32, [vp, vp, u32, u64, u64, u64, ctypes.POINTER(ctypes.POINTER(PubBatchStruct))]),
        "emqx_pub_batch_destroy": (i32, [ctypes.POINTER(PubBatchStruct)]),
        "emqx_pub_batch_reserve": (i32, [ctypes.POINTER(PubBatchStruct), u64, u64, u64]),
        "emqx_pub_batch_submit": (i32, [ctypes.POINTER(PubBatchStruct)]),
        "emqx_pub_batch_wait": (i32, [ctypes.POINTER(PubBatchStruct)]),
        "emqx_pub_batch_query": (i32, [ctypes.POINTER(PubBatchStruct)]),
        "emqx_pub_batcher_create": (i32, [vp, vp, u32, u32, u32, PUB_CB, ctypes.POINTER(vp)]),
        "emqx_pub_batcher_submit": (i32, [vp, vp, u64, u32, vp]),
        "emqx_pub_batcher_try_submit": (i32, [vp, vp, u64, u32, vp]),
        "emqx_pub_batcher_submit_many": (i32, [vp, vp, vp, vp, u64, vp]),
        "emqx_pub_batcher_destroy": (i32, [vp]),
        "emqx_pub_batcher_stats_ext": (i32, [vp, vp, u32]),
        "emqx_fanout_batch_device": (i32, [vp, u32, vp, vp, u64, vp, vp, vp, vp, u64, ctypes.POINTER(u64), vp]),
        "emqx_fanout_batch_device_async": (i32, [vp, u32, vp, vp, u64, u64, vp, vp, vp, vp, u64, vp, vp]),
        "emqx_publish_batch": (i32, [vp, vp, u32, vp, vp, u64, vp, vp, vp, vp, u64, ctypes.POINTER(u64)]),
        "emqx_retain_create": (i32, [ctypes.c_int32, ctypes.POINTER(vp)]),
        "emqx_retain_destroy": (i32, [vp]),
        "emqx_retain_store": (i32, [vp, vp, vp, u64, vp, vp]),
        "emqx_retain_delete": (i32, [vp, vp, u64]),
        "emqx_retain_lookup": (i32, [vp, vp, u64, ctypes.POINTER(u32)]),
        "emqx_retain_topic": (i32, [vp, u32, vp, u64, ctypes.POINTER(u64)]),
        "emqx_retain_expired": (i32, [vp, ctypes.c_int64, vp, u64, ctypes.POINTER(u64)]),
        "emqx_retain_commit": (i32, [vp]),
        "emqx_retain_match_batch": (i32, [vp, vp, vp, u64, ctypes.c_int64, vp, vp, u64, ctypes.POINTER(u64)]),
        "emqx_retain_set_tuning": (i32, [vp, ctypes.c_char_p, ctypes.c_int64]),
        "emqx_retain_match_spec_batch": (i32, [vp, vp, vp, u64, ctypes.c_int64, vp, vp, u64, ctypes.POINTER(u64)]),
        "emqx_retain_match_batch_device": (i32, [vp, vp, vp, u64, ctypes.c_int64, vp, vp, u64,
                                                 ctypes.POINTER(u64), vp]),
        "emqx_retain_stats_get": (i32, [vp, ctypes.POINTER(RetainStats)]),
        "emqx_commit_stats": (i32, [vp, vp, u32]),
        "emqx_shard_owner": (i32, [vp, vp, u64, u32, u32, i32, vp]),
        "emqx_shard_owner_device": (i32, [vp, vp, u64, u32, u32, vp, vp]),
        "emqx_shard_plan": (i32, [vp, vp, u64, u32, u32, u32, vp, u32, ctypes.POINTER(u32)]),
        "emqx_shard_place": (i32, [vp, vp, u64, u32, vp, u32, vp, vp, vp]),
        "emqx_shard_route": (i32, [vp, vp, u64, u32, vp, u32, vp]),
        "emqx_shard_route_device": (i32, [vp, vp, u64, u32, vp, u32, vp, vp]),
        "emqx_permute_scratch_bytes": (u64, [u64]),
        "emqx_owner_sort_scratch_bytes": (u64, [u64, u32]),
        "emqx_owner_sort_device": (i32, [vp, u64, u32, vp, vp, vp]),
        "emqx_shard_step_create": (i32, [i32, u32, vp, u32, ctypes.POINTER(vp)]),
        "emqx_shard_step_destroy": (i32, [vp]),
        "emqx_shard_send_cap": (u64, [u64, u64, u32]),
        "emqx_shard_step_send": (i32, [vp, vp, vp, u64, vp, u64, vp, vp]),
        "emqx_shard_step_recv": (i32, [vp, vp, vp, vp, vp, vp]),
        "emqx_shard_step_answer": (i32, [vp, vp, vp, vp, u32, vp, vp, vp]),
        "emqx_shard_step_merge": (i32, [vp, vp, vp, vp, vp, vp]),
        "emqx_shard_step_send_fixed": (i32, [vp, vp, vp, u64, vp, u64, vp, vp]),
        "emqx_shard_step_recv_fixed": (i32, [vp, vp, vp, vp, vp, vp, vp]),
        "emqx_shard_step_answer_fixed": (i32, [vp, vp, vp, vp, u32, vp, u64, vp]),
        "emqx_shard_step_merge_fixed": (i32, [vp, vp, vp, vp, vp, vp]),
        "emqx_batch_permute_device": (i32, [vp, vp, u64, vp, vp, vp, vp, vp]),
        "emqx_csr_unpermute_device": (i32, [vp, vp, u64, vp, vp, vp, vp, vp]),
        "emqx_host_batch_create": (i32, [vp, u64, u64, u64, ctypes.POINTER(ctypes.POINTER(HostBatchStruct))]),
        "emqx_host_batch_destroy": (i32, [ctypes.POINTER(HostBatchStruct)]),
        "emqx_host_batch_reserve": (i32, [ctypes.POINTER(HostBatchStruct), u64, u64, u64]),
        "emqx_host_batch_submit": (i32, [ctypes.POINTER(HostBatchStruct), u32]),
        "emqx_host_batch_wait": (i32, [ctypes.POINTER(HostBatchStruct)]),
        "emqx_host_batch_query": (i32, [ctypes.POINTER(HostBatchStruct)]),
        "emqx_htrie_create": (i32, [u64, i32, ctypes.POINTER(vp)]),
        "emqx_htrie_destroy": (i32, [vp]),
        "emqx_htrie_insert": (i32, [vp, vp, vp, u64, vp]),
        "emqx_htrie_delete": (i32, [vp, vp, u64]),
        "emqx_htrie_commit": (i32, [vp, i32, vp]),
        "emqx_htrie_match": (i32, [vp, u32, vp, vp, u64, vp, vp, u64, ctypes.POINTER(u64)]),
        "emqx_htrie_check": (i32, [vp, ctypes.c_char_p, u64]),
        "emqx_htrie_walk_sim": (i32, [vp, vp, vp, u64, vp, vp, u32]),
        "emqx_strerror": (ctypes.c_char_p, [i32]),
        "emqx_version": (ctypes.c_char_p, []),
    }
    for name, (res, args) in sig.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(rc: int, what: str = "") -> int:
    if rc != EMQX_OK:
        raise EngineError(rc, what)
    return rc


def loaded_path() -> str:
    return LIB_PATH if _lib is not None else ""


if __name__ == "__main__":  # pragma: no cover
    print(lib().emqx_version().decode())
    sys.exit(0)
