"""Multi-GPU route lookup: one process per GPU, torch.distributed (RCCL over xGMI on MI355X).

SURVEY §8(e).  Two layouts:

* **Replicated** (tables that fit one GPU — 10M filters take a few GB of 288 GB): every rank
  holds the whole table and matches its own slice of the topic stream.  Pure data
  parallelism, no collective on the data path (``split_topics``).  The reference does the same
  across a cluster: every node holds a full mria copy of the route table
  (apps/emqx/src/emqx_router.erl:135, apps/emqx/src/emqx_trie.erl:72-77).

* **Filter-sharded** (``ShardedMatcher``, tables past one GPU): the filters are divided over
  the ranks by two key spaces (include/emqx_match.h emqx_shard_*, layout.h):
    - root-wildcard filters ('#', '+', '+/#', '+/+/...') live on every rank (engine A);
    - space L: a filter with a literal first level l1 lives on the rank of l1 (engine A);
    - space P: a filter '+/x/...' lives on the rank of x (engine B);
    - a key with many filters (the plan, ``shard_plan``: Zipf-hot first words) is split over
      consecutive ranks by the next level, its filters whose next level is a wildcard on all
      of them.
  A topic l1/l2/... makes one request to its L-space rank's engine A and, if it has a second
  level and is not a '$' topic, one to its P-space rank's engine B; every filter that can match
  it lives, once, on one of the two, so the answers concatenate (``shard_route``).  A rank
  holds three engines: A, B, and AB (its A and B filters in one table); a topic whose two
  requests name the same rank, or that makes only one, asks that rank's AB engine once
  (``fold_requests``) — at world 1 that is every topic, one walk each, as replication.  Each
  rank partitions its batch's requests by (rank, engine slot), one all-to-all carries them to
  their owners, each rank matches what it received on its engines, and one all-to-all brings
  the results back, where they are merged per topic in batch order.  The busiest rank holds
  18 % of config C's filters at G = 8 (the replicated share was 29 % with the
  round-2 layout), and each rank walks ~1/G of the topics' node visits.
  Each engine is built with GLOBAL filter ids (``emqx_insert_filters_ext``).
"""

from __future__ import annotations

import contextlib
import ctypes
import os
import sys
import time
from typing import Callable, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

SHARD_ALL = 0xFFFFFFFF
SHARD_LEVELS = 2


def split_topics(packed: Tuple[np.ndarray, np.ndarray], rank: int, world: int):
    """Replicated mode: this rank's contiguous slice of a packed topic batch."""
    from .workloads import take
    n = len(packed[1]) - 1
    lo, hi = (n * rank) // world, (n * (rank + 1)) // world
    return take(packed, np.arange(lo, hi))


def shard_owner(packed: Tuple[np.ndarray, np.ndarray], world: int, levels: int = SHARD_LEVELS,
                topics: bool = False) -> np.ndarray:
    """Owner rank of each filter (uint32; SHARD_ALL = replicated) or topic, emqx_shard_owner."""
    from . import _lib
    buf, offs = packed
    offs = np.ascontiguousarray(np.asarray(offs, dtype=np.uint64))
    n = len(offs) - 1
    out = np.zeros(max(n, 1), dtype=np.uint32)
    b = np.ascontiguousarray(buf) if len(buf) else np.zeros(1, np.uint8)
    _lib.check(_lib.lib().emqx_shard_owner(b.ctypes.data, offs.ctypes.data, n, world, levels, int(topics),
                                           out.ctypes.data), "emqx_shard_owner")
    return out[:n]


def shard_filters(packed: Tuple[np.ndarray, np.ndarray], rank: int, world: int):
    """(packed filters of this rank's shard, their global ids): the filters whose key levels
    hash to `rank`, plus every replicated filter."""
    from .workloads import take
    own = shard_owner(packed, world)
    gids = np.nonzero((own == rank) | (own == SHARD_ALL))[0]
    return take(packed, gids), gids.astype(np.uint32)


def topic_owner(tb: torch.Tensor, to: torch.Tensor, world: int, levels: int = SHARD_LEVELS) -> torch.Tensor:
    """Owner rank of each topic of a batch (int64); on the batch's device (HIP kernel for a
    GPU batch).  Wildcard key levels (wildcard "topics") go to rank 0."""
    from . import _lib
    n = to.numel() - 1
    if tb.is_cuda:
        own = torch.empty(max(n, 1), dtype=torch.int32, device=tb.device)
        _lib.check(_lib.lib().emqx_shard_owner_device(
            ctypes.c_void_p(tb.data_ptr()), ctypes.c_void_p(to.data_ptr()), n, world, levels,
            ctypes.c_void_p(own.data_ptr()),
            ctypes.c_void_p(torch.cuda.current_stream(tb.device).cuda_stream)), "emqx_shard_owner_device")
        return own[:n].to(torch.int64)
    return torch.from_numpy(shard_owner((tb.numpy(), to.numpy().view(np.uint64)), world, levels,
                                        topics=True).astype(np.int64))


def partition(tb: torch.Tensor, to: torch.Tensor, owner: torch.Tensor, world: int):
    """Reorders a packed batch by owner rank (stable).  Returns (perm, lens in perm order,
    bytes in perm order, topics per rank, bytes per rank): part r is perm[sum(n_to[:r]) :
    sum(n_to[:r+1])]; the permuted bytes are the first sum(bytes_to) of `bytes`.
    Vectorized; no host round trip.  A device batch takes three HIP kernels
    (owner sort, lengths + scan, byte gather: emqx_owner_sort_device, emqx_batch_permute_device)
    and no atomics."""
    dev = tb.device
    n = owner.numel()
    lens = (to[1:] - to[:-1]).to(torch.int64)
    n_to = torch.bincount(owner, minlength=world)
    if tb.is_cuda and n:
        from . import _lib
        L = _lib.lib()
        stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
        perm32 = torch.empty(n, dtype=torch.int32, device=dev)
        scratch = torch.empty(int(L.emqx_owner_sort_scratch_bytes(n, world)), dtype=torch.uint8, device=dev)
        own32 = owner.to(torch.int32).contiguous()
        _lib.check(L.emqx_owner_sort_device(ctypes.c_void_p(own32.data_ptr()), n, world,
                                            ctypes.c_void_p(perm32.data_ptr()), ctypes.c_void_p(scratch.data_ptr()),
                                            stream), "emqx_owner_sort_device")
        perm = perm32.to(torch.int64)
        lens_p = lens[perm]
        # the permuted bytes (capacity: the whole buffer, so no host read of the byte total)
        bytes_p = torch.empty(tb.numel() + 16, dtype=torch.uint8, device=dev)
        ooffs = torch.empty(n + 1, dtype=torch.int64, device=dev)
        _device_call("emqx_batch_permute_device", tb, to, n, perm32, bytes_p, ooffs)
        ends = torch.cumsum(n_to, 0)
        bytes_to = ooffs[ends] - ooffs[ends - n_to]
        return perm, lens_p, bytes_p, n_to, bytes_to
    perm = torch.argsort(owner, stable=True)
    bytes_to = torch.zeros(world, dtype=torch.int64, device=dev).index_add_(0, owner, lens)
    lens_p = lens[perm]
    total = int(to[-1] - to[0]) if n else 0
    if total:
        starts_p = (to[:-1] - to[0])[perm]
        new_off = torch.cumsum(lens_p, 0) - lens_p
        seg = torch.repeat_interleave(torch.arange(n, device=dev), lens_p, output_size=total)
        src = starts_p[seg] + (torch.arange(total, device=dev) - new_off[seg])
        bytes_p = tb[int(to[0]):int(to[0]) + total][src]
    else:
        bytes_p = torch.zeros(0, dtype=torch.uint8, device=dev)
    return perm, lens_p, bytes_p, n_to, bytes_to


def merge_csr(recv_counts: torch.Tensor, recv_ids: torch.Tensor, perm: torch.Tensor):
    """Puts per-topic results back in batch order.  recv_counts (n,) are the counts of the
    topics in perm order (ranks' parts one after the other), recv_ids their ids laid out topic
    by topic; perm[k] = the batch index of received topic k.  Returns (offsets (n+1,) int64,
    ids int32) in batch order.  One host sync (the id total, for the allocation)."""
    dev = recv_counts.device
    n = perm.numel()
    if recv_counts.is_cuda:  # one scatter kernel (emqx_csr_unpermute_device)
        offsets = torch.empty(n + 1, dtype=torch.int64, device=dev)
        out = torch.empty(max(int(recv_ids.numel()), 1), dtype=torch.int32, device=dev)
        _device_call("emqx_csr_unpermute_device", recv_counts.to(torch.int32).contiguous(),
                     recv_ids.to(torch.int32).contiguous(), n, perm.to(torch.int32), offsets, out)
        return offsets, out[:int(recv_ids.numel())]
    counts = torch.zeros(n, dtype=torch.int64, device=dev).scatter_(0, perm, recv_counts.to(torch.int64))
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    offsets[1:] = torch.cumsum(counts, 0)
    total = int(recv_ids.numel())
    out = torch.empty(total, dtype=torch.int32, device=dev)
    if total:
        rc = recv_counts.to(torch.int64)
        recv_off = torch.cumsum(rc, 0) - rc
        k = torch.repeat_interleave(torch.arange(n, device=dev), rc, output_size=total)
        dest = offsets[perm[k]] + (torch.arange(total, device=dev) - recv_off[k])
        out[dest] = recv_ids.to(torch.int32)
    return offsets, out


def _device_call(name: str, *args):
    """A (un)permute entry point of the C ABI on the current stream, with its scratch."""
    from . import _lib
    L = _lib.lib()
    n = next(a for a in args if isinstance(a, int))
    dev = next(a for a in args if isinstance(a, torch.Tensor)).device
    scratch = torch.empty(int(L.emqx_permute_scratch_bytes(n)), dtype=torch.uint8, device=dev)
    conv = [a if isinstance(a, int) else ctypes.c_void_p(a.data_ptr()) for a in args]
    _lib.check(getattr(L, name)(*conv, ctypes.c_void_p(scratch.data_ptr()),
                                ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)), name)


def _a2a(out_t: torch.Tensor, in_t: torch.Tensor, out_splits: List[int], in_splits: List[int], group):
    if out_t.is_cuda and dist.get_backend(group) == "gloo":
        # device tensors over gloo (rehearsals of the N-rank path on a box with fewer GPUs):
        # exchange host copies, ordered after the producing stream by the copy itself
        host = torch.empty(out_t.shape, dtype=out_t.dtype)
        dist.all_to_all_single(host, in_t.cpu(), out_splits, in_splits, group=group)
        out_t.copy_(host)
        return
    dist.all_to_all_single(out_t, in_t, out_splits, in_splits, group=group)


_HIP = None


def _hip():
    """The HIP runtime torch already loaded (for hipHostGetDevicePointer)."""
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so", mode=ctypes.RTLD_GLOBAL)
        _HIP.hipHostGetDevicePointer.restype = ctypes.c_int
        _HIP.hipHostGetDevicePointer.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_uint]
    return _HIP


def _exchange_chunks(send: torch.Tensor, out_sz: List[int], in_sz: List[int], recv_buf: Callable, group,
                     rank: int) -> List[int]:
    """Chunk r of ``send`` (sizes ``out_sz`` in rank order, contiguous) to rank r; returns the
    device addresses of the chunks every source sent this rank.  The rank's own chunk is not
    moved: its address is where it lies in ``send`` (an all-to-all over one rank is no call at
    all).  RCCL: one grouped all_to_all of the other ranks' chunks.  gloo (rehearsals with
    device tensors through host copies) has no list all-to-all: all_to_all_single, the own chunk
    copied along and not read."""
    G = len(out_sz)
    base = send.data_ptr()
    if G == 1:
        return [base]
    es = send.element_size()
    gloo = dist.get_backend(group) == "gloo"
    out_off, in_off, _ = chunk_offsets(out_sz, in_sz, rank, skip_own=not gloo)
    recv = recv_buf(int(in_off[-1]))
    if gloo:
        _a2a(recv[: int(in_off[-1])], send[: int(out_off[-1])], in_sz, out_sz, group)
    else:
        empty = send[:0]
        outs = [recv[int(in_off[r]): int(in_off[r + 1])] if r != rank else empty for r in range(G)]
        ins = [send[int(out_off[r]): int(out_off[r + 1])] if r != rank else empty for r in range(G)]
        dist.all_to_all(outs, ins, group=group)
    return chunk_offsets(out_sz, in_sz, rank, skip_own=not gloo, base=base, rbase=recv.data_ptr(), es=es)[2]


def chunk_offsets(out_sz: List[int], in_sz: List[int], rank: int, skip_own: bool, base: int = 0, rbase: int = 0,
                  es: int = 1):
    """The chunk exchange's arithmetic (``_exchange_chunks``): (send offsets, receive offsets,
    the address of every source's chunk for this rank).  Chunk r of the send buffer starts at the
    prefix of out_sz; source s's chunk lands in the receive buffer at the prefix of in_sz, where
    with ``skip_own`` (RCCL's list all_to_all: the own entry empty) the own chunk takes no room;
    the own chunk is always read where it was packed (base + its send offset)."""
    G = len(out_sz)
    out_off = np.concatenate([[0], np.cumsum(out_sz)]).astype(np.int64)
    in_eff = [0 if (skip_own and r == rank) else x for r, x in enumerate(in_sz)]
    in_off = np.concatenate([[0], np.cumsum(in_eff)]).astype(np.int64)
    addrs = [base + es * int(out_off[r]) if r == rank else rbase + es * int(in_off[r]) for r in range(G)]
    return out_off, in_off, addrs


SHARD_NONE = 0xFFFFFFFF
SHARD_ENGINES = 3  # engine slots of a rank: 0 = A, 1 = B, 2 = AB (include/emqx_match.h)
MAX_PIECE_PM = 250  # a key is split when its filters exceed a quarter of a rank's share


P_SPACE = {"auto": 0, "sharded": 1, "replicated": 2}  # emqx_shard_plan p_space (include/emqx_match.h)


def fixed_steps() -> bool:
    """``ShardedMatcher.match_stream`` in the fixed-capacity form (env ``EMQX_SHARD_FIXED``, 1)."""
    return os.environ.get("EMQX_SHARD_FIXED", "1") != "0"


def step_priority() -> bool:
    """Fixed-form steps: the step's kernels on a high-priority stream (env ``EMQX_SHARD_PRIO``)."""
    return os.environ.get("EMQX_SHARD_PRIO", "0") == "1"


def stream_depth() -> int:
    """Steps in flight in ``ShardedMatcher.match_stream`` (env ``EMQX_SHARD_DEPTH``)."""
    return int(os.environ.get("EMQX_SHARD_DEPTH", "3"))


def shard_plan(filters: Tuple[np.ndarray, np.ndarray], world: int, max_piece_pm: int = MAX_PIECE_PM,
               p_space: str = "auto") -> np.ndarray:
    """The hot keys of a filter set (emqx_shard_plan): (k, 2) uint32 rows (key, first rank | span
    << 16), sorted by key.  Every rank computes the same plan from the same filters.  p_space:
    "sharded" (two key spaces: a topic asks its L-space rank and its P-space rank), "replicated"
    (the '+/x/...' filters on every rank: one request a topic), "auto" (replicated when they are
    at most a rank's share of the filters)."""
    from . import _lib
    buf, offs = filters
    offs = np.ascontiguousarray(np.asarray(offs, dtype=np.uint64))
    n = len(offs) - 1
    b = np.ascontiguousarray(buf) if len(buf) else np.zeros(1, np.uint8)
    cap = 1024
    while True:
        out = np.zeros((cap, 2), dtype=np.uint32)
        got = ctypes.c_uint32(0)
        rc = _lib.lib().emqx_shard_plan(b.ctypes.data, offs.ctypes.data, n, world, max_piece_pm, P_SPACE[p_space],
                                        out.ctypes.data, cap, ctypes.byref(got))
        if rc == _lib.EMQX_EOVERFLOW:
            cap = int(got.value)
            continue
        _lib.check(rc, "emqx_shard_plan")
        return out[: got.value].copy()


def plan_p_replicated(plan: np.ndarray) -> bool:
    """Whether the plan replicates space P (layout.h SHARD_P_REPLICATED): every topic then makes
    one request, to its rank's AB slot, and engines A and B are never asked."""
    return bool(len(plan)) and bool(((plan[:, 0] == 0x80000000) & (plan[:, 1] == 0x0000FFFF)).any())


def shard_place(filters: Tuple[np.ndarray, np.ndarray], world: int, plan: np.ndarray):
    """(first rank, span, engine) per filter (emqx_shard_place): filter i lives on ranks
    first[i] .. first[i] + span[i] - 1 (mod world), in engine A (0) or B (1)."""
    from . import _lib
    buf, offs = filters
    offs = np.ascontiguousarray(np.asarray(offs, dtype=np.uint64))
    n = len(offs) - 1
    first, span, eng = (np.zeros(max(n, 1), np.uint32) for _ in range(3))
    b = np.ascontiguousarray(buf) if len(buf) else np.zeros(1, np.uint8)
    pl = np.ascontiguousarray(plan, dtype=np.uint32) if len(plan) else np.zeros((1, 2), np.uint32)
    _lib.check(_lib.lib().emqx_shard_place(b.ctypes.data, offs.ctypes.data, n, world, pl.ctypes.data, len(plan),
                                           first.ctypes.data, span.ctypes.data, eng.ctypes.data), "emqx_shard_place")
    return first[:n], span[:n], eng[:n]


def shard_local_ids(filters: Tuple[np.ndarray, np.ndarray], rank: int, world: int, plan: np.ndarray):
    """[global ids of engine A, of engine B, of engine AB (A and B together)] for this rank
    (uint32, ascending)."""
    first, span, eng = shard_place(filters, world, plan)
    held = ((rank - first.astype(np.int64)) % world) < span
    return [np.nonzero(held & (eng == e))[0].astype(np.uint32) for e in (0, 1)] + [
        np.nonzero(held)[0].astype(np.uint32)]


def fold_requests(req: torch.Tensor, world: int) -> torch.Tensor:
    """(n, 2) raw requests (topic_requests) -> (n, 2) engine-slot keys rank * 3 + slot (3 * world
    = none), as the device step folds them (shard_step.hip shard_fold): two requests to two
    ranks stay A (slot 0) and B (slot 1); two to one rank, or a single one, become one request to
    that rank's AB engine (slot 2), in the first column."""
    E = SHARD_ENGINES
    none = torch.full_like(req[:, 0], E * world)
    a, b = req[:, 0] >= 0, req[:, 1] >= 0
    ra, rb = torch.div(req[:, 0], 2, rounding_mode="floor"), torch.div(req[:, 1], 2, rounding_mode="floor")
    split = a & b & (ra != rb)
    k0 = torch.where(split, E * ra, torch.where(a, E * ra + 2, torch.where(b, E * rb + 2, none)))
    k1 = torch.where(split, E * rb + 1, none)
    return torch.stack([k0, k1], 1)


def shard_engines(filters: Tuple[np.ndarray, np.ndarray], rank: int, world: int, plan: np.ndarray):
    """[(packed filters, global ids) of engine A, ... of engine B, ... of engine AB] for this
    rank."""
    from .workloads import take
    return [(take(filters, gids), gids) for gids in shard_local_ids(filters, rank, world, plan)]


def topic_requests(tb: torch.Tensor, to: torch.Tensor, world: int, plan: np.ndarray,
                   plan_dev: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(n, 2) int64 requests of each topic (emqx_shard_route): column 0 = rank * 2 of its engine-A
    request, column 1 = rank * 2 + 1 of its engine-B request; -1 = none.  On the batch's
    device (a HIP kernel for a GPU batch)."""
    from . import _lib
    n = to.numel() - 1
    if tb.is_cuda:
        req = torch.empty(max(2 * n, 2), dtype=torch.int32, device=tb.device)
        if plan_dev is None:
            plan_dev = torch.from_numpy(np.ascontiguousarray(plan, dtype=np.uint32).view(np.int32)).to(tb.device)
        _lib.check(_lib.lib().emqx_shard_route_device(
            ctypes.c_void_p(tb.data_ptr()), ctypes.c_void_p(to.data_ptr()), n, world,
            ctypes.c_void_p(plan_dev.data_ptr()) if len(plan) else None, len(plan), ctypes.c_void_p(req.data_ptr()),
            ctypes.c_void_p(torch.cuda.current_stream(tb.device).cuda_stream)), "emqx_shard_route_device")
        return req[: 2 * n].to(torch.int64).reshape(n, 2)
    buf = tb.numpy() if tb.numel() else np.zeros(1, np.uint8)
    offs = np.ascontiguousarray(to.numpy().astype(np.uint64))
    req = np.zeros(max(2 * n, 2), dtype=np.uint32)
    pl = np.ascontiguousarray(plan, dtype=np.uint32) if len(plan) else np.zeros((1, 2), np.uint32)
    _lib.check(_lib.lib().emqx_shard_route(np.ascontiguousarray(buf).ctypes.data, offs.ctypes.data, n, world,
                                           pl.ctypes.data, len(plan), req.ctypes.data), "emqx_shard_route")
    return torch.from_numpy(req[: 2 * n].view(np.int32).astype(np.int64)).reshape(n, 2)


def _p2p(t: Optional[torch.Tensor], peer: int, send: bool, group, like: Optional[torch.Tensor] = None):
    """Point-to-point copy of a tensor (host copies when a device tensor goes over gloo)."""
    gloo = dist.get_backend(group) == "gloo"
    if send:
        dist.send(t.cpu() if (gloo and t.is_cuda) else t, dst=peer, group=group)
        return None
    host = gloo and like.is_cuda
    buf = torch.empty(like.shape, dtype=like.dtype) if host else like
    dist.recv(buf, src=peer, group=group)
    if host:
        like.copy_(buf)
    return like


class _DeviceStep:
    """An emqx_shard_step (shard_step.hip) on this rank's device, for the rank's plan; on a CPU
    device its host mode (the kernels' per-item bodies as loops over host memory)."""

    def __init__(self, device: torch.device, world: int, plan: np.ndarray):
        from . import _lib
        self._lib = _lib
        pl = np.ascontiguousarray(plan, dtype=np.uint32) if len(plan) else np.zeros((1, 2), np.uint32)
        h = ctypes.c_void_p()
        dev = -1 if device.type != "cuda" else (device.index if device.index is not None else 0)
        _lib.check(_lib.lib().emqx_shard_step_create(dev, world, pl.ctypes.data, len(plan), ctypes.byref(h)),
                   "emqx_shard_step_create")
        self.h = h

    def close(self):
        if self.h:
            self._lib.lib().emqx_shard_step_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# EMQX_SHARD_PROF=1 (experiments): host time between the device step's calls, averaged per
# step and printed at exit: 0-1 send call, 1-2 host sync 1, 2-3 recv, 3-4 engine launches,
# 4-5 answer call, 5-6 host sync 2, 6-7 merge call.
_SHARD_PROF = os.environ.get("EMQX_SHARD_PROF") == "1"
_PROF_SUM = [0.0] * 8
_PROF_N = [0]


def _host_marks():
    t = [0.0] * 8

    def mark(k):
        t[k] = time.perf_counter()
        if k:
            _PROF_SUM[k] += t[k] - t[k - 1]
        if k == 7:
            _PROF_N[0] += 1
    return mark


if _SHARD_PROF:
    import atexit

    @atexit.register
    def _print_prof():
        n = max(_PROF_N[0], 1)
        print("EMQX_SHARD_PROF steps %d us/step: %s" % (_PROF_N[0], " ".join(
            "%d-%d %.1f" % (k - 1, k, 1e6 * _PROF_SUM[k] / n) for k in range(1, 8))), file=sys.stderr)


class _HostEngine:
    """Engine slot `slot` of a rank on the CPU: ``match_device_async`` / ``match_device`` over host
    memory, answered by a match function (counts, ids) = fn(slot, topic bytes, topic offsets) —
    what the device step's host mode calls where a rank's HIP engine would run (the CPU tests
    inject the oracle, tests/test_dist_gloo.py)."""

    def __init__(self, fn: Callable, slot: int):
        self.fn, self.slot = fn, slot

    def _run(self, b_addr, o_addr, n, off_addr, ids_addr, cap):
        offs = np.ctypeslib.as_array((ctypes.c_uint64 * (n + 1)).from_address(o_addr)).astype(np.int64)
        lo, hi = int(offs[0]), int(offs[-1])  # (a batch matched in place starts past its chunk's header)
        buf = np.ctypeslib.as_array((ctypes.c_uint8 * max(hi, 1)).from_address(b_addr))[lo:hi]
        cnt, ids = self.fn(self.slot, torch.from_numpy(buf.copy()), torch.from_numpy(offs - offs[0]))
        cnt = cnt.numpy().astype(np.int64)
        out = np.ctypeslib.as_array((ctypes.c_uint64 * (n + 1)).from_address(off_addr))
        out[0] = 0
        out[1:] = np.cumsum(cnt)
        total = int(out[-1])
        if total <= cap and total:
            np.ctypeslib.as_array((ctypes.c_int32 * total).from_address(ids_addr))[:] = ids.numpy().astype(np.int32)
        return total

    def match_device_async(self, b_addr, o_addr, n, off_addr, ids_addr, cap, sum_addr, mode=0, stream=None):
        total = self._run(b_addr, o_addr, n, off_addr, ids_addr, cap)
        sm = np.ctypeslib.as_array((ctypes.c_int64 * 8).from_address(sum_addr))
        sm[:] = 0
        sm[0] = 1 if total > cap else 0  # (engine summary: word 0 = flags, 0 when complete; word 1 = total)
        sm[1] = total

    def match_device(self, b_addr, o_addr, n, off_addr, ids_addr, cap, mode=0, stream=None):
        total = self._run(b_addr, o_addr, n, off_addr, ids_addr, cap)
        if total > cap:
            from .engine import EngineError
            from . import _lib
            err = EngineError(_lib.EMQX_EOVERFLOW, "match_device")
            err.needed = total
            raise err
        return total


class _Lane:
    """One step in flight of a ShardedMatcher: its device step (emqx_shard_step: the in-flight
    step's scratch), its reused buffers and pinned words, its streams."""

    def __init__(self, step: Optional[_DeviceStep]):
        self.step = step
        self.bufs = {}
        self.stream = None
        self.stream_b = None
        self.stream_hi = None  # (fixed form with step_priority(): the step kernels' stream
        self.stream_e = None   #  and the first engine's)


class ShardedMatcher:
    """A filter-sharded table over the ranks of a process group (two engines per rank).

    ``match_fn(engine, local_topics_bytes, local_topic_offsets) -> (counts int64 (n,), ids int32)``
    does the per-shard match on engine 0 (A) or 1 (B); the default is this rank's two HIP
    engines (device tensors).  Tests inject the oracle to check the distribution logic over gloo
    on CPU."""

    def __init__(self, filters: Tuple[np.ndarray, np.ndarray], group=None, device: Optional[torch.device] = None,
                 mode: int = 0, match_fn: Optional[Callable] = None, max_piece_pm: int = MAX_PIECE_PM,
                 engines: Optional[list] = None, rank_world: Optional[Tuple[int, int]] = None,
                 plan: Optional[np.ndarray] = None, local_ids: Optional[list] = None, p_space: str = "auto"):
        """``engines``: this rank's engines already built ([A, B, AB], each holding exactly the
        filters shard_local_ids names for it, reporting global ids; A and B may be None at world
        1, where every request is an AB request); they are adopted, not copied (e.g. a table
        held whole on one GPU is engine AB at world 1, tests/test_gpu_c100m.py).
        ``rank_world``: (rank, world) of a rank with no process group (``EmulatedWorld``: G
        ranks in one process); ``plan`` / ``local_ids``: the plan and this rank's ids when the
        caller computed them already (both are functions of the filters and the world).
        ``p_space``: the plan's space-P layout (``shard_plan``)."""
        self.group = group
        if rank_world is not None:
            self.rank, self.world = rank_world
        else:
            self.rank = dist.get_rank(group)
            self.world = dist.get_world_size(group)
        self.device = device or (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
                                 else torch.device("cpu"))
        self.mode = mode
        self.plan = shard_plan(filters, self.world, max_piece_pm, p_space) if plan is None else plan
        self.plan_dev = (torch.from_numpy(self.plan.view(np.int32).copy()).to(self.device)
                         if self.device.type == "cuda" and len(self.plan) else None)
        self.local_ids = (shard_local_ids(filters, self.rank, self.world, self.plan) if local_ids is None
                          else local_ids)
        self.last_exchange_out = [None, None]
        self.engines = []
        self.last_local_topics = 0
        self.last_slot_topics = [0, 0, 0]
        if engines is not None:
            assert match_fn is None and len(engines) == SHARD_ENGINES
            assert (self.world > 1 and not plan_p_replicated(self.plan)) or engines[2] is not None
            self.engines = list(engines)
            match_fn = self._engine_match
        elif match_fn is not None:  # (tests: a per-slot match function over host memory)
            assert self.device.type != "cuda", "an injected match_fn runs the step's host mode (CPU device)"
            self.engines = [_HostEngine(match_fn, e) for e in range(SHARD_ENGINES)]
            match_fn = self._engine_match
        else:
            from .engine import Engine
            from .workloads import take
            one_request = self.world == 1 or plan_p_replicated(self.plan)
            for slot, gids in enumerate(self.local_ids):
                if one_request and slot < 2:  # no request ever names A or B alone
                    self.engines.append(None)
                    continue
                e = Engine(self.device.index if self.device.type == "cuda" else -1)
                if len(gids):
                    e.insert_packed_ext(*take(filters, gids), gids)
                e.commit()
                self.engines.append(e)
            match_fn = self._engine_match
        self.match_fn = match_fn
        # the device step (emqx_shard_step_*) when this rank's own HIP engines do the matching;
        # an injected match_fn (tests on CPU over gloo) takes the tensor path below
        # a lane = the resources of one step in flight (step object, buffers, streams);
        # match_stream keeps two steps in flight on two lanes.  A CPU device runs the step's host
        # mode (the same protocol and chunk formats; the CPU tests over gloo)
        self._lanes = [_Lane(_DeviceStep(self.device, self.world, self.plan))]
        self._cuda = self.device.type == "cuda"
        self._lane = self._lanes[0]
        if self._cuda:  # the lanes' streams made together, so they land on different hardware queues
            for i in range(max(2, stream_depth())):
                ln = self._lane_n(i)
                ln.stream = torch.cuda.Stream(device=self.device)
        self._caps = [1 << 20] * SHARD_ENGINES
        self._ids_floor = 1 << 16  # (an engine call's id buffer is never smaller; tests lower it)
        self._fixed = None        # the fixed form's agreed capacities (_learn_fixed)
        self._last_sizes = None   # the last classic step's sizes (what _learn_fixed learns from)
        self.last_fixed_redo = 0
        self.last_fixed_enqueue_ms = 0.0

    # (the step's resources are the current lane's)
    _step = property(lambda self: self._lane.step)
    _bufs = property(lambda self: self._lane.bufs)
    _stream = property(lambda self: self._lane.stream, lambda self, v: setattr(self._lane, "stream", v))
    _stream_b = property(lambda self: self._lane.stream_b, lambda self, v: setattr(self._lane, "stream_b", v))

    def _engine_stream(self, i: int):
        """The lane's stream for its (i + 2)-th engine call of a step, made when first needed: a
        process has few hardware queues (GPU_MAX_HW_QUEUES, 4 here) and streams share them in
        creation order, so an unused stream can put two lanes on one queue."""
        if self._stream_b is None:
            self._stream_b = []
        while len(self._stream_b) <= i:
            self._stream_b.append(torch.cuda.Stream(device=self.device))
        return self._stream_b[i]

    def _lane_n(self, k: int) -> "_Lane":
        while len(self._lanes) <= k:
            self._lanes.append(_Lane(_DeviceStep(self.device, self.world, self.plan)))
        return self._lanes[k]

    def close(self):
        """Frees the device steps (the engines stay with their owner)."""
        for ln in self._lanes:
            if ln.step is not None:
                ln.step.close()

    @property
    def n_local_filters(self) -> int:
        return int(len(self.local_ids[2]))

    def _engine_match(self, which: int, tb: torch.Tensor, to: torch.Tensor):
        d_off, d_ids = self._engine_csr(which, tb, to)
        return d_off[1:] - d_off[:-1], d_ids

    def _engine_csr(self, which: int, tb, to: torch.Tensor, n: Optional[int] = None):
        """Synchronous match on engine `which`, growing the id buffer to the exact need (tb: a
        byte tensor, or a device address)."""
        n = to.numel() - 1 if n is None else n
        tb_addr = tb if isinstance(tb, int) else tb.data_ptr()
        d_off = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        caps = getattr(self, "_caps", [1 << 20] * SHARD_ENGINES)
        cap = max(1 << 16, caps[which])
        stream = torch.cuda.current_stream(self.device).cuda_stream if self._cuda else None
        while True:
            d_ids = torch.empty(cap, dtype=torch.int32, device=self.device)
            try:
                m = self.engines[which].match_device(tb_addr, to.data_ptr(), n, d_off.data_ptr(),
                                                     d_ids.data_ptr(), cap, mode=self.mode, stream=stream)
                break
            except Exception as e:  # EMQX_EOVERFLOW: retry with the exact capacity
                need = getattr(e, "needed", None)
                if need is None:
                    raise
                cap = need + 1
        caps[which] = max(cap, caps[which])
        self._caps = caps
        return d_off, d_ids[:m]

    def match_all(self, topics: Tuple[torch.Tensor, torch.Tensor], fixed: Optional[bool] = None):
        """Every rank matches its own batch against the sharded table and gets its own CSR
        (offsets int64 (n+1,), ids int32) in batch order — the layout's weak-scaling use, one
        publishing node per rank.  The classic form has two host synchronisations per call (the
        split sizes of the requests and of the answers); once the fixed form's capacities are
        learnt (a ``match_stream`` call), the call runs the fixed form (``fixed``, default
        ``fixed_steps()``): one host read at its end, the flag and the CSR's length."""
        if fixed is None:
            fixed = self._fixed is not None and fixed_steps()
        if fixed:
            return self._match_stream_fixed([topics], 1)[0]
        return self._match_all_classic(topics)

    def _match_all_classic(self, topics: Tuple[torch.Tensor, torch.Tensor]):
        if not self._cuda:
            return self._match_all_device(topics)
        if self._step is not None:
            # on a stream of its own: the engines take a null stream handle for "their own
            # stream", so the step's kernels and the engine calls must share a real one
            caller = torch.cuda.current_stream(self.device)
            if self._stream is None:
                self._stream = torch.cuda.Stream(device=self.device)
            self._stream.wait_stream(caller)
            with torch.cuda.stream(self._stream):
                res = self._match_all_device(topics)
            caller.wait_stream(self._stream)
            for t in res:
                t.record_stream(caller)
            return res
        raise RuntimeError("no device step")

    def _pinned(self, name: str, n: int):
        """A reused page-locked int64 buffer the device writes directly (its host tensor and the
        device address it is mapped at): words the host reads after a stream sync, with no copy."""
        got = self._bufs.get("_pin_" + name)
        if not self._cuda and (got is None or got[0].numel() < n):  # (host mode: plain memory)
            t = torch.zeros(max(n, 16), dtype=torch.int64)
            got = (t, t.data_ptr())
            self._bufs["_pin_" + name] = got
        if got is None or got[0].numel() < n:
            t = torch.zeros(max(n, 16), dtype=torch.int64, pin_memory=True)
            d = ctypes.c_void_p()
            rc = _hip().hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(t.data_ptr()), 0)
            if rc != 0:
                raise RuntimeError(f"hipHostGetDevicePointer: {rc}")
            got = (t, d.value)
            self._bufs["_pin_" + name] = got
        return got

    def _to_host(self, *parts: torch.Tensor) -> np.ndarray:
        """The device tensors' values (int64) on the host: one copy into a reused pinned buffer
        and a wait for this stream (no allocation per call)."""
        k = sum(int(t.numel()) for t in parts)
        if not self._cuda:
            return torch.cat([t.reshape(-1) for t in parts]).numpy().astype(np.int64)
        hb = self._bufs.get("_host")
        if hb is None or hb.numel() < k:
            hb = torch.empty(max(k, 256), dtype=torch.int64, pin_memory=True)
            self._bufs["_host"] = hb
        dv = torch.cat([t.reshape(-1) for t in parts]) if len(parts) > 1 else parts[0].reshape(-1)
        hb[:k].copy_(dv, non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return hb[:k].numpy().copy()

    def _buf(self, name: str, n: int, dtype) -> torch.Tensor:
        """A reused device buffer of at least n elements (every use is ordered on one stream)."""
        b = self._bufs.get(name)
        if b is None or b.numel() < n:
            b = torch.empty(max(int(n * 1.25), 64), dtype=dtype, device=self.device)
            self._bufs[name] = b
        return b

    def _match_all_device(self, topics: Tuple[torch.Tensor, torch.Tensor]):
        """match_all on device kernels: the step (``_step_gen``) driven over this rank's process
        group, one collective per exchange point."""
        gen = self._step_gen(topics)
        try:
            op = next(gen)
            while True:
                op = gen.send(self._exchange(op))
        except StopIteration as stop:
            return stop.value

    def match_stream(self, batches: List[Tuple[torch.Tensor, torch.Tensor]], exchange: Optional[Callable] = None,
                     depth: Optional[int] = None, fixed: Optional[bool] = None):
        """match_all over a sequence of this rank's batches with ``depth`` steps in flight (device
        step only; default ``stream_depth()``), one lane each: step k + depth - 1's send runs
        while the earlier steps' engines walk, and its requests are exchanged, unpacked and handed
        to its engines before the host waits for step k's answers, so the device always has a walk
        queued while the host synchronises.  With two lanes, step k + 2's send queues on its lane
        behind step k's merge, which waits for step k + 1's walk to free the CUs; a third lane
        gives that merge and send a whole walk to run under.  Every rank runs the same schedule,
        so the collectives pair up.  ``exchange``: the exchange-point function (default
        ``_exchange``: the process group; ``EmulatedWorld`` passes a recorded one).  ``fixed``
        (default ``fixed_steps()`` over this rank's own process group): the fixed-capacity form
        (``_match_stream_fixed``), no host synchronisation between the steps.  Returns every
        batch's (offsets, ids)."""
        D = max(1, int(depth or stream_depth()))
        if fixed is None:
            fixed = exchange is None and fixed_steps()
        if fixed:
            return self._match_stream_fixed(batches, D, exchange)
        assert self._cuda, "match_stream keeps steps in flight on device streams"
        ex = exchange or self._exchange
        caller = torch.cuda.current_stream(self.device)
        lanes = [self._lane_n(i) for i in range(D)]
        for ln in lanes:
            if ln.stream is None:
                ln.stream = torch.cuda.Stream(device=self.device)
            ln.stream.wait_stream(caller)
        K = len(batches)
        gens, ops, res = {}, {}, [None] * K

        def on_lane(k, fn):
            self._lane = lanes[k % D]
            with torch.cuda.stream(self._lane.stream):
                return fn()

        def adv(k, value):
            def seg():
                try:
                    return next(gens[k]) if value is None else gens[k].send(value)
                except StopIteration as stop:
                    return ("done", stop.value)
            ops[k] = on_lane(k, seg)

        def start(k):  # the send
            gens[k] = self._step_gen(batches[k])
            adv(k, None)

        def to_answer(k):  # up to the answers' sizes: recv, engines, answer enqueued
            seen = 0
            while ops[k][0] != "done":
                if ops[k][0] in ("sizes", "local_sizes"):
                    seen += 1
                    if seen == 2:
                        return
                op = ops[k]
                adv(k, on_lane(k, lambda: ex(op)))

        def finish(k):  # the answers exchanged and merged
            while ops[k][0] != "done":
                op = ops[k]
                adv(k, on_lane(k, lambda: ex(op)))
            res[k] = ops.pop(k)[1]
            del gens[k]

        try:
            for k in range(min(K, D - 1)):  # the first D - 1 steps up to their answers
                start(k)
                to_answer(k)
            if K >= D:
                start(D - 1)
            for k in range(K):
                if k + D - 1 < K and D > 1:
                    to_answer(k + D - 1)
                finish(k)
                if k + D < K:
                    start(k + D)
        finally:
            self._lane = self._lanes[0]
        for ln in lanes:
            caller.wait_stream(ln.stream)
        for r in res:
            for t in r:
                t.record_stream(caller)
        return res

    def _match_stream_fixed(self, batches: List[Tuple[torch.Tensor, torch.Tensor]], D: int,
                            exchange: Optional[Callable] = None):
        """match_stream in the fixed-capacity form: every step enqueued on its lane (D lanes)
        with no host read — send, chunk exchange, recv, engines, answer, answer exchange, merge —
        then one synchronisation for all of them: each step's flag, and each CSR cut to its
        length.  A flagged step (some chunk, slot or engine over its capacity; the flag is the
        same on every rank) is redone in the classic form, which also teaches larger capacities.
        The first call learns the capacities from a classic step (its batch's result).  Runs in
        host mode too (CPU device: the steps one after another).  ``exchange`` (EmulatedWorld's
        replay): capacities learnt beforehand, and a flagged step is an error (no classic redo)."""
        K = len(batches)
        res = [None] * K
        if not K:
            return res
        ex = exchange or self._exchange
        first = 0
        if self._fixed is None:
            assert exchange is None, "the fixed form over a replayed exchange needs learnt capacities"
            res[0] = self._match_all_classic(batches[0])
            self._learn_fixed()
            first = 1
        cuda = self._cuda
        flags = torch.zeros(K, dtype=torch.int64, pin_memory=cuda)
        if cuda:
            d = ctypes.c_void_p()
            rc = _hip().hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(flags.data_ptr()), 0)
            if rc != 0:
                raise RuntimeError(f"hipHostGetDevicePointer: {rc}")
            faddr = d.value
            caller = torch.cuda.current_stream(self.device)
        else:
            faddr = flags.data_ptr()
        lanes = [self._lane_n(i) for i in range(D)]
        prio = cuda and step_priority()
        if cuda:
            for ln in lanes:
                if ln.stream is None:
                    ln.stream = torch.cuda.Stream(device=self.device)
                if prio and ln.stream_hi is None:
                    # the step's own kernels on a high-priority stream, the engines on the lane's
                    # normal ones: a send gets CUs as the other lanes' walks drain
                    ln.stream_hi = torch.cuda.Stream(device=self.device, priority=-1)
                    ln.stream_e = torch.cuda.Stream(device=self.device)
                ln.stream.wait_stream(caller)
                if prio:
                    ln.stream_hi.wait_stream(caller)
        t_enq = time.perf_counter()
        try:
            for k in range(first, K):
                self._lane = lanes[k % D]
                ctx = (torch.cuda.stream(self._lane.stream_hi if prio else self._lane.stream) if cuda
                       else contextlib.nullcontext())
                with ctx:
                    gen = self._step_gen_fixed(batches[k], faddr + 8 * k)
                    try:
                        op = next(gen)
                        while True:
                            op = gen.send(ex(op))
                    except StopIteration as stop:
                        res[k] = stop.value
        finally:
            self._lane = self._lanes[0]
        # (host time to enqueue the steps, per step: the stream is host-bound when it nears the
        # step time)
        self.last_fixed_enqueue_ms = 1e3 * (time.perf_counter() - t_enq) / max(K - first, 1)
        if cuda:
            for ln in lanes:
                caller.wait_stream(ln.stream)
                if prio:
                    caller.wait_stream(ln.stream_hi)
            caller.synchronize()
        ends = torch.stack([res[k][0][-1] for k in range(first, K)]).cpu().tolist() if K > first else []
        fl = flags.tolist()
        self.last_fixed_redo = 0
        for k in range(first, K):
            if fl[k]:
                if exchange is not None:
                    raise RuntimeError(f"fixed-capacity step {k} flagged ({fl[k]}) over a replayed exchange")
                res[k] = self._match_all_classic(batches[k])
                self._learn_fixed()
                self.last_fixed_redo += 1
            else:
                res[k] = (res[k][0], res[k][1][: int(ends[k - first])])
        if cuda:
            for r in res:
                for t in r:
                    t.record_stream(caller)
        return res

    def _exchange(self, op):
        """One exchange point of ``_step_gen`` over the process group:
        ("local_sizes", pinned words, W) at world 1: the stream synchronised, the words read;
        ("sizes", words, W): an all-to-all of W int64 words per rank, both sides read on the host
        (a host sync) -> (words sent, words received, the received words as a numpy array);
        ("chunks", buf, out sizes, in sizes, name): chunk r of buf to rank r -> the device address
        of every source's chunk for this rank (``_exchange_chunks``)."""
        if op[0] == "local_sizes":  # world 1: words the device wrote into mapped pinned memory
            _, words, W = op
            if self._cuda:
                torch.cuda.current_stream(self.device).synchronize()
            lst = words[: W * self.world].tolist()
            return lst, lst, words
        if op[0] == "fixed":  # equal splits of c elements: chunk r of buf to rank r
            _, buf, c, name = op
            G, es = self.world, buf.element_size()
            recv = self._buf("f" + name, G * c, buf.dtype)
            _a2a(recv[: G * c], buf[: G * c], [c] * G, [c] * G, self.group)
            return [buf.data_ptr() + es * c * r if r == self.rank else recv.data_ptr() + es * c * r for r in range(G)]
        if op[0] == "sizes":
            _, words, W = op
            G = self.world
            words_in = torch.empty_like(words)
            _a2a(words_in, words, [W] * G, [W] * G, self.group)
            h = self._to_host(words, words_in)  # host sync
            mi = np.ascontiguousarray(h[W * G: 2 * W * G], dtype=np.int64)
            return h[: W * G].tolist(), mi.tolist(), mi
        _, buf, out_sz, in_sz, name = op
        return _exchange_chunks(buf, out_sz, in_sz, lambda k: self._buf(name, k + 16, buf.dtype), self.group,
                                self.rank)

    def _step_gen(self, topics: Tuple[torch.Tensor, torch.Tensor]):  # noqa: C901
        """One step of match_all on device kernels (emqx_shard_step_*, shard_step.hip), as a
        generator that yields at each exchange point and is sent its result (``_exchange`` over a
        process group; ``EmulatedWorld`` for G ranks in one process): route + fold + stable sort
        + pack the requests, one exchange of sizes and one of chunks, unpack into the engine
        slots' batches, the engines matched asynchronously into learnt capacities, the answers
        packed per source, one exchange of sizes and one of answers, merged back in batch order.
        The host only reads the split sizes (two syncs; at world 1 from mapped pinned words, no
        exchange).  Runs on the current stream; returns (offsets int64 (n+1,), ids int32)."""
        from . import _lib
        L = _lib.lib()
        E = SHARD_ENGINES
        dev, G = self.device, self.world
        st = self._step.h
        mark = _host_marks() if _SHARD_PROF else (lambda k: None)
        mark(0)
        stream = torch.cuda.current_stream(dev).cuda_stream if self._cuda else None
        P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        PA = lambda ts: (ctypes.c_void_p * E)(*[None if t is None else t.data_ptr() for t in ts])  # noqa: E731
        S = ctypes.c_void_p(stream)
        MW = 1 + 2 * E  # meta words per destination
        tb, to = topics
        tb = tb.to(dev)
        to = to.to(dev).to(torch.int64)
        if tb.numel() == 0:
            tb = torch.zeros(16, dtype=torch.uint8, device=dev)
        n = to.numel() - 1
        # 1. requests -> one chunk per destination
        cap = int(L.emqx_shard_send_cap(n, tb.numel(), G))
        send = self._buf("send", cap, torch.uint8)
        # (world 1: the sizes go straight into mapped pinned memory, read after the stream sync)
        hmeta, dmeta = self._pinned("meta", MW * G) if G == 1 else (None, None)
        meta = None if G == 1 else torch.empty(MW * G, dtype=torch.int64, device=dev)
        _lib.check(L.emqx_shard_step_send(st, P(tb), P(to), n, P(send), send.numel(),
                                          ctypes.c_void_p(dmeta) if G == 1 else P(meta), S), "emqx_shard_step_send")
        cur = torch.cuda.current_stream(dev) if self._cuda else None
        mark(1)
        # (the split sizes as Python ints: this bookkeeping sits between the host sync and the
        # next launch, on the step's critical path, where numpy calls on a few words cost more
        # than the arithmetic)
        # host sync 1 (world 1: the stream, then the mapped words; recv reads them on the host)
        mo_l, mi_l, mi = yield (("local_sizes", hmeta, MW) if G == 1 else ("sizes", meta, MW))
        mi_ptr = mi.data_ptr() if G == 1 else mi.ctypes.data
        mark(2)
        out_b = mo_l[0::MW]
        in_b = mi_l[0::MW]
        if min(out_b) < 0 or min(in_b) < 0:
            raise RuntimeError("emqx_shard_step_send: chunks over the send buffer")
        self.last_exchange_out = [[x for x in out_b], None]
        chunks = [send.data_ptr()] if G == 1 else (yield ("chunks", send, out_b, in_b, "recv"))
        NQ = [sum(mi_l[1 + e::MW]) for e in range(E)]
        self._last_sizes = {"chunk": max(out_b), "q": NQ, "y": [sum(mi_l[1 + E + e::MW]) for e in range(E)]}
        # a slot fed by one source only is matched in place in that source's chunk (recv
        # replaces its byte buffer's address); the others are gathered into these buffers
        one = [sum(1 for x in mi_l[1 + e::MW] if x) <= 1 for e in range(E)]
        qbytes = [None if one[e] else self._buf(f"q_bytes{e}", sum(mi_l[1 + E + e::MW]) + 16, torch.uint8)
                  for e in range(E)]
        qoff = [self._buf(f"q_off{e}", NQ[e] + 1, torch.int64) for e in range(E)]
        qb = PA(qbytes)
        _lib.check(L.emqx_shard_step_recv(st, (ctypes.c_void_p * G)(*chunks), ctypes.c_void_p(mi_ptr), qb, PA(qoff),
                                          S), "emqx_shard_step_recv")
        mark(3)
        qaddr = [qb[e] for e in range(E)]
        self.last_local_topics = sum(NQ)
        self.last_slot_topics = NQ
        # 2. the engines, asynchronously, into learnt capacities; each on a stream of its own
        # after the first, so the walks overlap
        batches = [(qaddr[e], qoff[e], NQ[e]) for e in range(E)]
        outs = []
        hsumm, dsumm = self._pinned("summary", 8 * E)  # written by each engine call that runs

        used = []
        for e, (eb, eo, ne) in enumerate(batches):
            ro = self._buf(f"off{e}", ne + 1, torch.int64)
            if not ne:  # (a slot no source asked: the answer kernel reads nothing of it)
                outs.append([ro, self._buf(f"ids{e}", 16, torch.int32)])
                continue
            cap_e = max(self._caps[e], self._ids_floor)
            ri = self._buf(f"ids{e}", cap_e, torch.int32)
            es = cur if not used or not self._cuda else self._engine_stream(len(used) - 1)
            if es is not cur:
                es.wait_stream(cur)
            used.append(es)
            self.engines[e].match_device_async(eb, eo.data_ptr(), ne, ro.data_ptr(), ri.data_ptr(),
                                               ri.numel(), dsumm + 64 * e, mode=self.mode,
                                               stream=es.cuda_stream if es is not None else None)
            outs.append([ro, ri])
        for es in used:
            if es is not cur:
                cur.wait_stream(es)
        mark(4)
        # 3. answers, one chunk per source; a call that did not complete is redone before the
        # exchange (every rank learns every rank's flag from the size exchange)
        redo = False
        while True:
            ans = self._buf("answer", 8 * G + sum(NQ) + sum(o[1].numel() for o in outs), torch.int32)
            # per source: words, redo, ids (world 1: into mapped pinned memory)
            hans, dans = self._pinned("ans_meta", 3 * G) if G == 1 else (None, None)
            ans_meta = None if G == 1 else torch.empty(3 * G, dtype=torch.int64, device=dev)
            sp = None if redo else (ctypes.c_void_p * E)(*[dsumm + 64 * e if NQ[e] else None for e in range(E)])
            # (this rank's own answers stay in the engines' outputs: the merge reads them from there)
            _lib.check(L.emqx_shard_step_answer(st, PA([o[0] for o in outs]), PA([o[1] for o in outs]), sp, self.rank,
                                                P(ans), ctypes.c_void_p(dans) if G == 1 else P(ans_meta), S),
                       "emqx_shard_step_answer")
            mark(5)
            # host sync 2 (world 1: the mapped words; merge reads them on the host)
            am_l, ai_l, ai = yield (("local_sizes", hans, 3) if G == 1 else ("sizes", ans_meta, 3))
            ai_ptr = ai.data_ptr() if G == 1 else ai.ctypes.data
            mark(6)
            sm = hsumm[: 8 * E].tolist()
            if not redo:
                for e in range(E):  # learn the id capacities from this call's totals
                    if NQ[e] and sm[8 * e] == 0:
                        self._caps[e] = max(self._caps[e], int(sm[8 * e + 1] * 1.25) + 4096)
            if not any(ai_l[1::3]):
                break
            if am_l[1]:  # this rank's call did not complete: redo it synchronously, exact size
                for e, (eb, eo, ne) in enumerate(batches):
                    if ne and sm[8 * e]:
                        outs[e] = list(self._engine_csr(e, eb, eo[: ne + 1], n=ne))
                        self._caps[e] = max(self._caps[e], int(outs[e][1].numel() * 1.25) + 4096)
            redo = True
        # 4. answers back to their sources, merged per topic in batch order
        out_w, in_w = am_l[0::3], ai_l[0::3]
        self._last_sizes["answer"] = max(out_w)
        self.last_exchange_out[1] = [4 * x for x in out_w]
        back = [ans.data_ptr()] if G == 1 else (yield ("chunks", ans, out_w, in_w, "back"))
        total = sum(ai_l[2::3])
        out_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        out_ids = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
        _lib.check(L.emqx_shard_step_merge(st, (ctypes.c_void_p * G)(*back), ctypes.c_void_p(ai_ptr), P(out_off),
                                           P(out_ids), S), "emqx_shard_step_merge")
        mark(7)
        return out_off, out_ids[:total]

    def _allreduce_max(self, vals: List[int]) -> List[int]:
        if self.world == 1 or self.group is None and not dist.is_initialized():
            return list(vals)
        on_dev = self._cuda and dist.get_backend(self.group) != "gloo"
        t = torch.tensor(vals, dtype=torch.int64, device=self.device if on_dev else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return [int(x) for x in t.cpu().tolist()]

    def _learn_fixed(self):
        """The fixed form's capacities from the last classic step's sizes (every rank at the same
        point: the chunk capacities are agreed by an all-reduce of their maxima), never shrinking:
        request chunks, answer chunks (u32 words), per slot requests and bytes (this rank's)."""
        ls = self._last_sizes
        old = self._fixed or {"chunk": 0, "answer": 0, "q": [0] * SHARD_ENGINES, "y": [0] * SHARD_ENGINES}
        # (margins: a rank's requests and chunks vary by ~sqrt between batches of one stream, so
        # 1/128 + 2048 requests covers them; the engines walk every padding topic, so a wide
        # margin costs walk time, and a step over it only costs its classic redo)
        c1 = (ls["chunk"] + ls["chunk"] // 64 + 4096 + 15) // 16 * 16
        c2 = ls["answer"] + ls["answer"] // 32 + 16384
        c1, c2 = self._allreduce_max([max(c1, old["chunk"]), max(c2, old["answer"])])
        q = [0 if self.engines[e] is None else max(old["q"][e], x + x // 128 + 2048) for e, x in enumerate(ls["q"])]
        y = [0 if self.engines[e] is None else max(old["y"][e], x + x // 64 + 65536) for e, x in enumerate(ls["y"])]
        self._fixed = {"chunk": c1, "answer": c2, "q": q, "y": y}

    def _step_gen_fixed(self, topics: Tuple[torch.Tensor, torch.Tensor], flag_addr: int):
        """One step in the fixed-capacity form (``emqx_shard_step_*_fixed``): the same kernels
        with chunks at the agreed capacities (``_learn_fixed``), so the only exchange points are
        the two chunk exchanges (equal splits; none at world 1) and nothing is read on the host.
        The engines match each slot's fixed-size batch (padding topics past its requests) into
        their learnt id capacities.  The step's flag (u32 at ``flag_addr``: 0 = valid) is
        written by the merge; a flagged step is redone by the caller.  Returns (offsets int64
        (n+1,), ids int32 with room to spare: the topics' ids end at offsets[n])."""
        from . import _lib
        L = _lib.lib()
        E, fx = SHARD_ENGINES, self._fixed
        dev, G = self.device, self.world
        st = self._step.h
        stream = torch.cuda.current_stream(dev).cuda_stream if self._cuda else None
        S = ctypes.c_void_p(stream)
        P = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        PA = lambda ts: (ctypes.c_void_p * E)(*[None if t is None else t.data_ptr() for t in ts])  # noqa: E731
        tb, to = topics
        tb = tb.to(dev)
        to = to.to(dev).to(torch.int64)
        if tb.numel() == 0:
            tb = torch.zeros(16, dtype=torch.uint8, device=dev)
        n = to.numel() - 1
        c1, c2, capq, capy = fx["chunk"], fx["answer"], list(fx["q"]), fx["y"]
        if G == 1 and self.engines[0] is None and self.engines[1] is None:
            capq[2] = n  # (world 1, one request a topic: at most n requests, so no padding)
        send = self._buf("fsend", G * c1, torch.uint8)
        meta = self._buf("fmeta", (1 + 2 * E) * G, torch.int64)
        _lib.check(L.emqx_shard_step_send_fixed(st, P(tb), P(to), n, P(send), c1, P(meta), S),
                   "emqx_shard_step_send_fixed")
        chunks = [send.data_ptr()] if G == 1 else (yield ("fixed", send, c1, "recv"))
        in_place = G == 1  # (world 1: every slot matched where send packed it)
        qbytes = [None] * E if in_place else [self._buf(f"q_bytes{e}", capy[e] + 16, torch.uint8) for e in range(E)]
        qoff = [self._buf(f"q_off{e}", capq[e] + 1, torch.int64) for e in range(E)]
        _lib.check(L.emqx_shard_step_recv_fixed(st, (ctypes.c_void_p * G)(*chunks), (ctypes.c_uint64 * E)(*capq),
                                                (ctypes.c_uint64 * E)(*capy), None if in_place else PA(qbytes),
                                                PA(qoff), S), "emqx_shard_step_recv_fixed")
        hsumm, dsumm = self._pinned("summary", 8 * E)
        cur = torch.cuda.current_stream(dev) if self._cuda else None
        outs, used, room = [], [], 0
        for e in range(E):
            ro = self._buf(f"off{e}", capq[e] + 1, torch.int64)
            if not capq[e]:
                outs.append([ro, self._buf(f"ids{e}", 16, torch.int32)])
                continue
            ri = self._buf(f"ids{e}", max(self._caps[e], self._ids_floor), torch.int32)
            room += ri.numel()
            es = cur if not used or not self._cuda else self._engine_stream(len(used) - 1)
            if self._cuda and self._lane.stream_e is not None and cur is not None and cur == self._lane.stream_hi:
                es = self._lane.stream_e if not used else self._engine_stream(len(used) - 1)
            if es is not cur:
                es.wait_stream(cur)
            used.append(es)
            eb = send.data_ptr() if in_place else qbytes[e].data_ptr()
            self.engines[e].match_device_async(eb, qoff[e].data_ptr(), capq[e], ro.data_ptr(), ri.data_ptr(),
                                               ri.numel(), dsumm + 64 * e, mode=self.mode,
                                               stream=es.cuda_stream if es is not None else None)
            outs.append([ro, ri])
        for es in used:
            if es is not cur:
                cur.wait_stream(es)
        ans = self._buf("fanswer", G * c2, torch.int32)
        sp = (ctypes.c_void_p * E)(*[dsumm + 64 * e if capq[e] else None for e in range(E)])
        _lib.check(L.emqx_shard_step_answer_fixed(st, PA([o[0] for o in outs]), PA([o[1] for o in outs]), sp,
                                                  self.rank, P(ans), c2, S), "emqx_shard_step_answer_fixed")
        back = [ans.data_ptr()] if G == 1 else (yield ("fixed", ans, c2, "back"))
        out_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        out_ids = torch.empty(G * c2 + room + 16, dtype=torch.int32, device=dev)
        _lib.check(L.emqx_shard_step_merge_fixed(st, (ctypes.c_void_p * G)(*back), P(out_off), P(out_ids),
                                                 ctypes.c_void_p(flag_addr), S), "emqx_shard_step_merge_fixed")
        return out_off, out_ids

    def match(self, topics: Optional[Tuple[torch.Tensor, torch.Tensor]], src: int = 0, dst: int = 0):
        """Match a batch held by rank ``src``; rank ``dst`` gets the CSR in batch order
        (offsets int64 (n+1,), ids int32), the other ranks None.  Every rank takes part (the
        others with empty batches)."""
        dev = self.device
        empty = (torch.zeros(0, dtype=torch.uint8, device=dev), torch.zeros(1, dtype=torch.int64, device=dev))
        res = self.match_all(topics if self.rank == src else empty)
        if src == dst:
            return res if self.rank == dst else None
        if self.rank == src:
            off, ids = res
            _p2p(torch.tensor([off.numel(), ids.numel()], dtype=torch.int64), dst, True, self.group)
            _p2p(off, dst, True, self.group)
            _p2p(ids, dst, True, self.group)
            return None
        if self.rank == dst:
            sz = _p2p(None, src, False, self.group, like=torch.zeros(2, dtype=torch.int64))
            off = _p2p(None, src, False, self.group, like=torch.empty(int(sz[0]), dtype=torch.int64, device=dev))
            ids = _p2p(None, src, False, self.group, like=torch.empty(int(sz[1]), dtype=torch.int32, device=dev))
            return off, ids
        return None


class EmulatedWorld:
    """G ranks of the filter-sharded layout in ONE process on one GPU, for measuring one rank's
    step at world G without G GPUs.  Every rank is a real ``ShardedMatcher`` with its
    own engines (A / B / AB over exactly the filters the G-way plan gives it), its own device step
    (emqx_shard_step_* built for world G) and its own buffers; every rank's step is the product's
    ``_step_gen``.  Only the exchanges differ: a chunk for rank r is read where its source packed
    it (the device address any all-to-all would have delivered it to is just another buffer on
    the same GPU), so a step costs the ranks' own work, run one rank at a time, and the
    exchanges' bytes are counted per (source, destination) pair for a projection over xGMI links
    instead of being moved.

    ``step(batches)`` runs one step of every rank (rank s publishing batches[s]) and returns every
    rank's CSR.  With ``timing``: "wall" times each rank's segments between exchange points on
    the host (device synchronised before and after: launches, host bookkeeping and kernels);
    "gpu" times them with HIP events on the rank's stream behind a spin kernel, so the launches
    are enqueued before the first kernel starts (kernel time only)."""

    PHASES = ("send", "sizes1", "recv_match_answer", "sizes2", "merge")
    PHASES_1 = ("send", "recv_match_answer", "merge")  # world 1: no exchange, two host syncs
    PHASES_FIXED = ("send", "recv_match_answer", "merge")  # the fixed form: the two chunk exchanges
    PHASES_FIXED_1 = ("step",)  # the fixed form at world 1: no exchange point at all

    def __init__(self, filters: Tuple[np.ndarray, np.ndarray], world: int, device: torch.device, mode: int = 0,
                 max_piece_pm: int = MAX_PIECE_PM, on_rank: Optional[Callable] = None, p_space: str = "auto"):
        self.world = world
        self.device = device
        self.plan = shard_plan(filters, world, max_piece_pm, p_space)
        self.p_replicated = plan_p_replicated(self.plan)
        first, span, eng = shard_place(filters, world, self.plan)
        first = first.astype(np.int64)
        self.matchers: List[ShardedMatcher] = []
        self.filters_per_rank = []
        for r in range(world):
            held = ((r - first) % world) < span
            ids = [np.nonzero(held & (eng == e))[0].astype(np.uint32) for e in (0, 1)] + [
                np.nonzero(held)[0].astype(np.uint32)]
            del held
            self.filters_per_rank.append([int(len(x)) for x in ids])
            self.matchers.append(ShardedMatcher(filters, device=device, mode=mode, rank_world=(r, world),
                                                plan=self.plan, local_ids=ids))
            if on_rank is not None:
                on_rank(r)
        self.bytes_out = np.zeros((2, world, world), dtype=np.int64)  # [requests, answers][src][dst]
        self.last_times = None
        self.recorded = [dict() for _ in range(world)]  # per rank: what its last step's exchanges gave it

    def close(self):
        for m in self.matchers:
            for e in m.engines:
                if e is not None:
                    e.close()
            m.close()
        self.matchers = []

    def learn_fixed(self):
        """The fixed form's capacities from the last (classic) ``step``: every rank's own, the
        chunk capacities agreed as their maxima (what the ranks' all-reduce would give)."""
        for m in self.matchers:
            m._learn_fixed()
        c1 = max(m._fixed["chunk"] for m in self.matchers)
        c2 = max(m._fixed["answer"] for m in self.matchers)
        for m in self.matchers:
            m._fixed["chunk"], m._fixed["answer"] = c1, c2

    def rank_stream(self, r: int, batch: Tuple[torch.Tensor, torch.Tensor], steps: int, fixed: bool = False):
        """Rank r alone running ``steps`` steps of its batch with two in flight
        (``ShardedMatcher.match_stream``), the other ranks' side replayed from the last ``step``
        (which must have used the same batches): their size words and their chunks for r, which
        stay where they were packed since no other rank runs; r's own chunks are its lane's.
        This is rank r's pipelined step — the device work it does per step at world G, with the
        collectives themselves left to the projection.  Returns (ms per step, the results)."""
        m = self.matchers[r]
        rec = self.recorded[r]
        if m._cuda:
            # fresh lane streams, made together: in one process the G ranks' streams share the
            # process's few hardware queues, and a rank of a real run has them to itself
            torch.cuda.synchronize(self.device)
            for i in range(max(2, stream_depth())):
                m._lane_n(i).stream = torch.cuda.Stream(device=self.device)

        def replay(op):
            if op[0] == "fixed":
                addrs = list(rec[("fixed", op[3])])
                addrs[r] = op[1].data_ptr() + op[1].element_size() * op[2] * r
                return addrs
            if op[0] == "local_sizes":
                return m._exchange(op)
            if op[0] == "sizes":
                return rec[("sizes", op[2])]
            addrs = list(rec[("chunks", op[4])])
            own = np.concatenate([[0], np.cumsum(op[2])]).astype(np.int64)
            addrs[r] = op[1].data_ptr() + op[1].element_size() * int(own[r])
            return addrs

        m.match_stream([batch] * max(2, stream_depth()), exchange=replay, fixed=fixed)  # (every lane's buffers)
        torch.cuda.synchronize(self.device)
        t0 = time.perf_counter()
        res = m.match_stream([batch] * steps, exchange=replay, fixed=fixed)
        torch.cuda.synchronize(self.device)
        return 1e3 * (time.perf_counter() - t0) / max(steps, 1), res

    def _run(self, r: int, gen, value, timing: Optional[str]):
        """Advances rank r's step to its next exchange point (or its end) on the rank's stream;
        returns (op or ("done", result), seconds or ms, or None)."""
        m = self.matchers[r]
        if m._stream is None:
            m._stream = torch.cuda.Stream(device=self.device)
        t = None
        with torch.cuda.stream(m._stream):
            if timing == "gpu":
                torch.cuda.synchronize(self.device)
                torch.cuda._sleep(2_000_000)  # (launches queue up behind it: the events time kernels)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(m._stream)
            elif timing == "wall":
                torch.cuda.synchronize(self.device)
                t0 = time.perf_counter()
            try:
                op = next(gen) if value is None else gen.send(value)
            except StopIteration as stop:
                op = ("done", stop.value)
            if timing == "gpu":
                e1.record(m._stream)
                e1.synchronize()
                t = e0.elapsed_time(e1)
            elif timing == "wall":
                torch.cuda.synchronize(self.device)
                t = 1e3 * (time.perf_counter() - t0)
        return op, t

    def step(self, batches: List[Tuple[torch.Tensor, torch.Tensor]], timing: Optional[str] = None,
             fixed: bool = False):
        """One step of every rank (see the class); ``fixed``: the fixed-capacity form (after
        ``learn_fixed``; a flagged step is an error here)."""
        G = self.world
        assert len(batches) == G
        flags = None
        if fixed:
            flags = torch.zeros(G, dtype=torch.int64, pin_memory=True)
            d = ctypes.c_void_p()
            if _hip().hipHostGetDevicePointer(ctypes.byref(d), ctypes.c_void_p(flags.data_ptr()), 0) != 0:
                raise RuntimeError("hipHostGetDevicePointer")
            gens = [m._step_gen_fixed(b, d.value + 8 * r) for r, (m, b) in enumerate(zip(self.matchers, batches))]
        else:
            gens = [m._step_gen(b) for m, b in zip(self.matchers, batches)]
        ops, times = [None] * G, [[] for _ in range(G)]
        vals = [None] * G
        rounds = 0
        chunk_round = 0
        while True:
            for r in range(G):
                ops[r], t = self._run(r, gens[r], vals[r], timing)
                times[r].append(t)
            kinds = {op[0] for op in ops}
            if len(kinds) != 1:
                raise RuntimeError(f"ranks out of step at exchange {rounds}: {kinds}")
            kind = kinds.pop()
            rounds += 1
            if kind == "done":
                break
            torch.cuda.synchronize(self.device)
            if kind == "local_sizes":  # world 1
                vals = [self.matchers[r]._exchange(ops[r]) for r in range(G)]
            elif kind == "sizes":
                W = ops[0][2]
                words = [op[1].cpu().numpy().astype(np.int64) for op in ops]
                for r in range(G):
                    mi = np.ascontiguousarray(np.concatenate([words[s][W * r: W * (r + 1)] for s in range(G)]))
                    vals[r] = (words[r].tolist(), mi.tolist(), mi)
                    self.recorded[r][("sizes", W)] = vals[r]
            elif kind == "fixed":  # chunk r of source s at s's buffer + r * the capacity
                c, es = ops[0][2], ops[0][1].element_size()
                for r in range(G):
                    vals[r] = [ops[s][1].data_ptr() + es * c * r for s in range(G)]
                    self.recorded[r][("fixed", ops[r][3])] = vals[r]
                self.bytes_out[min(chunk_round, 1)] = es * c
                chunk_round += 1
            elif kind == "chunks":
                # chunk r of source s lies at s's buffer + the prefix of s's sizes before r
                offs = [np.concatenate([[0], np.cumsum(op[2])]).astype(np.int64) for op in ops]
                for r in range(G):
                    vals[r] = [ops[s][1].data_ptr() + ops[s][1].element_size() * int(offs[s][r]) for s in range(G)]
                    self.recorded[r][("chunks", ops[r][4])] = vals[r]
                k = min(chunk_round, 1)
                for s in range(G):
                    self.bytes_out[k, s, :] = np.asarray(ops[s][2], dtype=np.int64) * ops[s][1].element_size()
                chunk_round += 1
            else:
                raise RuntimeError(f"unknown exchange {kind}")
        self.last_times = times if timing else None
        out = [op[1] for op in ops]
        if fixed:
            torch.cuda.synchronize(self.device)
            if any(flags.tolist()):
                raise RuntimeError(f"fixed-capacity step flagged: {flags.tolist()}")
            out = [(o, i[: int(o[-1].item())]) for o, i in out]
        return out
