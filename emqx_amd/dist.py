"""Multi-GPU route lookup: one process per GPU, torch.distributed (RCCL over xGMI on MI355X).

SURVEY §8(e).  Two layouts:

* **Replicated** (tables that fit one GPU — 10M filters take a few GB of 288 GB): every rank
  holds the whole table and matches its own slice of the topic stream.  Pure data
  parallelism, no collective on the data path (``split_topics``).  The reference does the same
  across a cluster: every node holds a full mria copy of the route table
  (apps/emqx/src/emqx_router.erl:135, apps/emqx/src/emqx_trie.erl:72-77).

* **Filter-sharded** (``ShardedMatcher``): a filter lives on the rank its first SHARD_LEVELS
  (2) levels hash to (``emqx_shard_owner``); a filter with ``+`` or ``#`` among those levels, or
  with fewer levels, can match topics of several keys and is replicated on every rank (about a
  tenth of config B's filters).  Two key levels instead of one keep a Zipf-hot first level
  (a third of the topics on config C's generator) from landing on one rank.  So every filter that can match a topic
  lives on the topic's owner rank, and each topic is matched on exactly one rank: a batch is
  partitioned by owner on its source rank, the parts are exchanged with one all-to-all, every
  rank matches only its part against its shard, and the per-topic results go back to the
  destination with a second all-to-all, where they are put back in batch order.  Per-rank walk
  work falls as 1/G; the collectives move each topic and each result once.
  Each rank builds its shard's trie with GLOBAL filter ids (``emqx_insert_filters_ext``).
"""

from __future__ import annotations

import ctypes
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


class ShardedMatcher:
    """A filter-sharded table over the ranks of a process group.

    ``match_fn(local_topics_bytes, local_topic_offsets) -> (counts int64 (n,), ids int32)`` does
    the per-shard match; the default is this rank's HIP engine (device tensors).  Tests inject
    the oracle to check the distribution logic over gloo on CPU."""

    def __init__(self, filters: Tuple[np.ndarray, np.ndarray], group=None, device: Optional[torch.device] = None,
                 mode: int = 0, match_fn: Optional[Callable] = None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.device = device or (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
                                 else torch.device("cpu"))
        self.mode = mode
        self.local_filters, self.global_ids = shard_filters(filters, self.rank, self.world)
        self.engine = None
        self.last_local_topics = 0
        if match_fn is None:
            from .engine import Engine
            self.engine = Engine(self.device.index if self.device.type == "cuda" else -1)
            self.engine.insert_packed_ext(*self.local_filters, self.global_ids)
            self.engine.commit()
            match_fn = self._engine_match
        self.match_fn = match_fn

    def _engine_match(self, tb: torch.Tensor, to: torch.Tensor):
        n = to.numel() - 1
        d_off = torch.empty(n + 1, dtype=torch.int64, device=self.device)
        cap = max(1 << 16, getattr(self, "_cap", 1 << 20))
        while True:
            d_ids = torch.empty(cap, dtype=torch.int32, device=self.device)
            try:
                m = self.engine.match_device(tb.data_ptr(), to.data_ptr(), n, d_off.data_ptr(), d_ids.data_ptr(),
                                             cap, mode=self.mode,
                                             stream=torch.cuda.current_stream(self.device).cuda_stream)
                break
            except Exception as e:  # EMQX_EOVERFLOW: retry with the exact capacity
                need = getattr(e, "needed", None)
                if need is None:
                    raise
                cap = need + 1
        self._cap = max(cap, getattr(self, "_cap", 0))
        return d_off[1:] - d_off[:-1], d_ids[:m]

    def match(self, topics: Optional[Tuple[torch.Tensor, torch.Tensor]], src: int = 0, dst: int = 0):
        """Match a batch held by rank ``src`` against the sharded table; rank ``dst`` gets the
        CSR in batch order (offsets int64 (n+1,), ids int32), other ranks get None."""
        dev, G, me, grp = self.device, self.world, self.rank, self.group
        i64 = dict(dtype=torch.int64, device=dev)
        # 1. the source partitions its batch by owner rank
        if me == src:
            tb, to = topics
            tb, to = tb.to(dev), to.to(dev).to(torch.int64)
            owner = topic_owner(tb, to, G)
            perm, lens_p, bytes_p, n_to, bytes_to = partition(tb, to, owner, G)
            send_meta = torch.stack([n_to, bytes_to], 1).reshape(-1)
        else:
            send_meta = torch.zeros(2 * G, **i64)
        # 2. sizes: every rank learns what it receives from the source
        recv_meta = torch.empty(2 * G, **i64)
        _a2a(recv_meta, send_meta, [2] * G, [2] * G, grp)
        rm = recv_meta.reshape(G, 2).cpu()
        n_in, b_in = int(rm[src, 0]), int(rm[src, 1])
        if me == src:
            sm = send_meta.reshape(G, 2).cpu()
            n_out_splits, b_out_splits = sm[:, 0].tolist(), sm[:, 1].tolist()
        else:
            lens_p = torch.zeros(0, **i64)
            bytes_p = torch.zeros(0, dtype=torch.uint8, device=dev)
            n_out_splits, b_out_splits = [0] * G, [0] * G
        in_splits_n = [n_in if r == src else 0 for r in range(G)]
        in_splits_b = [b_in if r == src else 0 for r in range(G)]
        # 3. the parts: topic lengths and bytes (a rank's part may be empty)
        my_lens = torch.empty(n_in, **i64)
        _a2a(my_lens, lens_p, in_splits_n, n_out_splits, grp)
        my_bytes = torch.empty(max(b_in, 1), dtype=torch.uint8, device=dev)
        _a2a(my_bytes[:b_in], bytes_p[:sum(b_out_splits)], in_splits_b, b_out_splits, grp)
        my_offs = torch.zeros(n_in + 1, **i64)
        if n_in:
            my_offs[1:] = torch.cumsum(my_lens, 0)
        # 4. the local match, against this rank's shard only
        counts, ids = self.match_fn(my_bytes, my_offs)
        counts = counts.to(torch.int64).to(dev)
        ids = ids.to(torch.int32).to(dev)
        self.last_local_topics = n_in
        # 5. results back to the destination: counts first (with the id totals), then ids
        tot = torch.zeros(G, **i64)
        tot[dst] = int(ids.numel())
        tot_in = torch.empty(G, **i64)
        _a2a(tot_in, tot, [1] * G, [1] * G, grp)
        n_parts = [0] * G
        if me == dst:
            if me == src:
                n_parts = n_out_splits
            else:  # the destination learns the part sizes and the order from the source
                np_t = torch.zeros(G, **i64)
                dist.recv(np_t, src=src, group=grp)
                n_parts = np_t.cpu().tolist()
                perm = torch.empty(sum(n_parts), **i64)
                dist.recv(perm, src=src, group=grp)
        elif me == src:
            dist.send(torch.tensor(n_out_splits, **i64), dst=dst, group=grp)
            dist.send(perm.contiguous(), dst=dst, group=grp)
        ids_in_splits = tot_in.cpu().tolist() if me == dst else [0] * G
        cnt_in = torch.empty(sum(n_parts), **i64)
        _a2a(cnt_in, counts, n_parts, [n_in if r == dst else 0 for r in range(G)], grp)
        ids_in = torch.empty(sum(ids_in_splits), dtype=torch.int32, device=dev)
        _a2a(ids_in, ids, ids_in_splits, [int(ids.numel()) if r == dst else 0 for r in range(G)], grp)
        # 6. the destination puts the results back in batch order
        if me != dst:
            return None
        return merge_csr(cnt_in, ids_in, perm)

    def match_all(self, topics: Tuple[torch.Tensor, torch.Tensor]):
        """Every rank matches its own batch against the sharded table and gets its own CSR
        (offsets int64 (n+1,), ids int32) in batch order — the layout's weak-scaling use, one
        publishing node per rank.  Each rank partitions its batch by owner; one all-to-all
        sends every part to its owner, every rank matches all it received (from all sources)
        in one engine call, and one all-to-all (counts, then ids) returns each source's
        results, which it puts back in batch order.  The collectives move each topic and each
        result once; the fixed cost per step does not grow with the number of sources."""
        dev, G, grp = self.device, self.world, self.group
        i64 = dict(dtype=torch.int64, device=dev)
        tb, to = topics
        tb, to = tb.to(dev), to.to(dev).to(torch.int64)
        owner = topic_owner(tb, to, G)
        perm, lens_p, bytes_p, n_to, bytes_to = partition(tb, to, owner, G)
        # sizes: what every source sends to every owner
        send_meta = torch.stack([n_to, bytes_to], 1).reshape(-1)
        recv_meta = torch.empty(2 * G, **i64)
        _a2a(recv_meta, send_meta, [2] * G, [2] * G, grp)
        sm = send_meta.reshape(G, 2).cpu()
        rm = recv_meta.reshape(G, 2).cpu()
        n_out, b_out = sm[:, 0].tolist(), sm[:, 1].tolist()
        n_in, b_in = rm[:, 0].tolist(), rm[:, 1].tolist()
        # the parts, source after source
        my_lens = torch.empty(sum(n_in), **i64)
        _a2a(my_lens, lens_p, n_in, n_out, grp)
        my_bytes = torch.empty(max(sum(b_in), 1), dtype=torch.uint8, device=dev)
        _a2a(my_bytes[:sum(b_in)], bytes_p[:sum(b_out)], b_in, b_out, grp)
        my_offs = torch.zeros(sum(n_in) + 1, **i64)
        if sum(n_in):
            my_offs[1:] = torch.cumsum(my_lens, 0)
        counts, ids = self.match_fn(my_bytes, my_offs)
        counts = counts.to(torch.int64).to(dev)
        ids = ids.to(torch.int32).to(dev)
        self.last_local_topics = sum(n_in)
        # results back: counts per received part, and the id total of each part
        bounds = torch.tensor([0] + list(np.cumsum(n_in)), **i64)
        csum = torch.zeros(sum(n_in) + 1, **i64)
        if sum(n_in):
            csum[1:] = torch.cumsum(counts, 0)
        ids_out = (csum[bounds[1:]] - csum[bounds[:-1]]).cpu().tolist()
        ids_in_t = torch.empty(G, **i64)
        _a2a(ids_in_t, torch.tensor(ids_out, **i64), [1] * G, [1] * G, grp)
        ids_in = ids_in_t.cpu().tolist()
        cnt_back = torch.empty(int(perm.numel()), **i64)
        _a2a(cnt_back, counts, n_out, n_in, grp)
        ids_back = torch.empty(sum(ids_in), dtype=torch.int32, device=dev)
        _a2a(ids_back, ids, ids_in, ids_out, grp)
        return merge_csr(cnt_back, ids_back, perm)
