"""Multi-GPU route lookup: one process per GPU, torch.distributed (RCCL over xGMI on MI355X).

SURVEY §8(e).  Two layouts:

* **Replicated** (tables that fit one GPU — 10M filters take a few GB of 288 GB): every rank
  holds the whole table and matches its own slice of the topic stream.  Pure data
  parallelism, no collective on the data path (``split_topics``).  The reference does the same
  across a cluster: every node holds a full mria copy of the route table
  (apps/emqx/src/emqx_router.erl:135, apps/emqx/src/emqx_trie.erl:72-77).

* **Filter-sharded** (``ShardedMatcher``): filter ``i`` lives on rank ``i mod G``; each rank builds
  the level trie of its shard with GLOBAL filter ids (``emqx_insert_filters_ext``).  A topic
  batch is broadcast from its source rank, every rank matches it against its shard, and the
  per-topic union — a concatenation, the shards being disjoint — is assembled on the
  destination rank from an all-gather of per-topic counts and a gather of the id lists.

Collective payloads per 1M-topic batch of config B: the batch (~44 MB) broadcast once, counts
4 MB per rank, ids ~56 MB in total — large, few collectives, as ring collectives over the
point-to-point xGMI links want.
"""

from __future__ import annotations

from typing import Callable, List, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist


def split_topics(packed: Tuple[np.ndarray, np.ndarray], rank: int, world: int):
    """Replicated mode: this rank's contiguous slice of a packed topic batch."""
    from .workloads import take
    n = len(packed[1]) - 1
    lo, hi = (n * rank) // world, (n * (rank + 1)) // world
    return take(packed, np.arange(lo, hi))


def shard_of(ids: np.ndarray, world: int) -> np.ndarray:
    """Filter-sharded mode: the rank that owns each global filter id."""
    return (np.asarray(ids, dtype=np.int64) % world).astype(np.int64)


def shard_filters(packed: Tuple[np.ndarray, np.ndarray], rank: int, world: int):
    """(packed filters of this rank's shard, their global ids)."""
    from .workloads import take
    n = len(packed[1]) - 1
    gids = np.nonzero(shard_of(np.arange(n), world) == rank)[0]
    return take(packed, gids), gids.astype(np.uint32)


def concat_csr(counts: Sequence[torch.Tensor], ids: Sequence[torch.Tensor]):
    """Per-topic concatenation of G CSR results of the same n topics (shard order).

    counts[r]: (n,) int64, ids[r]: (sum counts[r],) int32 laid out topic by topic.
    Returns (offsets (n+1,) int64, ids (total,) int32) on the tensors' device."""
    dev = counts[0].device
    n = counts[0].numel()
    C = torch.stack([c.to(torch.int64) for c in counts])          # (G, n)
    total_per_topic = C.sum(0)
    offsets = torch.zeros(n + 1, dtype=torch.int64, device=dev)
    offsets[1:] = torch.cumsum(total_per_topic, 0)
    before = torch.cumsum(C, 0) - C                                  # ids of earlier shards per topic
    out = torch.empty(int(offsets[-1].item()), dtype=torch.int32, device=dev)
    topic = torch.arange(n, device=dev)
    for r in range(C.shape[0]):
        c = C[r]
        m = int(c.sum().item())
        if m == 0:
            continue
        t_of = torch.repeat_interleave(topic, c)
        local_off = torch.cumsum(c, 0) - c
        j = torch.arange(m, device=dev) - local_off[t_of]
        pos = offsets[t_of] + before[r][t_of] + j
        out[pos] = ids[r][:m].to(torch.int32)
    return offsets, out


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
        """Match a batch held by rank ``src`` against every shard; rank ``dst`` gets the merged
        CSR (offsets int64 (n+1,), ids int32), other ranks get None."""
        dev = self.device
        # 1. broadcast the batch: sizes, offsets, bytes
        meta = torch.zeros(2, dtype=torch.int64, device=dev)
        if self.rank == src:
            tb, to = topics
            meta[0], meta[1] = to.numel() - 1, tb.numel()
        dist.broadcast(meta, src, group=self.group)
        n, nbytes = int(meta[0].item()), int(meta[1].item())
        if self.rank != src:
            to = torch.empty(n + 1, dtype=torch.int64, device=dev)
            tb = torch.empty(max(nbytes, 1), dtype=torch.uint8, device=dev)
        dist.broadcast(to, src, group=self.group)
        dist.broadcast(tb, src, group=self.group)
        # 2. local match against this rank's shard (global filter ids)
        counts, ids = self.match_fn(tb, to)
        counts = counts.to(torch.int64)
        # 3. all-gather per-topic counts, gather the id lists (padded to the largest shard)
        all_counts = [torch.empty_like(counts) for _ in range(self.world)]
        dist.all_gather(all_counts, counts, group=self.group)
        sizes = [int(c.sum().item()) for c in all_counts]
        pad = max(max(sizes), 1)
        send = torch.zeros(pad, dtype=torch.int32, device=dev)
        send[: ids.numel()] = ids.to(torch.int32)
        gathered = [torch.empty(pad, dtype=torch.int32, device=dev) for _ in range(self.world)] \
            if self.rank == dst else None
        dist.gather(send, gathered, dst=dst, group=self.group)
        if self.rank != dst:
            return None
        # 4. per-topic concatenation in shard order
        return concat_csr(all_counts, [g[:s] for g, s in zip(gathered, sizes)])
