"""Multi-process (world_size 2, gloo, CPU) checks of the multi-GPU layouts in emqx_amd/dist.py.

The per-shard match is injected from the oracle (test infrastructure) so that the
distribution logic — filter sharding, topic broadcast, count all-gather, id gather and the
per-topic CSR concatenation — is checked against a single-table oracle run.  The HIP match
itself is covered by the GPU tests."""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_match_fn(local_filters, global_ids):
    from oracle import cpp as C

    def fn(tb, to):
        o = C.CppOracle(True)
        ids = o.add_packed(*local_filters)
        l2g = np.zeros(len(ids), dtype=np.uint32)
        l2g[ids] = global_ids
        buf = tb.numpy().astype(np.uint8)
        offs = to.numpy().astype(np.uint64)
        counts, oids, _ = o.match_packed(buf, offs, mode=0, threads=2, stride=512)
        flat = np.concatenate([l2g[oids[i, :counts[i]]] for i in range(len(counts))]) if len(counts) else np.zeros(0)
        return torch.from_numpy(counts.astype(np.int64)), torch.from_numpy(flat.astype(np.int32))
    return fn


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from emqx_amd import dist as D
        from emqx_amd import workloads as W
        wl = W.config_b(n_filters=60_000, n_topics=3000, seed=7)
        local, gids = D.shard_filters(wl.filters, rank, world)
        sm = D.ShardedMatcher.__new__(D.ShardedMatcher)
        sm.group, sm.rank, sm.world, sm.device, sm.mode = None, rank, world, torch.device("cpu"), 0
        sm.local_filters, sm.global_ids, sm.engine = local, gids, None
        sm.match_fn = _oracle_match_fn(local, gids)
        topics = (torch.from_numpy(wl.topics[0].copy()), torch.from_numpy(wl.topics[1].view(np.int64).copy())) \
            if rank == 0 else None
        res = sm.match(topics, src=0, dst=0)
        # replicated mode: slices cover the batch exactly once
        part = D.split_topics(wl.topics, rank, world)
        if rank == 0:
            off, ids = res
            q.put(("sharded", off.numpy(), ids.numpy()))
        q.put(("split", rank, len(part[1]) - 1))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_equals_single_table():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world + 1)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    from emqx_amd import workloads as W
    from oracle import cpp as C
    wl = W.config_b(n_filters=60_000, n_topics=3000, seed=7)
    o = C.CppOracle(True)
    o.add_packed(*wl.filters)
    counts, oids, _ = o.match_packed(*wl.topics, mode=0, threads=4, stride=512)
    sharded = [g for g in got if g[0] == "sharded"][0]
    off, ids = sharded[1], sharded[2]
    assert np.array_equal(np.diff(off), counts.astype(np.int64))
    for i in range(len(counts)):
        assert np.array_equal(np.sort(ids[off[i]:off[i + 1]]), oids[i, :counts[i]])
    splits = sorted(g[2] for g in got if g[0] == "split")
    assert sum(splits) == wl.n_topics


def test_concat_csr_layout():
    from emqx_amd.dist import concat_csr
    c0 = torch.tensor([1, 0, 2])
    c1 = torch.tensor([0, 3, 1])
    i0 = torch.tensor([10, 20, 21], dtype=torch.int32)
    i1 = torch.tensor([5, 6, 7, 8], dtype=torch.int32)
    off, ids = concat_csr([c0, c1], [i0, i1])
    assert off.tolist() == [0, 1, 4, 7]
    assert ids.tolist() == [10, 5, 6, 7, 20, 21, 8]


def test_shard_partition_is_disjoint_and_complete():
    from emqx_amd import dist as D
    from emqx_amd import workloads as W
    wl = W.config_a(n_topics=10)
    seen = []
    for r in range(4):
        _, g = D.shard_filters(wl.filters, r, 4)
        seen.append(g)
    allg = np.sort(np.concatenate(seen))
    assert np.array_equal(allg, np.arange(wl.n_filters))
