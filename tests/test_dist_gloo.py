"""Multi-process (gloo, CPU, world sizes 2, 4 and 8) checks of the multi-GPU layouts in
emqx_amd/dist.py.

The match_all tests drive the product's step (dist.py ShardedMatcher._step_gen: the same
protocol, exchanges, chunk formats, redo and bookkeeping as on the GPUs) with the step object in
its host mode (emqx_shard_step_create(-1, ...): shard_step.hip's per-item bodies — routing and
fold (layout.h), layout, pack, unpack, answer, gather, merge — as loops over host memory) and
each rank's engines answered by the oracle (test infrastructure), over gloo; the result is
checked against a single-table oracle run.  So the CPU rehearsal and the device step cannot
drift apart: only the per-slot match and the tile sort's parallel form differ.  The layout
tests check the placement (two key spaces — first level, and second level under a root '+' —
or space P replicated; hot keys split by the next level; root wildcards on every rank) covers
every match.  The HIP match itself is covered by the GPU tests."""

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


def _oracle_match_fn(engines):
    """match_fn(engine, tb, to) over the oracle, one oracle table per engine of this rank."""
    from oracle import cpp as C
    tabs = []
    for local_filters, global_ids in engines:
        o = C.CppOracle(True)
        ids = o.add_packed(*local_filters) if len(global_ids) else np.zeros(0, np.uint32)
        l2g = np.zeros(max(len(ids), 1), dtype=np.uint32)
        l2g[ids] = global_ids
        tabs.append((o, l2g))

    def fn(e, tb, to):
        o, l2g = tabs[e]
        buf = tb.numpy().astype(np.uint8)
        offs = to.numpy().astype(np.uint64)
        off, oids, _ = o.match_csr(buf if len(buf) else np.zeros(1, np.uint8), offs, mode=0, threads=2)
        return (torch.from_numpy(np.diff(off.astype(np.int64))),
                torch.from_numpy(l2g[oids].astype(np.int32) if oids.size else np.zeros(0, np.int32)))
    return fn


def _matcher(filters, rank, world, p_space="auto"):
    from emqx_amd import dist as D
    plan = D.shard_plan(filters, world, p_space=p_space)
    return D.ShardedMatcher(filters, device=torch.device("cpu"), p_space=p_space,
                            match_fn=_oracle_match_fn(D.shard_engines(filters, rank, world, plan)))


def _batches():
    from emqx_amd import workloads as W
    wl = W.config_b(n_filters=60_000, n_topics=3000, seed=7)
    extra = [b"", b"/", b"+", b"#", b"+/x", b"$SYS/a", b"a/+", b"", b"+/x/y", b"/+", b"region0/+",
             b"region0", b"region0/#"]  # wildcard / empty / '$' / one-level topics
    from emqx_amd.engine import pack
    tb = np.concatenate([wl.topics[0][: int(wl.topics[1][-1])], pack(extra)[0][: sum(len(x) for x in extra)]])
    to = np.concatenate([wl.topics[1].astype(np.uint64),
                         wl.topics[1][-1] + np.cumsum([len(x) for x in extra]).astype(np.uint64)])
    have = set(W.unpack(wl.filters))
    more = [f for f in [b"+/x", b"#", b"a/+", b"+/x/y", b"+/x/#", b"+/x/+", b"+", b"+/#", b"region0", b"region0/#",
                        b"region0/+", b"/+", b"+/"] if f not in have]  # distinct filters, as the generator's
    filters = (np.concatenate([wl.filters[0][: int(wl.filters[1][-1])], np.frombuffer(b"".join(more), np.uint8)]),
               np.concatenate([wl.filters[1].astype(np.uint64),
                               wl.filters[1][-1] + np.cumsum([len(x) for x in more]).astype(np.uint64)]))
    return filters, (tb, to)


def _worker(rank, world, port, q, src, dst):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from emqx_amd import dist as D
        filters, topics = _batches()
        sm = _matcher(filters, rank, world)
        t = (torch.from_numpy(topics[0].copy()), torch.from_numpy(topics[1].astype(np.int64))) if rank == src else None
        res = sm.match(t, src=src, dst=dst)
        # an empty batch and a batch of empty topics go through the same collectives
        empty = (torch.zeros(0, dtype=torch.uint8), torch.zeros(1, dtype=torch.int64)) if rank == src else None
        r0 = sm.match(empty, src=src, dst=dst)
        blanks = (torch.zeros(0, dtype=torch.uint8), torch.zeros(4, dtype=torch.int64)) if rank == src else None
        r1 = sm.match(blanks, src=src, dst=dst)
        if rank == dst:
            q.put(("sharded", res[0].numpy(), res[1].numpy()))
            q.put(("empty", r0[0].tolist(), r0[1].numel(), r1[0].numpy(), r1[1].numpy()))
        else:
            assert res is None and r0 is None and r1 is None
        part = D.split_topics(topics, rank, world)
        q.put(("split", rank, len(part[1]) - 1))
    finally:
        dist.destroy_process_group()


def _expected():
    from oracle import cpp as C
    filters, topics = _batches()
    o = C.CppOracle(True)
    o.add_packed(*filters)
    return o.match_csr(*topics, mode=0, threads=4)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,src,dst", [(2, 0, 0), (4, 0, 0), (4, 2, 1), (8, 5, 3)])
def test_sharded_equals_single_table(world, src, dst):
    from oracle import cpp as C
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, src, dst)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world + 2)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    off_o, ids_o, _ = _expected()
    sharded = [g for g in got if g[0] == "sharded"][0]
    assert C.csr_mismatches(sharded[1], sharded[2], off_o, ids_o).size == 0
    empty = [g for g in got if g[0] == "empty"][0]
    assert empty[1] == [0] and empty[2] == 0
    o = C.CppOracle(True)
    o.add_packed(*_batches()[0])
    off3, ids3, _ = o.match_csr(np.zeros(1, np.uint8), np.zeros(4, np.uint64), mode=0)
    assert C.csr_mismatches(empty[3], empty[4], off3, ids3).size == 0
    splits = sorted(g[2] for g in got if g[0] == "split")
    assert sum(splits) == len(_batches()[1][1]) - 1


def _worker_all(rank, world, port, q, p_space):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from emqx_amd import dist as D
        filters, topics = _batches()
        sm = _matcher(filters, rank, world, p_space)
        # every rank publishes its own slice (rank 1 of 2+ an empty batch)
        part = D.split_topics(topics, rank, world)
        if rank == 1:
            part = (np.zeros(0, np.uint8), np.zeros(1, np.uint64))
        t = (torch.from_numpy(part[0].copy()), torch.from_numpy(part[1].astype(np.int64)))
        off, ids = sm.match_all(t)
        q.put((rank, part[0].copy(), part[1].copy(), off.numpy(), ids.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,p_space", [(2, "sharded"), (4, "sharded"), (8, "sharded"), (2, "replicated"),
                                           (8, "replicated")])
def test_sharded_match_all_sources(world, p_space):
    """ShardedMatcher.match_all: every rank a source of its own batch, each gets its own CSR
    equal to the single-table oracle's for that batch; both space-P layouts (two requests a
    topic, or space P on every rank and one request a topic)."""
    from oracle import cpp as C
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_all, args=(r, world, port, q, p_space)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    o = C.CppOracle(True)
    o.add_packed(*_batches()[0])
    for rank, tb, to, off, ids in got:
        off_o, ids_o, _ = o.match_csr(tb if len(tb) else np.zeros(1, np.uint8), to, mode=0, threads=2)
        assert C.csr_mismatches(off, ids, off_o, ids_o).size == 0, rank


def _worker_redo(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from emqx_amd import workloads as W
        wl = W.config_b(n_filters=60_000, n_topics=60_000, seed=7, topic_seed=None if rank == 0 else 70 + rank)
        sm = _matcher(wl.filters, rank, world, "sharded")
        sm._caps = [1, 1, 1]  # the 64 K-id floor is below a slot's ids: every engine call overflows
        t = (torch.from_numpy(wl.topics[0].copy()), torch.from_numpy(wl.topics[1].astype(np.int64)))
        off, ids = sm.match_all(t)
        learnt = max(sm._caps) > 65536
        again = sm.match_all(t)  # learnt capacities: no redo, the same CSR
        same = torch.equal(again[0], off) and torch.equal(again[1], ids)
        q.put((rank, wl.topics[0].copy(), wl.topics[1].copy(), off.numpy(), ids.numpy(), learnt, same, wl.filters))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_sharded_redo_on_small_capacities():
    """The redo protocol of the step at world 2: every rank's engine calls overflow their (forced)
    capacities, the answer chunks carry the flag, every rank redoes the answer exchange, and each
    source's CSR equals the oracle's; the learnt capacities then need no redo."""
    from oracle import cpp as C
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_redo, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(2)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    o = C.CppOracle(True)
    o.add_packed(*got[0][7])
    for rank, tb, to, off, ids, learnt, same, _ in got:
        off_o, ids_o, _ = o.match_csr(tb, to, mode=0, threads=2)
        assert int(off_o[-1]) > 3 * 65536
        assert C.csr_mismatches(off, ids, off_o, ids_o).size == 0, rank
        assert learnt and same


def _worker_fixed(rank, world, port, q, p_space):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from emqx_amd import dist as D
        filters, topics = _batches()
        sm = _matcher(filters, rank, world, p_space)
        part = D.split_topics(topics, rank, world)
        T = lambda b: (torch.from_numpy(b[0].copy()), torch.from_numpy(b[1].astype(np.int64)))  # noqa: E731
        blanks = (np.zeros(0, np.uint8), np.zeros(4, np.uint64))
        # the first batch teaches the capacities (a classic step); the whole topic set twice then
        # overflows them (a flagged step, redone on every rank alike), the rest fit
        nb = int(topics[1][-1])
        big = (np.concatenate([topics[0][:nb], topics[0][:nb]]),
               np.concatenate([topics[1].astype(np.uint64), nb + topics[1][1:].astype(np.uint64)]))
        batches = [part, part, blanks, big, part, (np.zeros(0, np.uint8), np.zeros(1, np.uint64))]
        res = sm.match_stream([T(b) for b in batches], fixed=True, depth=2)
        redo = sm.last_fixed_redo
        res2 = sm.match_stream([T(b) for b in batches[:3]], fixed=True, depth=3)  # learnt: no redo
        redo2 = sm.last_fixed_redo
        # match_all once the capacities are learnt: the fixed form, then the classic one
        res3 = [sm.match_all(T(part)), sm.match_all(T(part), fixed=False)]
        # engine id buffers cut to a 1 K floor: a slot over it flags its step (the engine's
        # summary), which is redone classically on every rank
        sm._caps, sm._ids_floor = [1, 1, 1], 1024
        for ln in sm._lanes:
            for e in range(3):
                ln.bufs.pop(f"ids{e}", None)
        res4 = sm.match_stream([T(big), T(big)], fixed=True)
        redo4 = sm.last_fixed_redo
        q.put((rank, batches + batches[:3] + [part, part, big, big],
               [(o.numpy(), i.numpy()) for o, i in res + res2 + res3 + res4], redo, redo2, redo4))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,p_space", [(1, "auto"), (2, "sharded"), (3, "replicated")])
def test_sharded_fixed_capacity_steps(world, p_space):
    """match_stream in the fixed-capacity form (emqx_shard_step_*_fixed: chunks at agreed
    capacities, the recv table built from the chunk headers, fixed-size engine batches with
    padding topics, the flag carried in every chunk): every step's CSR equals the single-table
    oracle's; a batch over the capacities is flagged on every rank and redone in the classic form,
    after which the learnt capacities need no redo.  World 1 matches every slot in place."""
    from oracle import cpp as C
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_fixed, args=(r, world, port, q, p_space)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    o = C.CppOracle(True)
    o.add_packed(*_batches()[0])
    for rank, batches, res, redo, redo2, redo4 in got:
        assert redo == 1 and redo2 == 0, (rank, redo, redo2)
        assert redo4 == 2, redo4  # (2 x 3 K topics: ~36 K ids, over every rank's 1 K buffers)
        assert len(res) == len(batches)
        for k, (b, (off, ids)) in enumerate(zip(batches, res)):
            tb, to = b
            off_o, ids_o, _ = o.match_csr(tb if len(tb) else np.zeros(1, np.uint8), to.astype(np.uint64), mode=0,
                                          threads=2)
            assert C.csr_mismatches(off, ids, off_o, ids_o).size == 0, (rank, k)


def test_shard_layout_covers_every_match():
    """Every filter that matches a topic is held by the rank of the topic's request to the
    filter's engine (so the two requests find every match, once); a filter is held by exactly
    `span` ranks, root wildcards by all; '$' and one-level topics make no engine-B request."""
    from emqx_amd import dist as D
    from oracle import cpp as C
    filters, topics = _batches()
    o = C.CppOracle(True)
    o.add_packed(*filters)
    off, ids, _ = o.match_csr(*topics, mode=0, threads=4)
    tid = np.repeat(np.arange(len(topics[1]) - 1), np.diff(off.astype(np.int64)))
    names = W_unpack(topics)
    for world, p_space in ((1, "auto"), (2, "sharded"), (3, "sharded"), (8, "sharded"), (2, "replicated"),
                           (8, "replicated")):
        plan = D.shard_plan(filters, world, max_piece_pm=50, p_space=p_space)  # small pieces: many split keys
        assert world == 1 or len(plan) > 0
        assert D.plan_p_replicated(plan) == (p_space == "replicated")
        first, span, eng = D.shard_place(filters, world, plan)
        req = D.topic_requests(torch.from_numpy(topics[0]), torch.from_numpy(topics[1].astype(np.int64)), world,
                               plan).numpy()
        r = req[tid, eng[ids]]
        assert np.all(r >= 0)
        assert np.all(r % 2 == eng[ids])
        assert np.all(((r // 2 - first[ids].astype(np.int64)) % world) < span[ids])
        held = np.zeros(len(first), np.int64)
        for k in range(world):
            ga, gb, gab = D.shard_local_ids(filters, k, world, plan)
            for e, g in enumerate((ga, gb)):
                held[g] += 1
                assert np.all(eng[g] == e)
            assert np.array_equal(gab, np.union1d(ga, gb))  # the AB engine: A and B in one table
        assert np.array_equal(held, span.astype(np.int64))
        for t, rq in zip(names, req):
            if t.startswith(b"$") or b"/" not in t:
                assert rq[1] == -1, t
        if p_space == "replicated":  # one request a topic; space P on every rank with engine A
            assert np.all(req[:, 1] == -1) and np.all(eng == 0)
            fnames = W_unpack(filters)
            is_p = np.array([f.startswith(b"+/") and f[2:3] not in (b"+", b"#") for f in fnames])
            assert is_p.any() and np.all(span[is_p] == world)
        else:
            assert world == 1 or (eng == 1).any()
        # the folded keys (rank * 3 + slot): two requests to two ranks stay A and B; to one rank,
        # or a single request, one AB request in the first column; at world 1 only AB
        key = D.fold_requests(torch.from_numpy(req), world).numpy()
        a, b = req[:, 0] >= 0, req[:, 1] >= 0
        split = a & b & (req[:, 0] // 2 != req[:, 1] // 2)
        assert np.array_equal(key[split, 0], 3 * (req[split, 0] // 2))
        assert np.array_equal(key[split, 1], 3 * (req[split, 1] // 2) + 1)
        one = ~split & (a | b)
        assert np.all(key[one, 0] % 3 == 2) and np.all(key[one, 1] == 3 * world)
        assert np.array_equal(key[one, 0] // 3, np.where(a[one], req[one, 0], req[one, 1]) // 2)
        if world == 1:
            assert np.all(key[:, 0] == 2) and not split.any()


def W_unpack(packed):
    from emqx_amd import workloads as W
    return W.unpack(packed)


def test_shard_plan_divides_config_c_capacity():
    """On config C's generator (vocab x4, seed 3; reduced), the busiest of 8 ranks holds at most
    1.5 / 8 of the filters (29 % with the round-2 layout)."""
    from emqx_amd import dist as D
    from emqx_amd import workloads as W
    wl = W.config_b(n_filters=400_000, n_topics=10, seed=3, vocab_scale=4)
    names = W.unpack(wl.filters)
    p_share = sum(1 for f in names if f.startswith(b"+/") and not f[2:3] in (b"+", b"#", b"")) / wl.n_filters
    for world in (2, 4, 8):
        for p_space in ("sharded", "auto"):
            plan = D.shard_plan(wl.filters, world, p_space=p_space)
            # auto: space P (~7 % of config C) replicated, at most a rank's share
            assert D.plan_p_replicated(plan) == (p_space == "auto" and p_share * world <= 1.0)
            first, span, eng = D.shard_place(wl.filters, world, plan)
            held = np.zeros(world, np.int64)
            for k in range(world):
                held[k] = int(np.count_nonzero(((k - first.astype(np.int64)) % world) < span))
            bound = 1.5 / world + (p_share if D.plan_p_replicated(plan) else 0.0)
            assert held.max() / wl.n_filters <= bound, (world, p_space, held.max() / wl.n_filters)


def test_partition_and_merge_roundtrip():
    from emqx_amd import dist as D
    from emqx_amd.engine import pack
    topics = [b"a/b", b"", b"x", b"a/c/d", b"q", b"+/z"]
    buf, offs = pack(topics)
    tb, to = torch.from_numpy(buf.copy()), torch.from_numpy(offs.astype(np.int64))
    owner = torch.tensor([1, 0, 2, 1, 0, 0])
    perm, lens_p, bytes_p, n_to, bytes_to = D.partition(tb, to, owner, 3)
    assert perm.tolist() == [1, 4, 5, 0, 3, 2] and n_to.tolist() == [3, 2, 1]
    parts = bytes(bytes_p.numpy()).decode()
    assert parts == "q+/za/ba/c/dx" and bytes_to.tolist() == [4, 8, 1]
    # results of the received topics (perm order), merged back into batch order
    rc = torch.tensor([0, 2, 1, 1, 3, 0])
    ri = torch.tensor([40, 41, 50, 0, 30, 31, 32], dtype=torch.int32)
    off, ids = D.merge_csr(rc, ri, perm)
    assert off.tolist() == [0, 1, 1, 1, 4, 6, 7]
    assert ids.tolist() == [0, 30, 31, 32, 40, 41, 50]


@pytest.mark.parametrize("skip_own", [False, True])
def test_chunk_exchange_addresses(skip_own):
    """dist.py chunk_offsets, the address arithmetic of _exchange_chunks for both exchanges:
    gloo's all_to_all_single (every chunk, the own one included, in rank order) and RCCL's list
    all_to_all (the own entry empty; ADVICE r5: that branch has not run on several GPUs).  Both
    collectives are simulated on host arrays from their definitions, and every source's chunk
    is read back through the returned address."""
    from emqx_amd import dist as D
    rng = np.random.default_rng(3)
    for G in (2, 3, 8):
        sizes = rng.integers(0, 40, size=(G, G))  # sizes[s][r]: bytes source s sends rank r
        sends = [rng.integers(0, 255, size=int(sizes[s].sum()), dtype=np.uint8) for s in range(G)]
        for rank in range(G):
            out_sz = sizes[rank].tolist()
            in_sz = sizes[:, rank].tolist()
            out_off, in_off, addrs = D.chunk_offsets(out_sz, in_sz, rank, skip_own, base=0, rbase=1 << 20)
            recv = np.zeros(int(in_off[-1]), np.uint8)
            for s in range(G):  # the collective: source s's chunk for `rank` at its receive offset
                if skip_own and s == rank:
                    continue
                lo = int(np.sum(sizes[s][:rank]))
                recv[int(in_off[s]): int(in_off[s + 1])] = sends[s][lo: lo + int(sizes[s][rank])]
            for s in range(G):
                lo = int(np.sum(sizes[s][:rank]))
                want = sends[s][lo: lo + int(sizes[s][rank])]
                a = addrs[s]
                got = sends[rank][a: a + len(want)] if s == rank else recv[a - (1 << 20): a - (1 << 20) + len(want)]
                assert np.array_equal(got, want), (G, rank, s)
