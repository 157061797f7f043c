"""The filter-sharded step on device kernels (emqx_amd/csrc/shard_step.hip, emqx_shard_step_*,
driven by emqx_amd/dist.py ShardedMatcher.match_all), ID-for-ID against the oracle
(oracle/trie_oracle.cpp: emqx_trie DFS + match_routes/1, apps/emqx/src/emqx_router.erl:128-133):

* edge batches at world 1 over RCCL: an empty batch, one-level topics (no engine-B request),
  '$' topics (no '+/x' match, emqx_topic.erl:71-74), wildcard topic names (one request, to
  their byte-identical filter), topics whose only matches are root wildcards;
* the redo path: id capacities far too small, so the engine call overflows and is redone
  before the answer exchange;
* two ranks sharing the one GPU over gloo (a rehearsal of the N-rank exchange on real device
  kernels), each rank's own batch checked ID-for-ID.
"""

import os

import numpy as np
import pytest

from oracle import cpp as C

pytestmark = pytest.mark.gpu

FILTERS = [b"#", b"+", b"+/#", b"+/+", b"+/+/#", b"a", b"a/b", b"a/+", b"a/#", b"+/b", b"+/b/c", b"+/b/#",
           b"$SYS/#", b"$SYS/x", b"$SYS/+/y", b"a/b/c/d/e", b"q/+/+/+/#", b"x/y", b"+/y/z", b"m/#",
           b"s/+", b"s/t/#", b"a/+/c", b"+/+/c"]
TOPICS = [b"a", b"a/b", b"a/b/c", b"$SYS/x", b"$SYS/x/y", b"$SYS", b"x/y", b"x/y/z", b"q/1/2/3",
          b"q/1/2/3/4/5", b"m", b"zz", b"s/t", b"s/t/u", b"a/+", b"+/b", b"#", b"a/#", b"+/y/z",
          b"a/b/c/d/e", b"/", b"a//", b"//b", b"c", b"a/q/c"]


def _init(port):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))


def _dev_topics(packed):
    import torch
    buf, offs = packed
    dev = torch.device("cuda:0")
    tb = torch.from_numpy(np.array(buf, dtype=np.uint8)).to(dev) if len(buf) else torch.zeros(0, dtype=torch.uint8, device=dev)
    return tb, torch.from_numpy(np.asarray(offs).astype(np.int64)).to(dev)


def _oracle(filters, topics):
    o = C.CppOracle(True)
    o.add_packed(*filters)
    o.freeze()
    off, ids, _ = o.match_csr(*topics, mode=C.MODE_ROUTES, threads=4)
    return off, ids


def _check(res, filters, topics):
    off, ids = res[0].cpu().numpy(), res[1].cpu().numpy().view(np.uint32)
    off_o, ids_o = _oracle(filters, topics)
    assert len(off) == len(off_o)
    bad = C.csr_mismatches(off.astype(np.uint64), ids, off_o, ids_o)
    assert bad.size == 0, bad[:10]
    return int(off_o[-1])


def test_shard_step_edge_batches_world1():
    import torch
    import torch.distributed as dist
    from emqx_amd.dist import ShardedMatcher
    from emqx_amd.engine import pack
    filters = pack(FILTERS)
    _init(29561)
    try:
        sm = ShardedMatcher(filters, device=torch.device("cuda:0"))
        assert sm._step is not None  # the device step, not the tensor path
        topics = pack(TOPICS)
        got = sm.match_all(_dev_topics(topics))
        assert _check(got, filters, topics) > 0
        # the same batch through the step's host mode (tests/test_dist_gloo.py's path: the same
        # protocol, the kernels' bodies as loops) with this GPU's engine as the slot matcher:
        # the same CSR, in the same order
        def on_gpu(e, tb, to):
            off, ids = sm._engine_csr(2, tb.cuda(), to.cuda())
            return (off[1:] - off[:-1]).cpu(), ids.cpu()
        host = ShardedMatcher(filters, device=torch.device("cpu"), match_fn=on_gpu)
        off_h, ids_h = host.match_all((torch.from_numpy(topics[0].copy()), torch.from_numpy(topics[1].astype(np.int64))))
        assert torch.equal(off_h, got[0].cpu()) and torch.equal(ids_h, got[1].cpu())
        host.close()
        # an empty batch, a one-topic batch, and a batch of topics no filter besides roots matches
        empty = (np.zeros(0, np.uint8), np.zeros(1, np.uint64))
        off, ids = sm.match_all(_dev_topics(empty))
        assert off.cpu().tolist() == [0] and ids.numel() == 0
        for batch in ([b"a/b"], [b"zz/yy/xx"] * 7, [b"$SYS"] * 3):
            t = pack(batch)
            _check(sm.match_all(_dev_topics(t)), filters, t)
        # steps in flight (match_stream), in both forms (fixed capacities: no host read between
        # the steps, the first call learning its capacities; classic: the size syncs): every
        # batch's CSR, an empty one among them, and in the fixed form a batch over the learnt
        # capacities (flagged, redone in the classic form)
        big = pack(TOPICS * 400)
        for fixed in (True, False):
            seq = [topics, pack([b"a/b"]), empty, pack(TOPICS[::-1]), topics] + ([big, topics] if fixed else [])
            outs = sm.match_stream([_dev_topics(t) for t in seq], fixed=fixed)
            assert len(outs) == len(seq)
            for t, got in zip(seq, outs):
                if len(t[1]) == 1:
                    assert got[0].cpu().tolist() == [0] and got[1].numel() == 0
                else:
                    _check(got, filters, t)
            if fixed:
                assert sm.last_fixed_redo == 1
                outs = sm.match_stream([_dev_topics(t) for t in (big, topics, big)], fixed=True, depth=2)
                assert sm.last_fixed_redo == 0
                for t, got in zip((big, topics, big), outs):
                    _check(got, filters, t)
    finally:
        dist.destroy_process_group()


def test_shard_step_redo_on_small_capacities():
    """The engine call (world 1: every request on the AB slot) overflows its (forced) tiny id
    buffer: the answer kernel flags it, every rank learns it from the size exchange, the call is
    redone, and the CSR is exact."""
    import torch
    import torch.distributed as dist
    from emqx_amd import workloads as W
    from emqx_amd.dist import ShardedMatcher
    wl = W.config_b(n_filters=300_000, n_topics=30_000, seed=3, vocab_scale=4)
    _init(29563)
    try:
        sm = ShardedMatcher(wl.filters, device=torch.device("cuda:0"))
        sm._caps = [1, 1, 1]  # the floor of 64K ids is below this batch's ids
        got = sm.match_all(_dev_topics(wl.topics))
        total = _check(got, wl.filters, wl.topics)
        assert total > 2 * 65536
        assert max(sm._caps) > 65536  # learnt from the redo
        again = sm.match_all(_dev_topics(wl.topics))  # learnt capacities: no redo
        assert torch.equal(again[0].cpu(), got[0].cpu()) and torch.equal(again[1].cpu(), got[1].cpu())
    finally:
        dist.destroy_process_group()


def _rank_main(rank, world, port, q, p_space="sharded"):
    import torch
    import torch.distributed as dist
    from emqx_amd import workloads as W
    from emqx_amd.dist import ShardedMatcher
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        wl = W.config_b(n_filters=200_000, n_topics=8000, seed=3, vocab_scale=4,
                        topic_seed=None if rank == 0 else 1000 + rank)
        sm = ShardedMatcher(wl.filters, device=torch.device("cuda:0"), p_space=p_space)
        assert sm._step is not None
        # two steps: the second reuses the learnt buffers; a third with an empty batch on rank 1
        sm.match_all(_dev_topics(wl.topics))
        got = sm.match_all(_dev_topics(wl.topics))
        empty = (np.zeros(0, np.uint8), np.zeros(1, np.uint64))
        third = sm.match_all(_dev_topics(empty if rank == 1 else wl.topics))
        # steps in flight over the process group (the fixed form, then the classic one): the
        # collectives of the steps pair up
        streamed = sm.match_stream([_dev_topics(wl.topics)] * 3) + sm.match_stream([_dev_topics(wl.topics)] * 3,
                                                                                  fixed=False)
        assert sm.last_fixed_redo == 0
        off, ids = got[0].cpu().numpy(), got[1].cpu().numpy().view(np.uint32)
        off_o, ids_o = _oracle(wl.filters, wl.topics)
        bad = C.csr_mismatches(off.astype(np.uint64), ids, off_o, ids_o)
        for st_off, st_ids in streamed:
            bad = np.concatenate([bad, C.csr_mismatches(st_off.cpu().numpy().astype(np.uint64),
                                                        st_ids.cpu().numpy().view(np.uint32), off_o, ids_o)])
        if rank == 1:
            third_ok = third[0].numel() == 1 and third[1].numel() == 0
        else:  # the same topics on a smaller exchange: the same sets (in-topic order may differ)
            third_ok = C.csr_mismatches(third[0].cpu().numpy().astype(np.uint64),
                                        third[1].cpu().numpy().view(np.uint32), off_o, ids_o).size == 0
        q.put((rank, int(bad.size), int(off_o[-1]), sm.last_local_topics, bool(third_ok), sm.n_local_filters,
               list(sm.last_slot_topics)))
    except Exception as e:  # reported to the parent
        q.put((rank, -1, repr(e), 0, False, 0, [0, 0, 0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,p_space", [(2, "sharded"), (3, "sharded"), (4, "sharded"), (3, "replicated")])
def test_shard_step_ranks_share_one_gpu(world, p_space):
    """The device step (emqx_shard_step_*, dist.py _match_all_device) at world 2, 3 and 4 with
    every rank a process on the one GPU (gloo for the exchanges): each rank's CSR ID-for-ID
    against the oracle over the whole table; a rehearsal of the protocol, not a measurement.
    Both space-P layouts (dist.py shard_plan)."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29565 + world + (10 if p_space == "replicated" else 0)
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, q, p_space)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=200) for _ in range(world)]
    for p in ps:
        p.join(30)
    res.sort()
    for rank, bad, ids, local, third_ok, nf, slots in res:
        assert bad == 0, (rank, ids)
        assert ids > 0 and local > 0 and third_ok
    # every rank holds part of the table (two key spaces), not all of it; some topics' two
    # requests met on one rank (AB slot) and some did not (A and B slots) — both paths ran
    assert all(r[5] < 200_000 for r in res)
    slots = np.sum([r[6] for r in res], axis=0)
    if p_space == "sharded":
        assert slots[0] > 0 and slots[1] > 0 and slots[2] > 0, slots
    else:  # one request a topic, always to the AB slot
        assert slots[0] == 0 and slots[1] == 0 and slots[2] > 0, slots


def test_device_routing_equals_host_routing():
    """The device scanner (16-B windows, shard_step.hip topic_levels_dev) routes every topic as
    the host's shard_route_topic does: config C topics and edge names (wildcards, '$', one level,
    empty levels, long names, the batch's last bytes), at world 1, 2 and 8 with a split plan."""
    import torch
    from emqx_amd import dist as D
    from emqx_amd import workloads as W
    from emqx_amd.engine import pack
    wl = W.config_b(n_filters=200_000, n_topics=20_000, seed=3, vocab_scale=4)
    extra = TOPICS + [b"", b"/", b"//", b"$", b"+", b"#", b"a/+/b", b"x" * 100 + b"/" + b"y" * 37,
                      b"/".join([b"l%d" % i for i in range(40)]), b"$share/g/a", b"a/b/c/"]
    # past the third level the scanner works on 16-byte masks: wildcard levels (and near misses:
    # '++', '+x', 'x+', '#/', '/#') at every offset against the window edges
    for k in range(40):
        head = b"a/b/c/" + b"x" * k
        for tail in (b"/+", b"/#", b"/+/", b"/#/z", b"/++", b"/+x", b"/x+", b"/+/+", b"+", b"#/", b"/+x/y",
                     b"/a+/#b"):
            extra.append(head + tail)
        extra.append(b"+/" * (k + 3) + b"q")
        extra.append(b"a/b/c/" + b"/" * k + b"#")
    eb, eo = pack(extra)
    buf = np.concatenate([wl.topics[0][: int(wl.topics[1][-1])], eb])
    offs = np.concatenate([wl.topics[1].astype(np.uint64), eo[1:].astype(np.uint64) + np.uint64(wl.topics[1][-1])])
    for world in (1, 2, 8):
        plan = D.shard_plan(wl.filters, world)
        tb_c = torch.from_numpy(buf.copy())
        to_c = torch.from_numpy(offs.astype(np.int64))
        host = D.topic_requests(tb_c, to_c, world, plan)
        dev = D.topic_requests(tb_c.cuda(), to_c.cuda(), world, plan).cpu()
        assert torch.equal(host, dev), world


@pytest.mark.parametrize("world,p_space", [(2, "sharded"), (3, "sharded"), (8, "sharded"), (2, "replicated"),
                                           (8, "replicated")])
def test_emulated_world_every_source_id_for_id(world, p_space):
    """dist.py EmulatedWorld: the G ranks of the G-way plan in this one process, every rank's
    step the product's _step_gen with chunks read in place; every source's merged CSR ID-for-ID
    against the oracle over the whole table, in both timing modes and untimed, and the exchange
    bytes accounted for (every request chunk is at least its header)."""
    import torch
    from emqx_amd import workloads as W
    from emqx_amd.dist import EmulatedWorld
    dev = torch.device("cuda:0")
    wl = W.config_b(n_filters=200_000, n_topics=6000, seed=3, vocab_scale=4,
                    extra_topic_seeds=tuple(1000 + s for s in range(1, world)))
    srcs = [wl.topics] + list(wl.extra_topics[: world - 1])
    ew = EmulatedWorld(wl.filters, world, dev, p_space=p_space)
    assert ew.p_replicated == (p_space == "replicated")
    try:
        assert sum(x[2] for x in ew.filters_per_rank) < world * 200_000  # sharded, not replicated
        for timing in (None, "wall", "gpu", None):
            res = ew.step([_dev_topics(s) for s in srcs], timing=timing)
            if timing:
                assert len(ew.last_times) == world and all(len(t) == len(EmulatedWorld.PHASES) for t in ew.last_times)
                assert all(x >= 0 for t in ew.last_times for x in t)
            for s in range(world):
                _check(res[s], wl.filters, srcs[s])
        assert (ew.bytes_out[0] >= 32).all() and (ew.bytes_out[1] >= 32).all()
        for r in range(world):  # each rank alone, two steps in flight, the others' side replayed
            ms, rs = ew.rank_stream(r, _dev_topics(srcs[r]), 3)
            assert ms > 0 and len(rs) == 3
            for got in rs:
                _check(got, wl.filters, srcs[r])
        slots = np.sum([m.last_slot_topics for m in ew.matchers], axis=0)
        if p_space == "sharded":
            assert slots[0] > 0 and slots[1] > 0 and slots[2] > 0, slots
        else:
            assert slots[0] == 0 and slots[1] == 0 and slots[2] > 0, slots
            assert all(m.engines[0] is None and m.engines[1] is None for m in ew.matchers)
        # the fixed-capacity form: capacities learnt from the classic steps above and agreed,
        # every rank's step with no size exchange; every source ID-for-ID, pipelined too
        ew.learn_fixed()
        assert len({(m._fixed["chunk"], m._fixed["answer"]) for m in ew.matchers}) == 1
        for timing in (None, "gpu"):
            res = ew.step([_dev_topics(s) for s in srcs], timing=timing, fixed=True)
            if timing:
                assert all(len(t) == len(EmulatedWorld.PHASES_FIXED) for t in ew.last_times)
            for s in range(world):
                _check(res[s], wl.filters, srcs[s])
        assert (ew.bytes_out[0] == ew.matchers[0]._fixed["chunk"]).all()
        for r in range(world):
            ms, rs = ew.rank_stream(r, _dev_topics(srcs[r]), 3, fixed=True)
            for got in rs:
                _check(got, wl.filters, srcs[r])
    finally:
        ew.close()
