"""Retained-message index on the GPU against the oracle of the reference's
mnesia retainer (oracle/retain_ref.py): the emqx_retainer_SUITE KATs through the
emqx_retainer_mnesia mirror, fuzzed tables/filters/expiry guards compared as sorted topic-id
sets, deletes and recommits, wide '+' fan-outs, root '#', deep topics, and a config-B-scale
table through the device entry point."""

import random

import numpy as np
import pytest

from oracle import retain_ref as RR

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mod():
    import torch  # noqa: F401
    from emqx_amd import _lib, retainer
    _lib.lib()
    return retainer


def test_retainer_suite_kats(mod, kats):
    for case in kats["retain_cases"]:
        st = mod.MnesiaRetainer()

        def apply(op):
            if op[0] == "store":
                st.store_retained(mod.Message(op[1].encode(), b"payload", 0, op[2]))
            elif op[0] == "publish_empty":
                st.on_message_publish(mod.Message(op[1].encode(), b"", 0, 0))
            else:
                st.delete_message(op[1].encode())

        def check(queries):
            for now, filt, exp in queries:
                got = sorted(m.topic.decode() for m in st.dispatch(filt.encode(), now))
                assert got == sorted(exp), (case["name"], filt, now)

        for op in case["ops"]:
            apply(op)
        check(case["queries"])
        for op in case.get("then", []):
            apply(op)
        check(case.get("after", []))


VOCAB = [b"a", b"b", b"c", b"", b"$SYS", b"dev", b"x$", b"long-word-over-sixteen-bytes"]


def rand_topic(rng, maxd=6):
    return b"/".join(rng.choice(VOCAB) for _ in range(rng.randint(1, maxd)))


def rand_filter(rng, maxd=6):
    lv = [rng.choice(VOCAB + [b"+", b"+", b"nope"]) for _ in range(rng.randint(1, maxd))]
    r = rng.random()
    if r < 0.35:
        lv[-1] = b"#"
    elif r < 0.38:
        lv.insert(0, b"#")  # invalid: a non-final '#'
    return b"/".join(lv)


@pytest.mark.parametrize("seed", range(5))
def test_fuzz_parity(mod, seed):
    rng = random.Random(700 + seed)
    idx = mod.RetainIndex()
    names = sorted({rand_topic(rng) for _ in range(rng.randint(20, 400))})
    expiry = [rng.choice([0, 0, 0, 90, 100, 110]) for _ in names]
    ids = idx.store(names, expiry)
    assert list(ids) == list(range(len(names)))
    live = [True] * len(names)
    idx.commit()
    filters = [rand_filter(rng) for _ in range(700)] + [b"#", b"+", b"+/#", b"", b"/", b"$SYS/#"]
    for step in range(3):
        tt = RR.TokenTrie(names, expiry, live)
        for now in (100, -1, 0):
            got = idx.match(filters, now)
            for f, g in zip(filters, got):
                assert g == tt.dispatch(f, now), (step, f, now)
        # deletes, re-stores with a new expiry, new topics
        dead = rng.sample(range(len(names)), len(names) // 5)
        idx.delete(dead)
        for i in dead:
            live[i] = False
        back = rng.sample(dead, len(dead) // 2)
        for i in back:
            expiry[i] = rng.choice([0, 95, 105])
        idx.store([names[i] for i in back], [expiry[i] for i in back])
        for i in back:
            live[i] = True
        new = sorted({rand_topic(rng) for _ in range(40)} - set(names))
        nid = idx.store(new, [0] * len(new))
        assert list(nid) == list(range(len(names), len(names) + len(new)))
        names += new
        expiry += [0] * len(new)
        live += [True] * len(new)
        idx.commit()


def test_wide_fanout_and_root_hash(mod):
    idx = mod.RetainIndex()
    names = [b"w/%d/x" % i for i in range(20000)] + [b"w/%d/y/z" % i for i in range(0, 20000, 7)] + [b"$SYS/s"]
    idx.store(names)
    idx.commit()
    filters = [b"w/+/x", b"w/+/y/#", b"#", b"+/+/x", b"w/#", b"+/s", b"w/+/+/z", b"w/7/y/z"]
    tt = RR.TokenTrie(names, [0] * len(names))
    got = idx.match(filters, 1)
    for f, g in zip(filters, got):
        assert g == tt.dispatch(f, 1), f
    assert len(got[2]) == len(names)  # '#' selects '$SYS/...' too: the match spec has no '$' rule


def test_wide_records_under_guard_and_depth_floor(mod):
    """Checked records (expiry guard, '+'-then-'#' depth floor) of both sizes: the count pass
    keeps each one's live-rank mask and the write pass emits from it (retain_out_kernel)."""
    rng = random.Random(11)
    idx = mod.RetainIndex()
    names = [b"w/%d" % i for i in range(3000)] + [b"w/%d/x" % i for i in range(5000)]
    names += [b"w/%d/x/%d" % (i, j) for i in range(0, 300, 3) for j in range(rng.randint(1, 90))]
    names += [b"v/%d" % i for i in range(70)] + [b"v/%d/q" % i for i in range(40)]
    expiry = [rng.choice([0, 0, 90, 100, 110]) for _ in names]
    idx.store(names, expiry)
    idx.commit()
    filters = [b"#", b"w/#", b"w/+/#", b"+/+/#", b"w/+/x/#", b"v/+/#", b"v/#", b"w/+/x", b"+/+"]
    tt = RR.TokenTrie(names, expiry)
    for now in (100, -1, 95):
        for f, g in zip(filters, idx.match(filters, now)):
            assert g == tt.dispatch(f, now), (f, now)


def test_deep_topics(mod):
    rng = random.Random(3)
    idx = mod.RetainIndex()
    names = [b"/".join(b"l%d" % (j % 3) for j in range(rng.randint(50, 120))) for _ in range(200)]
    names = sorted(set(names))
    idx.store(names)
    idx.commit()
    filters = [b"/".join([b"+"] * 60) + b"/#", b"/".join([b"+"] * 100), b"l0/#", b"/".join([b"l0", b"l1", b"l2"] * 20)]
    filters += [b"/".join(rng.choice([b"l0", b"l1", b"l2", b"+"]) for _ in range(rng.randint(40, 130))) + b"/#"
                for _ in range(100)]
    tt = RR.TokenTrie(names, [0] * len(names))
    for f, g in zip(filters, idx.match(filters, 1)):
        assert g == tt.dispatch(f, 1)


def test_empty_index_and_batches(mod):
    idx = mod.RetainIndex()
    assert idx.match([b"#", b"a"], 5) == [[], []]
    idx.store([b"a"])
    idx.commit()
    assert idx.match([], 5) == []
    with pytest.raises(Exception):
        idx.store([b"a/+"])  # published topics carry no wildcard levels


def test_large_table_device_api(mod):
    """A config-B-scale store of retained topics (the topic generator of config B), 20k
    subscription filters from its filter generator, through the device entry point."""
    import torch
    from emqx_amd import workloads as W
    from emqx_amd.engine import pack
    wl = W.config_b(n_filters=20_000, n_topics=300_000, seed=31)
    names = sorted(set(W.unpack(wl.topics)))
    rng = np.random.default_rng(1)
    expiry = np.where(rng.random(len(names)) < 0.1, 1000 + rng.integers(0, 200, len(names)), 0).astype(np.int64)
    idx = mod.RetainIndex()
    idx.store_packed(*pack(names), expiry)
    idx.commit()
    filters = W.unpack(wl.filters)
    dev = torch.device("cuda:0")
    fb, fo = pack(filters)
    d_fb = torch.from_numpy(np.array(fb)).to(dev)
    d_fo = torch.from_numpy(fo.view(np.int64)).to(dev)
    d_off = torch.empty(len(filters) + 1, dtype=torch.int64, device=dev)
    cap = 4_000_000
    d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
    try:
        n = idx.match_device(d_fb.data_ptr(), d_fo.data_ptr(), len(filters), 1100, d_off.data_ptr(),
                             d_ids.data_ptr(), cap)
    except mod.EngineError as err:
        cap = err.needed
        d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
        n = idx.match_device(d_fb.data_ptr(), d_fo.data_ptr(), len(filters), 1100, d_off.data_ptr(),
                             d_ids.data_ptr(), cap)
    off = d_off.cpu().numpy().view(np.uint64)
    ids = d_ids[:n].cpu().numpy().view(np.uint32)
    tt = RR.TokenTrie(names, expiry.tolist())
    total = 0
    for i in range(0, len(filters), 3):
        g = sorted(ids[off[i]:off[i + 1]].tolist())
        x = tt.dispatch(filters[i], 1100)
        assert g == x, (i, filters[i])
        total += len(x)
    assert total > 0 and n == off[-1]
    st = idx.stats()
    assert st["n_live"] == len(names) and st["last_total"] == n


@pytest.mark.parametrize("budget", [1, 2, 7])
def test_spill_rounds_parity(mod, budget):
    """Load-balanced walk: with a tiny step budget every wave spills its stack and the items
    are dealt over many waves for round after round (emqx_retain_set_tuning "step_budget",
    "spill_rounds"; the rounds are enqueued without host round trips, the last one without a
    budget).  The result, the node-visit count and the range count must equal the unbudgeted
    walk's."""
    rng = random.Random(900 + budget)
    idx = mod.RetainIndex()
    names = sorted({rand_topic(rng) for _ in range(400)})
    names += [b"w/%d/x" % i for i in range(3000)] + [b"w/%d/y/z" % i for i in range(0, 3000, 7)]
    expiry = [rng.choice([0, 0, 0, 90, 100, 110]) for _ in names]
    idx.store(names, expiry)
    idx.commit()
    filters = [rand_filter(rng) for _ in range(500)] + [b"#", b"+", b"+/#", b"w/+/x", b"+/+/x", b"w/+/+/z"]
    tt = RR.TokenTrie(names, expiry)
    idx.set_tuning("balance", 0)  # the spill rounds (the default is the work-sharing walk)
    idx.set_tuning("step_budget", 0)
    ref = idx.match(filters, 100)
    st0 = idx.stats()
    assert st0["last_spill_rounds"] == 0
    idx.set_tuning("step_budget", budget)
    for rounds, spill_budget in ((0, 0), (1, 0), (6, 3), (40, 1), (46, 0)):
        idx.set_tuning("spill_rounds", rounds)
        idx.set_tuning("spill_budget", spill_budget)
        got = idx.match(filters, 100)
        st1 = idx.stats()
        assert 0 < st1["last_spill_rounds"] <= rounds + 1 and st1["last_spilled"] > 0
        assert st1["last_spill_full"] == 0
        assert st1["last_visits"] == st0["last_visits"] and st1["last_ranges"] == st0["last_ranges"]
        for f, g, r in zip(filters, got, ref):
            assert g == r == tt.dispatch(f, 100), f
    with pytest.raises(Exception):
        idx.set_tuning("spill_rounds", 47)


def test_spill_buffer_full_parity(mod):
    """A spill buffer too small for what the waves spill (emqx_retain_set_tuning "spill_cap"):
    a wave whose reservation does not fit walks its stack on itself, and the part of its
    reservation below the cap is padded with empty items the next round skips.  The result and
    the visit and range counts stay the unbudgeted walk's."""
    rng = random.Random(977)
    idx = mod.RetainIndex()
    names = sorted({rand_topic(rng) for _ in range(300)})
    names += [b"v/%d/x" % i for i in range(4000)] + [b"v/%d/y/%d" % (i, i % 5) for i in range(0, 4000, 3)]
    idx.store(names, [0] * len(names))
    idx.commit()
    filters = [rand_filter(rng) for _ in range(300)] + [b"#", b"+/+", b"v/+/x", b"+/+/y/+", b"v/#"] * 8
    tt = RR.TokenTrie(names, [0] * len(names))
    idx.set_tuning("balance", 0)
    idx.set_tuning("step_budget", 0)
    ref = idx.match(filters, 100)
    st0 = idx.stats()
    idx.set_tuning("step_budget", 1)
    idx.set_tuning("spill_budget", 1)
    idx.set_tuning("spill_rounds", 3)
    idx.set_tuning("spill_cap", 64)
    got = idx.match(filters, 100)
    st1 = idx.stats()
    assert st1["last_spill_full"] > 0 and st1["last_spill_rounds"] > 0
    assert st1["last_visits"] == st0["last_visits"] and st1["last_ranges"] == st0["last_ranges"]
    for f, g, r in zip(filters, got, ref):
        assert g == r == tt.dispatch(f, 100), f


def _sharing_case(seed):
    rng = random.Random(seed)
    names = sorted({rand_topic(rng) for _ in range(400)})
    names += [b"w/%d/x" % i for i in range(6000)] + [b"w/%d/y/z" % i for i in range(0, 6000, 7)]
    names += [b"q/%d/%d/e" % (i % 50, i) for i in range(4000)]
    expiry = [rng.choice([0, 0, 0, 90, 100, 110]) for _ in names]
    filters = [rand_filter(rng) for _ in range(500)]
    filters += [b"#", b"+", b"+/#", b"w/+/x", b"+/+/x", b"w/+/+/z", b"q/+/+/e", b"+/+/+/e", b"q/+/#"] * 3
    return names, expiry, filters


@pytest.mark.parametrize("balance", [1, 0])
def test_lane_map_modes_agree(mod, balance):
    """A walk step maps its lanes to its items by a ballot of the items' first lanes (tuning
    "lane_map" 1, the default) or by a binary search of the items' prefixes per lane (0, the
    round-5 A/B): same results, visits and ranges, in the work-sharing walk and in the spill
    rounds (whose padding items have no nodes and flag no lane)."""
    names, expiry, filters = _sharing_case(4242 + balance)
    idx = mod.RetainIndex()
    idx.store(names, expiry)
    idx.commit()
    tt = RR.TokenTrie(names, expiry)
    idx.set_tuning("balance", balance)
    if not balance:
        idx.set_tuning("step_budget", 2)
        idx.set_tuning("spill_cap", 64)
    out = {}
    for lm in (0, 1):
        idx.set_tuning("lane_map", lm)
        got = idx.match(filters, 100)
        st = idx.stats()
        out[lm] = (got, st["last_visits"], st["last_ranges"])
    assert out[0] == out[1]
    for f, g in zip(filters, out[1][0]):
        assert g == tt.dispatch(f, 100), f
    with pytest.raises(Exception):
        idx.set_tuning("lane_map", 2)


@pytest.mark.parametrize("piece,check,shards,roam", [(64, 1, 1, 0), (64, 2, 4, 3), (256, 8, 64, 8), (1024, 64, 16, 15),
                                                     (512, 4, 64, 0)])
def test_queue_sharing_parity(mod, piece, check, shards, roam):
    """The work-sharing walk (balance 1, the default): waves out of tiles wait on tickets of
    their shard's queue of shared pieces, busy waves share the bottom of their stacks every
    `check` steps while waves of their shard wait, in pieces of `piece` nodes.  Results, visit
    and range counts equal the one-wave-per-tile walk with no budget (balance 0, step_budget 0);
    the safety valve never fires.  Waves whose shard is done help `roam` other shards."""
    names, expiry, filters = _sharing_case(1300 + piece + check)
    idx = mod.RetainIndex()
    idx.store(names, expiry)
    idx.commit()
    tt = RR.TokenTrie(names, expiry)
    idx.set_tuning("balance", 0)
    idx.set_tuning("step_budget", 0)
    ref = idx.match(filters, 100)
    st0 = idx.stats()
    idx.set_tuning("balance", 1)
    idx.set_tuning("queue_piece", piece)
    idx.set_tuning("queue_check", check)
    idx.set_tuning("queue_shards", shards)
    idx.set_tuning("queue_roam", roam)
    shared = 0
    for tile in (10, 1, 64):
        idx.set_tuning("tile", tile)
        for _ in range(2):  # the queue is left all zero for the next call
            got = idx.match(filters, 100)
            st1 = idx.stats()
            assert st1["queue_aborts"] == 0 and st1["last_spill_rounds"] == 0
            assert st1["last_visits"] == st0["last_visits"] and st1["last_ranges"] == st0["last_ranges"]
            for f, g, r in zip(filters, got, ref):
                assert g == r == tt.dispatch(f, 100), (f, tile)
            shared += st1["last_shares"]
    if check <= 2:
        assert shared > 0
    for key, bad in (("queue_check", 3), ("queue_piece", 63), ("balance", 2), ("queue_shards", 0)):
        with pytest.raises(Exception):
            idx.set_tuning(key, bad)


def test_queue_full_parity(mod):
    """A queue too small for what the waves share (emqx_retain_set_tuning "queue_cap"): a share
    whose reservation does not fit is not made (the wave walks on), the tickets past the cap wait
    for the walk's end.  Same results and counts; then a full-size queue again."""
    names, expiry, filters = _sharing_case(1399)
    idx = mod.RetainIndex()
    idx.store(names, expiry)
    idx.commit()
    tt = RR.TokenTrie(names, expiry)
    idx.set_tuning("balance", 0)
    idx.set_tuning("step_budget", 0)
    ref = idx.match(filters, 100)
    st0 = idx.stats()
    idx.set_tuning("balance", 1)
    idx.set_tuning("queue_piece", 64)
    idx.set_tuning("queue_check", 1)
    idx.set_tuning("queue_shards", 4)
    for cap in (64, 4 << 20):
        idx.set_tuning("queue_cap", cap)
        got = idx.match(filters, 100)
        st1 = idx.stats()
        assert st1["queue_aborts"] == 0
        assert st1["last_visits"] == st0["last_visits"] and st1["last_ranges"] == st0["last_ranges"]
        if cap == 64:
            assert st1["last_spilled"] <= 64
        for f, g, r in zip(filters, got, ref):
            assert g == r == tt.dispatch(f, 100), (f, cap)


def test_queue_abort_reruns_in_spill_mode(mod):
    """The work-sharing walk's safety valve, forced: with the poll limit at 1
    (emqx_retain_set_tuning "queue_poll_limit") a waiting wave gives up after its second empty
    poll (RC_QABORT), the kernel drains, and the host reruns the call in spill-round mode
    (retain.cpp, queue_aborts counts it).  The reruns' results equal the oracle's; with the limit
    back, calls run without aborts and give the same results."""
    names, expiry, filters = _sharing_case(1401)
    idx = mod.RetainIndex()
    idx.store(names, expiry)
    idx.commit()
    tt = RR.TokenTrie(names, expiry)
    idx.set_tuning("balance", 1)
    idx.set_tuning("queue_check", 1)
    idx.set_tuning("queue_shards", 4)
    a0 = idx.stats()["queue_aborts"]
    idx.set_tuning("queue_poll_limit", 1)
    for _ in range(3):
        got = idx.match(filters, 100)
        for f, g in zip(filters, got):
            assert g == tt.dispatch(f, 100), f
    a1 = idx.stats()["queue_aborts"]
    assert a1 > a0
    idx.set_tuning("queue_poll_limit", 1 << 20)
    got = idx.match(filters, 100)
    assert idx.stats()["queue_aborts"] == a1
    for f, g in zip(filters, got):
        assert g == tt.dispatch(f, 100), f
    with pytest.raises(Exception):
        idx.set_tuning("queue_poll_limit", 0)


@pytest.mark.parametrize("tile", [1, 5, 64])
def test_tile_sizes_parity(mod, tile):
    """Filters per wave tile of the first walk round (emqx_retain_set_tuning "tile"): any
    size from 1 to 64 gives the oracle's sets and the same visit and range counts."""
    rng = random.Random(950 + tile)
    idx = mod.RetainIndex()
    names = sorted({rand_topic(rng) for _ in range(300)})
    expiry = [rng.choice([0, 0, 90, 110]) for _ in names]
    idx.store(names, expiry)
    idx.commit()
    filters = [rand_filter(rng) for _ in range(333)] + [b"#", b"+/#"]
    tt = RR.TokenTrie(names, expiry)
    idx.set_tuning("tile", 64)
    ref = idx.match(filters, 100)
    st0 = idx.stats()
    idx.set_tuning("tile", tile)
    got = idx.match(filters, 100)
    st1 = idx.stats()
    assert st1["last_visits"] == st0["last_visits"] and st1["last_ranges"] == st0["last_ranges"]
    for f, g, r in zip(filters, got, ref):
        assert g == r == tt.dispatch(f, 100), f


@pytest.mark.parametrize("search", [0, 1])
def test_search_variants_parity(mod, search):
    """The postings / per-depth rank-list slices are cut by two-level binary searches
    (search 0) or 16-ary search trees (search 1, several levels deep here: postings groups of
    thousands of nodes).  Both give the oracle's sets and the same visit and range counts."""
    rng = random.Random(1200 + search)
    names = sorted({b"/".join([b"r%d" % rng.randrange(6), b"m%d" % rng.randrange(400),
                               b"x%d" % rng.randrange(3), b"l%d" % rng.randrange(900)][: rng.randrange(2, 5)])
                    for _ in range(20000)})
    expiry = [rng.choice([0, 0, 0, 90, 110]) for _ in names]
    idx = mod.RetainIndex()
    idx.store(names, expiry)
    idx.commit()
    filters = [b"+/+/x1", b"+/+/x2/+", b"+/m7/+/#", b"r1/+/x0", b"+/+/+/l5", b"+/+/+", b"+/#", b"#", b"r2/+/+/+",
               b"+/m3", b"r3/m9/+/l1", b"+/+/x0/l77", b"+/m400/#"]
    filters += [b"/".join(rng.choice([b"+", b"r%d" % rng.randrange(6), b"m%d" % rng.randrange(400),
                                      b"x%d" % rng.randrange(3), b"l%d" % rng.randrange(900)])
                          for _ in range(rng.randrange(1, 5))) for _ in range(300)]
    tt = RR.TokenTrie(names, expiry)
    idx.set_tuning("search", 1 - search)
    ref = idx.match(filters, 100)
    st0 = idx.stats()
    idx.set_tuning("search", search)
    got = idx.match(filters, 100)
    st1 = idx.stats()
    assert st1["last_visits"] == st0["last_visits"] and st1["last_ranges"] == st0["last_ranges"]
    for f, g, r in zip(filters, got, ref):
        assert g == r == tt.dispatch(f, 100), f


@pytest.mark.parametrize("seed", range(3))
def test_match_spec_strict_guard_for_plain_filters(mod, seed):
    """match_messages/3 and page_read/4 run make_match_spec/1 for plain topics too, whose guard
    is Et > Now (emqx_retainer_mnesia.erl:233-246); dispatch/4 reads a plain topic with
    read_messages/1's Et >= Now (:197-208).  At expiry == now the two differ."""
    rng = random.Random(900 + seed)
    names = sorted({rand_topic(rng) for _ in range(300)})
    expiry = [rng.choice([0, 99, 100, 101]) for _ in names]
    idx = mod.RetainIndex()
    idx.store(names, expiry)
    idx.commit()
    tab = RR.RetainTable()
    for t, e in zip(names, expiry):
        tab.store(t, e)
    filters = names[::3] + [rand_filter(rng) for _ in range(200)]
    now = 100
    spec = idx.match(filters, now, match_spec=True)
    disp = idx.match(filters, now)
    for f, s_, d in zip(filters, spec, disp):
        assert s_ == sorted(tab.match_messages(f, now)), f
        assert d == sorted(tab.dispatch(f, now)), f
    at_now = [t for t, e in zip(names, expiry) if e == now]
    assert at_now
    for t in at_now:  # the expiry == now topic: dispatched, not selected by the match spec
        assert idx.match([t], now)[0] == [names.index(t)]
        assert idx.match([t], now, match_spec=True)[0] == []
    # and the mnesia mirror's page_read/4 on a plain topic follows the match spec
    st = mod.MnesiaRetainer()
    st.store_retained(mod.Message(b"p/q", b"x", 0, now))
    assert st.page_read(b"p/q", 1, 10, now=now) == []
    assert [m.topic for m in st.dispatch(b"p/q", now)] == [b"p/q"]


def test_concurrent_callers_parity(mod):
    """Calls from several host threads at once, each on its own stream and buffers (the R line
    runs two such callers): each call takes its own work area (its own queue shards), the
    work-sharing walks of concurrent calls share the GPU, and every result equals the oracle's."""
    import threading

    import torch
    from emqx_amd.engine import pack
    names, expiry, filters = _sharing_case(1444)
    idx = mod.RetainIndex()
    idx.store(names, expiry)
    idx.commit()
    tt = RR.TokenTrie(names, expiry)
    want = [tt.dispatch(f, 100) for f in filters]
    dev = torch.device("cuda:0")
    fb, fo = pack(filters)
    d_fb = torch.from_numpy(fb.copy()).to(dev)
    d_fo = torch.from_numpy(fo.view(np.int64).copy()).to(dev)
    n, cap, T, rounds = len(filters), 1 << 20, 3, 6
    streams = [torch.cuda.Stream(device=dev) for _ in range(T)]
    outs = [(torch.empty(n + 1, dtype=torch.int64, device=dev), torch.empty(cap, dtype=torch.int32, device=dev))
            for _ in range(T)]
    errs, bad = [], []

    def worker(t):
        try:
            off_d, ids_d = outs[t]
            for _ in range(rounds):
                tot = idx.match_device(d_fb.data_ptr(), d_fo.data_ptr(), n, 100, off_d.data_ptr(), ids_d.data_ptr(), cap,
                                       stream=streams[t].cuda_stream)
                off = off_d.cpu().numpy().view(np.uint64)
                ids = ids_d[:tot].cpu().numpy().view(np.uint32)
                for i in range(n):
                    if sorted(ids[off[i]:off[i + 1]].tolist()) != want[i]:
                        bad.append((t, i))
                        return
        except Exception as e:  # noqa: BLE001 - re-raised below
            errs.append(e)

    threads = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
    for th in threads:
        th.start()
    for th in threads:
        th.join()
    if errs:
        raise errs[0]
    assert not bad, bad[:5]
    assert idx.stats()["queue_aborts"] == 0
