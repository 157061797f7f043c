"""GPU parity of the publish fan-out (emqx_amd/csrc/fanout_kernels.hip) against the fan-out
oracle (oracle/broker_ref.py) and a direct restatement of the dispatch rules on config E.

Deliveries are compared per topic as sorted multisets of (filter, subscriber, shared).
Hash strategies are exact (keys = the caller's phash2 values); round_robin / sticky / random
are checked by their invariants (the reference's are per-process and randomly seeded)."""

import collections
import random

import numpy as np
import pytest

from oracle import broker_ref as B

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def F():
    import torch
    assert torch.cuda.is_available()
    from emqx_amd import fanout
    return fanout


def scenario_ops(seed, n_filters=60, n_subs=40, n_ops=600):
    rng = random.Random(seed)
    words = [b"a", b"b", b"c", b"", b"$SYS"]
    filters = set()
    while len(filters) < n_filters:
        d = rng.randint(1, 4)
        lv = [rng.choice(words + [b"+"]) for _ in range(d)]
        if rng.random() < 0.3:
            lv.append(b"#")
        filters.add(b"/".join(lv))
    filters = sorted(filters)
    ops = []
    for _ in range(n_ops):
        f = rng.choice(filters)
        s = "s%d" % rng.randrange(n_subs)
        g = rng.choice([None, None, b"g1", b"g2"])
        ops.append(("sub" if rng.random() < 0.85 else "unsub", f, s, g))
    topics = []
    for _ in range(300):
        d = rng.randint(1, 5)
        topics.append(b"/".join(rng.choice(words) for _ in range(d)))
    topics += [b"a/+", b"#", b"$SYS/a"]
    return ops, topics


def canon(rows):
    return sorted((f, str(s), sh) for f, s, sh in rows)


@pytest.mark.parametrize("seed", range(4))
@pytest.mark.parametrize("strategy", [B.HASH_CLIENTID, B.HASH_TOPIC])
def test_broker_hash_strategies_exact(F, seed, strategy):
    ops, topics = scenario_ops(seed)
    ref = B.Broker()
    dev = F.Broker(0, node=B.NODE, strategy=strategy)
    for op, f, s, g in ops:
        getattr(ref, "subscribe" if op == "sub" else "unsubscribe")(f, s, g)
        getattr(dev, "subscribe" if op == "sub" else "unsubscribe")(f, s, g)
    keys = [random.Random(seed * 7 + i).randrange(1 << 27) for i in range(len(topics))]
    got = dev.publish_batch(topics, keys)
    for t, k, row in zip(topics, keys, got):
        assert canon(row) == canon(ref.publish(t, k, strategy)), t


def test_two_messages_scenarios(F):
    """emqx_shared_sub_SUITE test_two_messages/2 on the device for every strategy."""
    for name in ["random", "round_robin", "sticky", "hash", "hash_clientid"]:
        b = F.Broker(0, strategy=name)
        b.subscribe(b"foo/bar", "ConnPid1", share=b"group1")
        b.subscribe(b"foo/bar", "ConnPid2", share=b"group1")
        r1 = b.publish(b"foo/bar", key=99)
        r2 = b.publish(b"foo/bar", key=99)
        assert len(r1) == len(r2) == 1 and r1[0][2] and r2[0][2]
        if name == "sticky" or name.startswith("hash"):
            assert r1[0][1] == r2[0][1], name
        if name == "round_robin":
            assert r1[0][1] != r2[0][1]


def test_not_so_sticky_and_dispatch(F):
    b = F.Broker(0, strategy="sticky")
    assert b.publish(b"foo/bar") == []
    b.subscribe(b"foo/bar", "C1", share=b"group1")
    assert b.publish(b"foo/bar") == [(b"foo/bar", "C1", True)]
    b.unsubscribe(b"foo/bar", "C1", share=b"group1")
    b.subscribe(b"foo/#", "C1", share=b"group1")
    assert b.publish(b"foo/bar") == [(b"foo/#", "C1", True)]
    # a sticky member that leaves but stays alive keeps the publisher's messages
    # (is_active_sub/2 is process liveness, emqx_shared_sub.erl:234-240,385-393); once its
    # process is down it is replaced by another member
    b.subscribe(b"foo/#", "C2", share=b"group1")
    first = b.publish(b"foo/bar")[0][1]
    b.unsubscribe(b"foo/#", first, share=b"group1")
    other = "C2" if first == "C1" else "C1"
    assert [b.publish(b"foo/bar")[0][1] for _ in range(3)] == [first] * 3
    b.down(first)
    assert [b.publish(b"foo/bar")[0][1] for _ in range(3)] == [other] * 3


def test_round_robin_and_random_invariants(F):
    b = F.Broker(0, strategy="round_robin")
    members = ["m%d" % i for i in range(5)]
    for m in members:
        b.subscribe(b"x/+", m, share=b"g")
    b.subscribe(b"x/+", "lone", share=b"solo")
    topics = [b"x/%d" % i for i in range(1000)]
    rows = b.publish_batch(topics)
    picks = collections.Counter(r[1] for row in rows for r in row if r[0] == b"x/+" and r[1] != "lone")
    assert sum(picks.values()) == 1000 and set(picks) == set(members)
    assert all(v == 200 for v in picks.values())  # 1000 consecutive counter values, 5 members
    assert all(sum(1 for r in row if r[1] == "lone") == 1 for row in rows)
    rows = b.publish_batch(topics, strategy="random")
    picks = collections.Counter(r[1] for row in rows for r in row if r[1] != "lone")
    assert set(picks) == set(members) and min(picks.values()) > 120


def expected_fanout(moff, mids, fw, keys, lo, hi):
    """Per-topic sorted (sub, filter|shared_bit) pairs for topics [lo, hi) with hash picks:
    plain subscribers of each matched filter, plus lists:nth(1 + key rem N, Members) for each
    group (members in subscription order)."""
    from emqx_amd.workloads import NO_GROUP
    plain = collections.defaultdict(list)
    groups = collections.defaultdict(dict)
    for f, s, g in zip(fw.sub_filter.tolist(), fw.sub_id.tolist(), fw.sub_group.tolist()):
        if g == NO_GROUP:
            plain[f].append(s)
        else:
            groups[f].setdefault(g, []).append(s)
    out = []
    for t in range(lo, hi):
        row = []
        for f in mids[moff[t]:moff[t + 1]].tolist():
            row += [(s, f) for s in plain.get(f, [])]
            for g, mem in groups.get(f, {}).items():
                row.append((mem[keys[t] % len(mem)], f | 0x80000000))
        out.append(sorted(row))
    return out


def test_config_e_reduced_device_pipeline(F):
    """Config E generator at reduced scale through the device-pointer API: match CSR in HBM ->
    emqx_fanout_batch_device -> compared with the dispatch rules applied to the same CSR."""
    import torch
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine
    fw = W.config_e(n_filters=200_000, n_subscribers=100_000, n_topics=50_000, seed=5)
    eng = Engine(0)
    eng.insert_packed(*fw.wl.filters)
    eng.commit()
    st = F.SubTable(0)
    st.add(fw.sub_filter, fw.sub_id, fw.sub_group)
    st.commit()
    stats = st.stats()
    assert stats["plain"] + stats["shared_members"] == fw.n_subscriptions
    dev = torch.device("cuda", 0)
    tb = torch.from_numpy(fw.wl.topics[0]).to(dev)
    to = torch.from_numpy(fw.wl.topics[1].view(np.int64)).to(dev)
    n = fw.wl.n_topics
    moff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    mids = torch.empty(64 * n, dtype=torch.int32, device=dev)
    nm = eng.match_device(tb.data_ptr(), to.data_ptr(), n, moff.data_ptr(), mids.data_ptr(), 64 * n)
    keys = torch.from_numpy(fw.keys.view(np.int32)).to(dev)
    ooff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    with pytest.raises(Exception) as ei:
        st.fanout_device("hash_clientid", moff.data_ptr(), mids.data_ptr(), n, keys.data_ptr(), ooff.data_ptr(),
                         0, 0, 0)
    need = ei.value.needed
    osubs = torch.empty(need, dtype=torch.int32, device=dev)
    ofil = torch.empty(need, dtype=torch.int32, device=dev)
    tot = st.fanout_device("hash_clientid", moff.data_ptr(), mids.data_ptr(), n, keys.data_ptr(), ooff.data_ptr(),
                           osubs.data_ptr(), ofil.data_ptr(), need)
    torch.cuda.synchronize()
    assert tot == need
    mo, mi = moff.cpu().numpy(), mids[:nm].cpu().numpy().view(np.uint32)
    oo, os_, of = ooff.cpu().numpy(), osubs.cpu().numpy().view(np.uint32), ofil.cpu().numpy().view(np.uint32)
    assert oo[0] == 0 and oo[-1] == tot and np.all(np.diff(oo) >= 0)
    exp = expected_fanout(mo, mi, fw, fw.keys, 0, 4000)
    for t in range(4000):
        got = sorted(zip(os_[oo[t]:oo[t + 1]].tolist(), of[oo[t]:oo[t + 1]].tolist()))
        assert got == exp[t], t
    # whole batch: per-topic delivery counts
    from emqx_amd.workloads import NO_GROUP
    per_f = np.zeros(fw.wl.n_filters, dtype=np.int64)
    np.add.at(per_f, fw.sub_filter[fw.sub_group == NO_GROUP].astype(np.int64), 1)
    gk = np.unique((fw.sub_filter[fw.sub_group != NO_GROUP].astype(np.uint64) << np.uint64(8))
                   | fw.sub_group[fw.sub_group != NO_GROUP].astype(np.uint64))
    np.add.at(per_f, (gk >> np.uint64(8)).astype(np.int64), 1)
    cnt = np.add.reduceat(per_f[mi.astype(np.int64)], mo[:-1].astype(np.int64)) if nm else np.zeros(n)
    cnt = np.where(np.diff(mo) > 0, cnt, 0)
    assert np.array_equal(np.diff(oo), cnt)


def test_empty_batches_and_tables(F):
    from emqx_amd.engine import Engine
    eng = Engine(0)
    st = F.SubTable(0)
    off, subs, fils = F.publish_packed(eng, st, "round_robin", np.zeros(1, np.uint8), np.zeros(1, np.uint64))
    assert len(off) == 1 and off[0] == 0 and subs.size == 0
    eng.insert([b"a/#"])
    eng.commit()
    from emqx_amd.engine import pack
    off, subs, fils = F.publish_packed(eng, st, "round_robin", *pack([b"a/b", b"a"]))
    assert list(off) == [0, 0, 0]
    with pytest.raises(Exception):  # hash strategies need keys
        F.publish_packed(eng, st, "hash_topic", *pack([b"a/b"]))


def test_async_fanout_pipelined_streams(F):
    """emqx_fanout_batch_device_async: match + fan-out enqueued on three streams without host
    synchronisation equals the synchronous call; an undersized output sets the overflow flag
    and writes nothing; a CSR slice whose offsets do not start at 0 (moff[0] > 0) is read
    from its own base."""
    import torch
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine
    fw = W.config_e(n_filters=100_000, n_subscribers=50_000, n_topics=20_000, seed=6)
    eng = Engine(0)
    eng.insert_packed(*fw.wl.filters)
    eng.commit()
    st = F.SubTable(0)
    st.add(fw.sub_filter, fw.sub_id, fw.sub_group)
    st.commit()
    dev = torch.device("cuda", 0)
    tb = torch.from_numpy(fw.wl.topics[0]).to(dev)
    to = torch.from_numpy(fw.wl.topics[1].view(np.int64)).to(dev)
    keys = torch.from_numpy(fw.keys.view(np.int32)).to(dev)
    n = fw.wl.n_topics
    mcap = 64 * n
    moff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    mids = torch.empty(mcap, dtype=torch.int32, device=dev)
    nm = eng.match_device(tb.data_ptr(), to.data_ptr(), n, moff.data_ptr(), mids.data_ptr(), mcap)
    ooff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    cap = 64 * n
    osubs = torch.empty(cap, dtype=torch.int32, device=dev)
    ofil = torch.empty(cap, dtype=torch.int32, device=dev)
    tot = st.fanout_device("hash_clientid", moff.data_ptr(), mids.data_ptr(), n, keys.data_ptr(), ooff.data_ptr(),
                           osubs.data_ptr(), ofil.data_ptr(), cap)
    ref = (ooff.cpu().numpy(), osubs[:tot].cpu().numpy(), ofil[:tot].cpu().numpy())

    streams = [torch.cuda.Stream(device=dev) for _ in range(3)]
    outs = [[torch.empty_like(t) for t in (moff, mids, ooff, osubs, ofil)] for _ in streams]
    summ = torch.zeros((6, st.SUMMARY_WORDS), dtype=torch.int64, device=dev)
    msum = torch.zeros((6, eng.SUMMARY_WORDS), dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    for k in range(6):
        j = k % 3
        mo, mi, oo, os_, of = outs[j]
        s = streams[j].cuda_stream
        eng.match_device_async(tb.data_ptr(), to.data_ptr(), n, mo.data_ptr(), mi.data_ptr(), mcap,
                               msum[k].data_ptr(), stream=s)
        st.fanout_device_async("hash_clientid", mo.data_ptr(), mi.data_ptr(), n, mcap, keys.data_ptr(),
                               oo.data_ptr(), os_.data_ptr(), of.data_ptr(), cap, summ[k].data_ptr(), stream=s)
    torch.cuda.synchronize()
    sm = summ.cpu().numpy()
    assert (sm[:, 0] == 0).all() and (sm[:, 1] == tot).all() and (sm[:, 2] == nm).all()
    for mo, mi, oo, os_, of in outs:
        assert np.array_equal(oo.cpu().numpy(), ref[0])
        assert np.array_equal(os_[:tot].cpu().numpy(), ref[1])
        assert np.array_equal(of[:tot].cpu().numpy(), ref[2])

    # overflow: flag set, the total reported, the offsets complete, the id arrays untouched
    osubs.fill_(-7)
    ooff.fill_(-7)
    st.fanout_device_async("hash_clientid", moff.data_ptr(), mids.data_ptr(), n, mcap, keys.data_ptr(),
                           ooff.data_ptr(), osubs.data_ptr(), ofil.data_ptr(), tot - 1, summ[0].data_ptr())
    torch.cuda.synchronize()
    s0 = summ[0].cpu().numpy()
    assert s0[0] & 1 and s0[1] == tot
    assert (osubs.cpu().numpy() == -7).all()
    assert np.array_equal(ooff.cpu().numpy(), ref[0])

    # a slice of the CSR (topics [h, n)): offsets start at moff[h] > 0
    h = n // 2
    oo_ref = ref[0]
    sl = st.fanout_device("hash_clientid", moff[h:].data_ptr(), mids.data_ptr(), n - h, keys[h:].data_ptr(),
                          ooff.data_ptr(), osubs.data_ptr(), ofil.data_ptr(), cap)
    assert sl == int(oo_ref[n] - oo_ref[h])
    assert np.array_equal(osubs[:sl].cpu().numpy(), ref[1][oo_ref[h]:])
    assert np.array_equal(ooff[:n - h + 1].cpu().numpy(), oo_ref[h:] - oo_ref[h])


def test_publish_batch_overflow_retry_10k_subscribers():
    """emqx_publish_batch on a topic with 10K subscribers (plus a $share group) through the
    NIF's protocol (emqx_amd/csrc/nif/grow_retry.h): the 64-per-topic first guess overflows,
    n_out reports the deliveries needed, the retry at that size returns every subscriber
    (emqx_broker.erl:500-524) and one pick of the group (emqx_shared_sub.erl:251-288)."""
    import ctypes
    import torch  # noqa: F401
    from emqx_amd import _lib
    from emqx_amd.engine import Engine, pack
    from emqx_amd.fanout import SubTable
    e = Engine()
    ids = e.insert([b"hot/topic", b"hot/+", b"other/x"])
    e.commit()
    st = SubTable()
    subs = np.arange(10_000, dtype=np.uint32)
    st.add(np.full(10_000, ids[0], np.uint32), subs)
    st.add(np.full(5, ids[1], np.uint32), np.arange(20_000, 20_005, dtype=np.uint32), np.full(5, 3, np.uint32))
    st.add(np.array([ids[2]], np.uint32), np.array([7], np.uint32))
    st.commit()
    buf, offs = pack([b"hot/topic", b"other/x"])
    keys = np.array([11, 12], np.uint32)
    L = _lib.lib()
    out_off = np.zeros(3, np.uint64)
    cap = 64 * 2 + 64
    n_out = ctypes.c_uint64(0)
    sb, fb = np.zeros(cap, np.uint32), np.zeros(cap, np.uint32)
    rc = L.emqx_publish_batch(e._h, st.handle, _lib.SHARE_HASH_CLIENTID, buf.ctypes.data, offs.ctypes.data, 2,
                              keys.ctypes.data, out_off.ctypes.data, sb.ctypes.data, fb.ctypes.data, cap,
                              ctypes.byref(n_out))
    assert rc == _lib.EMQX_EOVERFLOW and n_out.value == 10_000 + 1 + 1
    cap = int(n_out.value)
    sb, fb = np.zeros(cap, np.uint32), np.zeros(cap, np.uint32)
    rc = L.emqx_publish_batch(e._h, st.handle, _lib.SHARE_HASH_CLIENTID, buf.ctypes.data, offs.ctypes.data, 2,
                              keys.ctypes.data, out_off.ctypes.data, sb.ctypes.data, fb.ctypes.data, cap,
                              ctypes.byref(n_out))
    assert rc == 0 and out_off.tolist() == [0, 10_001, 10_002]
    first = sb[:10_001]
    plain = first[(fb[:10_001] & _lib.FANOUT_SHARED_BIT) == 0]
    shared = first[(fb[:10_001] & _lib.FANOUT_SHARED_BIT) != 0]
    assert sorted(plain.tolist()) == subs.tolist()
    assert shared.tolist() == [20_000 + 11 % 5]   # hash_clientid: lists:nth(1 + Key rem N, Members)
    assert sb[10_001] == 7


def test_config_e_full_size_id_for_id(F):
    """Config E at its full size (SURVEY §8 d: 2M filters, 1M subscribers x 10 = 10M
    subscriptions, 10% in $share groups): a 100K-topic batch matched and fanned out on the
    device (hash_clientid), every topic's (subscriber, filter) multiset compared ID-for-ID with
    the C++ restatement of route/aggre/do_dispatch (oracle/fanout_oracle.cpp) over the C++ DFS's
    match CSR — and that match CSR with the device's."""
    import os
    import torch
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine
    from oracle import cpp as C
    threads = min(16, os.cpu_count() or 4)
    fw = W.config_e(n_topics=100_000)
    assert fw.n_subscriptions > 9_900_000 and fw.wl.n_filters == 2_000_000
    eng = Engine(0)
    eng.insert_packed(*fw.wl.filters)
    eng.commit()
    st = F.SubTable(0)
    st.add(fw.sub_filter, fw.sub_id, fw.sub_group)
    st.commit()
    dev = torch.device("cuda", 0)
    n = fw.wl.n_topics
    tb = torch.from_numpy(fw.wl.topics[0]).to(dev)
    to = torch.from_numpy(fw.wl.topics[1].view(np.int64)).to(dev)
    moff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    mids = torch.empty(64 * n, dtype=torch.int32, device=dev)
    nm = eng.match_device(tb.data_ptr(), to.data_ptr(), n, moff.data_ptr(), mids.data_ptr(), 64 * n)
    keys = torch.from_numpy(fw.keys.view(np.int32)).to(dev)
    ooff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    with pytest.raises(Exception) as ei:
        st.fanout_device("hash_clientid", moff.data_ptr(), mids.data_ptr(), n, keys.data_ptr(), ooff.data_ptr(),
                         0, 0, 0)
    need = ei.value.needed
    osubs = torch.empty(need, dtype=torch.int32, device=dev)
    ofil = torch.empty(need, dtype=torch.int32, device=dev)
    tot = st.fanout_device("hash_clientid", moff.data_ptr(), mids.data_ptr(), n, keys.data_ptr(), ooff.data_ptr(),
                           osubs.data_ptr(), ofil.data_ptr(), need)
    torch.cuda.synchronize()
    assert tot == need > 30 * n
    # the match CSR against the C++ DFS
    o = C.CppOracle(True)
    o.add_packed(*fw.wl.filters)
    off_o, ids_o, _ = o.match_csr(*fw.wl.topics, mode=C.MODE_ROUTES, threads=threads)
    mo = moff.cpu().numpy().view(np.uint64)
    assert C.csr_mismatches(mo, mids[:nm].cpu().numpy().view(np.uint32), off_o, ids_o).size == 0
    # deliveries, ID-for-ID per topic
    fo = C.FanoutOracle(fw.sub_filter, fw.sub_id, fw.sub_group)
    off_d, subs_d, fils_d = fo.publish_list(off_o, ids_o, fw.keys, threads=threads)
    oo = ooff.cpu().numpy().view(np.uint64)
    bad = C.pair_csr_mismatches(oo, osubs.cpu().numpy().view(np.uint32), ofil.cpu().numpy().view(np.uint32),
                                off_d, subs_d, fils_d)
    assert bad.size == 0, bad[:10]


@pytest.mark.parametrize("publishers", [1, 3, 5000])
def test_round_robin_seeded_zero_pick_exact(F, publishers):
    """emqx_subtab "rr_seed0" (SURVEY §8 d: config E's round_robin, counter seeded 0): every pick of
    two consecutive calls (the state carried over) equals the oracle's restatement of
    do_pick_subscriber/6 (oracle/fanout_oracle.cpp orf_publish_list_rr, itself checked against
    broker_ref in tests/test_fanout_oracle.py) — one publisher (one long run per group: the
    large resolve path), a few, and many (short runs); forgetting the publishers restarts them."""
    import torch
    from oracle import cpp as C
    rng = np.random.default_rng(publishers)
    nf, rows = 3000, []
    for f in range(nf):
        for s in rng.choice(100_000, size=int(rng.integers(0, 4)), replace=False):
            rows.append((f, int(s), 0xFFFFFFFF))
        for g in range(int(rng.integers(0, 3))):
            for s in rng.choice(100_000, size=int(rng.integers(1, 17)), replace=False):
                rows.append((f, int(s), g))
    filt, sub, grp = (np.array(x, np.uint32) for x in zip(*rows))
    st = F.SubTable(0)
    st.set_tuning("rr_seed0", 1)
    st.add(filt, sub, grp)
    st.commit()
    fo = C.FanoutOracle(filt, sub, grp)
    n = 20_000
    counts = rng.integers(0, 6, size=n)
    moff = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    mids = rng.integers(0, nf, size=int(moff[-1])).astype(np.uint32)
    keys = rng.integers(0, publishers, size=n).astype(np.uint32)
    dev = torch.device("cuda:0")
    d_moff = torch.from_numpy(moff.view(np.int64)).to(dev)
    d_mids = torch.from_numpy(mids.view(np.int32)).to(dev)
    d_keys = torch.from_numpy(keys.view(np.int32)).to(dev)
    cap = 64 * n
    ooff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    osubs = torch.empty(cap, dtype=torch.int32, device=dev)
    ofil = torch.empty(cap, dtype=torch.int32, device=dev)
    for call in range(3):
        if call == 2:  # forgotten: both sides start again from the first member
            st.forget_publishers(np.unique(keys))
            fo.rr_reset()
        nd = st.fanout_device("round_robin", d_moff.data_ptr(), d_mids.data_ptr(), n, d_keys.data_ptr(),
                              ooff.data_ptr(), osubs.data_ptr(), ofil.data_ptr(), cap)
        off_o, subs_o, fils_o = fo.publish_list(moff, mids, keys, round_robin=True)
        assert nd == len(subs_o)
        bad = C.pair_csr_mismatches(ooff.cpu().numpy().view(np.uint64), osubs[:nd].cpu().numpy().view(np.uint32),
                                    ofil[:nd].cpu().numpy().view(np.uint32), off_o, subs_o, fils_o)
        assert bad.size == 0, (call, bad[:10])
    st.close()
