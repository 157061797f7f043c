"""GPU tests of round 3's fan-out paths (emqx_amd/csrc/fanout.cpp, fanout_kernels.hip):

* incremental subscription-table commits (patched in place, lists moved when they outgrow their
  extent, compaction) against the fan-out oracle (oracle/broker_ref.py) after every commit, and
  against a table built in one commit from the same subscriptions;
* round_robin / sticky state per (group, publisher), as the reference keeps it in the
  publishing process's dictionary (apps/emqx/src/emqx_shared_sub.erl:234-247,279-285): several
  publishers interleaved in one batch and across batches, checked pick by pick against the
  oracle, which replays each rand draw the device made (and checks it drew from the right
  candidates);
* an over-capacity call consumes no pick state;
* the cross-caller publish batcher (emqx_pub_batcher) from many threads against publish_batch.
"""

import collections
import random
import threading

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


def canon(rows):
    return sorted((f, str(s), sh) for f, s, sh in rows)


def rand_topic_filter(rng, words, plus=True):
    d = rng.randint(1, 4)
    lv = [rng.choice(words + ([b"+"] if plus else [])) for _ in range(d)]
    if plus and rng.random() < 0.3:
        lv.append(b"#")
    return b"/".join(lv)


@pytest.mark.parametrize("seed", range(3))
def test_incremental_commits_match_oracle_every_round(F, seed):
    """Rounds of subscribe/unsubscribe (plain and $share, a few hot filters whose lists outgrow
    their extents many times) with a commit after each round; hash picks are exact, so every
    topic's deliveries must equal the oracle's after every commit."""
    rng = random.Random(100 + seed)
    words = [b"a", b"b", b"c", b"", b"$SYS"]
    filters = sorted({rand_topic_filter(rng, words) for _ in range(80)})
    hot = filters[:3]
    topics = sorted({rand_topic_filter(rng, words, plus=False) for _ in range(200)}) + [b"a/+", b"#"]
    ref = B.Broker()
    dev = F.Broker(0, node=B.NODE, strategy="hash_clientid")
    live = set()
    kinds = []
    for rnd in range(12):
        for _ in range(rng.randint(50, 400)):
            f = rng.choice(hot) if rng.random() < 0.4 else rng.choice(filters)
            s = "s%d" % rng.randrange(300)
            g = rng.choice([None, None, None, b"g1", b"g2", b"g3"])
            if (f, s, g) in live and rng.random() < 0.45:
                live.discard((f, s, g))
                ref.unsubscribe(f, s, g)
                dev.unsubscribe(f, s, g)
            else:
                live.add((f, s, g))
                ref.subscribe(f, s, g)
                dev.subscribe(f, s, g)
        keys = [rng.randrange(1 << 27) for _ in topics]
        got = dev.publish_batch(topics, keys)
        kinds.append(dev.subs.commit_stats()["kind"])
        for t, k, row in zip(topics, keys, got):
            assert canon(row) == canon(ref.publish(t, k, B.HASH_CLIENTID)), (rnd, t)
    st = dev.subs.commit_stats()
    assert st["commits"] >= 12 and st["moves"] > 0
    assert 1 in kinds[1:]  # later rounds patch in place


@pytest.mark.parametrize("small", [1, 0])
def test_inline_list_boundaries_every_commit(F, small):
    """Device records hold up to FO_INLINE = 7 plain subscribers inline (fanout.h DevRec: three in
    the head, four in ext).  Each round moves every filter's plain count to a fresh target in
    0..11 (across the 3/4 head boundary and the 7/8 inline boundary, both ways), some filters
    also carry a $share group (never inline); after every commit each topic's deliveries must
    equal the oracle's, through the one-launch small path (small = 1) and the batched fan-out
    kernels (small = 0)."""
    rng = random.Random(7 + small)
    filters = [b"x/%d" % i for i in range(40)] + [b"x/+", b"y/#"]
    topics = [b"x/%d" % i for i in range(40)] + [b"y/z", b"x/none"]
    ref = B.Broker()
    dev = F.Broker(0, node=B.NODE, strategy="hash_clientid")
    dev.router.engine.set_tuning("small_batch", small)
    plain = {f: [] for f in filters}
    for rnd in range(10):
        for f in filters:
            want = rng.randint(0, 11)
            while len(plain[f]) > want:
                s = plain[f].pop(rng.randrange(len(plain[f])))
                ref.unsubscribe(f, s)
                dev.unsubscribe(f, s)
            while len(plain[f]) < want:
                s = "s%d" % rng.randrange(500)
                if s in plain[f]:
                    continue
                plain[f].append(s)
                ref.subscribe(f, s)
                dev.subscribe(f, s)
            if rng.random() < 0.1:
                s = "m%d" % rng.randrange(20)
                ref.subscribe(f, s, b"g")
                dev.subscribe(f, s, b"g")
        keys = [rng.randrange(1 << 27) for _ in topics]
        got = dev.publish_batch(topics, keys)
        for t, k, row in zip(topics, keys, got):
            assert canon(row) == canon(ref.publish(t, k, B.HASH_CLIENTID)), (rnd, t)


def test_config_e_churn_equals_one_shot_build(F):
    """Config E's generator (reduced): the table built by 20 incremental commits of 4K-op churn
    (unsubscribes and resubscribes, plain and shared) gives the same deliveries per topic as a
    table built in one commit from the final subscriptions; each commit writes words and records
    in proportion to its ops, not to the table."""
    import torch
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine
    fw = W.config_e(n_filters=100_000, n_subscribers=40_000, n_topics=20_000, seed=9)
    eng = Engine(0)
    eng.insert_packed(*fw.wl.filters)
    eng.commit()
    st = F.SubTable(0)
    st.add(fw.sub_filter, fw.sub_id, fw.sub_group)
    st.commit()
    rng = np.random.default_rng(3)
    plain_idx = np.flatnonzero(fw.sub_group == W.NO_GROUP)
    shared_idx = np.flatnonzero(fw.sub_group != W.NO_GROUP)
    present = np.ones(len(fw.sub_id), bool)
    words = []
    extra_plain, extra_shared = [], []
    next_sub = 2_000_000
    for _ in range(20):
        # plain churn: unsubscribes and re-subscribes (plain order carries no meaning)
        idx = rng.choice(plain_idx, 4000, replace=False)
        rem = idx[present[idx]][:2000]
        add = idx[~present[idx]]
        st.remove(fw.sub_filter[rem], fw.sub_id[rem])
        present[rem] = False
        st.add(fw.sub_filter[add], fw.sub_id[add])
        present[add] = True
        # new subscriptions concentrated on 2000 filters: their lists outgrow extents and move
        nf = rng.integers(0, 2000, 1500).astype(np.uint32)
        ns = rng.integers(0, 40_000, 1500).astype(np.uint32) + np.uint32(1_000_000)
        st.add(nf, ns)
        extra_plain.append((nf, ns))
        # new members appended to existing $share groups (subscription order is kept)
        gi = rng.choice(shared_idx, 300)
        gs = np.arange(next_sub, next_sub + 300, dtype=np.uint32)
        next_sub += 300
        st.add(fw.sub_filter[gi], gs, fw.sub_group[gi])
        extra_shared.append((fw.sub_filter[gi], gs, fw.sub_group[gi]))
        before = st.commit_stats()
        st.commit()
        after = st.commit_stats()
        assert after["kind"] == 1
        words.append(after["words"] - before["words"] + after["records"] - before["records"])
    assert max(words) < 200_000, words  # each commit: its own ops (plus moved lists), not 10^6 words

    one = F.SubTable(0)  # the same subscriptions, in subscription order, one commit
    one.add(fw.sub_filter[present], fw.sub_id[present], fw.sub_group[present])
    for nf, ns in extra_plain:
        one.add(nf, ns)
    for gf, gs, gg in extra_shared:
        one.add(gf, gs, gg)
    one.commit()
    assert one.commit_stats()["kind"] == 0
    assert one.stats()["plain"] == st.stats()["plain"]
    assert one.stats()["shared_members"] == st.stats()["shared_members"]

    dev = torch.device("cuda", 0)
    tb = torch.from_numpy(fw.wl.topics[0]).to(dev)
    to = torch.from_numpy(fw.wl.topics[1].view(np.int64)).to(dev)
    n = fw.wl.n_topics
    moff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    mids = torch.empty(64 * n, dtype=torch.int32, device=dev)
    eng.match_device(tb.data_ptr(), to.data_ptr(), n, moff.data_ptr(), mids.data_ptr(), 64 * n)
    keys = torch.from_numpy(fw.keys.view(np.int32)).to(dev)
    outs = []
    for table in (st, one):
        cap = 256 * n
        ooff = torch.empty(n + 1, dtype=torch.int64, device=dev)
        osubs = torch.empty(cap, dtype=torch.int32, device=dev)
        ofil = torch.empty(cap, dtype=torch.int32, device=dev)
        tot = table.fanout_device("hash_clientid", moff.data_ptr(), mids.data_ptr(), n, keys.data_ptr(),
                                  ooff.data_ptr(), osubs.data_ptr(), ofil.data_ptr(), cap)
        outs.append((ooff.cpu().numpy(), osubs[:tot].cpu().numpy(), ofil[:tot].cpu().numpy()))
    (o1, s1, f1), (o2, s2, f2) = outs
    assert np.array_equal(o1, o2)
    for t in range(n):
        a = sorted(zip(s1[o1[t]:o1[t + 1]].tolist(), f1[o1[t]:o1[t + 1]].tolist()))
        b = sorted(zip(s2[o2[t]:o2[t + 1]].tolist(), f2[o2[t]:o2[t + 1]].tolist()))
        assert a == b, t


def build_groups(F, strategy):
    b = F.Broker(0, node=B.NODE, strategy=strategy)
    r = B.Broker()
    for m in ["m%d" % i for i in range(5)]:
        b.subscribe(b"x/+", m, share=b"g")
        r.subscribe(b"x/+", m, b"g")
    for m in ["k%d" % i for i in range(3)]:
        b.subscribe(b"x/#", m, share=b"h")
        r.subscribe(b"x/#", m, b"h")
    b.subscribe(b"x/#", "plain")
    r.subscribe(b"x/#", "plain")
    return b, r


def replay(dev_pick, firsts=None, key=None):
    """A draw for the oracle: the index of the device's pick among the reference's candidates
    (rand:uniform's draw), failing when the device picked outside them.  ``dev_pick`` may be a
    list (the device's $share deliveries of one filter, several groups): the one among the
    candidates is the draw."""
    def draw(cands):
        picks = dev_pick if isinstance(dev_pick, list) else [dev_pick]
        hits = [p for p in picks if p in cands]
        assert len(hits) == 1, (dev_pick, cands)
        if firsts is not None:
            firsts.setdefault(key, cands.index(hits[0]))
        return cands.index(hits[0])
    return draw


def check_against_oracle(rows, topics, pubs, ref, strategy, firsts=None):
    """Replays the device's deliveries through the oracle in message order; every rand draw
    (a publisher's first pick per group, sticky re-picks) is the device's, checked to be one of
    the reference's candidates, and every other pick must equal the reference's."""
    for t, p, row in zip(topics, pubs, rows):
        by_filter = {}
        for f, s, sh in row:
            if sh:
                by_filter.setdefault(f, []).append(s)
        exp = []
        for to, dest in B.Broker.aggre(ref.router.match_routes(t)):
            if dest == B.NODE:
                exp += [(to, s, False) for s in ref.subscriber.get(to, [])]
                continue
            sub = ref.shared.pick(strategy, p, dest, to, draw=replay(by_filter.get(to, []), firsts, (p, dest, to)))
            if sub is not False:
                exp.append((to, sub, True))
        assert canon(row) == canon(exp), (t, p, row, exp)


@pytest.mark.parametrize("strategy", ["round_robin", "sticky"])
def test_per_publisher_state_interleaved(F, strategy):
    code = B.ROUND_ROBIN if strategy == "round_robin" else B.STICKY
    dev, ref = build_groups(F, strategy)
    rng = random.Random(7)
    pubs_all = [11, 22, 33, 44, 55]
    firsts = {}
    for batch in range(4):
        n = rng.randint(20, 60)
        pubs = [rng.choice(pubs_all[:3] if batch < 2 else pubs_all) for _ in range(n)]
        topics = [b"x/%d" % rng.randrange(10) for _ in range(n)]
        rows = dev.publish_batch(topics, pubs)
        check_against_oracle(rows, topics, pubs, ref, code, firsts)
        if batch == 1:  # membership change between batches: state carries over ((Rem + 1) rem N);
            # a sticky publisher on m2 keeps it (alive, emqx_shared_sub.erl:234-240)
            dev.unsubscribe(b"x/+", "m2", share=b"g")
            ref.unsubscribe(b"x/+", "m2", b"g")
            dev.subscribe(b"x/+", "m9", share=b"g")
            ref.subscribe(b"x/+", "m9", b"g")
    # each publisher rotates (or sticks) on its own: 5 publishers x 2 groups seeded separately
    assert len(firsts) == 10
    if strategy == "sticky":
        # with 16 publishers, not every one sticks to the same member of a 5-member group
        pubs = list(range(1000, 1016))
        rows = dev.publish_batch([b"x/1"] * 16, pubs)
        picks = {r[1] for row in rows for r in row if r[0] == b"x/+"}
        assert len(picks) >= 2


def test_round_robin_overflow_consumes_no_state(F):
    from emqx_amd import _lib
    from emqx_amd.engine import pack
    dev, _ = build_groups(F, "round_robin")
    dev._sync()
    buf, offs = pack([b"x/1"])
    keys = np.array([5], np.uint32)

    def one(cap):
        import ctypes
        out_off = np.zeros(2, np.uint64)
        subs, fils = np.zeros(max(cap, 1), np.uint32), np.zeros(max(cap, 1), np.uint32)
        n_out = ctypes.c_uint64(0)
        rc = _lib.lib().emqx_publish_batch(dev.router.engine._h, dev.subs.handle, _lib.SHARE_ROUND_ROBIN,
                                           buf.ctypes.data, offs.ctypes.data, 1, keys.ctypes.data, out_off.ctypes.data,
                                           subs.ctypes.data, fils.ctypes.data, cap, ctypes.byref(n_out))
        return rc, int(n_out.value), subs, fils

    rc, need, subs, fils = one(64)
    assert rc == 0 and need == 3  # x/+ pick, x/# pick, x/# plain
    g_first = [int(s) for s, f in zip(subs[:need], fils[:need]) if f & _lib.FANOUT_SHARED_BIT]
    for _ in range(3):
        rc, need2, _, _ = one(2)
        assert rc == _lib.EMQX_EOVERFLOW and need2 == 3
    rc, _, subs, fils = one(64)
    g_next = [int(s) for s, f in zip(subs[:3], fils[:3]) if f & _lib.FANOUT_SHARED_BIT]
    # exactly one rotation step per group since the first call: overflowed calls advanced nothing
    names = {dev._sid(m): m for m in ["m%d" % i for i in range(5)] + ["k%d" % i for i in range(3)]}
    for a, b in zip(sorted(g_first, key=lambda v: names[v][0]), sorted(g_next, key=lambda v: names[v][0])):
        ma, mb = names[a], names[b]
        n = 5 if ma[0] == "m" else 3
        assert (int(ma[1:]) + 1) % n == int(mb[1:]), (ma, mb)


def test_forget_publishers_restarts_their_rotation(F):
    dev, _ = build_groups(F, "round_robin")
    rows = dev.publish_batch([b"x/1"] * 8, [77] * 8)
    seq = [r[1] for row in rows for r in row if r[0] == b"x/+"]
    assert all((int(seq[i][1:]) + 1) % 5 == int(seq[i + 1][1:]) for i in range(7))
    dev.subs.forget_publishers([77])
    # the state is gone: its next pick is a fresh first pick (random), and rotation resumes from it
    rows = dev.publish_batch([b"x/1"] * 6, [77] * 6)
    seq2 = [r[1] for row in rows for r in row if r[0] == b"x/+"]
    assert all((int(seq2[i][1:]) + 1) % 5 == int(seq2[i + 1][1:]) for i in range(5))


def test_pub_batcher_many_threads_equals_publish_batch(F):
    """64 threads x 200 single-message submissions through emqx_pub_batcher (hash_clientid):
    every callback's deliveries equal publish_batch's for the same (topic, key)."""
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine, pack
    fw = W.config_e(n_filters=50_000, n_subscribers=20_000, n_topics=4000, seed=12)
    eng = Engine(0)
    eng.insert_packed(*fw.wl.filters)
    eng.commit()
    st = F.SubTable(0)
    st.add(fw.sub_filter, fw.sub_id, fw.sub_group)
    st.commit()
    topics = W.unpack(fw.wl.topics)
    keys = fw.keys
    off, subs, fils = F.publish_packed(eng, st, "hash_clientid", *pack(topics), keys)
    exp = [sorted(zip(subs[off[i]:off[i + 1]].tolist(), fils[off[i]:off[i + 1]].tolist())) for i in range(len(topics))]
    pb = F.PubBatcher(eng, st, "hash_clientid", max_batch=512, max_wait_us=100)
    got = {}
    lock = threading.Lock()
    errors = []

    def worker(w):
        for j in range(200):
            i = (w * 200 + j) % len(topics)
            ev = threading.Event()

            def done(status, s, f, _i=i, _ev=ev):
                if status != 0:
                    errors.append(status)
                with lock:
                    got[_i] = sorted(zip(s.tolist(), f.tolist()))
                _ev.set()

            pb.submit(topics[i], int(keys[i]), done)
            assert ev.wait(30)

    th = [threading.Thread(target=worker, args=(w,)) for w in range(64)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    stats = pb.stats()
    pb.close()
    assert not errors
    assert len(got) == min(len(topics), 64 * 200)
    for i, rows in got.items():
        assert rows == exp[i], i
    assert stats["messages"] == 64 * 200 and stats["batches"] < 64 * 200


def test_commit_wait_rebuild_alloc_failure_is_enomem(F):
    """emqx_subtab_commit_wait rebuilds the tables when the last commit's device half
    failed; an allocation failure of that rebuild is EMQX_ENOMEM (no exception through the C
    ABI), and the next commit rebuilds and serves the fan-out again."""
    from emqx_amd import _lib
    t = F.SubTable(0)
    try:
        t.add([0, 1, 1], [5, 6, 7])
        t.commit()
        assert t.commit_wait() == _lib.EMQX_OK
        with pytest.raises(Exception):
            t.set_tuning("no_such_key", 1)
        t.set_tuning("inject_drain_error", 1)
        t.set_tuning("inject_bad_alloc", 1)
        assert t.commit_wait() == _lib.EMQX_ENOMEM
        # the failed rebuild left need_full set: the next commit is a full one and succeeds
        full0 = t.commit_stats()["full_commits"]
        t.add([2], [8])
        t.commit()
        assert t.commit_wait() == _lib.EMQX_OK
        assert t.commit_stats()["full_commits"] == full0 + 1
        st = t.stats()
        assert st["plain"] == 4 and st["device_bytes"] > 0
    finally:
        t.close()
