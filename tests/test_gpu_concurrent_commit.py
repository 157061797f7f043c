"""Matches in flight while commits publish changes.

The reference's readers never lock: emqx_trie's tables are ETS with read_concurrency
(apps/emqx/src/emqx_trie.erl:69-71), and a route change becomes visible when its mria
transaction commits (apps/emqx/src/emqx_router_utils.erl:97-125), so a lookup that overlaps a
batch of changes sees each change made or not made, never a broken table.  The engine's
incremental commit patches the committed table in place on the device while matches run
(whole 16-B slot stores, new extents before the slots that point at them).
For every topic of every overlapped match:   old ∩ new  ⊆  result  ⊆  old ∪ new,
where old / new are the results before / after the commit; and a commit that relocates nodes
is among the overlapped ones.

The subscription table (fan-out) and the retained index take the other two routes: fan-outs
are ordered against subscription commits by device events (a fan-out sees the table wholly
before or wholly after a commit), and the retained index swaps whole snapshots (a match reads
the old snapshot or the new one).  Both are checked here too."""

import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def pairs(off, ids, n_check):
    """Sorted unique (topic << 32 | id) keys of the first n_check topics of a CSR."""
    off = np.asarray(off, dtype=np.int64)[: n_check + 1]
    cnt = np.diff(off)
    t = np.repeat(np.arange(n_check, dtype=np.uint64), cnt)
    return np.unique((t << np.uint64(32)) | np.asarray(ids[: off[-1]], dtype=np.uint64))


def test_matches_overlapping_incremental_commits():
    import torch
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine, pack
    dev = torch.device("cuda", 0)
    wl = W.config_b(n_filters=460_000, n_topics=400_000, seed=31)
    allf = W.unpack(wl.filters)
    base, extra = allf[:400_000], allf[400_000:]
    # new words and deeper tails: new chains and relocated nodes in every commit
    rng = np.random.default_rng(5)
    extra = [f + b"/x%d" % i if i % 3 == 0 else b"n%d/" % (i % 97) + f for i, f in enumerate(extra)]
    e = Engine(0)
    e.insert(base)
    e.commit()
    n = wl.n_topics
    n_check = 100_000
    tb = torch.from_numpy(wl.topics[0]).to(dev)
    to = torch.from_numpy(wl.topics[1].view(np.int64)).to(dev)
    cap = 64 * n
    K = 24
    outs = [(torch.empty(n + 1, dtype=torch.int64, device=dev), torch.empty(cap, dtype=torch.int32, device=dev))
            for _ in range(K)]
    summ = torch.zeros((K, e.SUMMARY_WORDS), dtype=torch.int64, device=dev)
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]
    ref = outs[0]

    def sync_pairs():
        m = e.match_device(tb.data_ptr(), to.data_ptr(), n, ref[0].data_ptr(), ref[1].data_ptr(), cap)
        return pairs(ref[0].cpu().numpy(), ref[1][:m].cpu().numpy().view(np.uint32), n_check)

    live = np.ones(len(base), bool)
    relocated = 0
    mixed = 0
    for r in range(3):
        old = sync_pairs()
        dels = rng.choice(np.flatnonzero(live), 10_000, replace=False)
        e.delete(sorted(int(i) for i in dels))
        live[dels] = False
        e.insert(extra[r * 10_000:(r + 1) * 10_000])
        torch.cuda.synchronize()
        for k in range(K):  # ~K x 0.3 ms of matches queued on two streams ...
            o = outs[k]
            e.match_device_async(tb.data_ptr(), to.data_ptr(), n, o[0].data_ptr(), o[1].data_ptr(), cap,
                                 summ[k].data_ptr(), stream=streams[k % 2].cuda_stream)
        e.commit()  # ... while the commit patches the table they read
        torch.cuda.synchronize()
        assert e.stats()["last_commit_kind"] == 1
        relocated += e.commit_stats()["relocations"]
        new = sync_pairs()
        both = np.intersect1d(old, new, assume_unique=True)
        either = np.union1d(old, new)
        sm = summ.cpu().numpy()
        assert (sm[:, 0] == 0).all()
        for k in range(K):
            o = outs[k]
            got = pairs(o[0].cpu().numpy(), o[1][: int(sm[k, 1])].cpu().numpy().view(np.uint32), n_check)
            assert np.isin(both, got, assume_unique=True).all(), (r, k, "a filter in both old and new is missing")
            assert np.isin(got, either, assume_unique=True).all(), (r, k, "an id outside old and new")
            if not (np.array_equal(got, old) or np.array_equal(got, new)):
                mixed += 1
    assert relocated > 0  # the overlapped commits moved nodes


def test_fanout_ordered_around_subscription_commit():
    """A fan-out enqueued before a subscription commit sees the old table, one enqueued after it
    the new one (hash_clientid: exact), whatever the streams."""
    import torch
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine
    from emqx_amd.fanout import SubTable
    dev = torch.device("cuda", 0)
    fw = W.config_e(n_filters=100_000, n_subscribers=50_000, n_topics=100_000, seed=17)
    eng = Engine(0)
    eng.insert_packed(*fw.wl.filters)
    eng.commit()
    st = SubTable(0)
    st.add(fw.sub_filter, fw.sub_id, fw.sub_group)
    st.commit()
    n = fw.wl.n_topics
    tb = torch.from_numpy(fw.wl.topics[0]).to(dev)
    to = torch.from_numpy(fw.wl.topics[1].view(np.int64)).to(dev)
    keys = torch.from_numpy(fw.keys.view(np.int32)).to(dev)
    mcap = 64 * n
    moff = torch.empty(n + 1, dtype=torch.int64, device=dev)
    mids = torch.empty(mcap, dtype=torch.int32, device=dev)
    eng.match_device(tb.data_ptr(), to.data_ptr(), n, moff.data_ptr(), mids.data_ptr(), mcap)
    ocap = 128 * n
    bufs = [tuple(torch.empty(x, dtype=d, device=dev) for x, d in ((n + 1, torch.int64), (ocap, torch.int32),
                                                                   (ocap, torch.int32))) for _ in range(4)]
    summ = torch.zeros((4, st.SUMMARY_WORDS), dtype=torch.int64, device=dev)
    streams = [torch.cuda.Stream(device=dev) for _ in range(2)]

    def fan(k, stream):
        b = bufs[k]
        st.fanout_device_async("hash_clientid", moff.data_ptr(), mids.data_ptr(), n, mcap, keys.data_ptr(),
                               b[0].data_ptr(), b[1].data_ptr(), b[2].data_ptr(), ocap, summ[k].data_ptr(),
                               stream=stream.cuda_stream)

    def result(k):
        b, tot = bufs[k], int(summ[k, 1].item())
        return b[0].cpu().numpy(), b[1][:tot].cpu().numpy(), b[2][:tot].cpu().numpy()

    fan(0, streams[0])
    fan(1, streams[1])
    # churn: unsubscribe 20% of the plain subscriptions of the busiest filters, add new ones
    plain = np.flatnonzero(fw.sub_group == W.NO_GROUP)
    rm = plain[: len(plain) // 5]
    st.remove(fw.sub_filter[rm], fw.sub_id[rm])
    st.add(fw.sub_filter[rm], fw.sub_id[rm] + np.uint32(5_000_000))
    st.commit()
    fan(2, streams[0])
    fan(3, streams[1])
    torch.cuda.synchronize()
    assert (summ.cpu().numpy()[:, 0] == 0).all()
    r = [result(k) for k in range(4)]
    for a, b in ((0, 1), (2, 3)):
        assert all(np.array_equal(x, y) for x, y in zip(r[a], r[b]))
    assert not np.array_equal(r[0][1], r[2][1])  # the commit changed the deliveries


def test_retain_matches_during_commits_see_a_whole_snapshot():
    """Two host threads: one matches a filter batch in a loop, the other stores / deletes and
    commits; every match result equals the result of one of the committed snapshots."""
    from emqx_amd.retainer import RetainIndex
    from emqx_amd import workloads as W
    rng = np.random.default_rng(8)
    wl = W.config_b(n_filters=60_000, n_topics=2_000, seed=12)
    topics = [t for t in W.unpack(wl.filters) if b"+" not in t and b"#" not in t][:20_000]
    filters = W.unpack(wl.filters)[:2000]
    idx = RetainIndex(0)
    idx.store(topics[:10_000])
    idx.commit()
    snaps = [idx.match(filters, now=0)]
    results = []
    stop = threading.Event()
    errors = []

    def reader():
        try:
            while not stop.is_set():
                results.append(idx.match(filters, now=0))
        except Exception as ex:  # noqa: BLE001
            errors.append(ex)

    th = threading.Thread(target=reader)
    th.start()
    try:
        for r in range(6):
            idx.store(topics[10_000 + 1000 * r: 10_000 + 1000 * (r + 1)])
            idx.delete([int(i) for i in rng.choice(10_000, 300, replace=False)])
            idx.commit()
            snaps.append(idx.match(filters, now=0))
    finally:
        stop.set()
        th.join()
    assert not errors
    canon = [[sorted(x) for x in s] for s in snaps]
    assert len(results) > 0
    for res in results:
        assert [sorted(x) for x in res] in canon
