"""Parity of the HIP engine with the oracle (GPU).

Every result is compared bit-exactly as sorted filter-id sets against the
oracle: the reference KATs (tests/golden/kats.json), fuzzed tables in all three modes, the
BASELINE configs at sizes the oracle finishes in seconds, and the edge cases the reference
tests (empty levels, '$' topics, wildcard topics, 26-level topics, deletes) plus the engine's
own capacity paths (deep topics, slab overflow, long words, unknown words)."""

import random

import numpy as np
import pytest

from oracle import cpp as C
from oracle import emqx_ref as R
from tests.test_oracle_fuzz import rand_filter, rand_topic

pytestmark = pytest.mark.gpu

MODES = {"routes": 0, "trie": 1, "trie_wildcard": 2}


@pytest.fixture(scope="module")
def Engine():
    import torch  # noqa: F401  (shares the HIP runtime with the engine)
    from emqx_amd.engine import Engine as E
    from emqx_amd import _lib
    _lib.lib()
    return E


def engine_with(Engine, filters):
    e = Engine()
    ids = e.insert(filters)
    assert list(ids) == list(range(len(filters)))
    e.commit()
    return e


def expected(filters, topics, mode):
    if mode == 0:
        return [R.brute_force_routes(filters, t) for t in topics]
    if mode == 1:
        return [R.brute_force_trie(filters, t) for t in topics]
    wild = [f if R.wildcard(f) else b"\x00never" for f in filters]
    return [R.brute_force_trie(wild, t) for t in topics]


def test_trie_suite_kats(Engine, kats):
    for case in kats["trie_cases"]:
        e = Engine()
        names = {}
        for op, arg in case["ops"]:
            if op == "insert":
                fid = int(e.insert([arg.encode()])[0])
                names[fid] = arg.encode()
            elif op == "delete":
                fid = e.lookup(arg.encode())
                if fid is not None:
                    e.delete([fid])
            elif op == "assert_empty":
                assert (e.stats()["n_filters"] == 0) == arg
        e.commit()
        for topic, exp in case["queries"]:
            got = sorted(names[i] for i in e.match([topic.encode()], mode=1)[0])
            assert got == sorted(x.encode() for x in exp), (case["name"], topic)
        for topic, n in case.get("len_queries", []):
            assert len(e.match([topic.encode()], mode=1)[0]) == n


def test_router_and_client_kats(Engine, kats):
    from emqx_amd.router import Router
    for case in kats["router_cases"]:
        r = Router()
        for t in case["add"]:
            r.add_route(t.encode())
        for topic, exp in case["queries"]:
            assert sorted(x.topic for x in r.match_routes(topic.encode())) == sorted(e.encode() for e in exp)
        for t in case["add"]:
            r.delete_route(t.encode())
        for topic, exp in case["then_delete_all"]:
            assert r.match_routes(topic.encode()) == []
    c = kats["client"]
    for key in ("overlapping", "dollar"):
        r = Router()
        for s in c[key]["subs"]:
            r.add_route(s.encode())
        got = sorted(x.topic for x in r.match_routes(c[key]["topic"].encode()))
        assert got == sorted(e.encode() for e in c[key]["expect"])


def test_topic_match_pairs_on_device(Engine, kats):
    """emqx_topic:match/2 KATs as one-filter tables (valid names only; the device implements
    the trie/router semantics, which equal match/2 for non-wildcard names)."""
    for name, filt, exp in kats["topic_match"]:
        if R.wildcard(name.encode()):
            continue
        e = engine_with(Engine, [filt.encode()])
        got = e.match([name.encode()], mode=0)[0]
        assert (got == [0]) is exp, (name, filt)


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_fuzz_parity(Engine, seed, mode):
    rng = random.Random(9000 + seed)
    filters = sorted({rand_filter(rng) for _ in range(rng.randint(20, 400))})
    topics = [rand_topic(rng) for _ in range(600)] + [b"", b"/", b"$", b"$/x", b"+", b"#", b"a/#/b"]
    e = engine_with(Engine, filters)
    got = e.match(topics, mode=mode)
    exp = expected(filters, topics, mode)
    for t, g, x in zip(topics, got, exp):
        assert g == x, (mode, t, g, x)


def test_deletes_and_recommit(Engine):
    rng = random.Random(77)
    filters = sorted({rand_filter(rng) for _ in range(300)})
    e = engine_with(Engine, filters)
    gone = set(rng.sample(range(len(filters)), 100))
    e.delete(sorted(gone))
    e.commit()
    live = [f if i not in gone else b"\x00dead" for i, f in enumerate(filters)]
    topics = [rand_topic(rng) for _ in range(500)]
    for t, g in zip(topics, e.match(topics, mode=0)):
        assert g == R.brute_force_routes(live, t)
    # re-insert keeps the old ids
    back = sorted(gone)[:10]
    ids = e.insert([filters[i] for i in back])
    assert list(ids) == back


def oracle_ids(filters_packed, topics_packed, mode=C.MODE_ROUTES, threads=8):
    o = C.CppOracle(True, trie_all=(mode == C.MODE_TRIE))
    o.add_packed(*filters_packed)
    counts, ids, _ = o.match_packed(*topics_packed, mode=mode, threads=threads, stride=512)
    return counts, ids


def csr_equal(off, ids, counts, oids):
    n = len(counts)
    assert off[-1] == ids.size
    got_counts = np.diff(off.astype(np.int64))
    bad = np.nonzero(got_counts != counts.astype(np.int64))[0]
    assert bad.size == 0, f"count mismatch at topics {bad[:10]}"
    for i in range(n):
        g = np.sort(ids[off[i]:off[i + 1]])
        x = oids[i, :counts[i]]
        assert np.array_equal(g, x), (i, g, x)


def test_config_a_sample(Engine):
    from emqx_amd import workloads as W
    a = W.config_a(n_topics=50_000)
    e = Engine()
    e.insert_packed(*a.filters)
    e.commit()
    off, ids = e.match_packed(*a.topics, mode=0)
    counts, oids = oracle_ids(a.filters, a.topics)
    csr_equal(off, ids, counts, oids)
    assert 0.7 < float(np.mean(counts == 1)) < 0.85   # ≈78% hit exactly one filter (SURVEY §8 d)


def test_config_a_prime_one_route(Engine):
    """emqx_broker_bench.erl:161-162: every publisher topic matches exactly one route."""
    from emqx_amd import workloads as W
    ap = W.config_a_prime()
    e = Engine()
    e.insert_packed(*ap.filters)
    e.commit()
    off, ids = e.match_packed(*ap.topics, mode=0)
    assert np.all(np.diff(off.astype(np.int64)) == 1)


def test_config_b_reduced(Engine):
    from emqx_amd import workloads as W
    b = W.config_b(n_filters=300_000, n_topics=40_000)
    e = Engine()
    e.insert_packed(*b.filters)
    e.commit()
    for mode in (0, 2):
        off, ids = e.match_packed(*b.topics, mode=mode)
        counts, oids = oracle_ids(b.filters, b.topics, mode=mode)
        csr_equal(off, ids, counts, oids)
    # evals: the engine's node-visit count equals the oracle's cost model
    o = C.CppOracle(True)
    o.add_packed(*b.filters)
    e.match_packed(*b.topics, mode=0)
    assert e.stats()["last_evals"] == int(o.evals_packed(*b.topics).sum())


def test_config_b_full_table(Engine):
    """The headline table itself (BASELINE configs[1]): all 10M config-B filters (seed 2, the
    bench's table), 20K topics of config B's generator, every topic compared ID-for-ID with the oracle (routes mode and
    the router's wildcard-only trie)."""
    from emqx_amd import workloads as W
    b = W.config_b(n_filters=10_000_000, n_topics=20_000)
    e = Engine()
    e.insert_packed(*b.filters)
    e.commit()
    o = C.CppOracle(True)  # the router's layout: wildcard filters in the trie
    o.add_packed(*b.filters)
    # routes (exact ∪ trie) and the router's wildcard-only trie (oracle mode 1 on that trie)
    for mode, omode in ((0, C.MODE_ROUTES), (2, C.MODE_TRIE)):
        off, ids = e.match_packed(*b.topics, mode=mode)
        off_o, ids_o, _ = o.match_csr(*b.topics, mode=omode, threads=8)
        bad = C.csr_mismatches(off, ids, off_o, ids_o)
        assert bad.size == 0, (mode, bad[:10])
        assert int(off_o[-1]) > 5 * len(off_o)


def test_config_d_reduced(Engine):
    from emqx_amd import workloads as W
    d = W.config_d(n_filters=30_000, n_topics=3000)
    e = Engine()
    e.insert_packed(*d.filters)
    e.commit()
    off, ids = e.match_packed(*d.topics, mode=0)
    counts, oids = oracle_ids(d.filters, d.topics)
    csr_equal(off, ids, counts, oids)
    assert counts.mean() > 3


def test_config_d_full_table(Engine):
    """Config D at its full size (1M adversarial filters, depth-16 topics): 16K topics
    compared ID-for-ID with the C++ DFS, in batch order and with the walk order forced on (the
    prefix-key sort and XCD dealing the engine turns on for D's 1M-topic batches)."""
    import os
    from emqx_amd import workloads as W
    d = W.config_d(n_filters=1_000_000, n_topics=16_384)
    e = Engine()
    e.insert_packed(*d.filters)
    e.commit()
    o = C.CppOracle(True)
    o.add_packed(*d.filters)
    off_o, ids_o, _ = o.match_csr(*d.topics, mode=C.MODE_ROUTES, threads=min(16, os.cpu_count() or 4))
    assert int(off_o[-1]) > 3 * (len(off_o) - 1)
    for order in (0, 1):
        e.set_tuning("order", order)
        off, ids = e.match_packed(*d.topics, mode=0)
        bad = C.csr_mismatches(off, ids, off_o, ids_o)
        assert bad.size == 0, (order, bad[:10])
    e.set_tuning("order", -1)


def test_deep_topics_take_deep_path(Engine):
    """Topics beyond the fast path's LDS budget (WID_CAP/8 levels) run on the deep path."""
    rng = random.Random(5)
    deep = b"/".join(b"w%d" % (i % 7) for i in range(300))
    filters = [b"#", b"w0/#", b"+/+/#", deep, deep + b"/#", b"/".join([b"+"] * 300),
               b"/".join([b"+"] * 150) + b"/#", b"w0/w1/+/w3/#"]
    topics = [deep, deep + b"/x", b"/".join([b"w0"] * 400), b"a/b"] + [rand_topic(rng) for _ in range(100)]
    e = engine_with(Engine, filters)
    for mode in (0, 1, 2):
        got = e.match(topics, mode=mode)
        for t, g, x in zip(topics, got, expected(filters, topics, mode)):
            assert g == x, (mode, t[:40])
    assert e.stats()["last_deferred"] >= 3


def test_many_matches_slab_growth(Engine):
    """One topic matched by thousands of filters: the per-tile slab grows and reruns."""
    filters = [b"a/b/c/d"] + [b"a/%s#" % (b"+/" * k) for k in range(3)]
    filters += [b"a/b/c/d/%d/#" % i for i in range(3000)] + [b"+/b/+/d"]
    filters += [b"a/+/c/d"] + [b"+/+/+/+"]
    topics = [b"a/b/c/d"] * 70 + [b"a/b/c/d/%d" % i for i in range(50)]
    e = engine_with(Engine, filters)
    got = e.match(topics, mode=0)
    for t, g, x in zip(topics, got, expected(filters, topics, 0)):
        assert g == x


def test_long_and_unknown_words(Engine):
    long_w = b"x" * 40
    filters = [long_w + b"/+", b"+/" + long_w, long_w + b"y/#", long_w[:-1] + b"/#", b"\xe4\xbd\xa0/+"]
    topics = [long_w + b"/a", b"q/" + long_w, long_w + b"y", long_w + b"z/k", b"\xe4\xbd\xa0/1",
              b"nope/nope", long_w[:-1]]
    e = engine_with(Engine, filters)
    got = e.match(topics, mode=0)
    assert got == expected(filters, topics, 0)


def test_empty_table_and_empty_batch(Engine):
    e = Engine()
    e.commit()
    assert e.match([b"a/b", b""], mode=0) == [[], []]
    e2 = engine_with(Engine, [b"#"])
    assert e2.match([], mode=0) == []


def test_device_api_matches_host_api(Engine):
    import torch
    from emqx_amd import workloads as W
    b = W.config_b(n_filters=100_000, n_topics=20_000)
    e = Engine()
    e.insert_packed(*b.filters)
    e.commit()
    off_h, ids_h = e.match_packed(*b.topics, mode=0)
    dev = torch.device("cuda:0")
    tb = torch.from_numpy(b.topics[0]).to(dev)
    to = torch.from_numpy(b.topics[1].view(np.int64)).to(dev)
    d_off = torch.empty(len(b.topics[1]), dtype=torch.int64, device=dev)
    d_ids = torch.empty(ids_h.size + 16, dtype=torch.int32, device=dev)
    n = e.match_device(tb.data_ptr(), to.data_ptr(), len(b.topics[1]) - 1, d_off.data_ptr(), d_ids.data_ptr(),
                       d_ids.numel(), mode=0, stream=torch.cuda.current_stream().cuda_stream)
    assert n == ids_h.size
    off_d = d_off.cpu().numpy().view(np.uint64)
    ids_d = d_ids[:n].cpu().numpy().view(np.uint32)
    assert np.array_equal(off_d, off_h)
    for i in range(0, len(off_h) - 1, 97):
        assert np.array_equal(np.sort(ids_d[off_d[i]:off_d[i + 1]]), np.sort(ids_h[off_h[i]:off_h[i + 1]]))


def test_device_api_null_stream_waits_for_default_stream(Engine):
    """A device call given no stream runs on the engine's own (non-blocking) stream after the
    work already enqueued on the null stream (include/emqx_match.h): offsets written there
    behind a long kernel must be the ones matched.  Unordered, the call would read the
    all-zero offsets written first (every topic empty: no out-of-bounds reads) and return no ids."""
    import torch
    from emqx_amd import workloads as W
    b = W.config_b(n_filters=50_000, n_topics=20_000)
    e = Engine()
    e.insert_packed(*b.filters)
    e.commit()
    off_h, ids_h = e.match_packed(*b.topics, mode=0)
    assert ids_h.size > 0
    dev = torch.device("cuda:0")
    tb = torch.from_numpy(b.topics[0]).to(dev)
    to_real = torch.from_numpy(b.topics[1].view(np.int64)).to(dev)
    to = torch.zeros_like(to_real)
    d_off = torch.empty(len(b.topics[1]), dtype=torch.int64, device=dev)
    d_ids = torch.empty(ids_h.size + 16, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    for _ in range(3):
        to.zero_()
        torch.cuda.synchronize()
        torch.cuda._sleep(100_000_000)  # tens of ms on the null stream
        to.copy_(to_real)               # the real offsets, behind it
        n = e.match_device(tb.data_ptr(), to.data_ptr(), len(b.topics[1]) - 1, d_off.data_ptr(),
                           d_ids.data_ptr(), d_ids.numel(), mode=0, stream=0)
        assert n == ids_h.size
        assert np.array_equal(d_off.cpu().numpy().view(np.uint64), off_h)


def test_async_device_api(Engine):
    """emqx_match_batch_device_async: pipelined calls on one stream give the synchronous
    call's CSR, each writes its summary, and the flags report a too-small id buffer and a
    slab that must grow (the synchronous call then sizes it)."""
    import torch
    from emqx_amd import workloads as W
    b = W.config_b(n_filters=100_000, n_topics=20_000)
    e = Engine()
    e.insert_packed(*b.filters)
    e.commit()
    off_h, ids_h = e.match_packed(*b.topics, mode=0)
    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream().cuda_stream
    tb = torch.from_numpy(b.topics[0]).to(dev)
    to = torch.from_numpy(b.topics[1].view(np.int64)).to(dev)
    n = len(b.topics[1]) - 1
    summ = torch.zeros((4, Engine.SUMMARY_WORDS), dtype=torch.int64, device=dev)
    outs = []
    for k in range(3):
        d_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        d_ids = torch.empty(ids_h.size + 16, dtype=torch.int32, device=dev)
        e.match_device_async(tb.data_ptr(), to.data_ptr(), n, d_off.data_ptr(), d_ids.data_ptr(), d_ids.numel(),
                             summ[k].data_ptr(), mode=0, stream=s)
        outs.append((d_off, d_ids))
    small = torch.empty(8, dtype=torch.int32, device=dev)
    d_off_s = torch.empty(n + 1, dtype=torch.int64, device=dev)
    e.match_device_async(tb.data_ptr(), to.data_ptr(), n, d_off_s.data_ptr(), small.data_ptr(), small.numel(),
                         summ[3].data_ptr(), mode=0, stream=s)
    torch.cuda.synchronize()
    sm = summ.cpu().numpy()
    assert (sm[:3, 0] == 0).all() and (sm[:, 1] == ids_h.size).all()
    assert sm[3, 0] == 2  # overflow: offsets complete, ids truncated
    assert np.array_equal(d_off_s.cpu().numpy().view(np.uint64), off_h)
    for d_off, d_ids in outs:
        off_d = d_off.cpu().numpy().view(np.uint64)
        ids_d = d_ids[:ids_h.size].cpu().numpy().view(np.uint32)
        assert np.array_equal(off_d, off_h)
        for i in range(0, n, 89):
            assert np.array_equal(np.sort(ids_d[off_d[i]:off_d[i + 1]]), np.sort(ids_h[off_h[i]:off_h[i + 1]]))
    # a fresh engine's first async call on a hot topic overflows its slab: flag 1, then the
    # synchronous call grows it and the async call completes.  The topic has 10 levels; the
    # filters are every literal/'+' pattern of it and every such prefix + '#' (3071 matches).
    from emqx_amd.engine import pack
    words = [b"w%d" % i for i in range(10)]
    pats = []
    for L in range(11):
        for m in range(1 << L):
            lv = [b"+" if (m >> i) & 1 else words[i] for i in range(L)]
            pats.append(b"/".join(lv + [b"#"]) if L < 10 else b"/".join(lv))
    e2 = engine_with(Engine, pats)
    hot = pack([b"/".join(words)] * 64)
    want = len(expected(pats, [b"/".join(words)], 0)[0])
    htb = torch.from_numpy(np.array(hot[0])).to(dev)
    hto = torch.from_numpy(hot[1].view(np.int64)).to(dev)
    d_off = torch.empty(65, dtype=torch.int64, device=dev)
    d_ids = torch.empty(64 * want + 16, dtype=torch.int32, device=dev)
    s2 = torch.zeros(Engine.SUMMARY_WORDS, dtype=torch.int64, device=dev)
    e2.match_device_async(htb.data_ptr(), hto.data_ptr(), 64, d_off.data_ptr(), d_ids.data_ptr(), d_ids.numel(),
                          s2.data_ptr(), mode=0, stream=s)
    torch.cuda.synchronize()
    assert int(s2[0]) & 1
    assert e2.match_device(htb.data_ptr(), hto.data_ptr(), 64, d_off.data_ptr(), d_ids.data_ptr(), d_ids.numel(),
                           mode=0, stream=s) == 64 * want
    e2.match_device_async(htb.data_ptr(), hto.data_ptr(), 64, d_off.data_ptr(), d_ids.data_ptr(), d_ids.numel(),
                          s2.data_ptr(), mode=0, stream=s)
    torch.cuda.synchronize()
    assert int(s2[0]) == 0 and int(s2[1]) == 64 * want
    got = d_ids[:want].cpu().numpy().view(np.uint32)
    assert sorted(got.tolist()) == expected(pats, [b"/".join(words)], 0)[0]


def test_sharded_matcher_world1_rccl(Engine):
    """The filter-sharded path end to end on one GPU over RCCL (world size 1): requests to the
    two engines (space L + root wildcards, space P), global-id shard tables, the exchange and
    the per-topic merge give the single-engine result."""
    import os
    import torch
    import torch.distributed as dist
    from emqx_amd import workloads as W
    from emqx_amd.dist import ShardedMatcher
    wl = W.config_b(n_filters=120_000, n_topics=5000, seed=9)
    dev = torch.device("cuda:0")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29541")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        sm = ShardedMatcher(wl.filters, device=dev)
        topics = (torch.from_numpy(wl.topics[0]).to(dev), torch.from_numpy(wl.topics[1].view(np.int64)).to(dev))
        off, ids = sm.match(topics)
        off, ids = off.cpu().numpy(), ids.cpu().numpy().view(np.uint32)
    finally:
        dist.destroy_process_group()
    counts, oids = oracle_ids(wl.filters, wl.topics)
    csr_equal(off.astype(np.uint64), ids, counts, oids)


def test_sharded_matcher_config_c_generator(Engine):
    """Config C's generator (BASELINE configs[2]: generator B, vocab x4, seed 3) through the
    filter-sharded path on one GPU over RCCL, 1M filters and 20K topics, every topic compared
    ID-for-ID with the oracle; the walk order forced on for the same batch gives the same CSR."""
    import os
    import torch
    import torch.distributed as dist
    from emqx_amd import workloads as W
    from emqx_amd.dist import ShardedMatcher
    wl = W.config_b(n_filters=1_000_000, n_topics=20_000, seed=3, vocab_scale=4)
    dev = torch.device("cuda:0")
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = "29543"
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    try:
        sm = ShardedMatcher(wl.filters, device=dev)
        topics = (torch.from_numpy(wl.topics[0]).to(dev), torch.from_numpy(wl.topics[1].view(np.int64)).to(dev))
        off, ids = sm.match(topics)
        off, ids = off.cpu().numpy(), ids.cpu().numpy().view(np.uint32)
        live = [e for e in sm.engines if e is not None]  # (world 1: the AB engine only)
        for e in live:
            e.set_tuning("order", 1)
        off2, ids2 = sm.match(topics)
        off2, ids2 = off2.cpu().numpy(), ids2.cpu().numpy().view(np.uint32)
        for e in live:
            e.set_tuning("order", -1)
        off3, ids3 = sm.match_all(topics)  # every rank its own source (here the one rank)
        off3, ids3 = off3.cpu().numpy(), ids3.cpu().numpy().view(np.uint32)
    finally:
        dist.destroy_process_group()
    o = C.CppOracle(True)
    o.add_packed(*wl.filters)
    off_o, ids_o, _ = o.match_csr(*wl.topics, mode=C.MODE_ROUTES, threads=8)
    for a, b in ((off, ids), (off2, ids2), (off3, ids3)):
        bad = C.csr_mismatches(a.astype(np.uint64), b, off_o, ids_o)
        assert bad.size == 0, bad[:10]


def test_batcher_coalesces_concurrent_callers(Engine):
    """Concurrent single-topic callers (one PUBLISH each, as emqx_broker:publish/1 calls
    match_routes/1) get exactly their own results, in batches larger than one."""
    import threading
    from emqx_amd import workloads as W
    from emqx_amd.batcher import Batcher
    wl = W.config_b(n_filters=50_000, n_topics=2000, seed=13)
    e = Engine()
    e.insert_packed(*wl.filters)
    e.commit()
    topics = W.unpack(wl.topics)
    expect = e.match(topics, mode=0)
    b = Batcher(e, mode=0, max_batch=512, max_wait_us=2000)
    got = [None] * len(topics)

    def worker(k):
        for i in range(k, len(topics), 32):
            got[i] = sorted(b.match(topics[i]))

    th = [threading.Thread(target=worker, args=(k,)) for k in range(32)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    st = b.stats()
    b.close()
    assert got == expect
    assert st["topics"] == len(topics)
    assert st["batches"] < len(topics) // 4


def test_batch_permute_and_csr_unpermute_device(Engine):
    """emqx_batch_permute_device / emqx_csr_unpermute_device (the sharded layout's regrouping)
    against their torch restatements, on a batch that does not start at byte 0, with empty
    topics and topics without results."""
    import torch
    from emqx_amd import dist as D
    rng = np.random.default_rng(5)
    n = 5000
    lens = rng.integers(0, 40, n)
    lens[::97] = 0
    pad = 7
    tb_np = rng.integers(32, 127, pad + int(lens.sum()), dtype=np.uint8)
    to_np = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64) + pad
    dev = torch.device("cuda:0")
    tb, to = torch.from_numpy(tb_np).to(dev), torch.from_numpy(to_np).to(dev)
    owner = torch.from_numpy(rng.integers(0, 4, n)).to(dev)
    perm, lens_p, bytes_p, n_to, bytes_to = D.partition(tb, to, owner, 4)
    p = perm.cpu().numpy()
    want = b"".join(bytes(tb_np[to_np[i]:to_np[i + 1]]) for i in p)
    assert int(bytes_to.sum()) == len(want)
    assert bytes(bytes_p[:len(want)].cpu().numpy()) == want
    assert n_to.cpu().tolist() == np.bincount(owner.cpu().numpy(), minlength=4).tolist()
    assert bytes_to.cpu().tolist() == [int(lens[owner.cpu().numpy() == r].sum()) for r in range(4)]
    counts = torch.from_numpy(rng.integers(0, 6, n)).to(dev)
    counts[::13] = 0
    ids = torch.from_numpy(rng.integers(0, 1 << 30, int(counts.sum()))).to(torch.int32).to(dev)
    off, out = D.merge_csr(counts, ids, perm)
    c, i = counts.cpu().numpy(), ids.cpu().numpy()
    roff = np.concatenate([[0], np.cumsum(c)])
    per = [None] * n
    for k in range(n):
        per[p[k]] = i[roff[k]:roff[k + 1]]
    o, u = off.cpu().numpy(), out.cpu().numpy()
    assert o[-1] == len(i)
    for t in range(n):
        assert np.array_equal(u[o[t]:o[t + 1]], per[t]), t
