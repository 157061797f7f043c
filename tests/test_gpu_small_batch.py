"""The one-launch small-batch path (kernels.h SmallArgs): host batches and publish
batches of at most 1024 topics run as ONE kernel that reads the pinned inputs, walks the batch in
16 narrow tiles, runs the deep path, scatters the CSR and either streams it back (match) or fans
it out with stateless $share picks (publish).  Every result is compared ID-for-ID with the oracle
(emqx_router:match_routes/1 / emqx_trie:match/1, apps/emqx/src/emqx_router.erl:128-140,
emqx_trie.erl:315-334; the publish fan-out of emqx_broker.erl:244-272,500-524 with the hash pick
of emqx_shared_sub.erl:265-285) and with the batched pipeline (emqx_set_tuning "small_batch" 0)
on the same inputs, including the paths the kernel hands back: slab overflow (rerun on the
batched path), a fan-out with more entries than the kernel takes (FO_SUM_F_SMALL), id and
delivery buffers too small (EMQX_EOVERFLOW), and deferred topics (the deep path inside the
launch)."""

import numpy as np
import pytest

from oracle import cpp as C
from oracle import emqx_ref as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def table():
    import torch  # noqa: F401
    from emqx_amd import workloads as W
    from emqx_amd.engine import Engine
    wl = W.config_b(n_filters=150_000, n_topics=4096, seed=41)
    e = Engine()
    e.insert_packed(*wl.filters)
    e.commit()
    o = C.CppOracle(True, trie_all=False)
    o.add_packed(*wl.filters)
    o.freeze()
    return e, wl, o


def _host_batch(e, packed, mode, cap_ids=1 << 16):
    from emqx_amd.engine import HostBatch
    hb = HostBatch(e, cap_topics=2048, cap_bytes=1 << 20, cap_ids=cap_ids)
    hb.pack(*packed)
    hb.submit(mode)
    off, ids = hb.wait()
    hb.close()
    return off, ids


@pytest.mark.parametrize("n", [1, 3, 17, 48, 64, 65, 200, 511, 1024, 1025])
@pytest.mark.parametrize("mode", [0, 2])
def test_small_host_batches_id_for_id(table, n, mode):
    from emqx_amd import workloads as W
    e, wl, o = table
    part = W.take(wl.topics, np.arange(100, 100 + n))
    off_o, ids_o, _ = o.match_csr(*part, mode=mode, threads=4)
    off, ids = _host_batch(e, part, mode)
    assert C.csr_mismatches(off, ids, off_o, ids_o).size == 0
    e.set_tuning("small_batch", 0)
    try:
        off2, ids2 = _host_batch(e, part, mode)
    finally:
        e.set_tuning("small_batch", 1)
    assert np.array_equal(off, off2)
    assert C.csr_mismatches(off2, ids2, off_o, ids_o).size == 0  # (id order within a topic is free)


def _deep_topic_batch():
    """'#'-rich table: every literal / '+' combination of an 8-level topic, with and without a
    '#' after each prefix (767 filters that all match a/b/c/d/e/f/g/h), plus the edge topics."""
    import itertools
    lv = [b"a", b"b", b"c", b"d", b"e", b"f", b"g", b"h"]
    filters = set()
    for k in range(0, 9):
        for mask in itertools.product([0, 1], repeat=k):
            pre = [b"+" if m else lv[i] for i, m in enumerate(mask)]
            if k == 8:
                filters.add(b"/".join(pre))
            filters.add(b"/".join(pre + [b"#"]))
    filters |= {b"$SYS/#", b"$SYS/x", b"+/x", b"/+", b"/", b"a" * 5000, b"a" * 5000 + b"/#"}
    topics = [b"a/b/c/d/e/f/g/h", b"a/b/c", b"$SYS/x", b"x/x", b"", b"/", b"a/+/c", b"#",
              b"/".join([b"a"] * 120),                     # over 80 levels: the deep path
              b"a" * 5000, b"a" * 5000 + b"/q",            # a level over 4094 bytes: the deep path
              b"a/b/c/d/e/f/g/h/i/j/k"]
    return sorted(filters), topics


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_small_batch_deep_topics_and_slab_rerun(mode):
    """One topic with 767 matches fills its tile's slab past the learnt size (a rerun on the
    batched path); topics over 80 levels or with a 5000-byte level go to the deep path inside the
    launch; wildcard, '$', empty and '/' topics follow the reference's rules."""
    from emqx_amd.engine import Engine
    filters, topics = _deep_topic_batch()
    if mode == 0:
        exp = [R.brute_force_routes(filters, t) for t in topics]
    elif mode == 1:
        exp = [R.brute_force_trie(filters, t) for t in topics]
    else:  # the router's trie: wildcard filters only (emqx_router.erl:117-123)
        exp = [[i for i in R.brute_force_trie(filters, t) if R.wildcard(filters[i])] for t in topics]
    for reps in (1, 5):
        batch = topics * reps
        for small in (1, 0):
            e = Engine()
            e.insert(filters)
            e.commit()
            e.set_tuning("small_batch", small)
            got = e.match(batch, mode=mode)
            e.close()
            bad = [(i, len(g), len(x), sorted(set(g) ^ set(x))[:8]) for i, (g, x) in enumerate(zip(got, exp * reps))
                   if g != x]
            assert not bad, (reps, small, bad[:4])


def test_small_host_batch_overflow(table):
    """More ids than the pinned buffer holds: EMQX_EOVERFLOW with the count, then the rerun."""
    from emqx_amd import _lib
    from emqx_amd import workloads as W
    from emqx_amd.engine import HostBatch
    e, wl, o = table
    part = W.take(wl.topics, np.arange(0, 300))
    off_o, ids_o, _ = o.match_csr(*part, mode=0, threads=4)
    hb = HostBatch(e, cap_topics=2048, cap_bytes=1 << 20, cap_ids=32)
    hb.pack(*part)
    hb.submit(0)
    assert _lib.lib().emqx_host_batch_wait(hb._p) == _lib.EMQX_EOVERFLOW
    assert hb.s.n_out == int(off_o[-1])
    hb.submit(0)
    off, ids = hb.wait()
    hb.close()
    assert C.csr_mismatches(off, ids, off_o, ids_o).size == 0


def _broker(strategy, filters, n_subs=3000, seed=5):
    """Device broker and oracle broker with the same subscriptions; members[filter] = the
    subscribers of its one $share group (every fifth filter has one)."""
    from emqx_amd.fanout import Broker
    from oracle import broker_ref as BR
    rng = np.random.default_rng(seed)
    b, rb = Broker(0, node=BR.NODE, strategy=strategy), BR.Broker()
    members = {}
    for i, f in enumerate(filters):
        for s in rng.choice(n_subs, size=int(rng.integers(1, 7)), replace=False):
            for x in (b, rb):
                x.subscribe(f, "s%d" % s)
        if i % 5 == 0:
            ms = ["m%d" % s for s in rng.choice(n_subs, size=int(rng.integers(1, 6)), replace=False)]
            members[f] = set(ms)
            for m in ms:
                for x in (b, rb):
                    x.subscribe(f, m, b"g%d" % (i % 3))
    return b, rb, members


@pytest.mark.parametrize("n", [1, 47, 300, 1024])
def test_small_publish_batches_hash_pick(n):
    """Publish batches through the one-launch path (hash_clientid): every (filter, subscriber,
    shared) delivery equals the oracle's, and the batched pipeline's."""
    from emqx_amd import workloads as W
    from oracle import broker_ref as BR
    wl = W.config_b(n_filters=20_000, n_topics=n, seed=43)
    filters = W.unpack(wl.filters)[:4000]
    topics = W.unpack(wl.topics)
    b, rb, _ = _broker("hash_clientid", filters)
    keys = [int(k) for k in np.random.default_rng(7).integers(0, 1 << 32, len(topics))]
    got = b.publish_batch(topics, keys)
    for t, k, row in zip(topics, keys, got):
        exp = rb.publish(t, k, BR.HASH_CLIENTID)
        assert sorted(map(repr, row)) == sorted(map(repr, exp)), t
    b.router.engine.set_tuning("small_batch", 0)
    got2 = b.publish_batch(topics, keys)
    assert [sorted(map(repr, r)) for r in got] == [sorted(map(repr, r)) for r in got2]


def test_small_publish_random_pick_invariants():
    """random: the plain deliveries equal the oracle's; each matched filter with a group gets
    exactly one $share delivery, to one of that group's members."""
    from emqx_amd import workloads as W
    from oracle import broker_ref as BR
    wl = W.config_b(n_filters=20_000, n_topics=500, seed=44)
    filters = W.unpack(wl.filters)[:4000]
    topics = W.unpack(wl.topics)
    b, rb, members = _broker("random", filters)
    got = b.publish_batch(topics)
    for t, row in zip(topics, got):
        exp = rb.publish(t, 0, BR.HASH_CLIENTID)
        assert sorted(repr(d) for d in row if not d[2]) == sorted(repr(d) for d in exp if not d[2])
        shared = [(f, s) for f, s, sh in row if sh]
        assert sorted(f for f, _ in shared) == sorted(f for f, _, sh in exp if sh)
        for f, s in shared:
            assert s in members[f]


def test_small_publish_many_entries_falls_back():
    """A batch whose match entries exceed what the kernel's fan-out takes (16384): the match is
    kept, the fan-out runs on the batched kernels (FO_SUM_F_SMALL), deliveries equal the
    oracle's."""
    from oracle import broker_ref as BR
    filters, _ = _deep_topic_batch()
    filters = [f for f in filters if len(f) < 100 and f not in (b"", b"/")]
    b, rb, _ = _broker("hash_clientid", filters, n_subs=50)
    topics = [b"a/b/c/d/e/f/g/h"] * 30  # 30 x ~760 entries
    keys = list(range(30))
    got = b.publish_batch(topics, keys)
    exp = rb.publish(topics[0], 0, BR.HASH_CLIENTID)
    assert len(got[0]) == len(exp) > 700
    for t, k, row in zip(topics, keys, got):
        assert sorted(map(repr, row)) == sorted(map(repr, rb.publish(t, k, BR.HASH_CLIENTID)))
