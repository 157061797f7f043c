"""The fan-out oracle (oracle/broker_ref.py) against the reference's own scenarios.

Scenarios transcribed from apps/emqx/test/emqx_shared_sub_SUITE.erl (test_two_messages/2
:315-355, t_hash_topic :181-218, t_not_so_sticky :220-243, t_dispatch :297-309) and the
aggre/route rules of apps/emqx/src/emqx_broker.erl:244-272.  erlang:phash2 values are passed
in as keys (the suite only asserts phash2(T1) rem 2 =/= phash2(T2) rem 2, :192).
"""

import pytest

from oracle import broker_ref as B

NODE = B.NODE


def two_member_broker():
    b = B.Broker()
    b.subscribe(b"foo/bar", "ConnPid1", group=b"group1")
    b.subscribe(b"foo/bar", "ConnPid2", group=b"group1")
    return b


def picked(deliveries):
    assert len(deliveries) == 1 and deliveries[0][2]
    return deliveries[0][1]


@pytest.mark.parametrize("strategy", [B.HASH_CLIENTID])
def test_two_messages_hash_same_client_same_member(strategy):
    b = two_member_broker()
    key = 12345  # phash2(<<"ClientId1">>) stand-in: both messages come from ClientId1
    p1 = picked(b.publish(b"foo/bar", key, strategy))
    p2 = picked(b.publish(b"foo/bar", key, strategy))
    assert p1 == p2


def test_two_messages_round_robin_alternates():
    b = two_member_broker()
    p1 = picked(b.publish(b"foo/bar", 0, B.ROUND_ROBIN))
    p2 = picked(b.publish(b"foo/bar", 0, B.ROUND_ROBIN))
    assert p1 != p2
    assert picked(b.publish(b"foo/bar", 0, B.ROUND_ROBIN)) == p1


def test_hash_topic_different_parity_different_member():
    b = B.Broker()
    b.subscribe(b"foo/#", "ConnPid1", group=b"group1")
    b.subscribe(b"foo/#", "ConnPid2", group=b"group1")
    k1, k2 = 7, 10  # phash2(Topic1) rem 2 =/= phash2(Topic2) rem 2
    assert picked(b.publish(b"foo/bar1", k1, B.HASH_TOPIC)) != picked(b.publish(b"foo/bar2", k2, B.HASH_TOPIC))
    # lists:nth(1 + Key rem N, Subs) with Subs in subscription order
    assert picked(b.publish(b"foo/bar1", 7, B.HASH_TOPIC)) == "ConnPid2"
    assert picked(b.publish(b"foo/bar1", 10, B.HASH_TOPIC)) == "ConnPid1"


def test_not_so_sticky_follows_resubscription():
    b = B.Broker()
    b.subscribe(b"foo/bar", "C1", group=b"group1")
    assert b.publish(b"foo/bar", 0, B.HASH_CLIENTID) == [(b"foo/bar", "C1", True)]
    b.unsubscribe(b"foo/bar", "C1", group=b"group1")
    assert b.router.lookup_routes(b"foo/bar") == []  # last member gone: route deleted
    b.subscribe(b"foo/#", "C1", group=b"group1")
    assert b.publish(b"foo/bar", 0, B.HASH_CLIENTID) == [(b"foo/#", "C1", True)]


def test_dispatch_no_subscribers_then_one():
    b = B.Broker()
    assert b.publish(b"foo", 0) == []
    b.subscribe(b"foo", "S", group=b"group1")
    assert b.publish(b"foo", 0) == [(b"foo", "S", True)]


def test_plain_and_shared_on_overlapping_filters():
    b = B.Broker()
    b.subscribe(b"a/b", "p1")
    b.subscribe(b"a/+", "p1")          # same subscriber, second filter: delivered twice
    b.subscribe(b"a/#", "p2")
    b.subscribe(b"a/#", "g1", group=b"g")
    b.subscribe(b"a/#", "g2", group=b"g")
    b.subscribe(b"a/#", "h1", group=b"h")
    got = sorted(b.publish(b"a/b", 1, B.HASH_CLIENTID), key=repr)
    assert got == sorted([(b"a/b", "p1", False), (b"a/+", "p1", False), (b"a/#", "p2", False),
                          (b"a/#", "g2", True), (b"a/#", "h1", True)], key=repr)
    b.subscribe(b"a/b", "p1")          # idempotent
    assert len(b.publish(b"a/b", 1, B.HASH_CLIENTID)) == 5


def test_aggre_dedups_group_routes_across_nodes():
    routes = [(b"t", "n1@h"), (b"t", (b"g", "n1@h")), (b"t", (b"g", "n2@h"))]
    assert sorted(B.Broker.aggre(routes), key=repr) == sorted([(b"t", "n1@h"), (b"t", b"g")], key=repr)
    assert B.Broker.aggre([(b"t", (b"g", "n1@h"))]) == [(b"t", b"g")]
    assert B.Broker.aggre([]) == []


def test_dollar_and_wildcard_topics_follow_match_routes():
    b = B.Broker()
    b.subscribe(b"#", "all")
    b.subscribe(b"$SYS/#", "sys")
    b.subscribe(b"a/+", "exact-wild")  # a wildcard *topic* publish hits only the identical filter
    assert b.publish(b"$SYS/x", 0) == [(b"$SYS/#", "sys", False)]
    assert sorted(b.publish(b"a/+", 0), key=repr) == [(b"a/+", "exact-wild", False)]


def test_cpp_fanout_lists_agree_with_counts_and_checksums():
    """oracle/fanout_oracle.cpp: the listed deliveries (orf_publish_list, used for ID-for-ID
    checks at config E's full size) give the same per-topic counts and order-free checksums as
    orf_publish, and pair_csr_mismatches finds a swapped pair but not a reordering."""
    import numpy as np
    from oracle import cpp as C
    from emqx_amd import workloads as W
    fw = W.config_e(n_filters=20_000, n_subscribers=5_000, n_topics=2_000, seed=9)
    o = C.CppOracle(True)
    o.add_packed(*fw.wl.filters)
    moff, mids, _ = o.match_csr(*fw.wl.topics, mode=C.MODE_ROUTES, threads=4)
    fo = C.FanoutOracle(fw.sub_filter, fw.sub_id, fw.sub_group)
    counts, sums, total = fo.publish(moff, mids, fw.keys, threads=4)
    off, subs, fils = fo.publish_list(moff, mids, fw.keys, threads=4)
    assert int(off[-1]) == total > 1000
    assert np.array_equal(np.diff(off.astype(np.int64)), counts.astype(np.int64))
    assert np.array_equal(C.delivery_checksums(off, subs, fils), sums)
    assert C.pair_csr_mismatches(off, subs, fils, off, subs, fils).size == 0
    t = int(np.argmax(np.diff(off.astype(np.int64)) > 2))
    a, b = int(off[t]), int(off[t + 1])
    rev = subs.copy()
    rev[a:b] = rev[a:b][::-1]
    fr = fils.copy()
    fr[a:b] = fr[a:b][::-1]
    assert C.pair_csr_mismatches(off, rev, fr, off, subs, fils).size == 0  # order within a topic is free
    bad = subs.copy()
    bad[a] ^= 1
    assert C.pair_csr_mismatches(off, bad, fils, off, subs, fils).tolist() == [t]


# ---- round 4: sticky liveness and dispatch/4's retries (emqx_shared_sub.erl:113-130,234-263,
# 385-393), restated by SharedSub.pick_typed / dispatch -------------------------------------------

def three_member(strategy_members=("A", "B", "C")):
    b = B.Broker()
    for m in strategy_members:
        b.subscribe(b"t/+", m, group=b"g")
    return b


def test_sticky_keeps_an_alive_member_that_unsubscribed():
    """pick(sticky) checks is_active_sub(Sub0, []), i.e. is_process_alive, not membership."""
    b = three_member()
    first = picked(b.publish(b"t/1", 9, B.STICKY, draw=lambda c: c.index("B")))
    assert first == "B"
    b.unsubscribe(b"t/+", "B", group=b"g")
    assert picked(b.publish(b"t/1", 9, B.STICKY)) == "B"      # still alive: still sticky
    b.down("B")
    # dead: do_pick(random, ..., [Sub0]) over All -- [B] = [A, C]
    seen = []
    got = picked(b.publish(b"t/1", 9, B.STICKY, draw=lambda c: (seen.append(list(c)), 1)[1]))
    assert seen == [["A", "C"]] and got == "C"
    assert picked(b.publish(b"t/1", 9, B.STICKY)) == "C"


def test_sticky_dead_member_still_listed_is_excluded_then_retry_when_alone():
    b = three_member(("A",))
    assert picked(b.publish(b"t/1", 1, B.STICKY)) == "A"
    b.down("A")  # not yet cleaned up: still the only member
    assert b.shared.pick_typed(B.STICKY, 1, b"g", b"t/+") == ("retry", "A")
    b.subscribe(b"t/+", "A", group=b"g")  # a live process with that handle again
    assert b.shared.pick_typed(B.STICKY, 1, b"g", b"t/+") == ("fresh", "A")


def test_repick_excludes_failed_then_retries_over_all():
    """dispatch/4: [SubPid | FailedSubs]; do_pick: All -- FailedSubs, [] -> {retry, ...}."""
    b = three_member()
    sh = b.shared
    # hash: 1 + Key rem length(Subs) over the shrinking candidate list
    assert sh.pick_typed(B.HASH_CLIENTID, 4, b"g", b"t/+") == ("fresh", "B")          # 1 + 4 rem 3
    assert sh.pick_typed(B.HASH_CLIENTID, 4, b"g", b"t/+", ["B"]) == ("fresh", "A")   # [A, C]: 1 + 4 rem 2
    assert sh.pick_typed(B.HASH_CLIENTID, 4, b"g", b"t/+", ["A", "B"]) == ("fresh", "C")
    assert sh.pick_typed(B.HASH_CLIENTID, 4, b"g", b"t/+", ["C", "A", "B"]) == ("retry", "B")
    # round_robin: the publisher's Rem advances on every pick, modulo the candidate count
    assert sh.pick_typed(B.ROUND_ROBIN, 7, b"g", b"t/+") == ("fresh", "A")            # first draw: 0
    assert sh.pick_typed(B.ROUND_ROBIN, 7, b"g", b"t/+", ["A"]) == ("fresh", "C")     # (0+1) rem 2 over [B, C]
    assert sh.rr[(7, b"g", b"t/+")] == 1
    assert sh.pick_typed(B.ROUND_ROBIN, 7, b"g", b"t/+", ["B", "C"]) == ("fresh", "A")  # one left: no state
    assert sh.rr[(7, b"g", b"t/+")] == 1
    # sticky: a failed Sub0 is replaced and the replacement sticks
    assert sh.pick_typed(B.STICKY, 3, b"g", b"t/+", draw=lambda c: 2) == ("fresh", "C")
    assert sh.pick_typed(B.STICKY, 3, b"g", b"t/+", ["C"], draw=lambda c: c.index("A")) == ("fresh", "A")
    assert sh.sticky[(3, b"g", b"t/+")] == "A"


def test_dispatch_loop_until_ack_or_retry():
    b = three_member()
    attempts, res = b.shared.dispatch(B.HASH_CLIENTID, 4, b"g", b"t/+", deliver=lambda s: s == "C")
    assert attempts == [("fresh", "B"), ("fresh", "A"), ("fresh", "C")] and res == ("ok", 1)
    attempts, res = b.shared.dispatch(B.HASH_CLIENTID, 4, b"g", b"t/+", deliver=lambda s: False)
    assert attempts[-1] == ("retry", "B") and len(attempts) == 4 and res == ("ok", 1)
    attempts, res = b.shared.dispatch(B.HASH_CLIENTID, 4, b"nogroup", b"t/+", deliver=lambda s: True)
    assert attempts == [] and res == ("error", "no_subscribers")


def test_cleanup_down_removes_memberships_and_empty_group_routes():
    b = B.Broker()
    b.subscribe(b"t/+", "A", group=b"g")
    b.subscribe(b"u/#", "A", group=b"h")
    b.subscribe(b"u/#", "B", group=b"h")
    b.down("A")
    b.cleanup_down("A")
    assert b.shared.subscribers(b"g", b"t/+") == [] and b.shared.subscribers(b"h", b"u/#") == ["B"]
    assert b.publish(b"t/1", 0, B.HASH_CLIENTID) == []
    assert b.publish(b"u/1", 0, B.HASH_CLIENTID) == [(b"u/#", "B", True)]


def test_cpp_round_robin_equals_shared_sub_restatement():
    """oracle/fanout_oracle.cpp orf_publish_list_rr (bench.py's pick-exact check of config E's
    round_robin, counter seeded 0) against broker_ref.SharedSub.pick_subscriber (the restatement
    of emqx_shared_sub.erl:265-285) with the first draw 0: the picks of every message, over two
    calls that carry the state, on random groups of 1-5 members and a few publishers."""
    import numpy as np
    from oracle import cpp as C
    rng = np.random.default_rng(11)
    nf, rows = 40, []
    for f in range(nf):
        for s in rng.choice(50, size=int(rng.integers(0, 3)), replace=False):
            rows.append((f, int(s), 0xFFFFFFFF))
        for g in range(int(rng.integers(0, 3))):
            for s in rng.choice(50, size=int(rng.integers(1, 6)), replace=False):
                rows.append((f, 100 + int(s), g))
    filt, sub, grp = (np.array(x, np.uint32) for x in zip(*rows))
    fo = C.FanoutOracle(filt, sub, grp)
    ss = B.SharedSub()
    for f, s, g in rows:
        if g != 0xFFFFFFFF:
            ss.subscribe(g, f, s)
    n = 300
    counts = rng.integers(0, 4, size=n)
    moff = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    mids = rng.integers(0, nf, size=int(moff[-1])).astype(np.uint32)
    keys = rng.integers(0, 3, size=n).astype(np.uint32)  # three publishers
    for call in range(2):
        off, subs, fils = fo.publish_list(moff, mids, keys, round_robin=True)
        for t in range(n):
            want = []
            for j in range(int(moff[t]), int(moff[t + 1])):
                f = int(mids[j])
                want += [(s, f) for ff, s, g in rows if ff == f and g == 0xFFFFFFFF]
                groups = []
                for ff, s, g in rows:
                    if ff == f and g != 0xFFFFFFFF and g not in groups:
                        groups.append(g)
                for g in groups:
                    members = ss.subscribers(g, f)
                    pick = ss.pick_subscriber(g, f, B.ROUND_ROBIN, int(keys[t]), members, lambda c: 0)
                    want.append((pick, f | 0x80000000))
            got = list(zip(subs[int(off[t]):int(off[t + 1])].tolist(), fils[int(off[t]):int(off[t + 1])].tolist()))
            assert got == want, (call, t)
    fo.rr_reset()
    off2, subs2, _ = fo.publish_list(moff, mids, keys, round_robin=True)
    ss.rr.clear()
    assert subs2.size == subs.size
