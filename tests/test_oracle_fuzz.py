"""Cross-checks the oracle's three formulations on fuzzed tables:
compact DFS == non-compact DFS == brute-force emqx_topic:match/2, for emqx_trie:match
(trie holding exact AND wildcard filters, as emqx_trie_SUITE inserts) and for
emqx_router:match_routes (trie holding wildcard filters only)."""

import random

import pytest

from oracle import emqx_ref as R

VOCAB = [b"a", b"b", b"c", b"", b"$SYS", b"$x", b"dev", b"x$"]


def rand_filter(rng, maxd=6):
    d = rng.randint(1, maxd)
    ws = []
    for i in range(d):
        r = rng.random()
        if r < 0.25:
            ws.append(b"+")
        elif r < 0.32 and i == d - 1:
            ws.append(b"#")
        else:
            ws.append(rng.choice(VOCAB))
    return b"/".join(ws)


def rand_topic(rng, maxd=7, allow_wild=True):
    d = rng.randint(1, maxd)
    ws = []
    for _ in range(d):
        if allow_wild and rng.random() < 0.03:
            ws.append(rng.choice([b"+", b"#"]))
        else:
            ws.append(rng.choice(VOCAB))
    return b"/".join(ws)


@pytest.mark.parametrize("seed", range(12))
def test_trie_modes_equal_brute_force(seed):
    rng = random.Random(seed)
    filters = sorted({rand_filter(rng) for _ in range(rng.randint(5, 120))})
    index = {f: i for i, f in enumerate(filters)}
    tc, tn = R.Trie(True), R.Trie(False)
    for f in filters:
        tc.insert(f)
        tn.insert(f)
    for _ in range(300):
        t = rand_topic(rng)
        bf = R.brute_force_trie(filters, t)
        mc = tc.match(t)
        mn = tn.match(t)
        assert len(mc) == len(set(mc)) and len(mn) == len(set(mn))   # S6: no duplicates
        assert sorted(index[f] for f in mc) == bf, (t, mc, bf)
        assert sorted(index[f] for f in mn) == bf, (t, mn, bf)


@pytest.mark.parametrize("seed", range(8))
def test_router_equal_brute_force_with_deletes(seed):
    rng = random.Random(100 + seed)
    filters = sorted({rand_filter(rng) for _ in range(rng.randint(5, 100))})
    live = set(filters)
    rc, rn = R.Router(True), R.Router(False)
    for f in filters:
        rc.add_route(f)
        rn.add_route(f)
    for f in rng.sample(filters, len(filters) // 3):     # refcounted prefix removal
        rc.delete_route(f)
        rn.delete_route(f)
        live.discard(f)
    index = {f: i for i, f in enumerate(filters)}
    live_list = [f if f in live else None for f in filters]
    for _ in range(300):
        t = rand_topic(rng)
        bf = [i for i in R.brute_force_routes([f if f is not None else b"\x00dead" for f in live_list], t)
              if live_list[i] is not None]
        assert R.router_match_ids(rc, index, t) == bf, t
        assert R.router_match_ids(rn, index, t) == bf, t


def test_evals_counts_root_and_dollar():
    filters = [b"+/a", b"x/+", b"#", b"$SYS/#"]
    # a/b: F0={root}, F1={root/+}, F2={+/... none for b? '+/a' needs 'a'} -> 1 + 1 + 0
    assert R.evals(filters, [b"a/b"]) == [2]
    # x/a: F1={x, +}, F2={x/+, +/a} -> 1+2+2
    assert R.evals(filters, [b"x/a"]) == [5]
    # $SYS/a: root '+' skipped: F1={$SYS}, F2={} ('$SYS/#' is a node '#', never followed)
    assert R.evals(filters, [b"$SYS/a"]) == [2]
    assert R.evals(filters, [b"a/+"]) == [0]
