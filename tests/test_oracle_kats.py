"""Pins the oracle (oracle/emqx_ref.py) to the reference's own known-answer tests.

Every case in tests/golden/kats.json cites the reference test it was transcribed
from.  Trie cases run in both compaction modes, as emqx_trie_SUITE.erl:27-41 does.
"""

import pytest

from oracle import emqx_ref as R


def b(s):
    return s.encode() if isinstance(s, str) else s


def atomize(w):
    return {"''": R.EMPTY, "'+'": R.PLUS, "'#'": R.HASH}.get(w, b(w) if isinstance(w, str) else w)


@pytest.mark.parametrize("compact", [True, False])
def test_trie_suite(kats, compact):
    for case in kats["trie_cases"]:
        t = R.Trie(compact)
        for op, arg in case["ops"]:
            if op == "insert":
                t.insert(b(arg))
            elif op == "delete":
                t.delete(b(arg))
            elif op == "assert_empty":
                assert t.empty() == arg, case["name"]
        for topic, expect in case["queries"]:
            got = sorted(t.match(b(topic)))
            assert got == sorted(b(e) for e in expect), (case["name"], topic, got)
        for topic, n in case.get("len_queries", []):
            assert len(t.match(b(topic))) == n, case["name"]
        for topic, expect in case.get("lookup_topic", []):
            assert t.lookup_topic(b(topic)) == [b(e) for e in expect]


def test_eunit_make_keys(kats):
    for mode, compact in (("no_compact", False), ("compact", True)):
        t = R.Trie(compact)
        for topic, tkey, pkeys in kats["eunit"]["make_keys"][mode]:
            got = t.make_keys(b(topic))
            assert got[0] == (b(tkey[0]), tkey[1])
            assert got[1] == [(b(k), tag) for k, tag in pkeys]


def test_eunit_make_prefixes(kats):
    for mode, compact in (("no_compact", False), ("compact", True)):
        t = R.Trie(compact)
        for topic, expect in kats["eunit"]["make_prefixes"][mode]:
            assert t.make_prefixes(R.words(b(topic))) == [b(e) for e in expect]


def test_eunit_do_compact(kats):
    for topic, expect in kats["eunit"]["do_compact"]["cases"]:
        assert R.do_compact(R.words(b(topic))) == [b(e) for e in expect]


def test_topic_match_kats(kats):
    for name, filt, expect in kats["topic_match"]:
        assert R.match(b(name), b(filt)) is expect, (name, filt)


def test_topic_misc(kats):
    m = kats["topic_misc"]
    for topic, expect in m["wildcard"]["cases"]:
        assert R.wildcard(b(topic)) is expect
    for topic, expect in m["words"]["cases"]:
        assert R.words(b(topic)) == [atomize(w) for w in expect]
    for topic, expect in m["tokens"]["cases"]:
        assert R.tokens(b(topic)) == [b(w) for w in expect]
    for topic, n in m["levels"]["cases"]:
        assert R.levels(b(topic)) == n
    for arg, expect in m["join"]["cases"]:
        ws = R.words(b(arg["words_of"])) if isinstance(arg, dict) else [atomize(w) for w in arg]
        assert R.join(ws) == b(expect)
    for kind, topic in m["validate_ok"]["cases"]:
        assert R.validate((kind, b(topic))) is True
    for kind, topic, err in m["validate_err"]["cases"]:
        if isinstance(topic, dict):   # long_topic(): "0/1/.../66666/" (emqx_topic_SUITE.erl:193-194)
            topic = "".join("%d/" % i for i in range(66667))
        with pytest.raises(R.TopicError) as ei:
            R.validate((kind, b(topic)))
        assert ei.value.args[0] == err
    for parent, w, expect in m["prepend"]["cases"]:
        p = atomize(parent) if parent == "'+'" else (None if parent is None else b(parent))
        assert R.prepend(p, b(w)) == b(expect)
    for var, val, topic, expect in m["feed_var"]["cases"]:
        assert R.feed_var(b(var), b(val), b(topic)) == b(expect)
    for tf, opts, etf, eopts in m["parse_ok"]["cases"]:
        got_tf, got_opts = R.parse(b(tf), {k: b(v) if isinstance(v, str) else v for k, v in opts.items()})
        assert got_tf == b(etf)
        assert got_opts == {k: b(v) if isinstance(v, str) else v for k, v in eopts.items()}
    for tf, opts in m["parse_err"]["cases"]:
        with pytest.raises(R.TopicError):
            R.parse(b(tf), {k: b(v) for k, v in opts.items()})


@pytest.mark.parametrize("compact", [True, False])
def test_router_suite(kats, compact):
    for case in kats["router_cases"]:
        r = R.Router(compact)
        for t in case["add"]:
            r.add_route(b(t))
        for topic, expect in case["queries"]:
            got = sorted(t for t, _ in r.match_routes(b(topic)))
            assert got == sorted(b(e) for e in expect)
        for t in case["add"]:
            r.delete_route(b(t))
        for topic, expect in case["then_delete_all"]:
            assert r.match_routes(b(topic)) == []
        assert r.trie.empty()


@pytest.mark.parametrize("compact", [True, False])
def test_client_suite(kats, compact):
    c = kats["client"]
    for key in ("overlapping", "dollar"):
        r = R.Router(compact)
        for s in c[key]["subs"]:
            r.add_route(b(s))
        got = sorted(t for t, _ in r.match_routes(b(c[key]["topic"])))
        assert got == sorted(b(e) for e in c[key]["expect"])


@pytest.mark.parametrize("compact", [True, False])
def test_broker_bench_one_route(kats, compact):
    """emqx_broker_bench.erl:161-162: `[_] = emqx_router:match_routes(Topic)`."""
    bench = kats["bench"]
    r = R.Router(compact)
    sub = bench["sub_ptn"]
    subs, ops = 8, 50   # reduced: same pattern, fewer ids/nums
    for i in range(1, subs + 1):
        for n in range(1, ops + 1):
            r.add_route(b(sub.replace("{{id}}", str(i)).replace("{{num}}", str(n))))
    for pid in range(1, bench["publishers"] + 1):
        topic = bench["pub_ptn"].replace("{{id}}", str((pid % subs) + 1)).replace("{{num}}", "1")
        assert len(r.match_routes(b(topic))) == bench["expect_routes_per_topic"]
