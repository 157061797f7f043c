"""The retained-message oracle (oracle/retain_ref.py) pinned to the reference's retainer KATs
(tests/golden/kats.json "retain_cases", from emqx_retainer_SUITE), plus the match-spec
properties its restatement encodes (no '$' rule, '#' matches the parent level, '>' vs '>='
expiry guards)."""

import random

from oracle import emqx_ref as R
from oracle import retain_ref as RR


def run_case(case, table=None):
    t = table or RR.RetainTable()
    for op in case["ops"]:
        apply_op(t, op)
    for now, filt, exp in case["queries"]:
        got = sorted(t.names[i].decode() for i in t.dispatch(filt.encode(), now))
        assert got == sorted(exp), (case["name"], filt, now)
    for op in case.get("then", []):
        apply_op(t, op)
    for now, filt, exp in case.get("after", []):
        got = sorted(t.names[i].decode() for i in t.dispatch(filt.encode(), now))
        assert got == sorted(exp), (case["name"], "after", filt)


def apply_op(t, op):
    if op[0] == "store":
        t.store(op[1].encode(), op[2])
    elif op[0] in ("delete", "publish_empty"):
        t.delete_message(op[1].encode())
    else:
        raise AssertionError(op)


def test_retainer_suite_kats(kats):
    assert len(kats["retain_cases"]) >= 6
    for case in kats["retain_cases"]:
        run_case(case)


def test_condition_quirks():
    t = RR.RetainTable()
    for x in [b"$SYS/a", b"a", b"a/b", b"a//b", b"", b"/"]:
        t.store(x)
    names = lambda ids: sorted(t.names[i] for i in ids)  # noqa: E731
    # no '$' rule in the match spec (emqx_retainer_mnesia.erl:226-246)
    assert names(t.match_messages(b"#", 0)) == sorted(t.names)
    assert names(t.match_messages(b"+/a", 0)) == [b"$SYS/a"]
    # '#' matches the parent level; '+' matches an empty level
    assert names(t.match_messages(b"a/#", 0)) == [b"a", b"a//b", b"a/b"]
    assert names(t.match_messages(b"a/+/b", 0)) == [b"a//b"]
    assert names(t.match_messages(b"+", 0)) == [b"", b"a"]
    assert names(t.match_messages(b"+/+", 0)) == [b"$SYS/a", b"/", b"a/b"]
    # a non-final '#' is a literal token no stored topic has
    assert t.match_messages(b"a/#/b", 0) == []


def test_expiry_guards():
    t = RR.RetainTable()
    t.store(b"x/1", 100)
    t.store(b"x/2", 0)
    assert sorted(t.dispatch(b"x/+", 100)) == [1]          # wildcard: expiry > now
    assert t.dispatch(b"x/1", 100) == [0]                  # plain: expiry >= now
    assert t.dispatch(b"x/1", 101) == []
    assert sorted(t.match_messages(b"x/+", None)) == [0, 1]  # match_delete: no guard


def test_condition_equals_topic_match_without_dollar_rule():
    """For valid filters the match spec equals emqx_topic:match/2 minus its '$' rule."""
    rng = random.Random(3)
    vocab = [b"a", b"b", b"", b"$x"]
    for _ in range(3000):
        d = rng.randint(1, 5)
        topic = b"/".join(rng.choice(vocab) for _ in range(rng.randint(1, 5)))
        lv = [rng.choice(vocab + [b"+"]) for _ in range(d)]
        if rng.random() < 0.4:
            lv[-1] = b"#"
        filt = b"/".join(lv)
        got = RR.cond_match(RR.condition(R.words(filt)), RR.topic2tokens(topic))
        plain = R.match(topic.replace(b"$", b"_"), filt.replace(b"$", b"_"))
        assert got == plain, (topic, filt)


def test_token_trie_equals_brute_force():
    rng = random.Random(8)
    vocab = [b"a", b"b", b"", b"$SYS", b"x$"]
    for _ in range(20):
        names = sorted({b"/".join(rng.choice(vocab) for _ in range(rng.randint(1, 5))) for _ in range(80)})
        expiry = [rng.choice([0, 0, 50, 100, 150]) for _ in names]
        live = [rng.random() < 0.85 for _ in names]
        filters = []
        for _ in range(150):
            lv = [rng.choice(vocab + [b"+", b"+"]) for _ in range(rng.randint(1, 5))]
            if rng.random() < 0.35:
                lv[-1] = b"#"
            if rng.random() < 0.05:
                lv.insert(0, b"#")
            filters.append(b"/".join(lv))
        tt = RR.TokenTrie(names, expiry, live)
        for now in (100, -1):
            bf = RR.brute_force(names, expiry, live, filters, now) if now >= 0 else None
            for k, f in enumerate(filters):
                got = tt.dispatch(f, now)
                if bf is not None:
                    assert got == bf[k], (f, now)
                else:
                    t = RR.RetainTable()
                    for n, e in zip(names, expiry):
                        t.store(n, e)
                    t.delete_ids([i for i, v in enumerate(live) if not v])
                    exp = sorted(t.match_messages(f, None)) if R.wildcard(f) else sorted(
                        [t.ids[f]] if f in t.ids and t.live[t.ids[f]] else [])
                    assert got == exp, (f, "no guard")


def test_cpp_scan_equals_python_oracle():
    """oracle/retain_oracle.cpp (the bench's CPU baseline) == oracle/retain_ref.py."""
    import numpy as np
    from oracle import cpp as C
    rng = random.Random(12)
    vocab = [b"a", b"b", b"", b"$SYS", b"longer-than-sixteen-bytes"]
    names = sorted({b"/".join(rng.choice(vocab) for _ in range(rng.randint(1, 5))) for _ in range(300)})
    expiry = [rng.choice([0, 0, 50, 100, 150]) for _ in names]
    filters = []
    for _ in range(400):
        lv = [rng.choice(vocab + [b"+", b"zz"]) for _ in range(rng.randint(1, 5))]
        if rng.random() < 0.35:
            lv[-1] = b"#"
        filters.append(b"/".join(lv))
    filters += [b"#", b"+", b"", b"#/#"]
    sc = C.RetainScan(*C.pack(names), expiry)
    tt = RR.TokenTrie(names, expiry)
    for now in (100, -1):
        counts, sums = sc.select_packed(*C.pack(filters), now, threads=3)
        for k, f in enumerate(filters):
            x = tt.dispatch(f, now)
            assert int(counts[k]) == len(x) and int(sums[k]) == sum(x), (f, now)
    assert np.all(counts >= 0)
