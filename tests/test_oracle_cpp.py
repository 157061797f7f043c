"""Pins the C++ oracle (oracle/trie_oracle.cpp) to the Python oracle, which is pinned
to the reference's KATs (test_oracle_kats.py)."""

import random

import pytest

from oracle import cpp as C
from oracle import emqx_ref as R
from tests.test_oracle_fuzz import rand_filter, rand_topic


@pytest.fixture(scope="module", autouse=True)
def _built():
    C.lib()


@pytest.mark.parametrize("compact", [True, False])
def test_cpp_trie_suite_kats(kats, compact):
    for case in kats["trie_cases"]:
        if any(op == "assert_empty" for op, _ in case["ops"]):
            continue
        o = C.CppOracle(compact, trie_all=True)
        names = []
        for op, arg in case["ops"]:
            if op == "insert":
                o.add([arg.encode()])
                names.append(arg.encode())
            elif op == "delete":
                o.delete([arg.encode()])
        index = {}
        for f in names:
            index.setdefault(f, len(index))
        inv = {v: k for k, v in index.items()}
        for topic, expect in case["queries"]:
            got = sorted(inv[i] for i in o.match_lists([topic.encode()], C.MODE_TRIE)[0])
            assert got == sorted(e.encode() for e in expect), (case["name"], topic)


@pytest.mark.parametrize("seed", range(10))
@pytest.mark.parametrize("compact", [True, False])
def test_cpp_equals_python(seed, compact):
    rng = random.Random(7000 + seed)
    filters = sorted({rand_filter(rng) for _ in range(rng.randint(5, 150))})
    topics = [rand_topic(rng) for _ in range(400)]
    # router semantics (wildcard-only trie)
    o = C.CppOracle(compact)
    ids = o.add(filters)
    assert list(ids) == list(range(len(filters)))
    got = o.match_lists(topics, C.MODE_ROUTES, threads=2)
    for t, g in zip(topics, got):
        assert g == R.brute_force_routes(filters, t), t
    # trie semantics with every filter inserted (emqx_trie_SUITE style, incl. '$x' quirk)
    o2 = C.CppOracle(compact, trie_all=True)
    o2.add(filters)
    got2 = o2.match_lists(topics, C.MODE_TRIE)
    for t, g in zip(topics, got2):
        assert g == R.brute_force_trie(filters, t), t
    # evals cost model
    buf, offs = C.pack(topics)
    assert list(o.evals_packed(buf, offs)) == R.evals(filters, topics)


def test_cpp_topic_match_kats(kats):
    for name, filt, expect in kats["topic_match"]:
        assert C.topic_match(name.encode(), filt.encode()) is expect, (name, filt)


def test_cpp_delete_refcount():
    rng = random.Random(5)
    filters = sorted({rand_filter(rng) for _ in range(200)})
    o = C.CppOracle(True)
    o.add(filters)
    gone = set(rng.sample(filters, 70))
    o.delete(list(gone))
    topics = [rand_topic(rng, allow_wild=False) for _ in range(300)]
    live = [f if f not in gone else b"\x00" for f in filters]
    for t, g in zip(topics, o.match_lists(topics)):
        assert g == R.brute_force_routes(live, t)
