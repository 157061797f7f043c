"""Incremental commits (emqx_trie:insert/delete under emqx_router_utils.erl:33-70,
refcounted keys emqx_trie.erl:115-137,235-252) — parity of the HIP engine against brute-force
emqx_topic:match over the live filter set after every commit.

A commit after inserts/deletes either flips meta flags of base-trie slots in place (deleted /
revived filters of the last full build) and rebuilds the small delta trie of filters created
since then (last_commit_kind 1), or does a full rebuild (kind 0).  Match sets must be the same
either way, in all three modes, including '$' topics, wildcard topics (routes mode's byte-
identical lookup walks both tries), root '#', and words that only delta filters contain."""

import random

import pytest

from oracle import emqx_ref as R
from tests.test_oracle_fuzz import rand_filter, rand_topic

pytestmark = pytest.mark.gpu

DEAD = b"\x00dead"


@pytest.fixture(scope="module")
def Engine():
    import torch  # noqa: F401
    from emqx_amd.engine import Engine as E
    from emqx_amd import _lib
    _lib.lib()
    return E


def expected(names, live, topics, mode):
    filters = [f if live.get(i) else DEAD for i, f in enumerate(names)]
    if mode == 0:
        return [R.brute_force_routes(filters, t) for t in topics]
    if mode == 1:
        return [R.brute_force_trie(filters, t) for t in topics]
    wild = [f if R.wildcard(f) else DEAD for f in filters]
    return [R.brute_force_trie(wild, t) for t in topics]


class Model:
    """Engine + the id -> filter / liveness model the oracle checks against."""

    def __init__(self, e):
        self.e = e
        self.names = []
        self.live = {}

    def insert(self, fs):
        ids = self.e.insert(fs)
        for f, i in zip(fs, ids):
            i = int(i)
            if i == len(self.names):
                self.names.append(f)
            assert self.names[i] == f
            self.live[i] = True
        return ids

    def delete(self, ids):
        self.e.delete(ids)
        for i in ids:
            self.live[int(i)] = False

    def check(self, topics, modes=(0, 1, 2)):
        for mode in modes:
            got = self.e.match(topics, mode=mode)
            exp = expected(self.names, self.live, topics, mode)
            for t, g, x in zip(topics, got, exp):
                assert g == x, (mode, t, g, x)


NEW_WORDS = [b"n%d" % i for i in range(12)] + [b"long-word-beyond-sixteen-%d" % i for i in range(4)]


def rand_filter2(rng):
    f = rand_filter(rng)
    if rng.random() < 0.3:  # words the base build never saw
        lv = f.split(b"/")
        lv[rng.randrange(len(lv))] = rng.choice(NEW_WORDS)
        f = b"/".join(lv)
    return f


def rand_topic2(rng):
    t = rand_topic(rng)
    if rng.random() < 0.3:
        lv = t.split(b"/")
        lv[rng.randrange(len(lv))] = rng.choice(NEW_WORDS)
        t = b"/".join(lv)
    return t


@pytest.mark.parametrize("seed", range(4))
def test_incremental_fuzz(Engine, seed):
    rng = random.Random(4100 + seed)
    m = Model(Engine())
    m.insert(sorted({rand_filter(rng) for _ in range(rng.randint(50, 300))}))
    m.e.commit()
    assert m.e.stats()["last_commit_kind"] == 0
    m.e.set_tuning("delta_max", 1 << 20)  # every later commit incremental, however large the delta
    specials = [b"", b"/", b"$", b"$SYS/a", b"+", b"#", b"a/+", b"a/#", b"n1/#", b"+/n2"]
    for step in range(8):
        live_ids = [i for i, v in m.live.items() if v]
        if live_ids:
            m.delete(rng.sample(live_ids, min(len(live_ids), rng.randint(0, 40))))
        dead_ids = [i for i, v in m.live.items() if not v]
        revive = rng.sample(dead_ids, min(len(dead_ids), rng.randint(0, 20)))
        m.insert([m.names[i] for i in revive] + [rand_filter2(rng) for _ in range(rng.randint(0, 40))])
        if step % 3 == 2:  # '#' toggles the root flag of whichever trie holds it
            if m.e.lookup(b"#") is not None and m.live.get(m.e.lookup(b"#")):
                m.delete([m.e.lookup(b"#")])
            else:
                m.insert([b"#"])
        m.e.commit()
        assert m.e.stats()["last_commit_kind"] == 1, step
        m.check([rand_topic2(rng) for _ in range(300)] + specials)


def test_delete_everything_then_refill(Engine):
    rng = random.Random(17)
    m = Model(Engine())
    m.insert(sorted({rand_filter(rng) for _ in range(200)}))
    m.e.commit()
    m.e.set_tuning("delta_max", 1 << 20)
    m.delete([i for i, v in m.live.items() if v])
    m.e.commit()
    assert m.e.stats()["last_commit_kind"] == 1
    topics = [rand_topic(rng) for _ in range(200)]
    assert all(g == [] for g in m.e.match(topics, mode=0))
    m.insert([m.names[i] for i in range(0, len(m.names), 2)] + [b"n0/#", b"+/+/n1"])
    m.e.commit()
    m.check(topics + [b"n0", b"x/y/n1"])


def test_delta_overflow_forces_full_rebuild(Engine):
    rng = random.Random(23)
    m = Model(Engine())
    m.insert(sorted({rand_filter(rng) for _ in range(100)}))
    m.e.commit()
    m.e.set_tuning("delta_max", 10)
    m.insert([b"n%d/+/x%d" % (i, i) for i in range(5)])
    m.e.commit()
    assert m.e.stats()["last_commit_kind"] == 1 and m.e.stats()["delta_filters"] == 5
    m.insert([b"n%d/+/y%d/#" % (i, i) for i in range(20)])
    m.e.commit()
    st = m.e.stats()
    assert st["last_commit_kind"] == 0 and st["delta_filters"] == 0
    topics = [b"n%d/q/y%d/z" % (i, i) for i in range(20)] + [b"n%d/q/x%d" % (i, i) for i in range(5)]
    m.check(topics + [rand_topic2(rng) for _ in range(200)])
    # and incremental again on top of the new base
    m.delete([m.e.lookup(b"n3/+/y3/#")])
    m.e.commit()
    assert m.e.stats()["last_commit_kind"] == 1
    m.check(topics)


def test_incremental_off_matches(Engine):
    rng = random.Random(31)
    a, b = Model(Engine()), Model(Engine())
    b.e.set_tuning("incremental", 0)
    base = sorted({rand_filter(rng) for _ in range(200)})
    for m in (a, b):
        m.insert(base)
        m.e.commit()
    a.e.set_tuning("delta_max", 1 << 20)
    for step in range(4):
        dels = rng.sample(range(len(base)), 30)
        adds = [rand_filter2(rng) for _ in range(30)]
        topics = [rand_topic2(rng) for _ in range(300)]
        for m in (a, b):
            m.delete([i for i in dels if m.live.get(i)])
            m.insert(adds)
            m.e.commit()
        assert a.e.stats()["last_commit_kind"] == 1 and b.e.stats()["last_commit_kind"] == 0
        for mode in (0, 1):
            assert a.e.match(topics, mode=mode) == b.e.match(topics, mode=mode)
        a.check(topics, modes=(0,))


def test_incremental_on_config_b(Engine):
    """A 200k-filter base table, then rounds of 5k deletes + 5k subscribes per commit: every
    commit is incremental and the match CSR equals the oracle's over the live set."""
    import numpy as np
    from emqx_amd import workloads as W
    from emqx_amd.engine import pack
    from oracle import cpp as C
    wl = W.config_b(n_filters=220_000, n_topics=20_000, seed=21)
    allf = W.unpack(wl.filters)
    base, extra = allf[:200_000], allf[200_000:]
    e = Engine()
    e.insert(base)
    e.commit()
    rng = np.random.default_rng(3)
    live = np.zeros(len(allf), dtype=bool)
    live[:200_000] = True
    for r in range(4):
        dels = rng.choice(np.nonzero(live)[0], 5000, replace=False)
        e.delete(sorted(int(i) for i in dels))
        live[dels] = False
        adds = extra[r * 5000:(r + 1) * 5000]
        ids = e.insert(adds)
        assert int(ids[0]) == 200_000 + r * 5000
        live[ids] = True
        e.commit()
        assert e.stats()["last_commit_kind"] == 1
        off, ids_got = e.match_packed(*wl.topics, mode=0)
        # oracle over the live set, ids kept: dead filters become never-matching names
        names = [f if live[i] else b"\x00dead/%d" % i for i, f in enumerate(allf)]
        o = C.CppOracle(True)
        o.add_packed(*pack(names))
        off_o, ids_o, _ = o.match_csr(*wl.topics, mode=C.MODE_ROUTES, threads=8)
        bad = C.csr_mismatches(off, ids_got, off_o, ids_o)  # every topic, ID-for-ID
        assert bad.size == 0, (r, bad[:10])
