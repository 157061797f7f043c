"""Incremental commits patched into the committed table (emqx_amd/csrc/live_trie.cpp), on the
CPU: the engine's own filter store, builder and in-place patcher, walked on the host by the
kernels' lookup and emission rules (emqx_htrie_*, include/emqx_match.h).

Reference semantics: emqx_trie:insert/1 / delete/1 (apps/emqx/src/emqx_trie.erl:115-137) under
emqx_router_utils.erl:33-70; match sets as emqx_router:match_routes/1 (emqx_router.erl:128-140)
and the router's wildcard-only trie.  Every commit is followed by a full comparison with the
brute-force oracle (oracle/emqx_ref.py, pinned to the reference's KATs) and by the lookup
invariants of every reachable node; the same table rebuilt from scratch must agree too."""

import ctypes
import random

import numpy as np
import pytest

from oracle import emqx_ref as R
from tests.test_oracle_fuzz import rand_filter, rand_topic

DEAD = b"\x00dead"


def pack(items):
    offs = np.zeros(len(items) + 1, dtype=np.uint64)
    if items:
        offs[1:] = np.cumsum([len(x) for x in items])
    buf = np.frombuffer(b"".join(items) or b"\0", dtype=np.uint8).copy()
    return buf, offs


class HostTrie:
    def __init__(self, spare=0, threads=1):
        from emqx_amd import _lib
        self.L = _lib.lib()
        self.h = ctypes.c_void_p()
        assert self.L.emqx_htrie_create(spare, threads, ctypes.byref(self.h)) == 0

    def __del__(self):
        if getattr(self, "h", None):
            self.L.emqx_htrie_destroy(self.h)

    def insert(self, fs):
        buf, offs = pack(fs)
        ids = np.zeros(max(len(fs), 1), dtype=np.uint32)
        assert self.L.emqx_htrie_insert(self.h, buf.ctypes.data, offs.ctypes.data, len(fs), ids.ctypes.data) == 0
        return ids[:len(fs)].tolist()

    def delete(self, ids):
        a = np.asarray(ids, dtype=np.uint32)
        assert self.L.emqx_htrie_delete(self.h, a.ctypes.data if a.size else None, a.size) == 0

    def commit(self, full=False):
        st = np.zeros(8, dtype=np.uint64)
        assert self.L.emqx_htrie_commit(self.h, int(full), st.ctypes.data) == 0
        return dict(zip(["kind", "relocations", "in_place", "patches", "new_slots", "used", "cap", "garbage"],
                        st.tolist()))

    def match(self, topics, mode=0):
        buf, offs = pack(topics)
        out_off = np.zeros(len(topics) + 1, dtype=np.uint64)
        cap = 1 << 20
        ids = np.zeros(cap, dtype=np.uint32)
        n = ctypes.c_uint64()
        rc = self.L.emqx_htrie_match(self.h, mode, buf.ctypes.data, offs.ctypes.data, len(topics),
                                     out_off.ctypes.data, ids.ctypes.data, cap, ctypes.byref(n))
        assert rc == 0
        return [sorted(ids[out_off[i]:out_off[i + 1]].tolist()) for i in range(len(topics))]

    def check(self):
        err = ctypes.create_string_buffer(256)
        rc = self.L.emqx_htrie_check(self.h, err, 256)
        assert rc == 0, err.value.decode()


class Model:
    def __init__(self, t):
        self.t, self.names, self.live = t, [], {}

    def insert(self, fs):
        ids = self.t.insert(fs)
        for f, i in zip(fs, ids):
            if i == len(self.names):
                self.names.append(f)
            assert self.names[i] == f
            self.live[i] = True
        return ids

    def delete(self, ids):
        self.t.delete(ids)
        for i in ids:
            self.live[i] = False

    def filters(self):
        return [f if self.live.get(i) else DEAD for i, f in enumerate(self.names)]

    def check(self, topics):
        self.t.check()
        fl = self.filters()
        wild = [f if R.wildcard(f) else DEAD for f in fl]
        for mode in (0, 2):
            got = self.t.match(topics, mode=mode)
            for tp, g in zip(topics, got):
                x = R.brute_force_routes(fl, tp) if mode == 0 else R.brute_force_trie(wild, tp)
                assert g == x, (mode, tp, g, x)


NEW = [b"n%d" % i for i in range(10)] + [b"long-word-beyond-sixteen-bytes-%d" % i for i in range(3)]


def rand_filter2(rng):
    f = rand_filter(rng, maxd=8)
    if rng.random() < 0.4:
        lv = f.split(b"/")
        lv[rng.randrange(len(lv))] = rng.choice(NEW)
        f = b"/".join(lv)
    return f


def rand_topic2(rng):
    t = rand_topic(rng, maxd=9, allow_wild=False)
    if rng.random() < 0.4:
        lv = t.split(b"/")
        lv[rng.randrange(len(lv))] = rng.choice(NEW)
        t = b"/".join(lv)
    return t


SPECIALS = [b"", b"/", b"$", b"$SYS/a", b"a", b"n1", b"n1/n2", b"a/b/c/d/e/f/g/h/i"]


@pytest.mark.parametrize("seed", range(6))
def test_incremental_commits_equal_oracle(seed):
    rng = random.Random(7100 + seed)
    m = Model(HostTrie())
    m.insert(sorted({rand_filter(rng) for _ in range(rng.randint(0, 200))}))
    assert m.t.commit()["kind"] == 0
    for step in range(8):
        live = [i for i, v in m.live.items() if v]
        if live:
            m.delete(rng.sample(live, min(len(live), rng.randint(0, 30))))
        dead = [i for i, v in m.live.items() if not v]
        m.insert([m.names[i] for i in rng.sample(dead, min(len(dead), rng.randint(0, 15)))]
                 + [rand_filter2(rng) for _ in range(rng.randint(0, 60))])
        if step % 4 == 3:  # the root's '#' and '+' filters come and go
            for f in (b"#", b"+", b"+/#"):
                i = m.t.insert([f])[0] if f not in m.names else m.names.index(f)
                if i == len(m.names):
                    m.names.append(f)
                if m.live.get(i):
                    m.delete([i])
                else:
                    m.insert([f])
        st = m.t.commit()
        assert st["kind"] == 1, step
        m.check([rand_topic2(rng) for _ in range(150)] + SPECIALS)
    # the patched table and a fresh build agree
    topics = [rand_topic2(rng) for _ in range(400)] + SPECIALS
    before = m.t.match(topics)
    m.t.commit(full=True)
    m.t.check()
    assert m.t.match(topics) == before


def test_wide_nodes_relocate_and_fill_buckets():
    """A node grows from one child to thousands across commits: perfect-hash arrays fill and
    relocate, then turn into 2-slot bucket arrays that take further words in place or via
    their secondary bucket."""
    m = Model(HostTrie(spare=1 << 20))
    m.insert([b"root/x"])
    m.t.commit()
    rng = random.Random(3)
    stats = []
    for k in range(30):
        m.insert([b"root/w%d/%s" % (k * 100 + j, rng.choice([b"+", b"a", b"#"])) for j in range(100)])
        stats.append(m.t.commit())
    assert all(s["kind"] == 1 for s in stats)
    assert sum(s["relocations"] for s in stats) > 5
    assert sum(s["in_place"] for s in stats) > 1000
    topics = [b"root/w%d/a" % rng.randrange(3100) for _ in range(300)] + [b"root/x", b"root/w5/zz/q"]
    m.check(topics)


def test_spare_exhaustion_falls_back_to_full_build():
    m = Model(HostTrie(spare=64))
    m.insert([b"a/b"])
    m.t.commit()
    kinds = []
    for k in range(20):
        m.insert([b"a/%d/c/d" % k, b"x%d/+/#" % k])
        kinds.append(m.t.commit()["kind"])
    assert 0 in kinds and 1 in kinds
    m.check([b"a/%d/c/d" % k for k in range(20)] + [b"x%d/q/r" % k for k in range(20)] + [b"a/b"])


def test_commit_work_is_proportional_to_churn():
    """Per-commit slot traffic does not grow with earlier commits: the same churn costs about
    the same new slots and in-place rewrites in the first and in the last of 30 commits."""
    from emqx_amd import workloads as W
    wl = W.config_b(n_filters=60_000, n_topics=2000, seed=21)
    names = W.unpack(wl.filters)
    m = Model(HostTrie(spare=1 << 22))
    m.insert(names[:30_000])
    m.t.commit()
    rng = np.random.default_rng(5)
    new_slots = []
    nxt = 30_000
    for r in range(30):
        live = [i for i, v in m.live.items() if v]
        m.delete(sorted(int(i) for i in rng.choice(live, 500, replace=False)))
        m.insert(names[nxt:nxt + 500])
        nxt += 500
        st = m.t.commit()
        assert st["kind"] == 1
        new_slots.append(st["new_slots"] + 2 * st["patches"])
    assert np.mean(new_slots[-5:]) < 2.0 * np.mean(new_slots[:5])
    # every topic of the batch against the C++ oracle over the live set (ids kept)
    from oracle import cpp as C
    m.t.check()
    o = C.CppOracle(True)
    o.add([f if m.live.get(i) else b"\x00dead/%d" % i for i, f in enumerate(m.names)])  # ids kept
    off_o, ids_o, _ = o.match_csr(*wl.topics, mode=C.MODE_ROUTES, threads=4)
    got = m.t.match(W.unpack(wl.topics))
    off_g = np.concatenate([[0], np.cumsum([len(g) for g in got])])
    ids_g = np.array([x for g in got for x in g], dtype=np.uint32)
    assert C.csr_mismatches(off_g, ids_g, off_o, ids_o).size == 0


def test_threaded_commits_equal_oracle():
    """Commits large enough to run on several threads (flips in parallel, inserts grouped by
    first-level node): every topic of a config-B batch equals the C++ oracle over the live set,
    and the patched table equals the same churn applied on one thread."""
    from emqx_amd import workloads as W
    from oracle import cpp as C
    wl = W.config_b(n_filters=40_000, n_topics=3000, seed=23)
    names = W.unpack(wl.filters)
    ms = [Model(HostTrie(spare=1 << 22, threads=t)) for t in (1, 6)]
    for m in ms:
        m.insert(names[:20_000])
        m.t.commit()
    rng = np.random.default_rng(9)
    nxt = 20_000
    for r in range(4):
        live = [i for i, v in ms[0].live.items() if v]
        dels = sorted(int(i) for i in rng.choice(live, 3000, replace=False))
        for m in ms:
            m.delete(dels)
            m.insert(names[nxt:nxt + 5000] + [b"new%d/+/x" % (r * 10 + j) for j in range(5)])
            assert m.t.commit()["kind"] == 1
        nxt += 5000
    topics = W.unpack(wl.topics)
    outs = [m.t.match(topics) for m in ms]
    assert outs[0] == outs[1]
    m = ms[1]
    m.t.check()
    o = C.CppOracle(True)
    o.add([f if m.live.get(i) else b"\x00dead/%d" % i for i, f in enumerate(m.names)])
    off_o, ids_o, _ = o.match_csr(*wl.topics, mode=C.MODE_ROUTES, threads=4)
    off_g = np.concatenate([[0], np.cumsum([len(g) for g in outs[1]])])
    ids_g = np.array([x for g in outs[1] for x in g], dtype=np.uint32)
    assert C.csr_mismatches(off_g, ids_g, off_o, ids_o).size == 0


def test_partitioned_build_equals_single_thread_build():
    """A full build of >= 200K filters runs its trie pass in partitions by first level on
    several threads (tables.cpp build_tables); its table must answer exactly like the
    one-partition build, pass the lookup self-check, and survive incremental commits on top.
    Checked against the C++ oracle on a config-B sample (emqx_trie.erl:315-334 semantics)."""
    from emqx_amd import workloads as W
    from oracle import cpp as C
    b = W.config_b(n_filters=240_000, n_topics=3000, seed=21)
    fl = W.unpack(b.filters)
    topics = W.unpack(b.topics) + [b"", b"/", b"#", b"+/x"]
    one, many = HostTrie(threads=1), HostTrie(threads=6)
    for t in (one, many):
        t.insert(fl)
        t.commit(full=True)
        t.check()
    o = C.CppOracle(True)
    o.add_packed(*b.filters)
    tb, to = pack(topics)
    off_o, ids_o, _ = o.match_csr(tb, to, mode=C.MODE_ROUTES, threads=4)
    want = [sorted(ids_o[off_o[i]:off_o[i + 1]].tolist()) for i in range(len(topics))]
    for mode in (0, 2):
        a, m = one.match(topics, mode=mode), many.match(topics, mode=mode)
        assert a == m, mode
        if mode == 0:
            assert a == want
    # incremental commits patched into the partitioned build answer like a full rebuild
    rng = random.Random(3)
    extra = [b"zz%d/" % k + rand_filter(rng) for k in range(400)]
    sample = [rand_topic(rng) for _ in range(200)] + [b"zz%d/a/b" % k for k in range(0, 400, 7)]
    for t, full in ((many, False), (one, True)):
        ids = t.insert(extra)
        t.delete(ids[:50])
        t.commit(full=full)
        t.check()
    assert many.match(sample, mode=0) == one.match(sample, mode=0)
