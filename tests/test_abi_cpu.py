"""CPU-side checks of the drop-in boundary: the C-ABI library builds, loads and exports every
symbol include/emqx_match.h declares; its CPU entry points (emqx_topic:match/2, wildcard/1)
agree with the reference KATs; without a GPU the engine fails loudly (no CPU fallback)."""

import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def L():
    lib_path = os.path.join(ROOT, "emqx_amd", "_build", "libemqxmatch.so")
    if not os.path.exists(lib_path):
        subprocess.run(["make", "-C", os.path.join(ROOT, "emqx_amd", "csrc"), "-j4"], check=True,
                       capture_output=True)
    from emqx_amd import _lib
    return _lib.lib()


def header_functions(name="emqx_match.h"):
    src = open(os.path.join(ROOT, "include", name)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(emqx_[a-z_]+)\s*\(", src)))


def test_exports_every_declared_symbol(L):
    from emqx_amd import _lib
    declared = header_functions()
    assert len(declared) >= 14
    assert sorted(_lib.EXPORTS) == declared
    for name in declared:
        assert hasattr(L, name), name
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for name in declared:
        assert re.search(r"\bT %s\b" % name, nm), name


def test_exports_every_retain_symbol(L):
    from emqx_amd import _lib
    declared = header_functions("emqx_retain.h")
    assert sorted(_lib.RETAIN_EXPORTS) == declared
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for name in declared:
        assert re.search(r"\bT %s\b" % name, nm), name


def test_version_and_strerror(L):
    assert b"gfx950" in L.emqx_version()
    assert L.emqx_strerror(-4) == b"output capacity too small"


def test_topic_match_kats(L, kats):
    from emqx_amd import topic
    for name, filt, expect in kats["topic_match"]:
        assert topic.match(name.encode(), filt.encode()) is expect, (name, filt)


def test_topic_match_fuzz_vs_oracle(L):
    import random
    from emqx_amd import topic
    from oracle import emqx_ref as R
    from tests.test_oracle_fuzz import rand_filter, rand_topic
    rng = random.Random(3)
    for _ in range(4000):
        f, t = rand_filter(rng), rand_topic(rng)
        assert topic.match(t, f) == R.match(t, f), (t, f)
        assert topic.wildcard(t) == R.wildcard(t)


def test_topic_misc_kats(L, kats):
    from emqx_amd import topic as T
    m = kats["topic_misc"]
    for t, expect in m["wildcard"]["cases"]:
        assert T.wildcard(t.encode()) is expect
    for kind, t in m["validate_ok"]["cases"]:
        assert T.validate((kind, t.encode()))
    for kind, t, err in m["validate_err"]["cases"]:
        if isinstance(t, dict):
            t = "".join("%d/" % i for i in range(66667))
        with pytest.raises(T.TopicError) as ei:
            T.validate((kind, t.encode()))
        assert ei.value.reason == err
    for tf, opts, etf, eopts in m["parse_ok"]["cases"]:
        got = T.parse(tf.encode(), {k: v.encode() if isinstance(v, str) else v for k, v in opts.items()})
        assert got == (etf.encode(), {k: v.encode() if isinstance(v, str) else v for k, v in eopts.items()})
    for tf, opts in m["parse_err"]["cases"]:
        with pytest.raises(T.TopicError):
            T.parse(tf.encode(), {k: v.encode() for k, v in opts.items()})


def test_engine_without_gpu_fails_loudly(L):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from emqx_amd.engine import Engine, EngineError
    with pytest.raises(EngineError) as ei:
        Engine()
    assert ei.value.code == -3   # EMQX_EDEVICE


def test_subtab_without_gpu_fails_loudly(L):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from emqx_amd.fanout import SubTable
    from emqx_amd.engine import EngineError
    with pytest.raises(EngineError) as ei:
        SubTable()
    assert ei.value.code == -3


def test_config_e_shapes():
    import numpy as np
    from emqx_amd import workloads as W
    e = W.config_e(n_filters=20_000, n_subscribers=10_000, n_topics=500)
    shared = e.sub_group != W.NO_GROUP
    assert abs(int(shared.sum()) - 10_000) < 200          # 10% of 100k subscriptions
    assert e.n_subscriptions > 98_000 and e.keys.max() < (1 << 27)
    assert int(e.sub_filter.max()) < 20_000 and int(e.sub_group[shared].max()) < 8
    rows = np.stack([e.sub_filter, e.sub_group, e.sub_id], 1)
    assert len(np.unique(rows, axis=0)) == len(rows)        # no duplicate subscription
    gk = (e.sub_filter[shared].astype(np.uint64) << np.uint64(3)) | e.sub_group[shared].astype(np.uint64)
    sizes = np.unique(gk, return_counts=True)[1]
    assert sizes.max() <= 16 and np.median(sizes) >= 2


def test_workloads_shapes():
    from emqx_amd import workloads as W
    a = W.config_a(n_topics=2000)
    assert a.n_filters == 100_000
    assert W.unpack(a.filters, [0])[0] == b"site0/+/dev0/#"
    ap = W.config_a_prime(subscribers=4, sub_ops=10, publishers=8)
    assert W.unpack(ap.topics, [0])[0] == b"device/2/foo/1/bar/1/2/3/4/5"
    b = W.config_b(n_filters=50_000, n_topics=4000)
    fl = W.unpack(b.filters)
    assert len(set(fl)) == len(fl) == 50_000
    d = W.config_d(n_filters=5000, n_topics=100)
    assert d.n_filters == 5000
    assert all(t.count(b"/") == 15 for t in W.unpack(d.topics))


def build_check(packed):
    import ctypes
    import numpy as np
    from emqx_amd import _lib
    buf, offs = packed
    st = np.zeros(4, np.uint64)
    err = ctypes.create_string_buffer(256)
    rc = _lib.lib().emqx_build_check(buf.ctypes.data_as(ctypes.c_void_p), offs.ctypes.data_as(ctypes.c_void_p),
                                     len(offs) - 1, st.ctypes.data_as(ctypes.c_void_p), err, 256)
    return rc, err.value.decode(), st


@pytest.mark.parametrize("cfg", ["A", "B", "D", "fuzz", "kats"])
def test_builder_invariants(L, cfg, kats):
    """Host table builder (no device): every edge sits at its perfect-hash / cuckoo slot,
    '+' in slot 0, literal filters admit every present word."""
    import random
    from emqx_amd import workloads as W
    from emqx_amd.engine import pack
    from tests.test_oracle_fuzz import rand_filter
    if cfg == "A":
        packed = W.config_a(n_topics=10).filters
    elif cfg == "B":
        packed = W.config_b(n_filters=400_000, n_topics=10).filters
    elif cfg == "D":
        packed = W.config_d(n_filters=100_000, n_topics=10).filters
    elif cfg == "fuzz":
        rng = random.Random(11)
        packed = pack(sorted({rand_filter(rng, 9) for _ in range(20000)}))
    else:
        fl = sorted({op[1].encode() for c in kats["trie_cases"] for op in c["ops"] if op[0] == "insert"})
        packed = pack(fl + [b"a/#/b", b"+", b"#", b"", b"/"])
    rc, err, st = build_check(packed)
    assert rc == 0, err
    assert st[0] >= 1 and st[1] >= 1
