"""Every fast-kernel variant (items per lane K, LDS stack / word-id capacity, HBM spill)
must give the oracle's match sets: fuzzed tables, config B and config D (wide frontiers that
exercise the stack spill), and deep topics."""

import random

import numpy as np
import pytest

from oracle import cpp as C
from oracle import emqx_ref as R
from tests.test_oracle_fuzz import rand_filter, rand_topic

pytestmark = pytest.mark.gpu

N_VARIANTS = 18


@pytest.fixture(scope="module")
def Engine():
    import torch  # noqa: F401
    from emqx_amd.engine import Engine as E
    return E


@pytest.fixture(scope="module")
def datasets():
    from emqx_amd import workloads as W
    out = {}
    b = W.config_b(n_filters=150_000, n_topics=12_000)
    d = W.config_d(n_filters=40_000, n_topics=2_000)
    for name, wl in (("B", b), ("D", d)):
        o = C.CppOracle(True)
        o.add_packed(*wl.filters)
        counts, ids, _ = o.match_packed(*wl.topics, mode=0, threads=8, stride=1024)
        out[name] = (wl, counts, ids)
    return out


def check_csr(off, ids, counts, oids):
    assert np.array_equal(np.diff(off.astype(np.int64)), counts.astype(np.int64))
    for i in range(len(counts)):
        assert np.array_equal(np.sort(ids[off[i]:off[i + 1]]), oids[i, :counts[i]]), i


@pytest.mark.parametrize("variant", range(N_VARIANTS))
def test_variant_configs(Engine, datasets, variant):
    for name, (wl, counts, oids) in datasets.items():
        e = Engine()
        e.insert_packed(*wl.filters)
        e.commit()
        e.set_tuning("fast_variant", variant)
        off, ids = e.match_packed(*wl.topics, mode=0)
        check_csr(off, ids, counts, oids)
        st = e.stats()
        assert st["last_evals"] > 0


@pytest.mark.parametrize("variant", range(N_VARIANTS))
def test_variant_fuzz_and_deep(Engine, variant):
    rng = random.Random(31 + variant)
    filters = sorted({rand_filter(rng) for _ in range(300)})
    deep = b"/".join(b"w%d" % (i % 5) for i in range(200))
    filters += [deep, deep + b"/#", b"/".join([b"+"] * 120) + b"/#"]
    topics = [rand_topic(rng) for _ in range(700)] + [deep, b"/".join([b"w0"] * 90), b"$SYS/x", b""]
    e = Engine()
    e.insert(filters)
    e.commit()
    e.set_tuning("fast_variant", variant)
    for mode, ref in ((0, R.brute_force_routes), (1, R.brute_force_trie)):
        got = e.match(topics, mode=mode)
        for t, g in zip(topics, got):
            assert g == ref(filters, t), (variant, mode, t[:60])


def test_spill_is_exercised(Engine, datasets):
    """The smallest-stack variant must spill on config D and still be exact."""
    wl, counts, oids = datasets["D"]
    e = Engine()
    e.insert_packed(*wl.filters)
    e.commit()
    e.set_tuning("fast_variant", 5)   # stack 256
    off, ids = e.match_packed(*wl.topics, mode=0)
    check_csr(off, ids, counts, oids)
    assert e.stats()["last_max_stack"] > 256
