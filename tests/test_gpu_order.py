"""Walk order (emqx_set_tuning "order"): a batch walked in prefix-key order,
with tiles dealt to XCDs in contiguous ranges, must return exactly the CSR of the unordered
walk — same offsets in the caller's order, same per-topic filter-id sets — and equal the
oracle.  Covers deep (deferred) topics, empty topics, wildcard topics, a batch whose bytes
outgrow the reordered buffer's first guess (the CTRL_ERR_ORDER_CAP rerun) and batches that
do not start at byte 0."""

import random

import numpy as np
import pytest

from oracle import cpp as C
from tests.test_gpu_parity import csr_equal, oracle_ids
from tests.test_oracle_fuzz import rand_filter, rand_topic

pytestmark = pytest.mark.gpu

SETTINGS = [  # (level_bits, sort_bits, deal)
    (4, 64, 1), (8, 64, 1), (8, 16, 1), (6, 64, 0), (1, 3, 1),
]


@pytest.fixture(scope="module")
def Engine():
    import torch  # noqa: F401
    from emqx_amd.engine import Engine as E
    from emqx_amd import _lib
    _lib.lib()
    return E


def pack(topics):
    offs = np.zeros(len(topics) + 1, dtype=np.uint64)
    offs[1:] = np.cumsum([len(t) for t in topics])
    return np.frombuffer(b"".join(topics), dtype=np.uint8).copy(), offs


def ordered_csr(e, tb, to, mode, lb, sb, deal):
    e.set_tuning("order", 1)
    e.set_tuning("order_level_bits", lb)
    e.set_tuning("order_sort_bits", sb)
    e.set_tuning("order_deal", deal)
    try:
        return e.match_packed(tb, to, mode=mode)
    finally:
        e.set_tuning("order", 0)


def same_csr(a, b):
    (o1, i1), (o2, i2) = a, b
    if not np.array_equal(o1, o2):
        bad = np.nonzero(o1 != o2)[0]
        raise AssertionError(f"offsets differ at {bad.size} positions, first {bad[:8]}, n={len(o1) - 1}, "
                             f"totals {o1[-1]} vs {o2[-1]}, ids {i1.size} vs {i2.size}")
    for k in range(len(o1) - 1):
        assert np.array_equal(np.sort(i1[o1[k]:o1[k + 1]]), np.sort(i2[o2[k]:o2[k + 1]])), k


def test_order_config_d(Engine):
    from emqx_amd import workloads as W
    d = W.config_d(n_filters=30_000, n_topics=20_000)
    e = Engine()
    e.insert_packed(*d.filters)
    e.commit()
    e.set_tuning("order", 0)
    base = e.match_packed(*d.topics, mode=0)
    counts, oids = oracle_ids(d.filters, d.topics)
    csr_equal(*base, counts, oids)
    for lb, sb, deal in SETTINGS:
        same_csr(base, ordered_csr(e, *d.topics, 0, lb, sb, deal))
    assert e.stats()["last_evals"] > 0


def test_order_config_b(Engine):
    from emqx_amd import workloads as W
    b = W.config_b(n_filters=300_000, n_topics=50_000)
    e = Engine()
    e.insert_packed(*b.filters)
    e.commit()
    for mode in (0, 2):
        off, ids = ordered_csr(e, *b.topics, mode, 8, 64, 1)
        counts, oids = oracle_ids(b.filters, b.topics, mode=mode)
        csr_equal(off, ids, counts, oids)


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_order_fuzz_with_deep_and_long_topics(Engine, mode):
    rng = random.Random(4242 + mode)
    filters = sorted({rand_filter(rng) for _ in range(400)})
    deep = b"/".join(b"w%d" % (i % 5) for i in range(200))
    filters += [b"#", b"w0/#", deep + b"/#", b"/".join([b"+"] * 200)]
    topics = [rand_topic(rng) for _ in range(3000)]
    topics += [b"", b"/", b"$", b"$/x", b"+", b"#", b"a/#/b", deep, deep + b"/w1"]
    topics += [b"w0/" + b"L" * rng.randint(100, 600) + b"/x" for _ in range(300)]  # > 48 B per topic
    rng.shuffle(topics)
    e = Engine()
    e.insert(filters)
    e.commit()
    tb, to = pack(topics)
    e.set_tuning("order", 0)
    base = e.match_packed(tb, to, mode=mode)
    for lb, sb, deal in SETTINGS:
        same_csr(base, ordered_csr(e, tb, to, mode, lb, sb, deal))


def test_order_device_batch_not_at_byte_zero(Engine):
    """Device entry point with offsets that start inside the byte buffer."""
    import torch
    from emqx_amd import workloads as W
    d = W.config_d(n_filters=20_000, n_topics=5000)
    e = Engine()
    e.insert_packed(*d.filters)
    e.commit()
    tb, to = d.topics
    pad = 1000
    dev = torch.device("cuda", 0)
    t_bytes = torch.from_numpy(np.concatenate([np.full(pad, 0x41, np.uint8), tb])).to(dev)
    t_offs = torch.from_numpy((to.astype(np.int64) + pad)).to(dev)
    n = len(to) - 1
    cap = 1 << 24
    res = []
    for order in (0, 1):
        e.set_tuning("order", order)
        d_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
        d_ids = torch.empty(cap, dtype=torch.int32, device=dev)
        tot = e.match_device(t_bytes.data_ptr(), t_offs.data_ptr(), n, d_off.data_ptr(), d_ids.data_ptr(), cap)
        off = d_off.cpu().numpy()
        res.append((off, d_ids[:tot].cpu().numpy().view(np.uint32)))
    e.set_tuning("order", -1)
    same_csr(res[0], res[1])
    counts, oids = oracle_ids(d.filters, d.topics)
    csr_equal(*res[1], counts, oids)


def test_order_tuning_keys_validate(Engine):
    from emqx_amd.engine import EngineError
    e = Engine()
    for key, bad in (("order", 2), ("order_level_bits", 33), ("order_sort_bits", 0)):
        with pytest.raises(EngineError):
            e.set_tuning(key, bad)


def test_order_concurrent_callers(Engine):
    """Several host threads matching through one engine with the walk order forced on: each
    call reorders in its own workspace, and every caller gets the unordered walk's CSR."""
    import threading
    from emqx_amd import workloads as W
    d = W.config_d(n_filters=20_000, n_topics=16_000, seed=8)
    e = Engine()
    e.insert_packed(*d.filters)
    e.commit()
    tb, to = d.topics
    n = len(to) - 1
    slices = [(k * n // 4, (k + 1) * n // 4) for k in range(4)]

    def part(lo, hi):
        o = (to[lo:hi + 1] - to[lo]).astype(np.uint64)
        return tb[int(to[lo]):int(to[hi])].copy(), o

    e.set_tuning("order", 0)
    want = [e.match_packed(*part(lo, hi), mode=0) for lo, hi in slices]
    e.set_tuning("order", 1)
    got = [None] * 4
    errs = []

    def run(k):
        try:
            for _ in range(3):
                got[k] = e.match_packed(*part(*slices[k]), mode=0)
        except Exception as x:  # surfaced below
            errs.append(x)

    th = [threading.Thread(target=run, args=(k,)) for k in range(4)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    e.set_tuning("order", -1)
    assert not errs, errs
    for w, g in zip(want, got):
        same_csr(w, g)
