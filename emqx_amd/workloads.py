"""Synthetic subscription tables and topic streams for the BASELINE configs (SURVEY §8 d).

Everything is generated with numpy PCG64 at fixed seeds and returned PACKED:
``(uint8 bytes, uint64 offsets[n+1])`` — the engine's batch format — so 10M-filter tables
never become Python lists.  Filter ids are 0-based indices in the returned (deduplicated,
generation-ordered) filter list.

Level codes used while composing: >= 0 word id in that level's vocabulary, PLUS_CODE = '+',
HASH_CODE = '#', ABSENT = level not present.
"""

from __future__ import annotations

import os
from dataclasses import dataclass
from typing import List, Sequence, Tuple

import numpy as np

PLUS_CODE = -1
HASH_CODE = -2
ABSENT = -3

B_VOCAB = [64, 1024, 4096, 65536, 65536, 1024, 256, 64]
B_PREFIX = [b"region", b"site", b"bldg", b"dev", b"sensor", b"metric", b"unit", b"q"]


@dataclass
class Workload:
    name: str
    filters: Tuple[np.ndarray, np.ndarray]   # packed filters
    topics: Tuple[np.ndarray, np.ndarray]    # packed topics

    @property
    def n_filters(self) -> int:
        return len(self.filters[1]) - 1

    @property
    def n_topics(self) -> int:
        return len(self.topics[1]) - 1


# ---------------------------------------------------------------------------------------
# packing helpers
# ---------------------------------------------------------------------------------------

def vocab_table(words: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    offs = np.zeros(len(words) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(w) for w in words])
    buf = np.frombuffer(b"".join(words), dtype=np.uint8).copy() if offs[-1] else np.zeros(0, np.uint8)
    return buf, offs


PAD = 0xFF  # never a byte of a generated word


def _padded(vb: np.ndarray, vo: np.ndarray) -> np.ndarray:
    """(bytes, offsets) vocabulary -> [V, maxlen] uint8 table padded with PAD."""
    lens = np.diff(vo)
    V, W = len(lens), int(lens.max(initial=0))
    t = np.full((V, max(W, 1)), PAD, dtype=np.uint8)
    if V and W:
        col = np.arange(W)[None, :]
        inside = col < lens[:, None]
        t[inside] = vb[(vo[:-1, None] + col)[inside]]
    return t


def compose(codes: np.ndarray, level_vocabs: List[Tuple[np.ndarray, np.ndarray]],
            chunk: int = 1 << 20) -> Tuple[np.ndarray, np.ndarray]:
    """codes[N, D] level codes -> packed '/'-joined strings.  Levels must be contiguous from
    level 0 (ABSENT only as a suffix).  level_vocabs[l] = (bytes, offsets) of level l.

    Each chunk is laid out as a fixed-width byte matrix (padded words + separators) and
    compacted with one boolean mask, which keeps the 10M-filter tables to a few seconds."""
    N, D = codes.shape
    tables = []
    for l in range(D):
        vb, vo = level_vocabs[min(l, len(level_vocabs) - 1)]
        t = _padded(vb, vo)
        W = max(t.shape[1], 1)
        extra = np.full((3, W), PAD, dtype=np.uint8)   # rows: '+', '#', absent
        extra[0, 0] = ord("+")
        extra[1, 0] = ord("#")
        tables.append(np.concatenate([t, extra]))
    def one(c0):
        c = codes[c0:c0 + chunk]
        cols = []
        for l in range(D):
            tb = tables[l]
            V = tb.shape[0] - 3
            col = c[:, l]
            idx = np.where(col >= 0, col, np.where(col == PLUS_CODE, V, np.where(col == HASH_CODE, V + 1, V + 2)))
            if l > 0:
                sep = np.where(col != ABSENT, ord("/"), PAD).astype(np.uint8)[:, None]
                cols.append(sep)
            cols.append(tb[idx])
        mat = np.concatenate(cols, axis=1)
        keep = mat != PAD
        return keep.sum(1), mat[keep]

    # chunks are independent (numpy releases the GIL in these kernels): a thread pool, same bytes
    parts = _pmap(one, range(0, N, chunk))
    out_lens = [p[0] for p in parts]
    out_bufs = [p[1] for p in parts]
    lens = np.concatenate(out_lens) if out_lens else np.zeros(0, np.int64)
    offs = np.zeros(N + 1, dtype=np.uint64)
    offs[1:] = np.cumsum(lens)
    buf = np.concatenate(out_bufs) if out_bufs else np.zeros(0, np.uint8)
    if buf.size == 0:
        buf = np.zeros(1, np.uint8)
    return np.ascontiguousarray(buf), offs


def unpack(packed: Tuple[np.ndarray, np.ndarray], idx=None) -> List[bytes]:
    buf, offs = packed
    raw = buf.tobytes()
    n = len(offs) - 1
    it = range(n) if idx is None else idx
    return [raw[int(offs[i]):int(offs[i + 1])] for i in it]


def take(packed: Tuple[np.ndarray, np.ndarray], idx: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Sub-batch of a packed list (vectorized gather)."""
    buf, offs = packed
    idx = np.asarray(idx, dtype=np.int64)
    s = offs[:-1].astype(np.int64)[idx]
    ln = (offs[1:].astype(np.int64) - offs[:-1].astype(np.int64))[idx]
    o = np.zeros(len(idx) + 1, dtype=np.uint64)
    o[1:] = np.cumsum(ln)
    tot = int(o[-1])
    within = np.arange(tot, dtype=np.int64) - np.repeat(np.cumsum(ln) - ln, ln)
    nb = buf[np.repeat(s, ln) + within] if tot else np.zeros(1, np.uint8)
    return np.ascontiguousarray(nb), o


def dedupe_rows(codes: np.ndarray) -> np.ndarray:
    """Unique rows in first-occurrence order.  Rows are keyed by a 64-bit hash: a collision
    can only drop a distinct row, which the generators replace by drawing more rows.  (Hashes
    in row chunks, first occurrences per bucket of the hash's top bits, both on the thread
    pool: the same rows as one np.unique over all hashes.)"""
    n = codes.shape[0]

    def hashes(a):
        c = codes[a:a + (1 << 21)].astype(np.uint64)
        h = np.full(c.shape[0], 0x9E3779B97F4A7C15, dtype=np.uint64)
        with np.errstate(over="ignore"):
            for j in range(c.shape[1]):
                h ^= c[:, j] + np.uint64(0x632BE59BD9B4E019) + (h << np.uint64(6)) + (h >> np.uint64(2))
                h *= np.uint64(0xff51afd7ed558ccd)
                h ^= h >> np.uint64(29)
        return h
    h = np.concatenate(_pmap(hashes, range(0, n, 1 << 21))) if n else np.zeros(0, np.uint64)
    top = (h >> np.uint64(60)).astype(np.uint8)
    keep = np.zeros(n, dtype=bool)

    def bucket(b):
        idx = np.nonzero(top == b)[0]
        _, first = np.unique(h[idx], return_index=True)
        keep[idx[first]] = True
    _pmap(bucket, range(16))
    return codes[keep]


def _threads() -> int:
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    return max(1, min(n, 16))


def _pmap(fn, items):
    """[fn(x) for x in items] on a thread pool (the generators' numpy kernels release the GIL;
    results in order, so the output is the same as the serial loop's)."""
    items = list(items)
    if len(items) <= 1 or _threads() == 1:
        return [fn(x) for x in items]
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(_threads()) as ex:
        return list(ex.map(fn, items))


def zipf_sampler(rng: np.random.Generator, vsize: int, s: float = 1.1):
    p = 1.0 / np.arange(1, vsize + 1, dtype=np.float64) ** s
    cdf = np.cumsum(p)
    cdf /= cdf[-1]

    def draw(n):
        u = rng.random(n)  # one draw from the generator's stream, as before
        step = 1 << 21
        parts = _pmap(lambda a: np.searchsorted(cdf, u[a:a + step]), range(0, n, step))
        idx = np.concatenate(parts) if parts else np.zeros(0, np.int64)
        return np.minimum(idx, vsize - 1).astype(np.int32)
    return draw


def level_vocabs(prefixes: Sequence[bytes], sizes: Sequence[int]):
    return [vocab_table([p + b"%d" % k for k in range(v)]) for p, v in zip(prefixes, sizes)]


# ---------------------------------------------------------------------------------------
# Config A (CPU reference config) and A' (emqx_broker_bench run1 shape)
# ---------------------------------------------------------------------------------------

def config_a(n_filters: int = 100_000, n_topics: int = 1_000_000, seed: int = 1) -> Workload:
    """100k filters site{i mod 1000}/+/dev{i div 1000}/#; topics
    site{U[0,1000)}/gw{U[0,64)}/dev{U[0,128)}/m{U[0,8)} (SURVEY §8 d)."""
    i = np.arange(n_filters)
    vs = [vocab_table([b"site%d" % k for k in range(1000)]), vocab_table([b"gw%d" % k for k in range(64)]),
          vocab_table([b"dev%d" % k for k in range(max(128, n_filters // 1000 + 1))]),
          vocab_table([b"m%d" % k for k in range(8)])]
    fc = np.stack([i % 1000, np.full(n_filters, PLUS_CODE), i // 1000, np.full(n_filters, HASH_CODE)], 1)
    filters = compose(fc, vs)
    rng = np.random.default_rng(seed)
    tc = np.stack([rng.integers(0, 1000, n_topics), rng.integers(0, 64, n_topics),
                   rng.integers(0, 128, n_topics), rng.integers(0, 8, n_topics)], 1)
    topics = compose(tc, vs)
    return Workload("A", filters, topics)


def config_a_prime(subscribers: int = 80, sub_ops: int = 1000, publishers: int = 80) -> Workload:
    """emqx_broker_bench run1 (apps/emqx/src/emqx_broker_bench.erl:25-34,146-162): filters
    device/{id}/+/{num}/#, one topic per publisher device/{id rem subs + 1}/foo/1/bar/1/2/3/4/5."""
    ids = np.repeat(np.arange(1, subscribers + 1), sub_ops)
    nums = np.tile(np.arange(1, sub_ops + 1), subscribers)
    V = max(subscribers, sub_ops) + 2
    num_v = vocab_table([b"%d" % k for k in range(V)])
    vs = [vocab_table([b"device"]), num_v, vocab_table([b"foo"]), num_v, vocab_table([b"bar"])] + [num_v] * 5
    fc = np.stack([np.zeros_like(ids), ids, np.full_like(ids, PLUS_CODE), nums, np.full_like(ids, HASH_CODE)], 1)
    fc = np.concatenate([fc, np.full((len(ids), 5), ABSENT)], 1)
    filters = compose(fc, vs)
    pid = np.arange(1, publishers + 1)
    tc = np.stack([np.zeros_like(pid), pid % subscribers + 1, np.zeros_like(pid), np.ones_like(pid),
                   np.zeros_like(pid)] + [np.full_like(pid, k) for k in (1, 2, 3, 4, 5)], 1)
    topics = compose(tc, vs)
    return Workload("A'", filters, topics)


# ---------------------------------------------------------------------------------------
# Config B (1 x MI355X headline) — also C at larger scale
# ---------------------------------------------------------------------------------------

def _b_filter_codes(rng, n, vocab_sizes, samplers):
    D = len(vocab_sizes)
    # every draw from the generator's stream first, in the original order (the table depends on
    # it); the row-local arithmetic then runs over row chunks on the thread pool
    d = rng.integers(4, D + 1, n)  # U{4..8}
    words = [samplers[l](n) for l in range(D)]
    cls = rng.random(n)
    pm_u = rng.random((n, D))
    force = rng.integers(0, d)  # one level in [0, d)
    t = rng.integers(1, d + 1)
    lvl = np.arange(D)[None, :]
    codes9 = np.full((n, D + 1), ABSENT, dtype=np.int32)

    def rows(a):
        z = slice(a, min(n, a + (1 << 20)))
        dz, cz, tz = d[z], cls[z], t[z]
        codes = np.where(lvl < dz[:, None], np.stack([w[z] for w in words], 1), ABSENT).astype(np.int32)
        plus_cls = (cz >= 0.5) & (cz < 0.8)
        hash_cls = cz >= 0.8
        # '+' class: each level '+' w.p. 0.25, at least one
        pm = (pm_u[z] < 0.25) & (lvl < dz[:, None])
        none = plus_cls & ~pm.any(1)
        pm[np.nonzero(none)[0], force[z][none]] = True
        codes = np.where(plus_cls[:, None] & pm, PLUS_CODE, codes)
        # '#' class: keep t = U{1..d} literal levels, then '#'
        hrows = np.nonzero(hash_cls)[0]
        hc = codes[hrows]
        hc[lvl.repeat(len(hrows), 0) >= tz[hrows, None]] = ABSENT
        codes[hrows] = hc
        out = codes9[z]
        out[:, :D] = codes
        out[hrows, tz[hrows]] = HASH_CODE
    _pmap(rows, range(0, n, 1 << 20))
    return codes9


def config_b(n_filters: int = 10_000_000, n_topics: int = 1_000_000, seed: int = 2,
             vocab_scale: int = 1, prefixes=B_PREFIX, topic_seed=None, extra_topic_seeds=()) -> Workload:
    """10M mixed exact/'+'/'#' filters, depth U{4..8}, Zipf(1.1) per-level vocab
    [64,1024,4096,65536,65536,1024,256,64]; 50% exact / 30% '+' / 20% '#'.  Topics depth
    U{4..8}: 50% instantiated from a random filter ('+' -> random word, '#' -> 0-3 words),
    50% random (SURVEY §8 d).  extra_topic_seeds: more independent topic batches over the same
    table, as `.extra_topics` (the first batch is unchanged by them)."""
    rng = np.random.default_rng(seed)
    sizes = [v * vocab_scale for v in B_VOCAB]
    samplers = [zipf_sampler(rng, v) for v in sizes]
    vs = level_vocabs(prefixes, sizes)
    vs.append(vocab_table([b"x"]))  # level 8 only ever holds '#' or instantiated words
    got = np.zeros((0, 9), dtype=np.int32)
    want = n_filters
    while got.shape[0] < n_filters:
        extra = int((want - got.shape[0]) * 1.15) + 1024
        got = dedupe_rows(np.concatenate([got, _b_filter_codes(rng, extra, sizes, samplers)]))
    fcodes = got[:n_filters]
    filters = compose(fcodes, vs)
    if topic_seed is not None:  # an independent topic stream over the same table
        rng = np.random.default_rng(topic_seed)
        samplers = [zipf_sampler(rng, v) for v in sizes]
    topics, tcodes = _b_topics(rng, samplers, fcodes, vs, n_filters, n_topics, codes=True)
    wl = Workload("B", filters, topics)
    wl.fcodes, wl.tcodes = fcodes, tcodes  # level codes (oracle/pruned.py narrows the oracle's table)
    extra = []
    for ts in extra_topic_seeds:
        r2 = np.random.default_rng(ts)
        extra.append(_b_topics(r2, [zipf_sampler(r2, v) for v in sizes], fcodes, vs, n_filters, n_topics))
    wl.extra_topics = extra
    return wl


def _b_topics(rng, samplers, fcodes, vs, n_filters, n_topics, codes=False):
    """One topic batch of config B over the filter codes `fcodes` (see config_b)."""
    # topics (levels up to 8 + 3 for '#' expansion => pad to 11)
    TD = 11
    half = n_topics // 2
    src = fcodes[rng.integers(0, n_filters, half)]
    tcodes = np.full((n_topics, TD), ABSENT, dtype=np.int32)
    rand_words = np.stack([samplers[min(l, 7)](half) for l in range(TD)], 1)
    inst = np.full((half, TD), ABSENT, dtype=np.int32)
    inst[:, :9] = np.where(src == PLUS_CODE, rand_words[:, :9], src)
    # '#': replace by 0-3 random words at its position
    hpos = np.argmax(src == HASH_CODE, axis=1)
    has_h = (src == HASH_CODE).any(1)
    k = rng.integers(0, 4, half)
    lvl = np.arange(TD)[None, :]
    exp = has_h[:, None] & (lvl >= hpos[:, None]) & (lvl < (hpos + k)[:, None])
    inst = np.where(exp, rand_words, inst)
    inst = np.where(has_h[:, None] & (lvl >= (hpos + k)[:, None]), ABSENT, inst)
    # a '#' with zero expansion at position 0 would leave an empty topic: keep >= 1 level
    empty = inst[:, 0] == ABSENT
    inst[empty, 0] = rand_words[empty, 0]
    tcodes[:half] = inst
    nr = n_topics - half
    d = rng.integers(4, 9, nr)
    rw = np.stack([samplers[min(l, 7)](nr) for l in range(TD)], 1)
    tcodes[half:] = np.where(lvl < d[:, None], rw, ABSENT)
    perm = rng.permutation(n_topics)
    tcodes = tcodes[perm]
    # levels >= 8 use level-7 vocab words (instantiated '#' expansions)
    tv = vs[:8] + [vs[7]] * 3
    packed = compose(tcodes, tv)
    return (packed, tcodes) if codes else packed


# ---------------------------------------------------------------------------------------
# Config D (adversarial)
# ---------------------------------------------------------------------------------------

def config_d(n_filters: int = 1_000_000, n_topics: int = 100_000, seed: int = 4, depth: int = 16,
             vocab: int = 4) -> Workload:
    """Depth-16 templates over 4 words/level, each level '+' w.p. 0.5, 30% '#'-terminated,
    plus '#', '+/#', '+/+/#'; topics exactly 16 levels from the same vocab."""
    rng = np.random.default_rng(seed)
    got = np.zeros((0, depth + 1), dtype=np.int32)
    while got.shape[0] < n_filters:
        n = int((n_filters - got.shape[0]) * 1.1) + 64
        c = rng.integers(0, vocab, (n, depth)).astype(np.int32)
        c = np.where(rng.random((n, depth)) < 0.5, PLUS_CODE, c)
        c17 = np.full((n, depth + 1), ABSENT, dtype=np.int32)
        c17[:, :depth] = c
        hrows = np.nonzero(rng.random(n) < 0.3)[0]
        t = rng.integers(1, depth + 1, len(hrows))
        lvl = np.arange(depth + 1)[None, :]
        sub = c17[hrows]
        sub = np.where(lvl >= t[:, None], ABSENT, sub)
        sub[np.arange(len(hrows)), t] = HASH_CODE
        c17[hrows] = sub
        got = dedupe_rows(np.concatenate([got, c17]))
    special = np.full((3, depth + 1), ABSENT, dtype=np.int32)
    special[0, 0] = HASH_CODE
    special[1, :2] = [PLUS_CODE, HASH_CODE]
    special[2, :3] = [PLUS_CODE, PLUS_CODE, HASH_CODE]
    fcodes = dedupe_rows(np.concatenate([special, got]))[:n_filters]
    vs = [vocab_table([b"l%dw%d" % (l, k) for k in range(vocab)]) for l in range(depth + 1)]
    filters = compose(fcodes, vs)
    tcodes = rng.integers(0, vocab, (n_topics, depth)).astype(np.int32)
    topics = compose(tcodes, vs[:depth])
    return Workload("D", filters, topics)


# ---------------------------------------------------------------------------------------
# Config E (publish fan-out)
# ---------------------------------------------------------------------------------------

NO_GROUP = 0xFFFFFFFF


@dataclass
class FanoutWorkload:
    wl: Workload              # route table (filters) + topic stream
    sub_filter: np.ndarray    # uint32 filter id per subscription
    sub_id: np.ndarray        # uint32 subscriber id
    sub_group: np.ndarray     # uint32 $share group id, NO_GROUP for plain subscriptions
    keys: np.ndarray          # uint32 per-topic pick key (stands in for erlang:phash2, < 2^27)

    @property
    def n_subscriptions(self) -> int:
        return len(self.sub_id)


def config_e(n_filters: int = 2_000_000, n_subscribers: int = 1_000_000, per_sub: int = 10,
             shared_frac: float = 0.1, n_topics: int = 1_000_000, seed: int = 5, groups: int = 8,
             min_group: int = 2, max_group: int = 16) -> FanoutWorkload:
    """SURVEY §8 d config E: n_subscribers x per_sub subscriptions over config B's generator
    table of n_filters; shared_frac of them in $share groups g0..g7 of U{2..16} members
    (one group instance = (filter, group, members)), the rest plain (deduplicated
    (filter, subscriber) pairs); topics from config B's topic generator."""
    wl = config_b(n_filters=n_filters, n_topics=n_topics, seed=seed)
    rng = np.random.default_rng(seed + 1000)
    total = n_subscribers * per_sub
    n_shared = int(total * shared_frac)
    # plain
    n_plain = total - n_shared
    ps = (np.arange(n_plain, dtype=np.uint64) % np.uint64(n_subscribers))
    pf = rng.integers(0, n_filters, n_plain).astype(np.uint64)
    key = np.unique((pf << np.uint64(32)) | ps)
    pf, ps = (key >> np.uint64(32)).astype(np.uint32), (key & np.uint64(0xFFFFFFFF)).astype(np.uint32)
    # shared group instances until n_shared memberships
    sizes = []
    acc = 0
    while acc < n_shared:
        k = int(rng.integers(min_group, max_group + 1))
        sizes.append(k)
        acc += k
    sizes = np.array(sizes, dtype=np.int64)
    ng = len(sizes)
    gf = rng.integers(0, n_filters, ng).astype(np.uint64)
    gg = rng.integers(0, groups, ng).astype(np.uint64)
    gkey, first = np.unique((gf << np.uint64(3)) | gg, return_index=True)  # one instance per (filter, group)
    sizes, gf, gg = sizes[first], gf[first], gg[first]
    sf = np.repeat(gf, sizes).astype(np.uint32)
    sg = np.repeat(gg, sizes).astype(np.uint32)
    ss = rng.integers(0, n_subscribers, int(sizes.sum())).astype(np.uint32)
    # members of one instance are distinct subscribers (duplicates dropped, order kept)
    mk = (sf.astype(np.uint64) << np.uint64(35)) | (sg.astype(np.uint64) << np.uint64(32)) | ss.astype(np.uint64)
    _, keep = np.unique(mk, return_index=True)
    keep.sort()
    sf, sg, ss = sf[keep], sg[keep], ss[keep]
    keys = rng.integers(0, 1 << 27, n_topics).astype(np.uint32)
    return FanoutWorkload(wl, np.concatenate([pf, sf]), np.concatenate([ps, ss]),
                          np.concatenate([np.full(len(pf), NO_GROUP, np.uint32), sg]), keys)


def config_by_name(name: str, **kw) -> Workload:
    return {"A": config_a, "A'": config_a_prime, "B": config_b, "D": config_d}[name](**kw)
