// Retained-message index kernels (retain.h): a batch of subscription filters against the
// trie of stored retained topics (reference: the match-spec select of
// apps/emqx_retainer/src/emqx_retainer_mnesia.erl:212-258 and read_messages/1 :199-208).
//
//   walk    one wavefront per tile of up to 64 filters (persistent waves).  Each lane tokenizes and
//           interns its own filter (filters are short; subscription-path work), then the wave
//           walks all 64 filters' frontiers from one shared work stack of RANGE items
//           {first node, node count, level, filter}: a '+' level pushes its node's whole child
//           range as one item, and every step hands the next 64 nodes of the stack's top items
//           to the 64 lanes, so a wide '+' fan-out keeps every lane busy.  A final '#' emits the
//           node's subtree as one rank range; a filter that ends on a stored topic emits its rank.
//           Load balance (retain.cpp "balance"): the work-sharing walk (retain_walk_queue_kernel,
//           the default) shares the bottom of busy waves' stacks as pieces through sharded ticket
//           queues while waves wait; the spill rounds (retain_walk_kernel + _spill_kernel) move
//           whatever is left after a step budget into rebalanced rounds.
//   count   live (unexpired) ranks per range; per-filter totals (one atomic per run of a
//           filter's records in a 64-record super-row)
//   write   rank -> topic id for the live ranks of each range, at the filter's CSR offset plus
//           a per-filter cursor: coalesced streaming reads of rank_id / rank_exp.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "kernels.h"
#include "retain.h"

namespace emqx {

namespace {

__device__ __forceinline__ uint32_t rintern(const RetainView& rv, uint32_t h, uint32_t len, uint32_t w0, uint32_t w1,
                                            uint32_t w2, uint32_t w3, const uint8_t* bytes, uint64_t ws) {
  uint32_t i = vocab_slot0(h) & rv.vocab_mask;
  for (uint32_t k = 0; k <= rv.vocab_mask; ++k) {
    const uint4* vp = reinterpret_cast<const uint4*>(rv.vocab + i);
    const uint4 hd = vp[0];  // hash, len, wid, off
    if (hd.z == WID_NONE) return WID_NONE;
    if (hd.x == h && hd.y == len) {
      const uint4 in = vp[1];
      bool eq = in.x == w0 && in.y == w1 && in.z == w2 && in.w == w3;
      for (uint32_t b = 16; b < len && eq; ++b) eq = rv.arena[hd.w + b] == bytes[ws + b];
      if (eq) return hd.z;
    }
    i = (i + 1) & rv.vocab_mask;
  }
  return WID_NONE;
}

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// exclusive prefix of `v` over the wave; *tot = the wave's sum
__device__ __forceinline__ uint32_t wave_excl(uint32_t v, uint32_t* tot) {
  uint32_t x = v;
  const uint32_t lane = lane_id();
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= static_cast<uint32_t>(d)) x += y;
  }
  *tot = __shfl(x, 63, 64);
  return x - v;
}

__device__ __forceinline__ bool rank_live(const RetainView& rv, uint32_t rank, int64_t now, uint32_t flags) {
  const int64_t e = rv.rank_exp[rank];
  return e == 0 || ((flags & RRANGE_STRICT) ? e > now : e >= now);
}

__device__ __forceinline__ bool rank_ok(const RetainView& rv, uint32_t rank, bool guard, int64_t now, uint32_t flags) {
  const uint32_t mind = flags >> RRANGE_MIND_SHIFT;
  return (!guard || rank_live(rv, rank, now, flags)) && (mind == 0 || rv.rank_depth[rank] >= mind);
}

__device__ __forceinline__ uint32_t rank_at(const RetainView& rv, uint32_t i, uint32_t flags) {
  return (flags & RRANGE_INDIRECT) ? rv.dterm[i] : i;
}

// Both lower bounds of x1 <= x2 in [l, h) at once: two independent load chains in flight
// instead of one after the other (the walk is latency-bound).  Same results as two calls.
__device__ __forceinline__ void lower_bound2_u32(const uint32_t* a, uint32_t stride, uint32_t l, uint32_t h,
                                                 uint32_t x1, uint32_t x2, uint32_t* r1, uint32_t* r2) {
  uint32_t l1 = l, h1 = h, l2 = l, h2 = h;
  while (l1 < h1 || l2 < h2) {
    const uint32_t m1 = l1 < h1 ? (l1 + h1) >> 1 : l;  // in [l, h) either way
    const uint32_t m2 = l2 < h2 ? (l2 + h2) >> 1 : l;
    const uint32_t v1 = a[static_cast<uint64_t>(m1) * stride], v2 = a[static_cast<uint64_t>(m2) * stride];
    if (l1 < h1) {
      if (v1 < x1) l1 = m1 + 1; else h1 = m1;
    }
    if (l2 < h2) {
      if (v2 < x2) l2 = m2 + 1; else h2 = m2;
    }
  }
  *r1 = l1;
  *r2 = l2;
}

// Two-level form of lower_bound2_u32 over keys a[i * stride], i in [L, H) (global indices of
// one sorted slice), with fence[b] = a[b * RFENCE * stride]: the fences whose block starts
// inside the slice are searched first (a small, L2-resident array), then each bound is found
// inside one block of RFENCE entries.  Same results as lower_bound2_u32(a, stride, L, H, ...).
__device__ __forceinline__ void fenced_lower_bound2(const uint32_t* a, uint32_t stride, const uint32_t* fence,
                                                    uint32_t L, uint32_t H, uint32_t x1, uint32_t x2, uint32_t* r1,
                                                    uint32_t* r2) {
  const uint32_t B0 = (L + RFENCE - 1) / RFENCE, B1 = (H + RFENCE - 1) / RFENCE;  // blocks starting in [L, H)
  uint32_t f1 = B0, f2 = B0;
  if (B1 > B0) lower_bound2_u32(fence, 1, B0, B1, x1, x2, &f1, &f2);
  // the bound lies after block f-1's first key (< x) and at or before block f's first key
  const uint32_t l1 = f1 > B0 ? (f1 - 1) * RFENCE + 1 : L, h1 = f1 < B1 ? f1 * RFENCE : H;
  const uint32_t l2 = f2 > B0 ? (f2 - 1) * RFENCE + 1 : L, h2 = f2 < B1 ? f2 * RFENCE : H;
  // interleaved final searches, each within one block
  uint32_t a1 = l1, b1 = h1, a2 = l2, b2 = h2;
  while (a1 < b1 || a2 < b2) {
    const uint32_t m1 = a1 < b1 ? (a1 + b1) >> 1 : L;
    const uint32_t m2 = a2 < b2 ? (a2 + b2) >> 1 : L;
    const uint32_t v1 = a[static_cast<uint64_t>(m1) * stride], v2 = a[static_cast<uint64_t>(m2) * stride];
    if (a1 < b1) {
      if (v1 < x1) a1 = m1 + 1; else b1 = m1;
    }
    if (a2 < b2) {
      if (v2 < x2) a2 = m2 + 1; else b2 = m2;
    }
  }
  *r1 = a1;
  *r2 = a2;
}

// ceil(x / 2^sh)
__device__ __forceinline__ uint32_t ceil_shr(uint32_t x, uint32_t sh) {
  return static_cast<uint32_t>((static_cast<uint64_t>(x) + (1ull << sh) - 1) >> sh);
}

// max(16 * blk, L) + #{j in block blk (16 keys, one 64-B line) and in [L, H) : a[j] < x}
__device__ __forceinline__ uint32_t scan_block(const uint32_t* a, uint32_t blk, uint32_t L, uint32_t H, uint32_t x) {
  const uint32_t b = blk * RST_FAN;
  const uint4* p = reinterpret_cast<const uint4*>(a + b);
  uint32_t lt = 0;  // bit i: key b + i < x
#pragma unroll
  for (uint32_t i = 0; i < RST_FAN / 4; ++i) {
    const uint4 v = p[i];
    lt |= ((v.x < x ? 1u : 0u) | (v.y < x ? 2u : 0u) | (v.z < x ? 4u : 0u) | (v.w < x ? 8u : 0u)) << (4 * i);
  }
  // keys of the block inside [L, H): one contiguous run of bits
  const uint32_t lo = L > b ? L - b : 0u, hi = H > b ? min(H - b, RST_FAN) : 0u;
  const uint32_t in = hi > lo ? ((1u << hi) - 1u) & ~((1u << lo) - 1u) : 0u;
  const uint32_t c = __popc(lt & in);
  return (b > L ? b : L) + c;
}

// Both lower bounds of x1 <= x2 in the slice [L, H) of t's level 0 (RSTree): from the lowest
// level at which the slice lies in one 16-key block, one block scan per level.  The bound P at
// level k+1 brackets level k's: key (P-1)*16 (if inside the slice) is < x, key P*16 (if inside)
// >= x, so level k's bound lies in block P-1 (or, P at the slice's start, the slice's first).
__device__ __forceinline__ void stree_lower_bound2(const RSTree& t, uint32_t L, uint32_t H, uint32_t x1, uint32_t x2,
                                                   uint32_t* r1, uint32_t* r2) {
  uint32_t k = 0, Lk = L, Hk = H, off = 0;  // off: level k's first word
  while (k + 1 < t.levels && Hk > Lk && (Lk >> RST_SH) != ((Hk - 1) >> RST_SH)) {
    off += rst_level_words(ceil_shr(t.n, RST_SH * k));
    ++k;
    Lk = ceil_shr(L, RST_SH * k);
    Hk = ceil_shr(H, RST_SH * k);
  }
  uint32_t b1 = Lk >> RST_SH, b2 = b1;
  for (;;) {
    const uint32_t* a = t.keys + off;
    const uint32_t p1 = scan_block(a, b1, Lk, Hk, x1), p2 = scan_block(a, b2, Lk, Hk, x2);
    if (k == 0) {
      *r1 = p1;
      *r2 = p2;
      return;
    }
    --k;
    off -= rst_level_words(ceil_shr(t.n, RST_SH * k));
    const uint32_t Ln = ceil_shr(L, RST_SH * k), Hn = ceil_shr(H, RST_SH * k);
    b1 = p1 > Lk ? p1 - 1 : (Ln >> RST_SH);
    b2 = p2 > Lk ? p2 - 1 : (Ln >> RST_SH);
    Lk = Ln;
    Hk = Hn;
  }
}

// RETAIN_PROF builds (make retain-prof, experiments only): per-phase wave cycles of the
// walk, summed into RetainArgs.prof[RPROF_SLOTS]: take (stack read + item split), node (its
// fields + filter words), probe (edge / postings-key probes), search, emit+push; then steps,
// active lanes, searching lanes.  Each mark waits for the wave's outstanding memory first.
constexpr uint32_t RPROF_SLOTS = 20;  // 8..15: queue mode (retain_walk_queue_kernel); 16..18: search groups
#ifdef RETAIN_PROF
#define RPROF_MARK(slot)                                   \
  do {                                                     \
    __builtin_amdgcn_s_waitcnt(0);                         \
    const uint64_t _t = clock64();                         \
    pacc[slot] += _t - tprev;                              \
    tprev = _t;                                            \
  } while (0)
#define RPROF_ADD(slot, v) (pacc[slot] += (v))
#define RPROF_NOW() clock64()
#else
#define RPROF_MARK(slot) do {} while (0)
#define RPROF_ADD(slot, v) do {} while (0)
#define RPROF_NOW() 0ull
#endif

#ifndef RW_WAVES_V
#define RW_WAVES_V 1  // waves per block of the walk kernels: their waves share nothing, so one-wave blocks
                      // (round 5: R call 1.045-1.054 against 1.051-1.059 ms for 4, profiles/r5_rw1_ab/)
#endif
constexpr int RW_WAVES = RW_WAVES_V;
#ifndef RW_OCC
#define RW_OCC 1  // waves per SIMD the walk kernels are compiled for (1: the compiler's choice)
#endif
// The walk's work stack: the top RSTK items of each wave in LDS (a step's reads and pushes stay
// on chip); on overflow the bottom half moves to the wave's global area (a.stack) and comes
// back when the LDS part runs empty.  192 items (3 KiB per wave) keeps 32 waves per CU.
constexpr uint32_t RSTK = 192;
constexpr uint32_t RSTK_HALF = 96;
constexpr uint32_t RWORDS = 128;  // LDS word ids per wave tile (first round)
// A wave's reservation of range records (emissions): [next, next + left) of a.ranges.
constexpr uint32_t RRES = 32;
struct RangeRes {
  uint32_t next = 0, left = 0, emitted = 0;
};
enum : uint32_t { SK_NONE = 0, SK_DTERM = 1, SK_POSTS = 2 };
constexpr uint32_t RBIG = 64;     // ranks of a small range record at most
constexpr uint32_t RCHUNK = 256;  // ranks per big range record (one unrolled wave pass)

// Reserve n slots of the spill buffer, all or nothing (a partial reservation would leave
// unwritten items inside the counted prefix).  Called by one lane.
__device__ __forceinline__ bool spill_reserve(uint32_t* ctr32, uint32_t n, uint32_t cap, uint32_t* base) {
  // one fetch-add, not a compare-and-swap loop: waves of a round reach their budget together,
  // and 4096 of them retrying one CAS serialised a round for ~20 ms (budget 32).  A reservation
  // past `cap` fails; its part below `cap` is padded with empty items by the caller.  The
  // counter is 64-bit (two ctrl words, zeroed per call), so the failed reservations' overshoot
  // cannot wrap it back under `cap` (a load before the add, tried in round 4, cost ~0.2 ms per
  // call: 8K waves reading one word together)
  unsigned long long* ctr = reinterpret_cast<unsigned long long*>(ctr32);
  const unsigned long long old = atomicAdd(ctr, static_cast<unsigned long long>(n));
  *base = static_cast<uint32_t>(min(old, static_cast<unsigned long long>(cap)));
  return old <= cap && n <= cap - old;
}

// The walk of one wave's stack until it is empty or the step budget runs out; then the
// remaining items go to a.spill_out (global filter ids) for the next, rebalanced round.
// TILE: items name a filter lane of the tile whose first filter is `fbase` (its level count
// and word base in LDS);
// else items name a global filter id and the lane reads both from global memory.
// SEARCH: how the postings / rank-list slices are found (RetainArgs.search): RSEARCH_FENCED
// two-level binary searches, RSEARCH_STREE the 16-ary search tree
// A filter word: from the tile's LDS copy (lwords, first round, when the tile's words fit) or
// from the per-call word array in global memory.
__device__ __forceinline__ uint32_t word_at(const RetainArgs& a, const uint32_t* lwords, uint64_t i) {
  return lwords ? lwords[i] : a.wids[i];
}

// The loads of one walk step — the node's fields (posts[name]), its edge bucket (three 16-B
// parts), the postings key after a '+' run — each on the lanes that need it, issued back to
// back under one wait, as one asm block: left to the compiler, a lane's node-field load sat in
// its own branch with its own wait before the others were issued (two dependent round trips
// per '+' step).  Masked-off lanes keep the defaults.  Vector loads and exec writes only.
typedef uint32_t ru32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void step_loads(const uint4* pa, const uint4* pb, const RPostKey* pc, bool na, bool nb,
                                           bool nc, uint4& a, uint4& b0, uint4& b1, uint4& b2, RPostKey& c) {
  const uint64_t ma = __ballot(na), mb = __ballot(nb), mc = __ballot(nc);
  ru32x4 va = {0u, 0u, 0u, 0u}, vb0 = {b0.x, b0.y, b0.z, b0.w}, vb1 = {b1.x, b1.y, b1.z, b1.w},
         vb2 = {b2.x, b2.y, b2.z, b2.w}, vc = {c.depth, c.wid, c.off, c.len};
  uint64_t save;
  asm volatile(
      "s_mov_b64 %[sv], exec\n\t"
      "s_and_b64 exec, %[sv], %[ma]\n\t"
      "global_load_dwordx4 %[a], %[pa], off\n\t"
      "s_and_b64 exec, %[sv], %[mb]\n\t"
      "global_load_dwordx4 %[b0], %[pb], off\n\t"
      "global_load_dwordx4 %[b1], %[pb], off offset:16\n\t"
      "global_load_dwordx4 %[b2], %[pb], off offset:32\n\t"
      "s_and_b64 exec, %[sv], %[mc]\n\t"
      "global_load_dwordx4 %[c], %[pc], off\n\t"
      "s_mov_b64 exec, %[sv]\n\t"
      "s_waitcnt vmcnt(0)"
      : [a] "+v"(va), [b0] "+v"(vb0), [b1] "+v"(vb1), [b2] "+v"(vb2), [c] "+v"(vc), [sv] "=&s"(save)
      : [pa] "v"(pa), [pb] "v"(pb), [pc] "v"(pc), [ma] "s"(ma), [mb] "s"(mb), [mc] "s"(mc)
      : "memory");
  a = make_uint4(va.x, va.y, va.z, va.w);
  b0 = make_uint4(vb0.x, vb0.y, vb0.z, vb0.w);
  b1 = make_uint4(vb1.x, vb1.y, vb1.z, vb1.w);
  b2 = make_uint4(vb2.x, vb2.y, vb2.z, vb2.w);
  c = RPostKey{vc.x, vc.y, vc.z, vc.w};
}

// A step descriptor stored / loaded at agent scope (two 8-B halves): queue mode's tiles write
// them and other waves of the same launch, on any XCD, read them.
__device__ __forceinline__ void desc_store_sc(uint4* p, uint4 d) {
  uint64_t* q = reinterpret_cast<uint64_t*>(p);
  __hip_atomic_store(q, static_cast<uint64_t>(d.x) | (static_cast<uint64_t>(d.y) << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(q + 1, static_cast<uint64_t>(d.z) | (static_cast<uint64_t>(d.w) << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint4 desc_load_sc(const uint4* p) {
  const uint64_t* q = reinterpret_cast<const uint64_t*>(p);
  const uint64_t a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint64_t b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return make_uint4(static_cast<uint32_t>(a), static_cast<uint32_t>(a >> 32), static_cast<uint32_t>(b),
                    static_cast<uint32_t>(b >> 32));
}

// Tokenize filter f and intern its words (one lane): word ids to a.wids (at foffs[f] - foffs[0]
// + f) and the step descriptors of the untiled walks to a.wdesc; returns nlev | wildcard << 31.
// DESC: the step descriptors are stored (the spill rounds read them) or not (queue mode
// publishes a filter's descriptors when it first shares one of its pieces: publish_desc).
template <bool DESC>
__device__ __forceinline__ uint32_t tokenize_filter(const RetainArgs& a, uint64_t f) {
  const RetainView& rv = a.rv;
  const uint64_t b0 = a.foffs[0];
  uint32_t nlev = 0, wild = 0;
  const uint64_t start = a.foffs[f], end = a.foffs[f + 1];
  uint32_t* wout = a.wids + (start - b0) + f;
  uint32_t len = 0, w0 = 0, w1 = 0, w2 = 0, w3 = 0;
  uint64_t ws = start;
  for (uint64_t i = start; i <= end; ++i) {
    const uint32_t c = (i < end) ? a.fbytes[i] : static_cast<uint32_t>('/');
    if (c != '/') {
      if (len < 16) {
        const uint32_t v = c << (8u * (len & 3u));
        const uint32_t q = len >> 2;
        w0 |= q == 0 ? v : 0u;
        w1 |= q == 1 ? v : 0u;
        w2 |= q == 2 ? v : 0u;
        w3 |= q == 3 ? v : 0u;
      }
      ++len;
    } else {
      uint32_t wid;
      if (len == 1 && w0 == '+') {
        wid = WID_PLUS;
        wild = 1;
      } else if (len == 1 && w0 == '#') {
        wid = i == end ? WID_HASH : WID_NONE;  // a non-final '#' is a token no topic has
        wild = 1;
      } else {
        const uint32_t h = len <= 16 ? word_hash16(len, w0, w1, w2, w3) : word_hash_bytes(a.fbytes + ws, len);
        wid = rv.n_nodes ? rintern(rv, h, len, w0, w1, w2, w3, a.fbytes, ws) : WID_NONE;
      }
      wout[nlev++] = wid;
      len = 0;
      w0 = w1 = w2 = w3 = 0;
      ws = i + 1;
    }
  }
  const uint32_t nw = nlev | (wild << 31);
  if (DESC) {  // the step descriptors of the untiled walks (RetainArgs.wdesc), last level first
    uint4* dout = a.wdesc + (start - b0) + 2 * f;
    dout[nlev] = make_uint4(WID_NONE, 0u, WID_HASH, nw);
    uint32_t jn = nlev, wn = WID_HASH;  // the first non-'+' level above l, its word
    for (uint32_t l = nlev; l-- > 0;) {
      const uint32_t wl = wout[l];
      dout[l] = make_uint4(wl, jn, wn, nw);
      if (wl != WID_PLUS) {
        jn = l;
        wn = wl;
      }
    }
  }
  return nw;
}

// Queue mode: filter f's step descriptors (as tokenize_filter's), stored at agent scope from its
// word ids (written by this wave): other waves of the launch, on any XCD, read them.
__device__ __forceinline__ void publish_desc(const RetainArgs& a, uint64_t f, uint32_t nw) {
  const uint64_t b0 = a.foffs[0], start = a.foffs[f];
  const uint32_t nlev = nw & 0x7FFFFFFFu;
  const uint32_t* wids = a.wids + (start - b0) + f;
  uint4* dout = a.wdesc + (start - b0) + 2 * f;
  desc_store_sc(dout + nlev, make_uint4(WID_NONE, 0u, WID_HASH, nw));
  uint32_t jn = nlev, wn = WID_HASH;
  for (uint32_t l = nlev; l-- > 0;) {
    const uint32_t wl = wids[l];
    desc_store_sc(dout + l, make_uint4(wl, jn, wn, nw));
    if (wl != WID_PLUS) {
      jn = l;
      wn = wl;
    }
  }
}

// ---- work sharing (queue mode) --------------------------------------------------------------
// A shared piece is one queue slot, written as two 8-B stores at agent scope in either order:
// {x, y} with y = node count >= 1 and {z | QREADY, w} with w = global filter id.  A waiting
// wave takes the slot of its ticket once both halves read as written.  The queue is all zero
// when a call starts (the host clears the slots below the previous call's ticket count).
constexpr uint32_t QREADY = 1u << 30;  // in z, above any level
constexpr uint32_t QEND = 0xFFFFFFFFu;  // y of the end marker: the walk is over
constexpr uint32_t QNLEV_SHIFT = 16;  // a queued piece's z: level | nlev << 16 | QREADY | RITEM_POST
constexpr uint32_t QDESC = 12;  // step descriptors of a piece's filter kept in LDS (levels 0..11; 7 blocks per CU)

// The queue is sharded: wave w works in shard w % qshards, with its own tiles (t = s + S*j), its
// own slots and its own control words (QS_*) on a line of their own, QS_STRIDE words from the
// next shard's (distinct memory channels): every ticket, reservation and retire is an atomic on
// one address, and one address serves ~40 M of them per second, so a single queue's counters
// became the walk's bottleneck (and slowed every load that shared their channel).
struct QShard {
  uint32_t* c;       // control words
  uint4* q;          // slots
  uint32_t cap;      // slots
  uint32_t ntiles;   // tiles of this shard
  uint32_t s;
};
__device__ __forceinline__ QShard qshard_at(const RetainArgs& a, uint32_t s) {
  const uint32_t S = a.qshards, cap = a.queue_cap / S;
  return QShard{a.qctl + static_cast<uint64_t>(s) * QS_STRIDE, a.queue + static_cast<uint64_t>(s) * cap, cap,
                a.ntiles > s ? (a.ntiles - s + S - 1) / S : 0u, s};
}
__device__ __forceinline__ QShard qshard(const RetainArgs& a, uint32_t gw) { return qshard_at(a, gw % a.qshards); }

__device__ __forceinline__ void queue_put(uint4* q, uint4 it) {
  uint64_t* p = reinterpret_cast<uint64_t*>(q);
  __hip_atomic_store(p + 1, static_cast<uint64_t>(it.z | QREADY) | (static_cast<uint64_t>(it.w) << 32),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(p, static_cast<uint64_t>(it.x) | (static_cast<uint64_t>(it.y) << 32), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// slot q if both halves are written (*it = the piece), else false; the second half is read only
// once the first is (one load per poll)
__device__ __forceinline__ bool queue_get(uint4* q, uint4* it) {
  uint64_t* p = reinterpret_cast<uint64_t*>(q);
  const uint64_t a = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if ((a >> 32) == 0) return false;
  const uint64_t b = __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!(static_cast<uint32_t>(b) & QREADY)) return false;
  *it = make_uint4(static_cast<uint32_t>(a), static_cast<uint32_t>(a >> 32), static_cast<uint32_t>(b) & ~QREADY,
                   static_cast<uint32_t>(b >> 32));
  return true;
}

// Share the bottom of this wave's stack with the waiting waves: the whole global part if there is
// one, else the bottom half of the LDS part, else (one item) all but its first qpiece nodes; as
// pieces of at most qpiece nodes.  The pending count is raised (and the raise performed) before
// any piece can be seen, so the walk cannot look finished while a piece is queued.  A full queue:
// nothing is shared (the wave keeps walking its stack).
// TILE: items name lanes of the tile at fbase; a filter's descriptors are published with its first
// shared piece (pub: the tile's lanes already published).  Else the wave walks one piece's filter,
// of `pnw` (nlev | wildcard flag), whose descriptors are out already.
template <bool TILE>
__device__ __forceinline__ void share_work(const RetainArgs& a, const QShard& qs, uint4* ls, uint32_t& top, uint4* stk,
                                           uint32_t& gtop, uint64_t fbase, uint32_t& npieces, const uint32_t* nlevs,
                                           uint64_t* pub, uint32_t pnw) {
  const uint32_t lane = lane_id();
  const uint32_t QP = a.qpiece;
  uint32_t kind, nd;  // 0: stk[0, nd)  1: ls[0, nd)  2: ls[0] beyond its first QP nodes
  if (gtop > 0) {
    kind = 0;
    nd = gtop;
  } else if (top >= 2) {
    kind = 1;
    nd = top / 2;
  } else if (top == 1 && ls[0].y > 2 * QP) {
    kind = 2;
    nd = 1;
  } else {
    return;
  }
  auto item = [&](uint32_t i) -> uint4 {
    if (kind == 0) return stk[i];
    uint4 it = ls[i];
    if (kind == 2) {
      it.x += QP;
      it.y -= QP;
    }
    return it;
  };
  uint32_t ptot = 0;
  for (uint32_t i0 = 0; i0 < nd; i0 += 64) {
    const uint32_t i = i0 + lane;
    const uint32_t np = i < nd ? (item(i).y + QP - 1) / QP : 0u;
    uint32_t t;
    (void)wave_excl(np, &t);
    ptot += t;
  }
  if (TILE && !*pub) {
    // the tile's first share publishes every filter's descriptors, a lane each (before the
    // pieces: the waitcnt below covers these stores too)
    if (nlevs[lane] != 0xFFFFFFFFu) publish_desc(a, fbase + lane, nlevs[lane]);
    *pub = 1;
  }
  uint32_t base = 0, ok = 0;
  if (lane == 0) {
    base = atomicAdd(&qs.c[QS_TAIL], ptot);
    ok = base <= qs.cap && ptot <= qs.cap - base ? 1u : 0u;
    if (!ok) atomicMax(&qs.c[QS_FAIL], ~base);  // slots from `base` on are never written
    if (ok) {
      atomicAdd(&qs.c[QS_PEND], ptot);
      __builtin_amdgcn_s_waitcnt(0);  // the raise is performed before a piece is written
    }
  }
  ok = __shfl(ok, 0, 64);
  base = __shfl(base, 0, 64);
  if (!ok) return;
  npieces += ptot;
  for (uint32_t i0 = 0; i0 < nd; i0 += 64) {
    const uint32_t i = i0 + lane;
    uint4 it = make_uint4(0, 0, 0, 0);
    if (i < nd) it = item(i);
    const uint32_t np = i < nd ? (it.y + QP - 1) / QP : 0u;
    uint32_t ctot;
    const uint32_t off = wave_excl(np, &ctot);
    const uint32_t nlev = (TILE ? nlevs[it.w & 63] : pnw) & 0x7FFFFFFFu;
    if (TILE) it.w += static_cast<uint32_t>(fbase);
    it.z |= min(nlev, (QREADY >> QNLEV_SHIFT) - 1u) << QNLEV_SHIFT;
    for (uint32_t k = 0; k < np; ++k) {
      uint4 pc = it;
      pc.x = it.x + QP * k;
      pc.y = min(QP, it.y - QP * k);
      queue_put(qs.q + base + off + k, pc);
    }
    base += ctot;
  }
  __builtin_amdgcn_wave_barrier();
  if (kind == 0) {
    gtop = 0;
  } else if (kind == 1) {
    for (uint32_t i0 = 0; i0 < top - nd; i0 += 64) {  // shift down (reads stay ahead of writes)
      const uint32_t i = i0 + lane;
      uint4 x = make_uint4(0, 0, 0, 0);
      if (i < top - nd) x = ls[nd + i];
      __builtin_amdgcn_wave_barrier();
      if (i < top - nd) ls[i] = x;
    }
    top -= nd;
  } else if (lane == 0) {
    ls[0].y = QP;
  }
  __builtin_amdgcn_wave_barrier();
}

template <bool TILE, int SEARCH, bool QUEUE>
__device__ __forceinline__ void walk_stack(const RetainArgs& a, uint4* ls, uint32_t top, uint4* stk, uint32_t gtop,
                                           uint64_t fbase, const uint32_t* nlevs, const uint64_t* wbase,
                                           const uint32_t* lwords,
                                           uint32_t* pref, uint4* itm, uint32_t& visits, bool& overflow,
                                           RangeRes& res, uint64_t* pacc, const QShard* qs = nullptr,
                                           uint32_t* qstat = nullptr, const uint4* ldesc = nullptr,
                                           uint32_t ldn = 0, uint64_t* pub = nullptr, uint32_t pnw = 0) {
  const uint32_t lane = lane_id();
  const RetainView& rv = a.rv;
  const uint64_t b0 = a.foffs[0];
  uint32_t steps = 0;
#ifdef RETAIN_PROF
  uint64_t tprev = clock64();
#endif
  while (top + gtop > 0) {
    RPROF_MARK(4);
    // queue mode: every qcheck steps lane 0 reads the waiting count (tickets - reserved slots);
    // the load overlaps the step, its answer is used after the pushes
    uint64_t ht = 0;
    const bool look = QUEUE && (++steps & (a.qcheck - 1)) == 0;
    if (look && lane == 0)
      ht = __hip_atomic_load(reinterpret_cast<const uint64_t*>(qs->c + QS_HEAD), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
    if (!QUEUE && steps++ == a.step_budget) {
      // the rest goes out: items wider than 64 nodes as 64-node pieces, so the next round can
      // deal one wide '+' slice over many waves (global part first, then the LDS part)
      const uint32_t all = gtop + top;
      uint32_t pieces = 0;
      for (uint32_t i = lane; i < all; i += 64) pieces += ((i < gtop ? stk[i].y : ls[i - gtop].y) + 63) >> 6;
      uint32_t ptot;
      (void)wave_excl(pieces, &ptot);
      uint32_t base = 0, ok = 0;
      if (lane == 0) {
        ok = spill_reserve(&a.ctrl[a.spill_word], ptot, a.spill_cap, &base) ? 1u : 0u;
        atomicMax(&a.ctrl[RC_SPILLMAX], ptot);
        if (!ok) atomicAdd(&a.ctrl[RC_SPILLFAIL], 1u);
      }
      ok = __shfl(ok, 0, 64);
      base = __shfl(base, 0, 64);
      if (!ok)  // the reserved slots below the cap: empty items (no nodes), which the next round skips
        for (uint32_t i = base + lane; i < a.spill_cap && i - base < ptot; i += 64) a.spill_out[i] = make_uint4(0, 0, 0, 0);
      if (ok) {
        for (uint32_t i0 = 0; i0 < all; i0 += 64) {
          const uint32_t i = i0 + lane;
          uint4 it = make_uint4(0, 0, 0, 0);
          if (i < all) it = i < gtop ? stk[i] : ls[i - gtop];
          const uint32_t np = i < all ? (it.y + 63) >> 6 : 0u;
          uint32_t ctot;
          const uint32_t off = wave_excl(np, &ctot);
          if (TILE) it.w += static_cast<uint32_t>(fbase);
          for (uint32_t k = 0; k < np; ++k) {
            uint4 pc = it;
            pc.x = it.x + 64 * k;
            pc.y = min(64u, it.y - 64 * k);
            a.spill_out[base + off + k] = pc;
          }
          base += ctot;
        }
        return;
      }
      // no room: this wave finishes its stack itself (the budget is checked once)
    }
    if (top == 0) {
      // refill the LDS stack from the global part's top
      const uint32_t m = gtop < RSTK_HALF ? gtop : RSTK_HALF;
      for (uint32_t i = lane; i < m; i += 64) ls[i] = stk[gtop - m + i];
      gtop -= m;
      top = m;
      __builtin_amdgcn_wave_barrier();
    }
    // ---- take the next (up to) 64 nodes from the top items ----------------------------
    const uint32_t navail = top < 64 ? top : 64;
    uint4 it = make_uint4(0, 0, 0, 0);
    if (lane < navail) it = ls[top - 1 - lane];
    uint32_t ctot;
    const uint32_t cex = wave_excl(lane < navail ? it.y : 0u, &ctot);
    pref[lane] = cex + (lane < navail ? it.y : 0u);  // inclusive
    itm[lane] = it;
    if (a.ownmap) pref[64 + lane] = 0;
    __builtin_amdgcn_wave_barrier();
    // ownmap: lane -> item by the items' first lanes (their exclusive prefixes; distinct among
    // items with nodes, and the spill rounds' padding items have none) flagged in LDS with the
    // item's index and balloted, instead of a binary search over pref per lane
    uint64_t starts = 0;
    if (a.ownmap) {
      if (lane < navail && it.y && cex < 64) pref[64 + cex] = lane + 1;
      __builtin_amdgcn_wave_barrier();
      starts = __ballot(pref[64 + lane] != 0);
    }
    // items fully consumed: inclusive prefix <= 64
    const uint64_t full = __ballot(lane < navail && pref[lane] <= 64);
    const uint32_t kfull = __popcll(full);  // a prefix of the lanes (counts >= 1)
    const uint32_t taken = ctot < 64 ? ctot : 64;
    if (kfull < navail && lane == 0) {  // the partially consumed item stays, shortened
      const uint32_t used = 64 - (kfull ? pref[kfull - 1] : 0u);
      uint4 p = itm[kfull];
      p.x += used;
      p.y -= used;
      ls[top - 1 - kfull] = p;
    }
    top -= kfull;
    RPROF_MARK(0);
    // ---- this lane's node ---------------------------------------------------------------
    // A node is named by its postings index (RNAME_ROOT: the root), so its child lookup (the
    // edge bucket), the postings key after a '+' run and its own fields (posts[name]) are
    // all issued at once from the item and the filter's words: one round trip per step.
    bool act = lane < taken;
    uint32_t name = RNAME_ROOT, lev = 0, fl = 0, nl = 0, fn = 0, w_cur = WID_NONE, j = 0, wl = WID_HASH;
    uint64_t fg = 0;
    RNode rn{0, 0, 0, 0};
    uint4 ka = make_uint4(WID_NONE, 0, WID_NONE, 0), kb = ka, kc = make_uint4(0, 0, 0, 0);
    RPostKey pk{WID_NONE, 0, 0, 0};
    uint32_t bk = 0, ps = 0;
    bool nA = false, nB = false, nC = false;  // loads: node fields, edge bucket, postings key
    uint32_t iidx = 0xFFFFFFFFu;  // (RETAIN_PROF: the lane's item in this step)
    if (act) {
      uint32_t lo = 0, hi = navail - 1;  // first j with pref[j] > lane
      if (a.ownmap) {  // the last item start at or before this lane (lane 0 is always one)
        const uint64_t le = starts & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
        lo = pref[64 + 63 - static_cast<uint32_t>(__builtin_clzll(le))] - 1u;
      } else {
        while (lo < hi) {
          const uint32_t mid = (lo + hi) >> 1;
          if (pref[mid] > lane) hi = mid; else lo = mid + 1;
        }
      }
      iidx = lo;
      const uint32_t before = lo ? pref[lo - 1] : 0u;
      const uint4 q = itm[lo];
      lev = q.z & RITEM_LEVEL;
      fl = q.w;
      uint64_t wb;
      if (TILE) {
        nl = nlevs[fl];
        wb = wbase[fl];
        fg = fbase + fl;
        fn = nl & 0x7FFFFFFFu;
        w_cur = lev < fn ? word_at(a, lwords, wb + lev) : WID_NONE;
        if (w_cur == WID_PLUS) {  // the '+' run and the word after it
          j = lev + 1;
          while (j < fn && word_at(a, lwords, wb + j) == WID_PLUS) ++j;
          wl = j < fn ? word_at(a, lwords, wb + j) : WID_HASH;
        }
      } else {
        // a spill round: the level's descriptor, written by the first round, holds the word,
        // the '+' run's end and the word after it (one load, not a chain of word loads)
        // (queue mode: a piece's walk is one filter's, its first levels' descriptors in LDS,
        // deeper ones read at agent scope: its tile's wave wrote them in this launch)
        fg = fl;
        const uint4 d = !QUEUE         ? a.wdesc[(a.foffs[fg] - b0) + 2 * fg + lev]
                        : lev < ldn    ? ldesc[lev]
                                       : desc_load_sc(a.wdesc + (a.foffs[fg] - b0) + 2 * fg + lev);
        nl = d.w;
        fn = nl & 0x7FFFFFFFu;
        w_cur = d.x;
        if (w_cur == WID_PLUS) {
          j = d.y;
          wl = d.z;
        }
      }
      // A literal step needs only the edge bucket: a node without that child (a leaf
      // included) has no key for it there, so its own fields are not loaded (one random line
      // fewer per step of an exact filter).  Every other step reads them.
      if (q.z & RITEM_POST) {
        name = q.x + (lane - before);
        nA = w_cur >= WID_HASH;
      } else {
        rn = RNode{0, rv.root_ncld, rv.root_lo, rv.root_hi};
      }
      if (w_cur < WID_HASH) {  // a literal: its bucket
        bk = redge_slot0(name, w_cur) & rv.edge_mask;
        nB = true;
      } else if (w_cur == WID_PLUS && wl < WID_HASH && j < fn) {  // '+' run, then a literal
        ps = rpost_slot0(j + 1, wl) & rv.pkey_mask;
        nC = true;
      }
    }
    {  // the step's loads, one group under one wait (step_loads)
      uint4 pa;
      step_loads(rv.posts + name, reinterpret_cast<const uint4*>(rv.edges + bk), rv.pkeys + ps, nA, nB, nC, pa, ka, kb,
                 kc, pk);
      if (nA) rn = RNode{0, pa.z, pa.x, pa.w};
    }
    __builtin_amdgcn_wave_barrier();
    RPROF_MARK(1);
    RPROF_ADD(5, 1);
    RPROF_ADD(6, __popcll(__ballot(act)));
    bool emit = false, push = false;
    RRange rg{0, 0, 0, 0};
    uint4 np = make_uint4(0, 0, 0, 0);
    // a slice to cut to this node's rank interval: every lane that needs one searches at
    // one call site below (SK_DTERM: the per-depth rank list, SK_POSTS: a postings group)
    uint32_t skind = SK_NONE, sL = 0, sH = 0, plev = 0;
    if (act) {
      ++visits;
      rg.f = static_cast<uint32_t>(fg);
      // the match spec's strict guard for wildcard filters, and for every filter of a match
      // spec call (match_messages/3, page_read/4); read_message/2's `>=` otherwise
      rg.flags = (nl >> 31) | a.strict_all;
      const uint32_t ncld = rn.ncld & ~RNODE_TERM;
      if (lev == fn) {
        if (rn.ncld & RNODE_TERM) {
          emit = true;
          rg.lo = rn.lo;
          rg.hi = rn.lo + 1;
        }
      } else if (w_cur == WID_HASH) {
        emit = rn.hi > rn.lo;
        rg.lo = rn.lo;
        rg.hi = rn.hi;
      } else if (w_cur == WID_PLUS) {
        // the '+' run from this level, then: a literal -> its postings at the depth after the
        // run, inside this node's rank interval; the filter's end -> a slice of the per-depth
        // rank list; the final '#' -> the subtree's ranks with a depth floor
        if (ncld == 0 || wl == WID_NONE) {
          push = false;
        } else if (j == fn) {
          if (fn <= rv.max_depth) {
            skind = SK_DTERM;
            sL = rv.dterm_off[fn];
            sH = rv.dterm_off[fn + 1];
          }
        } else if (wl == WID_HASH) {
          emit = rn.hi > rn.lo;
          rg.lo = rn.lo;
          rg.hi = rn.hi;
          rg.flags |= j << RRANGE_MIND_SHIFT;
        } else {
          for (uint32_t k = 0; k <= rv.pkey_mask; ++k) {
            if (pk.depth == WID_NONE) break;
            if (pk.depth == j + 1 && pk.wid == wl) {
              skind = SK_POSTS;
              sL = pk.off;
              sH = pk.off + pk.len;
              plev = j + 1;
              break;
            }
            ps = (ps + 1) & rv.pkey_mask;
            pk = rv.pkeys[ps];
          }
        }
      } else if (w_cur < WID_HASH) {
        // the bucket's four keys and child names; a bucket that overflowed (REDGE_OVF)
        // continues in the next
        for (uint32_t k = 0; k <= rv.edge_mask; ++k) {
          const uint32_t hit = (ka.x == name && (ka.y & ~REDGE_OVF) == w_cur) ? kc.x
                               : (ka.z == name && ka.w == w_cur)             ? kc.y
                               : (kb.x == name && kb.y == w_cur)             ? kc.z
                               : (kb.z == name && kb.w == w_cur)             ? kc.w
                                                                             : RNAME_ROOT;
          if (hit != RNAME_ROOT) {
            push = true;
            np = make_uint4(hit, 1u, (lev + 1) | RITEM_POST, fl);
            break;
          }
          if (!(ka.y & REDGE_OVF)) break;
          bk = (bk + 1) & rv.edge_mask;
          const uint4* kp = reinterpret_cast<const uint4*>(rv.edges + bk);
          ka = kp[0];
          kb = kp[1];
          kc = kp[2];
        }
      }
    }
    RPROF_MARK(2);
    RPROF_ADD(7, __popcll(__ballot(skind != SK_NONE)));
#ifdef RETAIN_PROF
    {  // searching lanes of one item search one postings group: groups, lanes in groups of >= 8, >= 32
      const bool srch = skind != SK_NONE && name != RNAME_ROOT;
      uint32_t size = 0;
      for (uint32_t d = 0; d < 64; ++d) {
        const uint32_t v = __shfl(iidx, d, 64);
        const uint32_t sd = __shfl(srch ? 1u : 0u, d, 64);
        size += (srch && sd && v == iidx) ? 1u : 0u;
      }
      const uint32_t pi = __shfl_up(iidx, 1, 64), ps_ = __shfl_up(srch ? 1u : 0u, 1, 64);
      const bool first = srch && (lane == 0 || !ps_ || pi != iidx);
      RPROF_ADD(16, __popcll(__ballot(first)));
      RPROF_ADD(17, __popcll(__ballot(srch && size >= 8)));
      RPROF_ADD(18, __popcll(__ballot(srch && size >= 32)));
    }
#endif
    if (skind != SK_NONE) {
      uint32_t b = sL, e = sH;
      if (name != RNAME_ROOT) {  // the root's interval holds every rank: the whole slice
        const bool dt = skind == SK_DTERM;
        if (SEARCH == RSEARCH_STREE) {
          stree_lower_bound2(dt ? rv.dst : rv.pst, sL, sH, rn.lo, rn.hi, &b, &e);
        } else {
          const uint32_t* keys = dt ? rv.dterm : reinterpret_cast<const uint32_t*>(rv.posts);
          fenced_lower_bound2(keys, dt ? 1u : 4u, dt ? rv.dfence : rv.pfence, sL, sH, rn.lo, rn.hi, &b, &e);
        }
      }
      if (skind == SK_DTERM) {
        emit = e > b;
        rg.lo = b;
        rg.hi = e;
        rg.flags |= RRANGE_INDIRECT;
      } else {
        push = e > b;
        np = make_uint4(b, e - b, plev | RITEM_POST, fl);
      }
    }
    RPROF_MARK(3);
    // ---- emissions -----------------------------------------------------------------------
    // a range of at most RBIG ranks is one small record (lane-parallel in the output
    // kernels), from this wave's reservation, refilled RRES at a time (unused reserved slots
    // stay zeroed: empty); a longer one goes out as RCHUNK-rank big records (one wave each
    // in the output kernels), taken from the top of the buffer
    const uint32_t len = emit ? rg.hi - rg.lo : 0u;
    const uint32_t nsmall = emit && len <= RBIG ? 1u : 0u;
    const uint32_t nbig = len > RBIG ? (len + RCHUNK - 1) / RCHUNK : 0u;
    uint32_t etot, btot;
    const uint32_t epos = wave_excl(nsmall, &etot);
    const uint32_t bpos = wave_excl(nbig, &btot);
    if (etot) {
      if (etot > res.left) {
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&a.ctrl[RC_RANGES], etot + RRES);
        res.next = __shfl(base, 0, 64);
        res.left = etot + RRES;
      }
      if (nsmall && res.next + epos < a.range_cap) a.ranges[res.next + epos] = rg;
      res.next += etot;
      res.left -= etot;
      res.emitted += etot;
    }
    if (btot) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(&a.ctrl[RC_BIG], btot);
      base = __shfl(base, 0, 64);
      for (uint32_t k = 0; k < nbig; ++k) {
        const uint32_t at = base + bpos + k;  // from the top: ranges[range_cap - 1 - at]
        if (at >= a.range_cap) break;
        RRange part = rg;
        part.lo = rg.lo + k * RCHUNK;
        part.hi = min(rg.hi, part.lo + RCHUNK);
        a.ranges[a.range_cap - 1 - at] = part;
      }
      res.emitted += btot;
    }
    // ---- pushes ---------------------------------------------------------------------------
    uint32_t qtot;
    const uint32_t qpos = wave_excl(push ? 1u : 0u, &qtot);
    if (top + qtot > RSTK) {
      // the LDS stack's bottom half moves to the global part (top > RSTK - 64 >= RSTK_HALF)
      if (gtop + RSTK_HALF > a.stack_cap) {
        overflow = true;
        return;
      }
      for (uint32_t i = lane; i < RSTK_HALF; i += 64) stk[gtop + i] = ls[i];
      __builtin_amdgcn_wave_barrier();
      for (uint32_t i0 = 0; i0 < top - RSTK_HALF; i0 += 64) {  // shift down (reads stay ahead of writes)
        const uint32_t i = i0 + lane;
        uint4 x = make_uint4(0, 0, 0, 0);
        if (i < top - RSTK_HALF) x = ls[RSTK_HALF + i];
        __builtin_amdgcn_wave_barrier();
        if (i < top - RSTK_HALF) ls[i] = x;
      }
      gtop += RSTK_HALF;
      top -= RSTK_HALF;
      __threadfence_block();  // the global part is read back by other lanes
    }
    if (push) ls[top + qpos] = np;
    top += qtot;
    __builtin_amdgcn_wave_barrier();
    if (QUEUE && look) {  // the waiting count, loaded at the step's start
      const uint32_t hungry =
          static_cast<int32_t>(static_cast<uint32_t>(ht) - static_cast<uint32_t>(ht >> 32)) > 0 ? 1u : 0u;
      if (__shfl(hungry, 0, 64)) {
        const uint64_t ts = RPROF_NOW();
        share_work<TILE>(a, *qs, ls, top, stk, gtop, fbase, qstat[0], nlevs, pub, pnw);
        ++qstat[1];
        RPROF_ADD(11, RPROF_NOW() - ts);
      }
    }
  }
}

}  // namespace

template <int SEARCH>
__global__ __launch_bounds__(RW_WAVES * 64, RW_OCC) void retain_walk_kernel(RetainArgs a) {
  const uint32_t lane = lane_id();
  const uint32_t wib = threadIdx.x >> 6;
  const uint32_t gw = blockIdx.x * RW_WAVES + wib;
  __shared__ uint32_t s_pref[RW_WAVES][128];  // [64, 128): the step's item-start flags
  __shared__ uint4 s_item[RW_WAVES][64];
  __shared__ uint32_t s_nlev[RW_WAVES][64];
  __shared__ uint64_t s_wb[RW_WAVES][64];
  __shared__ uint4 s_stk[RW_WAVES][RSTK];
  __shared__ uint32_t s_words[RW_WAVES][RWORDS];
  uint32_t* nlevs = s_nlev[wib];
  uint64_t* wbase = s_wb[wib];  // per filter of the tile: its first word id in a.wids
  uint4* stk = a.stack + static_cast<uint64_t>(gw) * a.stack_cap;
  const RetainView& rv = a.rv;
  const uint32_t tf = a.tile_filters;  // filters per wave tile (1..64): fewer = more waves in flight
  const uint64_t ntiles = (a.n + tf - 1) / tf;
  const uint64_t b0 = a.foffs[0];
  uint32_t visits = 0;
  bool overflow = false;
  uint64_t pacc[RPROF_SLOTS] = {};
  RangeRes res;

  // tiles beyond the first wave-full are taken first come, first served (one atomic per
  // tile): a wave whose tile was light takes the next one instead of a fixed stride's
  for (uint64_t t = gw; t < ntiles;) {
    const uint64_t f = t * tf + lane;
    const bool valid = lane < tf && f < a.n;
    // ---- tokenize + intern (per lane) -------------------------------------------------
    const uint32_t nw = valid ? tokenize_filter<true>(a, f) : 0u;
    const uint32_t nlev = nw & 0x7FFFFFFFu;
    nlevs[lane] = nw;
    // the tile's words into LDS when they fit (the walk reads one or two per node visit)
    uint32_t wtot;
    const uint32_t wofs = wave_excl(valid ? nlev : 0u, &wtot);
    const bool lds_words = wtot <= RWORDS;
    if (lds_words && valid) {
      const uint32_t* wsrc = a.wids + (a.foffs[f] - b0) + f;  // this lane's own stores above
      for (uint32_t l = 0; l < nlev; ++l) s_words[wib][wofs + l] = wsrc[l];
    }
    wbase[lane] = !valid ? 0 : lds_words ? wofs : (a.foffs[f] - b0) + f;
    // root items
    const bool push0 = valid && rv.n_nodes != 0;
    uint32_t ptot;
    const uint32_t ppos = wave_excl(push0 ? 1u : 0u, &ptot);
    if (push0) s_stk[wib][ppos] = make_uint4(0u, 1u, 0u, lane);
    __builtin_amdgcn_wave_barrier();
    walk_stack<true, SEARCH, false>(a, s_stk[wib], ptot, stk, 0, t * tf, nlevs, wbase,
                             lds_words ? s_words[wib] : nullptr, s_pref[wib], s_item[wib], visits,
                             overflow, res, pacc);
    if (overflow) break;
    uint32_t nx = 0;
    if (lane == 0) nx = atomicAdd(&a.ctrl[RC_TILE], 1u);
    t = a.waves + static_cast<uint64_t>(__shfl(nx, 0, 64));
  }
  if (overflow && lane == 0) atomicOr(&a.ctrl[RC_STACK], 1u);
  // visits: one atomic per wave
  uint32_t vtot;
  (void)wave_excl(visits, &vtot);
  if (lane == 0 && vtot) atomicAdd(&a.ctrl[RC_STAT + 16 * (gw % RC_STAT_LINES)], vtot);
  if (lane == 0 && res.emitted) atomicAdd(&a.ctrl[RC_STAT + 16 * (gw % RC_STAT_LINES) + 1], res.emitted);
#ifdef RETAIN_PROF
  if (lane == 0 && a.prof)
    for (uint32_t i = 0; i < RPROF_SLOTS; ++i) atomicAdd(reinterpret_cast<unsigned long long*>(a.prof + i), pacc[i]);
#else
  (void)pacc;
#endif
}

// A spill round: the items the previous round left (global filter ids), their count read
// from ctrl[in_word], dealt `per_wave` to a wave over at most gridDim waves, each walking its
// share under the same step budget.  No items: every wave returns at once.
template <int SEARCH>
__global__ __launch_bounds__(RW_WAVES * 64, RW_OCC) void retain_walk_spill_kernel(RetainArgs a, const uint4* in,
                                                                          uint32_t in_word, uint32_t per_wave) {
  const uint32_t lane = lane_id();
  const uint32_t wib = threadIdx.x >> 6;
  const uint32_t gw = blockIdx.x * RW_WAVES + wib;
  __shared__ uint32_t s_pref[RW_WAVES][128];  // [64, 128): the step's item-start flags
  __shared__ uint4 s_item[RW_WAVES][64];
  __shared__ uint4 s_stk[RW_WAVES][RSTK];
  const uint32_t n_in = static_cast<uint32_t>(
      min(__hip_atomic_load(reinterpret_cast<const unsigned long long*>(a.ctrl + in_word), __ATOMIC_RELAXED,
                            __HIP_MEMORY_SCOPE_AGENT),
          static_cast<unsigned long long>(a.spill_cap)));
  if (n_in == 0) return;
  if (gw == 0 && lane == 0) {
    atomicAdd(&a.ctrl[RC_ROUNDS], 1u);
    atomicAdd(&a.ctrl[RC_SPILLED], n_in);
  }
  const uint32_t waves = max(1u, min(a.waves, (n_in + per_wave - 1) / per_wave));
  if (gw >= waves) return;
  uint4* stk = a.stack + static_cast<uint64_t>(gw) * a.stack_cap;
  const uint32_t per = (n_in + waves - 1) / waves;
  const uint64_t lo = static_cast<uint64_t>(gw) * per;
  const uint64_t hi = lo + per < n_in ? lo + per : static_cast<uint64_t>(n_in);
  const uint32_t top = hi > lo ? static_cast<uint32_t>(hi - lo) : 0u;
  uint32_t visits = 0;
  bool overflow = top > a.stack_cap;
  uint64_t pacc[RPROF_SLOTS] = {};
  RangeRes res;
  if (!overflow) {
    for (uint32_t i = lane; i < top; i += 64) stk[i] = in[lo + i];
    __threadfence_block();
    walk_stack<false, SEARCH, false>(a, s_stk[wib], 0, stk, top, 0, nullptr, nullptr, nullptr, s_pref[wib],
                              s_item[wib], visits,
                              overflow, res, pacc);
  }
  if (overflow && lane == 0) atomicOr(&a.ctrl[RC_STACK], 1u);
  uint32_t vtot;
  (void)wave_excl(visits, &vtot);
  if (lane == 0 && vtot) atomicAdd(&a.ctrl[RC_STAT + 16 * (gw % RC_STAT_LINES)], vtot);
  if (lane == 0 && res.emitted) atomicAdd(&a.ctrl[RC_STAT + 16 * (gw % RC_STAT_LINES) + 1], res.emitted);
#ifdef RETAIN_PROF
  if (lane == 0 && a.prof)
    for (uint32_t i = 0; i < RPROF_SLOTS; ++i) atomicAdd(reinterpret_cast<unsigned long long*>(a.prof + i), pacc[i]);
#else
  (void)pacc;
#endif
}

// Retire one unit of the shard (a tile or a piece walked to its end, or a tile ticket that found
// none).  A retire that leaves nothing held or queued once the shard's tiles are all taken ends
// the shard's walk: the wave sets QS_DONE, then writes the end marker into every slot a waiting
// wave can hold: tickets below the head it reads after setting QS_DONE, from the reserved count
// (or the first never-written slot) on.  A wave whose ticket comes later reads QS_DONE after
// taking it; one past the shard's slots polls QS_DONE.  (Two waves may both end it: the markers
// are the same.)
__device__ __forceinline__ void retire_unit(const QShard& qs) {
  const uint32_t lane = lane_id();
  uint32_t lo = 0, hi = 0;
  if (lane == 0) {
    const uint32_t old = atomicAdd(&qs.c[QS_PEND], 0xFFFFFFFFu);
    if (old == 1u &&
        __hip_atomic_load(&qs.c[QS_TILES], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= qs.ntiles) {
      __hip_atomic_store(&qs.c[QS_DONE], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_s_waitcnt(0);  // done is set before the head is read
      const uint64_t ht = __hip_atomic_load(reinterpret_cast<const uint64_t*>(qs.c + QS_HEAD), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t fail = ~__hip_atomic_load(&qs.c[QS_FAIL], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      lo = min(static_cast<uint32_t>(ht >> 32), fail);
      hi = min(static_cast<uint32_t>(ht), qs.cap);
    }
  }
  lo = __shfl(lo, 0, 64);
  hi = __shfl(hi, 0, 64);
  for (uint32_t k = lo + lane; k < hi; k += 64) queue_put(qs.q + k, make_uint4(0u, QEND, 0u, 0u));
}

// Queue mode, the walk.  Wave w works in shard s = w % qshards: it takes the shard's tiles by
// ticket (QS_TILES), then its shared pieces by ticket (QS_HEAD; a ticket names a slot).  Busy
// waves share when waves of their shard wait (share_work).  QS_PEND counts the units held or
// queued, and only a wave holding one (or announcing a tile ticket, raised before the ticket is
// taken) raises it, so once it is 0 with the tiles all taken nothing is held or queued and no
// piece can come: the wave whose retire saw that wakes the waiting ones (retire_unit).  A wave
// holds work only after it started, so waves not yet resident hold nothing and the grid drains;
// a waiting wave also gives up after qpoll_limit polls (RC_QABORT; the host reruns the call in
// spill mode), a safety valve that a correct walk never reaches.
// compiled for 4 waves per SIMD (<= 128 VGPRs): 16 resident waves per CU instead of 12
#ifndef QW_OCC
#define QW_OCC 4
#endif
template <int SEARCH>
__global__ __launch_bounds__(RW_WAVES * 64, QW_OCC) void retain_walk_queue_kernel(RetainArgs a) {
  const uint32_t lane = lane_id();
  const uint32_t wib = threadIdx.x >> 6;
  const uint32_t gw = blockIdx.x * RW_WAVES + wib;
  __shared__ uint32_t s_pref[RW_WAVES][128];  // [64, 128): the step's item-start flags
  __shared__ uint4 s_item[RW_WAVES][64];
  __shared__ uint32_t s_nlev[RW_WAVES][64];
  __shared__ uint64_t s_wb[RW_WAVES][64];
  __shared__ uint4 s_stk[RW_WAVES][RSTK];
  __shared__ uint32_t s_words[RW_WAVES][RWORDS];
  __shared__ uint4 s_desc[RW_WAVES][QDESC];
  uint32_t* nlevs = s_nlev[wib];
  uint64_t* wbase = s_wb[wib];
  uint4* stk = a.stack + static_cast<uint64_t>(gw) * a.stack_cap;
  const RetainView& rv = a.rv;
  const uint32_t tf = a.tile_filters;
  const uint64_t b0 = a.foffs[0];
  const QShard qs = qshard(a, gw);
  const uint32_t maxwait = max(2u, a.qmaxwait / a.qshards);
  uint32_t visits = 0, qstat[2] = {0, 0};
  bool overflow = false;
  uint64_t pacc[RPROF_SLOTS] = {};
  RangeRes res;
  // ---- the shard's tiles ----------------------------------------------------------------------
  for (;;) {
    uint32_t t = 0;
    uint64_t tq = RPROF_NOW();
    if (lane == 0) {
      atomicAdd(&qs.c[QS_PEND], 1u);  // announced before the ticket: see retire_unit
      __builtin_amdgcn_s_waitcnt(0);
      t = qs.s + a.qshards * atomicAdd(&qs.c[QS_TILES], 1u);
    }
    t = __shfl(t, 0, 64);
    RPROF_ADD(9, RPROF_NOW() - tq);
    if (t >= a.ntiles) {
      retire_unit(qs);  // no tile: the announcement is withdrawn
      break;
    }
    const uint64_t f = static_cast<uint64_t>(t) * tf + lane;
    const bool valid = lane < tf && f < a.n;
    uint32_t nw = 0;
    uint64_t wsrc = 0;
    if (valid) {
      nw = tokenize_filter<false>(a, f);  // descriptors: published with the filter's first piece
      wsrc = (a.foffs[f] - b0) + f;
    }
    const uint32_t nlev = nw & 0x7FFFFFFFu;
    nlevs[lane] = valid ? nw : 0xFFFFFFFFu;  // (no filter: share_work publishes nothing for it)
    uint32_t wtot;
    const uint32_t wofs = wave_excl(valid ? nlev : 0u, &wtot);
    const bool lds_words = wtot <= RWORDS;
    if (lds_words && valid)
      for (uint32_t l = 0; l < nlev; ++l) s_words[wib][wofs + l] = a.wids[wsrc + l];
    wbase[lane] = !valid ? 0 : lds_words ? wofs : wsrc;
    const bool push0 = valid && rv.n_nodes != 0;
    uint32_t ptot;
    const uint32_t ppos = wave_excl(push0 ? 1u : 0u, &ptot);
    if (push0) s_stk[wib][ppos] = make_uint4(0u, 1u, 0u, lane);
    __builtin_amdgcn_wave_barrier();
    uint64_t t0 = RPROF_NOW();
    uint64_t pub = 0;  // tile lanes whose step descriptors are published (share_work)
    walk_stack<true, SEARCH, true>(a, s_stk[wib], ptot, stk, 0, static_cast<uint64_t>(t) * tf, nlevs, wbase,
                                   lds_words ? s_words[wib] : nullptr, s_pref[wib], s_item[wib], visits, overflow,
                                   res, pacc, &qs, qstat, nullptr, 0, &pub);
    uint64_t t1 = RPROF_NOW();
    RPROF_ADD(13, t1 - t0);
    retire_unit(qs);  // this tile is walked (or abandoned)
    RPROF_ADD(10, RPROF_NOW() - t1);
    if (overflow) break;
  }
  // ---- shared pieces: the home shard's, then (roaming) other shards' ------------------------
  // At most `maxwait` waves of a shard wait at once: a wave that finds that many tickets beyond
  // the reserved slots moves on instead of taking one.  Safe: a shared piece's slot is below the
  // reserved count, so either its ticket is taken already or fewer than maxwait wait and the next
  // wave to come (at the latest the one that shared it, once its own stack is empty) takes one.
  // A wave whose shard's walk is over visits up to qroam other shards (an odd stride over the
  // ring, so each visit is a new one) and helps the ones still walking: the shards' work is
  // uneven (a few broad filters), and the launch lasts as long as its slowest shard.
  uint32_t polls = 0, hops = 0;
  const uint32_t stride = 2u * ((gw / a.qshards) % max(1u, a.qshards / 2)) + 1u;
  QShard cur = qs;
  while (!overflow) {
    uint32_t k = 0, state = 0;  // 1: a piece, 2: this shard's walk is over (or enough waves wait)
    uint64_t tq = RPROF_NOW();
    if (lane == 0) {
      // a shard is worth waiting in if its walk is not over and one of its own waves has
      // started: that wave takes all its tiles in turn, so the shard ends.  (A shard none of
      // whose waves is resident yet must not collect waiting visitors: they would hold the slots
      // its waves need.)
      const uint64_t td = __hip_atomic_load(reinterpret_cast<const uint64_t*>(cur.c + QS_TILES), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
      if ((td >> 32) != 0 || static_cast<uint32_t>(td) == 0) {
        state = 2;
      } else {
        const uint64_t ht = __hip_atomic_load(reinterpret_cast<const uint64_t*>(cur.c + QS_HEAD), __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
        if (static_cast<int32_t>(static_cast<uint32_t>(ht) - static_cast<uint32_t>(ht >> 32)) >=
            static_cast<int32_t>(maxwait))
          state = 2;
        else
          k = atomicAdd(&cur.c[QS_HEAD], 1u);
      }
    }
    state = __shfl(state, 0, 64);
    k = __shfl(k, 0, 64);
    uint4 it = make_uint4(0, 0, 0, 0);
    if (state == 0) {
      if (lane == 0 && __hip_atomic_load(&cur.c[QS_DONE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) state = 2;
      state = __shfl(state, 0, 64);
    }
    const uint64_t tw = RPROF_NOW();
    RPROF_ADD(9, tw - tq);
    while (state == 0) {
      if (lane == 0) {
        if (k < cur.cap) {
          if (queue_get(cur.q + k, &it)) state = it.y == QEND ? 2u : 1u;
        } else if (__hip_atomic_load(&cur.c[QS_DONE], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
          state = 2;
        }
        if (state == 0 && ++polls > a.qpoll_limit) {
          atomicOr(&a.ctrl[RC_QABORT], 1u);
          state = 3;  // give up entirely
        }
      }
      state = __shfl(state, 0, 64);
      if (state) break;
      for (uint32_t z = 0; z < a.qsleep; ++z) __builtin_amdgcn_s_sleep(16);
    }
    const uint64_t tp = RPROF_NOW();
    RPROF_ADD(8, tp - tw);
    if (state == 3) break;
    if (state == 2) {
      if (hops++ >= a.qroam) {
        RPROF_ADD(15, 1);
        break;
      }
      cur = qshard_at(a, (cur.s + stride) % a.qshards);
      continue;
    }
    RPROF_ADD(12, 1);
    // the piece: its level, its filter's level count (carried in z), and the filter's step
    // descriptors from the piece's level down (one round trip; the walk only goes deeper and
    // stays inside this filter) into LDS
    const uint32_t pz = __shfl(it.z, 0, 64), pw = __shfl(it.w, 0, 64);
    const uint32_t lev0 = pz & ((1u << QNLEV_SHIFT) - 1u), pnlev = (pz & ~RITEM_POST) >> QNLEV_SHIFT;
    if (lane == 0) s_stk[wib][0] = make_uint4(it.x, it.y, lev0 | (pz & RITEM_POST), pw);
    const uint64_t dbase = (a.foffs[pw] - b0) + 2ull * pw;
    const uint32_t ldn = min(QDESC, pnlev + 1u);
    if (lane >= lev0 && lane < ldn) s_desc[wib][lane] = desc_load_sc(a.wdesc + dbase + lane);
    __builtin_amdgcn_wave_barrier();
    walk_stack<false, SEARCH, true>(a, s_stk[wib], 1, stk, 0, 0, nullptr, nullptr, nullptr, s_pref[wib],
                                    s_item[wib], visits, overflow, res, pacc, &cur, qstat, s_desc[wib], ldn, nullptr,
                                    pnlev);
    const uint64_t te = RPROF_NOW();
    RPROF_ADD(14, te - tp);
    retire_unit(cur);
    RPROF_ADD(10, RPROF_NOW() - te);
  }
  if (overflow && lane == 0) atomicOr(&a.ctrl[RC_STACK], 1u);
  uint32_t vtot;
  (void)wave_excl(visits, &vtot);
  uint32_t* st = a.ctrl + RC_STAT + 16 * (gw % RC_STAT_LINES);
  if (lane == 0 && vtot) atomicAdd(&st[0], vtot);
  if (lane == 0 && res.emitted) atomicAdd(&st[1], res.emitted);
  if (lane == 0 && qstat[0]) atomicAdd(&st[2], qstat[0]);
  if (lane == 0 && qstat[1]) atomicAdd(&st[3], qstat[1]);
#ifdef RETAIN_PROF
  if (lane == 0 && a.prof)
    for (uint32_t i = 0; i < RPROF_SLOTS; ++i) atomicAdd(reinterpret_cast<unsigned long long*>(a.prof + i), pacc[i]);
#else
  (void)pacc;
#endif
}

// Queue mode, the call's last walk step: every shard's written slots (below its ticket and
// reserved counts) and its control words back to zero for the next call.
// grid (x, shard): the slots the call used, cleared by many blocks per shard (one block per
// shard was bandwidth-starved: ~0.1 ms a call); the control words after, by
// retain_queue_reset_kernel (every block here reads them first).
constexpr uint32_t QCLEAR_BLOCKS = 32;
__global__ __launch_bounds__(256) void retain_queue_clear_kernel(RetainArgs a) {
  const uint32_t* c = a.qctl + static_cast<uint64_t>(blockIdx.y) * QS_STRIDE;
  const uint32_t cap = a.queue_cap / a.qshards;
  const uint32_t n = min(max(c[QS_HEAD], c[QS_TAIL]), cap);
  uint4* q = a.queue + static_cast<uint64_t>(blockIdx.y) * cap;
  for (uint32_t k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x)
    q[k] = make_uint4(0, 0, 0, 0);
}

__global__ __launch_bounds__(64) void retain_queue_reset_kernel(RetainArgs a) {
  uint32_t* c = a.qctl + static_cast<uint64_t>(blockIdx.x) * QS_STRIDE;
  if (threadIdx.x < 16) c[threadIdx.x] = 0;
}

namespace {

// count (mode 0) / write (mode 1), grid-stride over work units: a ROW of 8 consecutive small
// records, one per 8-lane group, each lane of a group taking every 8th rank of the record
// (at most RBIG / 8 = 8, all loads in flight at once); or one BIG record (its RCHUNK ranks, the
// whole wave in one pass).  A record is one round trip (two when indirect), not one per rank.
constexpr uint32_t RUNROLL = RCHUNK / 64;
constexpr uint32_t RGROUP = 8;                // lanes per small record
constexpr uint32_t RPER = RBIG / RGROUP;      // ranks per lane of a small record, at most
template <int MODE>
__global__ __launch_bounds__(256, MODE == 1 ? 7 : 6) void retain_out_kernel(RetainArgs a) {
  const uint32_t lane = lane_id();
  const uint32_t gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
  const uint32_t grp = lane / RGROUP, sub = lane % RGROUP;
  const RetainView& rv = a.rv;
  const uint32_t ns = a.ctrl[RC_RANGES], nb = a.ctrl[RC_BIG];
  if (static_cast<uint64_t>(ns) + nb > a.range_cap) return;  // the host reruns with more room
  if (MODE == 1 && a.out_off[a.n] > a.out_cap) return;      // too many ids: the caller grows
                                                            // its buffer and asks again
  const bool guard = rv.has_expiring && a.now_ms >= 0;
  // units: SUPER-ROWS of 64 consecutive small records (8 rows of 8), then the big records
  const uint64_t nrows = (static_cast<uint64_t>(ns) + 63) / 64;
#ifdef RETAIN_PROF
  // ablations (timing experiments only): bit 0 no small rows, 1 no big records, 2 no atomics
  const uint32_t abl = a.ablate;
#else
  const uint32_t abl = 0;
#endif
  for (uint64_t u = gw; u < nrows + nb; u += nw) {
    if ((abl & 1) && u < nrows) continue;
    if ((abl & 2) && u >= nrows) continue;
    if (u < nrows) {
      // ---- a super-row: lane i holds record u*64 + i for the per-filter totals; each of its 8
      // rows gives every record 8 lanes (every 8th rank, all loads of the record in flight) ----
      const uint64_t rme = u * 64 + lane;
      RRange mine{0, 0, 0, 0};
      if (rme < ns) mine = a.ranges[rme];  // an unused reserved slot reads as lo == hi
      // Per-filter totals: a filter's records sit side by side (a wave's step emits them
      // together), so runs of equal filters over the 64 records take one atomic per run, from
      // the run's last lane (a broad filter's thousands of records would otherwise queue on one
      // address).  Empty records end runs.
      const uint32_t fme = mine.hi > mine.lo ? mine.f : 0xFFFFFFFFu;
      const uint32_t fprev = __shfl_up(fme, 1, 64), fnext = __shfl_down(fme, 1, 64);
      const uint64_t hm = __ballot(lane == 0 || fprev != fme), tm = __ballot(lane == 63 || fnext != fme);
      const uint32_t rstart = 63u - __clzll(hm & (~0ull >> (63 - lane)));  // this run's first lane
      const uint32_t rend = lane + __ffsll(static_cast<long long>(tm >> lane)) - 1u;  // its last
      const bool tail = (tm >> lane) & 1u;
      uint32_t cme = 0;  // this lane's record's live ranks
      uint64_t pos = 0;  // write pass: its first output position
      if (MODE == 1) {
        cme = fme != 0xFFFFFFFFu ? a.rcount[rme] : 0u;
        uint32_t tot;
        const uint32_t incl = wave_excl(cme, &tot) + cme;
        const uint32_t prev = __shfl(incl, rstart ? rstart - 1 : 0, 64);  // every lane takes part
        const uint32_t before = rstart ? prev : 0u;
        const uint32_t rincl = incl - before;
        uint64_t base = 0;
        if (tail && fme != 0xFFFFFFFFu && rincl)
          base = a.out_off[fme] + ((abl & 4) ? 0u : atomicAdd(&a.fcursor[fme], rincl));
        const uint32_t blo = __shfl(static_cast<uint32_t>(base), rend, 64);
        const uint32_t bhi = __shfl(static_cast<uint32_t>(base >> 32), rend, 64);
        pos = ((static_cast<uint64_t>(bhi) << 32) | blo) + (rincl - cme);
      }
#pragma unroll 1
      for (uint32_t row = 0; row < 8; ++row) {
        const uint32_t src = row * 8 + grp;  // the lane holding this group's record
        const uint64_t r = u * 64 + src;
        RRange rg;
        rg.f = __shfl(mine.f, src, 64);
        rg.lo = __shfl(mine.lo, src, 64);
        rg.hi = __shfl(mine.hi, src, 64);
        rg.flags = __shfl(mine.flags, src, 64);
        const bool check = guard || (rg.flags >> RRANGE_MIND_SHIFT) != 0;
        uint32_t rk[RPER];
        bool live[RPER];
#pragma unroll
        for (uint32_t k = 0; k < RPER; ++k) {
          const uint32_t i = rg.lo + sub + RGROUP * k;
          rk[k] = i < rg.hi ? rank_at(rv, i, rg.flags) : 0u;
        }
        // a checked record's live ranks: the count pass tests them (expiry, depth) and keeps the
        // mask (bit sub + RGROUP * k), the write pass takes the mask instead of loading them again
        uint64_t lm = 0;
        if (MODE == 1 && check && rg.hi > rg.lo) lm = a.rlive[r];
#pragma unroll
        for (uint32_t k = 0; k < RPER; ++k) {
          const bool in = rg.lo + sub + RGROUP * k < rg.hi;
          if (MODE == 1 && check)
            live[k] = (lm >> (sub + RGROUP * k)) & 1u;
          else
            live[k] = in && (!check || rank_ok(rv, rk[k], guard, a.now_ms, rg.flags));
        }
        if (MODE == 0) {
          uint32_t c = 0;
          uint64_t m = 0;
#pragma unroll
          for (uint32_t k = 0; k < RPER; ++k) {
            c += live[k] ? 1u : 0u;
            m |= ((__ballot(live[k]) >> (grp * RGROUP)) & 0xFFull) << (RGROUP * k);
          }
          c += __shfl_xor(c, 1, 64);
          c += __shfl_xor(c, 2, 64);
          c += __shfl_xor(c, 4, 64);
          if (sub == 0 && rg.hi > rg.lo) {
            a.rcount[r] = c;
            if (check) a.rlive[r] = m;
          }
          const uint32_t cr = __shfl(c, (lane & 7) * 8, 64);  // row `row`'s group (lane & 7)
          if ((lane >> 3) == row) cme = cr;
        } else {
          uint64_t p = (static_cast<uint64_t>(__shfl(static_cast<uint32_t>(pos >> 32), src, 64)) << 32) |
                       __shfl(static_cast<uint32_t>(pos), src, 64);
          uint32_t id[RPER];
#pragma unroll
          for (uint32_t k = 0; k < RPER; ++k) id[k] = live[k] ? rv.rank_id[rk[k]] : 0u;
#pragma unroll
          for (uint32_t k = 0; k < RPER; ++k) {
            const uint32_t bits = static_cast<uint32_t>(__ballot(live[k]) >> (grp * RGROUP)) & 0xFFu;
            const uint32_t rank = __popc(bits & ((1u << sub) - 1u));
            if (live[k] && p + rank < a.out_cap) a.out_ids[p + rank] = id[k];
            p += __popc(bits);
          }
        }
      }
      if (MODE == 0) {
        uint32_t tot;
        const uint32_t incl = wave_excl(cme, &tot) + cme;
        const uint32_t prev = __shfl(incl, rstart ? rstart - 1 : 0, 64);  // every lane takes part
        const uint32_t before = rstart ? prev : 0u;
        const uint32_t rincl = incl - before;
        if (tail && fme != 0xFFFFFFFFu && rincl && !(abl & 4)) atomicAdd(&a.fcount[fme], rincl);
      }
    } else {
      // ---- one big record: RCHUNK ranks over the wave, every load of the pass in flight ----
      const uint32_t br = a.range_cap - 1 - static_cast<uint32_t>(u - nrows);
      const RRange rg = a.ranges[br];
      const bool check = guard || (rg.flags >> RRANGE_MIND_SHIFT) != 0;
      uint32_t rk[RUNROLL];
      bool live[RUNROLL];
#pragma unroll
      for (uint32_t k = 0; k < RUNROLL; ++k) {
        const uint32_t i = rg.lo + k * 64 + lane;
        rk[k] = i < rg.hi ? rank_at(rv, i, rg.flags) : 0u;
      }
      uint64_t* const bm = a.rlive + a.range_cap + static_cast<uint64_t>(u - nrows) * RUNROLL;
      if (MODE == 1 && check) {
#pragma unroll
        for (uint32_t k = 0; k < RUNROLL; ++k) live[k] = (bm[k] >> lane) & 1u;
      } else {
#pragma unroll
        for (uint32_t k = 0; k < RUNROLL; ++k)
          live[k] = rg.lo + k * 64 + lane < rg.hi && (!check || rank_ok(rv, rk[k], guard, a.now_ms, rg.flags));
      }
      if (MODE == 0) {
        uint32_t cnt = 0;
#pragma unroll
        for (uint32_t k = 0; k < RUNROLL; ++k) {
          cnt += live[k] ? 1u : 0u;
          const uint64_t m = __ballot(live[k]);
          if (check && lane == k) bm[k] = m;
        }
        uint32_t tot;
        (void)wave_excl(cnt, &tot);
        if (lane == 0) {
          a.rcount[br] = tot;
          if (tot && !(abl & 4)) atomicAdd(&a.fcount[rg.f], tot);
        }
      } else {
        uint32_t id[RUNROLL];
#pragma unroll
        for (uint32_t k = 0; k < RUNROLL; ++k) id[k] = live[k] ? rv.rank_id[rk[k]] : 0u;
        const uint32_t c = a.rcount[br];
        uint64_t p = 0;
        if (lane == 0 && c) p = a.out_off[rg.f] + ((abl & 4) ? 0u : atomicAdd(&a.fcursor[rg.f], c));
        p = __shfl(p, 0, 64);
#pragma unroll
        for (uint32_t k = 0; k < RUNROLL; ++k) {
          const uint64_t m = __ballot(live[k]);
          const uint32_t rank = __popcll(m & ((1ull << lane) - 1ull));
          if (live[k] && p + rank < a.out_cap) a.out_ids[p + rank] = id[k];
          p += __popcll(m);
        }
      }
    }
  }
}

}  // namespace

hipError_t launch_retain_walk(const RetainArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  const uint32_t blocks = (a.waves + RW_WAVES - 1) / RW_WAVES;
  if (a.search == RSEARCH_STREE)
    hipLaunchKernelGGL(retain_walk_kernel<RSEARCH_STREE>, dim3(blocks), dim3(RW_WAVES * 64), 0, s, a);
  else
    hipLaunchKernelGGL(retain_walk_kernel<RSEARCH_FENCED>, dim3(blocks), dim3(RW_WAVES * 64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_retain_walk_queue(const RetainArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  const uint32_t blocks = (a.waves + RW_WAVES - 1) / RW_WAVES;
  if (a.search == RSEARCH_STREE)
    hipLaunchKernelGGL(retain_walk_queue_kernel<RSEARCH_STREE>, dim3(blocks), dim3(RW_WAVES * 64), 0, s, a);
  else
    hipLaunchKernelGGL(retain_walk_queue_kernel<RSEARCH_FENCED>, dim3(blocks), dim3(RW_WAVES * 64), 0, s, a);
  hipLaunchKernelGGL(retain_queue_clear_kernel, dim3(QCLEAR_BLOCKS, a.qshards), dim3(256), 0, s, a);
  hipLaunchKernelGGL(retain_queue_reset_kernel, dim3(a.qshards), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_retain_walk_spill(const RetainArgs& a, const uint4* in, uint32_t in_word, uint32_t per_wave,
                                    hipStream_t s) {
  if (a.waves == 0) return hipSuccess;
  const uint32_t blocks = (a.waves + RW_WAVES - 1) / RW_WAVES;
  if (a.search == RSEARCH_STREE)
    hipLaunchKernelGGL(retain_walk_spill_kernel<RSEARCH_STREE>, dim3(blocks), dim3(RW_WAVES * 64), 0, s, a, in,
                       in_word, std::max(1u, per_wave));
  else
    hipLaunchKernelGGL(retain_walk_spill_kernel<RSEARCH_FENCED>, dim3(blocks), dim3(RW_WAVES * 64), 0, s, a, in,
                       in_word, std::max(1u, per_wave));
  return hipGetLastError();
}

// grid of the output kernels: sized by the range capacity (the range count is on the device)
static uint32_t out_blocks(uint32_t cap) {
  const uint64_t waves = (static_cast<uint64_t>(cap) + 7) / 8;  // one per 8 slots (super-rows of 64 + big records)
  return static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>((waves + 3) / 4, 8192)));
}

hipError_t launch_retain_count(const RetainArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(retain_out_kernel<0>, dim3(out_blocks(a.range_cap)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_retain_write(const RetainArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(retain_out_kernel<1>, dim3(out_blocks(a.range_cap)), dim3(256), 0, s, a);
  return hipGetLastError();
}

}  // namespace emqx
