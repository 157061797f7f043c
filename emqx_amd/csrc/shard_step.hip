// Filter-sharded match step on the device (include/emqx_match.h emqx_shard_step_*, driven by
// emqx_amd/dist.py ShardedMatcher.match_all): the regrouping around the two all-to-alls, with
// no host work beyond the split sizes the collectives need.
//
// The reference replicates every route on every node (emqx_router.erl:135, mria) and matches a
// publish on the node that receives it (emqx_broker.erl:213 -> emqx_router:match_routes/1); a
// table past one GPU is sharded here instead, and one rank's step is
//
//   send    route every topic to its (rank, engine) requests (layout.h shard_route_topic),
//           fold them onto the rank's three engine slots (shard_fold: a topic whose requests
//           meet on one rank, or that makes only one, asks that rank's AB engine once), a
//           stable counting sort of the requests by destination whose scatter packs one chunk
//           per destination (layout first, from the sort's bucket starts and byte prefixes):
//             [u32 n0 n1 n2 0 bytes0 bytes1 bytes2 0][u32 offsets of the n0 slot-0 requests + 1]
//             [slot 1 + 1][slot 2 + 1] pad 16 [slot 0 topic bytes][slot 1][slot 2] pad 16
//   recv    the received chunks (this rank's own read where it was packed) -> three batches
//           (every source's slot-e requests; a slot with one source is matched in place)
//   answer  the three engines' CSRs -> one answer chunk per source:
//             [u32 n0 n1 n2 ids0 ids1 ids2 0 0][per request the end of its ids][ids 0][1][2]
//           (this rank's own chunk without ids: the merge reads them from the CSRs)
//   merge   per request its ids' address and count (at the request's own index), per topic
//           the total, a scan, then in topic order each topic's first request's ids and its
//           second's (engine A then engine B) -> the CSR of the rank's batch in batch order
//
// Engine slots of a rank: 0 = A (space L + root wildcards), 1 = B (space P), 2 = AB (both, one
// table).  A topic's two raw requests (A at rank rA, B at rank rB) become ONE request to slot 2
// when rA == rB — AB holds exactly A_r + B_r, disjoint, so its answer is the two answers'
// union — and a topic with one request (one level, '$', a wildcard name) asks slot 2 of its
// rank as well (no B filter '+/x/...' can match it, and a wildcard name's filter is in AB).
// At world 1 every request is a slot-2 request: one walk per topic over the rank's whole
// table, as replication does; at world G a topic's two requests meet with probability ~1/G.
//
// Per-source / per-destination tables (chunk starts, batch bases) come from the host, which
// holds the exchanged sizes anyway, as one kernel argument (world <= 64).  The fixed-capacity
// form (emqx_shard_step_*_fixed) has no size exchange: chunks sit at agreed capacities, the
// tables are built on the device from the chunks' headers, the engines run fixed-size batches
// (padding topics past the requests) and a flag word, carried in every chunk's header, marks a
// step that did not fit (the caller redoes it with the calls above).  Requests are u32
// indices (2 per topic), so a batch holds fewer than 2^31 topics.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/emqx_match.h"
#include "kernels.h"
#include "layout.h"

namespace emqx {
namespace {

constexpr uint32_t kMaxWorld = EMQX_SHARD_MAX_WORLD;
constexpr uint32_t kNone = 0xFFFFFFFFu;
constexpr uint32_t kE = EMQX_SHARD_ENGINES;  // engine slots per rank: A, B, AB
constexpr uint32_t kHW = 8;                  // header words of a request / answer chunk

struct ShardTab {
  uint64_t chunk[kMaxWorld];       // each source's received chunk (device address; a rank's own
                                   // chunk is read in place where it was packed)
  uint32_t q0[kE][kMaxWorld + 1];  // first slot-e request of each source in the slot-e batch
  uint64_t y0[kE][kMaxWorld + 1];  // first slot-e byte of each source in the slot-e batch
  uint64_t w0[kMaxWorld + 1];      // answer chunks: prefix of (kHW + n0 + n1 + n2) words
};
static_assert(sizeof(ShardTab) <= 3584, "kernel argument");

__host__ __device__ inline uint64_t al16(uint64_t x) { return (x + 15) & ~15ull; }

typedef uint4 __attribute__((aligned(1))) u4u;  // (gfx950 global loads and stores take any alignment)
// One thread's copy of a topic's bytes (any alignment): 16-B moves, then 8 / 4 / 2 / 1.
__host__ __device__ inline void copy_topic(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint32_t len) {
  typedef uint2 __attribute__((aligned(1))) u2u;
  typedef uint32_t __attribute__((aligned(1))) u1u;
  typedef uint16_t __attribute__((aligned(1))) h1u;
  uint32_t j = 0;
  for (; j + 16 <= len; j += 16) *reinterpret_cast<u4u*>(dst + j) = *reinterpret_cast<const u4u*>(src + j);
  if (j + 8 <= len) {
    *reinterpret_cast<u2u*>(dst + j) = *reinterpret_cast<const u2u*>(src + j);
    j += 8;
  }
  if (j + 4 <= len) {
    *reinterpret_cast<u1u*>(dst + j) = *reinterpret_cast<const u1u*>(src + j);
    j += 4;
  }
  if (j + 2 <= len) {
    *reinterpret_cast<h1u*>(dst + j) = *reinterpret_cast<const h1u*>(src + j);
    j += 2;
  }
  if (j < len) dst[j] = src[j];
}

uint32_t grid_of(uint64_t items, uint32_t per_block, uint32_t cap = 8192) {
  return static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>((items + per_block - 1) / per_block, cap)));
}


// A topic's raw requests (r[0]: rank * 2 of engine A, r[1]: rank * 2 + 1 of engine B, or kNone)
// -> its bucket keys (rank * kE + slot; kE * world = none), see the header.
__host__ __device__ inline uint2 shard_fold(const uint32_t (&r)[2], uint32_t world) {
  const uint32_t none = kE * world;
  const bool a = r[0] != kNone, b = r[1] != kNone;
  if (a && b && (r[0] >> 1) != (r[1] >> 1)) return make_uint2(kE * (r[0] >> 1), kE * (r[1] >> 1) + 1);
  if (a || b) return make_uint2(kE * ((a ? r[0] : r[1]) >> 1) + 2, none);
  return make_uint2(none, none);
}

// Destination r's chunk size from the sorted buckets (its requests and bytes per slot).
__host__ __device__ inline uint64_t dest_size(uint32_t r, const uint32_t* start, const uint64_t* bpre, bool* wide) {
  uint64_t ball = 0, nall = 0;
  for (uint32_t e = 0; e < kE; ++e) {
    const uint32_t b = kE * r + e;
    nall += start[b + 1] - start[b];
    ball += bpre[b + 1] - bpre[b];
    *wide |= bpre[b + 1] - bpre[b] > 0xFFFFFFFFull;
  }
  return 4 * kHW + al16(4ull * (nall + kE)) + al16(ball);
}

// Destination r of the send: its meta words, its chunk's header and final offsets, and per
// bucket where the sorted scatter puts its requests (obase[b] + p = the offset word of sorted
// request p, dbase[r] + byte prefix = its bytes); base = the chunk's start, over = the send does
// not fit.  (shard_layout_kernel; the host step's send.)
__host__ __device__ inline void layout_dest(uint32_t r, uint64_t size, uint64_t base, bool over,
                                            const uint32_t* __restrict__ start, const uint64_t* __restrict__ bpre,
                                            uint8_t* __restrict__ send, int64_t* __restrict__ meta,
                                            int64_t* __restrict__ obase, int64_t* __restrict__ dbase) {
  uint32_t nq[kE], nall = 0;
  uint64_t by[kE];
  for (uint32_t e = 0; e < kE; ++e) {
    const uint32_t b = kE * r + e;
    nq[e] = start[b + 1] - start[b];
    by[e] = bpre[b + 1] - bpre[b];
    nall += nq[e];
  }
  int64_t* m = meta + (1 + 2 * kE) * r;
  m[0] = over ? -1 : static_cast<int64_t>(size);
  for (uint32_t e = 0; e < kE; ++e) {
    m[1 + e] = nq[e];
    m[1 + kE + e] = static_cast<int64_t>(by[e]);
  }
  if (over) return;
  uint32_t* h = reinterpret_cast<uint32_t*>(send + base);
  uint32_t o = kHW;
  for (uint32_t e = 0; e < kE; ++e) {
    const uint32_t b = kE * r + e;
    obase[b] = static_cast<int64_t>(base / 4 + o) - static_cast<int64_t>(start[b]);
    h[e] = nq[e];
    h[4 + e] = static_cast<uint32_t>(by[e]);
    o += nq[e];
    h[o++] = static_cast<uint32_t>(by[e]);  // slot e's offsets[n_e]
  }
  h[3] = 0;
  h[7] = 0;
  dbase[r] = static_cast<int64_t>(base + 4 * kHW + al16(4ull * (nall + kE))) - static_cast<int64_t>(bpre[kE * r]);
}

// The fixed-capacity form's chunk of a step that does not fit: no requests, flag bit 1 in header
// word 3 (every receiver's step then carries the flag), slot offsets 0.
__host__ __device__ inline void flagged_chunk(uint8_t* __restrict__ chunk) {
  uint32_t* h = reinterpret_cast<uint32_t*>(chunk);
  for (uint32_t w = 0; w < kHW + kE; ++w) h[w] = w == 3 ? 1u : 0u;
}

// Sorted request `pos` (bucket k < the no-request bucket, byte x among the sorted requests') packed
// where it lands: its offset word and its topic's bytes into its destination's chunk.
__host__ __device__ inline void pack_request(uint8_t* __restrict__ send, uint32_t k, uint32_t pos, uint64_t x,
                                             const int64_t* obase, const uint64_t* bpre, const int64_t* dbase,
                                             const uint8_t* __restrict__ topic, uint32_t len) {
  reinterpret_cast<uint32_t*>(send)[obase[k] + pos] = static_cast<uint32_t>(x - bpre[k]);
  copy_topic(topic, send + (dbase[k / kE] + static_cast<int64_t>(x)), len);
}

// ---- send -------------------------------------------------------------------------------

// Bit k (k < 4) set iff byte k of v is zero (exact: no borrow crosses bytes).
__device__ __forceinline__ uint32_t byte_zero4(uint32_t v) {
  const uint32_t t = ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v) & 0x80808080u;
  return (t * 0x00204081u) >> 28;
}

// shard_topic_levels (layout.h) over the topic's bytes read as 16-B aligned windows (a window
// holding a topic byte lies inside the batch's allocation; the batch's last window only up to
// its end): the same summary, one load per 16 bytes instead of one per byte.  Each window is
// scanned as byte masks: its levels are its '/' bits (the end counts as one), a wildcard level a
// '+' / '#' bit with a '/' (or the topic's start) before it and a '/' (or the end) after it; the
// first three levels' ends are kept, and those levels are hashed a 32-bit word at a time
// (shard_level_hash) — a byte-wise scan of the first three levels made the kernel VALU-bound
// (~3600 VALU instructions a wave, `profiles/r6/`).
__device__ __forceinline__ uint32_t ld_u32_any(const uint8_t* p) {
  typedef uint32_t __attribute__((aligned(1))) u1u;
  return *reinterpret_cast<const u1u*>(p);
}

// shard_level_hash of tb[a, b) (b <= lim, the batch's end): whole words read unaligned, the tail
// word masked (read as a word when 4 bytes from it are inside the batch, else byte by byte).
__device__ __forceinline__ uint32_t level_hash_dev(const uint8_t* __restrict__ tb, uint64_t a, uint64_t b,
                                                   uint64_t lim) {
  uint32_t h = 0x811C9DC5u;
  uint64_t i = a;
  for (; i + 4 <= b; i += 4) h = shard_word_step(h, ld_u32_any(tb + i));
  if (i < b) {
    const uint32_t r = static_cast<uint32_t>(b - i);  // 1..3
    uint32_t w;
    if (i + 4 <= lim) {
      w = ld_u32_any(tb + i) & ((1u << (8u * r)) - 1u);
    } else {
      w = 0;
      for (uint32_t k = 0; k < r; ++k) w |= static_cast<uint32_t>(tb[i + k]) << (8u * k);
    }
    h = shard_word_step(h, w);
  }
  return mix32(h ^ static_cast<uint32_t>(b - a));
}

__device__ __forceinline__ void topic_levels_dev(const uint8_t* __restrict__ tb, uint64_t s, uint64_t e,
                                                 uint64_t lim, ShardTopicLevels* L) {
  // (the windows and the three level ends in named registers: an indexed private array would
  // live in scratch memory; four windows are loaded before any is scanned)
  uint32_t nl = 0;
  uint64_t c0 = e, c1 = e, c2 = e;  // the ends of levels 0, 1, 2
  bool wild = false;
  const uintptr_t abeg = reinterpret_cast<uintptr_t>(tb + s), aend = reinterpret_cast<uintptr_t>(tb + e);
  const uintptr_t alim = reinterpret_cast<uintptr_t>(tb + lim);
  auto window = [&](uintptr_t w0, uint64_t& lo, uint64_t& hi) {
    lo = hi = 0;
    if (w0 > aend) return;
    if (w0 + 16 <= alim) {
      const uint4 v = *reinterpret_cast<const uint4*>(w0);
      lo = (static_cast<uint64_t>(v.y) << 32) | v.x;
      hi = (static_cast<uint64_t>(v.w) << 32) | v.z;
    } else if (w0 < aend) {
      for (uint32_t b = 0; b < 8; ++b) {
        if (w0 + b < alim) lo |= static_cast<uint64_t>(*reinterpret_cast<const uint8_t*>(w0 + b)) << (8u * b);
        if (w0 + 8 + b < alim) hi |= static_cast<uint64_t>(*reinterpret_cast<const uint8_t*>(w0 + 8 + b)) << (8u * b);
      }
    }
  };
  // carry: the byte before the window ends a level (or is the start); pend: that byte is a '+' /
  // '#' that began its level, so a '/' first in this window makes its level a wildcard.
  bool carry = true, pend = false;
  auto masks16 = [&](uintptr_t w0, uint64_t lo, uint64_t hi) {
    const uint32_t i0 = abeg > w0 ? static_cast<uint32_t>(abeg - w0) : 0u;  // < 16
    const uint64_t ie = aend - w0;  // the virtual '/' at the end, if < 16
    const uint32_t real = (ie >= 16 ? 0xFFFFu : ((1u << ie) - 1u)) & ~((1u << i0) - 1u);
    const uint32_t d[4] = {static_cast<uint32_t>(lo), static_cast<uint32_t>(lo >> 32), static_cast<uint32_t>(hi),
                           static_cast<uint32_t>(hi >> 32)};
    uint32_t sl = 0, wc = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      sl |= byte_zero4(d[k] ^ 0x2F2F2F2Fu) << (4 * k);
      wc |= (byte_zero4(d[k] ^ 0x2B2B2B2Bu) | byte_zero4(d[k] ^ 0x23232323u)) << (4 * k);
    }
    uint32_t S = (sl & real) | (ie < 16 ? 1u << ie : 0u);
    const uint32_t P = ((S << 1) | (carry ? 1u : 0u) | (i0 ? 1u << i0 : 0u)) & 0xFFFFu;
    const uint32_t cand = wc & real & P;
    wild |= (cand & (S >> 1)) != 0 || (pend && (S & 1u));
    pend = ((cand >> 15) & 1u) != 0;
    carry = ((S >> 15) & 1u) != 0;
    // the first three level ends (at most three bits of this window matter)
    for (uint32_t k = nl; k < 3 && S; ++k) {
      const uint64_t pos = (w0 - reinterpret_cast<uintptr_t>(tb)) + static_cast<uint32_t>(__builtin_ctz(S));
      c0 = k == 0 ? pos : c0;
      c1 = k == 1 ? pos : c1;
      c2 = k == 2 ? pos : c2;
      S &= S - 1;
    }
    nl += static_cast<uint32_t>(__popc((sl & real) | (ie < 16 ? 1u << ie : 0u)));
  };
  for (uintptr_t w0 = abeg & ~static_cast<uintptr_t>(15); w0 <= aend; w0 += 64) {
    uint64_t l0, g0, l1, g1, l2, g2, l3, g3;
    window(w0, l0, g0);
    window(w0 + 16, l1, g1);
    window(w0 + 32, l2, g2);
    window(w0 + 48, l3, g3);
    masks16(w0, l0, g0);
    if (w0 + 16 <= aend) masks16(w0 + 16, l1, g1);
    if (w0 + 32 <= aend) masks16(w0 + 32, l2, g2);
    if (w0 + 48 <= aend) masks16(w0 + 48, l3, g3);
  }
  L->n_levels = nl;
  L->wild = wild;
  L->h[0] = nl > 0 ? level_hash_dev(tb, s, c0, lim) : 0u;
  L->h[1] = nl > 1 ? level_hash_dev(tb, c0 + 1, c1, lim) : 0u;
  L->h[2] = nl > 2 ? level_hash_dev(tb, c1 + 1, c2, lim) : 0u;
}

// The split plan in LDS when it fits (routing binary-searches it twice per topic: from global
// memory that is ~14 dependent L2 round trips a topic).
constexpr uint32_t kLdsSplits = 2048;
__device__ __forceinline__ const ShardSplitE* stage_splits(const ShardSplitE* sp, uint32_t nsp, ShardSplitE* lds) {
  if (nsp > kLdsSplits) return sp;
  for (uint32_t i = threadIdx.x; i < nsp; i += blockDim.x) lds[i] = sp[i];
  __syncthreads();
  return lds;
}

// ---- the requests sorted by destination: a counting sort over the kE G + 1 buckets -------
// Tiles of kSortTile requests (topics [tile * kSortTile / 2, ...)): the key kernel counts each
// tile's requests and bytes per bucket, one block scans the (bucket, tile) table, and the
// scatter kernel ranks each request inside its tile (stable: wave ballots per key, then the
// waves and rows in order) — the sorted keys, the permutation, each request's byte length and
// its byte offset among the sorted requests, the bucket starts.
constexpr uint32_t kSortTile = 512;  // requests per tile (256 topics: one a thread, so the grid fills the chip)
constexpr uint32_t kMaxBuckets = kE * kMaxWorld + 1;

__device__ __forceinline__ uint32_t lane_id() { return __lane_id(); }

// Adds the wave's requests to the block's per-bucket counts and bytes: one LDS atomic per
// distinct key in the wave (most of a wave's requests share a bucket: same-address atomics from
// every lane would serialise).  Lanes past the batch pass k = kNone.
__device__ __forceinline__ void wave_count(uint32_t k, uint32_t len, uint32_t nb, uint32_t* c_cnt,
                                           uint32_t* c_by) {
  const uint32_t lane = lane_id();
  uint64_t left = __ballot(k != kNone);
  while (left) {
    const uint32_t first = static_cast<uint32_t>(__builtin_ctzll(left));
    const uint32_t kk = __shfl(k, first, 64);
    const uint64_t mask = __ballot(k == kk);
    uint32_t v = k == kk && kk < nb - 1 ? len : 0u;
    for (uint32_t d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
    if (lane == first) {
      atomicAdd(&c_cnt[kk], static_cast<uint32_t>(__popcll(mask)));
      if (v) atomicAdd(&c_by[kk], v);
    }
    left &= ~mask;
  }
}

__global__ __launch_bounds__(256) void shard_key_kernel(const uint8_t* __restrict__ tb,
                                                        const uint64_t* __restrict__ to, uint64_t n, uint32_t world,
                                                        const ShardSplitE* __restrict__ gsp, uint32_t nsp,
                                                        uint32_t* __restrict__ key, uint32_t ntiles,
                                                        uint32_t* __restrict__ tcnt, uint32_t* __restrict__ tbytes,
                                                        uint32_t one) {
  __shared__ ShardSplitE lsp[kLdsSplits];
  __shared__ uint32_t c_cnt[kMaxBuckets];
  __shared__ uint32_t c_by[kMaxBuckets];  // (a tile's bytes: 512 requests of <= 64 KB topics)
  const uint32_t nb = kE * world + 1;
  for (uint32_t k = threadIdx.x; k < nb; k += blockDim.x) {
    c_cnt[k] = 0;
    c_by[k] = 0;
  }
  const ShardSplitE* sp = stage_splits(gsp, nsp, lsp);  // (its barrier covers the clearing)
  const uint64_t lim = n ? to[n] : 0;
  const uint32_t tpt = one ? kSortTile : kSortTile / 2;  // topics a tile
  const uint64_t t0 = static_cast<uint64_t>(blockIdx.x) * tpt;
  const uint64_t t1 = min<uint64_t>(n, t0 + tpt);
  for (uint64_t tr = t0; tr < t1; tr += blockDim.x) {  // block-uniform rows (wave_count is wave-wide)
    const uint64_t t = tr + threadIdx.x;
    if (t >= t1) {
      wave_count(kNone, 0, nb, c_cnt, c_by);
      if (!one) wave_count(kNone, 0, nb, c_cnt, c_by);
      continue;
    }
    const uint64_t a = to[t], b = to[t + 1];
    ShardTopicLevels L;
    topic_levels_dev(tb, a, b, lim, &L);
    uint32_t r[2];
    shard_route_levels(tb + a, b - a, L, world, sp, nsp, r);
    const uint2 k = shard_fold(r, world);
    wave_count(k.x, static_cast<uint32_t>(b - a), nb, c_cnt, c_by);
    if (one) {  // (one request a topic: every request is an AB request, k.y none)
      key[t] = k.x;
      continue;
    }
    *reinterpret_cast<uint2*>(key + 2 * t) = k;
    wave_count(k.y, static_cast<uint32_t>(b - a), nb, c_cnt, c_by);
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < nb; k += blockDim.x) {
    tcnt[static_cast<uint64_t>(k) * ntiles + blockIdx.x] = c_cnt[k];
    tbytes[static_cast<uint64_t>(k) * ntiles + blockIdx.x] = c_by[k];
  }
}

// One block: the (bucket, tile) table -> exclusive prefixes (bucket-major: a bucket's tiles in
// order, then the next bucket): counts in place, bytes into pbytes (u64), start[b] for b = 0 ..
// nb, sc[m] = the byte total.  A thread takes a chunk of consecutive entries (a multiple of 4,
// read as 16-B vectors, every load of a round issued before any is used; the tables are padded
// past the last chunk, the padding masked off).
constexpr uint32_t kScanThreads = 1024;
constexpr uint32_t kOneBlockScan = 8192;  // table entries up to which one block scans it (below: 3 kernels)
__global__ __launch_bounds__(kScanThreads) void shard_sort_scan_kernel(uint32_t* __restrict__ tcnt,
                                                                       const uint32_t* __restrict__ tbytes,
                                                                       uint64_t* __restrict__ pbytes, uint32_t nb,
                                                                       uint32_t ntiles, uint64_t m,
                                                                       uint32_t* __restrict__ start,
                                                                       uint64_t* __restrict__ bpre) {
  __shared__ uint64_t wc[kScanThreads / 64], wb[kScanThreads / 64];
  const uint32_t N = nb * ntiles;
  const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const uint32_t per = ((N + kScanThreads - 1) / kScanThreads + 3) & ~3u;
  const uint32_t i0 = min(N, tid * per), i1 = min(N, i0 + per);
  constexpr uint32_t R = 16;  // entries a round (4 vectors of each table)
  auto load_round = [&](uint32_t g, uint32_t (&vc)[R], uint32_t (&vb)[R]) {
    const uint4* pc = reinterpret_cast<const uint4*>(tcnt + g);
    const uint4* pb = reinterpret_cast<const uint4*>(tbytes + g);
    uint4 c4[R / 4], b4[R / 4];
#pragma unroll
    for (uint32_t q = 0; q < R / 4; ++q) {
      c4[q] = pc[q];
      b4[q] = pb[q];
    }
#pragma unroll
    for (uint32_t q = 0; q < R / 4; ++q) {
      const uint32_t cc[4] = {c4[q].x, c4[q].y, c4[q].z, c4[q].w}, bb[4] = {b4[q].x, b4[q].y, b4[q].z, b4[q].w};
#pragma unroll
      for (uint32_t k = 0; k < 4; ++k) {
        const bool in = g + 4 * q + k < i1;
        vc[4 * q + k] = in ? cc[k] : 0u;
        vb[4 * q + k] = in ? bb[k] : 0u;
      }
    }
  };
  uint64_t c = 0, by = 0;
  for (uint32_t g = i0; g < i1; g += R) {
    uint32_t vc[R], vb[R];
    load_round(g, vc, vb);
#pragma unroll
    for (uint32_t j = 0; j < R; ++j) {
      c += vc[j];
      by += vb[j];
    }
  }
  uint64_t ic = c, ib = by;  // inclusive wave scans
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t xc = __shfl_up(ic, d, 64), xb = __shfl_up(ib, d, 64);
    if (lane >= d) {
      ic += xc;
      ib += xb;
    }
  }
  if (lane == 63) {
    wc[w] = ic;
    wb[w] = ib;
  }
  __syncthreads();
  uint64_t bc = 0, bb = 0;
  for (uint32_t k = 0; k < w; ++k) {
    bc += wc[k];
    bb += wb[k];
  }
  uint64_t xc = bc + ic - c, xb = bb + ib - by;  // exclusive prefix of this thread's chunk
  uint32_t nxt = (i0 + ntiles - 1) / ntiles * ntiles;  // the first bucket start at or after i0
  for (uint32_t g = i0; g < i1; g += R) {
    uint32_t vc[R], vb[R];
    load_round(g, vc, vb);
#pragma unroll
    for (uint32_t j = 0; j < R; ++j) {
      const uint32_t i = g + j;
      if (i >= i1) break;
      if (i == nxt) {  // a bucket's first tile: its first request and first byte
        start[nxt / ntiles] = static_cast<uint32_t>(xc);
        bpre[nxt / ntiles] = xb;
        nxt += ntiles;
      }
      tcnt[i] = static_cast<uint32_t>(xc);
      pbytes[i] = xb;
      xc += vc[j];
      xb += vb[j];
    }
  }
  if (tid == kScanThreads - 1) {
    start[nb] = static_cast<uint32_t>(m);
    bpre[nb] = xb;  // (the no-request bucket is last and holds no bytes)
  }
}

// The same prefixes over many blocks (a table of kE G + 1 buckets x ntiles tiles grows with the
// world: 98 K entries at world 8 for 1 M topics, 166 us in the one-block kernel above): segments of
// kScanSeg entries; per segment its totals, one block scans the segment totals, then each segment
// is scanned from its base.
constexpr uint32_t kScanSeg = 2048;  // table entries per block: 8 per thread
constexpr uint32_t kScanPer = kScanSeg / 256;

// Block-wide exclusive scan of (c, b) pairs over 256 threads; returns this thread's prefixes and
// the block's totals.
__device__ __forceinline__ void block_scan2(uint64_t c, uint64_t b, uint64_t* xc, uint64_t* xb, uint64_t* tc,
                                            uint64_t* tb) {
  __shared__ uint64_t wc[4], wb[4];
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  uint64_t ic = c, ib = b;
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t yc = __shfl_up(ic, d, 64), yb = __shfl_up(ib, d, 64);
    if (lane >= d) {
      ic += yc;
      ib += yb;
    }
  }
  if (lane == 63) {
    wc[w] = ic;
    wb[w] = ib;
  }
  __syncthreads();
  uint64_t bc = 0, bb = 0, ac = 0, ab = 0;
  for (uint32_t k = 0; k < 4; ++k) {
    if (k < w) {
      bc += wc[k];
      bb += wb[k];
    }
    ac += wc[k];
    ab += wb[k];
  }
  *xc = bc + ic - c;
  *xb = bb + ib - b;
  *tc = ac;
  *tb = ab;
}

// A thread's kScanPer consecutive entries from i (16-B loads; entries at or past N read as 0: the
// tables are padded by a segment's worth past the last tile).
__device__ __forceinline__ void load_seg(const uint32_t* __restrict__ tcnt, const uint32_t* __restrict__ tbytes,
                                         uint32_t i, uint32_t N, uint32_t (&vc)[kScanPer], uint32_t (&vb)[kScanPer]) {
  const uint4* pc = reinterpret_cast<const uint4*>(tcnt + i);
  const uint4* pb = reinterpret_cast<const uint4*>(tbytes + i);
#pragma unroll
  for (uint32_t q = 0; q < kScanPer / 4; ++q) {
    const uint4 c4 = pc[q], b4 = pb[q];
    const uint32_t cc[4] = {c4.x, c4.y, c4.z, c4.w}, bb[4] = {b4.x, b4.y, b4.z, b4.w};
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const bool in = i + 4 * q + k < N;
      vc[4 * q + k] = in ? cc[k] : 0u;
      vb[4 * q + k] = in ? bb[k] : 0u;
    }
  }
}

__global__ __launch_bounds__(256) void shard_seg_sums_kernel(const uint32_t* __restrict__ tcnt,
                                                             const uint32_t* __restrict__ tbytes, uint32_t N,
                                                             uint64_t* __restrict__ seg) {
  const uint32_t i = blockIdx.x * kScanSeg + threadIdx.x * kScanPer;
  uint32_t vc[kScanPer], vb[kScanPer];
  uint64_t c = 0, b = 0;
  if (i < N) {
    load_seg(tcnt, tbytes, i, N, vc, vb);
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; ++j) {
      c += vc[j];
      b += vb[j];
    }
  }
  uint64_t xc, xb, tc, tb;
  block_scan2(c, b, &xc, &xb, &tc, &tb);
  if (threadIdx.x == 0) {
    seg[2 * blockIdx.x] = tc;
    seg[2 * blockIdx.x + 1] = tb;
  }
}

// One block: the segment totals -> exclusive prefixes, in place (any number of segments).
__global__ __launch_bounds__(256) void shard_seg_scan_kernel(uint64_t* __restrict__ seg, uint32_t nseg) {
  const uint32_t per = (nseg + 255) / 256;
  const uint32_t s0 = min(nseg, threadIdx.x * per), s1 = min(nseg, s0 + per);
  uint64_t c = 0, b = 0;
  for (uint32_t k = s0; k < s1; ++k) {
    c += seg[2 * k];
    b += seg[2 * k + 1];
  }
  uint64_t xc, xb, tc, tb;
  block_scan2(c, b, &xc, &xb, &tc, &tb);
  for (uint32_t k = s0; k < s1; ++k) {
    const uint64_t vc = seg[2 * k], vb = seg[2 * k + 1];
    seg[2 * k] = xc;
    seg[2 * k + 1] = xb;
    xc += vc;
    xb += vb;
  }
}

// Each segment from its base: counts in place, byte prefixes into pbytes, the bucket starts at
// every multiple of ntiles, and (block of entry N - 1) start[nb] = m, bpre[nb] = the byte total.
__global__ __launch_bounds__(256) void shard_seg_final_kernel(uint32_t* __restrict__ tcnt,
                                                              const uint32_t* __restrict__ tbytes,
                                                              uint64_t* __restrict__ pbytes, uint32_t N,
                                                              uint32_t ntiles, uint32_t nb, uint64_t m,
                                                              const uint64_t* __restrict__ seg,
                                                              uint32_t* __restrict__ start,
                                                              uint64_t* __restrict__ bpre) {
  const uint32_t i = blockIdx.x * kScanSeg + threadIdx.x * kScanPer;
  uint32_t vc[kScanPer], vb[kScanPer];
  uint64_t c = 0, b = 0;
  if (i < N) {
    load_seg(tcnt, tbytes, i, N, vc, vb);
#pragma unroll
    for (uint32_t j = 0; j < kScanPer; ++j) {
      c += vc[j];
      b += vb[j];
    }
  }
  uint64_t xc, xb, tc, tb;
  block_scan2(c, b, &xc, &xb, &tc, &tb);
  xc += seg[2 * blockIdx.x];
  xb += seg[2 * blockIdx.x + 1];
  if (i >= N) return;
#pragma unroll
  for (uint32_t j = 0; j < kScanPer; ++j) {
    const uint32_t e = i + j;
    if (e >= N) break;
    if (e % ntiles == 0) {  // a bucket's first tile: its first request and first byte
      start[e / ntiles] = static_cast<uint32_t>(xc);
      bpre[e / ntiles] = xb;
    }
    tcnt[e] = static_cast<uint32_t>(xc);
    pbytes[e] = xb;
    xc += vc[j];
    xb += vb[j];
    if (e == N - 1) {
      start[nb] = static_cast<uint32_t>(m);
      bpre[nb] = xb;  // (the no-request bucket is last and holds no bytes)
    }
  }
}

// Stable scatter of one tile's requests to their sorted positions (see above).
// ... and each request packed where it lands (shard_layout_kernel's bases): its offset word and
// its topic's bytes into its destination's chunk.
__global__ __launch_bounds__(256) void shard_sort_scatter_kernel(const uint32_t* __restrict__ key,
                                                                 const uint8_t* __restrict__ tb,
                                                                 const uint64_t* __restrict__ to, uint64_t m,
                                                                 uint32_t nb, uint32_t ntiles,
                                                                 const uint32_t* __restrict__ tcnt,
                                                                 const uint64_t* __restrict__ tbytes,  // (prefixes)
                                                                 const uint64_t* __restrict__ bpre,
                                                                 const int64_t* __restrict__ obase,
                                                                 const int64_t* __restrict__ dbase,
                                                                 const uint32_t* __restrict__ err,
                                                                 uint8_t* __restrict__ send,
                                                                 uint32_t* __restrict__ key_s, uint32_t* __restrict__ perm,
                                                                 uint32_t one, uint32_t* __restrict__ tpos) {
  __shared__ uint32_t run_c[kMaxBuckets];
  __shared__ uint64_t run_b[kMaxBuckets];
  __shared__ uint32_t w_c[4][kMaxBuckets];
  __shared__ uint64_t w_b[4][kMaxBuckets];
  __shared__ int64_t s_ob[kMaxBuckets], s_db[kMaxWorld];
  __shared__ uint64_t s_bp[kMaxBuckets];
  __shared__ uint64_t cp_src[256], cp_dst[256];  // the row's topic copies, made by 4 lanes each
  __shared__ uint32_t cp_len[256];
  const uint32_t tid = threadIdx.x, lane = lane_id(), w = tid >> 6;
  const bool pack = err[0] == 0;
  const uint32_t world = (nb - 1) / kE;
  for (uint32_t k = tid; k < nb - 1; k += 256) {
    s_ob[k] = obase[k];
    s_bp[k] = bpre[k];
  }
  for (uint32_t r = tid; r < world; r += 256) s_db[r] = dbase[r];
  for (uint32_t k = tid; k < nb; k += 256) {
    run_c[k] = tcnt[static_cast<uint64_t>(k) * ntiles + blockIdx.x];
    run_b[k] = tbytes[static_cast<uint64_t>(k) * ntiles + blockIdx.x];
    for (uint32_t j = 0; j < 4; ++j) {
      w_c[j][k] = 0;
      w_b[j][k] = 0;
    }
  }
  __syncthreads();
  const uint64_t p0 = static_cast<uint64_t>(blockIdx.x) * kSortTile;
  const uint64_t p1 = min<uint64_t>(m, p0 + kSortTile);
  for (uint64_t row = p0; row < p1; row += 256) {  // block-uniform
    const uint64_t p = row + tid;
    const bool ok = p < p1;
    const uint32_t k = ok ? key[p] : 0xFFFFFFFFu;
    uint32_t l = 0;
    uint64_t a = 0;
    if (ok && k < nb - 1) {
      const uint64_t t = one ? p : p >> 1;
      a = to[t];
      l = static_cast<uint32_t>(to[t + 1] - a);
    }
    // rank among the wave's lanes with the same key, and the wave's totals per key
    uint32_t rc = 0;
    uint64_t rb = 0;
    uint64_t left = __ballot(ok);
    while (left) {
      const uint32_t first = static_cast<uint32_t>(__builtin_ctzll(left));
      const uint32_t kk = __shfl(k, first, 64);
      const uint64_t mask = __ballot(ok && k == kk);
      const bool mine = ok && k == kk;
      const uint64_t below = mask & ((1ull << lane) - 1ull);
      // byte prefix among the key's lanes (inclusive scan of l on those lanes)
      uint64_t v = mine ? l : 0, incl = v;
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint64_t x = __shfl_up(incl, d, 64);
        if (lane >= d) incl += x;
      }
      if (mine) {
        rc = static_cast<uint32_t>(__popcll(below));
        rb = incl - v;
      }
      const uint64_t tot = __shfl(incl, 63, 64);
      if (lane == first) {
        w_c[w][kk] = static_cast<uint32_t>(__popcll(mask));
        w_b[w][kk] = tot;
      }
      left &= ~mask;
    }
    __syncthreads();
    if (ok) {
      uint32_t pc = run_c[k];
      uint64_t pb = run_b[k];
      for (uint32_t j = 0; j < w; ++j) {
        pc += w_c[j][k];
        pb += w_b[j][k];
      }
      const uint32_t pos = pc + rc;
      key_s[pos] = k;
      perm[pos] = static_cast<uint32_t>(p);
      if (one) tpos[p] = pos;  // (request p = topic p)
      if (pack && k < nb - 1) {  // pack_request's offset word here, its bytes below
        const uint64_t x = pb + rb;
        reinterpret_cast<uint32_t*>(send)[s_ob[k] + pos] = static_cast<uint32_t>(x - s_bp[k]);
        cp_src[tid] = a;
        cp_dst[tid] = static_cast<uint64_t>(s_db[k / kE] + static_cast<int64_t>(x));
      }
    }
    cp_len[tid] = ok && pack && k < nb - 1 ? l : 0u;
    __syncthreads();
    // the row's topic bytes, 4 lanes a request (16-B moves side by side: a wave's loads cover 16
    // topics' consecutive bytes instead of 64 lanes' strided 16-B pieces)
    for (uint32_t r = tid >> 2; r < 256; r += 64) {
      const uint32_t len = cp_len[r];
      if (!len) continue;
      const uint8_t* src = tb + cp_src[r];
      uint8_t* dst = send + cp_dst[r];
      for (uint32_t j = 16 * (tid & 3u); j < len; j += 64) {
        if (j + 16 <= len) *reinterpret_cast<u4u*>(dst + j) = *reinterpret_cast<const u4u*>(src + j);
        else copy_topic(src + j, dst + j, len - j);
      }
    }
    for (uint32_t kk = tid; kk < nb; kk += 256) {
      uint32_t c = 0;
      uint64_t b = 0;
      for (uint32_t j = 0; j < 4; ++j) {
        c += w_c[j][kk];
        b += w_b[j][kk];
        w_c[j][kk] = 0;
        w_b[j][kk] = 0;
      }
      run_c[kk] += c;
      run_b[kk] += b;
    }
    __syncthreads();
  }
}

// One block: per destination rank the chunk's sizes, start, header and final offsets, and per
// bucket where the sorted scatter puts its requests (pack fused into shard_sort_scatter_kernel).
__global__ __launch_bounds__(64) void shard_layout_kernel(const uint32_t* __restrict__ start,
                                                          const uint64_t* __restrict__ bpre, uint32_t world,
                                                          uint8_t* __restrict__ send, uint64_t cap,
                                                          int64_t* __restrict__ meta, uint64_t* __restrict__ cbase,
                                                          int64_t* __restrict__ obase, int64_t* __restrict__ dbase,
                                                          uint32_t* __restrict__ err, uint64_t fixed,
                                                          uint32_t* __restrict__ flagw) {
  __shared__ uint64_t sz[kMaxWorld];
  __shared__ uint32_t wide_any;
  const uint32_t r = threadIdx.x;
  if (r == 0) wide_any = 0;
  __syncthreads();
  bool wide = false;
  if (r < world) {
    sz[r] = dest_size(r, start, bpre, &wide);
    if (wide || (fixed && sz[r] > fixed)) atomicOr(&wide_any, 1u);
  }
  __syncthreads();
  if (r >= world) return;
  uint64_t base = 0, total = 0;
  for (uint32_t j = 0; j < r; ++j) base += sz[j];
  for (uint32_t j = 0; j < world; ++j) total += sz[j];
  if (fixed) base = fixed * r;  // (fixed capacities: chunk r at r * fixed; over = one does not fit)
  cbase[r] = base;
  const bool over = (!fixed && total > cap) || wide_any;
  layout_dest(r, sz[r], base, over, start, bpre, send, meta, obase, dbase);
  if (fixed && over) flagged_chunk(send + base);
  if (r == 0) {
    err[0] = over ? 1u : 0u;
    if (flagw) flagw[0] = over ? 1u : 0u;  // (the step's flag word starts here)
  }
}
// emqx_shard_route_device: the raw requests (req2[2t], req2[2t + 1]) with the same scanner.
__global__ __launch_bounds__(256) void shard_route_kernel(const uint8_t* __restrict__ tb,
                                                          const uint64_t* __restrict__ to, uint64_t n, uint32_t world,
                                                          const ShardSplitE* __restrict__ gsp, uint32_t nsp,
                                                          uint32_t* __restrict__ req2) {
  __shared__ ShardSplitE lsp[kLdsSplits];
  const ShardSplitE* sp = stage_splits(gsp, nsp, lsp);
  const uint64_t lim = n ? to[n] : 0;
  for (uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < n;
       t += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint64_t a = to[t], b = to[t + 1];
    ShardTopicLevels L;
    topic_levels_dev(tb, a, b, lim, &L);
    uint32_t r[2];
    shard_route_levels(tb + a, b - a, L, world, sp, nsp, r);
    req2[2 * t] = r[0];
    req2[2 * t + 1] = r[1];
  }
}

// ---- recv -------------------------------------------------------------------------------

// Words before slot e's offsets in a request chunk with slot sizes n[]: the header, then each
// earlier slot's n + 1 offsets.
__host__ __device__ inline uint32_t offs_words(const uint32_t* n, uint32_t e) {
  uint32_t w = kHW;
  for (uint32_t k = 0; k < e; ++k) w += n[k] + 1;
  return w;
}

// grid (x, source, slot): the source's offsets rebased into the slot's batch, and its bytes (one
// contiguous region per (source, slot) on both sides) moved into the slot's byte buffer — one
// launch for every source, where one copy-engine call per source cost ~5 us each.  A slot read in
// place (one source: bytes.p[e] null) moves no bytes.
struct SlotOffsets {
  uint64_t* p[kE];
};
struct SlotBytes {
  uint8_t* p[kE];
  uint32_t rel;  // (fixed form, world 1: every slot matched in place, offsets from the chunk's start)
};

// (source s, slot e) of the recv: items tid, tid + stride, ... (the kernel's grid-stride; the host
// step's loop: 0, 1).
__host__ __device__ inline void unpack_part(const ShardTab& tab, const SlotOffsets& dst_off, const SlotBytes& dst_bytes,
                                            uint32_t s, uint32_t e, uint64_t tid, uint64_t stride) {
  uint32_t nq[kE], nall = 0;
  uint64_t before = 0;  // this source's bytes of the slots before e
  for (uint32_t k = 0; k < kE; ++k) {
    nq[k] = tab.q0[k][s + 1] - tab.q0[k][s];
    nall += nq[k];
    before += k < e ? tab.y0[k][s + 1] - tab.y0[k][s] : 0;
  }
  const uint32_t* offs = reinterpret_cast<const uint32_t*>(tab.chunk[s]) + offs_words(nq, e);
  const uint32_t n = nq[e];
  const uint64_t dbase = dst_bytes.rel ? 4 * kHW + al16(4ull * (nall + kE)) + before : tab.y0[e][s];
  uint64_t* doff = dst_off.p[e] + tab.q0[e][s];
  for (uint64_t k = tid; k <= n; k += stride) doff[k] = dbase + offs[k];
  if (!dst_bytes.p[e]) return;
  const uint64_t by = tab.y0[e][s + 1] - dbase;
  const uint8_t* src = reinterpret_cast<const uint8_t*>(tab.chunk[s]) + 4 * kHW + al16(4ull * (nall + kE)) + before;
  uint8_t* dst = dst_bytes.p[e] + dbase;
  for (uint64_t j = 16 * tid; j + 16 <= by; j += 16 * stride)
    *reinterpret_cast<u4u*>(dst + j) = *reinterpret_cast<const u4u*>(src + j);
  const uint64_t tail = by & ~15ull;
  for (uint64_t j = tail + tid; j < by; j += stride) dst[j] = src[j];
}

__global__ __launch_bounds__(256) void shard_unpack_kernel(ShardTab tab, SlotOffsets dst_off, SlotBytes dst_bytes) {
  unpack_part(tab, dst_off, dst_bytes, blockIdx.y, blockIdx.z, static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x,
              static_cast<uint64_t>(gridDim.x) * blockDim.x);
}

// ---- the fixed-capacity form's tables ---------------------------------------------------------

// Per-slot capacities of the fixed form (requests, bytes) and the padding offset of each slot.
struct SlotCaps {
  uint64_t q[kE], y[kE];
};

// The recv table from the received chunks' headers (the host mode's and one device thread's
// body): per source its slot counts and bytes, prefixes over sources; a flagged chunk, or a slot
// over its capacity, flags the step and empties every slot batch.  pad[e]: slot e's offset after
// its last request (the engines' padding topics are empty topics there).
// (hdr[r]: where chunk r's header words are read — the chunk itself, or a copy in LDS)
__host__ __device__ inline void recv_table(const uint64_t* chunk, const uint64_t* hdr, uint32_t G, const SlotCaps& cap,
                                           bool rel, ShardTab* t, uint64_t* pad, uint32_t* flagw) {
  uint32_t f = flagw[0];
  for (uint32_t r = 0; r < G; ++r) f |= reinterpret_cast<const uint32_t*>(hdr[r])[3];
  for (int pass = 0; pass < 2; ++pass) {
    const bool empty = f != 0;
    uint64_t words = 0;
    for (uint32_t e = 0; e < kE; ++e) {
      t->q0[e][0] = 0;
      t->y0[e][0] = 0;
    }
    for (uint32_t r = 0; r < G; ++r) {
      const uint32_t* h = reinterpret_cast<const uint32_t*>(hdr[r]);
      t->chunk[r] = chunk[r];
      uint64_t nall = 0;
      for (uint32_t e = 0; e < kE; ++e) {
        const uint32_t nq = empty ? 0u : h[e];
        t->q0[e][r + 1] = t->q0[e][r] + nq;
        t->y0[e][r + 1] = t->y0[e][r] + (empty ? 0u : h[4 + e]);
        nall += nq;
      }
      t->w0[r] = words;
      words += kHW + nall;
    }
    t->w0[G] = words;
    for (uint32_t e = 0; e < kE; ++e)
      if (t->q0[e][G] > cap.q[e] || (!rel && t->y0[e][G] > cap.y[e])) f |= 2u;
    if (!f || empty) break;  // (over a capacity: again, every batch empty)
  }
  uint64_t nall0 = 0, y = 0;
  for (uint32_t e = 0; e < kE; ++e) nall0 += t->q0[e][1];
  for (uint32_t e = 0; e < kE; ++e) {
    y += t->y0[e][G];
    pad[e] = rel ? 4 * kHW + al16(4ull * (nall0 + kE)) + y : t->y0[e][G];
  }
  flagw[0] = f;
}

// Slot e's offsets from its request count to its capacity = pad[e] (the recv kernel's padding blocks).
__host__ __device__ inline void pad_slot(const ShardTab& tab, uint32_t G, const SlotOffsets& dst_off, const SlotCaps& cap,
                                         const uint64_t* pad, uint32_t e, uint64_t tid, uint64_t stride) {
  for (uint64_t k = tab.q0[e][G] + tid; k <= cap.q[e]; k += stride) dst_off.p[e][k] = pad[e];
}

// The fixed form's recv in ONE launch (the table, the unpack and the padding were three, each a
// few microseconds of latency on the path to the walk): every block builds the recv table from
// the chunk headers in LDS (the same table in each; block (0, 0, 0) publishes it and the
// padding offsets for the later kernels), then grid (x, source or G = padding, slot) does its
// part.
__global__ __launch_bounds__(256) void shard_recv_fixed_kernel(ShardTab chunks, uint32_t G, SlotCaps cap, uint32_t rel,
                                                               SlotOffsets dst_off, SlotBytes dst_bytes,
                                                               ShardTab* __restrict__ t_out, uint64_t* __restrict__ pad_out,
                                                               uint32_t* __restrict__ flagw) {
  __shared__ ShardTab t;
  __shared__ uint64_t pad[kE];
  __shared__ uint32_t f[1];
  __shared__ uint4 hw[kMaxWorld][2];  // every chunk's header, loaded in parallel
  __shared__ uint64_t hp[kMaxWorld];
  if (threadIdx.x < G) {
    const uint4* h = reinterpret_cast<const uint4*>(chunks.chunk[threadIdx.x]);
    hw[threadIdx.x][0] = h[0];
    hw[threadIdx.x][1] = h[1];
    hp[threadIdx.x] = reinterpret_cast<uint64_t>(&hw[threadIdx.x][0]);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    f[0] = flagw[0];
    recv_table(chunks.chunk, hp, G, cap, rel != 0, &t, pad, f);
  }
  __syncthreads();
  const bool first = blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0;
  if (first) {
    const uint32_t* src = reinterpret_cast<const uint32_t*>(&t);
    uint32_t* dst = reinterpret_cast<uint32_t*>(t_out);
    for (uint32_t w = threadIdx.x; w < sizeof(ShardTab) / 4; w += blockDim.x) dst[w] = src[w];
    if (threadIdx.x < kE) pad_out[threadIdx.x] = pad[threadIdx.x];
    if (threadIdx.x == 0) flagw[0] = f[0];
  }
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  if (blockIdx.y == G) {
    pad_slot(t, G, dst_off, cap, pad, blockIdx.z, tid, stride);
  } else if (!f[0]) {
    unpack_part(t, dst_off, dst_bytes, blockIdx.y, blockIdx.z, tid, stride);
  }
}

// ---- answer -----------------------------------------------------------------------------

struct EngineCsrs {
  const uint64_t* off[kE];
  const uint32_t* ids[kE];
  const uint64_t* sum[kE];  // emqx_match_batch_device_async summaries, or null
};

// grid (x, source): the source's answer chunk from the three CSRs.  An engine call that did not
// complete (summary flags) leaves its ids unread: the step is redone.  The chunk for this rank
// itself (source `self`) carries no ids: the merge reads them in place from the CSRs.
constexpr uint32_t kAnsMeta = 3;  // per source: chunk words, redo flag, ids
// Source s of G: items tid, tid + stride, ... (meta: this item writes the source's meta words).
// fixed > 0 (the fixed form): chunk s at s * fixed words, no meta; `flag` set: the chunk is a
// header only, flag in word 7.
__host__ __device__ inline void answer_source(const EngineCsrs& cs, const ShardTab& tab, uint32_t self,
                                              uint32_t* __restrict__ out, int64_t* __restrict__ ans_meta, uint32_t s,
                                              uint32_t G, uint64_t tid, uint64_t stride, bool meta, uint64_t fixed = 0,
                                              uint32_t flag = 0) {
  if (fixed && flag) {
    for (uint64_t w = tid; w < kHW; w += stride) out[fixed * s + w] = w == 7 ? flag : 0u;
    return;
  }
  bool bad = false;
  uint32_t q0[kE], nq[kE];
  uint64_t i0[kE], ni[kE], nall = 0, iall = 0, ibefore = 0;
  for (uint32_t e = 0; e < kE; ++e) {
    bad |= cs.sum[e] && cs.sum[e][0];
    q0[e] = tab.q0[e][s];
    nq[e] = tab.q0[e][s + 1] - q0[e];
    nall += nq[e];
  }
  for (uint32_t e = 0; e < kE; ++e) {
    i0[e] = tab.q0[e][G] ? cs.off[e][q0[e]] : 0;  // (a slot no source asked: never read)
    ni[e] = bad || !nq[e] ? 0 : cs.off[e][q0[e] + nq[e]] - i0[e];
    iall += ni[e];
    ibefore += bad ? 0 : i0[e];  // this source's ids start after every earlier source's
  }
  if (!bad && self < s)  // the own chunk before this one holds no ids
    for (uint32_t e = 0; e < kE; ++e) {
      const uint32_t a0 = tab.q0[e][self], a1 = tab.q0[e][self + 1];
      if (a1 > a0) ibefore -= cs.off[e][a1] - cs.off[e][a0];
    }
  const uint64_t cb = fixed ? fixed * s : tab.w0[s] + ibefore;
  if (meta && !fixed) {
    ans_meta[kAnsMeta * s] = static_cast<int64_t>(kHW + nall + (s == self ? 0 : iall));
    ans_meta[kAnsMeta * s + 1] = bad ? 1 : 0;
    ans_meta[kAnsMeta * s + 2] = static_cast<int64_t>(iall);
  }
  if (bad) return;
  const bool copy_ids = s != self;
  uint32_t* c = out + cb;
  for (uint64_t w = tid; w < kHW; w += stride) {
    uint32_t v = 0;
    if (w < kE) v = nq[w];
    else if (w >= 3 && w < 3 + kE) v = static_cast<uint32_t>(ni[w - 3]);
    c[w] = v;
  }
  // per request the END of its ids within the chunk's id region (the merge reads begin and end
  // without a scan), then the ids
  uint32_t* end = c + kHW;
  uint32_t* ids = c + kHW + nall;
  uint64_t before = 0;
  for (uint32_t e = 0; e < kE; ++e) {
    const uint64_t* off = cs.off[e] + q0[e];
    for (uint64_t k = tid; k < nq[e]; k += stride) end[k] = static_cast<uint32_t>(before + off[k + 1] - i0[e]);
    const uint32_t* src = cs.ids[e] + i0[e];
    if (copy_ids) {  // 16-B moves (any 4-B alignment), then the last < 4 ids
      for (uint64_t j = 4 * tid; j + 4 <= ni[e]; j += 4 * stride)
        *reinterpret_cast<u4u*>(ids + j) = *reinterpret_cast<const u4u*>(src + j);
      const uint64_t r = ni[e] & ~3ull;
      for (uint64_t j = r + tid; j < ni[e]; j += stride) ids[j] = src[j];
    }
    end += nq[e];
    ids += ni[e];
    before += ni[e];
  }
}

__global__ __launch_bounds__(256) void shard_answer_kernel(EngineCsrs cs, ShardTab tab, uint32_t self,
                                                           uint32_t* __restrict__ out, int64_t* __restrict__ ans_meta) {
  answer_source(cs, tab, self, out, ans_meta, blockIdx.y, gridDim.y,
                static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x, static_cast<uint64_t>(gridDim.x) * blockDim.x,
                blockIdx.x == 0 && threadIdx.x == 0);
}

// The fixed form's answer plan (one thread): an engine call that did not complete, or an answer
// chunk over `fixed` words, flags the step — decided for every chunk before any is written, so
// each destination gets the same flag.
__host__ __device__ inline void answer_plan(const EngineCsrs& cs, const ShardTab& tab, uint32_t self, uint32_t G,
                                            uint64_t fixed, uint32_t* flagw) {
  uint32_t f = flagw[0];
  for (uint32_t e = 0; e < kE; ++e)
    if (cs.sum[e] && cs.sum[e][0]) f |= 4u;
  if (!f)
    for (uint32_t s = 0; s < G; ++s) {
      uint64_t nall = 0, iall = 0;
      for (uint32_t e = 0; e < kE; ++e) {
        const uint32_t q0 = tab.q0[e][s], nq = tab.q0[e][s + 1] - q0;
        nall += nq;
        if (nq) iall += cs.off[e][q0 + nq] - cs.off[e][q0];
      }
      if (kHW + nall + (s == self ? 0 : iall) > fixed) f |= 8u;
    }
  flagw[0] = f;
}

// The plan and the chunks in one launch: every block makes the (deterministic) plan itself,
// block (0, 0) publishes the flag.
__global__ __launch_bounds__(256) void shard_answer_fixed_kernel(EngineCsrs cs, const ShardTab* __restrict__ tab,
                                                                 uint32_t self, uint32_t* __restrict__ out,
                                                                 uint64_t fixed, uint32_t* __restrict__ flagw) {
  // (answer_plan with its G x kE terms computed by as many threads)
  __shared__ uint32_t f[1];
  __shared__ unsigned long long a_n[kMaxWorld], a_i[kMaxWorld];
  const uint32_t G = gridDim.y, j = threadIdx.x;
  if (j < G) a_n[j] = a_i[j] = 0;
  if (j == 0) f[0] = flagw[0];
  __syncthreads();
  if (j < G * kE) {
    const uint32_t sj = j / kE, e = j - kE * sj;
    const uint32_t q0 = tab->q0[e][sj], nq = tab->q0[e][sj + 1] - q0;
    if (nq) {
      atomicAdd(&a_n[sj], static_cast<unsigned long long>(nq));
      atomicAdd(&a_i[sj], static_cast<unsigned long long>(cs.off[e][q0 + nq] - cs.off[e][q0]));
    }
  }
  if (j < kE && cs.sum[j] && cs.sum[j][0]) atomicOr(&f[0], 4u);
  __syncthreads();
  if (j == 0 && !f[0])
    for (uint32_t sj = 0; sj < G; ++sj)
      if (kHW + a_n[sj] + (sj == self ? 0 : a_i[sj]) > fixed) f[0] |= 8u;
  __syncthreads();
  if (blockIdx.x == 0 && blockIdx.y == 0 && j == 0) flagw[0] = f[0];
  answer_source(cs, *tab, self, out, nullptr, blockIdx.y, gridDim.y,
                static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x, static_cast<uint64_t>(gridDim.x) * blockDim.x,
                false, fixed, f[0]);
}

// ---- merge ------------------------------------------------------------------------------

// This rank's own answers, read in place: per slot its engine's ids from the first id of this
// rank's own requests (self = kNone: every answer came in a chunk).
struct SelfIds {
  const uint32_t* ids[kE];
  const uint64_t* off[kE];
  uint32_t q0[kE];
  uint32_t self;
  const ShardTab* rtab;     // (fixed form: q0 from the recv table on the device)
  const uint32_t* flagw;    // (fixed form: the step's flag; set = no answer is read)
};

// Per sorted request p: where its answer's ids are (an answer chunk's id region, or this rank's
// own engine output) and how many, stored at the request's own index perm[p] (2t: a topic's
// first request, 2t + 1 its second) — the merge then reads them per topic, coalesced.  With one
// request a topic (`one`: perm[p] = the topic) it goes to 2t and 2t + 1 says none.
// Sorted request p's answer: its ids' count and where they are.
__host__ __device__ inline uint32_t request_answer(const ShardTab& tab, const SelfIds& me,
                                                   const uint32_t* __restrict__ key_s,
                                                   const uint32_t* __restrict__ start, uint64_t p, uint64_t* src_out) {
  const uint32_t b = key_s[p], r = b / kE, e = b - kE * r;
  const uint32_t* ch = reinterpret_cast<const uint32_t*>(tab.chunk[r]);
  uint32_t before = 0, ibefore = 0;  // the chunk's requests / ids of the earlier slots
  for (uint32_t k = 0; k < e; ++k) {
    before += ch[k];
    ibefore += ch[3 + k];
  }
  const uint32_t k = before + (p - start[b]);
  const uint32_t b0 = k ? ch[kHW + k - 1] : 0u;
  const uint32_t q0 = me.rtab ? me.rtab->q0[e][me.self] : me.q0[e];
  const uint32_t* src = r == me.self ? me.ids[e] + me.off[e][q0] + (b0 - ibefore)
                                     : ch + kHW + ch[0] + ch[1] + ch[2] + b0;
  *src_out = reinterpret_cast<uint64_t>(src);
  return ch[kHW + k] - b0;
}

// One request a topic, in topic order: topic t's request sits at sorted position tpos[t]; its
// count and address go to the topic's pair (2t; 2t + 1 says none) and its total straight to
// tcnt — coalesced writes, and no separate topic-count pass.
__host__ __device__ inline void gather_topic(const ShardTab& tab, const SelfIds& me, const uint32_t* __restrict__ key_s,
                                             const uint32_t* __restrict__ tpos, const uint32_t* __restrict__ start,
                                             uint32_t nreq, uint64_t t, uint32_t* __restrict__ rq_cnt,
                                             uint64_t* __restrict__ rq_src, uint32_t* __restrict__ tcnt) {
  const uint32_t p = tpos[t];
  uint64_t src = 0;
  const bool none = p >= nreq || (me.flagw && me.flagw[0]);
  const uint32_t c = none ? 0u : request_answer(tab, me, key_s, start, p, &src);
  *reinterpret_cast<uint2*>(rq_cnt + 2 * t) = make_uint2(c, 0u);
  rq_src[2 * t] = src;
  tcnt[t] = c;
}

__host__ __device__ inline void gather_request(const ShardTab& tab, const SelfIds& me, const uint32_t* __restrict__ key_s,
                                               const uint32_t* __restrict__ perm, const uint32_t* __restrict__ start,
                                               uint32_t nreq, uint64_t p, uint32_t* __restrict__ rq_cnt,
                                               uint64_t* __restrict__ rq_src, uint32_t one) {
  {
    const uint32_t q = one ? 2 * perm[p] : perm[p];
    if (one) rq_cnt[q + 1] = 0;
    if (p >= nreq || (me.flagw && me.flagw[0])) {
      rq_cnt[q] = 0;
      return;
    }
    uint64_t src = 0;
    rq_cnt[q] = request_answer(tab, me, key_s, start, p, &src);
    rq_src[q] = src;
  }
}

__global__ __launch_bounds__(256) void shard_gather_kernel(ShardTab tab, SelfIds me,
                                                           const uint32_t* __restrict__ key_s,
                                                           const uint32_t* __restrict__ perm,
                                                           const uint32_t* __restrict__ start, uint64_t m,
                                                           uint32_t world, uint32_t* __restrict__ rq_cnt,
                                                           uint64_t* __restrict__ rq_src, uint32_t one) {
  const uint32_t nreq = start[kE * world];
  for (uint64_t p = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; p < m;
       p += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    gather_request(tab, me, key_s, perm, start, nreq, p, rq_cnt, rq_src, one);
}

__global__ __launch_bounds__(256) void shard_gather_topic_kernel(ShardTab tab, SelfIds me,
                                                                 const uint32_t* __restrict__ key_s,
                                                                 const uint32_t* __restrict__ tpos,
                                                                 const uint32_t* __restrict__ start, uint64_t n,
                                                                 uint32_t world, uint32_t* __restrict__ rq_cnt,
                                                                 uint64_t* __restrict__ rq_src, uint32_t* __restrict__ tcnt) {
  const uint32_t nreq = start[kE * world];
  for (uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < n;
       t += static_cast<uint64_t>(gridDim.x) * blockDim.x)
    gather_topic(tab, me, key_s, tpos, start, nreq, t, rq_cnt, rq_src, tcnt);
}

__global__ __launch_bounds__(256) void shard_topic_counts_kernel(const uint32_t* __restrict__ rq_cnt, uint64_t n,
                                                                 uint32_t* __restrict__ tcnt) {
  for (uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < n;
       t += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint2 c = *reinterpret_cast<const uint2*>(rq_cnt + 2 * t);
    tcnt[t] = c.x + c.y;
  }
}

// The fixed form's merge plan (one thread): the step's flag ORed with every answer chunk's (word
// 7), the same on every rank; copied to `out` (the caller's mapped word) as well.
__host__ __device__ inline void merge_plan(const uint64_t* chunk, uint32_t G, uint32_t* flagw, uint32_t* out) {
  uint32_t f = flagw[0];
  for (uint32_t r = 0; r < G; ++r) f |= reinterpret_cast<const uint32_t*>(chunk[r])[7];
  flagw[0] = f;
  if (out) out[0] = f;
}

__global__ __launch_bounds__(64) void shard_merge_plan_kernel(ShardTab t, uint32_t G, uint32_t* __restrict__ flagw,
                                                              uint32_t* __restrict__ out) {
  __shared__ uint32_t f[1];  // (merge_plan, the chunks' words read by G threads at once)
  if (threadIdx.x == 0) f[0] = flagw[0];
  __syncthreads();
  if (threadIdx.x < G) atomicOr(&f[0], reinterpret_cast<const uint32_t*>(t.chunk[threadIdx.x])[7]);
  __syncthreads();
  if (threadIdx.x == 0) {
    flagw[0] = f[0];
    if (out) out[0] = f[0];
  }
}

// c ids from src to dst by the 4 lanes `sub` of a quad: 16-B moves (4 ids a lane, any 4-B
// alignment), the last < 4 ids one by one.
__host__ __device__ inline void quad_copy_ids(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t c,
                                              uint32_t sub) {
  uint32_t j = 4 * sub;
  for (; j + 4 <= c; j += 16) *reinterpret_cast<u4u*>(dst + j) = *reinterpret_cast<const u4u*>(src + j);
  const uint32_t r = c & ~3u;  // the ids past the last whole group of 4
  if (sub < c - r) dst[r + sub] = src[r + sub];
}

// Topic t's ids by lane `sub` of its quad: its first request's ids, then its second's.
__host__ __device__ inline void merge_topic(const uint32_t* __restrict__ rq_cnt, const uint64_t* __restrict__ rq_src,
                                            uint64_t t, const uint64_t* __restrict__ out_off,
                                            uint32_t* __restrict__ out_ids, uint32_t sub) {
  const uint2 c = *reinterpret_cast<const uint2*>(rq_cnt + 2 * t);
  const uint32_t cx = c.x, cy = c.y;
  if ((cx | cy) == 0) return;
  const uint64_t dst = out_off[t];
  if (cx) quad_copy_ids(reinterpret_cast<const uint32_t*>(rq_src[2 * t]), out_ids + dst, cx, sub);
  if (cy) quad_copy_ids(reinterpret_cast<const uint32_t*>(rq_src[2 * t + 1]), out_ids + dst + cx, cy, sub);
}

// 4 lanes per topic, in topic order: its first request's ids, then its second's, to the topic's
// place in the output (the counts, addresses and offsets read coalesced, no dependent chain).
__global__ __launch_bounds__(256) void shard_merge_kernel(const uint32_t* __restrict__ rq_cnt,
                                                          const uint64_t* __restrict__ rq_src, uint64_t n,
                                                          const uint64_t* __restrict__ out_off,
                                                          uint32_t* __restrict__ out_ids) {
  const uint32_t sub = threadIdx.x & 3u;
  for (uint64_t t = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 2; t < n;
       t += (static_cast<uint64_t>(gridDim.x) * blockDim.x) >> 2) {
    merge_topic(rq_cnt, rq_src, t, out_off, out_ids, sub);
  }
}

}  // namespace

hipError_t launch_shard_route(const uint8_t* tbytes, const uint64_t* toffs, uint64_t n, uint32_t world,
                              const ShardSplitE* splits, uint32_t n_splits, uint32_t* req2, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(shard_route_kernel, dim3(grid_of(n, 256, 4096)), dim3(256), 0, s, tbytes, toffs, n, world, splits,
                     n_splits, req2);
  return hipGetLastError();
}

}  // namespace emqx

using namespace emqx;

struct emqx_shard_step {
  int device = 0;
  uint32_t world = 1;
  ShardSplitE* d_splits = nullptr;
  uint32_t n_splits = 0;
  // request scratch, sized for m_cap requests
  uint64_t m_cap = 0;
  uint32_t *key = nullptr, *key_s = nullptr, *perm = nullptr, *pos = nullptr, *tcnt = nullptr,
           *tcnt_tab = nullptr, *tbytes_tab = nullptr;  // (tab: the sort's (bucket, tile) table)
  uint64_t *partials = nullptr, *pbytes_tab = nullptr, *rq_src = nullptr;  // (pos: merge's rq_cnt)
  uint64_t* segsum = nullptr;  // the sort scan's segment totals (2 per kScanSeg table entries)
  uint32_t* tpos = nullptr;    // one request a topic: topic t's sorted position
  uint32_t* start = nullptr;  // [kE G + 2]
  uint64_t* cbase = nullptr;  // [G]
  uint64_t* bpre = nullptr;   // [kE G + 2]: each bucket's first byte among the sorted requests'
  int64_t* obase = nullptr;   // [kE G + 2]: offset-word base per bucket (pack)
  int64_t* dbase = nullptr;   // [G]: byte base per destination (pack)
  uint32_t* err = nullptr;
  // the fixed form: the recv table built on the device, the slots' padding offsets, the flag word
  ShardTab* d_tab = nullptr;
  uint64_t* d_pad = nullptr;
  uint32_t* d_flagw = nullptr;
  uint64_t fixed_q = 0;  // the last recv_fixed's request capacity (all slots)
  // the step in flight
  uint64_t n = 0, m = 0;                // topics and requests of the last send
  uint32_t one = 0;                     // one request a topic (world 1 or space P replicated):
                                        // m = n, request p = topic p
  ShardTab recv_tab{};                  // the last recv's per-source table (answer uses it)
  SelfIds self_ids{};                   // the last answer's in-place own ids (merge uses them)
  bool have_recv = false, have_send = false;
  // host mode (device < 0): every pointer is host memory and each call runs on the caller's
  // thread — the kernels' per-item bodies (layout_dest, pack_request, unpack_part,
  // answer_source, gather_request, merge_topic; routing and fold from layout.h / shard_fold) as
  // loops, the tile sort as a stable counting sort.  The CPU rehearsal of the protocol over gloo
  // (tests/test_dist_gloo.py drives dist.py's step with it).
  bool host = false;
  std::vector<ShardSplitE> h_splits;
  std::vector<uint32_t> h_key, h_key_s, h_perm, h_pos, h_tcnt, h_start, h_tpos;
  std::vector<uint64_t> h_rq_src, h_bpre, h_cbase;
  std::vector<int64_t> h_obase, h_dbase;
  ShardTab h_tab{};
  uint64_t h_pad[kE] = {};
  uint32_t h_flagw[4] = {};
};

namespace {

void free_scratch(emqx_shard_step* st) {
  for (void* p : {static_cast<void*>(st->key), static_cast<void*>(st->tcnt_tab), static_cast<void*>(st->key_s),
                  static_cast<void*>(st->perm), static_cast<void*>(st->pos),
                  static_cast<void*>(st->tcnt), static_cast<void*>(st->partials),
                  static_cast<void*>(st->rq_src), static_cast<void*>(st->tbytes_tab), static_cast<void*>(st->pbytes_tab),
                  static_cast<void*>(st->segsum), static_cast<void*>(st->tpos)})
    if (p) (void)hipFree(p);
  st->key = st->tcnt_tab = st->key_s = st->perm = st->pos = st->tcnt = st->tbytes_tab = st->tpos = nullptr;
  st->partials = st->pbytes_tab = st->rq_src = st->segsum = nullptr;
  st->m_cap = 0;
}

// Scratch for m requests (grown geometrically; hipFree waits for the device, so nothing in
// flight still reads the old buffers).
hipError_t ensure_scratch(emqx_shard_step* st, uint64_t m) {
  if (m <= st->m_cap && st->key) return hipSuccess;
  free_scratch(st);
  const uint64_t cap = std::max<uint64_t>(std::max<uint64_t>(m, 1) + m / 4, 1 << 16);
  hipError_t e = hipSuccess;
  auto al = [&](auto** p, uint64_t bytes) {
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(p), std::max<uint64_t>(bytes, 16));
  };
  al(&st->key, 4 * cap);
  // (+ padding: the scans read whole 16-entry rounds / 8-entry thread chunks)
  const uint64_t tab = (kE * st->world + 1ull) * ((cap + kSortTile - 1) / kSortTile + 1) + 16;
  al(&st->tcnt_tab, 4 * tab);
  al(&st->tbytes_tab, 4 * tab);
  al(&st->pbytes_tab, 8 * tab);
  al(&st->segsum, 16 * (tab / kScanSeg + 2));
  al(&st->key_s, 4 * cap);
  al(&st->perm, 4 * cap);
  al(&st->pos, 4 * cap);
  al(&st->rq_src, 8 * cap);
  al(&st->tcnt, 4 * (cap / 2 + 1));
  al(&st->tpos, 4 * (cap / 2 + 1));
  al(&st->partials, 8 * scan_partials(cap));
  if (e != hipSuccess) {
    free_scratch(st);
    return e;
  }
  st->m_cap = cap;
  return hipSuccess;
}

int hip_rc(hipError_t e) { return e == hipSuccess ? EMQX_OK : (e == hipErrorOutOfMemory ? EMQX_ENOMEM : EMQX_EDEVICE); }

// ---- host mode ----------------------------------------------------------------------------

// The send on the host: routing and fold per topic, a stable counting sort by bucket (what the
// tiles' counting sort computes), then the same layout and packing as the kernels.
int host_send(emqx_shard_step* st, const uint8_t* tb, const uint64_t* to, uint64_t n, uint8_t* send, uint64_t cap,
              int64_t* meta, uint64_t fixed) {
  const uint32_t G = st->world, nb = kE * G + 1;
  const uint64_t m = st->one ? n : 2 * n;
  st->h_key.assign(m, 0);
  st->h_key_s.assign(m, 0);
  st->h_perm.assign(m, 0);
  st->h_tpos.assign(st->one ? n : 0, 0);
  for (uint64_t t = 0; t < n; ++t) {
    ShardTopicLevels L;
    shard_topic_levels(tb + to[t], to[t + 1] - to[t], &L);
    uint32_t r[2];
    shard_route_levels(tb + to[t], to[t + 1] - to[t], L, G, st->d_splits, st->n_splits, r);
    const uint2 k = shard_fold(r, G);
    if (st->one) {
      st->h_key[t] = k.x;
    } else {
      st->h_key[2 * t] = k.x;
      st->h_key[2 * t + 1] = k.y;
    }
  }
  auto topic_of = [&](uint64_t p) { return st->one ? p : p >> 1; };
  std::vector<uint64_t> cnt(nb, 0), byb(nb, 0);
  for (uint64_t p = 0; p < m; ++p) {
    const uint32_t k = st->h_key[p];
    ++cnt[k];
    if (k < nb - 1) byb[k] += to[topic_of(p) + 1] - to[topic_of(p)];
  }
  uint64_t c = 0, b = 0;
  for (uint32_t k = 0; k < nb; ++k) {
    st->start[k] = static_cast<uint32_t>(c);
    st->bpre[k] = b;
    c += cnt[k];
    b += byb[k];
  }
  st->start[nb] = static_cast<uint32_t>(m);
  st->bpre[nb] = b;
  bool wide = false;
  std::vector<uint64_t> sz(G);
  uint64_t total = 0;
  for (uint32_t r = 0; r < G; ++r) {
    sz[r] = dest_size(r, st->start, st->bpre, &wide);
    st->cbase[r] = fixed ? fixed * r : total;
    total += sz[r];
    wide |= fixed && sz[r] > fixed;
  }
  const bool over = (!fixed && total > cap) || wide;
  for (uint32_t r = 0; r < G; ++r) {
    layout_dest(r, sz[r], st->cbase[r], over, st->start, st->bpre, send, meta, st->obase, st->dbase);
    if (fixed && over) flagged_chunk(send + st->cbase[r]);
  }
  st->h_flagw[0] = over ? 1u : 0u;
  std::vector<uint64_t> nextp(st->start, st->start + nb), nextx(st->bpre, st->bpre + nb);
  for (uint64_t p = 0; p < m; ++p) {  // in request order: stable
    const uint32_t k = st->h_key[p];
    const uint64_t pos = nextp[k]++;
    st->h_key_s[pos] = k;
    st->h_perm[pos] = static_cast<uint32_t>(p);
    if (st->one) st->h_tpos[p] = static_cast<uint32_t>(pos);
    if (k == nb - 1 || over) continue;
    const uint64_t a = to[topic_of(p)];
    const uint32_t len = static_cast<uint32_t>(to[topic_of(p) + 1] - a);
    pack_request(send, k, static_cast<uint32_t>(pos), nextx[k], st->obase, st->bpre, st->dbase, tb + a, len);
    nextx[k] += len;
  }
  st->key_s = st->h_key_s.data();
  st->perm = st->h_perm.data();
  st->tpos = st->h_tpos.data();
  return EMQX_OK;
}

// The merge on the host: gather per request, the topics' totals and offsets, then the copies.
int host_merge(emqx_shard_step* st, const ShardTab& t, uint64_t* out_off, uint32_t* out_ids) {
  const uint64_t n = st->n, m = st->m;
  st->h_pos.assign(2 * n + 2, 0);
  st->h_rq_src.assign(2 * n + 2, 0);
  const uint32_t nreq = st->start[kE * st->world];
  st->h_tcnt.assign(n + 1, 0);
  if (st->one)
    for (uint64_t q = 0; q < n; ++q)
      gather_topic(t, st->self_ids, st->key_s, st->tpos, st->start, nreq, q, st->h_pos.data(), st->h_rq_src.data(),
                   st->h_tcnt.data());
  else
    for (uint64_t p = 0; p < m; ++p)
      gather_request(t, st->self_ids, st->key_s, st->perm, st->start, nreq, p, st->h_pos.data(), st->h_rq_src.data(),
                     st->one);
  out_off[0] = 0;
  for (uint64_t q = 0; q < n; ++q) out_off[q + 1] = out_off[q] + st->h_pos[2 * q] + st->h_pos[2 * q + 1];
  if (n && !out_ids && out_off[n]) return EMQX_EINVAL;
  for (uint64_t q = 0; q < n; ++q)
    for (uint32_t sub = 0; sub < 4; ++sub) merge_topic(st->h_pos.data(), st->h_rq_src.data(), q, out_off, out_ids, sub);
  return EMQX_OK;
}

#define SS_TRY(x)                    \
  do {                               \
    hipError_t e_ = (x);             \
    if (e_ != hipSuccess) return hip_rc(e_); \
  } while (0)

}  // namespace

extern "C" {

uint64_t emqx_shard_send_cap(uint64_t n, uint64_t batch_bytes, uint32_t world) {
  return 96ull * std::max<uint32_t>(world, 1) + 8 * n + 2 * batch_bytes + 64;
}

int emqx_shard_step_create(int device, uint32_t world, const emqx_shard_split* splits, uint32_t n_splits,
                           emqx_shard_step** out) {
  if (!out || world == 0 || world > kMaxWorld || (n_splits && !splits) || world > 0xFFFF) return EMQX_EINVAL;
  *out = nullptr;
  auto* st = new (std::nothrow) emqx_shard_step();
  if (!st) return EMQX_ENOMEM;
  st->device = device;
  st->world = world;
  st->n_splits = n_splits;
  st->one = world == 1 || shard_p_replicated(reinterpret_cast<const ShardSplitE*>(splits), n_splits) ? 1u : 0u;
  if (device < 0) {  // host mode
    try {
      st->host = true;
      const auto* sp = reinterpret_cast<const ShardSplitE*>(splits);
      st->h_splits.assign(sp, sp + n_splits);
      st->d_splits = st->h_splits.data();
      st->h_start.assign(kE * world + 2, 0);
      st->h_bpre.assign(kE * world + 2, 0);
      st->h_obase.assign(kE * world + 2, 0);
      st->h_dbase.assign(world, 0);
      st->h_cbase.assign(world, 0);
    } catch (const std::bad_alloc&) {
      delete st;
      return EMQX_ENOMEM;
    }
    st->start = st->h_start.data();
    st->bpre = st->h_bpre.data();
    st->obase = st->h_obase.data();
    st->dbase = st->h_dbase.data();
    st->cbase = st->h_cbase.data();
    st->d_tab = &st->h_tab;
    st->d_pad = st->h_pad;
    st->d_flagw = st->h_flagw;
    *out = st;
    return EMQX_OK;
  }
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&st->d_splits), std::max<uint64_t>(8ull * n_splits, 16));
  if (e == hipSuccess && n_splits)
    e = hipMemcpy(st->d_splits, splits, 8ull * n_splits, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipStreamSynchronize(nullptr);  // (the DMA has landed: steps run on other streams)
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&st->start), 4ull * (kE * world + 2));
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&st->cbase), 8ull * world);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&st->bpre), 8ull * (kE * world + 2));
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&st->obase), 8ull * (kE * world + 2));
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&st->dbase), 8ull * world);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&st->err), 16);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&st->d_tab), sizeof(ShardTab));
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&st->d_pad), 8 * kE);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&st->d_flagw), 16);
  if (e == hipSuccess) e = hipMemset(st->d_flagw, 0, 16);
  if (e != hipSuccess) {
    emqx_shard_step_destroy(st);
    return hip_rc(e);
  }
  *out = st;
  return EMQX_OK;
}

int emqx_shard_step_destroy(emqx_shard_step* st) {
  if (!st) return EMQX_EINVAL;
  if (st->host) {
    delete st;
    return EMQX_OK;
  }
  (void)hipSetDevice(st->device);
  (void)hipDeviceSynchronize();
  free_scratch(st);
  for (void* p : {static_cast<void*>(st->d_splits), static_cast<void*>(st->start), static_cast<void*>(st->cbase),
                  static_cast<void*>(st->bpre), static_cast<void*>(st->obase), static_cast<void*>(st->dbase),
                  static_cast<void*>(st->err), static_cast<void*>(st->d_tab), static_cast<void*>(st->d_pad),
                  static_cast<void*>(st->d_flagw)})
    if (p) (void)hipFree(p);
  delete st;
  return EMQX_OK;
}

}  // extern "C"

namespace {

int merge_launch(emqx_shard_step* st, const ShardTab& t, uint64_t* d_out_offsets, uint32_t* d_out_ids, hipStream_t s);

int send_impl(emqx_shard_step* st, const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n, uint8_t* d_send,
              uint64_t send_cap, int64_t* d_meta, uint64_t fixed, void* stream) {
  if (!st || !d_send || !d_meta || (n && (!d_bytes || !d_offsets)) || n >= (1ull << 31)) return EMQX_EINVAL;
  if (st->host) {
    try {
      const int rc = host_send(st, d_bytes, d_offsets, n, d_send, send_cap, d_meta, fixed);
      if (rc != EMQX_OK) return rc;
    } catch (const std::bad_alloc&) {
      return EMQX_ENOMEM;
    }
    st->n = n;
    st->m = st->one ? n : 2 * n;
    st->have_send = true;
    st->have_recv = false;
    return EMQX_OK;
  }
  const hipStream_t s = static_cast<hipStream_t>(stream);
  SS_TRY(hipSetDevice(st->device));
  const uint64_t m = st->one ? n : 2 * n;
  SS_TRY(ensure_scratch(st, 2 * n));  // (the merge's per-topic request pairs: 2 n either way)
  const uint32_t G = st->world;
  if (m) {
    const uint32_t nb = kE * G + 1;
    const uint32_t ntiles = static_cast<uint32_t>((m + kSortTile - 1) / kSortTile);
    hipLaunchKernelGGL(shard_key_kernel, dim3(ntiles), dim3(256), 0, s, d_bytes, d_offsets, n, G, st->d_splits,
                       st->n_splits, st->key, ntiles, st->tcnt_tab, st->tbytes_tab, st->one);
    const uint32_t N = nb * ntiles;
    if (N <= kOneBlockScan) {
      hipLaunchKernelGGL(shard_sort_scan_kernel, dim3(1), dim3(kScanThreads), 0, s, st->tcnt_tab, st->tbytes_tab,
                         st->pbytes_tab, nb, ntiles, m, st->start, st->bpre);
    } else {
      const uint32_t nseg = (N + kScanSeg - 1) / kScanSeg;
      hipLaunchKernelGGL(shard_seg_sums_kernel, dim3(nseg), dim3(256), 0, s, st->tcnt_tab, st->tbytes_tab, N,
                         st->segsum);
      hipLaunchKernelGGL(shard_seg_scan_kernel, dim3(1), dim3(256), 0, s, st->segsum, nseg);
      hipLaunchKernelGGL(shard_seg_final_kernel, dim3(nseg), dim3(256), 0, s, st->tcnt_tab, st->tbytes_tab,
                         st->pbytes_tab, N, ntiles, nb, m, st->segsum, st->start, st->bpre);
    }
    hipLaunchKernelGGL(shard_layout_kernel, dim3(1), dim3(64), 0, s, st->start, st->bpre, G, d_send, send_cap, d_meta,
                       st->cbase, st->obase, st->dbase, st->err, fixed, fixed ? st->d_flagw : nullptr);
    hipLaunchKernelGGL(shard_sort_scatter_kernel, dim3(ntiles), dim3(256), 0, s, st->key, d_bytes, d_offsets, m, nb,
                       ntiles, st->tcnt_tab, st->pbytes_tab, st->bpre, st->obase, st->dbase, st->err, d_send,
                       st->key_s, st->perm, st->one, st->tpos);
  } else {
    SS_TRY(hipMemsetAsync(st->start, 0, 4ull * (kE * G + 2), s));
    SS_TRY(hipMemsetAsync(st->bpre, 0, 8ull * (kE * G + 2), s));
    hipLaunchKernelGGL(shard_layout_kernel, dim3(1), dim3(64), 0, s, st->start, st->bpre, G, d_send, send_cap, d_meta,
                       st->cbase, st->obase, st->dbase, st->err, fixed, fixed ? st->d_flagw : nullptr);
  }
  SS_TRY(hipGetLastError());
  st->n = n;
  st->m = m;
  st->have_send = true;
  st->have_recv = false;
  return EMQX_OK;
}

}  // namespace

extern "C" {

int emqx_shard_step_send(emqx_shard_step* st, const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n,
                         uint8_t* d_send, uint64_t send_cap, int64_t* d_meta, void* stream) {
  return send_impl(st, d_bytes, d_offsets, n, d_send, send_cap, d_meta, 0, stream);
}

int emqx_shard_step_send_fixed(emqx_shard_step* st, const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n,
                               uint8_t* d_send, uint64_t chunk_bytes, int64_t* d_meta, void* stream) {
  if (!st || chunk_bytes < 4 * (kHW + kE) || chunk_bytes % 16) return EMQX_EINVAL;
  return send_impl(st, d_bytes, d_offsets, n, d_send, chunk_bytes * st->world, d_meta, chunk_bytes, stream);
}

int emqx_shard_step_recv(emqx_shard_step* st, const uint8_t* const* d_chunks, const int64_t* meta_in,
                         uint8_t** d_bytes, uint64_t* const* d_offsets, void* stream) {
  if (!st || !d_chunks || !meta_in || !d_bytes || !d_offsets) return EMQX_EINVAL;
  for (uint32_t e = 0; e < kE; ++e)
    if (!d_offsets[e]) return EMQX_EINVAL;
  const uint32_t G = st->world;
  ShardTab& t = st->recv_tab;
  t = ShardTab{};
  uint64_t words = 0;
  for (uint32_t r = 0; r < G; ++r) {
    const int64_t* m = meta_in + (1 + 2 * kE) * r;
    for (uint32_t k = 0; k < 1 + 2 * kE; ++k)
      if (m[k] < 0) return EMQX_EINVAL;
    if (m[0] && !d_chunks[r]) return EMQX_EINVAL;
    t.chunk[r] = reinterpret_cast<uint64_t>(d_chunks[r]);
    uint64_t nall = 0;
    for (uint32_t e = 0; e < kE; ++e) {
      t.q0[e][r + 1] = t.q0[e][r] + static_cast<uint32_t>(m[1 + e]);
      t.y0[e][r + 1] = t.y0[e][r] + static_cast<uint64_t>(m[1 + kE + e]);
      nall += static_cast<uint64_t>(m[1 + e]);
    }
    t.w0[r] = words;
    words += kHW + nall;
  }
  t.w0[G] = words;
  // a slot whose requests all come from one source is read in place from that source's chunk
  // (its offsets rebased from 0 are already relative to its byte region): no copy
  int only[kE];
  for (uint32_t e = 0; e < kE; ++e) {
    only[e] = -1;
    for (uint32_t r = 0; r < G; ++r)
      if (t.q0[e][r + 1] != t.q0[e][r]) only[e] = only[e] == -1 ? static_cast<int>(r) : -2;
    if (only[e] < 0 && t.y0[e][G] && !d_bytes[e]) return EMQX_EINVAL;
  }
  SlotOffsets so{};
  for (uint32_t e = 0; e < kE; ++e) so.p[e] = d_offsets[e];
  uint64_t qall = 0;
  for (uint32_t e = 0; e < kE; ++e) qall += t.q0[e][G];
  uint64_t yall = 0;
  for (uint32_t e = 0; e < kE; ++e) yall += t.y0[e][G];
  // (blocks per (source, slot): its offsets, or its bytes in 16-B moves, whichever is more work)
  const uint64_t per = std::max<uint64_t>(qall, yall / 16) / (kE * G) + 1;
  const uint32_t x = grid_of(per, 256, std::max<uint32_t>(1, 1024 / G));
  SlotBytes sb{};
  for (uint32_t e = 0; e < kE; ++e) sb.p[e] = only[e] >= 0 ? nullptr : d_bytes[e];
  if (st->host) {
    for (uint32_t r = 0; r < G; ++r)
      for (uint32_t e = 0; e < kE; ++e) unpack_part(t, so, sb, r, e, 0, 1);
  } else {
    const hipStream_t s = static_cast<hipStream_t>(stream);
    SS_TRY(hipSetDevice(st->device));
    hipLaunchKernelGGL(shard_unpack_kernel, dim3(x, G, kE), dim3(256), 0, s, t, so, sb);
    SS_TRY(hipGetLastError());
  }
  for (uint32_t r = 0; r < G; ++r) {  // a slot with one source: matched where that source packed it
    uint64_t nall = 0;
    for (uint32_t e = 0; e < kE; ++e) nall += t.q0[e][r + 1] - t.q0[e][r];
    const uint8_t* data = d_chunks[r] + 4 * kHW + al16(4ull * (nall + kE));
    for (uint32_t e = 0; e < kE; ++e) {
      if (only[e] == static_cast<int>(r)) d_bytes[e] = const_cast<uint8_t*>(data);
      data += t.y0[e][r + 1] - t.y0[e][r];
    }
  }
  st->have_recv = true;
  return EMQX_OK;
}

int emqx_shard_step_answer(emqx_shard_step* st, const uint64_t* const* d_offsets, const uint32_t* const* d_ids,
                           const uint64_t* const* d_summaries, uint32_t self_rank, uint32_t* d_answer,
                           int64_t* d_ans_meta, void* stream) {
  if (!st || !st->have_recv || !d_offsets || !d_ids || !d_answer || !d_ans_meta) return EMQX_EINVAL;
  const uint32_t G = st->world;
  if (self_rank >= G && self_rank != kNone) return EMQX_EINVAL;
  const ShardTab& t = st->recv_tab;
  EngineCsrs cs{};
  uint64_t qall = 0;
  st->self_ids = SelfIds{};
  st->self_ids.self = self_rank;
  for (uint32_t e = 0; e < kE; ++e) {
    if (!d_offsets[e] || (t.q0[e][G] && !d_ids[e])) return EMQX_EINVAL;
    cs.off[e] = d_offsets[e];
    cs.ids[e] = d_ids[e];
    cs.sum[e] = d_summaries ? d_summaries[e] : nullptr;
    qall += t.q0[e][G];
    st->self_ids.ids[e] = d_ids[e];
    st->self_ids.off[e] = d_offsets[e];
    st->self_ids.q0[e] = self_rank < G ? t.q0[e][self_rank] : 0;
  }
  if (st->host) {
    for (uint32_t r = 0; r < G; ++r) answer_source(cs, t, self_rank, d_answer, d_ans_meta, r, G, 0, 1, true);
    return EMQX_OK;
  }
  const hipStream_t s = static_cast<hipStream_t>(stream);
  SS_TRY(hipSetDevice(st->device));
  const uint32_t x = grid_of(8 * qall / G + 1, 256, std::max<uint32_t>(1, 1024 / G));  // ~8 ids a request
  hipLaunchKernelGGL(shard_answer_kernel, dim3(x, G), dim3(256), 0, s, cs, t, self_rank, d_answer, d_ans_meta);
  SS_TRY(hipGetLastError());
  return EMQX_OK;
}

int emqx_shard_step_merge(emqx_shard_step* st, const uint32_t* const* d_chunks, const int64_t* ans_meta_in,
                          uint64_t* d_out_offsets, uint32_t* d_out_ids, void* stream) {
  if (!st || !st->have_send || !d_chunks || !ans_meta_in || !d_out_offsets) return EMQX_EINVAL;
  const uint32_t G = st->world;
  ShardTab t{};
  for (uint32_t r = 0; r < G; ++r) {
    if (ans_meta_in[kAnsMeta * r] < kHW || ans_meta_in[kAnsMeta * r + 1] != 0 || !d_chunks[r]) return EMQX_EINVAL;
    t.chunk[r] = reinterpret_cast<uint64_t>(d_chunks[r]);
  }
  if (st->host) {
    try {
      return host_merge(st, t, d_out_offsets, d_out_ids);
    } catch (const std::bad_alloc&) {
      return EMQX_ENOMEM;
    }
  }
  const hipStream_t s = static_cast<hipStream_t>(stream);
  SS_TRY(hipSetDevice(st->device));
  return merge_launch(st, t, d_out_offsets, d_out_ids, s);
}

}  // extern "C"

namespace {

int merge_launch(emqx_shard_step* st, const ShardTab& t, uint64_t* d_out_offsets, uint32_t* d_out_ids, hipStream_t s) {
  const uint32_t G = st->world;
  const uint64_t n = st->n, m = st->m;
  if (m && st->one) {
    hipLaunchKernelGGL(shard_gather_topic_kernel, dim3(grid_of(n, 256)), dim3(256), 0, s, t, st->self_ids, st->key_s,
                       st->tpos, st->start, n, G, st->pos, st->rq_src, st->tcnt);
  } else if (m) {
    hipLaunchKernelGGL(shard_gather_kernel, dim3(grid_of(m, 256)), dim3(256), 0, s, t, st->self_ids, st->key_s,
                       st->perm, st->start, m, G, st->pos, st->rq_src, st->one);
    hipLaunchKernelGGL(shard_topic_counts_kernel, dim3(grid_of(n, 256)), dim3(256), 0, s, st->pos, n, st->tcnt);
  }
  SS_TRY(launch_scan(st->tcnt, n, d_out_offsets, st->partials, s));
  if (n) {
    if (!d_out_ids) return EMQX_EINVAL;
    hipLaunchKernelGGL(shard_merge_kernel, dim3(grid_of(n, 64)), dim3(256), 0, s, st->pos, st->rq_src, n, d_out_offsets,
                       d_out_ids);
  }
  SS_TRY(hipGetLastError());
  return EMQX_OK;
}

}  // namespace

extern "C" {

// ---- the fixed-capacity form --------------------------------------------------------------

int emqx_shard_step_recv_fixed(emqx_shard_step* st, const uint8_t* const* d_chunks, const uint64_t* cap_requests,
                               const uint64_t* cap_bytes, uint8_t* const* d_bytes, uint64_t* const* d_offsets,
                               void* stream) {
  if (!st || !st->have_send || !d_chunks || !cap_requests || !cap_bytes || !d_offsets) return EMQX_EINVAL;
  const uint32_t G = st->world;
  bool rel = true;
  SlotCaps cap{};
  SlotOffsets so{};
  SlotBytes sb{};
  uint64_t qall = 0, yall = 0;
  for (uint32_t e = 0; e < kE; ++e) {
    if (!d_offsets[e] || cap_requests[e] >= (1ull << 31)) return EMQX_EINVAL;
    cap.q[e] = cap_requests[e];
    cap.y[e] = cap_bytes[e];
    so.p[e] = d_offsets[e];
    sb.p[e] = d_bytes ? d_bytes[e] : nullptr;
    rel &= sb.p[e] == nullptr;
    qall += cap.q[e];
    yall += cap.y[e];
  }
  for (uint32_t e = 0; e < kE; ++e)
    if (!rel && !sb.p[e] && cap.q[e]) return EMQX_EINVAL;  // (in place: every slot, and only at world 1)
  if (rel && G != 1) return EMQX_EINVAL;
  sb.rel = rel ? 1u : 0u;
  ShardTab ch{};
  for (uint32_t r = 0; r < G; ++r) {
    if (!d_chunks[r]) return EMQX_EINVAL;
    ch.chunk[r] = reinterpret_cast<uint64_t>(d_chunks[r]);
  }
  st->fixed_q = qall;
  st->have_recv = true;
  if (st->host) {
    recv_table(ch.chunk, ch.chunk, G, cap, rel, st->d_tab, st->d_pad, st->d_flagw);
    if (!st->d_flagw[0])
      for (uint32_t r = 0; r < G; ++r)
        for (uint32_t e = 0; e < kE; ++e) unpack_part(*st->d_tab, so, sb, r, e, 0, 1);
    for (uint32_t e = 0; e < kE; ++e) pad_slot(*st->d_tab, G, so, cap, st->d_pad, e, 0, 1);
    return EMQX_OK;
  }
  const hipStream_t s = static_cast<hipStream_t>(stream);
  SS_TRY(hipSetDevice(st->device));
  const uint64_t per = std::max<uint64_t>(qall, yall / 16) / (kE * G) + 1;
  const uint32_t x = grid_of(per, 256, std::max<uint32_t>(1, 1024 / G));
  hipLaunchKernelGGL(shard_recv_fixed_kernel, dim3(x, G + 1, kE), dim3(256), 0, s, ch, G, cap, sb.rel, so, sb, st->d_tab,
                     st->d_pad, st->d_flagw);
  SS_TRY(hipGetLastError());
  return EMQX_OK;
}

int emqx_shard_step_answer_fixed(emqx_shard_step* st, const uint64_t* const* d_offsets, const uint32_t* const* d_ids,
                                 const uint64_t* const* d_summaries, uint32_t self_rank, uint32_t* d_answer,
                                 uint64_t chunk_words, void* stream) {
  if (!st || !st->have_recv || !d_offsets || !d_ids || !d_answer || chunk_words < kHW) return EMQX_EINVAL;
  const uint32_t G = st->world;
  if (self_rank >= G && self_rank != kNone) return EMQX_EINVAL;
  EngineCsrs cs{};
  st->self_ids = SelfIds{};
  st->self_ids.self = self_rank;
  st->self_ids.rtab = st->d_tab;
  st->self_ids.flagw = st->d_flagw;
  for (uint32_t e = 0; e < kE; ++e) {
    if (!d_offsets[e] || !d_ids[e]) return EMQX_EINVAL;
    cs.off[e] = d_offsets[e];
    cs.ids[e] = d_ids[e];
    cs.sum[e] = d_summaries ? d_summaries[e] : nullptr;
    st->self_ids.ids[e] = d_ids[e];
    st->self_ids.off[e] = d_offsets[e];
  }
  if (st->host) {
    answer_plan(cs, *st->d_tab, self_rank, G, chunk_words, st->d_flagw);
    for (uint32_t r = 0; r < G; ++r)
      answer_source(cs, *st->d_tab, self_rank, d_answer, nullptr, r, G, 0, 1, false, chunk_words, st->d_flagw[0]);
    return EMQX_OK;
  }
  const hipStream_t s = static_cast<hipStream_t>(stream);
  SS_TRY(hipSetDevice(st->device));
  const uint32_t x = grid_of(8 * st->fixed_q / G + 1, 256, std::max<uint32_t>(1, 1024 / G));  // ~8 ids a request
  hipLaunchKernelGGL(shard_answer_fixed_kernel, dim3(x, G), dim3(256), 0, s, cs, st->d_tab, self_rank, d_answer,
                     chunk_words, st->d_flagw);
  SS_TRY(hipGetLastError());
  return EMQX_OK;
}

int emqx_shard_step_merge_fixed(emqx_shard_step* st, const uint32_t* const* d_chunks, uint64_t* d_out_offsets,
                                uint32_t* d_out_ids, uint32_t* d_flag, void* stream) {
  if (!st || !st->have_send || !st->self_ids.flagw || !d_chunks || !d_out_offsets || (st->n && !d_out_ids))
    return EMQX_EINVAL;
  const uint32_t G = st->world;
  ShardTab t{};
  for (uint32_t r = 0; r < G; ++r) {
    if (!d_chunks[r]) return EMQX_EINVAL;
    t.chunk[r] = reinterpret_cast<uint64_t>(d_chunks[r]);
  }
  if (st->host) {
    merge_plan(t.chunk, G, st->d_flagw, d_flag);
    try {
      return host_merge(st, t, d_out_offsets, d_out_ids);
    } catch (const std::bad_alloc&) {
      return EMQX_ENOMEM;
    }
  }
  const hipStream_t s = static_cast<hipStream_t>(stream);
  SS_TRY(hipSetDevice(st->device));
  hipLaunchKernelGGL(shard_merge_plan_kernel, dim3(1), dim3(64), 0, s, t, G, st->d_flagw, d_flag);
  return merge_launch(st, t, d_out_offsets, d_out_ids, s);
}

}  // extern "C"
