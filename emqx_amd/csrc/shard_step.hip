// Filter-sharded match step on the device (include/emqx_match.h emqx_shard_step_*, driven by
// emqx_amd/dist.py ShardedMatcher.match_all): the regrouping around the two all-to-alls, with
// no host work beyond the split sizes the collectives need.
//
// The reference replicates every route on every node (emqx_router.erl:135, mria) and matches a
// publish on the node that receives it (emqx_broker.erl:213 -> emqx_router:match_routes/1); a
// table past one GPU is sharded here instead, and one rank's step is
//
//   send    route every topic to its (rank, engine) requests (layout.h shard_route_topic),
//           stable radix sort of the requests by destination, one chunk per destination:
//             [u32 nA nB bytesA bytesB][u32 offsets of the nA A-requests + 1][... B + 1] pad 16
//             [A topic bytes][B topic bytes] pad 16
//   recv    the received chunks -> two contiguous batches (every source's A requests, then B)
//   answer  the two engines' CSRs -> one answer chunk per source:
//             [u32 nA nB idsA idsB][counts of the A requests][counts of B][A ids][B ids]
//   merge   the answer chunks -> the CSR of the rank's batch in batch order, each topic's
//           engine-A ids then its engine-B ids
//
// Per-source / per-destination tables (chunk starts, batch bases) come from the host, which
// holds the exchanged sizes anyway, as one kernel argument (world <= 64).  Requests are u32
// indices (2 per topic), so a batch holds fewer than 2^31 topics.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
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

struct ShardTab {
  uint64_t base[kMaxWorld + 1];  // chunk starts (bytes: request chunks; u32 words: answer chunks)
  uint32_t a0[kMaxWorld + 1];    // first A request of each source in the A batch (prefix of nA)
  uint32_t b0[kMaxWorld + 1];
  uint64_t ab0[kMaxWorld + 1];   // first A byte of each source in the A batch
  uint64_t bb0[kMaxWorld + 1];
  uint64_t w0[kMaxWorld + 1];    // answer chunks: prefix of (4 + nA + nB) words
};

__host__ __device__ inline uint64_t al16(uint64_t x) { return (x + 15) & ~15ull; }

// A topic's bytes from src to dst (any alignment: gfx950 global loads and stores take
// unaligned addresses), `lanes` lanes of one request together (sub = this lane's index among
// them): 16-B moves, then the tail byte by byte.
typedef uint4 __attribute__((aligned(1))) u4u;
__device__ __forceinline__ void copy_bytes(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, uint64_t len,
                                           uint32_t sub, uint32_t lanes) {
  const uint64_t full = len & ~15ull;
  for (uint64_t j = 16ull * sub; j < full; j += 16ull * lanes)
    *reinterpret_cast<u4u*>(dst + j) = *reinterpret_cast<const u4u*>(src + j);
  for (uint64_t j = full + sub; j < len; j += lanes) dst[j] = src[j];
}

uint32_t grid_of(uint64_t items, uint32_t per_block, uint32_t cap = 8192) {
  return static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>((items + per_block - 1) / per_block, cap)));
}

uint32_t bucket_bits(uint32_t world) {  // keys 0 .. 2 * world (2 * world = no request)
  uint32_t b = 1;
  while ((1ull << b) < 2ull * world + 1) ++b;
  return b;
}

// ---- send -------------------------------------------------------------------------------

// shard_topic_levels (layout.h) over the topic's bytes read as 16-B aligned windows (a window
// holding a topic byte lies inside the batch's allocation; the batch's last window only up to
// its end): the same summary, one load per 16 bytes instead of one per byte.
__device__ __forceinline__ void topic_levels_dev(const uint8_t* __restrict__ tb, uint64_t s, uint64_t e,
                                                 uint64_t lim, ShardTopicLevels* L) {
  L->n_levels = 0;
  L->wild = false;
  L->h[0] = L->h[1] = L->h[2] = 0;
  uint32_t h = 0x811C9DC5u, len = 0, c0 = 0;
  const uintptr_t abeg = reinterpret_cast<uintptr_t>(tb + s), aend = reinterpret_cast<uintptr_t>(tb + e);
  const uintptr_t alim = reinterpret_cast<uintptr_t>(tb + lim);
  for (uintptr_t w0 = abeg & ~static_cast<uintptr_t>(15); w0 <= aend; w0 += 16) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (w0 + 16 <= alim) {
      v = *reinterpret_cast<const uint4*>(w0);
    } else if (w0 < aend) {
      uint32_t t4[4] = {0, 0, 0, 0};
      for (uint32_t b = 0; b < 16 && w0 + b < alim; ++b)
        t4[b >> 2] |= static_cast<uint32_t>(*reinterpret_cast<const uint8_t*>(w0 + b)) << (8u * (b & 3u));
      v = make_uint4(t4[0], t4[1], t4[2], t4[3]);
    }
    const uint32_t wd[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (uint32_t b = 0; b < 16; ++b) {
      const uintptr_t q = w0 + b;
      if (q < abeg || q > aend) continue;
      const uint32_t c = q < aend ? (wd[b >> 2] >> (8u * (b & 3u))) & 0xFFu : static_cast<uint32_t>('/');
      if (c == '/') {
        if (L->n_levels < 3) L->h[L->n_levels] = mix32(h ^ len);
        if (len == 1 && (c0 == '+' || c0 == '#')) L->wild = true;
        ++L->n_levels;
        h = 0x811C9DC5u;
        len = 0;
      } else {
        if (len == 0) c0 = c;
        h = (h ^ c) * 0x01000193u;
        ++len;
      }
    }
  }
}

__global__ __launch_bounds__(256) void shard_key_kernel(const uint8_t* __restrict__ tb,
                                                        const uint64_t* __restrict__ to, uint64_t n, uint32_t world,
                                                        const ShardSplitE* __restrict__ sp, uint32_t nsp,
                                                        uint32_t* __restrict__ key, uint32_t* __restrict__ idx) {
  const uint64_t lim = n ? to[n] : 0;
  for (uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < n;
       t += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint64_t a = to[t], b = to[t + 1];
    ShardTopicLevels L;
    topic_levels_dev(tb, a, b, lim, &L);
    uint32_t r[2];
    shard_route_levels(tb + a, b - a, L, world, sp, nsp, r);
    *reinterpret_cast<uint2*>(key + 2 * t) =
        make_uint2(r[0] == kNone ? 2 * world : r[0], r[1] == kNone ? 2 * world : r[1]);
    *reinterpret_cast<uint2*>(idx + 2 * t) = make_uint2(static_cast<uint32_t>(2 * t), static_cast<uint32_t>(2 * t + 1));
  }
}

// start[b] = first position of bucket b in the sorted requests (b = 0 .. 2G + 1; start[2G] =
// the request count, start[2G + 1] = m); len[p] = bytes of request p's topic (0 for no request).
__global__ __launch_bounds__(256) void shard_bounds_kernel(const uint32_t* __restrict__ key_s,
                                                           const uint32_t* __restrict__ perm,
                                                           const uint64_t* __restrict__ to, uint64_t m,
                                                           uint32_t world, uint32_t* __restrict__ start,
                                                           uint32_t* __restrict__ len) {
  const uint32_t nb = 2 * world + 1;
  for (uint64_t p = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; p < m;
       p += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint32_t k = key_s[p];
    const uint32_t lo = p ? key_s[p - 1] + 1 : 0;
    for (uint32_t b = lo; b <= k; ++b) start[b] = static_cast<uint32_t>(p);
    if (p == m - 1)
      for (uint32_t b = k + 1; b <= nb; ++b) start[b] = static_cast<uint32_t>(m);
    uint32_t l = 0;
    if (k < 2 * world) {
      const uint32_t t = perm[p] >> 1;
      l = static_cast<uint32_t>(to[t + 1] - to[t]);
    }
    len[p] = l;
  }
}

// One block: per destination rank the chunk's sizes, start, header and final offsets.
__global__ __launch_bounds__(64) void shard_layout_kernel(const uint32_t* __restrict__ start,
                                                          const uint64_t* __restrict__ sc, uint32_t world,
                                                          uint8_t* __restrict__ send, uint64_t cap,
                                                          int64_t* __restrict__ meta, uint64_t* __restrict__ cbase,
                                                          uint32_t* __restrict__ err) {
  __shared__ uint64_t sz[kMaxWorld];
  const uint32_t r = threadIdx.x;
  uint32_t nA = 0, nB = 0;
  uint64_t bA = 0, bB = 0, size = 0;
  if (r < world) {
    const uint32_t s0 = start[2 * r], s1 = start[2 * r + 1], s2 = start[2 * r + 2];
    nA = s1 - s0;
    nB = s2 - s1;
    bA = sc[s1] - sc[s0];
    bB = sc[s2] - sc[s1];
    size = 16 + al16(4ull * (nA + nB + 2)) + al16(bA + bB);
    sz[r] = size;
  }
  __syncthreads();
  if (r >= world) return;
  uint64_t base = 0;
  for (uint32_t j = 0; j < r; ++j) base += sz[j];
  uint64_t total = 0;
  for (uint32_t j = 0; j < world; ++j) total += sz[j];
  cbase[r] = base;
  const bool over = total > cap || bA > 0xFFFFFFFFull || bB > 0xFFFFFFFFull;
  meta[5 * r + 0] = over ? -1 : static_cast<int64_t>(size);
  meta[5 * r + 1] = nA;
  meta[5 * r + 2] = nB;
  meta[5 * r + 3] = static_cast<int64_t>(bA);
  meta[5 * r + 4] = static_cast<int64_t>(bB);
  if (over) {
    if (r == 0) err[0] = 1;
    return;
  }
  if (r == 0) err[0] = 0;
  uint32_t* h = reinterpret_cast<uint32_t*>(send + base);
  h[0] = nA;
  h[1] = nB;
  h[2] = static_cast<uint32_t>(bA);
  h[3] = static_cast<uint32_t>(bB);
  h[4 + nA] = static_cast<uint32_t>(bA);           // A offsets[nA]
  h[4 + nA + 1 + nB] = static_cast<uint32_t>(bB);  // B offsets[nB]
}

// 4 lanes per request (16 requests a wave, their loads in flight together): its offset entry
// and its topic's bytes (16-B moves) into the destination's chunk.
__global__ __launch_bounds__(256) void shard_pack_kernel(const uint8_t* __restrict__ tb,
                                                         const uint64_t* __restrict__ to,
                                                         const uint32_t* __restrict__ key_s,
                                                         const uint32_t* __restrict__ perm,
                                                         const uint32_t* __restrict__ start,
                                                         const uint64_t* __restrict__ sc,
                                                         const uint64_t* __restrict__ cbase, uint32_t world,
                                                         const uint32_t* __restrict__ err, uint8_t* __restrict__ send) {
  if (err[0]) return;
  const uint32_t nreq = start[2 * world];
  const uint32_t sub = threadIdx.x & 3u;
  for (uint64_t p = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 2; p < nreq;
       p += (static_cast<uint64_t>(gridDim.x) * blockDim.x) >> 2) {
    const uint32_t b = key_s[p], r = b >> 1, e = b & 1u;
    const uint32_t s0 = start[2 * r], s1 = start[2 * r + 1], s2 = start[2 * r + 2];
    const uint32_t nA = s1 - s0, nB = s2 - s1;
    const uint64_t rel = sc[p] - sc[start[b]];
    uint8_t* c = send + cbase[r];
    if (sub == 0)
      reinterpret_cast<uint32_t*>(c)[4 + (e ? nA + 1 : 0) + (p - start[b])] = static_cast<uint32_t>(rel);
    const uint64_t data = 16 + al16(4ull * (nA + nB + 2)) + (e ? sc[s1] - sc[s0] : 0) + rel;
    const uint32_t t = perm[p] >> 1;
    const uint64_t a = to[t], len = to[t + 1] - a;
    copy_bytes(tb + a, c + data, len, sub, 4);
  }
}

// emqx_shard_route_device: the raw requests (req2[2t], req2[2t + 1]) with the same scanner.
__global__ __launch_bounds__(256) void shard_route_kernel(const uint8_t* __restrict__ tb,
                                                          const uint64_t* __restrict__ to, uint64_t n, uint32_t world,
                                                          const ShardSplitE* __restrict__ sp, uint32_t nsp,
                                                          uint32_t* __restrict__ req2) {
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

// grid (x, source, engine): the source's offsets rebased into the batch (its bytes are one
// contiguous region each, moved by the copy engine: emqx_shard_step_recv).
__global__ __launch_bounds__(256) void shard_unpack_kernel(const uint8_t* __restrict__ recv, ShardTab tab,
                                                           uint64_t* __restrict__ a_off, uint64_t* __restrict__ b_off) {
  const uint32_t s = blockIdx.y, e = blockIdx.z;
  const uint32_t nA = tab.a0[s + 1] - tab.a0[s], nB = tab.b0[s + 1] - tab.b0[s];
  const uint32_t* offs = reinterpret_cast<const uint32_t*>(recv + tab.base[s]) + 4 + (e ? nA + 1 : 0);
  const uint32_t n = e ? nB : nA;
  const uint64_t dbase = e ? tab.bb0[s] : tab.ab0[s];
  uint64_t* doff = (e ? b_off : a_off) + (e ? tab.b0[s] : tab.a0[s]);
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t k = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; k <= n; k += stride)
    doff[k] = dbase + offs[k];
}

// ---- answer -----------------------------------------------------------------------------

// grid (x, source): the source's answer chunk from the two CSRs.  An engine call that did not
// complete (summary flags) leaves its ids unread: the step is redone.
__global__ __launch_bounds__(256) void shard_answer_kernel(const uint64_t* __restrict__ a_off,
                                                           const uint32_t* __restrict__ a_ids,
                                                           const uint64_t* __restrict__ a_sum,
                                                           const uint64_t* __restrict__ b_off,
                                                           const uint32_t* __restrict__ b_ids,
                                                           const uint64_t* __restrict__ b_sum, ShardTab tab,
                                                           uint32_t* __restrict__ out, int64_t* __restrict__ ans_meta) {
  const uint32_t s = blockIdx.y;
  const uint32_t a0 = tab.a0[s], nA = tab.a0[s + 1] - a0, b0 = tab.b0[s], nB = tab.b0[s + 1] - b0;
  const bool bad = (a_sum && a_sum[0]) || (b_sum && b_sum[0]);
  const uint64_t iA0 = a_off[a0], iB0 = b_off[b0];
  const uint64_t iA = bad ? 0 : a_off[a0 + nA] - iA0, iB = bad ? 0 : b_off[b0 + nB] - iB0;
  const uint64_t cb = tab.w0[s] + (bad ? 0 : iA0 + iB0);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    ans_meta[2 * s] = static_cast<int64_t>(4 + nA + nB + iA + iB);
    ans_meta[2 * s + 1] = bad ? 1 : 0;
  }
  if (bad) return;
  uint32_t* c = out + cb;
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  if (tid == 0) {
    c[0] = nA;
    c[1] = nB;
    c[2] = static_cast<uint32_t>(iA);
    c[3] = static_cast<uint32_t>(iB);
  }
  for (uint64_t k = tid; k < nA; k += stride) c[4 + k] = static_cast<uint32_t>(a_off[a0 + k + 1] - a_off[a0 + k]);
  for (uint64_t k = tid; k < nB; k += stride) c[4 + nA + k] = static_cast<uint32_t>(b_off[b0 + k + 1] - b_off[b0 + k]);
  uint32_t* ids = c + 4 + nA + nB;
  for (uint64_t j = tid; j < iA; j += stride) ids[j] = a_ids[iA0 + j];
  for (uint64_t j = tid; j < iB; j += stride) ids[iA + j] = b_ids[iB0 + j];
}

// ---- merge ------------------------------------------------------------------------------

// Per sorted request p: its answer count, and pos[request] = p (kNone for no request).
__global__ __launch_bounds__(256) void shard_gather_counts_kernel(const uint32_t* __restrict__ back, ShardTab tab,
                                                                  const uint32_t* __restrict__ key_s,
                                                                  const uint32_t* __restrict__ perm,
                                                                  const uint32_t* __restrict__ start, uint64_t m,
                                                                  uint32_t world, uint32_t* __restrict__ cnt,
                                                                  uint32_t* __restrict__ pos) {
  const uint32_t nreq = start[2 * world];
  for (uint64_t p = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; p < m;
       p += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    uint32_t c = 0;
    if (p < nreq) {
      const uint32_t b = key_s[p], r = b >> 1, e = b & 1u;
      const uint32_t* ch = back + tab.base[r];
      c = ch[4 + (e ? ch[0] : 0) + (p - start[b])];
      pos[perm[p]] = static_cast<uint32_t>(p);
    } else {
      pos[perm[p]] = kNone;
    }
    cnt[p] = c;
  }
}

__global__ __launch_bounds__(256) void shard_topic_counts_kernel(const uint32_t* __restrict__ cnt,
                                                                 const uint32_t* __restrict__ pos, uint64_t n,
                                                                 uint32_t* __restrict__ tcnt) {
  for (uint64_t t = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < n;
       t += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint2 q = *reinterpret_cast<const uint2*>(pos + 2 * t);
    tcnt[t] = (q.x != kNone ? cnt[q.x] : 0u) + (q.y != kNone ? cnt[q.y] : 0u);
  }
}

// 4 lanes per request, in request (send) order: its answer's ids, read from the answer chunk
// where they lie in that same order (coalesced), to its topic's place in the output: the
// topic's offset, after the topic's engine-A ids for an engine-B request.
__global__ __launch_bounds__(256) void shard_merge_kernel(const uint32_t* __restrict__ back, ShardTab tab,
                                                          const uint32_t* __restrict__ key_s,
                                                          const uint32_t* __restrict__ perm,
                                                          const uint32_t* __restrict__ start,
                                                          const uint32_t* __restrict__ cnt,
                                                          const uint64_t* __restrict__ csc,
                                                          const uint32_t* __restrict__ pos, uint32_t world,
                                                          const uint64_t* __restrict__ out_off,
                                                          uint32_t* __restrict__ out_ids) {
  const uint32_t nreq = start[2 * world];
  const uint32_t sub = threadIdx.x & 3u;
  for (uint64_t p = (static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 2; p < nreq;
       p += (static_cast<uint64_t>(gridDim.x) * blockDim.x) >> 2) {
    const uint32_t c = cnt[p];
    if (c == 0) continue;
    const uint32_t q = perm[p], t = q >> 1, e = q & 1u;
    const uint32_t b = key_s[p], r = b >> 1;
    const uint32_t* ch = back + tab.base[r];
    const uint64_t src = 4ull + ch[0] + ch[1] + (e ? ch[2] : 0u) + (csc[p] - csc[start[b]]);
    uint64_t dst = out_off[t];
    if (e) {
      const uint32_t pa = pos[2 * t];
      if (pa != kNone) dst += cnt[pa];
    }
    for (uint32_t j = sub; j < c; j += 4) out_ids[dst + j] = ch[src + j];
  }
}

using SortCfg = rocprim::default_config;

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
  uint32_t *key = nullptr, *idx = nullptr, *key_s = nullptr, *perm = nullptr, *len = nullptr, *pos = nullptr,
           *tcnt = nullptr;
  uint64_t *sc = nullptr, *partials = nullptr;
  void* sort_temp = nullptr;
  size_t sort_bytes = 0;
  uint32_t* start = nullptr;  // [2G + 2]
  uint64_t* cbase = nullptr;  // [G]
  uint32_t* err = nullptr;
  // the step in flight
  uint64_t n = 0;                       // topics of the last send
  ShardTab recv_tab{};                  // the last recv's per-source table (answer uses it)
  bool have_recv = false, have_send = false;
};

namespace {

void free_scratch(emqx_shard_step* st) {
  for (void* p : {static_cast<void*>(st->key), static_cast<void*>(st->idx), static_cast<void*>(st->key_s),
                  static_cast<void*>(st->perm), static_cast<void*>(st->len), static_cast<void*>(st->pos),
                  static_cast<void*>(st->tcnt), static_cast<void*>(st->sc), static_cast<void*>(st->partials),
                  st->sort_temp})
    if (p) (void)hipFree(p);
  st->key = st->idx = st->key_s = st->perm = st->len = st->pos = st->tcnt = nullptr;
  st->sc = st->partials = nullptr;
  st->sort_temp = nullptr;
  st->m_cap = 0;
  st->sort_bytes = 0;
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
  al(&st->idx, 4 * cap);
  al(&st->key_s, 4 * cap);
  al(&st->perm, 4 * cap);
  al(&st->len, 4 * cap);
  al(&st->pos, 4 * cap);
  al(&st->tcnt, 4 * (cap / 2 + 1));
  al(&st->sc, 8 * (cap + 1));
  al(&st->partials, 8 * scan_partials(cap));
  size_t tb = 0;
  if (e == hipSuccess)
    e = rocprim::radix_sort_pairs<SortCfg>(nullptr, tb, static_cast<const uint32_t*>(nullptr),
                                           static_cast<uint32_t*>(nullptr), static_cast<const uint32_t*>(nullptr),
                                           static_cast<uint32_t*>(nullptr), static_cast<size_t>(cap), 0u,
                                           bucket_bits(st->world));
  if (e == hipSuccess) {
    st->sort_bytes = tb;
    al(&st->sort_temp, tb);
  }
  if (e != hipSuccess) {
    free_scratch(st);
    return e;
  }
  st->m_cap = cap;
  return hipSuccess;
}

int hip_rc(hipError_t e) { return e == hipSuccess ? EMQX_OK : (e == hipErrorOutOfMemory ? EMQX_ENOMEM : EMQX_EDEVICE); }

#define SS_TRY(x)                    \
  do {                               \
    hipError_t e_ = (x);             \
    if (e_ != hipSuccess) return hip_rc(e_); \
  } while (0)

}  // namespace

extern "C" {

uint64_t emqx_shard_send_cap(uint64_t n, uint64_t batch_bytes, uint32_t world) {
  return 48ull * std::max<uint32_t>(world, 1) + 8 * n + 2 * batch_bytes + 64;
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
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&st->d_splits), std::max<uint64_t>(8ull * n_splits, 16));
  if (e == hipSuccess && n_splits)
    e = hipMemcpy(st->d_splits, splits, 8ull * n_splits, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipStreamSynchronize(nullptr);  // (the DMA has landed: steps run on other streams)
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&st->start), 4ull * (2 * world + 2));
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&st->cbase), 8ull * world);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&st->err), 16);
  if (e != hipSuccess) {
    emqx_shard_step_destroy(st);
    return hip_rc(e);
  }
  *out = st;
  return EMQX_OK;
}

int emqx_shard_step_destroy(emqx_shard_step* st) {
  if (!st) return EMQX_EINVAL;
  (void)hipSetDevice(st->device);
  (void)hipDeviceSynchronize();
  free_scratch(st);
  for (void* p : {static_cast<void*>(st->d_splits), static_cast<void*>(st->start), static_cast<void*>(st->cbase),
                  static_cast<void*>(st->err)})
    if (p) (void)hipFree(p);
  delete st;
  return EMQX_OK;
}

int emqx_shard_step_send(emqx_shard_step* st, const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n,
                         uint8_t* d_send, uint64_t send_cap, int64_t* d_meta, void* stream) {
  if (!st || !d_send || !d_meta || (n && (!d_bytes || !d_offsets)) || n >= (1ull << 31)) return EMQX_EINVAL;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  SS_TRY(hipSetDevice(st->device));
  const uint64_t m = 2 * n;
  SS_TRY(ensure_scratch(st, m));
  const uint32_t G = st->world;
  if (m) {
    hipLaunchKernelGGL(shard_key_kernel, dim3(grid_of(n, 256, 4096)), dim3(256), 0, s, d_bytes, d_offsets, n, G,
                       st->d_splits, st->n_splits, st->key, st->idx);
    size_t tb = 0;
    SS_TRY(rocprim::radix_sort_pairs<SortCfg>(nullptr, tb, st->key, st->key_s, st->idx, st->perm,
                                              static_cast<size_t>(m), 0u, bucket_bits(G), s));
    if (tb > st->sort_bytes) return EMQX_EDEVICE;  // (sized for m_cap >= m)
    tb = st->sort_bytes;
    SS_TRY(rocprim::radix_sort_pairs<SortCfg>(st->sort_temp, tb, st->key, st->key_s, st->idx, st->perm,
                                              static_cast<size_t>(m), 0u, bucket_bits(G), s));
    hipLaunchKernelGGL(shard_bounds_kernel, dim3(grid_of(m, 256)), dim3(256), 0, s, st->key_s, st->perm, d_offsets, m,
                       G, st->start, st->len);
  } else {
    SS_TRY(hipMemsetAsync(st->start, 0, 4ull * (2 * G + 2), s));
  }
  SS_TRY(launch_scan(st->len, m, st->sc, st->partials, s));
  hipLaunchKernelGGL(shard_layout_kernel, dim3(1), dim3(64), 0, s, st->start, st->sc, G, d_send, send_cap, d_meta,
                     st->cbase, st->err);
  if (m)
    hipLaunchKernelGGL(shard_pack_kernel, dim3(grid_of(m, 64)), dim3(256), 0, s, d_bytes, d_offsets, st->key_s,
                       st->perm, st->start, st->sc, st->cbase, G, st->err, d_send);
  SS_TRY(hipGetLastError());
  st->n = n;
  st->have_send = true;
  st->have_recv = false;
  return EMQX_OK;
}

int emqx_shard_step_recv(emqx_shard_step* st, const uint8_t* d_recv, const int64_t* meta_in, uint8_t* d_a_bytes,
                         uint64_t* d_a_offsets, uint8_t* d_b_bytes, uint64_t* d_b_offsets, void* stream) {
  if (!st || !meta_in || !d_a_offsets || !d_b_offsets) return EMQX_EINVAL;
  const uint32_t G = st->world;
  ShardTab& t = st->recv_tab;
  t = ShardTab{};
  uint64_t words = 0;
  for (uint32_t r = 0; r < G; ++r) {
    const int64_t* m = meta_in + 5 * r;
    if (m[0] < 0 || m[1] < 0 || m[2] < 0 || m[3] < 0 || m[4] < 0) return EMQX_EINVAL;
    t.base[r + 1] = t.base[r] + static_cast<uint64_t>(m[0]);
    t.a0[r + 1] = t.a0[r] + static_cast<uint32_t>(m[1]);
    t.b0[r + 1] = t.b0[r] + static_cast<uint32_t>(m[2]);
    t.ab0[r + 1] = t.ab0[r] + static_cast<uint64_t>(m[3]);
    t.bb0[r + 1] = t.bb0[r] + static_cast<uint64_t>(m[4]);
    t.w0[r] = words;
    words += 4 + static_cast<uint64_t>(m[1] + m[2]);
  }
  t.w0[G] = words;
  if ((t.base[G] && !d_recv) || (t.ab0[G] && !d_a_bytes) || (t.bb0[G] && !d_b_bytes)) return EMQX_EINVAL;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  SS_TRY(hipSetDevice(st->device));
  const uint64_t per = (t.a0[G] + t.b0[G]) / (2 * G) + 1;  // offsets per (source, engine)
  const uint32_t x = grid_of(per, 256, std::max<uint32_t>(1, 1024 / G));
  hipLaunchKernelGGL(shard_unpack_kernel, dim3(x, G, 2), dim3(256), 0, s, d_recv, t, d_a_offsets, d_b_offsets);
  SS_TRY(hipGetLastError());
  for (uint32_t r = 0; r < G; ++r) {  // each source's A bytes, then its B bytes: contiguous both sides
    const uint64_t nA = t.a0[r + 1] - t.a0[r], nB = t.b0[r + 1] - t.b0[r];
    const uint64_t bA = t.ab0[r + 1] - t.ab0[r], bB = t.bb0[r + 1] - t.bb0[r];
    const uint8_t* data = d_recv + t.base[r] + 16 + al16(4ull * (nA + nB + 2));
    if (bA) SS_TRY(hipMemcpyAsync(d_a_bytes + t.ab0[r], data, bA, hipMemcpyDeviceToDevice, s));
    if (bB) SS_TRY(hipMemcpyAsync(d_b_bytes + t.bb0[r], data + bA, bB, hipMemcpyDeviceToDevice, s));
  }
  st->have_recv = true;
  return EMQX_OK;
}

int emqx_shard_step_answer(emqx_shard_step* st, const uint64_t* d_a_offsets, const uint32_t* d_a_ids,
                           const uint64_t* d_a_summary, const uint64_t* d_b_offsets, const uint32_t* d_b_ids,
                           const uint64_t* d_b_summary, uint32_t* d_answer, int64_t* d_ans_meta, void* stream) {
  if (!st || !st->have_recv || !d_a_offsets || !d_b_offsets || !d_answer || !d_ans_meta) return EMQX_EINVAL;
  const uint32_t G = st->world;
  const ShardTab& t = st->recv_tab;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  SS_TRY(hipSetDevice(st->device));
  const uint32_t x = grid_of(8 * (t.a0[G] + t.b0[G]) / G + 1, 256, std::max<uint32_t>(1, 1024 / G));  // ~8 ids a request
  hipLaunchKernelGGL(shard_answer_kernel, dim3(x, G), dim3(256), 0, s, d_a_offsets, d_a_ids, d_a_summary, d_b_offsets,
                     d_b_ids, d_b_summary, t, d_answer, d_ans_meta);
  SS_TRY(hipGetLastError());
  return EMQX_OK;
}

int emqx_shard_step_merge(emqx_shard_step* st, const uint32_t* d_back, const int64_t* ans_meta_in,
                          uint64_t* d_out_offsets, uint32_t* d_out_ids, void* stream) {
  if (!st || !st->have_send || !ans_meta_in || !d_out_offsets) return EMQX_EINVAL;
  const uint32_t G = st->world;
  ShardTab t{};
  for (uint32_t r = 0; r < G; ++r) {
    if (ans_meta_in[2 * r] < 4 || ans_meta_in[2 * r + 1] != 0) return EMQX_EINVAL;
    t.base[r + 1] = t.base[r] + static_cast<uint64_t>(ans_meta_in[2 * r]);
  }
  if (!d_back) return EMQX_EINVAL;
  const hipStream_t s = static_cast<hipStream_t>(stream);
  SS_TRY(hipSetDevice(st->device));
  const uint64_t n = st->n, m = 2 * n;
  if (m) {
    hipLaunchKernelGGL(shard_gather_counts_kernel, dim3(grid_of(m, 256)), dim3(256), 0, s, d_back, t, st->key_s,
                       st->perm, st->start, m, G, st->len, st->pos);
    SS_TRY(launch_scan(st->len, m, st->sc, st->partials, s));
    hipLaunchKernelGGL(shard_topic_counts_kernel, dim3(grid_of(n, 256)), dim3(256), 0, s, st->len, st->pos, n,
                       st->tcnt);
  }
  SS_TRY(launch_scan(st->tcnt, n, d_out_offsets, st->partials, s));
  if (n) {
    if (!d_out_ids) return EMQX_EINVAL;
    hipLaunchKernelGGL(shard_merge_kernel, dim3(grid_of(m, 64)), dim3(256), 0, s, d_back, t, st->key_s, st->perm,
                       st->start, st->len, st->sc, st->pos, G, d_out_offsets, d_out_ids);
  }
  SS_TRY(hipGetLastError());
  return EMQX_OK;
}

}  // extern "C"
