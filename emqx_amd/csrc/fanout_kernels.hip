// HIP kernels for gfx950: publish fan-out — matched filter ids -> subscriber deliveries.
//
// Replaces emqx_broker:route/2 + do_dispatch/2,3 (apps/emqx/src/emqx_broker.erl:244-259,
// 500-524) and emqx_shared_sub:dispatch/3 -> pick/6 -> do_pick_subscriber/6
// (apps/emqx/src/emqx_shared_sub.erl:113-126,251-288) for a whole batch of published topics.
//
// Pipeline, all on one stream with no host synchronisation: the number of
// match entries m = moff[n] - moff[0] is read on the device, so every kernel below runs a
// fixed grid over a length it loads itself.
//   entry_topic  one thread per topic: entry -> topic map (hash strategies only)
//   count        FO_BLOCKS blocks, one contiguous chunk of entries each: per-entry count
//                n_plain + n_groups of its filter, and the chunk's sum
//   partials     one block: exclusive scan of the chunk sums, the total, the overflow flag
//                and the call summary
//   final        FO_BLOCKS blocks: per-entry output offsets (chunk scan + the chunk's base)
//   offsets      per-topic output offsets = per-entry offsets at the match CSR boundaries
//   write        one wavefront per 256 match entries: the wave walks its flattened outputs 64
//                at a time (each lane finds its entry by an 8-step search over LDS prefix
//                offsets), so plain-subscriber copies are coalesced reads and writes; each
//                $share group contributes exactly one pick.  Skipped entirely on overflow, so
//                no pick state is consumed by a call that wrote nothing.
// Bandwidth-bound streaming; no MFMA.
#include <hip/hip_runtime.h>

#include "../../include/emqx_match.h"
#include "fanout.h"
#include "layout.h"

namespace emqx {

namespace {

constexpr int FO_THREADS = 256;
constexpr uint32_t FO_UNROLL = 4;  // outputs per lane per round of the write kernel
constexpr uint32_t FO_WCHUNK = 256;  // match entries per wave chunk of the write kernel

__device__ __forceinline__ uint32_t fo_lane() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

__global__ __launch_bounds__(FO_THREADS) void fanout_entry_topic_kernel(FanoutArgs a) {
  const uint64_t base = a.moff[0];
  for (uint64_t t = blockIdx.x * uint64_t(FO_THREADS) + threadIdx.x; t < a.n;
       t += uint64_t(gridDim.x) * FO_THREADS) {
    const uint64_t b = a.moff[t] - base, e = a.moff[t + 1] - base;
    for (uint64_t i = b; i < e; ++i) a.entry_topic[i] = static_cast<uint32_t>(t);
  }
}

__device__ __forceinline__ uint64_t fo_entries(const FanoutArgs& a) { return a.moff[a.n] - a.moff[0]; }

// Chunk [lo, hi) of block b out of FO_BLOCKS over m entries (multiples of 64).
__device__ __forceinline__ void fo_chunk(uint64_t m, uint32_t b, uint64_t* lo, uint64_t* hi) {
  const uint64_t per = ((m + FO_BLOCKS - 1) / FO_BLOCKS + 63) & ~63ull;
  *lo = min<uint64_t>(m, per * b);
  *hi = min<uint64_t>(m, per * (b + 1));
}

__device__ __forceinline__ uint64_t fo_wave_sum(uint64_t v) {
#pragma unroll
  for (uint32_t d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// Block-wide exclusive scan of one u64 per thread (FO_THREADS threads).
__device__ __forceinline__ uint64_t fo_block_excl_scan(uint64_t v, uint64_t* total) {
  __shared__ uint64_t wsum[FO_THREADS / 64];
  const uint32_t lane = fo_lane(), w = threadIdx.x >> 6;
  uint64_t incl = v;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint64_t before = 0, all = 0;
#pragma unroll
  for (uint32_t k = 0; k < FO_THREADS / 64; ++k) {
    before += k < w ? wsum[k] : 0;
    all += wsum[k];
  }
  __syncthreads();
  *total = all;
  return before + incl - v;
}

__global__ __launch_bounds__(FO_THREADS) void fanout_count_kernel(FanoutArgs a) {
  __shared__ uint64_t bsum[FO_THREADS / 64];
  const uint64_t base = a.moff[0];
  uint64_t lo, hi;
  fo_chunk(fo_entries(a), blockIdx.x, &lo, &hi);
  uint64_t sum = 0;
  for (uint64_t i = lo + threadIdx.x; i < hi; i += FO_THREADS) {
    const uint32_t f = a.mids[base + i];
    uint32_t c = 0;
    if (f < a.n_recs) {
      const uint4 r = *reinterpret_cast<const uint4*>(a.recs + f);
      c = r.y + r.w;
    }
    a.ecount[i] = c;
    sum += c;
  }
  sum = fo_wave_sum(sum);
  if (fo_lane() == 0) bsum[threadIdx.x >> 6] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (uint32_t k = 0; k < FO_THREADS / 64; ++k) t += bsum[k];
    a.partials[blockIdx.x] = t;
  }
}

// One block of FO_BLOCKS threads: chunk bases, eoff[m] = total, the call summary.
__global__ __launch_bounds__(FO_BLOCKS) void fanout_partials_kernel(FanoutArgs a) {
  __shared__ uint64_t wsum[FO_BLOCKS / 64];
  const uint32_t lane = fo_lane(), w = threadIdx.x >> 6;
  const uint64_t v = a.partials[threadIdx.x];
  uint64_t incl = v;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint64_t y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint64_t before = 0, all = 0;
  for (uint32_t k = 0; k < FO_BLOCKS / 64; ++k) {
    before += k < w ? wsum[k] : 0;
    all += wsum[k];
  }
  a.partials[FO_BLOCKS + threadIdx.x] = before + incl - v;
  if (threadIdx.x == 0) {
    const uint64_t m = fo_entries(a);
    a.eoff[m] = all;
    uint64_t* sm = a.summary;
    sm[FO_SUM_FLAGS] = all > a.cap ? FO_SUM_F_OVERFLOW : 0u;
    sm[FO_SUM_TOTAL] = all;
    sm[FO_SUM_ENTRIES] = m;
    __threadfence_system();
  }
}

// Per-entry output offsets: each block rescans its chunk, FO_THREADS * 4 entries per round.
__global__ __launch_bounds__(FO_THREADS) void fanout_final_kernel(FanoutArgs a) {
  uint64_t lo, hi;
  fo_chunk(fo_entries(a), blockIdx.x, &lo, &hi);
  uint64_t carry = a.partials[FO_BLOCKS + blockIdx.x];
  for (uint64_t r0 = lo; r0 < hi; r0 += FO_THREADS * 4) {
    const uint64_t i0 = r0 + 4ull * threadIdx.x;
    uint32_t c[4];
    uint64_t sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      c[k] = i0 + k < hi ? a.ecount[i0 + k] : 0u;
      sum += c[k];
    }
    uint64_t tot;
    uint64_t p = carry + fo_block_excl_scan(sum, &tot);
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      if (i0 + k < hi) a.eoff[i0 + k] = p;
      p += c[k];
    }
    carry += tot;
  }
}

__global__ __launch_bounds__(FO_THREADS) void fanout_offsets_kernel(FanoutArgs a) {
  const uint64_t base = a.moff[0];
  for (uint64_t t = blockIdx.x * uint64_t(FO_THREADS) + threadIdx.x; t <= a.n;
       t += uint64_t(gridDim.x) * FO_THREADS)
    a.out_off[t] = a.eoff[a.moff[t] - base];
}

// One pick among n >= 1 members of group record g (entry i of topic t).
__device__ __forceinline__ uint32_t pick_member(const FanoutArgs& a, const GroupRec& g, uint64_t i, uint32_t t,
                                                uint32_t gidx) {
  const uint32_t n = g.n_members;
  if (a.strategy == EMQX_SHARE_STICKY) {
    GroupState* st = a.state + g.slot;
    uint32_t s = __hip_atomic_load(&st->sticky, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (s != SUB_NONE) return s;
    const uint32_t r = mix32(a.seed ^ mix32(static_cast<uint32_t>(i) * 0x9E3779B1u ^ gidx));
    const uint32_t cand = a.members[g.member_begin + (n > 1 ? r % n : 0u)];
    const uint32_t old = atomicCAS(&st->sticky, SUB_NONE, cand);
    return old == SUB_NONE ? cand : old;
  }
  // pick_subscriber/6 with one member returns it without consulting the strategy
  // (emqx_shared_sub.erl:266), so a lone member never advances round-robin state.
  if (n == 1) return a.members[g.member_begin];
  uint32_t idx;
  switch (a.strategy) {
    case EMQX_SHARE_HASH_CLIENTID:
    case EMQX_SHARE_HASH_TOPIC:
      idx = a.keys[t] % n;  // 1 + phash2(Key) rem Count, 1-based in the reference
      break;
    case EMQX_SHARE_ROUND_ROBIN:
      idx = atomicAdd(&a.state[g.slot].rr, 1u) % n;
      break;
    default:  // EMQX_SHARE_RANDOM
      idx = mix32(a.seed ^ mix32(static_cast<uint32_t>(i) * 0x9E3779B1u ^ (gidx + 0x632BE5ABu))) % n;
      break;
  }
  return a.members[g.member_begin + idx];
}

__global__ __launch_bounds__(FO_THREADS) void fanout_write_kernel(FanoutArgs a) {
  struct WaveLds {
    uint32_t pre[FO_WCHUNK];  // entry's first output, relative to the chunk's first output
    uint32_t fid[FO_WCHUNK];
    uint32_t pb[FO_WCHUNK];
    uint32_t np[FO_WCHUNK];
    uint32_t gb[FO_WCHUNK];
    uint32_t top[FO_WCHUNK];
  };
  __shared__ WaveLds lds_all[FO_THREADS / 64];
  constexpr uint32_t EU = FO_WCHUNK / 64;  // entries per lane per chunk
  const uint32_t lane = fo_lane();
  const uint32_t wv = threadIdx.x >> 6;
  WaveLds& L = lds_all[wv];
  const uint64_t base = a.moff[0];
  const uint64_t m = fo_entries(a);
  if (a.eoff[m] > a.cap) return;  // overflow: nothing is written, no pick state consumed
  const bool need_topic = a.strategy == EMQX_SHARE_HASH_CLIENTID || a.strategy == EMQX_SHARE_HASH_TOPIC;
  const uint64_t nwaves = uint64_t(gridDim.x) * (FO_THREADS / 64);
  for (uint64_t e0 = (uint64_t(blockIdx.x) * (FO_THREADS / 64) + wv) * FO_WCHUNK; e0 < m;
       e0 += nwaves * FO_WCHUNK) {
    const uint64_t e1 = min<uint64_t>(e0 + FO_WCHUNK, m);
    const uint64_t obase = a.eoff[e0];
    const uint32_t total = static_cast<uint32_t>(a.eoff[e1] - obase);
    // the chunk's entries, EU per lane: every first-level load of the chunk is in flight
    // before the filter records are fetched, and those before anything is stored to LDS
    uint32_t f[EU], tp[EU];
    uint64_t eo[EU];
#pragma unroll
    for (uint32_t u = 0; u < EU; ++u) {
      const uint64_t i = e0 + lane + 64u * u;
      const bool v = i < e1;
      f[u] = v ? a.mids[base + i] : FID_NONE;
      eo[u] = v ? a.eoff[i] : obase + total;
      tp[u] = (v && need_topic) ? a.entry_topic[i] : 0u;
    }
    uint4 r[EU];
#pragma unroll
    for (uint32_t u = 0; u < EU; ++u)
      r[u] = f[u] < a.n_recs ? *reinterpret_cast<const uint4*>(a.recs + f[u]) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t u = 0; u < EU; ++u) {
      const uint32_t k = lane + 64u * u;
      L.pre[k] = static_cast<uint32_t>(eo[u] - obase);  // past the chunk's end: `total`
      L.fid[k] = f[u];
      L.pb[k] = r[u].x;
      L.np[k] = r[u].y;
      L.gb[k] = r[u].z;
      L.top[k] = tp[u];
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // FO_UNROLL outputs per lane per round: all plain-subscriber loads of the round are in
    // flight before the first store ($share picks, ~10 % of entries, resolve after them).
    for (uint32_t j0 = 0; j0 < total; j0 += 64 * FO_UNROLL) {
      uint32_t sub[FO_UNROLL], fl[FO_UNROLL], kk[FO_UNROLL], rr[FO_UNROLL];
      bool act[FO_UNROLL], shr[FO_UNROLL];
#pragma unroll
      for (uint32_t u = 0; u < FO_UNROLL; ++u) {
        const uint32_t j = j0 + lane + 64u * u;
        act[u] = j < total;
        // largest k with pre[k] <= j (pre is non-decreasing, pre[0] = 0, slots past the
        // chunk's entries hold `total`); k + step never exceeds FO_WCHUNK - 1
        uint32_t k = 0;
#pragma unroll
        for (uint32_t step = FO_WCHUNK / 2; step >= 1; step >>= 1)
          if (L.pre[k + step] <= j) k += step;
        kk[u] = k;
        rr[u] = j - L.pre[k];
        fl[u] = L.fid[k];
        shr[u] = act[u] && rr[u] >= L.np[k];
        sub[u] = (act[u] && !shr[u]) ? a.plain[L.pb[k] + rr[u]] : 0u;
      }
#pragma unroll
      for (uint32_t u = 0; u < FO_UNROLL; ++u) {
        if (!shr[u]) continue;
        const uint32_t k = kk[u];
        const uint32_t gidx = L.gb[k] + (rr[u] - L.np[k]);
        const uint4 gr = *reinterpret_cast<const uint4*>(a.groups + gidx);
        const GroupRec g{gr.x, gr.y, gr.z, gr.w};
        sub[u] = pick_member(a, g, e0 + k, L.top[k], gidx);
        fl[u] |= FANOUT_SHARED_BIT;
      }
#pragma unroll
      for (uint32_t u = 0; u < FO_UNROLL; ++u) {
        if (!act[u]) continue;
        const uint32_t j = j0 + lane + 64u * u;
        a.out_subs[obase + j] = sub[u];
        if (a.out_filters) a.out_filters[obase + j] = fl[u];
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

uint32_t grid_for(uint64_t items, uint32_t per_block) {
  const uint64_t g = (items + per_block - 1) / per_block;
  return static_cast<uint32_t>(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

}  // namespace

hipError_t launch_fanout(const FanoutArgs& a, uint64_t m_cap, hipStream_t s) {
  const bool hash = a.strategy == EMQX_SHARE_HASH_CLIENTID || a.strategy == EMQX_SHARE_HASH_TOPIC;
  if (a.n && hash)
    hipLaunchKernelGGL(fanout_entry_topic_kernel, dim3(grid_for(a.n, FO_THREADS)), dim3(FO_THREADS), 0, s, a);
  hipLaunchKernelGGL(fanout_count_kernel, dim3(FO_BLOCKS), dim3(FO_THREADS), 0, s, a);
  hipLaunchKernelGGL(fanout_partials_kernel, dim3(1), dim3(FO_BLOCKS), 0, s, a);
  hipLaunchKernelGGL(fanout_final_kernel, dim3(FO_BLOCKS), dim3(FO_THREADS), 0, s, a);
  hipLaunchKernelGGL(fanout_offsets_kernel, dim3(grid_for(a.n + 1, FO_THREADS)), dim3(FO_THREADS), 0, s, a);
  // one wave per FO_WCHUNK entries up to m_cap (waves past m exit at once)
  hipLaunchKernelGGL(fanout_write_kernel, dim3(grid_for(m_cap, FO_WCHUNK * (FO_THREADS / 64))), dim3(FO_THREADS), 0, s,
                     a);
  return hipGetLastError();
}

}  // namespace emqx
