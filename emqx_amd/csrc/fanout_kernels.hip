// HIP kernels for gfx950: publish fan-out — matched filter ids -> subscriber deliveries.
//
// Replaces emqx_broker:route/2 + do_dispatch/2,3 (apps/emqx/src/emqx_broker.erl:244-259,
// 500-524) and emqx_shared_sub:dispatch/3 -> pick/6 -> do_pick_subscriber/6
// (apps/emqx/src/emqx_shared_sub.erl:113-126,251-288) for a whole batch of published topics.
//
// Pipeline, all on one stream, inputs = the match CSR left in HBM:
//   entry_topic  one thread per topic: entry -> topic map (segmented fill)
//   count        one thread per match entry: n_plain + n_groups of its filter
//   scan         (match_kernels.hip) per-entry counts -> per-entry output offsets
//   offsets      per-topic output offsets = per-entry offsets at the match CSR boundaries
//   write        one wavefront per 64 match entries: the wave walks its flattened outputs 64
//                at a time (each lane finds its entry by a 6-step search over LDS prefix
//                offsets), so plain-subscriber copies are coalesced reads and writes; each
//                $share group contributes exactly one pick.
// Bandwidth-bound streaming; no MFMA.
#include <hip/hip_runtime.h>

#include "../../include/emqx_match.h"
#include "fanout.h"
#include "layout.h"

namespace emqx {

namespace {

constexpr int FO_THREADS = 256;

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

__global__ __launch_bounds__(FO_THREADS) void fanout_count_kernel(FanoutArgs a) {
  for (uint64_t i = blockIdx.x * uint64_t(FO_THREADS) + threadIdx.x; i < a.m;
       i += uint64_t(gridDim.x) * FO_THREADS) {
    const uint32_t f = a.mids[i];
    uint32_t c = 0;
    if (f < a.n_recs) {
      const uint4 r = *reinterpret_cast<const uint4*>(a.recs + f);
      c = r.y + r.w;
    }
    a.ecount[i] = c;
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
    uint32_t pre[64];  // entry's first output, relative to the wave's first output
    uint32_t fid[64];
    uint32_t pb[64];
    uint32_t np[64];
    uint32_t gb[64];
    uint32_t top[64];
  };
  __shared__ WaveLds lds_all[FO_THREADS / 64];
  const uint32_t lane = fo_lane();
  const uint32_t wv = threadIdx.x >> 6;
  WaveLds& L = lds_all[wv];
  const uint64_t nwaves = uint64_t(gridDim.x) * (FO_THREADS / 64);
  for (uint64_t e0 = (uint64_t(blockIdx.x) * (FO_THREADS / 64) + wv) * 64; e0 < a.m; e0 += nwaves * 64) {
    const uint64_t e1 = min<uint64_t>(e0 + 64, a.m);
    const uint64_t obase = a.eoff[e0];
    const uint32_t total = static_cast<uint32_t>(a.eoff[e1] - obase);
    const uint64_t i = e0 + lane;
    if (i < e1) {
      const uint32_t f = a.mids[i];
      uint4 r = make_uint4(0, 0, 0, 0);
      if (f < a.n_recs) r = *reinterpret_cast<const uint4*>(a.recs + f);
      L.pre[lane] = static_cast<uint32_t>(a.eoff[i] - obase);
      L.fid[lane] = f;
      L.pb[lane] = r.x;
      L.np[lane] = r.y;
      L.gb[lane] = r.z;
      L.top[lane] = a.entry_topic[i];
    } else {
      L.pre[lane] = total;  // never <= a valid output index
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (uint32_t j0 = 0; j0 < total; j0 += 64) {
      const uint32_t j = j0 + lane;
      if (j < total) {
        // largest k with pre[k] <= j (pre is non-decreasing, pre[0] = 0, unused lanes hold
        // `total`); k + step never exceeds 63
        uint32_t k = 0;
#pragma unroll
        for (uint32_t step = 32; step >= 1; step >>= 1)
          if (L.pre[k + step] <= j) k += step;
        const uint32_t r = j - L.pre[k];
        const uint32_t f = L.fid[k];
        uint32_t sub, fl;
        if (r < L.np[k]) {
          sub = a.plain[L.pb[k] + r];
          fl = f;
        } else {
          const uint32_t gidx = L.gb[k] + (r - L.np[k]);
          const uint4 gr = *reinterpret_cast<const uint4*>(a.groups + gidx);
          const GroupRec g{gr.x, gr.y, gr.z, gr.w};
          sub = pick_member(a, g, e0 + k, L.top[k], gidx);
          fl = f | FANOUT_SHARED_BIT;
        }
        a.out_subs[obase + j] = sub;
        if (a.out_filters) a.out_filters[obase + j] = fl;
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

hipError_t launch_fanout_count(const FanoutArgs& a, hipStream_t s) {
  if (a.n) hipLaunchKernelGGL(fanout_entry_topic_kernel, dim3(grid_for(a.n, FO_THREADS)), dim3(FO_THREADS), 0, s, a);
  if (a.m) hipLaunchKernelGGL(fanout_count_kernel, dim3(grid_for(a.m, FO_THREADS)), dim3(FO_THREADS), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_fanout_offsets(const FanoutArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(fanout_offsets_kernel, dim3(grid_for(a.n + 1, FO_THREADS)), dim3(FO_THREADS), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_fanout_write(const FanoutArgs& a, hipStream_t s) {
  if (a.m) hipLaunchKernelGGL(fanout_write_kernel, dim3(grid_for(a.m, FO_THREADS)), dim3(FO_THREADS), 0, s, a);
  return hipGetLastError();
}

}  // namespace emqx
