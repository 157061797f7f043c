// HIP kernels for gfx950: publish fan-out — matched filter ids -> subscriber deliveries.
//
// Replaces emqx_broker:route/2 + do_dispatch/2,3 (apps/emqx/src/emqx_broker.erl:244-259,
// 500-524) and emqx_shared_sub:dispatch/3 -> pick/6 -> do_pick_subscriber/6
// (apps/emqx/src/emqx_shared_sub.erl:113-126,234-288) for a whole batch of published topics.
//
// Pipeline, all on one stream with no host synchronisation: the number of
// match entries m = moff[n] - moff[0] is read on the device, so every kernel below runs a
// fixed grid over a length it loads itself.
//   entry_topic  one thread per topic: entry -> topic map (strategies that read per-topic keys)
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
//   resolve      round_robin / sticky only: the picks of one (group slot, publisher) are made
//                in message order from that publisher's state, one thread per such pair
//   finish       one thread: pick-state occupancy into the summary
// Bandwidth-bound streaming; no MFMA.
#include <hip/hip_runtime.h>

#include "../../include/emqx_match.h"
#include "fanout.h"
#include "layout.h"

namespace emqx {

namespace {

constexpr int FO_THREADS = 256;
#ifndef FO_UNROLL_V
#define FO_UNROLL_V 4
#endif
#ifndef FO_WCHUNK_V
#define FO_WCHUNK_V 256
#endif
constexpr uint32_t FO_UNROLL = FO_UNROLL_V;  // outputs per lane per round of the write kernel
constexpr uint32_t FO_WCHUNK = FO_WCHUNK_V;  // match entries per wave chunk of the write kernel

__device__ __forceinline__ uint32_t fo_lane() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

// Match entries of the call: 0 when the match call reported a problem or its CSR is longer
// than the scratch was sized for (the partials kernel flags both).
__device__ __forceinline__ uint64_t fo_entries_raw(const FanoutArgs& a) { return a.moff[a.n] - a.moff[0]; }
__device__ __forceinline__ bool fo_refused(const FanoutArgs& a) {
  return (a.msum && a.msum[0] != 0) || fo_entries_raw(a) > a.m_cap;
}
__device__ __forceinline__ uint64_t fo_entries(const FanoutArgs& a) { return fo_refused(a) ? 0 : fo_entries_raw(a); }

__global__ __launch_bounds__(FO_THREADS) void fanout_entry_topic_kernel(FanoutArgs a) {
  if (fo_refused(a)) return;
  const uint64_t base = a.moff[0];
  for (uint64_t t = blockIdx.x * uint64_t(FO_THREADS) + threadIdx.x; t < a.n;
       t += uint64_t(gridDim.x) * FO_THREADS) {
    const uint64_t b = a.moff[t] - base, e = a.moff[t + 1] - base;
    for (uint64_t i = b; i < e; ++i) a.entry_topic[i] = static_cast<uint32_t>(t);
  }
}

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
    const bool refused = fo_refused(a);
    const uint64_t m = fo_entries(a);
    a.eoff[m] = all;
    uint64_t* sm = a.summary;
    sm[FO_SUM_FLAGS] = refused ? FO_SUM_F_MATCH : (all > a.cap ? FO_SUM_F_OVERFLOW : 0u);
    sm[FO_SUM_TOTAL] = all;
    sm[FO_SUM_ENTRIES] = refused ? fo_entries_raw(a) : m;
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
  const bool refused = fo_refused(a);
  for (uint64_t t = blockIdx.x * uint64_t(FO_THREADS) + threadIdx.x; t <= a.n;
       t += uint64_t(gridDim.x) * FO_THREADS)
    a.out_off[t] = refused ? 0 : a.eoff[a.moff[t] - base];
}

__device__ __forceinline__ uint32_t fo_rand(uint32_t seed, uint64_t i, uint32_t salt) {
  return mix32(seed ^ mix32(static_cast<uint32_t>(i) * 0x9E3779B1u ^ static_cast<uint32_t>(i >> 32) ^ salt));
}

__device__ __forceinline__ uint64_t ps_hash(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  return k;
}

// The state-table entry of `key`, inserting it when absent; PS_EMPTY when the table has no room
// within PS_MAX_PROBES.  *created: this lane inserted it.
__device__ __forceinline__ uint64_t ps_find_or_insert(const FanoutArgs& a, uint64_t key, bool* created) {
  *created = false;
  uint64_t i = ps_hash(key) & a.ps_mask;
  for (uint32_t p = 0; p < PS_MAX_PROBES; ++p, i = (i + 1) & a.ps_mask) {
    uint64_t cur = __hip_atomic_load(a.ps_keys + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) return i;
    if (cur == PS_EMPTY) {
      const unsigned long long old =
          atomicCAS(reinterpret_cast<unsigned long long*>(a.ps_keys + i), static_cast<unsigned long long>(PS_EMPTY),
                    static_cast<unsigned long long>(key));
      if (old == PS_EMPTY) {
        *created = true;
        return i;
      }
      if (old == key) return i;
    }
  }
  return PS_EMPTY;
}

// Appends one u32 per predicated lane to list[*counter ...] with one atomic per wave (every
// active lane must call it).
__device__ __forceinline__ void wave_append(unsigned long long* counter, uint32_t* list, bool pred, uint32_t v) {
  const uint64_t m = __ballot(pred);
  if (!m) return;
  const uint32_t leader = __ffsll(static_cast<long long>(m)) - 1;
  unsigned long long base = 0;
  if (fo_lane() == leader) base = atomicAdd(counter, static_cast<unsigned long long>(__popcll(m)));
  base = __shfl(base, leader, 64);
  if (pred) list[base + __popcll(m & ((1ull << fo_lane()) - 1))] = v;
}

__device__ __forceinline__ void wave_count(unsigned long long* counter, bool pred) {
  const uint64_t m = __ballot(pred);
  if (m && fo_lane() == static_cast<uint32_t>(__ffsll(static_cast<long long>(m)) - 1))
    atomicAdd(counter, static_cast<unsigned long long>(__popcll(m)));
}

// One stateless pick among n >= 1 members of group record g (entry i of topic t).
__device__ __forceinline__ uint32_t pick_stateless(const FanoutArgs& a, const GroupRec& g, uint64_t i, uint32_t t,
                                                   uint32_t gidx) {
  const uint32_t n = g.n_members;
  // pick_subscriber/6 with one member returns it without consulting the strategy
  // (emqx_shared_sub.erl:265)
  if (n == 1) return a.members[g.member_begin];
  uint32_t idx;
  if (a.strategy == EMQX_SHARE_HASH_CLIENTID || a.strategy == EMQX_SHARE_HASH_TOPIC)
    idx = a.keys[t] % n;  // 1 + phash2(Key) rem Count, 1-based in the reference
  else  // EMQX_SHARE_RANDOM (and the fallback of a stateful pick with no room for its state)
    idx = fo_rand(a.seed, i, gidx + 0x632BE5ABu) % n;
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
  const bool need_topic = a.keys && a.strategy != EMQX_SHARE_RANDOM;
  const bool stateful = fo_stateful(a.strategy);
  const uint64_t nwaves = uint64_t(gridDim.x) * (FO_THREADS / 64);
  for (uint64_t e0 = (uint64_t(blockIdx.x) * (FO_THREADS / 64) + wv) * FO_WCHUNK; e0 < m;
       e0 += nwaves * FO_WCHUNK) {
    const uint64_t e1 = min<uint64_t>(e0 + FO_WCHUNK, m);
    const uint64_t obase = a.eoff[e0];
    const uint32_t total = static_cast<uint32_t>(a.eoff[e1] - obase);
    // the chunk's entries, EU per lane: every first-level load of the chunk is in flight
    // before the filter records are fetched, and those before anything is stored to LDS
    // (loads are unconditional, from a clamped index, and masked after: under a per-lane
    // `if` the compiler waited for each entry's loads before issuing the next entry's)
    uint32_t f[EU], tp[EU];
    uint64_t eo[EU];
    bool v[EU];
#pragma unroll
    for (uint32_t u = 0; u < EU; ++u) {
      const uint64_t i = e0 + lane + 64u * u;
      v[u] = i < e1;
      const uint64_t ic = v[u] ? i : e0;
      f[u] = a.mids[base + ic];
      eo[u] = a.eoff[ic];
      tp[u] = need_topic ? a.entry_topic[ic] : 0u;
    }
#pragma unroll
    for (uint32_t u = 0; u < EU; ++u) {
      f[u] = v[u] ? f[u] : FID_NONE;
      eo[u] = v[u] ? eo[u] : obase + total;
      tp[u] = v[u] ? tp[u] : 0u;
    }
    uint4 r[EU];
    if (a.n_recs) {
#pragma unroll
      for (uint32_t u = 0; u < EU; ++u) {
        const bool in = f[u] < a.n_recs;
        const uint4 x = *reinterpret_cast<const uint4*>(a.recs + (in ? f[u] : 0u));
        r[u] = in ? x : make_uint4(0, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (uint32_t u = 0; u < EU; ++u) r[u] = make_uint4(0, 0, 0, 0);
    }
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
        const uint32_t k = kk[u];
        const uint32_t gidx = shr[u] ? L.gb[k] + (rr[u] - L.np[k]) : 0u;
        GroupRec g{0, 0, 0, 0};
        if (shr[u]) {
          const uint4 gr = *reinterpret_cast<const uint4*>(a.groups + gidx);
          g = GroupRec{gr.x, gr.y, gr.z, gr.w};
          fl[u] |= FANOUT_SHARED_BIT;
        }
        if (!stateful) {
          if (shr[u]) sub[u] = pick_stateless(a, g, e0 + k, L.top[k], gidx);
          continue;
        }
        // round_robin / sticky: the pick is deferred to the resolve kernel, which takes this
        // publisher's picks of the slot in message order.  The output holds the group record
        // until then, and the output position joins the (slot, publisher) entry's chain.
        const uint64_t pos = obase + j0 + lane + 64u * u;
        const uint32_t pub = a.keys ? a.keys[L.top[k]] : 0u;
        bool created = false;
        const uint64_t ent = shr[u] ? ps_find_or_insert(a, (uint64_t(g.slot) << 32) | pub, &created) : PS_EMPTY;
        wave_count(a.ps_count, created);
        bool first = false;
        if (shr[u] && ent == PS_EMPTY) {  // no room: a stateless random pick, flagged
          sub[u] = pick_stateless(a, g, e0 + k, 0u, gidx);
          if (g.n_members > 1) atomicOr(a.ctl + FO_CTL_FLAGS, static_cast<unsigned long long>(FO_SUM_F_STATE_FULL));
        } else if (shr[u]) {
          sub[u] = gidx;
          // a push onto the entry's chain: one exchange, no retry loop (many lanes of a hot
          // group push at once); the chain is read only by the resolve kernel, a later launch
          const unsigned long long mine = (static_cast<unsigned long long>(a.stamp) << 32) | static_cast<uint32_t>(pos);
          const unsigned long long old = atomicExch(a.heads + ent, mine);
          first = static_cast<uint32_t>(old >> 32) != a.stamp;
          a.next[pos] = first ? SUB_NONE : static_cast<uint32_t>(old);
        }
        wave_append(a.ctl + FO_CTL_TOUCHED, a.touched, first, static_cast<uint32_t>(ent));
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

__device__ __forceinline__ bool is_member(const FanoutArgs& a, const GroupRec& g, uint32_t sub) {
  for (uint32_t i = 0; i < g.n_members; ++i)
    if (a.members[g.member_begin + i] == sub) return true;
  return false;
}

// round_robin / sticky: one thread per (slot, publisher) entry touched by this call.  Its
// chain holds the output positions of its picks (any order); they are taken in increasing
// position — message order — as the publisher's process would make them one PUBLISH at a time.
//   round_robin (do_pick_subscriber/6, :279-285): Rem = rand:uniform(N) - 1 the first time,
//     else (Last + 1) rem N; one member: that member, the state untouched (:265)
//   sticky (pick/6, :234-247): the stored member while it is still subscribed to the group,
//     else a random member, which becomes the stored one
__global__ __launch_bounds__(FO_THREADS) void fanout_resolve_kernel(FanoutArgs a) {
  const uint64_t nt = a.ctl[FO_CTL_TOUCHED];
  for (uint64_t t = blockIdx.x * uint64_t(FO_THREADS) + threadIdx.x; t < nt; t += uint64_t(gridDim.x) * FO_THREADS) {
    const uint32_t ent = a.touched[t];
    const uint32_t head = static_cast<uint32_t>(a.heads[ent]);
    const uint32_t gidx = a.out_subs[head];
    const uint4 gr = *reinterpret_cast<const uint4*>(a.groups + gidx);
    const GroupRec g{gr.x, gr.y, gr.z, gr.w};
    const uint32_t n = g.n_members;
    uint32_t val = a.ps_vals[ent];
    // positions in increasing order: the smallest one above the last taken, per step
    int64_t last = -1;
    while (true) {
      uint32_t best = SUB_NONE;
      for (uint32_t p = head; p != SUB_NONE; p = a.next[p])
        if (static_cast<int64_t>(p) > last && (best == SUB_NONE || p < best)) best = p;
      if (best == SUB_NONE) break;
      last = best;
      uint32_t pick;
      if (a.strategy == EMQX_SHARE_ROUND_ROBIN) {
        if (n == 1) {
          pick = a.members[g.member_begin];
        } else {
          val = val == PS_NOVAL ? fo_rand(a.seed, best, ent) % n : (val + 1) % n;
          pick = a.members[g.member_begin + val];
        }
      } else {  // EMQX_SHARE_STICKY
        if (val == PS_NOVAL || !is_member(a, g, val))
          val = a.members[g.member_begin + (n > 1 ? fo_rand(a.seed, best, ent) % n : 0u)];
        pick = val;
      }
      a.out_subs[best] = pick;
    }
    a.ps_vals[ent] = val;
  }
}

__global__ void fanout_finish_kernel(FanoutArgs a) {
  const unsigned long long c = *a.ps_count;
  a.summary[FO_SUM_STATE] = c;
  a.summary[FO_SUM_FLAGS] |= a.ctl[FO_CTL_FLAGS];
  if (a.ps_seen) *a.ps_seen = c;
  __threadfence_system();
}

uint32_t grid_for(uint64_t items, uint32_t per_block) {
  const uint64_t g = (items + per_block - 1) / per_block;
  return static_cast<uint32_t>(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

// ---- incremental commits of the subscription table ----------------------------------------
__global__ __launch_bounds__(256) void subtab_word_patch_kernel(uint32_t* plain, uint32_t* members,
                                                                const WordPatch* wp, uint64_t n_plain,
                                                                uint64_t n_total) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n_total; i += uint64_t(gridDim.x) * 256) {
    const WordPatch p = wp[i];
    const uint64_t idx = (uint64_t(p.index_hi) << 32) | p.index_lo;
    (i < n_plain ? plain : members)[idx] = p.value;
  }
}

// Whole 16-B records (one dwordx4 store each): a reader sees a record old or new.
__global__ __launch_bounds__(256) void subtab_rec_patch_kernel(GroupRec* groups, FilterRec* recs,
                                                               const RecPatch* rp, uint64_t n_groups,
                                                               uint64_t n_total) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n_total; i += uint64_t(gridDim.x) * 256) {
    const RecPatch p = rp[i];
    uint4* dst = i < n_groups ? reinterpret_cast<uint4*>(groups + p.index) : reinterpret_cast<uint4*>(recs + p.index);
    *dst = p.value;
  }
}

__global__ __launch_bounds__(256) void ps_rehash_kernel(const uint64_t* old_keys, const uint32_t* old_vals,
                                                        uint64_t old_cap, uint64_t* keys, uint32_t* vals,
                                                        uint64_t mask, unsigned long long* count) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < old_cap; i += uint64_t(gridDim.x) * 256) {
    const uint64_t k = old_keys[i];
    if (k == PS_EMPTY || k == PS_TOMB) continue;
    for (uint64_t j = ps_hash(k) & mask;; j = (j + 1) & mask) {
      if (atomicCAS(reinterpret_cast<unsigned long long*>(keys + j), static_cast<unsigned long long>(PS_EMPTY),
                    static_cast<unsigned long long>(k)) == PS_EMPTY) {
        vals[j] = old_vals[i];
        atomicAdd(count, 1ull);
        break;
      }
    }
  }
}

__global__ __launch_bounds__(256) void ps_forget_kernel(uint64_t* keys, uint64_t cap, const uint32_t* pubs,
                                                        uint64_t n_pubs, unsigned long long* count) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < cap; i += uint64_t(gridDim.x) * 256) {
    const uint64_t k = keys[i];
    if (k == PS_EMPTY || k == PS_TOMB) continue;
    const uint32_t p = static_cast<uint32_t>(k);
    uint64_t lo = 0, hi = n_pubs;
    while (lo < hi) {
      const uint64_t mid = (lo + hi) >> 1;
      if (pubs[mid] < p) lo = mid + 1; else hi = mid;
    }
    if (lo < n_pubs && pubs[lo] == p) {
      keys[i] = PS_TOMB;  // probes continue past it; a rehash drops it
      atomicAdd(count, ~0ull);
    }
  }
}

__global__ __launch_bounds__(256) void fanout_to_host_kernel(const uint64_t* d_off, uint64_t n, const uint32_t* d_subs,
                                                             const uint32_t* d_fil, const uint64_t* d_summary,
                                                             uint64_t cap, uint64_t* h_off, uint32_t* h_subs,
                                                             uint32_t* h_fil) {
  const uint64_t stride = uint64_t(gridDim.x) * 256;
  const uint64_t t0 = blockIdx.x * 256ull + threadIdx.x;
  for (uint64_t t = t0; t <= n; t += stride) h_off[t] = d_off[t];
  const uint64_t total = (d_summary[FO_SUM_FLAGS] & (FO_SUM_F_OVERFLOW | FO_SUM_F_MATCH)) ? 0 : d_summary[FO_SUM_TOTAL];
  if (total > cap) return;
  for (uint64_t i = t0; i < total; i += stride) {
    h_subs[i] = d_subs[i];
    h_fil[i] = d_fil[i];
  }
}

}  // namespace

hipError_t launch_fanout(const FanoutArgs& a, uint64_t m_cap, hipStream_t s) {
  const bool need_topic = a.keys && a.strategy != EMQX_SHARE_RANDOM;
  if (a.n && need_topic)
    hipLaunchKernelGGL(fanout_entry_topic_kernel, dim3(grid_for(a.n, FO_THREADS)), dim3(FO_THREADS), 0, s, a);
  hipLaunchKernelGGL(fanout_count_kernel, dim3(FO_BLOCKS), dim3(FO_THREADS), 0, s, a);
  hipLaunchKernelGGL(fanout_partials_kernel, dim3(1), dim3(FO_BLOCKS), 0, s, a);
  hipLaunchKernelGGL(fanout_final_kernel, dim3(FO_BLOCKS), dim3(FO_THREADS), 0, s, a);
  hipLaunchKernelGGL(fanout_offsets_kernel, dim3(grid_for(a.n + 1, FO_THREADS)), dim3(FO_THREADS), 0, s, a);
  // one wave per FO_WCHUNK entries up to m_cap (waves past m exit at once)
  hipLaunchKernelGGL(fanout_write_kernel, dim3(grid_for(m_cap, FO_WCHUNK * (FO_THREADS / 64))), dim3(FO_THREADS), 0, s,
                     a);
  if (fo_stateful(a.strategy)) {
    const uint64_t most = a.ps_mask + 1 < a.cap ? a.ps_mask + 1 : a.cap;  // entries touched at most
    hipLaunchKernelGGL(fanout_resolve_kernel, dim3(grid_for(most, FO_THREADS)), dim3(FO_THREADS), 0, s, a);
  }
  hipLaunchKernelGGL(fanout_finish_kernel, dim3(1), dim3(1), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_subtab_patches(uint32_t* plain, uint32_t* members, const WordPatch* wp, uint64_t n_plain_w,
                                 uint64_t n_member_w, GroupRec* groups, FilterRec* recs, const RecPatch* rp,
                                 uint64_t n_group_p, uint64_t n_rec_p, hipStream_t s) {
  // words first (the lists), then the records that point at them
  if (n_plain_w + n_member_w)
    hipLaunchKernelGGL(subtab_word_patch_kernel, dim3(grid_for(n_plain_w + n_member_w, 256)), dim3(256), 0, s, plain,
                       members, wp, n_plain_w, n_plain_w + n_member_w);
  if (n_group_p)
    hipLaunchKernelGGL(subtab_rec_patch_kernel, dim3(grid_for(n_group_p, 256)), dim3(256), 0, s, groups, recs, rp,
                       n_group_p, n_group_p);
  if (n_rec_p)
    hipLaunchKernelGGL(subtab_rec_patch_kernel, dim3(grid_for(n_rec_p, 256)), dim3(256), 0, s, groups, recs,
                       rp + n_group_p, uint64_t(0), n_rec_p);
  return hipGetLastError();
}

hipError_t launch_ps_rehash(const uint64_t* old_keys, const uint32_t* old_vals, uint64_t old_cap, uint64_t* keys,
                            uint32_t* vals, uint64_t mask, unsigned long long* count, hipStream_t s) {
  if (old_cap)
    hipLaunchKernelGGL(ps_rehash_kernel, dim3(grid_for(old_cap, 256)), dim3(256), 0, s, old_keys, old_vals, old_cap,
                       keys, vals, mask, count);
  return hipGetLastError();
}

hipError_t launch_ps_forget(uint64_t* keys, uint64_t cap, const uint32_t* pubs, uint64_t n_pubs,
                            unsigned long long* count, hipStream_t s) {
  if (cap && n_pubs)
    hipLaunchKernelGGL(ps_forget_kernel, dim3(grid_for(cap, 256)), dim3(256), 0, s, keys, cap, pubs, n_pubs, count);
  return hipGetLastError();
}

hipError_t launch_fanout_to_host(const uint64_t* d_off, uint64_t n, const uint32_t* d_subs, const uint32_t* d_fil,
                                 const uint64_t* d_summary, uint64_t cap, uint64_t* h_off, uint32_t* h_subs,
                                 uint32_t* h_fil, hipStream_t s) {
  hipLaunchKernelGGL(fanout_to_host_kernel, dim3(1024), dim3(256), 0, s, d_off, n, d_subs, d_fil, d_summary, cap, h_off,
                     h_subs, h_fil);
  return hipGetLastError();
}

}  // namespace emqx
