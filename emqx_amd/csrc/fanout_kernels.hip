// HIP kernels for gfx950: publish fan-out — matched filter ids -> subscriber deliveries.
//
// Replaces emqx_broker:route/2 + do_dispatch/2,3 (apps/emqx/src/emqx_broker.erl:244-259,
// 500-524) and emqx_shared_sub:dispatch/3 -> pick/6 -> do_pick_subscriber/6
// (apps/emqx/src/emqx_shared_sub.erl:113-126,234-288) for a whole batch of published topics.
//
// Pipeline, all on one stream with no host synchronisation: the number of
// match entries m = moff[n] - moff[0] is read on the device, so every kernel below runs a
// fixed grid over a length it loads itself.
//   entry_topic  one thread per topic: entry -> topic map (a refused or empty CSR: zero
//                offsets, as nothing else runs)
//   count        FO_BLOCKS blocks, one contiguous range of entries each: per FO_WCHUNK-entry
//                chunk the deliveries (n_plain + n_groups of each entry's filter) and picks,
//                per block their sums
//   partials     one block: exclusive scan of the block sums, the totals, the flags and the
//                call summary
//   write        one wavefront per 256 match entries: the chunk's base (its block's base + the
//                block's earlier chunks), its entries' offsets by a wave scan of the counts of
//                the records it loads anyway, the per-topic output offsets of the topics that
//                start in the chunk; then the wave walks its flattened outputs 64 at a time
//                (each lane finds its entry by an 8-step search over LDS prefix offsets), so
//                plain-subscriber copies are coalesced reads and writes; each $share group
//                contributes exactly one pick.  On overflow only the offsets are written, so
//                no pick state is consumed by a call that wrote no deliveries.
//   probe, sort, round_robin / sticky only: the write kernel puts one {position, group record,
//   resolve      publisher} record per $share pick into a list in output order; the probe kernel
//                finds each pick's (group slot, publisher) state entry and names the call's run of
//                that entry with a small id; a stable radix sort by run id makes each run one
//                segment in message order; a head thread per run takes the stored state
//                (round_robin: the run's first index; sticky: the stored subscriber, re-picked
//                while it is not alive), then every pick is made from its rank in the run in
//                parallel (O(k) per run, no chains, no same-address atomics)
//   finish       one thread: pick-state occupancy into the summary
// Bandwidth-bound streaming; no MFMA.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include "../../include/emqx_match.h"
#include "fanout.h"
#include "layout.h"

namespace emqx {

namespace {

constexpr int FO_THREADS = 256;
#ifndef FO_UNROLL_V
#define FO_UNROLL_V 4
#endif
constexpr uint32_t FO_UNROLL = FO_UNROLL_V;  // outputs per lane per round of the write kernel

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
  // the call's control words start at zero (the first kernel of the call: no memset launch)
  if (blockIdx.x == 0) {
    if (threadIdx.x < FO_CTL_WORDS) a.ctl[threadIdx.x] = 0;
    __syncthreads();
  }
  if (fo_entries(a) == 0) {  // refused or no entries: every topic's deliveries start at 0, and
                             // no chunk runs, so the summary is written here
    for (uint64_t t = blockIdx.x * uint64_t(FO_THREADS) + threadIdx.x; t <= a.n; t += uint64_t(gridDim.x) * FO_THREADS)
      a.out_off[t] = 0;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      const bool refused = fo_refused(a);
      const uint64_t fl = refused ? FO_SUM_F_MATCH : 0;
      a.summary[FO_SUM_FLAGS] = fl;
      a.summary[FO_SUM_TOTAL] = 0;
      a.summary[FO_SUM_ENTRIES] = refused ? fo_entries_raw(a) : 0;
      a.ctl[FO_CTL_PICKS] = 0;
      if (fl) atomicOr(a.ctl + FO_CTL_FLAGS, static_cast<unsigned long long>(fl));
      __threadfence_system();
    }
    return;
  }
  // a wave per 64 topics: their 65 offsets, then the entries they span written lane by lane
  // (coalesced), each lane finding its entry's topic by a 6-step search over the offsets
  __shared__ uint64_t s_off[FO_THREADS / 64][65];
  const uint32_t lane = fo_lane(), wv = threadIdx.x >> 6;
  uint64_t* so = s_off[wv];
  const uint64_t base = a.moff[0];
  const uint64_t nwaves = uint64_t(gridDim.x) * (FO_THREADS / 64);
  for (uint64_t t0 = (uint64_t(blockIdx.x) * (FO_THREADS / 64) + wv) * 64; t0 < a.n; t0 += nwaves * 64) {
    const uint64_t nt = min<uint64_t>(64, a.n - t0);
    so[lane] = a.moff[t0 + min<uint64_t>(lane, nt)] - base;
    if (lane == 0) so[64] = a.moff[t0 + nt] - base;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    const uint64_t b = so[0], e = so[nt];
    for (uint64_t i = b + lane; i < e; i += 64) {
      uint32_t k = 0;  // largest k < nt with so[k] <= i
#pragma unroll
      for (uint32_t step = 32; step >= 1; step >>= 1)
        if (k + step < nt && so[k + step] <= i) k += step;
      a.entry_topic[i] = static_cast<uint32_t>(t0 + k);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

__device__ __forceinline__ uint64_t fo_wave_sum(uint64_t v) {
#pragma unroll
  for (uint32_t d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// Chunk offsets in two passes: count: per FO_WCHUNK-entry chunk the deliveries (csum) and $share
// picks (gchunk), per block their sums; partials: one block scans the block sums and writes the
// call's totals, flags and summary; the write kernel then adds the block's earlier chunks to
// its block's base.  (A one-pass decoupled look-back in the write kernel measured slower: its
// chains of unpublished predecessors at the kernel's start, and the registers it held, cost
// more than the count kernel, profiles/r4_v16_fanout_onepass_ab.txt.)
__device__ __forceinline__ uint64_t fo_per_block(uint64_t m) {
  return ((m + FO_BLOCKS - 1) / FO_BLOCKS + FO_WCHUNK - 1) & ~static_cast<uint64_t>(FO_WCHUNK - 1);
}

__global__ __launch_bounds__(FO_THREADS) void fanout_count_kernel(FanoutArgs a) {
  __shared__ uint64_t bsum[2][FO_THREADS / 64];
  const uint64_t base = a.moff[0];
  const bool stateful = fo_stateful(a.strategy);
  const uint32_t lane = fo_lane(), wv = threadIdx.x >> 6;
  constexpr uint32_t EU = FO_WCHUNK / 64;
  const uint64_t m = fo_entries(a), per = fo_per_block(m);
  const uint64_t lo = min<uint64_t>(m, per * blockIdx.x), hi = min<uint64_t>(m, per * (blockIdx.x + 1));
  uint64_t sum = 0, gsum = 0;
  for (uint64_t c0 = lo + uint64_t(wv) * FO_WCHUNK; c0 < hi; c0 += uint64_t(FO_THREADS / 64) * FO_WCHUNK) {
    uint32_t f[EU];
#pragma unroll
    for (uint32_t u = 0; u < EU; ++u) {
      const uint64_t i = c0 + lane + 64u * u;
      f[u] = i < hi ? a.mids[base + i] : FID_NONE;
    }
    uint64_t cs = 0, gl = 0;
    uint32_t w[EU];
#pragma unroll
    for (uint32_t u = 0; u < EU; ++u) w[u] = f[u] < a.n_recs ? a.fcnt[f[u]] : 0u;
#pragma unroll
    for (uint32_t u = 0; u < EU; ++u) {
      if (w[u] == 0xFFFFFFFFu) {  // saturated: the record itself (a filter with 16 M deliveries)
        const uint4 r = a.recs[f[u]].head;
        cs += fo_rec_plain(r) + fo_rec_groups(r);
        gl += fo_rec_groups(r);
      } else {
        cs += w[u] & FO_CNT_DELIV_MAX;
        gl += w[u] >> 24;
      }
    }
    cs = fo_wave_sum(cs);
    gl = fo_wave_sum(gl);
    if (lane == 0) {
      a.csum[c0 / FO_WCHUNK] = cs;
      if (stateful) a.gchunk[c0 / FO_WCHUNK] = gl;
    }
    sum += cs;
    gsum += gl;
  }
  if (lane == 0) {
    bsum[0][wv] = sum;
    bsum[1][wv] = gsum;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0, tg = 0;
    for (uint32_t k = 0; k < FO_THREADS / 64; ++k) {
      t += bsum[0][k];
      tg += bsum[1][k];
    }
    a.partials[blockIdx.x] = t;
    a.partials[2 * FO_BLOCKS + blockIdx.x] = tg;
  }
}

__device__ __forceinline__ uint64_t fo_blocks_excl_scan(uint64_t v, uint64_t* total) {
  __shared__ uint64_t wsum[FO_BLOCKS / 64];
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
  for (uint32_t k = 0; k < FO_BLOCKS / 64; ++k) {
    before += k < w ? wsum[k] : 0;
    all += wsum[k];
  }
  __syncthreads();
  *total = all;
  return before + incl - v;
}

__global__ __launch_bounds__(FO_BLOCKS) void fanout_partials_kernel(FanoutArgs a) {
  uint64_t all = 0, picks = 0;
  a.partials[FO_BLOCKS + threadIdx.x] = fo_blocks_excl_scan(a.partials[threadIdx.x], &all);
  const bool stateful = fo_stateful(a.strategy);
  if (stateful) a.partials[3 * FO_BLOCKS + threadIdx.x] = fo_blocks_excl_scan(a.partials[2 * FO_BLOCKS + threadIdx.x], &picks);
  if (threadIdx.x == 0 && fo_entries(a)) {  // (no entries: the entry-topic kernel wrote it)
    uint64_t fl = 0;
    if (all > a.cap) fl = FO_SUM_F_OVERFLOW;
    else if (stateful && picks + 1 > a.pk_cap) fl = FO_SUM_F_PICKS;
    uint64_t* sm = a.summary;
    sm[FO_SUM_FLAGS] = fl;
    sm[FO_SUM_TOTAL] = all;
    sm[FO_SUM_ENTRIES] = fo_entries(a);
    a.ctl[FO_CTL_PICKS] = stateful ? picks : 0;
    if (fl) atomicOr(a.ctl + FO_CTL_FLAGS, static_cast<unsigned long long>(fl));
    __threadfence_system();
  }
}

__device__ __forceinline__ uint64_t ps_hash(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  return k;
}

// The state-table entry of `key`, inserting it when absent; PS_EMPTY when the table has no room
// within PS_MAX_PROBES.  *created: this lane inserted it.
__device__ __forceinline__ uint64_t ps_probe_insert(uint64_t* keys, uint64_t mask, uint64_t key, bool* created) {
  *created = false;
  uint64_t i = ps_hash(key) & mask;
  for (uint32_t p = 0; p < PS_MAX_PROBES; ++p, i = (i + 1) & mask) {
    uint64_t cur = __hip_atomic_load(keys + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == key) return i;
    if (cur == PS_EMPTY) {
      const unsigned long long old =
          atomicCAS(reinterpret_cast<unsigned long long*>(keys + i), static_cast<unsigned long long>(PS_EMPTY),
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

__device__ __forceinline__ uint64_t ps_find_or_insert(const FanoutArgs& a, uint64_t key, bool* created) {
  return ps_probe_insert(a.ps_keys, a.ps_mask, key, created);
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
  // 1 + phash2(Key) rem Count for the hash strategies; random (and the fallback of a stateful
  // pick with no room for its state): fo_rand
  const bool hash = a.strategy == EMQX_SHARE_HASH_CLIENTID || a.strategy == EMQX_SHARE_HASH_TOPIC;
  const uint32_t idx = fo_stateless_index(hash ? a.strategy : 0u, hash ? a.keys[t] : 0u, a.seed, i, gidx, n);
  return a.members[g.member_begin + idx];
}

// (5 waves per SIMD: 96 VGPRs, no spill; the compiler's own choice, 98, rounds up to 104 and 4 waves)
__global__ __launch_bounds__(FO_THREADS, 5) void fanout_write_kernel(FanoutArgs a) {
  struct WaveLds {
    uint32_t pre[FO_WCHUNK];  // entry's first output, relative to the chunk's first output
    uint32_t fid[FO_WCHUNK];
    uint32_t pb[FO_WCHUNK];
    uint32_t np[FO_WCHUNK];
    uint32_t gb[FO_WCHUNK];
    uint32_t top[FO_WCHUNK];
    uint32_t go[FO_WCHUNK];   // stateful strategies: the entry's first pick-list index
  };
  __shared__ WaveLds lds_all[FO_THREADS / 64];
  constexpr uint32_t EU = FO_WCHUNK / 64;  // entries per lane per chunk
  const uint32_t lane = fo_lane();
  const uint32_t wv = threadIdx.x >> 6;
  WaveLds& L = lds_all[wv];
  const uint64_t base = a.moff[0];
  const uint64_t m = fo_entries(a);
  const bool stateful = fo_stateful(a.strategy);
  // over cap (deliveries or picks): offsets only, no ids, no pick state consumed
  const bool ids = !(a.ctl[FO_CTL_FLAGS] & (FO_SUM_F_OVERFLOW | FO_SUM_F_PICKS));
  const uint64_t per = fo_per_block(m);
  const uint64_t nwaves = uint64_t(gridDim.x) * (FO_THREADS / 64);
  for (uint64_t e0 = (uint64_t(blockIdx.x) * (FO_THREADS / 64) + wv) * FO_WCHUNK; e0 < m;
       e0 += nwaves * FO_WCHUNK) {
    const uint64_t e1 = min<uint64_t>(e0 + FO_WCHUNK, m);
    const uint64_t blk = e0 / per;
    // the chunk's entries, EU per lane: every first-level load of the chunk is in flight
    // before the filter records are fetched, and those before anything is stored to LDS
    // (loads are unconditional, from a clamped index, and masked after: under a per-lane
    // `if` the compiler waited for each entry's loads before issuing the next entry's)
    uint32_t f[EU], tp[EU];
    bool v[EU];
#pragma unroll
    for (uint32_t u = 0; u < EU; ++u) {
      const uint64_t i = e0 + lane + 64u * u;
      v[u] = i < e1;
      const uint64_t ic = v[u] ? i : e0;
      f[u] = a.mids[base + ic];
      tp[u] = a.entry_topic[ic];
    }
    const uint32_t prev_topic = e0 ? a.entry_topic[e0 - 1] : FID_NONE;
    // the chunk's first output: its block's base + the block's chunks before it; round_robin /
    // sticky also the chunk's first pick-list index the same way (the list is in output order,
    // one pick per $share group of an entry)
    uint64_t cl = 0, gl = 0;
    for (uint64_t q = blk * per / FO_WCHUNK + lane; q < e0 / FO_WCHUNK; q += 64) {
      cl += a.csum[q];
      if (stateful) gl += a.gchunk[q];
    }
    const uint64_t obase = a.partials[FO_BLOCKS + blk] + fo_wave_sum(cl);
    uint64_t gbase = stateful ? a.partials[3 * FO_BLOCKS + blk] + fo_wave_sum(gl) : 0;
#pragma unroll
    for (uint32_t u = 0; u < EU; ++u) f[u] = v[u] ? f[u] : FID_NONE;
    uint4 r[EU];
    if (a.n_recs) {
#pragma unroll
      for (uint32_t u = 0; u < EU; ++u) {
        const bool in = f[u] < a.n_recs;
        const uint4 x = a.recs[in ? f[u] : 0u].head;
        r[u] = in ? x : make_uint4(0, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (uint32_t u = 0; u < EU; ++u) r[u] = make_uint4(0, 0, 0, 0);
    }
    // entry offsets: exclusive scan of the entries' counts in entry order (k = lane + 64 u);
    // entries past the chunk count 0, so their offset is the chunk's total
    uint32_t total = 0;
    uint32_t pre[EU];
#pragma unroll
    for (uint32_t u = 0; u < EU; ++u) {
      const uint32_t c = fo_rec_plain(r[u]) + fo_rec_groups(r[u]);
      uint32_t incl = c;
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
      }
      pre[u] = total + incl - c;
      total += __shfl(incl, 63, 64);
    }
    // per-topic offsets: the first entry of a topic writes its offset for it and for the
    // entry-less topics just before it; the chunk holding the last entry, for those after it
#pragma unroll
    for (uint32_t u = 0; u < EU; ++u) {
      const uint32_t up = __shfl_up(tp[u], 1, 64);
      const uint32_t last_prev = u ? __shfl(tp[u ? u - 1 : 0], 63, 64) : prev_topic;
      const uint32_t pt = lane ? up : last_prev;
      if (v[u] && tp[u] != pt)
        for (uint64_t t = pt == FID_NONE ? 0 : uint64_t(pt) + 1; t <= tp[u]; ++t) a.out_off[t] = obase + pre[u];
    }
    if (e1 == m && lane == 0)
      for (uint64_t t = uint64_t(a.entry_topic[m - 1]) + 1; t <= a.n; ++t) a.out_off[t] = obase + total;
    if (!ids) continue;
#pragma unroll
    for (uint32_t u = 0; u < EU; ++u) {
      const uint32_t k = lane + 64u * u;
      L.pre[k] = pre[u];  // past the chunk's end: `total`
      L.fid[k] = f[u];
      L.pb[k] = r[u].x;   // inline record: its first subscriber
      L.np[k] = r[u].y;   // with FO_INLINE_BIT
      L.gb[k] = r[u].z;   // inline: the second
      L.go[k] = r[u].w;   // inline: the third (stateful: replaced below for records with groups)
      L.top[k] = v[u] ? tp[u] : 0u;
    }
    if (stateful) {  // entry k's first pick-list index: exclusive scan of n_groups in entry order
#pragma unroll
      for (uint32_t u = 0; u < EU; ++u) {
        const uint32_t g = fo_rec_groups(r[u]);
        uint32_t incl = g;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
          const uint32_t y = __shfl_up(incl, d, 64);
          if (lane >= d) incl += y;
        }
        if (g) L.go[lane + 64u * u] = static_cast<uint32_t>(gbase) + incl - g;
        gbase += __shfl(incl, 63, 64);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    // FO_UNROLL outputs per lane per round: all plain-subscriber loads of the round are in
    // flight before the first store ($share picks, ~10 % of entries, resolve after them).
    for (uint32_t j0 = 0; j0 < total; j0 += 64 * FO_UNROLL) {
      uint32_t sub[FO_UNROLL], fl[FO_UNROLL], kk[FO_UNROLL], rr[FO_UNROLL];
      bool act[FO_UNROLL], shr[FO_UNROLL];
      // per output j, the largest k with pre[k] <= j (pre is non-decreasing, pre[0] = 0, slots
      // past the chunk's entries hold `total`; k + step never exceeds FO_WCHUNK - 1): the
      // FO_UNROLL searches advance step by step together, their LDS reads in flight at once
      uint32_t jj[FO_UNROLL];
#pragma unroll
      for (uint32_t u = 0; u < FO_UNROLL; ++u) {
        jj[u] = j0 + lane + 64u * u;
        kk[u] = 0;
      }
#pragma unroll
      for (uint32_t step = FO_WCHUNK / 2; step >= 1; step >>= 1) {
        uint32_t c[FO_UNROLL];
#pragma unroll
        for (uint32_t u = 0; u < FO_UNROLL; ++u) c[u] = L.pre[kk[u] + step];
#pragma unroll
        for (uint32_t u = 0; u < FO_UNROLL; ++u) kk[u] += c[u] <= jj[u] ? step : 0u;
      }
#pragma unroll
      for (uint32_t u = 0; u < FO_UNROLL; ++u) {
        const uint32_t j = jj[u];
        act[u] = j < total;
        const uint32_t k = kk[u];
        rr[u] = j - L.pre[k];
        fl[u] = L.fid[k];
        const uint32_t npr = L.np[k], np = npr & ~FO_INLINE_BIT;
        const bool inl = (npr & FO_INLINE_BIT) != 0;
        shr[u] = act[u] && rr[u] >= np;
        // the load stays unconditional (all of a round's in flight together): an arena output
        // reads its plain entry, an inline one past the head its record's ext word (the line the
        // record load just brought in), any other output plain[0], discarded
        const bool arena = act[u] && !shr[u] && !inl;
        const bool ext = act[u] && !shr[u] && inl && rr[u] >= FO_INLINE_HEAD;
        const uint32_t x = *(ext ? fo_inline_ext(a.recs, fl[u], rr[u]) : a.plain + (arena ? L.pb[k] + rr[u] : 0u));
        const uint32_t iv = rr[u] == 0 ? L.pb[k] : (rr[u] == 1 ? L.gb[k] : L.go[k]);
        sub[u] = (act[u] && !shr[u]) ? ((inl && rr[u] < FO_INLINE_HEAD) ? iv : x) : 0u;
      }
#pragma unroll
      for (uint32_t u = 0; u < FO_UNROLL; ++u) {
        if (!shr[u]) continue;
        const uint32_t k = kk[u];
        const uint32_t gidx = L.gb[k] + (rr[u] - L.np[k]);  // (a record with groups is never inline)
        fl[u] |= FANOUT_SHARED_BIT;
        if (!stateful) {
          const uint4 gr = *reinterpret_cast<const uint4*>(a.groups + gidx);
          sub[u] = pick_stateless(a, GroupRec{gr.x, gr.y, gr.z, gr.w}, e0 + k, L.top[k], gidx);
          continue;
        }
        // round_robin / sticky: the pick is made after the write by the probe / resolve kernels,
        // which take each (slot, publisher) entry's picks in message order.  The output holds the
        // group record until then; the pick goes to the list at its place in output order (the
        // entry's first pick-list index + its group's rank in the entry) as {position, group
        // record, publisher} (the group's record is not loaded here: the probe kernel reads its
        // slot off this kernel's critical path).
        const uint32_t li = L.go[k] + (rr[u] - L.np[k]);
        a.pk_vals[li] = static_cast<uint32_t>(obase + j0 + lane + 64u * u);
        a.pk_skeys[li] = gidx;
        a.pk_svals[li] = a.keys ? a.keys[L.top[k]] : 0u;
        sub[u] = gidx;
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

// The pick list's runs: per pick, the (group slot, publisher) entry of the state table (inserted
// when absent; in parallel over the list, off the write kernel's critical path) and the call's
// run id of that entry: the list index of the first pick that names it (no counter, no atomics
// on a shared word); past the call's picks the pad key pk_cap - 1, which sorts last.  run_cnt
// (small path): picks per run.  Runs named, per block, to run_named[block] (the finish kernel
// adds them up).  A fixed grid of at most FO_BLOCKS blocks strides over the list.
__global__ __launch_bounds__(FO_THREADS) void fanout_pick_probe_kernel(FanoutArgs a) {
  __shared__ uint32_t s_named[FO_THREADS / 64];
  if (a.ctl[FO_CTL_FLAGS] & (FO_SUM_F_OVERFLOW | FO_SUM_F_PICKS | FO_SUM_F_MATCH)) {
    if (threadIdx.x == 0) a.run_named[blockIdx.x] = 0;
    return;
  }
  const uint64_t S = a.ctl[FO_CTL_PICKS];
  const uint32_t pad = static_cast<uint32_t>(a.pk_cap - 1);
  const uint64_t stride = uint64_t(gridDim.x) * FO_THREADS;
  uint32_t named = 0;
  for (uint64_t i0 = blockIdx.x * uint64_t(FO_THREADS); i0 < a.pk_cap; i0 += stride) {
    const uint64_t i = i0 + threadIdx.x;
    const bool pick = i < S;
    bool created = false;
    uint64_t ent = PS_EMPTY;
    if (pick) {
      const uint32_t slot = a.groups[a.pk_skeys[i]].slot;
      ent = ps_find_or_insert(a, (uint64_t(slot) << 32) | a.pk_svals[i], &created);
      if (ent == PS_EMPTY) atomicOr(a.ctl + FO_CTL_FLAGS, static_cast<unsigned long long>(FO_SUM_F_STATE_FULL));
      a.pk_svals[i] = static_cast<uint32_t>(ent);  // (the small path reads a pick's entry here)
    }
    wave_count(a.ps_count, created);
    uint32_t key = pad;
    if (ent != PS_EMPTY) {
      unsigned long long* t = a.tag + ent;
      const unsigned long long cur = __hip_atomic_load(t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (static_cast<uint32_t>(cur >> 32) == a.stamp) {
        key = static_cast<uint32_t>(cur);
      } else {
        const unsigned long long mine = (static_cast<unsigned long long>(a.stamp) << 32) | static_cast<uint32_t>(i);
        const unsigned long long prev = atomicCAS(t, cur, mine);
        if (prev == cur) {
          key = static_cast<uint32_t>(i);
          a.run_ent[i] = static_cast<uint32_t>(ent);
          ++named;
        } else {
          key = static_cast<uint32_t>(prev);  // another pick of this call named the run first
        }
      }
      if (a.run_cnt) atomicAdd(a.run_cnt + key, 1u);
    }
    if (i < a.pk_cap) a.pk_keys[i] = key;
  }
  const uint32_t wn = static_cast<uint32_t>(fo_wave_sum(named));
  if (fo_lane() == 0) s_named[threadIdx.x >> 6] = wn;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (uint32_t k = 0; k < FO_THREADS / 64; ++k) t += s_named[k];
    a.run_named[blockIdx.x] = t;
  }
}

// The idx-th member of g that is not `excl` (count = members - [excl] > idx); member order.
__device__ __forceinline__ uint32_t nth_member_except(const FanoutArgs& a, const GroupRec& g, uint32_t excl,
                                                      uint32_t idx) {
  for (uint32_t i = 0; i < g.n_members; ++i) {
    const uint32_t s = a.members[g.member_begin + i];
    if (s == excl) continue;
    if (idx == 0) return s;
    --idx;
  }
  return SUB_NONE;
}

__device__ __forceinline__ bool fo_busy_flags(const FanoutArgs& a) { return a.ctl[FO_CTL_FLAGS] != 0; }

__device__ __forceinline__ GroupRec fo_group(const FanoutArgs& a, uint32_t gidx) {
  const uint4 gr = *reinterpret_cast<const uint4*>(a.groups + gidx);
  return GroupRec{gr.x, gr.y, gr.z, gr.w};
}

// round_robin, one message (do_pick_subscriber/6, :279-285): Rem = rand:uniform(N) - 1 without
// state, else (Last + 1) rem N; with one member the state is neither consulted nor changed (:265).
__device__ __forceinline__ uint32_t rr_step(const FanoutArgs& a, const GroupRec& g, uint32_t* val, uint32_t pos,
                                            uint32_t ent) {
  const uint32_t n = g.n_members;
  if (n <= 1) return a.members[g.member_begin];
  *val = *val == PS_NOVAL ? (a.rr_first0 ? 0u : fo_rand(a.seed, pos, ent) % n) : (*val + 1) % n;
  return a.members[g.member_begin + *val];
}

// sticky, one message (pick/6, :234-247): the stored subscriber while its process is alive
// (is_active_sub/2 with no failed subscribers, :386-393; membership is not checked), else
// do_pick(random, ..., [Sub0]) (:243): a random member other than Sub0, or {retry, any member}
// when Sub0 is the only one (:251-263); the pick is stored (:245).
__device__ __forceinline__ uint32_t sticky_step(const FanoutArgs& a, const GroupRec& g, uint32_t* val, uint32_t pos,
                                                uint32_t ent, bool* retry) {
  *retry = false;
  if (fo_alive(a.alive, a.n_alive_words, *val)) return *val;
  const uint32_t n = g.n_members;
  bool in = false;  // Sub0 among the members?
  for (uint32_t q = 0; q < n && !in; ++q) in = a.members[g.member_begin + q] == *val;
  const uint32_t cnt = in ? n - 1 : n;
  uint32_t pick;
  if (cnt == 0) {  // All -- [Sub0] = []: {retry, the only member}
    pick = a.members[g.member_begin];
    *retry = true;
  } else {
    pick = nth_member_except(a, g, *val, cnt > 1 ? fo_rand(a.seed, pos, ent) % cnt : 0u);
  }
  *val = pick;
  return pick;
}

__device__ __forceinline__ void fo_put_pick(const FanoutArgs& a, uint32_t pos, uint32_t sub, bool retry) {
  a.out_subs[pos] = sub;
  if (retry && a.out_filters) a.out_filters[pos] |= FANOUT_RETRY_BIT;
}

// ---- large path (many picks per run: few publishers) ---------------------------------------
// Resolve, part 1: one thread per run (its first element in the sorted list; the run's positions
// are in message order): round_robin's first index of the run; sticky's picks made message by
// message until the stored subscriber is alive, from where on the run is constant.
__global__ __launch_bounds__(FO_THREADS) void fanout_resolve_heads_kernel(FanoutArgs a) {
  if (fo_busy_flags(a)) return;  // nothing resolved: the call is rerun
  const uint64_t S = a.ctl[FO_CTL_PICKS];
  const bool sticky = a.strategy == EMQX_SHARE_STICKY;
  for (uint64_t i = blockIdx.x * uint64_t(FO_THREADS) + threadIdx.x; i < S; i += uint64_t(gridDim.x) * FO_THREADS) {
    const uint32_t k = a.pk_skeys[i];
    if (k + 1 >= a.pk_cap || (i > 0 && a.pk_skeys[i - 1] == k)) continue;
    const uint32_t ent = a.run_ent[k];
    const uint32_t pos = a.pk_svals[i];
    const GroupRec g = fo_group(a, a.out_subs[pos]);
    uint32_t val = a.ps_vals[ent];
    if (!sticky) {
      const uint32_t n = g.n_members;
      const uint32_t first =
          n <= 1 ? 0u : (val == PS_NOVAL ? (a.rr_first0 ? 0u : fo_rand(a.seed, pos, ent) % n) : (val + 1) % n);
      a.seg[k] = static_cast<unsigned long long>(i) | (static_cast<unsigned long long>(first) << 32);
      continue;
    }
    uint64_t j = i;
    for (; j < S && a.pk_skeys[j] == k; ++j) {
      if (fo_alive(a.alive, a.n_alive_words, val)) break;  // constant from here on
      const uint32_t p = a.pk_svals[j];
      bool retry;
      fo_put_pick(a, p, sticky_step(a, g, &val, p, ent, &retry), retry);
    }
    a.seg[k] = static_cast<unsigned long long>(i) | (static_cast<unsigned long long>(val) << 32);
    a.seg_from[k] = static_cast<uint32_t>(j);
    a.ps_vals[ent] = val;
  }
}

// Resolve, part 2: every pick of the list from its run's first pick and its rank in the run;
// the last pick of a round_robin run stores the state.
__global__ __launch_bounds__(FO_THREADS) void fanout_resolve_apply_kernel(FanoutArgs a) {
  if (fo_busy_flags(a)) return;
  const uint64_t S = a.ctl[FO_CTL_PICKS];
  const bool sticky = a.strategy == EMQX_SHARE_STICKY;
  for (uint64_t i = blockIdx.x * uint64_t(FO_THREADS) + threadIdx.x; i < S; i += uint64_t(gridDim.x) * FO_THREADS) {
    const uint32_t k = a.pk_skeys[i];
    if (k + 1 >= a.pk_cap) continue;
    const uint32_t pos = a.pk_svals[i];
    const unsigned long long sg = a.seg[k];
    const uint32_t start = static_cast<uint32_t>(sg), first = static_cast<uint32_t>(sg >> 32);
    if (sticky) {
      if (i >= a.seg_from[k]) a.out_subs[pos] = first;  // (earlier ones: written by the head)
      continue;
    }
    const uint32_t gidx = a.out_subs[pos];
    const uint4 gr = *reinterpret_cast<const uint4*>(a.groups + gidx);
    const uint32_t n = gr.y;
    if (n <= 1) {
      a.out_subs[pos] = a.members[gr.x];
      continue;
    }
    const uint32_t idx = static_cast<uint32_t>((first + (i - start)) % n);
    a.out_subs[pos] = a.members[gr.x + idx];
    if (i + 1 == S || a.pk_skeys[i + 1] != k) a.ps_vals[a.run_ent[k]] = idx;
  }
}

// ---- small path (few picks per run: many publishers) -----------------------------------------
// No sort: a run of one pick (the common case) is resolved where it lies; the picks of runs with
// more than one are gathered (at most FO_MULTI_CAP of them), sorted by (run, list index) in LDS
// by one block and resolved run by run.  A call with more multi-pick picks is flagged before any
// state is consumed and rerun on the large path.
__global__ __launch_bounds__(FO_THREADS) void fanout_pick_classify_kernel(FanoutArgs a) {
  if (fo_busy_flags(a)) return;
  const uint64_t S = a.ctl[FO_CTL_PICKS];
  const uint32_t lane = fo_lane();
  const uint64_t stride = uint64_t(gridDim.x) * FO_THREADS;
  for (uint64_t i0 = blockIdx.x * uint64_t(FO_THREADS); i0 < S; i0 += stride) {
    const uint64_t i = i0 + threadIdx.x;
    const uint32_t k = i < S ? a.pk_keys[i] : a.pk_cap - 1;
    const bool multi = k + 1 < a.pk_cap && a.run_cnt[k] > 1;
    const uint64_t m = __ballot(multi);
    if (!m) continue;
    const uint32_t leader = __ffsll(static_cast<long long>(m)) - 1;
    unsigned long long base = 0;
    if (lane == leader) base = atomicAdd(a.ctl + FO_CTL_MULTI, static_cast<unsigned long long>(__popcll(m)));
    base = __shfl(base, leader, 64);
    const uint64_t slot = base + __popcll(m & ((1ull << lane) - 1));
    if (multi && slot < FO_MULTI_CAP) a.multi[slot] = (static_cast<unsigned long long>(k) << 32) | static_cast<uint32_t>(i);
  }
}

__global__ __launch_bounds__(1024) void fanout_resolve_small_kernel(FanoutArgs a) {
  __shared__ unsigned long long srt[FO_MULTI_CAP];
  if (fo_busy_flags(a)) return;
  const uint64_t M = a.ctl[FO_CTL_MULTI];
  if (M > FO_MULTI_CAP) {  // too many: nothing consumed, the host reruns on the large path
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr(a.ctl + FO_CTL_FLAGS, static_cast<unsigned long long>(FO_SUM_F_PICKS));
    return;
  }
  const uint64_t S = a.ctl[FO_CTL_PICKS];
  const bool sticky = a.strategy == EMQX_SHARE_STICKY;
  if (blockIdx.x == 0) {
    if (M == 0) return;
    uint32_t P = 1;
    while (P < M) P <<= 1;
    for (uint32_t t = threadIdx.x; t < P; t += 1024) srt[t] = t < M ? a.multi[t] : ~0ull;
    __syncthreads();
    for (uint32_t k2 = 2; k2 <= P; k2 <<= 1)  // bitonic sort by (run, list index)
      for (uint32_t j = k2 >> 1; j > 0; j >>= 1) {
        for (uint32_t t = threadIdx.x; t < P; t += 1024) {
          const uint32_t o = t ^ j;
          if (o > t) {
            const unsigned long long x = srt[t], y = srt[o];
            if (((t & k2) == 0) == (x > y)) {
              srt[t] = y;
              srt[o] = x;
            }
          }
        }
        __syncthreads();
      }
    for (uint32_t t = threadIdx.x; t < M; t += 1024) {  // a thread per run, in message order
      const uint32_t k = static_cast<uint32_t>(srt[t] >> 32);
      if (t > 0 && static_cast<uint32_t>(srt[t - 1] >> 32) == k) continue;
      const uint32_t ent = a.run_ent[k];
      uint32_t val = a.ps_vals[ent];
      for (uint32_t u = t; u < M && static_cast<uint32_t>(srt[u] >> 32) == k; ++u) {
        const uint32_t pos = a.pk_vals[static_cast<uint32_t>(srt[u])];
        const GroupRec g = fo_group(a, a.out_subs[pos]);
        bool retry = false;
        const uint32_t sub = sticky ? sticky_step(a, g, &val, pos, ent, &retry) : rr_step(a, g, &val, pos, ent);
        fo_put_pick(a, pos, sub, retry);
      }
      a.ps_vals[ent] = val;
    }
    return;
  }
  // the other blocks: runs of one pick (the pick's entry, group record and position were left
  // in the list by the write and probe kernels: no chain through out_subs / run_ent)
  for (uint64_t i = (blockIdx.x - 1) * 1024ull + threadIdx.x; i < S; i += uint64_t(gridDim.x - 1) * 1024) {
    const uint32_t k = a.pk_keys[i];
    const uint32_t ent = a.pk_svals[i], gidx = a.pk_skeys[i], pos = a.pk_vals[i];
    if (k + 1 >= a.pk_cap || a.run_cnt[k] != 1) continue;
    const GroupRec g = fo_group(a, gidx);
    uint32_t val = a.ps_vals[ent];
    bool retry = false;
    const uint32_t sub = sticky ? sticky_step(a, g, &val, pos, ent, &retry) : rr_step(a, g, &val, pos, ent);
    fo_put_pick(a, pos, sub, retry);
    a.ps_vals[ent] = val;
  }
}

// One block of FO_THREADS: the call summary's state words; stateful calls add up the probe
// kernel's per-block run counts.
__global__ __launch_bounds__(FO_THREADS) void fanout_finish_kernel(FanoutArgs a, uint32_t probe_blocks) {
  uint64_t named = 0;
  if (a.run_named)
    for (uint32_t b = threadIdx.x; b < probe_blocks; b += FO_THREADS) named += a.run_named[b];
  named = fo_wave_sum(named);
  __shared__ uint64_t s_n[FO_THREADS / 64];
  if (fo_lane() == 0) s_n[threadIdx.x >> 6] = named;
  __syncthreads();
  if (threadIdx.x != 0) return;
  named = 0;
  for (uint32_t k = 0; k < FO_THREADS / 64; ++k) named += s_n[k];
  const unsigned long long c = *a.ps_count;
  a.summary[FO_SUM_STATE] = c;
  a.summary[FO_SUM_FLAGS] |= a.ctl[FO_CTL_FLAGS];
  if (a.ps_seen) {
    a.ps_seen[0] = c;
    a.ps_seen[1] = *a.ps_tombs;
    a.ps_seen[2] = a.ctl[FO_CTL_PICKS];
    a.ps_seen[3] = named;
  }
  if (a.call_seen) {
    a.call_seen[0] = a.ctl[FO_CTL_PICKS];
    a.call_seen[1] = named;
  }
  __threadfence_system();
}

// ---- emqx_shared_sub:dispatch/4 retries (emqx_shared_sub.erl:118-130,234-288) ----------------
// One wave, requests in order (each sees the state the previous ones left).  Lanes share the
// member scans: a member is "failed" when it is in the request's FailedSubs (or is the excluded
// sticky subscriber).
__device__ __forceinline__ bool rp_excluded(const RepickArgs& a, uint64_t f0, uint64_t f1, uint32_t extra,
                                            uint32_t s) {
  if (s == extra) return true;
  for (uint64_t q = f0; q < f1; ++q)
    if (a.failed[q] == s) return true;
  return false;
}

// Lane 0 only: the request's state entry (inserted when absent) and its value.
__device__ __forceinline__ uint64_t rp_entry(const RepickArgs& a, uint64_t key, uint32_t* val) {
  bool created = false;
  const uint64_t ent = ps_probe_insert(a.ps_keys, a.ps_mask, key, &created);
  if (created) atomicAdd(a.ps_count, 1ull);
  if (ent == PS_EMPTY) atomicOr(a.ctl, static_cast<unsigned long long>(FO_SUM_F_STATE_FULL));
  *val = ent == PS_EMPTY ? PS_NOVAL : __hip_atomic_load(a.ps_vals + ent, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return ent;
}

__device__ __forceinline__ void rp_store(const RepickArgs& a, uint64_t ent, uint32_t v) {
  __hip_atomic_store(a.ps_vals + ent, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(64) void share_repick_kernel(RepickArgs a) {
  const uint32_t lane = fo_lane();
  for (uint64_t r = 0; r < a.n; ++r) {
    const uint32_t f = a.filter_ids[r], grp = a.group_ids[r], key = a.keys ? a.keys[r] : 0u;
    const uint64_t f0 = a.failed_off[r], f1 = a.failed_off[r + 1];
    // the group's record: the filter's live groups, searched by the lanes
    GroupRec g{0, 0, 0, 0};
    bool found = false;
    if (f < a.n_recs) {
      const uint4 h = a.recs[f].head;
      const FilterRec fr{h.x, h.y, h.z, h.w};
      const uint32_t ngr = fo_rec_groups(h);
      for (uint32_t q0 = 0; q0 < ngr && !found; q0 += 64) {
        const uint32_t q = q0 + lane;
        const bool hit = q < ngr && a.groups[fr.group_begin + q].group_id == grp;
        const uint64_t m = __ballot(hit);
        if (m) {
          g = a.groups[fr.group_begin + q0 + __ffsll(static_cast<long long>(m)) - 1];
          found = true;
        }
      }
    }
    uint32_t pick = SUB_NONE, kind = EMQX_PICK_NONE;
    if (found && g.n_members) {
      const uint64_t skey = (uint64_t(g.slot) << 32) | key;
      uint32_t extra = SUB_NONE;  // sticky: Sub0 joins the excluded list
      uint32_t strategy = a.strategy;
      uint64_t sent = PS_EMPTY;
      bool done = false;
      if (strategy == EMQX_SHARE_STICKY) {
        uint32_t v = PS_NOVAL;
        if (lane == 0) sent = rp_entry(a, skey, &v);
        sent = __shfl(sent, 0, 64);
        v = __shfl(v, 0, 64);
        if (fo_alive(a.alive, a.n_alive_words, v) && !rp_excluded(a, f0, f1, SUB_NONE, v)) {
          pick = v;  // is_active_sub(Sub0, FailedSubs): {fresh, Sub0}
          kind = EMQX_PICK_FRESH;
          done = true;
        } else {
          extra = v;
          strategy = EMQX_SHARE_RANDOM;  // do_pick(random, ..., [Sub0 | FailedSubs])
        }
      }
      if (!done) {
        // Subs = All -- Excluded (member order); [] -> {retry, pick over All}
        uint32_t cnt = 0;
        for (uint32_t q0 = 0; q0 < g.n_members; q0 += 64) {
          const uint32_t q = q0 + lane;
          const bool keep = q < g.n_members && !rp_excluded(a, f0, f1, extra, a.members[g.member_begin + q]);
          cnt += __popcll(__ballot(keep));
        }
        const bool retry = cnt == 0;
        const uint32_t count = retry ? g.n_members : cnt;
        uint32_t idx = 0;
        if (count > 1) {  // pick_subscriber/6 with one candidate: it, no strategy (:265)
          if (strategy == EMQX_SHARE_HASH_CLIENTID || strategy == EMQX_SHARE_HASH_TOPIC) {
            idx = key % count;
          } else if (strategy == EMQX_SHARE_ROUND_ROBIN) {
            if (lane == 0) {
              uint32_t last = PS_NOVAL;
              const uint64_t ent = rp_entry(a, skey, &last);
              idx = last == PS_NOVAL ? (a.rr_first0 ? 0u : fo_rand(a.seed, r, g.slot) % count) : (last + 1) % count;
              if (ent != PS_EMPTY) rp_store(a, ent, idx);
            }
            idx = __shfl(idx, 0, 64);
          } else {
            idx = fo_rand(a.seed, r, g.slot + 0x632BE5ABu) % count;
          }
        }
        // the idx-th kept member
        uint32_t seen = 0;
        for (uint32_t q0 = 0; q0 < g.n_members && pick == SUB_NONE; q0 += 64) {
          const uint32_t q = q0 + lane;
          const uint32_t s = q < g.n_members ? a.members[g.member_begin + q] : SUB_NONE;
          const bool keep = q < g.n_members && (retry || !rp_excluded(a, f0, f1, extra, s));
          const uint64_t m = __ballot(keep);
          const uint32_t c = __popcll(m);
          if (idx < seen + c) {
            // the (idx - seen)-th set bit of m
            uint64_t mm = m;
            for (uint32_t t = idx - seen; t; --t) mm &= mm - 1;
            const uint32_t src = __ffsll(static_cast<long long>(mm)) - 1;
            pick = __shfl(s, src, 64);
          }
          seen += c;
        }
        kind = retry ? EMQX_PICK_RETRY : EMQX_PICK_FRESH;
        if (a.strategy == EMQX_SHARE_STICKY && sent != PS_EMPTY && lane == 0)
          rp_store(a, sent, pick);  // stick to whatever was picked (:245)
      }
    }
    if (lane == 0) {
      a.out_subs[r] = pick;
      a.out_kind[r] = kind;
    }
    __threadfence();
    __builtin_amdgcn_wave_barrier();
  }
}

uint32_t grid_for(uint64_t items, uint32_t per_block) {
  const uint64_t g = (items + per_block - 1) / per_block;
  return static_cast<uint32_t>(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

uint32_t probe_blocks(uint64_t pk_cap) {
  const uint32_t g = grid_for(pk_cap, FO_THREADS);
  return g < FO_BLOCKS ? g : FO_BLOCKS;
}

// ---- incremental commits of the subscription table ----------------------------------------
__global__ __launch_bounds__(256) void subtab_word_patch_kernel(uint32_t* plain, uint32_t* members, uint32_t* alive,
                                                                const WordPatch* wp, uint64_t n_plain,
                                                                uint64_t n_plain_members, uint64_t n_total) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n_total; i += uint64_t(gridDim.x) * 256) {
    const WordPatch p = wp[i];
    const uint64_t idx = (uint64_t(p.index_hi) << 32) | p.index_lo;
    (i < n_plain ? plain : (i < n_plain_members ? members : alive))[idx] = p.value;
  }
}

// Whole records (a group's one dwordx4 store, a filter's two: head and ext; no fan-out reads them
// meanwhile, commits are ordered after the fan-outs in flight and before the next ones).
__global__ __launch_bounds__(256) void subtab_rec_patch_kernel(GroupRec* groups, DevRec* recs, uint32_t* fcnt,
                                                               const RecPatch* rp, uint64_t n_groups,
                                                               uint64_t n_total) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n_total; i += uint64_t(gridDim.x) * 256) {
    const RecPatch p = rp[i];
    if (i < n_groups) {
      *reinterpret_cast<uint4*>(groups + p.index) = p.value;
    } else {
      recs[p.index].head = p.value;
      recs[p.index].ext = p.ext;
      fcnt[p.index] = fo_cnt_word(p.value);
    }
  }
}

__global__ __launch_bounds__(256) void fcnt_from_recs_kernel(const DevRec* recs, uint64_t n, uint32_t* fcnt) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += uint64_t(gridDim.x) * 256)
    fcnt[i] = fo_cnt_word(recs[i].head);
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
                                                        uint64_t n_pubs, unsigned long long* count,
                                                        unsigned long long* tombs) {
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
      atomicAdd(tombs, 1ull);
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
  const uint64_t total =
      (d_summary[FO_SUM_FLAGS] & (FO_SUM_F_OVERFLOW | FO_SUM_F_MATCH | FO_SUM_F_PICKS)) ? 0 : d_summary[FO_SUM_TOTAL];
  if (total > cap) return;
  for (uint64_t i = t0; i < total; i += stride) {
    h_subs[i] = d_subs[i];
    h_fil[i] = d_fil[i];
  }
}

}  // namespace

hipError_t launch_fanout(const FanoutArgs& a, uint64_t m_cap, hipStream_t s) {
  hipLaunchKernelGGL(fanout_entry_topic_kernel, dim3(grid_for(a.n + 1, FO_THREADS)), dim3(FO_THREADS), 0, s, a);
  hipLaunchKernelGGL(fanout_count_kernel, dim3(FO_BLOCKS), dim3(FO_THREADS), 0, s, a);
  hipLaunchKernelGGL(fanout_partials_kernel, dim3(1), dim3(FO_BLOCKS), 0, s, a);
  // one wave per FO_WCHUNK entries up to m_cap (waves past m exit at once)
  hipLaunchKernelGGL(fanout_write_kernel, dim3(grid_for(m_cap, FO_WCHUNK * (FO_THREADS / 64))), dim3(FO_THREADS), 0, s,
                     a);
  if (fo_stateful(a.strategy))
    hipLaunchKernelGGL(fanout_pick_probe_kernel, dim3(probe_blocks(a.pk_cap)), dim3(FO_THREADS), 0, s, a);
  else
    hipLaunchKernelGGL(fanout_finish_kernel, dim3(1), dim3(FO_THREADS), 0, s, a, 0u);
  return hipGetLastError();
}

// Onesweep at every size (rocprim's default takes its merge sort below 1M items: three times
// slower on these keys).
using PickSortConfig = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                                  rocprim::default_config, 0>;

uint32_t pick_key_bits(uint64_t pk_cap) {  // run ids and the pad key are < pk_cap
  uint32_t b = 1;
  while (b < 32 && (1ull << b) < pk_cap) ++b;
  return b;
}

uint64_t fanout_sort_temp_bytes(uint64_t pk_cap) {
  size_t bytes = 0;
  (void)rocprim::radix_sort_pairs<PickSortConfig>(nullptr, bytes, static_cast<const uint32_t*>(nullptr),
                                                  static_cast<uint32_t*>(nullptr), static_cast<const uint32_t*>(nullptr),
                                                  static_cast<uint32_t*>(nullptr), static_cast<size_t>(pk_cap), 0u,
                                                  pick_key_bits(pk_cap));
  return bytes;
}

hipError_t launch_fanout_resolve(const FanoutArgs& a, void* sort_temp, uint64_t sort_temp_bytes, hipStream_t s) {
  if (a.run_cnt) {  // small path
    hipLaunchKernelGGL(fanout_pick_classify_kernel, dim3(grid_for(a.pk_cap, FO_THREADS * 4)), dim3(FO_THREADS), 0, s, a);
    hipLaunchKernelGGL(fanout_resolve_small_kernel, dim3(1 + grid_for(a.pk_cap, 1024)), dim3(1024), 0, s, a);
    hipLaunchKernelGGL(fanout_finish_kernel, dim3(1), dim3(FO_THREADS), 0, s, a, probe_blocks(a.pk_cap));
    return hipGetLastError();
  }
  // large path: stable by run: each run keeps output (message) order; the pad sorts last
  size_t tb = sort_temp_bytes;
  hipError_t e = rocprim::radix_sort_pairs<PickSortConfig>(sort_temp, tb, a.pk_keys, a.pk_skeys, a.pk_vals,
                                                           a.pk_svals, static_cast<size_t>(a.pk_cap), 0u,
                                                           pick_key_bits(a.pk_cap), s);
  if (e != hipSuccess) return e;
  const uint32_t grid = grid_for(a.pk_cap, FO_THREADS * 4);
  hipLaunchKernelGGL(fanout_resolve_heads_kernel, dim3(grid), dim3(FO_THREADS), 0, s, a);
  hipLaunchKernelGGL(fanout_resolve_apply_kernel, dim3(grid), dim3(FO_THREADS), 0, s, a);
  hipLaunchKernelGGL(fanout_finish_kernel, dim3(1), dim3(FO_THREADS), 0, s, a, probe_blocks(a.pk_cap));
  return hipGetLastError();
}

hipError_t launch_share_repick(const RepickArgs& a, hipStream_t s) {
  if (a.n) hipLaunchKernelGGL(share_repick_kernel, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_subtab_patches(uint32_t* plain, uint32_t* members, uint32_t* alive, const WordPatch* wp,
                                 uint64_t n_plain_w, uint64_t n_member_w, uint64_t n_alive_w, GroupRec* groups,
                                 DevRec* recs, uint32_t* fcnt, const RecPatch* rp, uint64_t n_group_p,
                                 uint64_t n_rec_p, hipStream_t s) {
  // words first (the lists), then the records that point at them
  const uint64_t nw = n_plain_w + n_member_w + n_alive_w;
  if (nw)
    hipLaunchKernelGGL(subtab_word_patch_kernel, dim3(grid_for(nw, 256)), dim3(256), 0, s, plain, members, alive, wp,
                       n_plain_w, n_plain_w + n_member_w, nw);
  if (n_group_p)
    hipLaunchKernelGGL(subtab_rec_patch_kernel, dim3(grid_for(n_group_p, 256)), dim3(256), 0, s, groups, recs, fcnt,
                       rp, n_group_p, n_group_p);
  if (n_rec_p)
    hipLaunchKernelGGL(subtab_rec_patch_kernel, dim3(grid_for(n_rec_p, 256)), dim3(256), 0, s, groups, recs, fcnt,
                       rp + n_group_p, uint64_t(0), n_rec_p);
  return hipGetLastError();
}

hipError_t launch_fcnt_from_recs(const DevRec* recs, uint64_t n, uint32_t* fcnt, hipStream_t s) {
  if (n)
    hipLaunchKernelGGL(fcnt_from_recs_kernel, dim3(std::min<uint32_t>(grid_for(n, 256), 4096)), dim3(256), 0, s,
                       recs, n, fcnt);
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
                            unsigned long long* count, unsigned long long* tombs, hipStream_t s) {
  if (cap && n_pubs)
    hipLaunchKernelGGL(ps_forget_kernel, dim3(grid_for(cap, 256)), dim3(256), 0, s, keys, cap, pubs, n_pubs, count,
                       tombs);
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
