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
//   count   live (unexpired) ranks per range; per-filter totals (one atomic per range)
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

constexpr int RW_WAVES = 4;
constexpr uint32_t RCHUNK = 2048;  // ranks per range record

// Reserve n slots of the spill buffer, all or nothing (a partial reservation would leave
// unwritten items inside the counted prefix).  Called by one lane.
__device__ __forceinline__ bool spill_reserve(uint32_t* ctr, uint32_t n, uint32_t cap, uint32_t* base) {
  uint32_t old = __hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  for (;;) {
    if (old > cap || n > cap - old) return false;
    const uint32_t prev = atomicCAS(ctr, old, old + n);
    if (prev == old) {
      *base = old;
      return true;
    }
    old = prev;
  }
}

// The walk of one wave's stack until it is empty or the step budget runs out; then the
// remaining items go to a.spill_out (global filter ids) for the next, rebalanced round.
// TILE: items name a filter lane of the tile whose first filter is `fbase` (its level count
// and word base in LDS);
// else items name a global filter id and the lane reads both from global memory.
template <bool TILE>
__device__ __forceinline__ void walk_stack(const RetainArgs& a, uint4* stk, uint32_t top, uint64_t fbase,
                                           const uint32_t* nlevs, const uint64_t* wbase, uint32_t* pref,
                                           uint4* itm, uint32_t& visits, bool& overflow) {
  const uint32_t lane = lane_id();
  const RetainView& rv = a.rv;
  const uint64_t b0 = a.foffs[0];
  uint32_t steps = 0;
  while (top > 0) {
    if (steps++ == a.step_budget) {
      // items wider than 64 nodes go out as 64-node pieces, so the next round can deal one
      // wide '+' slice over many waves
      uint32_t pieces = 0;
      for (uint32_t i = lane; i < top; i += 64) pieces += (stk[i].y + 63) >> 6;
      uint32_t ptot;
      (void)wave_excl(pieces, &ptot);
      uint32_t base = 0, ok = 0;
      if (lane == 0) ok = spill_reserve(&a.ctrl[RC_SPILL], ptot, a.spill_cap, &base) ? 1u : 0u;
      ok = __shfl(ok, 0, 64);
      base = __shfl(base, 0, 64);
      if (ok) {
        for (uint32_t i0 = 0; i0 < top; i0 += 64) {
          const uint32_t i = i0 + lane;
          uint4 it = make_uint4(0, 0, 0, 0);
          if (i < top) it = stk[i];
          const uint32_t np = i < top ? (it.y + 63) >> 6 : 0u;
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
    // ---- take the next (up to) 64 nodes from the top items ----------------------------
    const uint32_t navail = top < 64 ? top : 64;
    uint4 it = make_uint4(0, 0, 0, 0);
    if (lane < navail) it = stk[top - 1 - lane];
    uint32_t ctot;
    const uint32_t cex = wave_excl(lane < navail ? it.y : 0u, &ctot);
    pref[lane] = cex + (lane < navail ? it.y : 0u);  // inclusive
    itm[lane] = it;
    __builtin_amdgcn_wave_barrier();
    // items fully consumed: inclusive prefix <= 64
    const uint64_t full = __ballot(lane < navail && pref[lane] <= 64);
    const uint32_t kfull = __popcll(full);  // a prefix of the lanes (counts >= 1)
    const uint32_t taken = ctot < 64 ? ctot : 64;
    if (kfull < navail && lane == 0) {  // the partially consumed item stays, shortened
      const uint32_t used = 64 - (kfull ? pref[kfull - 1] : 0u);
      uint4 p = itm[kfull];
      p.x += used;
      p.y -= used;
      stk[top - 1 - kfull] = p;
    }
    top -= kfull;
    // ---- this lane's node ---------------------------------------------------------------
    bool act = lane < taken;
    uint32_t v = 0, lev = 0, fl = 0;
    if (act) {
      uint32_t lo = 0, hi = navail - 1;  // first j with pref[j] > lane
      while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (pref[mid] > lane) hi = mid; else lo = mid + 1;
      }
      const uint32_t before = lo ? pref[lo - 1] : 0u;
      const uint4 q = itm[lo];
      v = q.x + (lane - before);
      if (q.z & RITEM_POST) v = rv.posts[v].y;  // a postings slice: entry -> node
      lev = q.z & ~RITEM_POST;
      fl = q.w;
    }
    __builtin_amdgcn_wave_barrier();
    bool emit = false, push = false;
    RRange rg{0, 0, 0, 0};
    uint4 np = make_uint4(0, 0, 0, 0);
    if (act) {
      ++visits;
      const RNode rn = rv.nodes[v];
      uint32_t nl;
      uint64_t wb, fg;
      if (TILE) {
        nl = nlevs[fl];
        wb = wbase[fl];
        fg = fbase + fl;
      } else {
        fg = fl;
        nl = a.fnlev[fg];
        wb = (a.foffs[fg] - b0) + fg;
      }
      const uint32_t fn = nl & 0x7FFFFFFFu;
      rg.f = static_cast<uint32_t>(fg);
      // the match spec's strict guard for wildcard filters, and for every filter of a match
      // spec call (match_messages/3, page_read/4); read_message/2's `>=` otherwise
      rg.flags = (nl >> 31) | a.strict_all;
      if (lev == fn) {
        if (rn.ncld & RNODE_TERM) {
          emit = true;
          rg.lo = rn.lo;
          rg.hi = rn.lo + 1;
        }
      } else {
        const uint32_t w = a.wids[wb + lev];
        const uint32_t ncld = rn.ncld & ~RNODE_TERM;
        if (w == WID_HASH) {
          emit = rn.hi > rn.lo;
          rg.lo = rn.lo;
          rg.hi = rn.hi;
        } else if (w == WID_PLUS) {
          // the '+' run from this level, then: a literal -> its postings at the depth after
          // the run, inside this node's rank interval; else ('#', the filter's end) the
          // children range
          uint32_t j = lev + 1;
          while (j < fn && a.wids[wb + j] == WID_PLUS) ++j;
          const uint32_t wl = j < fn ? a.wids[wb + j] : WID_HASH;
          if (ncld == 0 || wl == WID_NONE) {
            push = false;
          } else if (j == fn) {
            // the filter ends with this '+' run: the stored topics of exactly fn levels in
            // this subtree = one slice of the depth-fn rank list
            if (fn <= rv.max_depth) {
              const uint32_t d0 = rv.dterm_off[fn], d1 = rv.dterm_off[fn + 1];
              uint32_t b = d0, e = d1;
              if (v) lower_bound2_u32(rv.dterm, 1, d0, d1, rn.lo, rn.hi, &b, &e);
              emit = e > b;
              rg.lo = b;
              rg.hi = e;
              rg.flags |= RRANGE_INDIRECT;
            }
          } else if (wl == WID_HASH) {
            // '+' run then the final '#': this subtree's topics of at least j levels — one
            // rank range with a depth floor, filtered by the output kernels
            emit = rn.hi > rn.lo;
            rg.lo = rn.lo;
            rg.hi = rn.hi;
            rg.flags |= j << RRANGE_MIND_SHIFT;
          } else {
            uint32_t s = rpost_slot0(j + 1, wl) & rv.pkey_mask;
            uint32_t off = 0, len = 0;
            for (uint32_t k = 0; k <= rv.pkey_mask; ++k) {
              const RPostKey pk = rv.pkeys[s];
              if (pk.depth == WID_NONE) break;
              if (pk.depth == j + 1 && pk.wid == wl) {
                off = pk.off;
                len = pk.len;
                break;
              }
              s = (s + 1) & rv.pkey_mask;
            }
            // slice of entries with lo in [rn.lo, rn.hi): two lower bounds
            const uint32_t* px = reinterpret_cast<const uint32_t*>(rv.posts);
            uint32_t b = 0, e = len;
            if (v) lower_bound2_u32(px + 2ull * off, 2, 0, len, rn.lo, rn.hi, &b, &e);
            push = e > b;
            np = make_uint4(off + b, e - b, (j + 1) | RITEM_POST, fl);
          }
        } else if (w != WID_NONE && ncld != 0) {
          uint32_t s = redge_slot0(v, w) & rv.edge_mask;
          for (uint32_t k = 0; k <= rv.edge_mask; ++k) {
            const REdge e = rv.edges[s];
            if (e.parent == WID_NONE) break;
            if (e.parent == v && e.wid == w) {
              push = true;
              np = make_uint4(e.child, 1u, lev + 1, fl);
              break;
            }
            s = (s + 1) & rv.edge_mask;
          }
        }
      }
    }
    // ---- emissions (one atomic per wave step) --------------------------------------------
    // a range longer than RCHUNK ranks goes out as several records, so the output kernels
    // spread one '#' over the whole subtree across many waves
    const uint32_t nrec = emit ? (rg.hi - rg.lo + RCHUNK - 1) / RCHUNK : 0u;
    uint32_t etot;
    const uint32_t epos = wave_excl(nrec, &etot);
    if (etot) {
      uint32_t base = 0;
      if (lane == 0) base = atomicAdd(&a.ctrl[RC_RANGES], etot);
      base = __shfl(base, 0, 64);
      for (uint32_t k = 0; k < nrec; ++k) {
        if (base + epos + k >= a.range_cap) break;
        RRange part = rg;
        part.lo = rg.lo + k * RCHUNK;
        part.hi = min(rg.hi, part.lo + RCHUNK);
        a.ranges[base + epos + k] = part;
      }
    }
    // ---- pushes ---------------------------------------------------------------------------
    uint32_t qtot;
    const uint32_t qpos = wave_excl(push ? 1u : 0u, &qtot);
    if (top + qtot > a.stack_cap) {
      overflow = true;
      return;
    }
    if (push) stk[top + qpos] = np;
    top += qtot;
    __threadfence_block();
  }
}

}  // namespace

__global__ __launch_bounds__(RW_WAVES * 64) void retain_walk_kernel(RetainArgs a) {
  const uint32_t lane = lane_id();
  const uint32_t wib = threadIdx.x >> 6;
  const uint32_t gw = blockIdx.x * RW_WAVES + wib;
  __shared__ uint32_t s_pref[RW_WAVES][64];
  __shared__ uint4 s_item[RW_WAVES][64];
  __shared__ uint32_t s_nlev[RW_WAVES][64];
  __shared__ uint64_t s_wb[RW_WAVES][64];
  uint32_t* nlevs = s_nlev[wib];
  uint64_t* wbase = s_wb[wib];  // per filter of the tile: its first word id in a.wids
  uint4* stk = a.stack + static_cast<uint64_t>(gw) * a.stack_cap;
  const RetainView& rv = a.rv;
  const uint32_t tf = a.tile_filters;  // filters per wave tile (1..64): fewer = more waves in flight
  const uint64_t ntiles = (a.n + tf - 1) / tf;
  const uint64_t b0 = a.foffs[0];
  uint32_t visits = 0;
  bool overflow = false;

  for (uint64_t t = gw; t < ntiles; t += a.waves) {
    const uint64_t f = t * tf + lane;
    const bool valid = lane < tf && f < a.n;
    // ---- tokenize + intern (per lane) -------------------------------------------------
    uint32_t nlev = 0, wild = 0;
    if (valid) {
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
      a.fnlev[f] = nlev | (wild << 31);  // for the spill rounds
    }
    nlevs[lane] = nlev | (wild << 31);
    wbase[lane] = valid ? (a.foffs[f] - b0) + f : 0;
    // root items
    const bool push0 = valid && rv.n_nodes != 0;
    uint32_t ptot;
    const uint32_t ppos = wave_excl(push0 ? 1u : 0u, &ptot);
    if (push0) stk[ppos] = make_uint4(0u, 1u, 0u, lane);
    __threadfence_block();  // the stack lives in global memory: order this wave's stores and loads
    walk_stack<true>(a, stk, ptot, t * tf, nlevs, wbase, s_pref[wib], s_item[wib], visits, overflow);
    if (overflow) break;
  }
  if (overflow && lane == 0) atomicOr(&a.ctrl[RC_STACK], 1u);
  // visits: one atomic per wave
  uint32_t vtot;
  (void)wave_excl(visits, &vtot);
  if (lane == 0 && vtot) atomicAdd(&a.ctrl[RC_VISITS], vtot);
}

// A spill round: the items the previous round left (global filter ids) dealt evenly over
// `a.waves` waves, each walking its share under the same step budget.
__global__ __launch_bounds__(RW_WAVES * 64) void retain_walk_spill_kernel(RetainArgs a, const uint4* in, uint32_t n_in) {
  const uint32_t lane = lane_id();
  const uint32_t wib = threadIdx.x >> 6;
  const uint32_t gw = blockIdx.x * RW_WAVES + wib;
  __shared__ uint32_t s_pref[RW_WAVES][64];
  __shared__ uint4 s_item[RW_WAVES][64];
  if (gw >= a.waves) return;
  uint4* stk = a.stack + static_cast<uint64_t>(gw) * a.stack_cap;
  const uint32_t per = (n_in + a.waves - 1) / a.waves;
  const uint64_t lo = static_cast<uint64_t>(gw) * per;
  const uint64_t hi = lo + per < n_in ? lo + per : static_cast<uint64_t>(n_in);
  const uint32_t top = hi > lo ? static_cast<uint32_t>(hi - lo) : 0u;
  uint32_t visits = 0;
  bool overflow = top > a.stack_cap;
  if (!overflow) {
    for (uint32_t i = lane; i < top; i += 64) stk[i] = in[lo + i];
    __threadfence_block();
    walk_stack<false>(a, stk, top, 0, nullptr, nullptr, s_pref[wib], s_item[wib], visits, overflow);
  }
  if (overflow && lane == 0) atomicOr(&a.ctrl[RC_STACK], 1u);
  uint32_t vtot;
  (void)wave_excl(visits, &vtot);
  if (lane == 0 && vtot) atomicAdd(&a.ctrl[RC_VISITS], vtot);
}

namespace {

// count (mode 0) / write (mode 1): one wave per 64 ranges (grid-stride, strided rows).  Ranges of at most
// RSHORT ranks are handled lane-parallel; longer ones by the whole wave, 64 ranks at a time.
constexpr uint32_t RSHORT = 32;
template <int MODE>
__global__ __launch_bounds__(256) void retain_out_kernel(RetainArgs a, uint32_t nr) {
  const uint32_t lane = lane_id();
  const uint32_t gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
  const RetainView& rv = a.rv;
  const bool guard = rv.has_expiring && a.now_ms >= 0;
  // lane l of row j takes range l * nrows + j: one emission's consecutive records (a root '#'
  // is hundreds of RCHUNK records) land in different waves instead of one wave's serial loop
  const uint64_t nrows = (static_cast<uint64_t>(nr) + 63) / 64;
  for (uint64_t row = gw; row < nrows; row += nw) {
    const uint64_t r = static_cast<uint64_t>(lane) * nrows + row;
    const bool valid = r < nr;
    RRange rg{0, 0, 0, 0};
    if (valid) rg = a.ranges[r];
    const uint32_t len = rg.hi - rg.lo;
    uint32_t c = 0;
    uint64_t pos = 0;
    const bool check = guard || (rg.flags >> RRANGE_MIND_SHIFT) != 0;  // per-rank filtering needed
    // ranges of at most RSHORT ranks: this lane alone (independent loads, no wave-wide pass
    // per range); longer ones: the whole wave
    if (MODE == 0) {
      if (valid && !check) {
        c = len;
      } else if (valid && len <= RSHORT) {
        for (uint32_t i = rg.lo; i < rg.hi; ++i) c += rank_ok(rv, rank_at(rv, i, rg.flags), guard, a.now_ms, rg.flags) ? 1u : 0u;
      }
    } else if (valid) {
      c = a.rcount[r];
      if (c) pos = a.out_off[rg.f] + atomicAdd(&a.fcursor[rg.f], c);
      if (c && len <= RSHORT) {
        uint64_t p = pos;
        for (uint32_t i = rg.lo; i < rg.hi; ++i) {
          const uint32_t rk = rank_at(rv, i, rg.flags);
          if (len == 1 || rank_ok(rv, rk, guard, a.now_ms, rg.flags)) {
            if (p < a.out_cap) a.out_ids[p] = rv.rank_id[rk];
            ++p;
          }
        }
      }
    }
    // wave-cooperative ranges: longer than RSHORT ranks (and, when counting, only under a guard)
    uint64_t big = __ballot(valid && len > RSHORT && (MODE == 1 ? c != 0 : check));
    while (big) {
      const uint32_t b = __ffsll(static_cast<unsigned long long>(big)) - 1;
      big &= big - 1;
      const uint32_t lo = __shfl(rg.lo, b, 64), hi = __shfl(rg.hi, b, 64), fg = __shfl(rg.flags, b, 64);
      uint64_t p = __shfl(pos, b, 64);
      uint32_t cnt = 0;
      for (uint32_t i0 = lo; i0 < hi; i0 += 64) {
        const uint32_t i = i0 + lane;
        const uint32_t rk = i < hi ? rank_at(rv, i, fg) : 0u;
        const bool live = i < hi && rank_ok(rv, rk, guard, a.now_ms, fg);
        if (MODE == 0) {
          cnt += live ? 1u : 0u;
        } else {
          const uint64_t m = __ballot(live);
          const uint32_t rank = __popcll(m & ((1ull << lane) - 1ull));
          if (live && p + rank < a.out_cap) a.out_ids[p + rank] = rv.rank_id[rk];
          p += __popcll(m);
        }
      }
      if (MODE == 0) {
        uint32_t tot;
        (void)wave_excl(cnt, &tot);
        if (lane == b) c = tot;
      }
    }
    if (MODE == 0 && valid) {
      a.rcount[r] = c;
      if (c) atomicAdd(&a.fcount[rg.f], c);
    }
  }
}

}  // namespace

hipError_t launch_retain_walk(const RetainArgs& a, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  const uint32_t blocks = (a.waves + RW_WAVES - 1) / RW_WAVES;
  hipLaunchKernelGGL(retain_walk_kernel, dim3(blocks), dim3(RW_WAVES * 64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_retain_walk_spill(const RetainArgs& a, const uint4* in, uint32_t n_in, hipStream_t s) {
  if (n_in == 0 || a.waves == 0) return hipSuccess;
  const uint32_t blocks = (a.waves + RW_WAVES - 1) / RW_WAVES;
  hipLaunchKernelGGL(retain_walk_spill_kernel, dim3(blocks), dim3(RW_WAVES * 64), 0, s, a, in, n_in);
  return hipGetLastError();
}

static uint32_t out_blocks(uint32_t nr) {
  const uint64_t waves = (static_cast<uint64_t>(nr) + 63) / 64;
  return static_cast<uint32_t>(std::max<uint64_t>(1, std::min<uint64_t>((waves + 3) / 4, 8192)));
}

hipError_t launch_retain_count(const RetainArgs& a, uint32_t nr, hipStream_t s) {
  if (nr == 0) return hipSuccess;
  hipLaunchKernelGGL(retain_out_kernel<0>, dim3(out_blocks(nr)), dim3(256), 0, s, a, nr);
  return hipGetLastError();
}

hipError_t launch_retain_write(const RetainArgs& a, uint32_t nr, hipStream_t s) {
  if (nr == 0) return hipSuccess;
  hipLaunchKernelGGL(retain_out_kernel<1>, dim3(out_blocks(nr)), dim3(256), 0, s, a, nr);
  return hipGetLastError();
}

}  // namespace emqx
