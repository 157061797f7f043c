// HIP kernels for gfx950 (MI355X): batched topic -> filter-id matching.
//
// Replaces the reference's per-topic DFS over ETS prefix keys
// (apps/emqx/src/emqx_trie.erl:272-334) and the exact-route union of
// emqx_router:match_routes/1 (apps/emqx/src/emqx_router.erl:128-133).
//
// Structure:
//   match_fast_kernel  one wavefront per tile of 64 published topics.
//     phase A  the tile's topic bytes are read with coalesced 16-B loads into an LDS level
//              map ('/' and wildcard bytes); each lane splits its topic from the map, then
//              every word of the tile is hashed and interned word-parallel in the vocab
//              table (exact byte check) -> word ids in LDS.
//     phase B  the frontier of all 64 topics is pooled in one LDS work stack.  Each step
//              pops up to 64*K (topic, node, level) items — K per lane, all their loads in
//              flight together — probes each node's '+' edge (slot 0, no search) and its
//              literal edge (perfect hash or 2-slot bucket), pushes the children and emits
//              the found children's '#' and terminal filter ids (inline in the slot of an
//              edgeless child, else a fids[] reference the scatter resolves: the walk never
//              waits on an id); pushes and emissions are stream-compacted with wave ballots
//              + popcount prefix sums.
//              The stack is LIFO, which bounds it by ~64*K x levels whatever the frontier
//              width.  No MFMA: this is pointer chasing.
//     phase C  per-topic counts + a per-tile slab of (topic, filter id or reference) entries.
//   match_deep_kernel  topics that did not fit the fast path's LDS budget (very deep
//              topics, or a frontier that overflowed the stack): one wavefront per topic,
//              word ids and stack in global scratch.
//   scan / scatter     counts -> CSR offsets; slab entries (references resolved) -> out_ids.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "fanout.h"
#include "kernels.h"

namespace emqx {

namespace {

constexpr uint32_t MODE_ROUTES = 0, MODE_TRIE = 1;  // MODE_TRIE_WILDCARD = 2: default branch

__device__ __forceinline__ uint32_t lane_id() {
  return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint64_t lanemask_lt(uint32_t lane) { return (1ull << lane) - 1ull; }

// Exclusive prefix of a small per-lane value (< 2^BITS) across the wave; *total = wave sum.
// (per bit: one ballot, v_mbcnt_lo/hi for the lanes below, a scalar popcount for the total)
template <int BITS>
__device__ __forceinline__ uint32_t wave_prefix(uint32_t v, uint32_t lane, uint32_t* total) {
  (void)lane;
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (int b = 0; b < BITS; ++b) {
    const uint64_t m = __ballot((v >> b) & 1u);
    pre += __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32), __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u))
           << b;
    tot += static_cast<uint32_t>(__popcll(m)) << b;
  }
  *total = tot;
  return pre;
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t o = __shfl_up(v, d, 64);
    if (lane >= d) v += o;
  }
  return v;
}

__device__ __forceinline__ uint64_t wave_incl_scan64(uint64_t v, uint32_t lane) {
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t lo = __shfl_up(static_cast<uint32_t>(v), d, 64);
    const uint32_t hi = __shfl_up(static_cast<uint32_t>(v >> 32), d, 64);
    if (lane >= d) v += (static_cast<uint64_t>(hi) << 32) | lo;
  }
  return v;
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (uint32_t d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}


__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
#pragma unroll
  for (uint32_t d = 32; d >= 1; d >>= 1) {
    const uint32_t lo = __shfl_xor(static_cast<uint32_t>(v), d, 64);
    const uint32_t hi = __shfl_xor(static_cast<uint32_t>(v >> 32), d, 64);
    v |= (static_cast<uint64_t>(hi) << 32) | lo;
  }
  return v;
}

// One edge slot (wid, child_base, child meta, child literal filter) and its index, which
// names the child's filter ids fids[2 * idx + kind] (see EdgeSlot).
struct Slot {
  uint4 a;
  uint32_t idx;
};

__device__ __forceinline__ Slot load_slot(const EdgeSlot* edges, uint32_t i) {
  Slot s;
  s.a = *reinterpret_cast<const uint4*>(edges + i);
  s.idx = i;
  return s;
}

// Slab / deep-slab entry: owner << 32 | value.  The value is a filter id, or — with
// ENTRY_REF set — a fids[] reference the scatter kernels resolve.
constexpr uint64_t ENTRY_REF = 1ull << 63;

// Emission value of a found child's '#' (kind 0) or terminal (kind 1) filter: the id itself
// when the slot carries it (edgeless child, or META_XFID), else a reference.
__device__ __forceinline__ uint64_t emit_value(const Slot& s, uint32_t kind) {
  if (!(s.a.z & META_HAS_EDGES)) return kind ? s.a.w : s.a.y;
  if (s.a.z & META_XFID) return s.a.w;  // the child's only filter id: the one asked for
  return ENTRY_REF | (2u * s.idx + kind);
}

__device__ __forceinline__ uint32_t resolve_entry(const TableView& tv, uint64_t e) {
  return (e & ENTRY_REF) ? tv.fids[static_cast<uint32_t>(e)] : static_cast<uint32_t>(e);
}

__device__ __forceinline__ Slot empty_slot() {
  Slot s;
  s.a = make_uint4(WID_NONE, 0, 0, 0);
  s.idx = 0;
  return s;
}


// Term-filter emission rule per mode (see include/emqx_match.h):
//  ROUTES          every filter ending here (exact ∪ wildcard), emqx_router.erl:128-133
//  TRIE_WILDCARD   wildcard filters only (the router's trie), emqx_router.erl:117-123
//  TRIE            wildcard filters, plus the one-level '$x' exact filter quirk of
//                  emqx_trie.erl:276-277 (lookup_topic/2 without the wildcard gate)
__device__ __forceinline__ bool term_ok(uint32_t meta, uint32_t mode, bool dollar_root_literal) {
  if (!(meta & META_HAS_TERM)) return false;
  if (mode == MODE_ROUTES) return true;
  if (meta & META_TERM_WILD) return true;
  return mode == MODE_TRIE && dollar_root_literal;
}

// Vocab lookup with exact byte verification.  w0..w3 hold the first 16 bytes of the word;
// longer words compare the tail against the arena.  Returns WID_NONE if absent.
__device__ __forceinline__ uint32_t intern_word(const TableView& tv, uint32_t h, uint32_t len, uint32_t w0,
                                uint32_t w1, uint32_t w2, uint32_t w3, const uint8_t* tbytes,
                                uint64_t wstart) {
  uint32_t i = vocab_slot0(h) & tv.vocab_mask;
  for (uint32_t k = 0; k <= tv.vocab_mask; ++k) {
    const uint4* vp = reinterpret_cast<const uint4*>(tv.vocab + i);
    const uint4 hd = vp[0];  // hash, len, wid, off
    if (hd.z == WID_NONE) return WID_NONE;
    if (hd.x == h && hd.y == len) {
      const uint4 in = vp[1];
      bool eq = in.x == w0 && in.y == w1 && in.z == w2 && in.w == w3;
      if (eq && len > 16) {
        for (uint32_t b = 16; b < len && eq; ++b) eq = tv.arena[hd.w + b] == tbytes[wstart + b];
      }
      if (eq) return hd.z;
    }
    i = (i + 1) & tv.vocab_mask;
  }
  return WID_NONE;
}

// Probe one node's edge array (slots [base, base + cap)) for `wid` ('+' sits in slot 0;
// literals perfect-hashed, or in 2-slot buckets, according to the node's meta).
__device__ __forceinline__ bool probe_one(const EdgeSlot* edges, uint32_t plus_mask, uint32_t base,
                                          uint32_t meta, uint32_t wid, Slot* out) {
  if (wid == WID_PLUS) {
    *out = load_slot(edges, base);
    return out->a.x == WID_PLUS;
  }
  const uint32_t mask = (1u << (meta & META_CAPLOG2_MASK)) - 1u;
  const uint32_t sd = (meta >> META_SEED_SHIFT) & 255u;
  if (meta & META_PH) {
    const bool cp = plus_copies(plus_mask, (meta & META_HAS_PLUS) != 0, meta & META_CAPLOG2_MASK);
    *out = load_slot(edges, base + lit_slot(wid, sd, mask, cp));
    return out->a.x == wid;
  }
  const bool cp = plus_copies(plus_mask, (meta & META_HAS_PLUS) != 0, meta & META_CAPLOG2_MASK);
  const uint32_t b1 = wide_slot(wid, sd, mask, cp, false);
  const Slot x = load_slot(edges, base + b1), y = load_slot(edges, base + b1 + 1);
  if (x.a.x == wid) { *out = x; return true; }
  if (y.a.x == wid) { *out = y; return true; }
  if (!(x.a.z & META_BUCKET_OVF)) return false;
  const uint32_t b2 = wide_slot(wid, sd, mask, cp, true);
  const Slot u = load_slot(edges, base + b2), v = load_slot(edges, base + b2 + 1);
  if (u.a.x == wid) { *out = u; return true; }
  if (v.a.x == wid) { *out = v; return true; }
  return false;
}

// Byte-identical lookup of a wildcard "topic" for match_routes (emqx_router.erl:130):
// walks literal/'+'/'#' edges; a final '#' is the node's hash filter.  Returns the fid or
// FID_NONE.
template <class WidAt>
__device__ uint32_t exact_walk1(const TableView& tv, uint32_t root_base, uint32_t root_meta, uint32_t root_hash_fid,
                                uint32_t nlev, WidAt wid_at) {
  uint32_t base = root_base, meta = root_meta, at = 0, term_inline = FID_NONE;
  bool root = true;
  for (uint32_t k = 0; k < nlev; ++k) {
    const uint32_t w = wid_at(k);
    if (w == WID_HASH && k + 1 == nlev) {
      if (!(meta & META_HAS_HASH)) return FID_NONE;
      if (root) return root_hash_fid;
      return (meta & META_HAS_EDGES) ? tv.fids[2u * at] : base;  // edgeless: inline in child_base
    }
    if (w == WID_NONE || !(meta & META_HAS_EDGES)) return FID_NONE;
    Slot s;
    if (!probe_one(tv.edges, tv.plus_mask, base, meta, w, &s)) return FID_NONE;
    base = s.a.y;
    meta = s.a.z;
    term_inline = s.a.w;
    at = s.idx;
    root = false;
  }
  if (root || !(meta & META_HAS_TERM)) return FID_NONE;
  return (meta & META_HAS_EDGES) ? tv.fids[2u * at + 1u] : term_inline;
}

template <class WidAt>
__device__ uint32_t exact_walk(const TableView& tv, uint32_t nlev, WidAt wid_at) {
  return exact_walk1(tv, tv.root_base, tv.root_meta, tv.root_hash_fid, nlev, wid_at);
}

// Item (8 B):  x = edge-array base of the node
//   y = widx (10) | topic (6) | dollar_root (1) | has_plus (1) | no_literal (1) | ph (1) |
//       hashing (12): ph ? caplog (4) | seed (8) << 4 : caplog (5) | cuckoo seed (7) << 5
constexpr uint32_t IT_TOPIC_SHIFT = 10;
constexpr uint32_t IT_DROOT = 1u << 16;
constexpr uint32_t IT_PLUS = 1u << 17;
constexpr uint32_t IT_NOLIT = 1u << 18;
constexpr uint32_t IT_PH = 1u << 19;
constexpr uint32_t IT_HASH_SHIFT = 20;

__device__ __forceinline__ uint2 make_item(uint32_t base, uint32_t meta, bool droot, bool nolit, uint32_t tl,
                                           uint32_t widx) {
  const bool ph = (meta & META_PH) != 0;
  const uint32_t caplog = meta & META_CAPLOG2_MASK;
  const uint32_t sd = (meta >> META_SEED_SHIFT) & 255u;
  const uint32_t hp = ph ? (caplog | (sd << 4)) : (caplog | (sd << 5));
  return make_uint2(base, widx | (tl << IT_TOPIC_SHIFT) | (droot ? IT_DROOT : 0u) |
                              ((meta & META_HAS_PLUS) ? IT_PLUS : 0u) | (nolit ? IT_NOLIT : 0u) |
                              (ph ? IT_PH : 0u) | (hp << IT_HASH_SHIFT));
}

__device__ __forceinline__ uint32_t item_topic(uint2 it) { return (it.y >> IT_TOPIC_SHIFT) & 63u; }

// The three probe loads of one item — '+' slot, literal slot, the bucket's second slot — each
// on the lanes that need it, issued back to back under one wait.  Written as one asm block
// because the compiler, given `if (need) x = load(...)`, tests the '+' slot inside its own
// branch (a wait there: two dependent round trips per step, measured), and narrows the
// literal loads to their key dwords, fetching the chosen slot's other 12 bytes after the
// compare (a third).  Masked-off lanes keep the empty slot.  Vector loads and exec writes
// only.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void load3_masked(const EdgeSlot* edges, uint32_t ip, uint32_t il, uint32_t ia, bool np,
                                             bool nl, bool na, Slot& p, Slot& l, Slot& a) {
  const uint64_t mp = __ballot(np), ml = __ballot(nl), ma = __ballot(na);
  const EdgeSlot* pp = edges + ip;
  const EdgeSlot* pl = edges + il;
  const EdgeSlot* pa = edges + ia;
  u32x4 vp = {WID_NONE, 0u, 0u, 0u}, vl = vp, va = vp;
  uint64_t save;
  asm volatile(
      "s_mov_b64 %[sv], exec\n\t"
      "s_and_b64 exec, %[sv], %[mp]\n\t"
      "global_load_dwordx4 %[p], %[ap], off\n\t"
      "s_and_b64 exec, %[sv], %[ml]\n\t"
      "global_load_dwordx4 %[l], %[al], off\n\t"
      "s_and_b64 exec, %[sv], %[ma]\n\t"
      "global_load_dwordx4 %[a], %[aa], off\n\t"
      "s_mov_b64 exec, %[sv]\n\t"
      "s_waitcnt vmcnt(0)"
      : [p] "+v"(vp), [l] "+v"(vl), [a] "+v"(va), [sv] "=&s"(save)
      : [ap] "v"(pp), [al] "v"(pl), [aa] "v"(pa), [mp] "s"(mp), [ml] "s"(ml), [ma] "s"(ma)
      : "memory");
  p.a = make_uint4(vp.x, vp.y, vp.z, vp.w);
  p.idx = ip;
  l.a = make_uint4(vl.x, vl.y, vl.z, vl.w);
  l.idx = il;
  a.a = make_uint4(va.x, va.y, va.z, va.w);
  a.idx = ia;
}

// K = 2: the six loads of two items per lane, one asm group under one wait (as load3_masked).
__device__ __forceinline__ void load6_masked(const EdgeSlot* edges, const uint32_t (&ip)[2], const uint32_t (&il)[2],
                                             const bool (&np)[2], const bool (&nl)[2], const bool (&na)[2],
                                             Slot (&p)[2], Slot (&l)[2], Slot (&a)[2]) {
  const uint64_t mp0 = __ballot(np[0]), ml0 = __ballot(nl[0]), ma0 = __ballot(na[0]);
  const uint64_t mp1 = __ballot(np[1]), ml1 = __ballot(nl[1]), ma1 = __ballot(na[1]);
  const EdgeSlot *pp0 = edges + ip[0], *pl0 = edges + il[0], *pa0 = edges + il[0] + 1;
  const EdgeSlot *pp1 = edges + ip[1], *pl1 = edges + il[1], *pa1 = edges + il[1] + 1;
  u32x4 vp0 = {WID_NONE, 0u, 0u, 0u}, vl0 = vp0, va0 = vp0, vp1 = vp0, vl1 = vp0, va1 = vp0;
  uint64_t save;
  asm volatile(
      "s_mov_b64 %[sv], exec\n\t"
      "s_and_b64 exec, %[sv], %[mp0]\n\t"
      "global_load_dwordx4 %[p0], %[ap0], off\n\t"
      "s_and_b64 exec, %[sv], %[ml0]\n\t"
      "global_load_dwordx4 %[l0], %[al0], off\n\t"
      "s_and_b64 exec, %[sv], %[ma0]\n\t"
      "global_load_dwordx4 %[a0], %[aa0], off\n\t"
      "s_and_b64 exec, %[sv], %[mp1]\n\t"
      "global_load_dwordx4 %[p1], %[ap1], off\n\t"
      "s_and_b64 exec, %[sv], %[ml1]\n\t"
      "global_load_dwordx4 %[l1], %[al1], off\n\t"
      "s_and_b64 exec, %[sv], %[ma1]\n\t"
      "global_load_dwordx4 %[a1], %[aa1], off\n\t"
      "s_mov_b64 exec, %[sv]\n\t"
      "s_waitcnt vmcnt(0)"
      : [p0] "+v"(vp0), [l0] "+v"(vl0), [a0] "+v"(va0), [p1] "+v"(vp1), [l1] "+v"(vl1), [a1] "+v"(va1),
        [sv] "=&s"(save)
      : [ap0] "v"(pp0), [al0] "v"(pl0), [aa0] "v"(pa0), [ap1] "v"(pp1), [al1] "v"(pl1), [aa1] "v"(pa1),
        [mp0] "s"(mp0), [ml0] "s"(ml0), [ma0] "s"(ma0), [mp1] "s"(mp1), [ml1] "s"(ml1), [ma1] "s"(ma1)
      : "memory");
  p[0].a = make_uint4(vp0.x, vp0.y, vp0.z, vp0.w);
  p[0].idx = ip[0];
  l[0].a = make_uint4(vl0.x, vl0.y, vl0.z, vl0.w);
  l[0].idx = il[0];
  a[0].a = make_uint4(va0.x, va0.y, va0.z, va0.w);
  a[0].idx = il[0] + 1;
  p[1].a = make_uint4(vp1.x, vp1.y, vp1.z, vp1.w);
  p[1].idx = ip[1];
  l[1].a = make_uint4(vl1.x, vl1.y, vl1.z, vl1.w);
  l[1].idx = il[1];
  a[1].a = make_uint4(va1.x, va1.y, va1.z, va1.w);
  a[1].idx = il[1] + 1;
}

// Probe the '+' edge and the literal edge of K nodes at once: every load is issued
// before any result is consumed, so a step costs one dependent round trip (plus one more for
// the ~1% of wide-node words displaced to their secondary bucket).  Perfect-hashed nodes
// answer in one slot load; wide nodes load their word's 2-slot bucket (one 32-B pair).
// RL (FAST_K1_S384R): the root node's edge array is staged in LDS (rl, rsz slots from
// root_base); a root item's three probes read it there and leave the global load group.
template <int K, bool RL = false>
__device__ __forceinline__ void probe_items(const EdgeSlot* __restrict__ edges, uint32_t plus_mask,
                                            const uint32_t (&base)[K],
                                            const uint32_t (&hparams)[K], const bool (&isph)[K],
                                            const bool (&cpy)[K], const bool (&needL)[K], const uint32_t (&wid)[K],
                                            const bool (&needP)[K], Slot (&lit)[K], bool (&fL)[K],
                                            Slot (&pls)[K], bool (&fP)[K], uint32_t& extra,
                                            const uint4* rl = nullptr, uint32_t rsz = 0, uint32_t root_base = 0) {
  Slot alt[K];
  bool wide[K], again[K];
  uint32_t sdk[K], msk[K], atp[K], atl[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const uint32_t caplog = isph[k] ? (hparams[k] & 15u) : (hparams[k] & 31u);
    sdk[k] = isph[k] ? (hparams[k] >> 4) : (hparams[k] >> 5);
    const uint32_t mask = (1u << caplog) - 1u;
    msk[k] = mask;
    wide[k] = needL[k] && !isph[k];
    const uint32_t h = node_hash(wid[k], sdk[k]);
    const uint32_t i1 = isph[k] ? ph_slot(h, mask, cpy[k]) : wide_slot1(h, mask, cpy[k]);
    // the '+' edge: its copy in the literal probe's line when the table has copies (one L2
    // request for both loads), else slot 0
    atp[k] = base[k] + (needL[k] ? plus_copy(i1, cpy[k]) : 0u);
    atl[k] = base[k] + i1;
  }
  if constexpr (K == 1 && RL) {
    const bool r = rsz != 0 && base[0] == root_base;
    load3_masked(edges, atp[0], atl[0], atl[0] + 1, needP[0] && !r, needL[0] && !r, wide[0] && !r, pls[0], lit[0],
                 alt[0]);
    if (r) {  // (slots of the root's own array: inside [root_base, root_base + rsz))
      if (needP[0]) pls[0].a = rl[atp[0] - root_base];
      if (needL[0]) lit[0].a = rl[atl[0] - root_base];
      if (wide[0]) alt[0].a = rl[atl[0] + 1 - root_base];
    }
  } else if constexpr (K == 1) {
    load3_masked(edges, atp[0], atl[0], atl[0] + 1, needP[0], needL[0], wide[0], pls[0], lit[0], alt[0]);
  } else if constexpr (K == 2) {
    load6_masked(edges, atp, atl, needP, needL, wide, pls, lit, alt);
  } else {
#pragma unroll
    for (int k = 0; k < K; ++k) {
      pls[k] = empty_slot();
      lit[k] = pls[k];
      alt[k] = pls[k];
      if (needP[k]) pls[k] = load_slot(edges, atp[k]);
      if (needL[k]) lit[k] = load_slot(edges, atl[k]);
      if (wide[k]) alt[k] = load_slot(edges, atl[k] + 1);  // same 32-B bucket
    }
  }
  bool any_again = false;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    fP[k] = needP[k] && pls[k].a.x == WID_PLUS;
    fL[k] = needL[k] && lit[k].a.x == wid[k];
    if (wide[k] && !fL[k] && alt[k].a.x == wid[k]) {
      lit[k] = alt[k];
      fL[k] = true;
    }
    again[k] = wide[k] && !fL[k] && (lit[k].a.z & META_BUCKET_OVF);
    any_again |= again[k];
  }
  if (__any(any_again)) {  // secondary buckets (rare): one more dependent round trip
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (!again[k]) continue;
      const uint32_t i2 = wide_slot(wid[k], sdk[k], msk[k], cpy[k], true);
      const Slot u = load_slot(edges, base[k] + i2), v = load_slot(edges, base[k] + i2 + 1);
      ++extra;
      if (u.a.x == wid[k]) { lit[k] = u; fL[k] = true; }
      else if (v.a.x == wid[k]) { lit[k] = v; fL[k] = true; }
    }
  }
}

}  // namespace

// ------------------------------------------------------------------------------------
// Fast path
// ------------------------------------------------------------------------------------

// Per-lane byte reader over the packed topic buffer: 16-B aligned register windows (one
// dwordx4 load per window; the last window of the buffer is filled bytewise).
struct ByteWin {
  const uint8_t* p;
  uint64_t lim;  // bytes [0, lim) are readable
  bool vec_ok;   // p is 16-B aligned
  uint64_t wbase;
  uint4 w;
  __device__ __forceinline__ ByteWin(const uint8_t* p_, uint64_t lim_)
      : p(p_), lim(lim_), vec_ok((reinterpret_cast<uintptr_t>(p_) & 15u) == 0), wbase(~0ull),
        w(make_uint4(0, 0, 0, 0)) {}
  __device__ __forceinline__ uint32_t operator()(uint64_t i) {
    const uint64_t b = i & ~15ull;
    if (b != wbase) {
      wbase = b;
      if (vec_ok && b + 16 <= lim) {
        w = *reinterpret_cast<const uint4*>(p + b);
      } else {
        uint64_t lo = 0, hi = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (b + k < lim) lo |= static_cast<uint64_t>(p[b + k]) << (8 * k);
          if (b + 8 + k < lim) hi |= static_cast<uint64_t>(p[b + 8 + k]) << (8 * k);
        }
        w = make_uint4(static_cast<uint32_t>(lo), static_cast<uint32_t>(lo >> 32), static_cast<uint32_t>(hi),
                       static_cast<uint32_t>(hi >> 32));
      }
    }
    // value selects + shifts (a select between members would become a scratch load)
    const uint32_t j = static_cast<uint32_t>(i & 15u);
    const uint64_t lo = (static_cast<uint64_t>(w.y) << 32) | w.x;
    const uint64_t hi = (static_cast<uint64_t>(w.w) << 32) | w.z;
    const uint64_t q = (j & 8u) ? hi : lo;
    return static_cast<uint32_t>(q >> (8u * (j & 7u))) & 0xFFu;
  }
};

// Per-lane 64-B register chunk over the packed topic buffer: four 16-B aligned windows
// loaded together (one round trip); bytes [0, lim) are readable, the rest reads as 0.
struct Chunk64 {
  const uint8_t* p;
  uint64_t lim;
  bool vec_ok;  // p is 16-B aligned
  uint64_t cb;  // chunk base, ~0 = empty
  uint4 w0, w1, w2, w3;
  __device__ __forceinline__ Chunk64(const uint8_t* p_, uint64_t lim_)
      : p(p_), lim(lim_), vec_ok((reinterpret_cast<uintptr_t>(p_) & 15u) == 0), cb(~0ull) {}
  __device__ __forceinline__ static uint4 win(const uint8_t* p, uint64_t lim, bool vec_ok, uint64_t b) {
    if (vec_ok && b + 16 <= lim) return *reinterpret_cast<const uint4*>(p + b);
    uint32_t v[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t k = 0; k < 16; ++k)
      if (b + k < lim) v[k >> 2] |= static_cast<uint32_t>(p[b + k]) << (8u * (k & 3u));
    return make_uint4(v[0], v[1], v[2], v[3]);
  }
  // the aligned dword at i (i % 4 == 0)
  __device__ __forceinline__ uint32_t dword(uint64_t i) {
    if (i < cb || i >= cb + 64) {
      cb = i & ~15ull;
      w0 = win(p, lim, vec_ok, cb);
      w1 = win(p, lim, vec_ok, cb + 16);
      w2 = win(p, lim, vec_ok, cb + 32);
      w3 = win(p, lim, vec_ok, cb + 48);
    }
    // component-wise value selects (an aggregate select becomes a scratch access)
    const uint32_t r = static_cast<uint32_t>(i - cb);
    const uint32_t q = r >> 4, d = (r >> 2) & 3u;
    return pick4(d, pick4(q, w0.x, w1.x, w2.x, w3.x), pick4(q, w0.y, w1.y, w2.y, w3.y),
                 pick4(q, w0.z, w1.z, w2.z, w3.z), pick4(q, w0.w, w1.w, w2.w, w3.w));
  }
  __device__ __forceinline__ static uint32_t pick4(uint32_t q, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
    return (q & 2u) ? ((q & 1u) ? d : c) : ((q & 1u) ? b : a);
  }
};

__device__ __forceinline__ uint32_t sel8(uint4 a, uint4 b, uint32_t i) {
  const uint32_t lo = Chunk64::pick4(i & 3u, a.x, a.y, a.z, a.w), hi = Chunk64::pick4(i & 3u, b.x, b.y, b.z, b.w);
  return (i & 4u) ? hi : lo;
}

// First 16 bytes of a word (zero padded past its length), given the two aligned windows
// that cover [ws, ws + 16) and sh = ws % 16 — the layout of VocabSlot::inl.
__device__ __forceinline__ void word_head(uint4 wa, uint4 wb, uint32_t sh, uint32_t len, uint32_t (&w)[4]) {
#pragma unroll
  for (uint32_t o = 0; o < 4; ++o) {
    const uint32_t i = (sh >> 2) + o;
    const uint32_t v = __builtin_amdgcn_alignbyte(sel8(wa, wb, i + 1), sel8(wa, wb, i), sh & 3u);
    const uint32_t nb = len > 4 * o ? min(len - 4 * o, 4u) : 0u;
    w[o] = nb >= 4 ? v : (v & ((1u << (8 * nb)) - 1u));
  }
}

// Phase A keeps a word record in wids[] until the word is interned: its offset from the
// tile's 16-B aligned first byte | its length << 20.  Values >= WID_RESOLVED are word ids
// already ('+' / '#' levels, or WID_NONE for a topic handed to the deep path).
constexpr uint32_t AUX_LEN_SHIFT = 20;
constexpr uint64_t AUX_OFF_LIM = 1ull << AUX_LEN_SHIFT;
constexpr uint32_t AUX_LEN_MAX = 4095;  // longer levels go to the deep path
constexpr uint32_t WID_RESOLVED = 0xFFFFFFF0u;

// 4-bit mask of the bytes of x equal to the byte replicated in pat (exact: no carry
// crosses a byte, and the gather multiply's partial products never overlap).
__device__ __forceinline__ uint32_t byte_eq_mask(uint32_t x, uint32_t pat) {
  const uint32_t y = x ^ pat;
  const uint32_t z = ~(((y & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | y) & 0x80808080u;
  return (((z >> 7) * 0x204081u) >> 21) & 0xFu;
}

// Level map of one aligned 16-B chunk: bit b = byte b is '/', bit 16 + b = byte b is '+' or '#'.
__device__ __forceinline__ uint32_t chunk_levelmap(uint4 v) {
  const uint32_t d[4] = {v.x, v.y, v.z, v.w};
  uint32_t m = 0;
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) {
    m |= byte_eq_mask(d[i], 0x2F2F2F2Fu) << (4 * i);
    m |= (byte_eq_mask(d[i], 0x2B2B2B2Bu) | byte_eq_mask(d[i], 0x23232323u)) << (16 + 4 * i);
  }
  return m;
}

// Bits of chunk k (bytes [16k, 16k + 16)) that fall inside [lo, hi); requires hi > 16k.
__device__ __forceinline__ uint32_t span_mask(uint32_t k, uint32_t lo, uint32_t hi) {
  const uint32_t c = 16u * k;
  const uint32_t b0 = lo > c ? lo - c : 0u, b1 = min(hi - c, 16u);
  return ((1u << b1) - 1u) & ~((1u << b0) - 1u);
}

constexpr int ceil_log2(int v) { return v <= 1 ? 0 : 1 + ceil_log2((v + 1) / 2); }

// One wave's LDS in the fast path.
template <int STACK_CAP, int WID_CAP>
struct FastLds {
  uint2 stack[STACK_CAP];  // work stack (LIFO); overflow spills its bottom half to HBM
  uint32_t wids[WID_CAP];  // word ids of the tile's topics, topic after topic
  uint32_t wend[64];       // per topic: end index of its word ids
  uint32_t cnt[64];        // per topic: emitted filter ids
};

// One wave walks one tile: topics [tile * tt, tile * tt + tt) of the batch (tt <= 64; the batched
// kernel's tiles are TILE_TOPICS wide, the small-batch kernel's narrower, so that a batch of a
// few dozen topics spreads over many waves).  Wave-uniform returns only; no block barrier.
// PA splits the tile over two kernels (FAST_K1_S384P, an A/B of round 5): 0 = one kernel,
// 1 = phase A only, its results parked in the tile's HBM spill area (idle until phase B):
// [0, 64) the topics' word-id ends, [64, 128) packed flags (pa_flags), [128] the tile's word
// count, [192, 192 + words) the word ids; 2 = phase B onward, starting from that record.
constexpr uint32_t PA_WIDS = 192;
// NH: each item's next word id is read from LDS before its probe loads are issued (in flight
// with them), not after they return (round 5, -0.9 % on config B; FAST_K1_S384N keeps the old
// order for the A/B harness).
template <int STACK_CAP, int WID_CAP, int K, bool DIAG, bool RL = false, int PA = 0, bool NH = true>
__device__ __forceinline__ void fast_tile(const MatchArgs& a, FastLds<STACK_CAP, WID_CAP>& L, uint64_t tile,
                                          uint32_t tt, const uint4* rl = nullptr, uint32_t rsz = 0) {
  static_assert(STACK_CAP >= 4 * 64 * K && STACK_CAP % 128 == 0, "stack must hold 4 pops");
  static_assert(WID_CAP <= 1024, "item word index is 10 bits");
  static_assert(PA == 0 || (!DIAG && PA_WIDS + WID_CAP <= 2 * 2048), "split tiles: no diagnostics; record fits the spill");
  const uint32_t lane = lane_id();
  const uint64_t t0 = tile * tt;
  if (t0 >= a.n) return;  // wave-uniform; the kernel uses no block-wide barrier
  if (a.perm && (a.ctrl[CTRL_ERROR] & CTRL_ERR_ORDER_CAP)) return;  // no reordered batch: rerun
  const uint64_t clk0 = DIAG ? wall_clock64() : 0;

  const TableView& tv = a.tv;
  const uint32_t tcount = static_cast<uint32_t>(min<uint64_t>(tt, a.n - t0));
  const bool valid = lane < tcount;
  const uint64_t t = t0 + lane;
  uint64_t start = 0, end = 0;
  if (valid) {
    start = a.toffs[t];
    end = a.toffs[t + 1];
  }

  uint32_t nlev = 0, wbase = 0;
  bool wild = false, dollar = false, defer = false;
  uint64_t defer_mask = 0;
  if constexpr (PA == 2) {
    const uint32_t* pa = reinterpret_cast<const uint32_t*>(a.spill + tile * a.spill_cap);
    const uint32_t fl = pa[64 + lane];
    L.wend[lane] = pa[lane];
    const uint32_t nw = pa[128];
    for (uint32_t j = lane; j < nw; j += 64) L.wids[j] = pa[PA_WIDS + j];
    nlev = fl & 0xFFFFu;
    defer = valid && ((fl >> 16) & 1u);
    wild = (fl >> 17) & 1u;
    dollar = (fl >> 18) & 1u;
    wbase = fl >> 20;
    defer_mask = __ballot(defer);
    L.cnt[lane] = 0;
    wave_sync();
  } else {
  // ---- phase A1: tokenize ----------------------------------------------------------
  // The tile's topics are one contiguous byte range.  The wave reads it with coalesced
  // 16-B loads and writes a level map (chunk_levelmap) to the stack area, idle until
  // phase B; then each lane counts its topic's levels with popcounts, and after a wave scan
  // of the counts writes one record per level to wids[].  A tile whose bytes exceed the
  // map falls back to a per-lane byte loop over 64-B register chunks.
  const uint64_t lim = a.toffs[a.n];  // bytes [0, lim) are readable
  const uint64_t A0 = a.toffs[t0] & ~15ull;
  const uint64_t tend = a.toffs[t0 + tcount];
  const bool vec_ok = (reinterpret_cast<uintptr_t>(a.tbytes) & 15u) == 0;
  constexpr uint32_t MAP_CHUNKS = 2 * STACK_CAP;  // one dword per 16-B chunk
  const bool use_map = tend - A0 <= 16ull * MAP_CHUNKS;  // wave-uniform
  uint32_t* lmap = reinterpret_cast<uint32_t*>(L.stack);
  const uint32_t lo = static_cast<uint32_t>(start - A0), hi = static_cast<uint32_t>(end - A0);  // map path only
  Chunk64 C(a.tbytes, lim);
  bool longw = false;
  if (use_map) {
    const uint32_t first = (valid && end > start) ? a.tbytes[start] : 0u;
    const uint32_t nch = static_cast<uint32_t>((tend - A0 + 15) >> 4);
    for (uint32_t c0 = 0; c0 < nch; c0 += 256) {
      uint4 v[4];
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) {
        const uint32_t c = c0 + lane + 64u * u;
        v[u] = c < nch ? Chunk64::win(a.tbytes, lim, vec_ok, A0 + 16ull * c) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (uint32_t u = 0; u < 4; ++u) {
        const uint32_t c = c0 + lane + 64u * u;
        if (c < nch) lmap[c] = chunk_levelmap(v[u]);
      }
    }
    dollar = first == '$';
    wave_sync();
    if (valid) {
      uint32_t cnt = 0;
      for (uint32_t k = lo >> 4; 16u * k < hi; ++k) cnt += __popc(lmap[k] & span_mask(k, lo, hi));
      nlev = cnt + 1;
    }
  } else if (valid) {
    nlev = 1;
    uint32_t llen = 0, first = 0;
    for (uint64_t i = start & ~3ull; i < end; i += 4) {
      const uint32_t d = C.dword(i);
#pragma unroll
      for (uint32_t b = 0; b < 4; ++b) {
        const uint64_t pos = i + b;
        if (pos < start || pos >= end) continue;
        const uint32_t c = (d >> (8u * b)) & 0xFFu;
        if (pos == start) dollar = c == '$';
        if (c == '/') {
          longw |= llen >= AUX_LEN_MAX;
          ++nlev;
          llen = 0;
        } else {
          if (llen == 0) first = c;
          ++llen;
        }
      }
    }
    longw |= llen >= AUX_LEN_MAX;
  }
  defer = valid && (nlev > static_cast<uint32_t>(WID_CAP / 8) || longw || end - A0 >= AUX_OFF_LIM);
  const uint32_t need = (valid && !defer) ? nlev : 0u;
  const uint32_t incl = wave_incl_scan(need, lane);
  wbase = incl - need;
  if (valid && !defer && incl > static_cast<uint32_t>(WID_CAP)) defer = true;
  L.wend[lane] = incl;  // end of the topic's word ids (= the next topic's first)

  if (valid && !defer) {
    uint32_t j = wbase;
    uint64_t ws = start;  // first byte of the current level
    // one record per level; '+' / '#' levels resolve here, over-long ones defer the topic
    auto put = [&](uint64_t wend_) {
      const uint32_t len = static_cast<uint32_t>(wend_ - ws);
      uint32_t v = static_cast<uint32_t>(ws - A0) | (len << AUX_LEN_SHIFT);
      if (len == 1) {
        const bool maybe = !use_map || ((lmap[(ws - A0) >> 4] >> (16u + ((ws - A0) & 15u))) & 1u);
        const uint32_t c = maybe ? static_cast<uint32_t>(a.tbytes[ws]) : 0u;
        v = c == '+' ? WID_PLUS : c == '#' ? WID_HASH : v;
      }
      v = len >= AUX_LEN_MAX ? WID_NONE : v;
      L.wids[j++] = v;
      return v;
    };
    uint32_t seen = 0;  // OR of the records' flags: bit 0 wildcard level, bit 1 over-long level
    auto note = [](uint32_t v) -> uint32_t {
      return (v == WID_PLUS || v == WID_HASH ? 1u : 0u) | (v == WID_NONE ? 2u : 0u);
    };
    if (use_map) {
      for (uint32_t k = lo >> 4; 16u * k < hi; ++k) {
        uint32_t m = lmap[k] & span_mask(k, lo, hi);
        while (m) {
          const uint64_t pos = A0 + 16u * k + static_cast<uint32_t>(__builtin_ctz(m));
          m &= m - 1u;
          seen |= note(put(pos));
          ws = pos + 1;
        }
      }
    } else {
      for (uint64_t i = start & ~3ull; i < end; i += 4) {
        const uint32_t d = C.dword(i);
#pragma unroll
        for (uint32_t b = 0; b < 4; ++b) {
          const uint64_t pos = i + b;
          if (pos < start || pos >= end) continue;
          if (((d >> (8u * b)) & 0xFFu) == '/') {
            seen |= note(put(pos));
            ws = pos + 1;
          }
        }
      }
    }
    seen |= note(put(end));
    wild = (seen & 1u) != 0;
    longw = (seen & 2u) != 0;
  }
  // words of the tile: entries [0, nwords) of wids belong to topics kept on the fast path
  uint32_t nwords = (valid && !defer) ? incl : 0u;
#pragma unroll
  for (uint32_t dd = 32; dd >= 1; dd >>= 1) nwords = max(nwords, static_cast<uint32_t>(__shfl_xor(nwords, dd, 64)));
  defer |= longw;
  defer_mask = __ballot(defer);
  wave_sync();

  // ---- phase A2: intern every word of the tile, word-parallel ------------------------
  // Each lane takes IW words per round: it loads their bytes (16-B windows, mostly L1/L2
  // hits after A1), hashes the head dwords (word_hash16) and loads their first vocab slot;
  // the exact byte check uses the same head dwords.
  constexpr uint32_t IW = 2;  // words per lane per intern round (two vocab probes in flight)
  for (uint32_t j0 = 0; j0 < nwords; j0 += 64u * IW) {
    uint32_t jj[IW], ln[IW], sh[IW], hh[IW], w[IW][4];
    uint64_t wsa[IW];
    bool act[IW];
    uint4 wa[IW], wb[IW], hd[IW], in[IW];
#pragma unroll
    for (uint32_t u = 0; u < IW; ++u) {
      jj[u] = j0 + lane + 64u * u;
      const uint32_t v = jj[u] < nwords ? L.wids[jj[u]] : WID_NONE;
      act[u] = v < WID_RESOLVED;
      ln[u] = v >> AUX_LEN_SHIFT;
      wsa[u] = A0 + (v & (AUX_OFF_LIM - 1));
      sh[u] = static_cast<uint32_t>(wsa[u] & 15u);
      const uint64_t w0 = wsa[u] & ~15ull;
      wa[u] = (act[u] && ln[u]) ? Chunk64::win(a.tbytes, lim, vec_ok, w0) : make_uint4(0, 0, 0, 0);
      wb[u] = (act[u] && sh[u] + min(ln[u], 16u) > 16u) ? Chunk64::win(a.tbytes, lim, vec_ok, w0 + 16)
                                                         : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (uint32_t u = 0; u < IW; ++u) {
      word_head(wa[u], wb[u], sh[u], ln[u], w[u]);
      hh[u] = !act[u] ? 0u : ln[u] <= 16 ? word_hash16(ln[u], w[u][0], w[u][1], w[u][2], w[u][3])
                          : word_hash_bytes(a.tbytes + wsa[u], ln[u]);
      const uint4* vp = reinterpret_cast<const uint4*>(tv.vocab + (vocab_slot0(hh[u]) & tv.vocab_mask));
      hd[u] = act[u] ? vp[0] : make_uint4(0, 0, WID_NONE, 0);
      in[u] = act[u] ? vp[1] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (uint32_t u = 0; u < IW; ++u) {
      if (!act[u]) continue;
      uint32_t wid;
      if (hd[u].z == WID_NONE) {
        wid = WID_NONE;
      } else if (hd[u].x == hh[u] && hd[u].y == ln[u] && ln[u] <= 16 && in[u].x == w[u][0] &&
                 in[u].y == w[u][1] && in[u].z == w[u][2] && in[u].w == w[u][3]) {
        wid = hd[u].z;
      } else {  // long word or a probe chain: the full lookup (rare)
        wid = intern_word(tv, hh[u], ln[u], w[u][0], w[u][1], w[u][2], w[u][3], a.tbytes, wsa[u]);
      }
      L.wids[jj[u]] = wid;
    }
  }
  L.cnt[lane] = 0;
  wave_sync();
  if constexpr (PA == 1) {
    uint32_t* pa = reinterpret_cast<uint32_t*>(a.spill + tile * a.spill_cap);
    pa[lane] = L.wend[lane];
    // nlev and wbase matter only for topics kept on the fast path (nlev <= WID_CAP / 8, wbase < WID_CAP)
    pa[64 + lane] = (nlev & 0xFFFFu) | (defer ? 1u << 16 : 0u) | (wild ? 1u << 17 : 0u) | (dollar ? 1u << 18 : 0u) |
                    ((wbase & 0xFFFu) << 20);
    if (lane == 0) pa[128] = nwords;
    for (uint32_t j = lane; j < nwords; j += 64) pa[PA_WIDS + j] = L.wids[j];
    return;
  }
  }
  const uint64_t clk1 = DIAG ? wall_clock64() : 0;

  // ---- phase B: pooled frontier walk ------------------------------------------------
  uint64_t* slab = a.slab + tile * a.slab_cap;
  uint2* spill = a.spill + tile * a.spill_cap;
  const uint32_t cap = a.slab_cap;
  const uint32_t mode = a.mode;
  uint32_t cursor = 0;    // wave-uniform
  uint32_t top = 0;       // wave-uniform
  uint32_t stop = 0;      // wave-uniform: items in the HBM spill
  uint32_t maxtop = 0;    // wave-uniform (LDS + spill)
  uint32_t evals = 0;     // per lane
  uint32_t dg[DIAG_NCOUNT] = {};  // diagnostic counters (per lane)

  // the root: '#' emission, exact walk of wildcard topics, the root item
  {
    bool e0 = false, e1 = false, push = false;
    uint32_t g1 = 0;
    uint2 it = make_uint2(0, 0);
    if (valid && !defer) {
      if (wild) {
        if (mode == MODE_ROUTES) {
          g1 = exact_walk(tv, nlev, [&](uint32_t k) { return L.wids[wbase + k]; });
          e1 = g1 != FID_NONE;
        }
      } else {
        evals = 1;  // the root visit, F_0
        // filter '#'; '$' rule (emqx_trie.erl:272-279): no root-level '+' or '#' for '$' topics
        e0 = !dollar && (tv.root_meta & META_HAS_HASH);
        if (tv.root_meta & META_HAS_EDGES) {
          push = true;
          const uint32_t rmeta = dollar ? (tv.root_meta & ~META_HAS_PLUS) : tv.root_meta;
          it = make_item(tv.root_base, rmeta, dollar, false, lane, wbase);
        }
      }
    }
    const uint32_t c = (e0 ? 1u : 0u) + (e1 ? 1u : 0u);
    uint32_t tot;
    uint32_t pos = wave_prefix<2>(c, lane, &tot);
    const uint64_t tag = static_cast<uint64_t>(lane) << 32;
    if (e0) { if (pos < cap) slab[pos] = tag | tv.root_hash_fid; ++pos; }
    if (e1) { if (pos < cap) slab[pos] = tag | g1; ++pos; }
    if (c) L.cnt[lane] = c;
    cursor = tot;
    uint32_t ptot;
    const uint32_t ppos = wave_prefix<2>(push ? 1u : 0u, lane, &ptot);
    if (push) L.stack[ppos] = it;
    top = ptot;
    maxtop = top;
    wave_sync();
  }

  if (DIAG && a.diag_stop) top = 0;  // phase A alone (diagnostic counter passes)
  constexpr uint32_t POP = 64u * K;
  constexpr uint32_t HALF = STACK_CAP / 2;
  while (true) {
    top = __builtin_amdgcn_readfirstlane(top);
    stop = __builtin_amdgcn_readfirstlane(stop);
    if (top < POP && stop > 0) {
      // refill from the HBM spill (its newest items first)
      const uint32_t r = min(stop, HALF - (top < HALF ? top : HALF));
      for (uint32_t i = lane; i < r; i += 64) L.stack[top + i] = spill[stop - r + i];
      top += r;
      stop -= r;
      wave_sync();
    }
    if (top == 0) break;
    if (top + POP > static_cast<uint32_t>(STACK_CAP)) {
      if (stop + HALF <= a.spill_cap) {
        // spill the bottom half of the LDS stack to HBM, slide the rest down
        for (uint32_t i = lane; i < HALF; i += 64) spill[stop + i] = L.stack[i];
        for (uint32_t i0 = 0; i0 < top - HALF; i0 += 64) {
          const uint32_t i = i0 + lane;
          uint2 v = make_uint2(0, 0);
          if (i < top - HALF) v = L.stack[HALF + i];
          wave_sync();
          if (i < top - HALF) L.stack[i] = v;
          wave_sync();
        }
        stop += HALF;
        top -= HALF;
        if (DIAG) dg[8] += lane == 0 ? 1u : 0u;
      } else {
        // spill full: hand every topic still pending to the deep path
        uint64_t m = 0;
        for (uint32_t i = lane; i < top; i += 64) m |= 1ull << item_topic(L.stack[i]);
        for (uint32_t i = lane; i < stop; i += 64) m |= 1ull << item_topic(spill[i]);
        defer_mask |= wave_or64(m);
        top = 0;
        stop = 0;
        break;
      }
    }
    const uint32_t nb = min(POP, top);
    uint2 it[K];
    bool act[K], needL[K], needP[K], leaf[K], droot[K], isph[K];
    uint32_t wid[K], tl[K], widx[K], ibase[K], hpar[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
      const uint32_t idx = lane + 64u * k;
      act[k] = idx < nb;
      it[k] = act[k] ? L.stack[top - nb + idx] : make_uint2(0, 0);
    }
    top -= nb;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      tl[k] = item_topic(it[k]);
      widx[k] = it[k].y & 1023u;
      droot[k] = (it[k].y & IT_DROOT) != 0;
      isph[k] = (it[k].y & IT_PH) != 0;
      hpar[k] = it[k].y >> IT_HASH_SHIFT;
      ibase[k] = it[k].x;
      wid[k] = act[k] ? L.wids[widx[k]] : WID_NONE;
      leaf[k] = act[k] && (widx[k] + 1 == L.wend[tl[k]]);
      needL[k] = act[k] && wid[k] != WID_NONE && !(it[k].y & IT_NOLIT);
      needP[k] = act[k] && (it[k].y & IT_PLUS);
    }
    wave_sync();
    Slot lit[K], pls[K];
    bool fL[K], fP[K];
    bool cpy[K];  // the node's array holds '+' copies (a '$' topic's root item keeps them too)
#pragma unroll
    for (int k = 0; k < K; ++k)
      cpy[k] = plus_copies(tv.plus_mask, (it[k].y & IT_PLUS) || (droot[k] && (tv.root_meta & META_HAS_PLUS)),
                           isph[k] ? (hpar[k] & 15u) : (hpar[k] & 31u));
    uint32_t nw0[K];
    if constexpr (NH) {
#pragma unroll
      for (int k = 0; k < K; ++k) nw0[k] = act[k] ? L.wids[widx[k] + 1] : WID_NONE;  // (wids[WID_CAP] is wend[0])
    }
    probe_items<K, RL>(tv.edges, tv.plus_mask, ibase, hpar, isph, cpy, needL, wid, needP, lit, fL, pls, fP, dg[4], rl,
                       rsz, tv.root_base);
    if (DIAG) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        dg[1] += act[k] ? 1u : 0u;
        dg[2] += needL[k] ? 1u : 0u;
        dg[3] += fL[k] ? 1u : 0u;
        dg[5] += needP[k] ? 1u : 0u;
        dg[6] += fP[k] ? 1u : 0u;
        if (act[k]) {
          const uint32_t lvl = widx[k] - (tl[k] ? L.wend[tl[k] - 1] : 0u);
#pragma unroll
          for (uint32_t q = 0; q < 8; ++q) dg[DIAG_LEVEL0 + q] += (lvl == q || (q == 7 && lvl > 7)) ? 1u : 0u;
          const uint32_t cl = isph[k] ? (hpar[k] & 15u) : (hpar[k] & 31u);
          dg[DIAG_SMALL] += cl <= 3 ? 1u : 0u;
          dg[DIAG_WIDE] += cl > 3 ? 1u : 0u;
        }
      }
      dg[0] += 1;
    }

    // emissions: per item ('#' and terminal filter of each found child)
    bool eLh[K], eLt[K], ePh[K], ePt[K], pL[K], pP[K], nlL[K], nlP[K];
    uint32_t ce[K], nwid[K], ecount = 0, pcount = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
      evals += (fL[k] ? 1u : 0u) + (fP[k] ? 1u : 0u);
      eLh[k] = fL[k] && (lit[k].a.z & META_HAS_HASH);
      eLt[k] = fL[k] && leaf[k] && term_ok(lit[k].a.z, mode, droot[k]);
      ePh[k] = fP[k] && (pls[k].a.z & META_HAS_HASH);
      ePt[k] = fP[k] && leaf[k] && term_ok(pls[k].a.z, mode, false);
      pL[k] = fL[k] && !leaf[k] && (lit[k].a.z & META_HAS_EDGES);
      pP[k] = fP[k] && !leaf[k] && (pls[k].a.z & META_HAS_EDGES);
      // the topic's next word decides whether a child's literal edges can matter at all;
      // a child with nothing left to probe is not pushed
      nwid[k] = (pL[k] || pP[k]) ? (NH ? nw0[k] : L.wids[widx[k] + 1]) : WID_NONE;
      nlL[k] = nwid[k] == WID_NONE || !litf_may_contain(lit[k].a.z, lit[k].a.w, nwid[k]);
      nlP[k] = nwid[k] == WID_NONE || !litf_may_contain(pls[k].a.z, pls[k].a.w, nwid[k]);
      pL[k] = pL[k] && !(nlL[k] && !(lit[k].a.z & META_HAS_PLUS));
      pP[k] = pP[k] && !(nlP[k] && !(pls[k].a.z & META_HAS_PLUS));
      ce[k] = (eLh[k] ? 1u : 0u) + (eLt[k] ? 1u : 0u) + (ePh[k] ? 1u : 0u) + (ePt[k] ? 1u : 0u);
      ecount += ce[k];
      pcount += (pL[k] ? 1u : 0u) + (pP[k] ? 1u : 0u);
    }
    {
      uint32_t ptot;
      uint32_t pos = top + wave_prefix<ceil_log2(2 * K + 1)>(pcount, lane, &ptot);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (pL[k]) L.stack[pos++] = make_item(lit[k].a.y, lit[k].a.z, false, nlL[k], tl[k], widx[k] + 1);
        if (pP[k]) L.stack[pos++] = make_item(pls[k].a.y, pls[k].a.z, false, nlP[k], tl[k], widx[k] + 1);
      }
      top += ptot;
      maxtop = max(maxtop, top + stop);
    }
    {
      uint32_t tot;
      uint32_t pos = cursor + wave_prefix<ceil_log2(4 * K + 1)>(ecount, lane, &tot);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const uint64_t tag = static_cast<uint64_t>(tl[k]) << 32;
        if (eLh[k]) { if (pos < cap) slab[pos] = tag | emit_value(lit[k], 0); ++pos; }
        if (eLt[k]) { if (pos < cap) slab[pos] = tag | emit_value(lit[k], 1); ++pos; }
        if (ePh[k]) { if (pos < cap) slab[pos] = tag | emit_value(pls[k], 0); ++pos; }
        if (ePt[k]) { if (pos < cap) slab[pos] = tag | emit_value(pls[k], 1); ++pos; }
        if (ce[k]) atomicAdd(&L.cnt[tl[k]], ce[k]);
      }
      cursor += tot;
      if (DIAG) dg[7] += ecount;
    }
    wave_sync();
  }

  // ---- phase C: per-topic counts, tile bookkeeping ---------------------------------
  wave_sync();
  if (DIAG && a.diag) {
    dg[0] = lane == 0 ? dg[0] : 0u;  // steps are wave-uniform
    dg[8] = lane == 0 ? dg[8] : 0u;
    const uint64_t clk2 = wall_clock64();  // 100 MHz constant clock
    dg[9] = lane == 0 ? static_cast<uint32_t>(clk1 - clk0) : 0u;
    dg[10] = lane == 0 ? static_cast<uint32_t>(clk2 - clk1) : 0u;
    dg[11] = lane == 0 ? 1u : 0u;
    if (a.timeline && lane == 0)
      a.timeline[tile] = make_uint4(static_cast<uint32_t>(clk0), static_cast<uint32_t>(clk0 >> 32),
                                    static_cast<uint32_t>(clk1 - clk0) | (static_cast<uint32_t>(__smid()) << 20),
                                    static_cast<uint32_t>(clk2 - clk0));
#pragma unroll
    for (int i = 0; i < DIAG_NCOUNT; ++i) {
      const uint32_t v = wave_sum(dg[i]);
      if (lane == 0 && v) atomicAdd(reinterpret_cast<unsigned long long*>(a.diag + i), static_cast<unsigned long long>(v));
    }
  }
  const uint32_t mine = (valid && !((defer_mask >> lane) & 1ull)) ? L.cnt[lane] : 0u;
  if (valid) a.counts[t] = mine;
  const uint32_t ev = wave_sum(evals);
  const uint32_t tsum = wave_sum(mine);
  if (lane == 0) {
    a.tile_sum[tile] = tsum;  // the deep path adds its topics' counts
    a.tile_stats[tile] = make_uint2(ev, maxtop);
    a.tile_fill[tile] = cursor;
    a.tile_defer[tile] = defer_mask;
    if (cursor > cap) atomicMax(&a.ctrl[CTRL_NEED_SLAB], cursor);
  }
  if (defer_mask) {
    uint32_t pos0 = 0;
    if (lane == 0) pos0 = atomicAdd(&a.ctrl[CTRL_DEFERRED], static_cast<uint32_t>(__popcll(defer_mask)));
    pos0 = __shfl(pos0, 0, 64);
    if ((defer_mask >> lane) & 1ull)
      a.deferred[pos0 + __popcll(defer_mask & lanemask_lt(lane))] = static_cast<uint32_t>(t);
  }
}

constexpr uint32_t ROOT_LDS_SLOTS = 256;  // FAST_K1_S384R: root arrays up to 4 KB staged in LDS

// (waves per SIMD asked of the compiler: 8 for K = 1, i.e. <= 64 VGPRs, which it exceeds (73, so 6
// waves); FAST_K1_S384W7 (448 word ids) asks for 7, which its 21.5 KiB of LDS per block allows)
constexpr int fast_waves_hint(int K, int WC) { return K == 1 ? (WC == 448 ? 7 : 8) : 5; }
template <int WAVES, int STACK_CAP, int WID_CAP, int K, bool DIAG, bool RL = false, int PA = 0, bool NH = true>
__global__ __launch_bounds__(WAVES * 64, fast_waves_hint(K, WID_CAP)) void match_fast_kernel(MatchArgs a) {
  __shared__ FastLds<STACK_CAP, WID_CAP> lds_all[WAVES];
  __shared__ uint4 rl[RL ? ROOT_LDS_SLOTS : 1];
  const uint32_t wv = threadIdx.x >> 6;
  uint32_t rsz = 0;
  if constexpr (RL) {  // the root's edge array, once per block (every tile's first step probes it)
    const TableView& tv = a.tv;
    const uint32_t cl = (tv.root_meta & META_PH) ? (tv.root_meta & 15u) : (tv.root_meta & META_CAPLOG2_MASK);
    const uint32_t n = (tv.root_meta & META_HAS_EDGES) ? (1u << cl) : 0u;
    rsz = n <= ROOT_LDS_SLOTS ? n : 0u;
    const uint4* src = reinterpret_cast<const uint4*>(tv.edges + tv.root_base);
    for (uint32_t i = threadIdx.x; i < rsz; i += blockDim.x) rl[i] = src[i];
    __syncthreads();
  }
  // With a reordered batch (a.deal), XCD x (blocks b = x mod 8, dispatched round robin)
  // takes one contiguous range of logical blocks: neighbouring keys share its L2.
  uint64_t blk = blockIdx.x;
  if (a.deal) {
    const uint32_t nb = gridDim.x, x = blockIdx.x & 7u, j = blockIdx.x >> 3, q = nb >> 3, r = nb & 7u;
    blk = static_cast<uint64_t>(x) * q + min(x, r) + j;
  }
  fast_tile<STACK_CAP, WID_CAP, K, DIAG, RL, PA, NH>(a, lds_all[wv], blk * WAVES + wv, TILE_TOPICS, rl, rsz);
}

// ------------------------------------------------------------------------------------
// Deep path: one wavefront per deferred topic; word ids and stack in global scratch.
// ------------------------------------------------------------------------------------
// Wave gw of nwaves walks deferred topics gw, gw + nwaves, ... (tt: the fast path's tile width,
// whose tile_sum the deep path adds its counts to).
__device__ __forceinline__ void deep_walk(const MatchArgs& a, uint32_t gw, uint32_t nwaves, uint32_t tt) {
  const uint32_t lane = lane_id();
  const TableView& tv = a.tv;
  const uint32_t ndef = __hip_atomic_load(&a.ctrl[CTRL_DEFERRED], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t* wids = a.deep_wids + static_cast<uint64_t>(gw) * DEEP_MAX_LEVELS;
  uint4* stack = a.deep_stack + static_cast<uint64_t>(gw) * a.deep_stack_cap;
  const uint32_t scap = a.deep_stack_cap;
  const uint32_t mode = a.mode;

  // Slab entries are reserved in chunks of DEEP_CHUNK per wave (no same-address atomic per
  // step); a chunk's unused tail is padded with DEEP_PAD, which the scatter skips.
  uint32_t ccur = 0, cend = 0;  // wave-uniform
  auto pad_chunk = [&]() {
    for (uint32_t p = ccur + lane; p < cend; p += 64)
      if (p < a.deep_slab_cap) a.deep_slab[p] = DEEP_PAD;
    ccur = cend;
  };
  for (uint32_t j = gw; j < ndef; j += nwaves) {
    const uint32_t t = a.deferred[j];
    if (lane == 0) a.deep_rank[j] = 0;
    const uint64_t start = a.toffs[t], end = a.toffs[t + 1];
    if (end - start > 65535u) {
      if (lane == 0) {
        atomicOr(&a.ctrl[CTRL_ERROR], CTRL_ERR_TOO_LONG);
        a.counts[t] = 0;
      }
      continue;
    }
    auto byte_at = [&](uint64_t i) -> uint32_t { return a.tbytes[i]; };
    // tokenize + intern (lane 0; rare path)
    uint32_t nlev = 0, wild = 0, dollar = 0;
    if (lane == 0) {
      uint32_t k = 0, len = 0, w0 = 0, w1 = 0, w2 = 0, w3 = 0;
      uint64_t ws = start;
      for (uint64_t i = start; i <= end; ++i) {
        const uint32_t c = (i < end) ? byte_at(i) : static_cast<uint32_t>('/');
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
          if (len == 1 && w0 == '+') { wid = WID_PLUS; wild = 1; }
          else if (len == 1 && w0 == '#') { wid = WID_HASH; wild = 1; }
          else {
            const uint32_t h = len <= 16 ? word_hash16(len, w0, w1, w2, w3) : word_hash_bytes(a.tbytes + ws, len);
            wid = intern_word(tv, h, len, w0, w1, w2, w3, a.tbytes, ws);
          }
          wids[k++] = wid;
          len = 0;
          w0 = w1 = w2 = w3 = 0;
          ws = i + 1;
        }
      }
      nlev = k;
      dollar = (end > start && byte_at(start) == '$') ? 1u : 0u;
    }
    __threadfence_block();
    nlev = __shfl(nlev, 0, 64);
    wild = __shfl(wild, 0, 64);
    dollar = __shfl(dollar, 0, 64);
    uint32_t count = 0, evals = 0;  // wave-uniform / per-lane

    auto emit = [&](bool e0, uint64_t g0, bool e1, uint64_t g1, bool e2, uint64_t g2, bool e3, uint64_t g3) {
      const uint32_t c = (e0 ? 1u : 0u) + (e1 ? 1u : 0u) + (e2 ? 1u : 0u) + (e3 ? 1u : 0u);
      uint32_t tot;
      const uint32_t rel = wave_prefix<3>(c, lane, &tot);
      if (tot == 0) return;
      if (ccur + tot > cend) {  // reserve the next chunk (one atomic per DEEP_CHUNK entries)
        pad_chunk();
        const uint32_t want = max(tot, DEEP_CHUNK);
        uint32_t base = 0;
        if (lane == 0) base = atomicAdd(&a.ctrl[CTRL_DEEP_FILL], want);
        ccur = __shfl(base, 0, 64);
        cend = ccur + want;
      }
      uint32_t pos = ccur + rel;
      ccur += tot;
      const uint64_t tag = static_cast<uint64_t>(j) << 32;
      bool over = false;
      if (e0) { if (pos < a.deep_slab_cap) a.deep_slab[pos] = tag | g0; else over = true; ++pos; }
      if (e1) { if (pos < a.deep_slab_cap) a.deep_slab[pos] = tag | g1; else over = true; ++pos; }
      if (e2) { if (pos < a.deep_slab_cap) a.deep_slab[pos] = tag | g2; else over = true; ++pos; }
      if (e3) { if (pos < a.deep_slab_cap) a.deep_slab[pos] = tag | g3; else over = true; ++pos; }
      if (over) atomicOr(&a.ctrl[CTRL_ERROR], CTRL_ERR_DEEP_SLAB);
      count += tot;
    };

    uint32_t top = 0;
    if (wild) {
      if (mode == MODE_ROUTES) {
        uint32_t f = FID_NONE;
        if (lane == 0) f = exact_walk(tv, nlev, [&](uint32_t k) { return wids[k]; });
        f = __shfl(f, 0, 64);
        emit(lane == 0 && f != FID_NONE, f, false, 0, false, 0, false, 0);
      }
    } else {
      if (lane == 0) evals = 1;
      const bool eh = lane == 0 && !dollar && (tv.root_meta & META_HAS_HASH);
      emit(eh, tv.root_hash_fid, false, 0, false, 0, false, 0);
      if (tv.root_meta & META_HAS_EDGES) {
        const uint32_t rmeta = dollar ? (tv.root_meta & ~META_HAS_PLUS) : tv.root_meta;
        if (lane == 0)
          stack[top] = make_uint4(tv.root_base, rmeta, 0u, dollar ? 1u : 0u);  // {base, meta, widx, droot}
        top += 1;
      }
    }
    __threadfence_block();

    while (top > 0) {
      const uint32_t nb = min(64u, min(top, scap - top));
      if (nb == 0) {
        if (lane == 0) atomicOr(&a.ctrl[CTRL_ERROR], CTRL_ERR_TOO_DEEP);
        break;
      }
      const bool act = lane < nb;
      uint4 q = make_uint4(0, 0, 0, 0);
      if (act) q = stack[top - nb + lane];
      top -= nb;
      __threadfence_block();
      const bool droot = (q.w & 1u) != 0;
      const uint32_t widx = q.z;
      const uint32_t qbase[1] = {q.x};
      const bool qph[1] = {(q.y & META_PH) != 0};
      const uint32_t qsd = (q.y >> META_SEED_SHIFT) & 255u;
      const uint32_t qhp[1] = {qph[0] ? ((q.y & 15u) | (qsd << 4)) : ((q.y & META_CAPLOG2_MASK) | (qsd << 5))};
      const uint32_t w[1] = {act ? wids[widx] : WID_NONE};
      const bool leaf = act && widx + 1 == nlev;
      const bool nL[1] = {act && w[0] != WID_NONE};
      const bool nP[1] = {act && (q.y & META_HAS_PLUS) != 0};
      Slot lit[1], pls[1];
      bool fL[1], fP[1];
      uint32_t extra = 0;
      const bool qcp[1] = {plus_copies(tv.plus_mask, (q.y & META_HAS_PLUS) || (droot && (tv.root_meta & META_HAS_PLUS)),
                                       q.y & META_CAPLOG2_MASK)};
      probe_items<1>(tv.edges, tv.plus_mask, qbase, qhp, qph, qcp, nL, w, nP, lit, fL, pls, fP, extra);
      evals += (fL[0] ? 1u : 0u) + (fP[0] ? 1u : 0u);
      const uint32_t m0 = lit[0].a.z, m1 = pls[0].a.z;
      const bool e0 = fL[0] && (m0 & META_HAS_HASH), e1 = fL[0] && leaf && term_ok(m0, mode, droot);
      const bool e2 = fP[0] && (m1 & META_HAS_HASH), e3 = fP[0] && leaf && term_ok(m1, mode, false);
      emit(e0, emit_value(lit[0], 0), e1, emit_value(lit[0], 1), e2, emit_value(pls[0], 0), e3,
           emit_value(pls[0], 1));
      const bool p0 = fL[0] && !leaf && (m0 & META_HAS_EDGES);
      const bool p1 = fP[0] && !leaf && (m1 & META_HAS_EDGES);
      uint32_t ptot;
      const uint32_t ppos = wave_prefix<2>((p0 ? 1u : 0u) + (p1 ? 1u : 0u), lane, &ptot);
      if (p0) stack[top + ppos] = make_uint4(lit[0].a.y, m0, widx + 1, 0u);
      if (p1) stack[top + ppos + (p0 ? 1u : 0u)] = make_uint4(pls[0].a.y, m1, widx + 1, 0u);
      top += ptot;
      __threadfence_block();
    }
    const uint32_t ev = wave_sum(evals);
    if (lane == 0) {
      a.counts[t] = count;
      if (count) atomicAdd(reinterpret_cast<unsigned long long*>(a.tile_sum + t / tt),
                           static_cast<unsigned long long>(count));
      atomicAdd(a.ctrl + CTRL_DEEP_EVALS, ev);
    }
  }
  pad_chunk();
}

__global__ __launch_bounds__(256) void match_deep_kernel(MatchArgs a) {
  const uint32_t gw = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if (gw >= a.deep_waves) return;
  deep_walk(a, gw, a.deep_waves, TILE_TOPICS);
}

// ------------------------------------------------------------------------------------
// Scan: counts[n] (u32) -> offsets[n+1] (u64, exclusive)
// ------------------------------------------------------------------------------------
namespace {
constexpr int SCAN_THREADS = 256;
constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = SCAN_THREADS * SCAN_ITEMS;

// Block-wide exclusive scan of one u64 per thread (SCAN_THREADS threads).
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t* total) {
  __shared__ uint64_t wsum[SCAN_THREADS / 64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t incl = wave_incl_scan64(v, lane);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint64_t before = 0, all = 0;
  for (uint32_t k = 0; k < SCAN_THREADS / 64; ++k) {
    if (k < w) before += wsum[k];
    all += wsum[k];
  }
  __syncthreads();
  *total = all;
  return before + incl - v;
}
}  // namespace

__global__ __launch_bounds__(SCAN_THREADS) void scan_reduce_kernel(const uint32_t* counts, uint64_t n,
                                                                   uint64_t* partials) {
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * SCAN_TILE;
  uint64_t s = 0;
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const uint64_t i = base + static_cast<uint64_t>(k) * SCAN_THREADS + threadIdx.x;
    if (i < n) s += counts[i];
  }
  uint64_t tot;
  block_excl_scan(s, &tot);
  if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

__global__ __launch_bounds__(SCAN_THREADS) void scan_partials_kernel(uint64_t* partials, uint64_t nb,
                                                                     uint64_t* offsets, uint64_t n) {
  uint64_t carry = 0;
  for (uint64_t b0 = 0; b0 < nb; b0 += SCAN_THREADS) {
    const uint64_t i = b0 + threadIdx.x;
    const uint64_t v = i < nb ? partials[i] : 0;
    uint64_t tot;
    const uint64_t ex = block_excl_scan(v, &tot);
    if (i < nb) partials[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) offsets[n] = carry;
}

__global__ __launch_bounds__(SCAN_THREADS) void scan_final_kernel(const uint32_t* counts, uint64_t n,
                                                                  const uint64_t* partials,
                                                                  uint64_t* offsets) {
  // thread-contiguous items: thread k owns [base + k*ITEMS, base + (k+1)*ITEMS)
  const uint64_t base = static_cast<uint64_t>(blockIdx.x) * SCAN_TILE + static_cast<uint64_t>(threadIdx.x) * SCAN_ITEMS;
  uint32_t v[SCAN_ITEMS];
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const uint64_t i = base + k;
    v[k] = i < n ? counts[i] : 0u;
    s += v[k];
  }
  uint64_t tot;
  uint64_t run = partials[blockIdx.x] + block_excl_scan(s, &tot);
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const uint64_t i = base + k;
    if (i < n) offsets[i] = run;
    run += v[k];
  }
}

// A scan of at most SCAN_TILE counts in one launch (small batches: the host batcher's calls,
// where each launch of the three-kernel scan costs more than the scan).
__global__ __launch_bounds__(SCAN_THREADS) void scan_single_kernel(const uint32_t* counts, uint64_t n,
                                                                   uint64_t* offsets) {
  const uint64_t base = static_cast<uint64_t>(threadIdx.x) * SCAN_ITEMS;
  uint32_t v[SCAN_ITEMS];
  uint64_t s = 0;
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const uint64_t i = base + k;
    v[k] = i < n ? counts[i] : 0u;
    s += v[k];
  }
  uint64_t tot;
  uint64_t run = block_excl_scan(s, &tot);
#pragma unroll
  for (int k = 0; k < SCAN_ITEMS; ++k) {
    const uint64_t i = base + k;
    if (i < n) offsets[i] = run;
    run += v[k];
  }
  if (threadIdx.x == 0) offsets[n] = tot;
}

// ------------------------------------------------------------------------------------
// Output assembly: tile scan -> per-tile offsets; scatter: slab entries -> CSR out_ids
// ------------------------------------------------------------------------------------
// Sum of v over lanes (u64).
__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
  for (uint32_t d = 32; d >= 1; d >>= 1)
    v += (static_cast<uint64_t>(__shfl_xor(static_cast<uint32_t>(v >> 32), d, 64)) << 32) |
         __shfl_xor(static_cast<uint32_t>(v), d, 64);
  return v;
}

// One block per group of GROUP_TILES tiles: its id total and its node visits / max stack
// (coalesced; no atomics — same-address atomics serialise at L2, ~50 ns each).
__global__ __launch_bounds__(GROUP_TILES) void group_reduce_kernel(MatchArgs a, uint64_t ntiles) {
  __shared__ uint64_t ws[GROUP_TILES / 64], we[GROUP_TILES / 64];
  __shared__ uint32_t wm[GROUP_TILES / 64];
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t i = static_cast<uint64_t>(blockIdx.x) * GROUP_TILES + threadIdx.x;
  uint64_t v = 0, ev = 0;
  uint32_t mx = 0;
  if (i < ntiles) {
    v = a.tile_sum[i];
    const uint2 st = a.tile_stats[i];
    ev = st.x;
    mx = st.y;
  }
  v = wave_sum64(v);
  ev = wave_sum64(ev);
  for (uint32_t d = 32; d >= 1; d >>= 1) mx = max(mx, static_cast<uint32_t>(__shfl_xor(mx, d, 64)));
  if (lane == 0) {
    ws[w] = v;
    we[w] = ev;
    wm[w] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t sv = 0, se = 0;
    uint32_t sm = 0;
    for (uint32_t k = 0; k < GROUP_TILES / 64; ++k) {
      sv += ws[k];
      se += we[k];
      sm = max(sm, wm[k]);
    }
    a.group_sum[blockIdx.x] = sv;
    a.group_stats[blockIdx.x] = make_uint2(static_cast<uint32_t>(min<uint64_t>(se, 0xFFFFFFFFull)), sm);
  }
}

// One wave per tile.  The tile's first output position is two short sums — the group sums
// before its group and its group's tile sums before it — plus a wave scan of its 64 counts.
// Then its slab entries, 64 at a time: lanes holding the same topic find each other with six
// ballots (one per bit of the topic index) and take ranks by popcount, and the same ballots
// advance every topic's running position — no atomics.  Ids beyond out_cap are dropped.
__device__ __forceinline__ void scatter_tile(const MatchArgs& a, uint64_t tile, uint64_t off);

__global__ __launch_bounds__(256) void scatter_fast_kernel(MatchArgs a) {
  const uint32_t lane = lane_id();
  const uint32_t wv = threadIdx.x >> 6;
  const uint64_t tile = static_cast<uint64_t>(blockIdx.x) * 4 + wv;
  const uint64_t t0 = tile * TILE_TOPICS;
  if (t0 >= a.n) return;
  const uint64_t t = t0 + lane;
  uint64_t off = 0;
  if (a.perm) {  // reordered batch: out_off (the caller's order) is already scanned
    if (a.ctrl[CTRL_ERROR] & CTRL_ERR_ORDER_CAP) return;
    off = t < a.n ? a.out_off[a.perm[t]] : 0;
  } else {
    const uint64_t g = tile / GROUP_TILES, g0 = g * GROUP_TILES;
    uint64_t before = 0;
    for (uint64_t k = lane; k < g; k += 64) before += a.group_sum[k];
    for (uint64_t j = g0 + lane; j < tile; j += 64) before += a.tile_sum[j];
    before = wave_sum64(before);
    const uint64_t c = t < a.n ? a.counts[t] : 0;
    off = before + wave_incl_scan64(c, lane) - c;
    if (t < a.n) a.out_off[t] = off;
  }
  scatter_tile(a, tile, off);
}

// Lane L keeps topic L's next output position in a register.  Per round of 64 entries the
// six topic-bit ballots give each entry its rank among the round's entries of its topic and
// each lane its topic's count in the round; positions travel by cross-lane reads.  No LDS
// and no fence in the loop, so the id stores never hold the next round's loads back.
// off: the output position of this lane's topic of the tile.
__device__ __forceinline__ void scatter_tile(const MatchArgs& a, uint64_t tile, uint64_t off) {
  const uint32_t lane = lane_id();
  uint64_t next = off;
  const uint32_t fill = min(a.tile_fill[tile], a.slab_cap);
  const uint64_t dmask = a.tile_defer[tile];
  const uint64_t* slab = a.slab + tile * a.slab_cap;
  const uint64_t lt = lanemask_lt(lane);
  constexpr uint32_t U = 4;  // rounds whose slab loads and id lookups are in flight together
  for (uint32_t i0 = 0; i0 < fill; i0 += 64 * U) {
    uint64_t e[U];
    uint32_t id[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t i = i0 + 64 * u + lane;
      e[u] = i < fill ? slab[i] : ~0ull;
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) id[u] = e[u] != ~0ull ? resolve_entry(a.tv, e[u]) : 0u;
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t tl = static_cast<uint32_t>(e[u] >> 32) & 63u;
      const bool keep = e[u] != ~0ull && !((dmask >> tl) & 1ull);
      const uint64_t km = __ballot(keep);
      uint64_t peers = km, mine = km;
#pragma unroll
      for (uint32_t bit = 0; bit < 6; ++bit) {
        const uint64_t m = __ballot(keep && ((tl >> bit) & 1u));
        peers &= ((tl >> bit) & 1u) ? m : ~m;
        mine &= ((lane >> bit) & 1u) ? m : ~m;
      }
      const uint32_t rk = static_cast<uint32_t>(__popcll(peers & lt));
      const uint32_t lo = __shfl(static_cast<uint32_t>(next), static_cast<int>(tl), 64);
      const uint32_t hi = __shfl(static_cast<uint32_t>(next >> 32), static_cast<int>(tl), 64);
      if (keep) {
        const uint64_t p = ((static_cast<uint64_t>(hi) << 32) | lo) + rk;
        if (p < a.out_cap) a.out_ids[p] = id[u];
      }
      next += static_cast<uint64_t>(__popcll(mine));
    }
  }
}

// One wave: out_off[n] and the call summary from the group sums and the ctrl words.
__global__ __launch_bounds__(64) void summary_kernel(MatchArgs a) {
  const uint32_t lane = lane_id();
  uint64_t tot = 0, ev = 0;
  uint32_t mx = 0;
  for (uint32_t k = lane; k < a.ngroups; k += 64) {
    tot += a.group_sum[k];
    const uint2 st = a.group_stats[k];
    ev += st.x;
    mx = max(mx, st.y);
  }
  tot = wave_sum64(tot);
  ev = wave_sum64(ev);
  for (uint32_t d = 32; d >= 1; d >>= 1) mx = max(mx, static_cast<uint32_t>(__shfl_xor(mx, d, 64)));
  if (lane == 0) {
    const uint32_t* c = a.ctrl;
    const uint32_t need = c[CTRL_NEED_SLAB], err = c[CTRL_ERROR];
    uint64_t flags = 0;
    if (need > a.slab_cap || (err & (CTRL_ERR_DEEP_SLAB | CTRL_ERR_TOO_DEEP | CTRL_ERR_ORDER_CAP))) flags |= SUM_F_RETRY;
    if (tot > a.out_cap) flags |= SUM_F_OVERFLOW;
    if (err & CTRL_ERR_TOO_LONG) flags |= SUM_F_ERROR;
    a.out_off[a.n] = tot;
    uint64_t* sm = a.summary;
    sm[SUM_TOTAL] = tot;
    sm[SUM_EVALS] = ev + c[CTRL_DEEP_EVALS];
    sm[SUM_MAXSTACK] = mx;
    sm[SUM_DEFERRED] = c[CTRL_DEFERRED];
    sm[SUM_NEED_SLAB] = need;
    sm[SUM_DEEP_FILL] = c[CTRL_DEEP_FILL];
    sm[SUM_ERROR] = err;
    sm[SUM_FLAGS] = flags;
    __threadfence_system();
  }
}

__global__ __launch_bounds__(256) void scatter_deep_kernel(MatchArgs a) {
  const uint32_t fill = min(a.ctrl[CTRL_DEEP_FILL], a.deep_slab_cap);
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < fill;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint64_t e = a.deep_slab[i];
    if (e == DEEP_PAD) continue;
    const uint32_t j = static_cast<uint32_t>(e >> 32) & 0x7FFFFFFFu;
    const uint32_t t = a.deferred[j];
    const uint64_t p = a.out_off[a.perm ? a.perm[t] : t] + atomicAdd(&a.deep_rank[j], 1u);
    if (p < a.out_cap) a.out_ids[p] = resolve_entry(a.tv, e);
  }
}

// Host batches (engine.cpp, emqx_host_batch_*): streams a finished CSR from HBM into the
// batch's pinned host buffers — offsets [n+1] and min(total, cap) ids, total read on the
// device — with 16-B stores, so the PCIe writes are full lines and the host needs no
// size-dependent D2H copy.
__global__ __launch_bounds__(256) void csr_to_host_kernel(const uint64_t* __restrict__ d_off, uint64_t n,
                                                          const uint32_t* __restrict__ d_ids, uint64_t cap,
                                                          uint64_t* h_off, uint32_t* h_ids) {
  const uint64_t tid = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const uint64_t nt = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  const uint64_t total = min(d_off[n], cap);
  const uint64_t no2 = (n + 1) / 2;  // offsets, two per 16-B store
  for (uint64_t i = tid; i < no2; i += nt)
    reinterpret_cast<uint4*>(h_off)[i] = reinterpret_cast<const uint4*>(d_off)[i];
  if (tid == 0 && ((n + 1) & 1)) h_off[n] = d_off[n];
  const uint64_t nv = total / 4;     // ids, four per 16-B store
  for (uint64_t i = tid; i < nv; i += nt)
    reinterpret_cast<uint4*>(h_ids)[i] = reinterpret_cast<const uint4*>(d_ids)[i];
  if (tid < total - 4 * nv) h_ids[4 * nv + tid] = d_ids[4 * nv + tid];
}

// Filter-sharded tables: the owner rank of each topic of a batch (layout.h shard_owner).
__global__ __launch_bounds__(256) void shard_owner_kernel(const uint8_t* __restrict__ tbytes,
                                                          const uint64_t* __restrict__ toffs, uint64_t n,
                                                          uint32_t world, uint32_t levels,
                                                          uint32_t* __restrict__ owner) {
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<uint64_t>(gridDim.x) * blockDim.x) {
    const uint64_t a = toffs[i], b = toffs[i + 1];
    owner[i] = shard_owner(tbytes + a, b - a, world, levels, true);
  }
}

// Incremental commits (live_trie.cpp): rewrites existing slots of the committed table in
// place.  Phase 0 writes the slots' filter ids, phase 1 (a later launch) the slots, each with
// one 16-B store, so a concurrent walk sees every slot either old or new, and never a slot
// whose filter id is not yet readable.
__global__ void slot_patch_kernel(EdgeSlot* edges, uint32_t* fids, const SlotPatch* patches, uint32_t n,
                                  int phase) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const SlotPatch& p = patches[i];
    if (phase == 0) {
      *reinterpret_cast<uint2*>(fids + 2ull * p.slot) = make_uint2(p.fid_h, p.fid_t);
    } else {
      *reinterpret_cast<uint4*>(edges + p.slot) = make_uint4(p.s.wid, p.s.child_base, p.s.meta, p.s.litf);
    }
  }
}

// ------------------------------------------------------------------------------------
// Small batches in one launch (kernels.h SmallArgs)
// ------------------------------------------------------------------------------------
namespace {

// Exclusive scan of one value per thread over a block of SMALL_WAVES waves; *total = the sum.
__device__ __forceinline__ uint64_t small_block_scan(uint64_t v, uint64_t* total, uint64_t* wsum) {
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  const uint64_t incl = wave_incl_scan64(v, lane);
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  uint64_t before = 0, all = 0;
  for (uint32_t k = 0; k < SMALL_WAVES; ++k) {
    before += k < w ? wsum[k] : 0;
    all += wsum[k];
  }
  __syncthreads();
  *total = all;
  return before + incl - v;
}

// A phase boundary of the small-batch kernel.  The phases hand data to each other through global
// memory (counts, slabs, the deferred list), but the kernel is ONE workgroup: all its waves sit
// on one CU and share its vector L1, so a workgroup-scope release/acquire (the barrier's own
// s_waitcnt) is all the hand-over needs.  An agent-scope fence here would write back and
// invalidate the XCD's whole L2 at every phase (buffer_wbl2 / buffer_inv sc1 on gfx950) and
// every later table read would miss.  Words that atomics update in L2 (ctrl, deep_rank) are
// read back with atomic loads, never through L1.
__device__ __forceinline__ void small_phase_barrier() {
  __syncthreads();
}

// Largest i in [0, n) with v[i] <= x (v non-decreasing, v[0] <= x).
__device__ __forceinline__ uint32_t small_floor(const uint32_t* v, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (v[mid] <= x) lo = mid; else hi = mid;
  }
  return lo;
}

}  // namespace

__global__ __launch_bounds__(SMALL_WAVES * 64) void small_batch_kernel(SmallArgs sa) {
  constexpr int SC = 384, WC = 640;  // the batched kernel's shallow-table variant (FAST_K1_S384)
  struct FoLds {
    uint32_t D[SMALL_FO_MAX_ENTRIES + 1];  // each entry's first delivery
    uint32_t off[SMALL_MAX_N + 1];         // each topic's first entry
  };
  union Lds {
    FastLds<SC, WC> w[SMALL_WAVES];
    FoLds f;
  };
  __shared__ Lds lds;
  __shared__ uint64_t wsum[SMALL_WAVES];
  const MatchArgs& a = sa.m;
  const uint32_t tid = threadIdx.x, lane = lane_id(), wv = tid >> 6;
  constexpr uint32_t NT = SMALL_WAVES * 64;
  const uint64_t n = a.n;
  // optional phase clock (thread 0; every mark follows a block barrier, so it dates the phase's end)
  uint64_t* const clk = sa.clk;
  uint64_t tprev = clk ? wall_clock64() : 0;
  auto mark = [&](uint32_t k) {
    if (clk && tid == 0) {
      const uint64_t now = wall_clock64();
      atomicAdd(reinterpret_cast<unsigned long long*>(clk + k), static_cast<unsigned long long>(now - tprev));
      tprev = now;
    }
  };
  auto finish = [&](uint32_t k) {  // block-uniform: the launch's last phase
    if (!clk) return;
    __syncthreads();
    mark(k);
    if (tid == 0) atomicAdd(reinterpret_cast<unsigned long long*>(clk + SMALL_CLK_LAUNCHES), 1ull);
  };

  // 0. the call's control words; the batch from pinned host memory into HBM (one round trip
  //    over PCIe: every load of the copy is issued before any store)
  if (tid < CTRL_WORDS) a.ctrl[tid] = 0;
  {
    uint64_t* toffs = const_cast<uint64_t*>(a.toffs);
    uint4* tb = reinterpret_cast<uint4*>(const_cast<uint8_t*>(a.tbytes));
    const uint4* hb = reinterpret_cast<const uint4*>(sa.h_tbytes);
    const uint64_t nch = (sa.nbytes + 15) / 16;
    for (uint64_t i = tid; i <= n; i += NT) toffs[i] = sa.h_toffs[i];
    for (uint64_t i = tid; i < nch; i += NT) tb[i] = hb[i];
    if (sa.has_fanout && sa.f.h_keys)
      for (uint64_t i = tid; i < n; i += NT) sa.f.d_keys[i] = sa.f.h_keys[i];
  }
  small_phase_barrier();
  mark(SMALL_CLK_COPY);

  // 1. the walk: wave w takes tile w (tt topics); 2. deferred topics on every wave
  const uint32_t tt = sa.tt;
  const uint64_t ntiles = (n + tt - 1) / tt;
  if (wv < ntiles) fast_tile<SC, WC, 1, false>(a, lds.w[wv], wv, tt);
  small_phase_barrier();
  mark(SMALL_CLK_WALK);
  auto ctrl = [&](uint32_t k) { return __hip_atomic_load(&a.ctrl[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  if (ctrl(CTRL_DEFERRED)) deep_walk(a, wv, SMALL_WAVES, tt);
  small_phase_barrier();
  mark(SMALL_CLK_DEEP);

  uint64_t* sm = a.summary;
  const uint32_t need = ctrl(CTRL_NEED_SLAB), err = ctrl(CTRL_ERROR);
  uint64_t flags = 0;
  if (need > a.slab_cap || (err & (CTRL_ERR_DEEP_SLAB | CTRL_ERR_TOO_DEEP))) flags |= SUM_F_RETRY;
  if (err & CTRL_ERR_TOO_LONG) flags |= SUM_F_ERROR;

  // 3. offsets (one topic per thread), 4. the tiles' slabs and the deep slab into the CSR
  uint64_t total = 0;
  {
    const uint64_t c = (tid < n && !flags) ? a.counts[tid] : 0;
    const uint64_t ex = small_block_scan(c, &total, wsum);
    if (tid < n) a.out_off[tid] = ex;
    if (tid == 0) a.out_off[n] = total;
  }
  if (total > a.out_cap) flags |= SUM_F_OVERFLOW;
  small_phase_barrier();
  mark(SMALL_CLK_SCAN);
  if (!(flags & (SUM_F_RETRY | SUM_F_ERROR))) {
    if (wv < ntiles) {
      const uint64_t t = uint64_t(wv) * tt + lane;
      scatter_tile(a, wv, (lane < tt && t < n) ? a.out_off[t] : 0);
    }
    const uint32_t fill = min(ctrl(CTRL_DEEP_FILL), a.deep_slab_cap);
    for (uint32_t i = tid; i < fill; i += NT) {
      const uint64_t e = a.deep_slab[i];
      if (e == DEEP_PAD) continue;
      const uint32_t j = static_cast<uint32_t>(e >> 32) & 0x7FFFFFFFu;
      const uint64_t p = a.out_off[a.deferred[j]] + atomicAdd(&a.deep_rank[j], 1u);
      if (p < a.out_cap) a.out_ids[p] = resolve_entry(a.tv, e);
    }
  }
  small_phase_barrier();
  mark(SMALL_CLK_SCATTER);
  if (tid == 0) {
    uint64_t ev = ctrl(CTRL_DEEP_EVALS);
    uint32_t mx = 0;
    for (uint64_t k = 0; k < ntiles; ++k) {
      const uint2 st = a.tile_stats[k];
      ev += st.x;
      mx = max(mx, st.y);
    }
    sm[SUM_TOTAL] = total;
    sm[SUM_EVALS] = ev;
    sm[SUM_MAXSTACK] = mx;
    sm[SUM_DEFERRED] = ctrl(CTRL_DEFERRED);
    sm[SUM_NEED_SLAB] = need;
    sm[SUM_DEEP_FILL] = ctrl(CTRL_DEEP_FILL);
    sm[SUM_ERROR] = err;
    sm[SUM_FLAGS] = flags;
  }

  // 5a. match only: the CSR into the pinned host buffers (16-B stores)
  if (sa.h_out_off) {
    if (!(flags & (SUM_F_RETRY | SUM_F_ERROR))) {
      const uint64_t no2 = (n + 1) / 2;
      for (uint64_t i = tid; i < no2; i += NT)
        reinterpret_cast<uint4*>(sa.h_out_off)[i] = reinterpret_cast<const uint4*>(a.out_off)[i];
      if (tid == 0 && ((n + 1) & 1)) sa.h_out_off[n] = a.out_off[n];
      const uint64_t ids = min(total, sa.h_cap), nv = ids / 4;
      for (uint64_t i = tid; i < nv; i += NT)
        reinterpret_cast<uint4*>(sa.h_out_ids)[i] = reinterpret_cast<const uint4*>(a.out_ids)[i];
      if (tid < ids - 4 * nv) sa.h_out_ids[4 * nv + tid] = a.out_ids[4 * nv + tid];
    }
    finish(SMALL_CLK_OUT);
    return;
  }
  if (!sa.has_fanout) {
    finish(SMALL_CLK_OUT);
    return;
  }

  // 5b. the fan-out (emqx_broker.erl:244-272,500-524; stateless $share picks,
  //     emqx_shared_sub.erl:251-288), straight into the pinned delivery buffers
  const SmallFanout& f = sa.f;
  const uint64_t m = total;
  if (flags || m > SMALL_FO_MAX_ENTRIES) {
    if (tid == 0) {
      f.h_sum[FO_SUM_FLAGS] = flags ? FO_SUM_F_MATCH : FO_SUM_F_SMALL;
      f.h_sum[FO_SUM_TOTAL] = 0;
      f.h_sum[FO_SUM_ENTRIES] = m;
      f.h_sum[FO_SUM_STATE] = f.ps_count ? *f.ps_count : 0;
    }
    finish(SMALL_CLK_OUT);
    return;
  }
  uint32_t* D = lds.f.D;
  uint32_t* off = lds.f.off;
  for (uint64_t t = tid; t <= n; t += NT) off[t] = static_cast<uint32_t>(a.out_off[t]);
  small_phase_barrier();
  // pass 1: each entry's record and topic; exclusive scan of the deliveries.  A thread takes
  // FU entries per round with every load of the round issued before any is used (the id, then
  // the record: two dependent round trips per round, not per entry).
  constexpr uint32_t FU = 4;
  uint64_t T = 0;
  for (uint32_t r0 = 0; r0 < m; r0 += FU * NT) {
    uint32_t fid[FU], c[FU];
    uint4 rec[FU];
#pragma unroll
    for (uint32_t u = 0; u < FU; ++u) {
      const uint32_t e = r0 + u * NT + tid;
      fid[u] = e < m ? a.out_ids[e] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (uint32_t u = 0; u < FU; ++u) rec[u] = fid[u] < f.n_recs ? f.recs[2u * fid[u]] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (uint32_t u = 0; u < FU; ++u) {
      const uint32_t e = r0 + u * NT + tid;
      c[u] = e < m ? fo_rec_plain(rec[u]) + fo_rec_groups(rec[u]) : 0u;
      if (e < m) {
        f.erec[e] = rec[u];
        f.etop[e] = small_floor(off, static_cast<uint32_t>(n), e);
      }
    }
#pragma unroll
    for (uint32_t u = 0; u < FU; ++u) {
      const uint32_t e = r0 + u * NT + tid;
      if (r0 + u * NT >= m) break;  // block-uniform
      uint64_t tc;
      const uint64_t ex = small_block_scan(c[u], &tc, wsum);
      if (e < m) D[e] = static_cast<uint32_t>(T + ex);
      T += tc;
    }
  }
  if (tid == 0) D[m] = static_cast<uint32_t>(min<uint64_t>(T, 0xFFFFFFFFull));
  small_phase_barrier();
  mark(SMALL_CLK_FO_PASS1);
  for (uint64_t t = tid; t <= n; t += NT) f.h_off[t] = t < n ? D[off[t]] : T;
  const bool fits = T <= f.cap;
  // pass 2: deliveries j, lane-consecutive (coalesced stores); each finds its entry in LDS.
  // FU deliveries per thread per round, loads batched as in pass 1: the entry's record, then
  // the plain subscriber or the group, then the group's member.
  if (fits) {
    const bool hash = f.strategy == 3u || f.strategy == 4u;
    for (uint64_t j0 = 0; j0 < T; j0 += FU * NT) {
      uint32_t e[FU], r[FU], fid[FU], sub[FU], key[FU];
      bool ok[FU], grp[FU];
      uint4 rec[FU], g[FU];
#pragma unroll
      for (uint32_t u = 0; u < FU; ++u) {
        const uint64_t j = j0 + u * NT + tid;
        ok[u] = j < T;
        e[u] = ok[u] ? small_floor(D, static_cast<uint32_t>(m), static_cast<uint32_t>(j)) : 0u;
        r[u] = ok[u] ? static_cast<uint32_t>(j) - D[e[u]] : 0u;
      }
#pragma unroll
      for (uint32_t u = 0; u < FU; ++u) {
        rec[u] = ok[u] ? f.erec[e[u]] : make_uint4(0, 0, 0, 0);
        fid[u] = ok[u] ? a.out_ids[e[u]] : 0u;
        key[u] = ok[u] && hash ? f.d_keys[f.etop[e[u]]] : 0u;
      }
#pragma unroll
      for (uint32_t u = 0; u < FU; ++u) {
        const uint32_t np = rec[u].y & ~FO_INLINE_BIT;
        grp[u] = ok[u] && r[u] >= np;
        sub[u] = 0;
        g[u] = make_uint4(0, 0, 0, 0);
        if (ok[u] && !grp[u]) {
          const bool inl = (rec[u].y & FO_INLINE_BIT) != 0;
          sub[u] = (inl && r[u] < FO_INLINE_HEAD)
                       ? fo_inline_head(rec[u], r[u])
                       : *(inl ? reinterpret_cast<const uint32_t*>(f.recs + 2u * fid[u] + 1u) + (r[u] - FO_INLINE_HEAD)
                               : f.plain + rec[u].x + r[u]);
        }
        if (grp[u]) g[u] = f.groups[rec[u].z + (r[u] - np)];  // {member_begin, n_members, slot, group_id}
      }
#pragma unroll
      for (uint32_t u = 0; u < FU; ++u) {
        if (!grp[u]) continue;
        const uint32_t np = rec[u].y & ~FO_INLINE_BIT;
        const uint32_t gidx = rec[u].z + (r[u] - np);
        const uint32_t idx = g[u].y <= 1 ? 0u : fo_stateless_index(f.strategy, key[u], f.seed, e[u], gidx, g[u].y);
        sub[u] = f.members[g[u].x + idx];
      }
#pragma unroll
      for (uint32_t u = 0; u < FU; ++u) {
        if (!ok[u]) continue;
        const uint64_t j = j0 + u * NT + tid;
        f.h_subs[j] = sub[u];
        f.h_fil[j] = grp[u] ? (fid[u] | FANOUT_SHARED_BIT) : fid[u];
      }
    }
  }
  if (tid == 0) {
    f.h_sum[FO_SUM_FLAGS] = fits ? 0 : FO_SUM_F_OVERFLOW;
    f.h_sum[FO_SUM_TOTAL] = T;
    f.h_sum[FO_SUM_ENTRIES] = m;
    f.h_sum[FO_SUM_STATE] = f.ps_count ? *f.ps_count : 0;
  }
  finish(SMALL_CLK_FO_PASS2);
}

// ------------------------------------------------------------------------------------
// Launch wrappers
// ------------------------------------------------------------------------------------
template <int W, int S, int WC, int K, bool RL = false, bool NH = true>
static void launch_fast_t(const MatchArgs& a, uint64_t ntiles, hipStream_t s) {
  const uint64_t grid = (ntiles + W - 1) / W;
  if (a.diag)
    hipLaunchKernelGGL((match_fast_kernel<W, S, WC, K, true, RL, 0, NH>), dim3(static_cast<uint32_t>(grid)),
                       dim3(W * 64), 0, s, a);
  else
    hipLaunchKernelGGL((match_fast_kernel<W, S, WC, K, false, RL, 0, NH>), dim3(static_cast<uint32_t>(grid)),
                       dim3(W * 64), 0, s, a);
}

hipError_t launch_match_fast(const MatchArgs& a, FastVariant v, hipStream_t s) {
  const uint64_t ntiles = (a.n + TILE_TOPICS - 1) / TILE_TOPICS;
  if (ntiles == 0) return hipSuccess;
  switch (v) {
    case FAST_K1_S1K: launch_fast_t<4, 1024, 1024, 1>(a, ntiles, s); break;
    case FAST_K2_S1K: launch_fast_t<4, 1024, 1024, 2>(a, ntiles, s); break;
    case FAST_K2_S2K: launch_fast_t<2, 2048, 1024, 2>(a, ntiles, s); break;
    case FAST_K2_S768: launch_fast_t<4, 768, 768, 2>(a, ntiles, s); break;
    case FAST_K4_S2K: launch_fast_t<2, 2048, 1024, 4>(a, ntiles, s); break;
    case FAST_K1_S256: launch_fast_t<4, 256, 512, 1>(a, ntiles, s); break;
    case FAST_K2_S512: launch_fast_t<4, 512, 640, 2>(a, ntiles, s); break;
    case FAST_K1_S384: launch_fast_t<4, 384, 640, 1>(a, ntiles, s); break;
    case FAST_K2_S512W: launch_fast_t<4, 512, 512, 2>(a, ntiles, s); break;
    case FAST_K1_S768W: launch_fast_t<4, 768, 1024, 1>(a, ntiles, s); break;
    case FAST_K1_S512W: launch_fast_t<4, 512, 1024, 1>(a, ntiles, s); break;
    case FAST_K1_S384R: launch_fast_t<4, 384, 640, 1, true>(a, ntiles, s); break;
    case FAST_K1_S384N: launch_fast_t<4, 384, 640, 1, false, false>(a, ntiles, s); break;
    case FAST_K1_S384W7: launch_fast_t<4, 384, 448, 1>(a, ntiles, s); break;
    case FAST_K1_S384B2: launch_fast_t<2, 384, 640, 1>(a, ntiles, s); break;
    case FAST_K1_S384B1: launch_fast_t<1, 384, 640, 1>(a, ntiles, s); break;
    case FAST_K1_S512WB1: launch_fast_t<1, 512, 1024, 1>(a, ntiles, s); break;
    case FAST_K1_S384P: {  // phase A and the walk as two kernels (diagnostic runs keep one)
      if (a.diag) {
        launch_fast_t<4, 384, 640, 1>(a, ntiles, s);
        break;
      }
      const dim3 grid(static_cast<uint32_t>((ntiles + 3) / 4));
      hipLaunchKernelGGL((match_fast_kernel<4, 384, 640, 1, false, false, 1>), grid, dim3(256), 0, s, a);
      hipLaunchKernelGGL((match_fast_kernel<4, 384, 640, 1, false, false, 2>), grid, dim3(256), 0, s, a);
      break;
    }
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_small_batch(const SmallArgs& a, hipStream_t s) {
  const uint64_t tiles = a.tt ? (a.m.n + a.tt - 1) / a.tt : 0;
  if (a.m.n == 0 || a.m.n > SMALL_MAX_N || a.tt == 0 || a.tt > TILE_TOPICS || tiles > SMALL_WAVES ||
      tiles > a.slab_tiles)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(small_batch_kernel, dim3(1), dim3(SMALL_WAVES * 64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_match_deep(const MatchArgs& a, hipStream_t s) {
  const uint32_t blocks = (a.deep_waves * 64 + 255) / 256;
  hipLaunchKernelGGL(match_deep_kernel, dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

uint64_t scan_partials(uint64_t n) { return (n + SCAN_TILE - 1) / SCAN_TILE + 1; }

hipError_t launch_scan(const uint32_t* counts, uint64_t n, uint64_t* offsets, uint64_t* partials,
                       hipStream_t s) {
  const uint64_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
  if (nb <= 1) {  // one tile (or none): one launch
    hipLaunchKernelGGL(scan_single_kernel, dim3(1), dim3(SCAN_THREADS), 0, s, counts, n, offsets);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(scan_reduce_kernel, dim3(static_cast<uint32_t>(nb)), dim3(SCAN_THREADS), 0, s, counts, n, partials);
  hipLaunchKernelGGL(scan_partials_kernel, dim3(1), dim3(SCAN_THREADS), 0, s, partials, nb, offsets, n);
  hipLaunchKernelGGL(scan_final_kernel, dim3(static_cast<uint32_t>(nb)), dim3(SCAN_THREADS), 0, s, counts, n, partials, offsets);
  return hipGetLastError();
}

hipError_t launch_assemble(const MatchArgs& a, hipStream_t s) {
  const uint64_t ntiles = (a.n + TILE_TOPICS - 1) / TILE_TOPICS;
  if (ntiles) {
    hipLaunchKernelGGL(group_reduce_kernel, dim3(a.ngroups), dim3(GROUP_TILES), 0, s, a, ntiles);
    if (a.perm) {  // the counts back in the caller's order, scanned into out_off
      hipError_t err = launch_order_counts(a.counts, a.perm, a.n, a.corig, s);
      if (err == hipSuccess) err = launch_scan(a.corig, a.n, a.out_off, a.partials, s);
      if (err != hipSuccess) return err;
    }
    hipLaunchKernelGGL(scatter_fast_kernel, dim3(static_cast<uint32_t>((ntiles + 3) / 4)), dim3(256), 0, s, a);
  }
  hipLaunchKernelGGL(scatter_deep_kernel, dim3(64), dim3(256), 0, s, a);
  hipLaunchKernelGGL(summary_kernel, dim3(1), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_csr_to_host(const uint64_t* d_off, uint64_t n, const uint32_t* d_ids, uint64_t cap,
                               uint64_t* h_off, uint32_t* h_ids, hipStream_t s) {
  const uint64_t work = std::max<uint64_t>((n + 1) / 2, cap / 4);
  const uint32_t blocks = static_cast<uint32_t>(std::min<uint64_t>((work + 255) / 256 + 1, 2048));
  hipLaunchKernelGGL(csr_to_host_kernel, dim3(blocks), dim3(256), 0, s, d_off, n, d_ids, cap, h_off, h_ids);
  return hipGetLastError();
}

hipError_t launch_shard_owner(const uint8_t* tbytes, const uint64_t* toffs, uint64_t n, uint32_t world,
                              uint32_t levels, uint32_t* owner, hipStream_t s) {
  if (!n) return hipSuccess;
  const uint32_t blocks = static_cast<uint32_t>(std::min<uint64_t>((n + 255) / 256, 4096));
  hipLaunchKernelGGL(shard_owner_kernel, dim3(blocks), dim3(256), 0, s, tbytes, toffs, n, world, levels, owner);
  return hipGetLastError();
}

hipError_t launch_slot_patches(EdgeSlot* edges, uint32_t* fids, const SlotPatch* patches, uint32_t n,
                               hipStream_t s) {
  if (!n) return hipSuccess;
  const dim3 grid(std::min<uint32_t>((n + 255) / 256, 1024));
  hipLaunchKernelGGL(slot_patch_kernel, grid, dim3(256), 0, s, edges, fids, patches, n, 0);
  hipLaunchKernelGGL(slot_patch_kernel, grid, dim3(256), 0, s, edges, fids, patches, n, 1);
  return hipGetLastError();
}

}  // namespace emqx
