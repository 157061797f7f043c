// Incremental commits: the committed level trie patched in place (tables.h, LiveTrie).
//
// Reference semantics (paths relative to /root/reference): emqx_trie:insert/1 and delete/1
// add / remove one filter's keys (apps/emqx/src/emqx_trie.erl:115-137), called per route
// change inside a mria transaction (apps/emqx/src/emqx_router_utils.erl:33-70); a filter is
// visible to match/1 as soon as its transaction commits.  Here a commit publishes a batch of
// such changes, and its cost is proportional to that batch:
//
//   * delete / re-insert of a filter already in the trie: flip its META_HAS_HASH / _TERM flag
//     in the slot that describes its node (the filter ids stay, so a revival is a flip too);
//   * insert of a new filter: walk the host image of the trie like the kernel does; at the
//     first missing edge, the rest of the filter becomes a chain of one-edge nodes in the spare
//     region, and the missing edge is placed into the existing node if that node's hashing has
//     a free slot for it (perfect-hash slot, '+' slot 0, or a free slot of its primary /
//     secondary 2-slot bucket), otherwise the node is relocated: rebuilt with one more entry,
//     with slack, into the spare region.  Then the slot that describes the node (in its
//     parent's array, or the table view for the root) is re-encoded: literal filter, XFID /
//     inline filter ids, hashing parameters.
//
// Device writes per commit: the new spare-region extents (one copy each), plus one whole 16-B
// slot store per rewritten existing slot (filter ids first, slots second), so a walk that
// overlaps a commit sees each slot old or new, and each new filter absent or present.
//
// Threads: flips touch one slot each (atomic flag updates); inserts under different
// first-level nodes touch disjoint parts of the table (the node, its descendants, their
// slots, their filters' ids), so after the inserts that must change the root itself have run
// serially, the rest run grouped by first-level node on up to `threads` threads, each
// allocating from its own chunk of the spare region.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>

#include "tables.h"

namespace emqx {

namespace {

constexpr uint32_t STRUCT_BITS =
    META_CAPLOG2_MASK | META_HAS_PLUS | META_HAS_EDGES | META_PH | (0xFFu << META_SEED_SHIFT);
constexpr uint32_t FILTER_BITS = META_HAS_HASH | META_HAS_TERM | META_TERM_WILD;
constexpr EdgeSlot EMPTY_SLOT{WID_NONE, 0, 0, 0};
constexpr uint32_t LINE = 8;  // slots per 128-B line
constexpr uint32_t FULL_LINE = 0xFFu;

uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

uint32_t log2u(uint64_t p) {
  uint32_t l = 0;
  while ((1ull << l) < p) ++l;
  return l;
}

}  // namespace

void LiveTrie::adopt(HostTables& ht, std::vector<uint64_t>& fid_loc, std::vector<uint32_t>& slot_ids,
                     uint64_t spare, VocabState* v) {
  const uint64_t n = ht.edges.size();
  edges.swap(ht.edges);
  fids.swap(ht.fids);
  sid.swap(slot_ids);
  cap = std::min<uint64_t>(n + spare, MAX_SLOTS);
  edges.resize(cap, EMPTY_SLOT);
  fids.resize(2 * cap, FID_NONE);
  sid.resize(2 * cap, WID_NONE);
  used = n;
  garbage = 0;
  root_base = ht.root_base;
  root_meta = ht.root_meta;
  root_hash_fid = ht.root_hash_fid;
  root_hash_id = WID_NONE;
  for (uint64_t id = 0; id < fid_loc.size(); ++id)
    if (fid_loc[id] == FIDLOC_ROOT_HASH) root_hash_id = static_cast<uint32_t>(id);
  n_nodes = ht.n_nodes;
  max_depth = ht.max_depth;
  loc.swap(fid_loc);
  vocab = v;
  plus_mask = ht.plus_mask;
  pcap.assign(plus_mask ? cap : 0, 0);
  if (plus_mask) {  // arrays whose '+' edge has copies: the root's and every slot's child array
    auto note = [&](uint32_t base, uint32_t meta) {
      const uint32_t cl = meta & META_CAPLOG2_MASK;
      if ((meta & META_HAS_EDGES) && plus_copies(plus_mask, meta & META_HAS_PLUS, cl)) pcap[base] = static_cast<uint8_t>(cl);
    };
    note(root_base, root_meta);
    for (uint64_t i = 0; i < n; ++i)
      if (edges[i].wid != WID_NONE) note(edges[i].child_base, edges[i].meta);
  }
  mark = used;
  dirty.clear();
  ranges.clear();
}

void LiveTrie::sync_plus(Ctx& c, uint64_t p) {
  if (!has_copies(p)) return;
  const uint64_t end = p + (1ull << pcap[p]);
  const EdgeSlot& h = edges[p];
  const EdgeSlot& c1 = edges[p + PLUS_LINE];
  if (c1.wid == h.wid && c1.child_base == h.child_base && c1.litf == h.litf &&
      ((c1.meta ^ h.meta) & ~META_BUCKET_OVF) == 0 && fids[2 * (p + PLUS_LINE)] == fids[2 * p] &&
      fids[2 * (p + PLUS_LINE) + 1] == fids[2 * p + 1])
    return;  // the copies hold this record already (every copy is written together)
  for (uint64_t q = p + PLUS_LINE; q < end; q += PLUS_LINE) {
    const uint32_t keep = edges[q].meta & META_BUCKET_OVF;
    edges[q] = edges[p];
    edges[q].meta = (edges[p].meta & ~META_BUCKET_OVF) | keep;
    fids[2 * q] = fids[2 * p];
    fids[2 * q + 1] = fids[2 * p + 1];
    sid[2 * q] = sid[2 * p];
    sid[2 * q + 1] = sid[2 * p + 1];
    touch(c, q);
  }
}

namespace {
constexpr uint64_t CHUNK = 8192;          // spare-region slots a thread takes at a time
constexpr uint32_t WID_UNKNOWN = 0xFFFFFFFCu;  // tokenize(intern = false): a word not interned yet
}  // namespace

// Spare-region allocation: arrays of >= 8 slots start on a 128-B line; smaller ones are packed
// first-fit into the thread's open line (an array never straddles a line), as the builder's
// line-packed layout does.  Large arrays come straight from the shared cursor.
bool LiveTrie::alloc(Ctx& c, uint32_t caplog, uint64_t* at) {
  const uint64_t n = 1ull << caplog;
  auto grab = [&](uint64_t want, uint64_t* a) -> bool {
    std::lock_guard<std::mutex> g(alloc_mu_);
    const uint64_t b = (used + LINE - 1) & ~uint64_t(LINE - 1);
    if (b + want > cap) return false;
    used = b + want;
    *a = b;
    return true;
  };
  if (n >= CHUNK / 4) {
    uint64_t a;
    if (!grab(n, &a)) return false;
    c.ranges.push_back({a, a + n});
    *at = a;
    return true;
  }
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (n >= LINE) {
      const uint64_t a = (c.cur + LINE - 1) & ~uint64_t(LINE - 1);
      if (a + n <= c.end) {
        c.cur = a + n;
        c.ranges[c.chunk_range].second = c.cur;
        c.line_used = FULL_LINE;
        *at = a;
        return true;
      }
    } else {
      const uint32_t want = (1u << n) - 1u;
      for (uint32_t o = 0; o < LINE; o += static_cast<uint32_t>(n))
        if (!(c.line_used & (want << o))) {
          c.line_used |= want << o;
          *at = c.line + o;
          return true;
        }
      const uint64_t l = (c.cur + LINE - 1) & ~uint64_t(LINE - 1);
      if (l + LINE <= c.end) {
        c.line = l;
        c.cur = l + LINE;
        c.ranges[c.chunk_range].second = c.cur;
        c.line_used = want;
        *at = l;
        return true;
      }
    }
    uint64_t a, len = CHUNK;  // a new chunk (what is left, near the end of the region)
    {
      std::lock_guard<std::mutex> g(alloc_mu_);
      const uint64_t b = (used + LINE - 1) & ~uint64_t(LINE - 1);
      len = b < cap ? std::min<uint64_t>(CHUNK, cap - b) : 0;
      if (len < std::max<uint64_t>(n, LINE)) return false;
      used = b + len;
      a = b;
    }
    c.garbage += c.end - c.cur;  // the old chunk's unused tail
    c.cur = a;
    c.end = a + len;
    c.line_used = FULL_LINE;
    c.chunk_range = c.ranges.size();
    c.ranges.push_back({a, a});
  }
  return false;
}

// The node's literal words, summarised as the builder does (tables.cpp pass 4).  Wide
// (bucketed) nodes are summarised as "many" (an all-ones filter: no false negatives).
void LiveTrie::lit_summary(uint32_t base, uint32_t meta, uint32_t* n_lit, uint32_t* only, uint32_t* bloom,
                           uint32_t* bloom8) const {
  *n_lit = 0;
  *only = WID_NONE;
  *bloom = 0;
  *bloom8 = 0;
  if (!(meta & META_HAS_EDGES)) return;
  if (!(meta & META_PH)) {
    *n_lit = LITF_BLOOM_MAX + 1;
    return;
  }
  const uint32_t c = 1u << (meta & META_CAPLOG2_MASK);
  for (uint32_t i = 0; i < c; ++i) {
    const uint32_t w = edges[base + i].wid;
    if (w == WID_NONE || w == WID_PLUS) continue;
    *n_lit += 1;
    *only = w;
    const uint32_t h = litf_hash(w);
    *bloom |= (1u << (h & 31u)) | (1u << ((h >> 5) & 31u));
    *bloom8 |= 1u << (h & 7u);
  }
}

// The slot that leads to a node: its structure (smeta & STRUCT_BITS), its filters (fmeta &
// FILTER_BITS, fid_h / fid_t present or FID_NONE) and its literal filter — encoded exactly as
// write_slot / meta_of in tables.cpp do.
EdgeSlot LiveTrie::encode(uint32_t wid, bool has_edges, uint32_t base, uint32_t smeta, uint32_t fid_h,
                          uint32_t fid_t, uint32_t fmeta) const {
  EdgeSlot r{wid, 0, 0, 0};
  if (!has_edges) {  // edgeless child: filter ids inline
    r.meta = (fmeta & FILTER_BITS) | META_LITF_NONE;
    r.child_base = fid_h;
    r.litf = fid_t;
    return r;
  }
  smeta = (smeta & STRUCT_BITS) | META_HAS_EDGES;
  uint32_t n_lit, only, bloom, bloom8;
  lit_summary(base, smeta, &n_lit, &only, &bloom, &bloom8);
  uint32_t lf = 0, lflag = 0;
  if (n_lit == 0) {
    lflag = META_LITF_NONE;
  } else if (n_lit == 1) {
    lflag = META_LITF_EXACT;
    lf = only;
  } else {
    lf = n_lit <= LITF_BLOOM_MAX ? bloom : ~0u;
  }
  const bool h = fid_h != FID_NONE, t = fid_t != FID_NONE;
  if (h != t) {
    uint32_t f8 = 0;
    if (lflag & META_LITF_EXACT) f8 = litf_hash(only) >> 24;
    else if (!(lflag & META_LITF_NONE)) f8 = n_lit > LITF_BLOOM_MAX ? 0xFFu : bloom8;
    lflag |= META_XFID | (t ? META_XFID_TERM : 0u) | (f8 << META_F8_SHIFT);
    lf = t ? fid_t : fid_h;
  }
  r.child_base = base;
  r.meta = smeta | (fmeta & FILTER_BITS) | lflag;
  r.litf = lf;
  return r;
}

// Re-encodes slot `p` from its current node structure and filter ids.
void LiveTrie::reencode(Ctx& c, uint64_t p) {
  const EdgeSlot s = edges[p];
  const bool he = (s.meta & META_HAS_EDGES) != 0;
  EdgeSlot r = encode(s.wid, he, he ? s.child_base : 0, s.meta, fids[2 * p], fids[2 * p + 1], s.meta);
  r.meta |= s.meta & META_BUCKET_OVF;
  edges[p] = r;
  touch(c, p);
  sync_plus(c, p);
}

// Points the node reached through `pslot` (or the root) at a new edge array / structure.
void LiveTrie::set_node(Ctx& c, bool root, uint64_t pslot, uint32_t base, uint32_t smeta) {
  if (root) {
    uint32_t n_lit, only, bloom, bloom8;
    const uint32_t sm = (smeta & STRUCT_BITS) | META_HAS_EDGES;
    lit_summary(base, sm, &n_lit, &only, &bloom, &bloom8);
    root_base = base;
    root_meta = sm | (root_meta & META_HAS_HASH) | (n_lit == 0 ? META_LITF_NONE : n_lit == 1 ? META_LITF_EXACT : 0u);
    return;
  }
  const EdgeSlot s = edges[pslot];
  EdgeSlot r = encode(s.wid, true, base, smeta, fids[2 * pslot], fids[2 * pslot + 1], s.meta);
  r.meta |= s.meta & META_BUCKET_OVF;
  edges[pslot] = r;
  touch(c, pslot);
  sync_plus(c, pslot);
}

bool LiveTrie::find_child(uint32_t base, uint32_t meta, uint32_t wid, uint32_t* slot) const {
  if (!(meta & META_HAS_EDGES)) return false;
  if (wid == WID_PLUS) {
    *slot = base;
    return edges[base].wid == WID_PLUS;
  }
  const uint32_t mask = (1u << (meta & META_CAPLOG2_MASK)) - 1u;
  const uint32_t sd = (meta >> META_SEED_SHIFT) & 255u;
  if (meta & META_PH) {
    *slot = base + lit_slot(wid, sd, mask, plus_copies(plus_mask, meta & META_HAS_PLUS, meta & META_CAPLOG2_MASK));
    return edges[*slot].wid == wid;
  }
  const bool cp = plus_copies(plus_mask, meta & META_HAS_PLUS, meta & META_CAPLOG2_MASK);
  const uint32_t b1 = wide_slot(wid, sd, mask, cp, false);
  for (uint32_t k = 0; k < 2; ++k)
    if (edges[base + b1 + k].wid == wid) {
      *slot = base + b1 + k;
      return true;
    }
  if (!(edges[base + b1].meta & META_BUCKET_OVF)) return false;
  const uint32_t b2 = wide_slot(wid, sd, mask, cp, true);
  for (uint32_t k = 0; k < 2; ++k)
    if (edges[base + b2 + k].wid == wid) {
      *slot = base + b2 + k;
      return true;
    }
  return false;
}

// Adds edge `wid` -> `child` (slot content; filter ids fh/ft, engine ids ih/it) to the node
// reached through `pslot` (or the root): in place when its hashing has room, else relocated.
bool LiveTrie::place(Ctx& cx, bool root, uint64_t pslot, uint32_t wid, const EdgeSlot& child, uint32_t fh,
                     uint32_t ft, uint32_t ih, uint32_t it) {
  const uint32_t base = root ? root_base : edges[pslot].child_base;
  uint32_t smeta = (root ? root_meta : edges[pslot].meta) & STRUCT_BITS;
  if (!(smeta & META_HAS_EDGES)) return relocate(cx, root, pslot, wid, child, fh, ft, ih, it);
  const uint32_t mask = (1u << (smeta & META_CAPLOG2_MASK)) - 1u;
  const uint32_t sd = (smeta >> META_SEED_SHIFT) & 255u;
  uint64_t target = ~0ull, ovf = ~0ull;
  if (wid == WID_PLUS) {
    bool free = edges[base].wid == WID_NONE;
    // with copies, the literals of a perfect-hashed array are hashed over the non-head slots:
    // a '+' joining one of more than PLUS_LINE slots rehashes it (relocation)
    // an array that would hold copies hashes its literals over the non-head slots once it has
    // '+' (lit_slot, wide_slot): a '+' joining one is placed by relocation, which rehashes
    if (plus_copies(plus_mask, true, smeta & META_CAPLOG2_MASK)) free = false;
    if (free) {
      target = base;
      smeta |= META_HAS_PLUS;
    }
  } else if (smeta & META_PH) {
    const uint32_t j =
        lit_slot(wid, sd, mask, plus_copies(plus_mask, smeta & META_HAS_PLUS, smeta & META_CAPLOG2_MASK));
    if (edges[base + j].wid == WID_NONE) target = base + j;
  } else {
    const bool cp = plus_copies(plus_mask, smeta & META_HAS_PLUS, smeta & META_CAPLOG2_MASK);
    const uint32_t b1 = wide_slot(wid, sd, mask, cp, false), b2 = wide_slot(wid, sd, mask, cp, true);
    for (uint32_t k = 0; k < 2 && target == ~0ull; ++k)
      if (edges[base + b1 + k].wid == WID_NONE) target = base + b1 + k;
    for (uint32_t k = 0; k < 2 && target == ~0ull; ++k)
      if (edges[base + b2 + k].wid == WID_NONE) {
        target = base + b2 + k;
        ovf = base + b1;
      }
  }
  if (target == ~0ull) return relocate(cx, root, pslot, wid, child, fh, ft, ih, it);
  const uint32_t keep = edges[target].meta & META_BUCKET_OVF;
  edges[target] = child;
  edges[target].meta = (child.meta & ~META_BUCKET_OVF) | keep;
  fids[2 * target] = fh;
  fids[2 * target + 1] = ft;
  sid[2 * target] = ih;
  sid[2 * target + 1] = it;
  if (ih != WID_NONE) loc[ih] = target << 2 | FIDLOC_HASH;
  if (it != WID_NONE) loc[it] = target << 2 | FIDLOC_TERM;
  touch(cx, target);
  if (wid == WID_PLUS && plus_copies(plus_mask, true, smeta & META_CAPLOG2_MASK)) {
    pcap[base] = static_cast<uint8_t>(smeta & META_CAPLOG2_MASK);
    sync_plus(cx, base);
  }
  if (ovf != ~0ull && !(edges[ovf].meta & META_BUCKET_OVF)) {
    edges[ovf].meta |= META_BUCKET_OVF;
    touch(cx, ovf);
  }
  set_node(cx, root, pslot, base, smeta);
  cx.in_place += 1;
  return true;
}

// Rebuilds the node's edge array with the new entry into the spare region (perfect hash for
// up to 32 literals, with 1.5x slack so later inserts usually fit in place; 2-slot buckets at
// load <= 1/8 beyond), then points the node's slot at it.
namespace {
bool commit_prof() {  // EMQX_COMMIT_PROF=1: commit phase times on stderr
  static const bool on = [] {
    const char* e = std::getenv("EMQX_COMMIT_PROF");
    return e && *e && *e != '0';
  }();
  return on;
}
// A relocation's perfect-hash search tries an array size only when its 256 seeds expect at
// least this many hits, else the next size up (EMQX_PH_MIN_HITS overrides).  0.02 spent 65 % of
// relocate's time on sizes that mostly failed; 2 cut the seed search 12.7 -> 4.8 thread-ms per
// 20K-op commit for 2 % more new slots.
double ph_min_hits() {
  static const double v = [] {
    const char* e = std::getenv("EMQX_PH_MIN_HITS");
    return e && *e ? std::atof(e) : 2.0;
  }();
  return v;
}
struct ProfTimer {  // adds the scope's duration to *acc when profiling
  uint64_t* acc;
  std::chrono::steady_clock::time_point t0;
  explicit ProfTimer(uint64_t* a) : acc(commit_prof() ? a : nullptr) {
    if (acc) t0 = std::chrono::steady_clock::now();
  }
  void stop() {
    if (acc) *acc += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    acc = nullptr;
  }
  ~ProfTimer() { stop(); }
};
}  // namespace

bool LiveTrie::relocate(Ctx& cx, bool root, uint64_t pslot, uint32_t wid, const EdgeSlot& child, uint32_t fh,
                        uint32_t ft, uint32_t ih, uint32_t it) {
  ProfTimer prof_all(&cx.reloc_ns);
  const uint32_t obase = root ? root_base : edges[pslot].child_base;
  const uint32_t ometa = (root ? root_meta : edges[pslot].meta) & STRUCT_BITS;
  std::vector<Entry>& ent = cx.ent;
  ent.clear();
  uint32_t ocap = 0;
  if (ometa & META_HAS_EDGES) {
    ocap = 1u << (ometa & META_CAPLOG2_MASK);
    for (uint32_t i = 0; i < ocap; ++i) {
      const uint64_t p = obase + i;
      const EdgeSlot& s = edges[p];
      if (s.wid == WID_NONE || (s.wid == WID_PLUS && i != 0)) continue;  // (a '+' copy: slot 0's edge)
      EdgeSlot c = s;
      c.meta &= ~META_BUCKET_OVF;
      ent.push_back({s.wid, c, fids[2 * p], fids[2 * p + 1], sid[2 * p], sid[2 * p + 1]});
    }
  }
  EdgeSlot c = child;
  c.meta &= ~META_BUCKET_OVF;
  ent.push_back({wid, c, fh, ft, ih, it});
  const uint32_t e = static_cast<uint32_t>(ent.size());
  bool has_plus = false;
  for (auto& x : ent) has_plus |= x.wid == WID_PLUS;
  const uint32_t n_lit = e - (has_plus ? 1u : 0u);

  uint32_t caplog = 0, seed = 0;
  bool ph = false;
  std::vector<uint32_t>& pos = cx.pos;
  pos.assign(e, 0);
  ProfTimer prof_ph(&cx.ph_ns);
  if (n_lit <= 32) {
    // perfect-hash seed search, one bitmap per trial (cap <= 512 here: 8 words); array sizes
    // where 256 seeds would almost surely all fail (birthday bound) are skipped
    const uint64_t cap0 = next_pow2(std::max<uint64_t>(2, e + e / 2));
    const uint64_t cap_max = next_pow2(std::max<uint64_t>(16, 8ull * e));
    for (uint64_t c2 = cap0; c2 <= cap_max && !ph && log2u(c2) <= PH_MAX_CAPLOG && c2 <= 512; c2 <<= 1) {
      double p_ok = 1.0;
      const bool cp = plus_copies(plus_mask, has_plus, log2u(c2));
      const uint32_t room = cp ? static_cast<uint32_t>(c2 / PLUS_LINE * (PLUS_LINE - 1)) : static_cast<uint32_t>(c2);
      const uint32_t avail = room - (has_plus && !cp ? 1u : 0u);
      for (uint32_t k = 0; k < n_lit; ++k) p_ok *= k < avail ? double(avail - k) / double(room) : 0.0;
      if (p_ok * 256.0 < ph_min_hits() && c2 < cap_max) continue;
      const uint32_t mask = static_cast<uint32_t>(c2 - 1);
      for (uint32_t sd = 0; sd < 256 && !ph; ++sd) {
        uint64_t bm[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (has_plus) bm[0] = 1;  // slot 0 (a copy array's literals never hash to a line head)
        bool ok = true;
        for (uint32_t k = 0; k < e && ok; ++k) {
          if (ent[k].wid == WID_PLUS) {
            pos[k] = 0;
            continue;
          }
          const uint32_t sl = lit_slot(ent[k].wid, sd, mask, cp);
          const uint64_t bit = 1ull << (sl & 63u);
          ok = !(bm[sl >> 6] & bit);
          bm[sl >> 6] |= bit;
          pos[k] = sl;
        }
        if (ok) {
          caplog = log2u(c2);
          seed = sd;
          ph = true;
        }
      }
    }
  }
  std::vector<uint32_t> ovf_at;
  if (!ph) {  // 2-slot buckets, two candidate buckets, random-walk eviction
    caplog = log2u(next_pow2(8ull * e + 8));
    bool ok = false;
    std::vector<int32_t> owner;
    const bool cp = plus_copies(plus_mask, has_plus, caplog);
    for (uint32_t sd = 0; sd < CUCKOO_SEEDS && !ok; ++sd) {
      const uint32_t cc = 1u << caplog, mk = cc - 1;
      owner.assign(cc, -1);
      ok = true;
      uint32_t rng = 0x9E3779B9u ^ (sd << 20) ^ e;
      for (uint32_t k = 0; k < e; ++k)  // '+' pinned at slot 0 (and its copies at every line head)
        if (ent[k].wid == WID_PLUS)
          for (uint32_t q = 0; q < cc; q += cp ? PLUS_LINE : cc) owner[q] = static_cast<int32_t>(k);
      for (uint32_t k0 = 0; k0 < e && ok; ++k0) {
        if (ent[k0].wid == WID_PLUS) continue;
        int32_t k = static_cast<int32_t>(k0);
        for (int kick = 0;; ++kick) {
          const uint32_t w = ent[k].wid, b1 = wide_slot(w, sd, mk, cp, false), b2 = wide_slot(w, sd, mk, cp, true);
          const uint32_t cand[4] = {b1, b1 + 1, b2, b2 + 1};
          bool placed = false;
          for (uint32_t q : cand)
            if (owner[q] < 0) {
              owner[q] = k;
              placed = true;
              break;
            }
          if (placed) break;
          if (kick > 500) {
            ok = false;
            break;
          }
          rng = rng * 1664525u + 1013904223u;
          const uint32_t victim = cand[(rng >> 16) & 3u];
          if (ent[owner[victim]].wid == WID_PLUS) continue;
          std::swap(k, owner[victim]);
        }
      }
      if (ok) {
        seed = sd;
        for (uint32_t q = cc; q-- > 0;)  // (the '+' entry ends at slot 0)
          if (owner[q] >= 0) pos[owner[q]] = q;
        for (uint32_t k = 0; k < e; ++k) {
          if (ent[k].wid == WID_PLUS) continue;
          const uint32_t b1 = wide_slot(ent[k].wid, sd, mk, cp, false);
          if (pos[k] != b1 && pos[k] != b1 + 1) ovf_at.push_back(b1);
        }
      }
    }
    if (!ok || caplog > 31) return false;
  }
  prof_ph.stop();
  uint64_t nb = 0;
  if (!alloc(cx, caplog, &nb)) return false;
  const uint32_t cc = 1u << caplog;
  for (uint32_t i = 0; i < cc; ++i) {
    edges[nb + i] = EMPTY_SLOT;
    fids[2 * (nb + i)] = fids[2 * (nb + i) + 1] = FID_NONE;
    sid[2 * (nb + i)] = sid[2 * (nb + i) + 1] = WID_NONE;
  }
  for (uint32_t k = 0; k < e; ++k) {
    const uint64_t p = nb + pos[k];
    edges[p] = ent[k].s;
    fids[2 * p] = ent[k].fh;
    fids[2 * p + 1] = ent[k].ft;
    sid[2 * p] = ent[k].ih;
    sid[2 * p + 1] = ent[k].it;
    if (ent[k].ih != WID_NONE) loc[ent[k].ih] = p << 2 | FIDLOC_HASH;
    if (ent[k].it != WID_NONE) loc[ent[k].it] = p << 2 | FIDLOC_TERM;
  }
  if (plus_mask) {
    pcap[nb] = plus_copies(plus_mask, has_plus, caplog) ? static_cast<uint8_t>(caplog) : 0u;
    sync_plus(cx, nb);  // (new slots: nothing to touch)
  }
  for (uint32_t q : ovf_at) edges[nb + q].meta |= META_BUCKET_OVF;
  const uint32_t smeta = (caplog & META_CAPLOG2_MASK) | META_HAS_EDGES | (has_plus ? META_HAS_PLUS : 0u) |
                         (ph ? META_PH : 0u) | (seed << META_SEED_SHIFT);
  set_node(cx, root, pslot, static_cast<uint32_t>(nb), smeta);
  cx.garbage += ocap;
  cx.relocations += 1;
  return true;
}

// Delete / revival of a filter already in the table: its flag in the slot of its node.
void LiveTrie::flip(Ctx& c, uint32_t id, bool want, bool atomic) {
  const uint64_t l = loc[id];
  c.flips += 1;
  if (l == FIDLOC_ROOT_HASH) {  // serial only
    root_meta = want ? (root_meta | META_HAS_HASH) : (root_meta & ~META_HAS_HASH);
    return;
  }
  const uint64_t p = l >> 2;
  const uint32_t bit = (l & 3) == FIDLOC_HASH ? META_HAS_HASH : META_HAS_TERM;
  if (((edges[p].meta & bit) != 0) == want) return;
  if (atomic) {  // the hash and the term filter of one node may flip on two threads
    if (want) __atomic_fetch_or(&edges[p].meta, bit, __ATOMIC_RELAXED);
    else __atomic_fetch_and(&edges[p].meta, ~bit, __ATOMIC_RELAXED);
  } else {
    edges[p].meta ^= bit;
  }
  touch(c, p);
  if (has_copies(p)) c.plus_heads.push_back(static_cast<uint32_t>(p));  // copies: after the flips
}

// emqx_topic:words/1 (emqx_topic.erl:153-164) to word ids; a final '#' is the parent level's
// hash filter.  intern = false: read-only lookups (thread-safe), unknown words -> WID_UNKNOWN.
bool LiveTrie::tokenize(const FilterStore& fs, uint32_t id, std::vector<uint32_t>& w, bool* wild,
                        bool* final_hash, bool intern) const {
  const uint8_t* p = fs.bytes.data() + fs.off[id];
  const uint64_t n = fs.off[id + 1] - fs.off[id];
  w.clear();
  *wild = *final_hash = false;
  bool unknown = false;
  uint64_t s = 0;
  for (uint64_t i = 0; i <= n; ++i) {
    if (i != n && p[i] != '/') continue;
    const uint64_t len = i - s;
    if (len == 1 && p[s] == '+') {
      w.push_back(WID_PLUS);
      *wild = true;
    } else if (len == 1 && p[s] == '#') {
      *wild = true;
      if (i == n) *final_hash = true;
      else w.push_back(WID_HASH);
    } else if (intern) {
      w.push_back(vocab->intern(p + s, len));
    } else {
      const VocabState& v = *vocab;
      auto res = [&v](uint32_t k, const uint8_t*& q, uint64_t& m) {
        q = v.arena.data() + v.off[k];
        m = v.off[k + 1] - v.off[k];
      };
      const uint32_t k = v.map.find(p + s, len, hash64_bytes(p + s, len), res);
      unknown |= k == WID_NONE;
      w.push_back(k == WID_NONE ? WID_UNKNOWN : k);
    }
    s = i + 1;
  }
  return !unknown;
}

bool LiveTrie::insert(Ctx& c, const FilterStore& fs, uint32_t id, const std::vector<uint32_t>& w, bool wild,
                      bool final_hash, bool root, uint64_t pslot, uint32_t i) {
  const uint32_t ext = fs.ext[id];
  const uint32_t L = static_cast<uint32_t>(w.size());
  for (; i < L; ++i) {
    const uint32_t base = root ? root_base : edges[pslot].child_base;
    const uint32_t meta = root ? root_meta : edges[pslot].meta;
    uint32_t ch;
    if (!find_child(base, meta, w[i], &ch)) break;
    root = false;
    pslot = ch;
  }
  if (i == L) {  // the filter's node exists: set its id and flag
    if (final_hash && root) {
      root_hash_fid = ext;
      root_hash_id = id;
      root_meta |= META_HAS_HASH;
      loc[id] = FIDLOC_ROOT_HASH;
      return true;
    }
    EdgeSlot& sl = edges[pslot];
    if (final_hash) {
      fids[2 * pslot] = ext;
      sid[2 * pslot] = id;
      sl.meta |= META_HAS_HASH;
      loc[id] = pslot << 2 | FIDLOC_HASH;
    } else {
      fids[2 * pslot + 1] = ext;
      sid[2 * pslot + 1] = id;
      sl.meta |= META_HAS_TERM | (wild ? META_TERM_WILD : 0u);
      loc[id] = pslot << 2 | FIDLOC_TERM;
    }
    reencode(c, pslot);
    return true;
  }

  // new chain for levels i+1 .. L (bottom-up): the last node carries the filter
  const uint32_t fmeta = final_hash ? META_HAS_HASH : (META_HAS_TERM | (wild ? META_TERM_WILD : 0u));
  const uint32_t fh = final_hash ? ext : FID_NONE, ft = final_hash ? FID_NONE : ext;
  const uint32_t ih = final_hash ? id : WID_NONE, it = final_hash ? WID_NONE : id;
  EdgeSlot cur = encode(w[L - 1], false, 0, 0, fh, ft, fmeta);
  uint32_t cfh = fh, cft = ft, cih = ih, cit = it;
  for (uint32_t j = L - 1; j > i; --j) {  // node at depth j holds the edge w[j]
    uint64_t nb = 0;
    if (!alloc(c, 1, &nb)) return false;
    const bool plus = w[j] == WID_PLUS;
    const uint32_t at = plus ? 0u : lit_slot(w[j], 0, 1, false);
    edges[nb] = edges[nb + 1] = EMPTY_SLOT;
    for (uint64_t q = 2 * nb; q < 2 * nb + 4; ++q) {
      fids[q] = FID_NONE;
      sid[q] = WID_NONE;
    }
    const uint64_t ps = nb + at;
    edges[ps] = cur;
    fids[2 * ps] = cfh;
    fids[2 * ps + 1] = cft;
    sid[2 * ps] = cih;
    sid[2 * ps + 1] = cit;
    if (cih != WID_NONE) loc[cih] = ps << 2 | FIDLOC_HASH;
    if (cit != WID_NONE) loc[cit] = ps << 2 | FIDLOC_TERM;
    const uint32_t sm = 1u | META_HAS_EDGES | META_PH | (plus ? META_HAS_PLUS : 0u);
    cur = encode(w[j - 1], true, static_cast<uint32_t>(nb), sm, FID_NONE, FID_NONE, 0);
    cfh = cft = FID_NONE;
    cih = cit = WID_NONE;
    c.nodes += 1;
  }
  c.nodes += 1;
  c.max_depth = std::max(c.max_depth, L);
  c.chains += 1;
  return place(c, root, pslot, w[i], cur, cfh, cft, cih, cit);
}

bool LiveTrie::commit(const FilterStore& fs, const std::vector<uint32_t>& ids, int threads) {
  const bool prof_phases = commit_prof();
  mark = used;
  dirty.clear();
  ranges.clear();
  relocations = in_place = chains = flips = 0;
  if (loc.size() < fs.n_ids()) loc.resize(fs.n_ids(), FIDLOC_NONE);
  threads = std::max(1, threads);
  std::vector<uint32_t> fl, ins;
  for (uint32_t id : ids) {
    if (loc[id] != FIDLOC_NONE) fl.push_back(id);
    else if (fs.live[id]) ins.push_back(id);
  }
  std::vector<Ctx> cx(threads);
  auto run = [&](uint64_t n, auto&& body) {  // body(ctx, i) over [0, n) on up to `threads` threads
    const int t = static_cast<int>(std::min<uint64_t>(threads, (n + 255) / 256));
    if (t <= 1) {
      for (uint64_t i = 0; i < n; ++i) body(cx[0], i);
      return;
    }
    std::vector<std::thread> th;
    for (int k = 0; k < t; ++k)
      th.emplace_back([&, k] {
        for (uint64_t i = n * k / t; i < n * (k + 1) / t; ++i) body(cx[k], i);
      });
    for (auto& x : th) x.join();
  };

  const auto t0 = std::chrono::steady_clock::now();
  // 1. flips (the root's '#' filter serially)
  for (uint32_t id : fl)
    if (loc[id] == FIDLOC_ROOT_HASH) flip(cx[0], id, fs.live[id] != 0, false);
  run(fl.size(), [&](Ctx& c, uint64_t i) {
    const uint32_t id = fl[i];
    if (loc[id] != FIDLOC_ROOT_HASH) flip(c, id, fs.live[id] != 0, true);
  });
  for (Ctx& c : cx) {  // '+' edges flipped in place: their copies, serially (two flips may share one)
    for (uint32_t p : c.plus_heads) sync_plus(cx[0], p);
    c.plus_heads.clear();
  }

  const auto t1 = std::chrono::steady_clock::now();
  // 2. tokenize (read-only vocab lookups in parallel; unknown words interned serially)
  const uint64_t ni = ins.size();
  std::vector<uint64_t> woff(ni + 1, 0);
  std::vector<uint8_t> flags(ni, 0);  // bit 0 wild, bit 1 final '#', bit 2 unknown words
  std::vector<std::vector<uint32_t>> wl(ni);
  run(ni, [&](Ctx&, uint64_t k) {
    bool wild, fh;
    const bool known = tokenize(fs, ins[k], wl[k], &wild, &fh, false);
    flags[k] = (wild ? 1 : 0) | (fh ? 2 : 0) | (known ? 0 : 4);
  });
  for (uint64_t k = 0; k < ni; ++k)
    if (flags[k] & 4) {
      bool wild, fh;
      tokenize(fs, ins[k], wl[k], &wild, &fh, true);
    }

  const auto t2 = std::chrono::steady_clock::now();
  // 3. inserts that change the root (a new first-level edge, or the filter '#'), serially
  Ctx& c0 = cx[0];
  if (c0.ranges.empty()) c0.cur = c0.end = 0;
  std::vector<uint8_t> done(ni, 0);
  for (uint64_t k = 0; k < ni; ++k) {
    uint32_t ch;
    if (wl[k].empty() || !find_child(root_base, root_meta, wl[k][0], &ch)) {
      if (!insert(c0, fs, ins[k], wl[k], flags[k] & 1, flags[k] & 2, true, 0, 0)) return false;
      done[k] = 1;
    }
  }
  const auto t3 = std::chrono::steady_clock::now();
  // 4. the rest grouped by first-level node, groups dealt to threads (largest first)
  std::vector<std::pair<uint32_t, uint32_t>> key;  // (first-level slot, insert)
  key.reserve(ni);
  for (uint64_t k = 0; k < ni; ++k) {
    if (done[k]) continue;
    uint32_t ch = 0;
    find_child(root_base, root_meta, wl[k][0], &ch);
    key.push_back({ch, static_cast<uint32_t>(k)});
  }
  std::sort(key.begin(), key.end());
  std::vector<std::pair<uint64_t, uint64_t>> groups;  // [begin, end) in key
  for (uint64_t a = 0; a < key.size();) {
    uint64_t b = a;
    while (b < key.size() && key[b].first == key[a].first) ++b;
    groups.push_back({a, b});
    a = b;
  }
  const int t = static_cast<int>(std::min<uint64_t>(threads, std::max<uint64_t>(1, key.size() / 512)));
  std::vector<std::vector<uint32_t>> mine(t);
  {
    std::vector<uint64_t> load(t, 0);
    std::vector<uint32_t> order(groups.size());
    for (uint32_t g = 0; g < groups.size(); ++g) order[g] = g;
    std::sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) {
      return groups[x].second - groups[x].first > groups[y].second - groups[y].first;
    });
    for (uint32_t g : order) {
      const int k = static_cast<int>(std::min_element(load.begin(), load.end()) - load.begin());
      mine[k].push_back(g);
      load[k] += groups[g].second - groups[g].first;
    }
  }
  const auto t4 = std::chrono::steady_clock::now();
  auto work = [&](int k) {
    Ctx& c = cx[k];
    for (uint32_t g : mine[k])
      for (uint64_t j = groups[g].first; j < groups[g].second && !c.failed; ++j) {
        const uint32_t q = key[j].second;
        if (!insert(c, fs, ins[q], wl[q], flags[q] & 1, flags[q] & 2, false, key[j].first, 1)) c.failed = true;
      }
  };
  if (t <= 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int k = 0; k < t; ++k) th.emplace_back(work, k);
    for (auto& x : th) x.join();
  }

  const auto t5 = std::chrono::steady_clock::now();
  // 5. merge
  bool ok = true;
  for (Ctx& c : cx) {
    ok &= !c.failed;
    dirty.insert(dirty.end(), c.dirty.begin(), c.dirty.end());
    for (auto& r : c.ranges)
      if (r.second > r.first) ranges.push_back(r);
    garbage += c.garbage + (c.end - c.cur);
    relocations += c.relocations;
    in_place += c.in_place;
    chains += c.chains;
    flips += c.flips;
    n_nodes += c.nodes;
    max_depth = std::max(max_depth, c.max_depth);
  }
  std::sort(ranges.begin(), ranges.end());
  std::vector<std::pair<uint64_t, uint64_t>> merged;
  for (auto& r : ranges) {
    if (!merged.empty() && merged.back().second == r.first) merged.back().second = r.second;
    else merged.push_back(r);
  }
  ranges.swap(merged);
  if (prof_phases) {
    const auto t6 = std::chrono::steady_clock::now();
    auto ms = [](auto a, auto b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
    uint64_t rns = 0, pns = 0;
    for (Ctx& c : cx) {
      rns += c.reloc_ns;
      pns += c.ph_ns;
      c.reloc_ns = c.ph_ns = 0;
    }
    std::fprintf(stderr, "COMMIT_PROF flips %.3f tokenize %.3f root %.3f group %.3f insert %.3f merge %.3f (fl %zu ins %llu) "
                 "relocate %.3f (seed search %.3f) thread-ms\n",
                 ms(t0, t1), ms(t1, t2), ms(t2, t3), ms(t3, t4), ms(t4, t5), ms(t5, t6), fl.size(),
                 static_cast<unsigned long long>(ni), rns * 1e-6, pns * 1e-6);
  }
  return ok;
}

uint64_t LiveTrie::new_slots() const {
  uint64_t n = 0;
  for (auto& r : ranges) n += r.second - r.first;
  return n;
}

void sort_unique_u32(std::vector<uint32_t>& v) {
  if (v.size() < 64) {
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    return;
  }
  uint32_t mx = 0;
  for (uint32_t x : v) mx = std::max(mx, x);
  std::vector<uint32_t> tmp(v.size());
  std::vector<uint32_t> cnt(1u << 11);
  for (uint32_t sh = 0; sh < 32 && (sh == 0 || (mx >> sh) != 0); sh += 11) {
    std::fill(cnt.begin(), cnt.end(), 0u);
    for (uint32_t x : v) ++cnt[(x >> sh) & 2047u];
    uint32_t sum = 0;
    for (uint32_t& c : cnt) {
      const uint32_t t = c;
      c = sum;
      sum += t;
    }
    for (uint32_t x : v) tmp[cnt[(x >> sh) & 2047u]++] = x;
    v.swap(tmp);
  }
  v.erase(std::unique(v.begin(), v.end()), v.end());
}

void LiveTrie::patches(std::vector<SlotPatch>& out) const {
  std::vector<uint32_t> d(dirty);
  sort_unique_u32(d);
  out.clear();
  out.reserve(d.size());
  for (uint32_t p : d) out.push_back(SlotPatch{p, fids[2 * uint64_t(p)], fids[2 * uint64_t(p) + 1], 0, edges[p]});
}

}  // namespace emqx
