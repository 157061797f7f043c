// Host-only self-check of incremental commits (include/emqx_match.h, emqx_htrie_*): the same
// FilterStore + builder + LiveTrie the engine uses, with no device.  `match` walks the host
// image of the table by the kernel's rules — '+' in slot 0, perfect-hash / 2-slot-bucket
// literal probes gated by the parent slot's literal filter, filter ids read from inline leaf
// fields, XFID or fids[] exactly as the kernels read them — so a CPU test can compare a table
// patched by many incremental commits with the oracle (tests/test_live_trie.py) before any of
// it runs on the GPU.  Not on the product path.
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "../../include/emqx_match.h"
#include "tables.h"

using namespace emqx;

// The table as the device holds it: written only the way the engine writes device memory
// (the full build's slots; per incremental commit the new extents and the slot patches), so the
// host walk below sees exactly what the kernels would.
struct DevImage {
  std::vector<EdgeSlot> edges;
  std::vector<uint32_t> fids;
  uint32_t root_base = 0, root_meta = 0, root_hash_fid = FID_NONE;
  uint32_t plus_mask = 0;  // layout.h plus_copy
  uint64_t used = 0;
};

struct emqx_htrie {
  DevImage dev;
  FilterStore fs;
  std::unique_ptr<VocabState> vocab;
  LiveTrie lt;
  std::vector<uint32_t> dirty;
  bool built = false;
  uint64_t spare = 0;
  uint64_t kind = 0;
  int threads = 1;
};

namespace {

void full_build(emqx_htrie* h) {
  h->vocab = std::make_unique<VocabState>();
  std::vector<uint64_t> loc;
  std::vector<uint32_t> sids;
  BuildOpts o;
  o.vocab = h->vocab.get();
  o.fid_loc = &loc;
  o.slot_ids = &sids;
  o.threads = h->threads;
  HostTables ht;
  std::string err;
  build_tables(h->fs, o, ht, &err);
  const uint64_t spare = h->spare ? h->spare : std::max<uint64_t>(1u << 16, ht.edges.size() / 2);
  h->dev.edges.assign(ht.edges.size() + spare, EdgeSlot{WID_NONE, 0, 0, 0});
  h->dev.fids.assign(2 * (ht.edges.size() + spare), FID_NONE);
  std::copy(ht.edges.begin(), ht.edges.end(), h->dev.edges.begin());
  std::copy(ht.fids.begin(), ht.fids.end(), h->dev.fids.begin());
  h->dev.plus_mask = ht.plus_mask;
  h->lt.adopt(ht, loc, sids, spare, h->vocab.get());
  h->dev.edges.resize(h->lt.cap);
  h->dev.fids.resize(2 * h->lt.cap);
  h->built = true;
  h->kind = 0;
  h->dirty.clear();
}

uint32_t hash_id_of(const DevImage& t, uint64_t c) {
  const EdgeSlot& s = t.edges[c];
  if (!(s.meta & META_HAS_EDGES)) return s.child_base;
  if ((s.meta & META_XFID) && !(s.meta & META_XFID_TERM)) return s.litf;
  return t.fids[2 * c];
}

uint32_t term_id_of(const DevImage& t, uint64_t c) {
  const EdgeSlot& s = t.edges[c];
  if (!(s.meta & META_HAS_EDGES)) return s.litf;
  if ((s.meta & META_XFID) && (s.meta & META_XFID_TERM)) return s.litf;
  return t.fids[2 * c + 1];
}

// Lookup by the kernel's rule (match_kernels.hip probe_one).
bool probe(const DevImage& t, uint32_t base, uint32_t meta, uint32_t wid, uint64_t* out) {
  if (wid == WID_PLUS) {
    *out = base;
    return t.edges[base].wid == WID_PLUS;
  }
  const uint32_t mask = (1u << (meta & META_CAPLOG2_MASK)) - 1u;
  const uint32_t sd = (meta >> META_SEED_SHIFT) & 255u;
  if (meta & META_PH) {
    *out = base + lit_slot(wid, sd, mask, plus_copies(t.plus_mask, meta & META_HAS_PLUS, meta & META_CAPLOG2_MASK));
    return t.edges[*out].wid == wid;
  }
  const bool cp = plus_copies(t.plus_mask, meta & META_HAS_PLUS, meta & META_CAPLOG2_MASK);
  const uint32_t b1 = wide_slot(wid, sd, mask, cp, false);
  for (uint32_t k = 0; k < 2; ++k)
    if (t.edges[base + b1 + k].wid == wid) {
      *out = base + b1 + k;
      return true;
    }
  if (!(t.edges[base + b1].meta & META_BUCKET_OVF)) return false;
  const uint32_t b2 = wide_slot(wid, sd, mask, cp, true);
  for (uint32_t k = 0; k < 2; ++k)
    if (t.edges[base + b2 + k].wid == wid) {
      *out = base + b2 + k;
      return true;
    }
  return false;
}

struct Item {
  uint32_t base, meta, litf;
  bool root;
};

// Level-by-level frontier walk of one non-wildcard topic (emqx_trie.erl:272-334 semantics):
// every reached node emits its '#' filter, the last level emits terminal filters (all of them
// in ROUTES mode, wildcard ones in TRIE_WILDCARD mode); '$' topics skip the root's '+' and '#'.
void walk(const DevImage& t, const VocabState& v, const uint8_t* p, uint64_t n, uint32_t mode,
          std::vector<uint32_t>& out) {
  std::vector<uint32_t> w;
  uint64_t s = 0;
  for (uint64_t i = 0; i <= n; ++i) {
    if (i != n && p[i] != '/') continue;
    const uint64_t len = i - s;
    if (len == 1 && (p[s] == '+' || p[s] == '#')) return;  // wildcard topic: not supported here
    uint64_t hh = hash64_bytes(p + s, len);
    auto res = [&v](uint32_t id, const uint8_t*& q, uint64_t& m) {
      q = v.arena.data() + v.off[id];
      m = v.off[id + 1] - v.off[id];
    };
    w.push_back(v.map.find(p + s, len, hh, res));
    s = i + 1;
  }
  const bool dollar = n > 0 && p[0] == '$';
  if (!dollar && (t.root_meta & META_HAS_HASH)) out.push_back(t.root_hash_fid);
  std::vector<Item> fr, nx;
  if (t.root_meta & META_HAS_EDGES) fr.push_back({t.root_base, t.root_meta, 0, true});
  for (size_t i = 0; i < w.size() && !fr.empty(); ++i) {
    nx.clear();
    for (const Item& it : fr) {
      uint64_t c[2];
      int nc = 0;
      if ((it.meta & META_HAS_PLUS) && !(it.root && dollar) && probe(t, it.base, it.meta, WID_PLUS, &c[nc])) ++nc;
      if (w[i] != WID_NONE && (it.root || litf_may_contain(it.meta, it.litf, w[i])) &&
          probe(t, it.base, it.meta, w[i], &c[nc]))
        ++nc;
      for (int k = 0; k < nc; ++k) {
        const EdgeSlot& cs = t.edges[c[k]];
        if (cs.meta & META_HAS_HASH) out.push_back(hash_id_of(t, c[k]));
        if (i + 1 == w.size()) {
          if ((cs.meta & META_HAS_TERM) && (mode == EMQX_MODE_ROUTES || (cs.meta & META_TERM_WILD)))
            out.push_back(term_id_of(t, c[k]));
        } else if (cs.meta & META_HAS_EDGES) {
          nx.push_back({cs.child_base, cs.meta, cs.litf, false});
        }
      }
    }
    fr.swap(nx);
  }
}

// ---- L2 model of the fast kernel's walk (emqx_htrie_walk_sim; a diagnostic, not product) ----
// Replays match_fast_kernel's loads on this image: tiles of 64 topics, a pooled LIFO stack
// popped 64 items per step, '+' probe (slot 0) and literal probe (perfect-hash slot or 2-slot
// bucket) per item, children pushed by the kernel's rules; phase A's vocab probes at the
// tile's start.  Tiles are dealt to XCDs as blocks of 4 (block b -> XCD b mod 8), each XCD runs
// `resident` tiles at once, advancing one step each per tick, against its own set-associative
// LRU L2 of `sector`-byte lines.  Counts what the PMC passes count (L2 accesses, misses), split
// by item level and node kind, so layout ideas can be priced on the CPU before they are built.
struct SimItem {
  uint32_t base, meta, litf, widx;
  uint8_t topic, flags;  // flags: 1 root, 2 dollar root, 4 no literal probe, 8 chain parent,
                         // 16 spine (reached from the root by literal edges only)
};

struct SimL2 {
  uint32_t sets = 0, ways = 0;
  std::vector<uint64_t> tag;  // sets x ways, ~0 empty
  std::vector<uint64_t> age;
  uint64_t clock = 0;
  void init(uint64_t bytes, uint32_t sector, uint32_t w) {
    ways = w;
    sets = static_cast<uint32_t>(std::max<uint64_t>(1, bytes / sector / w));
    tag.assign(uint64_t(sets) * ways, ~0ull);
    age.assign(uint64_t(sets) * ways, 0);
  }
  bool access(uint64_t line) {  // true = hit
    const uint64_t s = (mix32(static_cast<uint32_t>(line)) ^ static_cast<uint32_t>(line >> 32)) % sets;
    uint64_t* t = tag.data() + s * ways;
    uint64_t* a = age.data() + s * ways;
    ++clock;
    uint32_t lru = 0;
    for (uint32_t i = 0; i < ways; ++i) {
      if (t[i] == line) {
        a[i] = clock;
        return true;
      }
      if (a[i] < a[lru]) lru = i;
    }
    t[lru] = line;
    a[lru] = clock;
    return false;
  }
};

enum SimOut : uint32_t {
  SO_TOPICS, SO_TILES, SO_ITEMS, SO_LOADS, SO_ACC, SO_MISS, SO_VLOADS, SO_VMISS, SO_BOTH, SO_BOTH_SPLIT,
  SO_CHAIN, SO_CHAIN_MISS, SO_MISS_L0, SO_ITEMS_L0 = SO_MISS_L0 + 8, SO_WIDE = SO_ITEMS_L0 + 8, SO_WIDE_MISS,
  SO_STEPS, SO_PLUS_MISS, SO_LIT_MISS, SO_EMITS, SO_PLUS_LOADS, SO_PH_LOADS, SO_WIDE_LOADS, SO_HITS_L0,
  SO_SPINE = SO_HITS_L0 + 8, SO_SPINE_LIT_MISS, SO_N
};

struct SimTile {
  std::vector<uint32_t> wids, wend;  // tile's word ids; per topic end index
  std::vector<SimItem> stack;
  uint64_t tile = 0, cursor = 0;     // emissions so far (slab entries of 8 B)
};

void sim_tile_init(const DevImage& t, const VocabState& v, const uint8_t* tb, const uint64_t* to, uint64_t t0,
                   uint64_t t1, SimTile& st, std::vector<uint64_t>& vaddr) {
  st.wids.clear();
  st.wend.clear();
  st.stack.clear();
  for (uint64_t q = t0; q < t1; ++q) {
    const uint8_t* p = tb + to[q];
    const uint64_t n = to[q + 1] - to[q];
    const uint32_t wb = static_cast<uint32_t>(st.wids.size());
    bool wild = false;
    uint64_t s = 0;
    for (uint64_t i = 0; i <= n; ++i) {
      if (i != n && p[i] != '/') continue;
      const uint64_t len = i - s;
      if (len == 1 && (p[s] == '+' || p[s] == '#')) wild = true;
      auto res = [&v](uint32_t id, const uint8_t*& qq, uint64_t& m) {
        qq = v.arena.data() + v.off[id];
        m = v.off[id + 1] - v.off[id];
      };
      const uint32_t w = v.map.find(p + s, len, hash64_bytes(p + s, len), res);
      st.wids.push_back(w);
      vaddr.push_back((2ull << 40) + 32ull * ((w == WID_NONE ? mix32(static_cast<uint32_t>(len) ^ p[s])
                                                             : v.h32[w]) & v.mask));
      s = i + 1;
    }
    st.wend.push_back(static_cast<uint32_t>(st.wids.size()));
    if (wild || !(t.root_meta & META_HAS_EDGES)) continue;
    const bool dollar = n > 0 && p[0] == '$';
    const uint32_t rmeta = dollar ? (t.root_meta & ~META_HAS_PLUS) : t.root_meta;
    st.stack.push_back({t.root_base, rmeta, 0, wb, static_cast<uint8_t>(q - t0),
                        static_cast<uint8_t>(1 | 16 | (dollar ? 2 : 0))});
  }
}

// One step of a tile: pops up to 64 items, appends (address, class) of every load.
// class: bit 0-2 level (7 = 7+), bit 3 '+' probe, bit 4 wide node, bit 5 chain item
// what-if flags (params[7]): bit 0 = a '+' copy in every 64-B line of a node array (the '+'
// probe reads the literal probe's line whenever the item probes both)
void sim_tile_step(const DevImage& t, SimTile& st, std::vector<std::pair<uint64_t, uint32_t>>& acc, uint64_t* o,
                   uint32_t whatif) {
  const size_t nb = std::min<size_t>(64, st.stack.size());
  std::vector<SimItem> pop(st.stack.end() - nb, st.stack.end());
  st.stack.resize(st.stack.size() - nb);
  std::vector<SimItem> push;
  for (const SimItem& it : pop) {
    const uint32_t wid = st.wids[it.widx];
    const uint32_t tl = it.topic;
    const uint32_t first = tl ? st.wend[tl - 1] : 0u;
    const uint32_t lvl = std::min<uint32_t>(it.widx - first, 7);
    const bool leaf = it.widx + 1 == st.wend[tl];
    const bool needL = wid != WID_NONE && !(it.flags & 4);
    const bool needP = (it.meta & META_HAS_PLUS) != 0;
    const uint32_t caplog = it.meta & META_CAPLOG2_MASK;
    const bool wide = needL && !(it.meta & META_PH);
    // a chain item: a node whose only edge is one literal (a unique filter suffix, typically)
    const bool chain = (it.meta & META_LITF_EXACT) && !needP && !(it.flags & 1);
    const bool spine = (it.flags & 16) != 0;
    const uint32_t cls = lvl | (wide ? 16u : 0u) | (chain ? 32u : 0u);
    const uint32_t lcls = cls | (spine ? 128u : 0u);  // (its literal probe: class bit 7 on the spine)
    o[SO_ITEMS] += 1;
    o[SO_SPINE] += spine ? 1 : 0;
    o[SO_ITEMS_L0 + lvl] += 1;
    o[SO_WIDE] += wide ? 1 : 0;
    o[SO_CHAIN] += chain ? 1 : 0;
    uint64_t c[2];
    int nc = 0, lit_k = -1;  // (lit_k: which child came through the literal edge)
    uint64_t pa = ~0ull, la = ~0ull;
    size_t plus_at = ~size_t(0);
    if (needP) {
      pa = it.base;
      plus_at = acc.size();
      acc.push_back({16ull * it.base, cls | 8u});
      o[SO_PLUS_LOADS] += 1;
      if (t.edges[it.base].wid == WID_PLUS) c[nc++] = it.base;
    }
    if (needL) {
      const uint32_t mask = (1u << caplog) - 1u, sd = (it.meta >> META_SEED_SHIFT) & 255u;
      uint64_t f = ~0ull;
      if (it.meta & META_PH) {
        la = it.base + lit_slot(wid, sd, mask, plus_copies(t.plus_mask, it.meta & META_HAS_PLUS, caplog));
        acc.push_back({16ull * la, lcls});
        o[SO_PH_LOADS] += 1;
        if (t.edges[la].wid == wid) f = la;
      } else {
        const bool cp = plus_copies(t.plus_mask, it.meta & META_HAS_PLUS, caplog);
        la = it.base + wide_slot(wid, sd, mask, cp, false);
        acc.push_back({16ull * la, lcls});
        acc.push_back({16ull * la + 16, lcls});
        o[SO_WIDE_LOADS] += 2;
        for (uint32_t k = 0; k < 2 && f == ~0ull; ++k)
          if (t.edges[la + k].wid == wid) f = la + k;
        if (f == ~0ull && (t.edges[la].meta & META_BUCKET_OVF)) {
          const uint64_t l2 = it.base + wide_slot(wid, sd, mask, cp, true);
          acc.push_back({16ull * l2, lcls});
          acc.push_back({16ull * l2 + 16, lcls});
          for (uint32_t k = 0; k < 2 && f == ~0ull; ++k)
            if (t.edges[l2 + k].wid == wid) f = l2 + k;
        }
      }
      if (f != ~0ull) {
        lit_k = nc;
        c[nc++] = f;
      }
    }
    if (plus_copies(t.plus_mask, needP, caplog) && plus_at != ~size_t(0) && la != ~0ull) {  // the copy in the literal's line
      acc[plus_at].first = 16ull * (it.base + plus_copy(static_cast<uint32_t>(la - it.base), true));
      std::swap(acc[plus_at], acc[plus_at + 1]);
    } else if ((whatif & 1u) && plus_at != ~size_t(0) && la != ~0ull) {  // '+' copy in the literal's line
      acc[plus_at].first = (16ull * la) & ~63ull;
      std::swap(acc[plus_at], acc[plus_at + 1]);  // next to the literal probe (one request)
    }
    if (pa != ~0ull && la != ~0ull) {
      o[SO_BOTH] += 1;
      o[SO_BOTH_SPLIT] += (pa * 16 / 64) != (la * 16 / 64) ? 1 : 0;
    }
    for (int k = 0; k < nc; ++k) {  // slab entries: the found child's '#' and terminal filters
      const EdgeSlot& cs = t.edges[c[k]];
      const uint32_t ne = ((cs.meta & META_HAS_HASH) ? 1u : 0u) + ((leaf && (cs.meta & META_HAS_TERM)) ? 1u : 0u);
      for (uint32_t e = 0; e < ne; ++e, ++st.cursor) acc.push_back({(3ull << 40) + (st.tile << 16) + 8 * st.cursor, 64u});
      o[SO_EMITS] += ne;
    }
    if (leaf) continue;
    const uint32_t nwid = st.wids[it.widx + 1];
    for (int k = 0; k < nc; ++k) {
      const EdgeSlot& cs = t.edges[c[k]];
      if (!(cs.meta & META_HAS_EDGES)) continue;
      const bool nl = nwid == WID_NONE || !litf_may_contain(cs.meta, cs.litf, nwid);
      if (nl && !(cs.meta & META_HAS_PLUS)) continue;
      push.push_back({cs.child_base, cs.meta, cs.litf, it.widx + 1, it.topic,
                      static_cast<uint8_t>((nl ? 4 : 0) | (spine && k == lit_k ? 16 : 0))});
    }
  }
  st.stack.insert(st.stack.end(), push.begin(), push.end());
}

// Lookup invariants of every node reachable from the root (garbage arrays left behind by
// relocations are not checked: nothing reaches them).
bool check(const DevImage& t, std::string* err) {
  std::vector<Item> st;
  if (t.root_meta & META_HAS_EDGES) st.push_back({t.root_base, t.root_meta, ~0u, true});
  while (!st.empty()) {
    const Item it = st.back();
    st.pop_back();
    const uint32_t cap = 1u << (it.meta & META_CAPLOG2_MASK);
    if (uint64_t(it.base) + cap > t.used) {
      *err = "edge array beyond the allocated slots";
      return false;
    }
    for (uint32_t i = 0; i < cap; ++i) {
      const uint64_t p = it.base + i;
      const EdgeSlot& s = t.edges[p];
      if (s.wid == WID_NONE) continue;
      uint64_t f = 0;
      if (s.wid == WID_PLUS) {
        if (!plus_position(i, plus_copies(t.plus_mask, true, it.meta & META_CAPLOG2_MASK)) ||
            !(it.meta & META_HAS_PLUS)) {
          *err = "'+' edge outside slot 0";
          return false;
        }
      } else {
        if (!probe(t, it.base, it.meta, s.wid, &f) || f != p) {
          *err = "edge not at its lookup slot";
          return false;
        }
        if (!it.root && !litf_may_contain(it.meta, it.litf, s.wid)) {
          *err = "literal filter rejects a present word";
          return false;
        }
      }
      if (((s.meta & META_HAS_HASH) && hash_id_of(t, p) == FID_NONE) ||
          ((s.meta & META_HAS_TERM) && term_id_of(t, p) == FID_NONE)) {
        *err = "a set filter flag without its filter id";
        return false;
      }
      if ((s.meta & META_HAS_EDGES) && (s.meta & META_XFID) &&
          s.litf != t.fids[2 * p + ((s.meta & META_XFID_TERM) ? 1 : 0)]) {
        *err = "XFID id disagrees with fids[]";
        return false;
      }
      if ((s.meta & META_HAS_EDGES) && !(s.wid == WID_PLUS && i != 0))  // (a '+' copy: slot 0's child)
        st.push_back({s.child_base, s.meta, s.litf, false});
    }
    if ((it.meta & META_HAS_PLUS) && t.edges[it.base].wid != WID_PLUS) {
      *err = "missing '+' edge";
      return false;
    }
    if (plus_copies(t.plus_mask, it.meta & META_HAS_PLUS, it.meta & META_CAPLOG2_MASK))  // line heads = slot 0
      for (uint32_t q = PLUS_LINE; q < cap; q += PLUS_LINE) {
        const EdgeSlot& a = t.edges[it.base], &b = t.edges[it.base + q];
        if (a.wid != b.wid || a.child_base != b.child_base || a.litf != b.litf ||
            (a.meta & ~META_BUCKET_OVF) != (b.meta & ~META_BUCKET_OVF) ||
            t.fids[2 * uint64_t(it.base)] != t.fids[2 * uint64_t(it.base + q)] ||
            t.fids[2 * uint64_t(it.base) + 1] != t.fids[2 * uint64_t(it.base + q) + 1]) {
          *err = "a '+' copy differs from slot 0";
          return false;
        }
      }
  }
  return true;
}

}  // namespace

extern "C" {

int emqx_htrie_create(uint64_t spare_slots, int threads, emqx_htrie** out) {
  if (!out) return EMQX_EINVAL;
  auto* h = new (std::nothrow) emqx_htrie();
  if (!h) return EMQX_ENOMEM;
  h->spare = spare_slots;
  h->threads = std::max(1, threads);
  *out = h;
  return EMQX_OK;
}

int emqx_htrie_destroy(emqx_htrie* h) {
  delete h;
  return EMQX_OK;
}

int emqx_htrie_insert(emqx_htrie* h, const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint32_t* ids_out) {
  if (!h || (n && !offsets)) return EMQX_EINVAL;
  for (uint64_t i = 0; i < n; ++i) {
    bool created = false;
    const uint32_t id = h->fs.insert(bytes + offsets[i], offsets[i + 1] - offsets[i], &created);
    h->dirty.push_back(id);
    if (ids_out) ids_out[i] = id;
  }
  return EMQX_OK;
}

int emqx_htrie_delete(emqx_htrie* h, const uint32_t* ids, uint64_t n) {
  if (!h || (n && !ids)) return EMQX_EINVAL;
  for (uint64_t i = 0; i < n; ++i) {
    if (ids[i] >= h->fs.n_ids()) return EMQX_ENOTFOUND;
    if (h->fs.live[ids[i]]) {
      h->fs.live[ids[i]] = 0;
      h->fs.n_live -= 1;
      h->dirty.push_back(ids[i]);
    }
  }
  return EMQX_OK;
}

int emqx_htrie_commit(emqx_htrie* h, int full, uint64_t* stats8) {
  if (!h) return EMQX_EINVAL;
  if (full || !h->built) {
    full_build(h);
  } else {
    std::vector<uint32_t> ids(h->dirty);
    std::sort(ids.begin(), ids.end());
    ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
    const bool ok = h->lt.commit(h->fs, ids, h->threads);
    h->kind = 1;
    if (ok) {  // the engine's device writes: new extents, then filter ids, then slots
      for (const auto& r : h->lt.ranges) {
        std::copy(h->lt.edges.begin() + r.first, h->lt.edges.begin() + r.second, h->dev.edges.begin() + r.first);
        std::copy(h->lt.fids.begin() + 2 * r.first, h->lt.fids.begin() + 2 * r.second,
                  h->dev.fids.begin() + 2 * r.first);
      }
      std::vector<SlotPatch> p;
      h->lt.patches(p);
      for (const SlotPatch& q : p) {
        h->dev.fids[2 * uint64_t(q.slot)] = q.fid_h;
        h->dev.fids[2 * uint64_t(q.slot) + 1] = q.fid_t;
      }
      for (const SlotPatch& q : p) h->dev.edges[q.slot] = q.s;
    } else {
      full_build(h);  // spare region exhausted
    }
    h->dirty.clear();
  }
  h->dev.root_base = h->lt.root_base;  // the snapshot's table view
  h->dev.root_meta = h->lt.root_meta;
  h->dev.root_hash_fid = h->lt.root_hash_fid;
  h->dev.used = h->lt.used;
  if (stats8) {
    std::vector<SlotPatch> p;
    h->lt.patches(p);
    const uint64_t v[8] = {h->kind, h->lt.relocations, h->lt.in_place, p.size(), h->lt.new_slots(),
                           h->lt.used, h->lt.cap, h->lt.garbage};
    std::memcpy(stats8, v, sizeof(v));
  }
  return EMQX_OK;
}

int emqx_htrie_match(emqx_htrie* h, uint32_t mode, const uint8_t* topic_bytes, const uint64_t* topic_offsets,
                     uint64_t n, uint64_t* out_offsets, uint32_t* out_ids, uint64_t cap, uint64_t* n_out) {
  if (!h || !h->built || !out_offsets || !n_out || (mode != EMQX_MODE_ROUTES && mode != EMQX_MODE_TRIE_WILDCARD))
    return EMQX_EINVAL;
  std::vector<uint32_t> acc, one;
  out_offsets[0] = 0;
  for (uint64_t i = 0; i < n; ++i) {
    one.clear();
    walk(h->dev, *h->vocab, topic_bytes + topic_offsets[i], topic_offsets[i + 1] - topic_offsets[i], mode, one);
    acc.insert(acc.end(), one.begin(), one.end());
    out_offsets[i + 1] = acc.size();
  }
  *n_out = acc.size();
  if (acc.size() > cap) return EMQX_EOVERFLOW;
  if (!acc.empty()) std::memcpy(out_ids, acc.data(), acc.size() * sizeof(uint32_t));
  return EMQX_OK;
}

int emqx_htrie_walk_sim(emqx_htrie* h, const uint8_t* topic_bytes, const uint64_t* topic_offsets, uint64_t n,
                        const uint64_t* params, uint64_t* out, uint32_t n_out) {
  if (!h || !h->built || !params || !out || (n && !topic_offsets)) return EMQX_EINVAL;
  const uint32_t xcds = static_cast<uint32_t>(std::max<uint64_t>(1, params[0]));
  const uint64_t l2_bytes = params[1];
  const uint32_t sector = static_cast<uint32_t>(std::max<uint64_t>(16, params[2]));
  const uint32_t ways = static_cast<uint32_t>(std::max<uint64_t>(1, params[3]));
  const uint32_t resident = static_cast<uint32_t>(std::max<uint64_t>(1, params[4]));
  const uint32_t a_ticks = static_cast<uint32_t>(params[5]);  // ticks a tile spends in phase A
  const uint32_t slab_mode = static_cast<uint32_t>(params[6]);  // 1: slab writes allocate in L2
  const uint32_t whatif = static_cast<uint32_t>(params[7]);
  std::vector<uint64_t> o(SO_N, 0);
  const uint64_t ntiles = (n + 63) / 64;
  std::vector<std::vector<uint64_t>> queue(xcds);
  for (uint64_t tile = 0; tile < ntiles; ++tile) queue[(tile / 4) % xcds].push_back(tile);
  std::vector<SimL2> l2(xcds);
  for (auto& c : l2) c.init(l2_bytes, sector, ways);
  struct Slot {
    SimTile st;
    uint64_t tile = ~0ull;
    uint32_t wait = 0;
  };
  std::vector<std::pair<uint64_t, uint32_t>> acc;
  std::vector<uint64_t> vaddr;
  for (uint32_t x = 0; x < xcds; ++x) {
    std::vector<Slot> slots(resident);
    size_t next = 0;
    SimL2& c = l2[x];
    bool any = true;
    while (any) {
      any = false;
      for (Slot& s : slots) {
        if (s.tile == ~0ull) {
          if (next >= queue[x].size()) continue;
          s.tile = queue[x][next++];
          const uint64_t t0 = s.tile * 64, t1 = std::min<uint64_t>(n, t0 + 64);
          vaddr.clear();
          sim_tile_init(h->dev, *h->vocab, topic_bytes, topic_offsets, t0, t1, s.st, vaddr);
          s.st.tile = s.tile;
          s.st.cursor = 0;
          for (uint64_t a : vaddr) {
            o[SO_VLOADS] += 1;
            o[SO_VMISS] += c.access(a / sector) ? 0 : 1;
          }
          o[SO_TILES] += 1;
          o[SO_TOPICS] += t1 - t0;
          s.wait = a_ticks;
        }
        any = true;
        if (s.wait) {
          --s.wait;
          continue;
        }
        if (s.st.stack.empty()) {
          s.tile = ~0ull;
          continue;
        }
        acc.clear();
        sim_tile_step(h->dev, s.st, acc, o.data(), whatif);
        o[SO_STEPS] += 1;
        uint64_t last = ~0ull;
        for (const auto& [addr, cls] : acc) {
          const uint64_t line = addr / sector;
          if (cls & 64u) {  // a slab write: allocates in L2 (write-back) unless streamed past it
            if (slab_mode == 1 && line != last) (void)c.access(line);
            last = line;
            continue;
          }
          o[SO_LOADS] += 1;
          if (line == last) continue;  // the second slot of a bucket: same line, one request
          last = line;
          o[SO_ACC] += 1;
          if (c.access(line)) {
            o[SO_HITS_L0 + (cls & 7u)] += 1;
          } else {
            o[SO_MISS] += 1;
            o[SO_MISS_L0 + (cls & 7u)] += 1;
            o[SO_WIDE_MISS] += (cls & 16u) ? 1 : 0;
            o[SO_CHAIN_MISS] += (cls & 32u) ? 1 : 0;
            o[(cls & 8u) ? SO_PLUS_MISS : SO_LIT_MISS] += 1;
            o[SO_SPINE_LIT_MISS] += (cls & 128u) ? 1 : 0;
          }
        }
      }
    }
  }
  for (uint32_t i = 0; i < n_out && i < SO_N; ++i) out[i] = o[i];
  return EMQX_OK;
}

int emqx_htrie_check(emqx_htrie* h, char* err, uint64_t err_cap) {
  if (!h || !h->built) return EMQX_EINVAL;
  std::string e;
  const bool ok = check(h->dev, &e);
  if (!ok && err && err_cap) {
    strncpy(err, e.c_str(), err_cap - 1);
    err[err_cap - 1] = 0;
  }
  return ok ? EMQX_OK : EMQX_EINVAL;
}

}  // extern "C"
