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
    *out = base + lit_slot(wid, sd, mask);
    return t.edges[*out].wid == wid;
  }
  const uint32_t nbm = mask >> 1, b1 = bucket1(wid, sd, nbm);
  for (uint32_t k = 0; k < 2; ++k)
    if (t.edges[base + 2 * b1 + k].wid == wid) {
      *out = base + 2 * b1 + k;
      return true;
    }
  if (!(t.edges[base + 2 * b1].meta & META_BUCKET_OVF)) return false;
  const uint32_t b2 = bucket2(wid, sd, nbm);
  for (uint32_t k = 0; k < 2; ++k)
    if (t.edges[base + 2 * b2 + k].wid == wid) {
      *out = base + 2 * b2 + k;
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
        if (i != 0 || !(it.meta & META_HAS_PLUS)) {
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
      if (s.meta & META_HAS_EDGES) st.push_back({s.child_base, s.meta, s.litf, false});
    }
    if ((it.meta & META_HAS_PLUS) && t.edges[it.base].wid != WID_PLUS) {
      *err = "missing '+' edge";
      return false;
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
