// Host builder: live filter set -> level trie in the device layout of layout.h.
//
// Semantics carried over from the reference (paths relative to /root/reference):
//  * levels are the '/'-split tokens, empty levels kept (emqx_topic.erl:153-164);
//  * '+' and '#' are wildcards only when a level is exactly that byte (emqx_topic.erl:161-163);
//  * a filter is a wildcard filter iff some level is '+' or '#' (emqx_topic.erl:53-62) —
//    recorded per terminal node (META_TERM_WILD) so the kernel can serve
//    emqx_trie:match (wildcard filters only) and emqx_router:match_routes (all filters);
//  * a final '#' matches the parent level and anything below (emqx_topic.erl:80), so it is
//    stored as the parent's hash filter; a non-final '#' (never matched by a topic, only by
//    a byte-identical wildcard "topic", emqx_router.erl:130) is an ordinary edge WID_HASH.
#include "tables.h"

#include <algorithm>
#include <cstring>

namespace emqx {

namespace {

inline uint64_t rd64(const uint8_t* p) {
  uint64_t v;
  std::memcpy(&v, p, 8);
  return v;
}

inline uint64_t mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

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

// Open-addressed u64 -> u32 map for (parent, word) -> child.
class EdgeMap {
 public:
  static constexpr uint64_t EMPTY = ~0ull;
  void reserve(uint64_t n) {
    uint64_t cap = next_pow2(n * 2 + 16);
    if (cap > keys_.size()) rehash(cap);
  }
  // returns existing value or inserts `v` and returns it; *inserted set accordingly
  uint32_t get_or_insert(uint64_t key, uint32_t v, bool* inserted) {
    if ((size_ + 1) * 2 > keys_.size()) rehash(keys_.empty() ? 1024 : keys_.size() * 2);
    uint64_t mask = keys_.size() - 1;
    for (uint64_t i = mix64(key) & mask;; i = (i + 1) & mask) {
      if (keys_[i] == key) {
        *inserted = false;
        return vals_[i];
      }
      if (keys_[i] == EMPTY) {
        keys_[i] = key;
        vals_[i] = v;
        ++size_;
        *inserted = true;
        return v;
      }
    }
  }
  template <class F>
  void for_each(F&& f) const {
    for (uint64_t i = 0; i < keys_.size(); ++i)
      if (keys_[i] != EMPTY) f(keys_[i], vals_[i]);
  }
  uint64_t size() const { return size_; }

 private:
  void rehash(uint64_t cap) {
    std::vector<uint64_t> ok;
    std::vector<uint32_t> ov;
    ok.swap(keys_);
    ov.swap(vals_);
    keys_.assign(cap, EMPTY);
    vals_.assign(cap, 0);
    uint64_t mask = cap - 1;
    for (uint64_t j = 0; j < ok.size(); ++j) {
      if (ok[j] == EMPTY) continue;
      uint64_t i = mix64(ok[j]) & mask;
      while (keys_[i] != EMPTY) i = (i + 1) & mask;
      keys_[i] = ok[j];
      vals_[i] = ov[j];
    }
  }
  std::vector<uint64_t> keys_;
  std::vector<uint32_t> vals_;
  uint64_t size_ = 0;
};

struct VocabBuilder {
  std::vector<uint8_t> arena;
  std::vector<uint32_t> off{0};
  std::vector<uint32_t> h32;
  StrIdMap map;

  uint32_t intern(const uint8_t* p, uint64_t n) {
    uint64_t h = hash64_bytes(p, n);
    auto res = [this](uint32_t id, const uint8_t*& q, uint64_t& m) {
      q = arena.data() + off[id];
      m = off[id + 1] - off[id];
    };
    uint32_t id = map.find(p, n, h, res);
    if (id != WID_NONE) return id;
    id = static_cast<uint32_t>(h32.size());
    arena.insert(arena.end(), p, p + n);
    off.push_back(static_cast<uint32_t>(arena.size()));
    uint32_t f = FNV_BASIS;
    for (uint64_t i = 0; i < n; ++i) f = fnv1a_step(f, p[i]);
    h32.push_back(f);
    map.insert_new(h, id);
    return id;
  }
};

}  // namespace

uint64_t hash64_bytes(const uint8_t* p, uint64_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ULL ^ (n * 0xff51afd7ed558ccdULL);
  uint64_t i = 0;
  for (; i + 8 <= n; i += 8) h = mix64(h ^ rd64(p + i)) + 0x632BE59BD9B4E019ULL;
  uint64_t t = 0;
  for (uint64_t k = 0; i + k < n; ++k) t |= uint64_t(p[i + k]) << (8 * k);
  h = mix64(h ^ t ^ 0x94D049BB133111EBULL);
  return h == EdgeMap::EMPTY ? 0 : h;
}

void StrIdMap::reserve(uint64_t n) {
  uint64_t cap = next_pow2(n * 2 + 16);
  if (cap <= keys_.size()) return;
  std::vector<uint64_t> ok;
  std::vector<uint32_t> ov;
  ok.swap(keys_);
  ov.swap(vals_);
  keys_.assign(cap, 0);
  vals_.assign(cap, WID_NONE);
  uint64_t mask = cap - 1;
  for (uint64_t j = 0; j < ok.size(); ++j) {
    if (ov[j] == WID_NONE) continue;
    uint64_t i = ok[j] & mask;
    while (vals_[i] != WID_NONE) i = (i + 1) & mask;
    keys_[i] = ok[j];
    vals_[i] = ov[j];
  }
}

void StrIdMap::grow() { reserve(keys_.empty() ? 512 : keys_.size()); }

void StrIdMap::insert_new(uint64_t h, uint32_t id) {
  if ((size_ + 1) * 2 > keys_.size()) grow();
  uint64_t mask = keys_.size() - 1;
  uint64_t i = h & mask;
  while (vals_[i] != WID_NONE) i = (i + 1) & mask;
  keys_[i] = h;
  vals_[i] = id;
  ++size_;
}

uint32_t FilterStore::find(const uint8_t* p, uint64_t n) const {
  uint64_t h = hash64_bytes(p, n);
  auto res = [this](uint32_t id, const uint8_t*& q, uint64_t& m) {
    q = bytes.data() + off[id];
    m = off[id + 1] - off[id];
  };
  return index.find(p, n, h, res);
}

uint32_t FilterStore::insert(const uint8_t* p, uint64_t n, bool* created) {
  uint64_t h = hash64_bytes(p, n);
  auto res = [this](uint32_t id, const uint8_t*& q, uint64_t& m) {
    q = bytes.data() + off[id];
    m = off[id + 1] - off[id];
  };
  uint32_t id = index.find(p, n, h, res);
  if (id != WID_NONE) {
    *created = false;
    if (!live[id]) {
      live[id] = 1;
      ++n_live;
    }
    return id;
  }
  id = static_cast<uint32_t>(live.size());
  bytes.insert(bytes.end(), p, p + n);
  off.push_back(bytes.size());
  live.push_back(1);
  ++n_live;
  index.insert_new(h, id);
  *created = true;
  return id;
}

bool build_tables(const FilterStore& fs, HostTables& out, std::string* err) {
  // ---- pass 1: intern words, build the level trie (old node ids) -----------------
  VocabBuilder vb;
  vb.map.reserve(1024);
  EdgeMap em;
  em.reserve(fs.n_live * 2 + 16);
  std::vector<uint32_t> depth{0}, n_edges{0};
  std::vector<uint8_t> has_plus{0}, term_wild{0};
  std::vector<uint32_t> hash_fid{FID_NONE}, term_fid{FID_NONE};
  uint32_t max_depth = 0;

  const uint64_t n_ids = fs.n_ids();
  for (uint64_t id = 0; id < n_ids; ++id) {
    if (!fs.live[id]) continue;
    const uint8_t* p = fs.bytes.data() + fs.off[id];
    const uint64_t n = fs.off[id + 1] - fs.off[id];
    // wildcard? (emqx_topic:wildcard/1)
    bool wild = false;
    {
      uint64_t s = 0;
      for (uint64_t i = 0; i <= n; ++i) {
        if (i == n || p[i] == '/') {
          if (i - s == 1 && (p[s] == '+' || p[s] == '#')) wild = true;
          s = i + 1;
        }
      }
    }
    uint32_t node = 0;
    bool ended_hash = false;
    uint64_t s = 0;
    for (uint64_t i = 0; i <= n; ++i) {
      if (i != n && p[i] != '/') continue;
      const uint64_t len = i - s;
      uint32_t wid;
      if (len == 1 && p[s] == '+') {
        wid = WID_PLUS;
      } else if (len == 1 && p[s] == '#') {
        if (i == n) {  // final '#': the parent level's hash filter
          hash_fid[node] = static_cast<uint32_t>(id);
          ended_hash = true;
          break;
        }
        wid = WID_HASH;
      } else {
        wid = vb.intern(p + s, len);
      }
      const uint64_t key = (uint64_t(node) << 32) | wid;
      bool inserted = false;
      const uint32_t next_id = static_cast<uint32_t>(depth.size());
      const uint32_t child = em.get_or_insert(key, next_id, &inserted);
      if (inserted) {
        if (depth.size() >= 0xFFFFFFF0u) {
          if (err) *err = "too many trie nodes";
          return false;
        }
        depth.push_back(depth[node] + 1);
        max_depth = std::max(max_depth, depth[node] + 1);
        n_edges.push_back(0);
        has_plus.push_back(0);
        term_wild.push_back(0);
        hash_fid.push_back(FID_NONE);
        term_fid.push_back(FID_NONE);
        n_edges[node] += 1;
        if (wid == WID_PLUS) has_plus[node] = 1;
      }
      node = child;
      s = i + 1;
    }
    if (!ended_hash) {
      term_fid[node] = static_cast<uint32_t>(id);
      term_wild[node] = wild ? 1 : 0;
    }
  }

  const uint64_t n_nodes = depth.size();
  // ---- pass 2: layout — BFS by depth, larger arrays first (natural alignment) -------
  std::vector<uint32_t> caplog(n_nodes, 0);
  for (uint64_t v = 0; v < n_nodes; ++v) {
    uint32_t e = n_edges[v];
    caplog[v] = e ? log2u(next_pow2(uint64_t(e) + e / 2 + 1)) : 0;
  }
  std::vector<uint32_t> order(n_nodes);
  for (uint64_t v = 0; v < n_nodes; ++v) order[v] = static_cast<uint32_t>(v);
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
    if (depth[a] != depth[b]) return depth[a] < depth[b];
    return caplog[a] > caplog[b];
  });
  std::vector<uint32_t> new_id(n_nodes), base(n_nodes, 0);
  uint64_t total_slots = 0;
  for (uint64_t k = 0; k < n_nodes; ++k) {
    const uint32_t v = order[k];
    new_id[v] = static_cast<uint32_t>(k);
    if (n_edges[v]) {
      base[v] = static_cast<uint32_t>(total_slots);
      total_slots += 1ull << caplog[v];
      if (total_slots >= 0xFFFFFFF0ull) {
        if (err) *err = "edge slot array exceeds 2^32 slots";
        return false;
      }
    }
  }
  auto meta_of = [&](uint32_t v) -> uint32_t {
    uint32_t m = caplog[v] & META_CAPLOG2_MASK;
    if (n_edges[v]) m |= META_HAS_EDGES;
    if (has_plus[v]) m |= META_HAS_PLUS;
    if (hash_fid[v] != FID_NONE) m |= META_HAS_HASH;
    if (term_fid[v] != FID_NONE) m |= META_HAS_TERM;
    if (term_wild[v]) m |= META_TERM_WILD;
    return m;
  };

  out.edges.assign(std::max<uint64_t>(total_slots, 1),
                   EdgeSlot{WID_NONE, 0, 0, 0, FID_NONE, FID_NONE, 0, 0});
  auto fill = [&](uint32_t parent, uint32_t wid, uint32_t child) {
    const uint32_t mask = (1u << caplog[parent]) - 1;
    uint32_t i = (wid == WID_PLUS) ? 0u : (mix32(wid) & mask);  // '+' pinned at slot 0
    while (out.edges[base[parent] + i].wid != WID_NONE) i = (i + 1) & mask;
    EdgeSlot& s = out.edges[base[parent] + i];
    s.wid = wid;
    s.child_base = base[child];
    s.meta = meta_of(child);
    s.child = new_id[child];
    s.hash_fid = hash_fid[child];
    s.term_fid = term_fid[child];
  };
  // '+' edges first so that each one lands in slot 0 of its parent's array
  em.for_each([&](uint64_t key, uint32_t child) {
    if (static_cast<uint32_t>(key) == WID_PLUS) fill(static_cast<uint32_t>(key >> 32), WID_PLUS, child);
  });
  em.for_each([&](uint64_t key, uint32_t child) {
    const uint32_t wid = static_cast<uint32_t>(key);
    if (wid != WID_PLUS) fill(static_cast<uint32_t>(key >> 32), wid, child);
  });
  out.root_hash_fid = hash_fid[0];
  out.root_base = base[0];
  out.root_meta = meta_of(0);
  out.n_nodes = n_nodes;
  out.max_depth = max_depth;

  // ---- vocab device table ----------------------------------------------------------
  const uint64_t nw = vb.h32.size();
  const uint64_t vcap = next_pow2(std::max<uint64_t>(nw * 2, 2));
  out.vocab.assign(vcap, VocabSlot{0, 0, WID_NONE, 0, {0, 0, 0, 0}});
  out.vocab_mask = static_cast<uint32_t>(vcap - 1);
  for (uint64_t w = 0; w < nw; ++w) {
    const uint32_t h = vb.h32[w];
    uint32_t i = vocab_slot0(h) & out.vocab_mask;
    while (out.vocab[i].wid != WID_NONE) i = (i + 1) & out.vocab_mask;
    VocabSlot& s = out.vocab[i];
    s.hash = h;
    s.off = vb.off[w];
    s.len = vb.off[w + 1] - vb.off[w];
    s.wid = static_cast<uint32_t>(w);
    uint8_t tmp[16] = {0};
    std::memcpy(tmp, vb.arena.data() + s.off, std::min<uint32_t>(s.len, 16));
    std::memcpy(s.inl, tmp, 16);
  }
  out.arena.swap(vb.arena);
  if (out.arena.empty()) out.arena.push_back(0);
  out.n_words = nw;
  return true;
}

}  // namespace emqx
