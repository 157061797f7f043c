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
#include <atomic>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstdlib>
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
  void swap_into(EdgeMap& o) {  // o takes this (empty) map's state: frees o's memory
    keys_.swap(o.keys_);
    vals_.swap(o.vals_);
    std::swap(size_, o.size_);
  }

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

// fn(begin, end, thread) over [0, n) in chunks taken first come, first served by `threads`
// host threads (the calling thread is one of them).  The per-node passes of build_tables write
// disjoint per-node state, so they need no other synchronisation.
template <class F>
void parallel_chunks(uint64_t n, int threads, uint64_t chunk, F&& fn) {
  const int t = static_cast<int>(std::max<uint64_t>(1, std::min<uint64_t>(threads, (n + chunk - 1) / chunk)));
  if (t <= 1) {
    if (n) fn(0, n, 0);
    return;
  }
  std::atomic<uint64_t> next{0};
  auto run = [&](int k) {
    for (;;) {
      const uint64_t b = next.fetch_add(chunk);
      if (b >= n) return;
      fn(b, std::min(n, b + chunk), k);
    }
  };
  std::vector<std::thread> th;
  for (int k = 1; k < t; ++k) th.emplace_back(run, k);
  run(0);
  for (auto& x : th) x.join();
}

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

uint32_t VocabState::intern(const uint8_t* p, uint64_t n) {
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
  h32.push_back(word_hash_bytes(p, static_cast<uint32_t>(n)));
  map.insert_new(h, id);
  return id;
}

namespace {
void vocab_put(VocabState& v, uint64_t w, uint32_t* at) {
  uint32_t i = vocab_slot0(v.h32[w]) & v.mask;
  while (v.table[i].wid != WID_NONE) i = (i + 1) & v.mask;
  VocabSlot& s = v.table[i];
  s.hash = v.h32[w];
  s.off = v.off[w];
  s.len = v.off[w + 1] - v.off[w];
  s.wid = static_cast<uint32_t>(w);
  uint8_t tmp[16] = {0};
  std::memcpy(tmp, v.arena.data() + s.off, std::min<uint32_t>(s.len, 16));
  std::memcpy(s.inl, tmp, 16);
  *at = i;
}
}  // namespace

void VocabState::build_table() {
  const uint64_t nw = n_words();
  const uint64_t vcap = next_pow2(std::max<uint64_t>(nw * 3, 1024));  // load <= 1/3: room to grow
  table.assign(vcap, VocabSlot{0, 0, WID_NONE, 0, {0, 0, 0, 0}});
  mask = static_cast<uint32_t>(vcap - 1);
  uint32_t at;
  for (uint64_t w = 0; w < nw; ++w) vocab_put(*this, w, &at);
}

bool VocabState::insert_table(uint64_t from, std::vector<uint32_t>* dirty) {
  if (n_words() * 2 > table.size()) return false;
  uint32_t at;
  for (uint64_t w = from; w < n_words(); ++w) {
    vocab_put(*this, w, &at);
    if (dirty) dirty->push_back(at);
  }
  return true;
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
  ext.push_back(id);
  ++n_live;
  index.insert_new(h, id);
  *created = true;
  return id;
}

bool build_tables(const FilterStore& fs, const BuildOpts& opts, HostTables& out, std::string* err) {
  // ---- pass 1: intern words, build the level trie (old node ids) -----------------
  // Filters are partitioned by their first level's bytes, so no two partitions create the
  // same edge (the root's edges are split by word, everything below hangs off one of them).
  // Each partition builds its own sub-trie with its own interner on its own thread; the
  // merge renumbers nodes (root shared, then partition after partition) and maps each
  // partition's words to the global interner in partition order.  One partition (few
  // filters or one thread) interns into the global interner directly.
  VocabState own;
  VocabState& vb = opts.vocab ? *opts.vocab : own;
  vb.map.reserve(1024);
  const uint64_t n_sel = opts.ids ? opts.ids->size() : fs.n_live;
  const int nthreads = std::max(1, opts.threads);
  const uint64_t n_ids = fs.n_ids();
  const uint64_t n_iter = opts.ids ? opts.ids->size() : n_ids;
  const uint32_t nparts = n_sel >= 200000 ? static_cast<uint32_t>(std::min(nthreads, 64)) : 1u;

  struct Part {
    VocabState lv;  // partition interner (nparts > 1)
    EdgeMap em;
    std::vector<uint32_t> ids;
    std::vector<uint32_t> depth{0}, n_edges{0}, hash_fid{FID_NONE}, term_fid{FID_NONE};
    std::vector<uint32_t> hash_id{WID_NONE}, term_id{WID_NONE}, parent_of{0}, wid_of{WID_NONE};
    std::vector<uint8_t> has_plus{0}, term_wild{0};
    uint32_t max_depth = 0;
    bool too_many = false;
  };
  std::vector<Part> parts(nparts);
  for (uint64_t k = 0; k < n_iter; ++k) {
    const uint64_t id = opts.ids ? (*opts.ids)[k] : k;
    if (id >= n_ids || !fs.live[id]) continue;
    uint32_t pt = 0;
    if (nparts > 1) {
      const uint8_t* p = fs.bytes.data() + fs.off[id];
      const uint64_t n = fs.off[id + 1] - fs.off[id];
      uint64_t e = 0;
      while (e < n && p[e] != '/') ++e;
      pt = static_cast<uint32_t>(hash64_bytes(p, e) % nparts);
    }
    parts[pt].ids.push_back(static_cast<uint32_t>(id));
  }
  auto insert_part = [&](Part& P, VocabState& iv) {
    P.lv.map.reserve(1024);
    P.em.reserve(P.ids.size() * 2 + 16);
    for (uint32_t id : P.ids) {
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
            P.hash_fid[node] = fs.ext[id];
            P.hash_id[node] = id;
            ended_hash = true;
            break;
          }
          wid = WID_HASH;
        } else {
          wid = iv.intern(p + s, len);
        }
        const uint64_t key = (uint64_t(node) << 32) | wid;
        bool inserted = false;
        const uint32_t next_id = static_cast<uint32_t>(P.depth.size());
        const uint32_t child = P.em.get_or_insert(key, next_id, &inserted);
        if (inserted) {
          if (P.depth.size() >= 0xFFFFFFF0u / nparts) {
            P.too_many = true;
            return;
          }
          P.depth.push_back(P.depth[node] + 1);
          P.max_depth = std::max(P.max_depth, P.depth[node] + 1);
          P.n_edges.push_back(0);
          P.has_plus.push_back(0);
          P.term_wild.push_back(0);
          P.hash_fid.push_back(FID_NONE);
          P.term_fid.push_back(FID_NONE);
          P.hash_id.push_back(WID_NONE);
          P.term_id.push_back(WID_NONE);
          P.parent_of.push_back(node);
          P.wid_of.push_back(wid);
          P.n_edges[node] += 1;
          if (wid == WID_PLUS) P.has_plus[node] = 1;
        }
        node = child;
        s = i + 1;
      }
      if (!ended_hash) {
        P.term_fid[node] = fs.ext[id];
        P.term_id[node] = id;
        P.term_wild[node] = wild ? 1 : 0;
      }
    }
    EdgeMap().swap_into(P.em);  // the edge map is not needed past pass 1
  };
  if (nparts == 1) {
    insert_part(parts[0], vb);
  } else {
    std::vector<std::thread> th;
    for (uint32_t t = 1; t < nparts; ++t) th.emplace_back([&, t] { insert_part(parts[t], parts[t].lv); });
    insert_part(parts[0], parts[0].lv);
    for (auto& x : th) x.join();
  }
  uint64_t total_nodes = 1;
  for (const Part& P : parts) {
    if (P.too_many) {
      if (err) *err = "too many trie nodes";
      return false;
    }
    total_nodes += P.depth.size() - 1;
  }
  if (total_nodes >= 0xFFFFFFF0u) {
    if (err) *err = "too many trie nodes";
    return false;
  }
  std::vector<uint32_t> depth, n_edges, hash_fid, term_fid, hash_id, term_id, parent_of, wid_of;
  std::vector<uint8_t> has_plus, term_wild;
  uint32_t max_depth = 0;
  if (nparts == 1) {
    Part& P = parts[0];
    depth.swap(P.depth);
    n_edges.swap(P.n_edges);
    hash_fid.swap(P.hash_fid);
    term_fid.swap(P.term_fid);
    hash_id.swap(P.hash_id);
    term_id.swap(P.term_id);
    parent_of.swap(P.parent_of);
    wid_of.swap(P.wid_of);
    has_plus.swap(P.has_plus);
    term_wild.swap(P.term_wild);
    max_depth = P.max_depth;
  } else {
    // global word ids of each partition's words, partition after partition
    std::vector<std::vector<uint32_t>> gw(nparts);
    for (uint32_t t = 0; t < nparts; ++t) {
      const VocabState& lv = parts[t].lv;
      gw[t].resize(lv.n_words());
      for (uint64_t w = 0; w < lv.n_words(); ++w)
        gw[t][w] = vb.intern(lv.arena.data() + lv.off[w], lv.off[w + 1] - lv.off[w]);
    }
    std::vector<uint64_t> base(nparts + 1, 1);
    for (uint32_t t = 0; t < nparts; ++t) base[t + 1] = base[t] + parts[t].depth.size() - 1;
    depth.assign(total_nodes, 0);
    n_edges.assign(total_nodes, 0);
    hash_fid.assign(total_nodes, FID_NONE);
    term_fid.assign(total_nodes, FID_NONE);
    hash_id.assign(total_nodes, WID_NONE);
    term_id.assign(total_nodes, WID_NONE);
    parent_of.assign(total_nodes, 0);
    wid_of.assign(total_nodes, WID_NONE);
    has_plus.assign(total_nodes, 0);
    term_wild.assign(total_nodes, 0);
    // the root's fields, then every partition's nodes into its own range (in parallel)
    for (const Part& P : parts) {
      n_edges[0] += P.n_edges[0];
      has_plus[0] |= P.has_plus[0];
      if (P.hash_fid[0] != FID_NONE) {
        hash_fid[0] = P.hash_fid[0];
        hash_id[0] = P.hash_id[0];
      }
      max_depth = std::max(max_depth, P.max_depth);
    }
    std::vector<std::thread> th;
    auto copy_part = [&](uint32_t t) {
      Part& P = parts[t];
      const uint64_t b = base[t];
      for (uint64_t l = 1; l < P.depth.size(); ++l) {
        const uint64_t g = b + l - 1;
        depth[g] = P.depth[l];
        n_edges[g] = P.n_edges[l];
        hash_fid[g] = P.hash_fid[l];
        term_fid[g] = P.term_fid[l];
        hash_id[g] = P.hash_id[l];
        term_id[g] = P.term_id[l];
        has_plus[g] = P.has_plus[l];
        term_wild[g] = P.term_wild[l];
        const uint32_t pp = P.parent_of[l];
        parent_of[g] = pp ? static_cast<uint32_t>(b + pp - 1) : 0u;
        const uint32_t w = P.wid_of[l];
        wid_of[g] = w < WID_HASH ? gw[t][w] : w;
      }
      P = Part();  // free the partition
    };
    for (uint32_t t = 1; t < nparts; ++t) th.emplace_back(copy_part, t);
    copy_part(0);
    for (auto& x : th) x.join();
  }

  // ---- pass 2: per-node child lists -----------------------------------------------
  // (children in creation order: one linear pass over the nodes' in-edges, not two scans of
  // the edge hash map)
  const uint64_t n_nodes = depth.size();
  std::vector<uint64_t> coff(n_nodes + 1, 0);
  for (uint64_t v = 0; v < n_nodes; ++v) coff[v + 1] = coff[v] + n_edges[v];
  std::vector<uint32_t> cwid(coff[n_nodes]), cid(coff[n_nodes]);
  {
    std::vector<uint64_t> fillp(coff.begin(), coff.end() - 1);
    for (uint64_t c = 1; c < n_nodes; ++c) {
      const uint32_t p = parent_of[c];
      cwid[fillp[p]] = wid_of[c];
      cid[fillp[p]] = static_cast<uint32_t>(c);
      fillp[p] += 1;
    }
  }
  // EMQX_CHILD_ORDER=hash|size (A/B runs only): each node's children in the pseudo-random
  // order of a hash of (node, word) — the order round 1's edge-map scan produced — or by
  // subtree size, largest first, instead of creation order; the child order decides the
  // line-packed layout below
  static const int child_order = [] {
    const char* v = getenv("EMQX_CHILD_ORDER");
    return !v ? 0 : std::strcmp(v, "hash") == 0 ? 1 : std::strcmp(v, "size") == 0 ? 2 : 0;
  }();
  if (child_order == 2) {
    std::vector<uint32_t> sub(n_nodes, 1);  // subtree node counts (a child's id exceeds its parent's)
    for (uint64_t c = n_nodes; c-- > 1;) sub[parent_of[c]] += sub[c];
    parallel_chunks(n_nodes, nthreads, 1 << 14, [&](uint64_t v0, uint64_t v1, int) {
      std::vector<std::pair<uint64_t, uint32_t>> tmp;
      for (uint64_t v = v0; v < v1; ++v) {
        const uint64_t a = coff[v], b = coff[v + 1];
        if (b - a < 2) continue;
        tmp.clear();
        for (uint64_t j = a; j < b; ++j) tmp.emplace_back(~uint64_t(sub[cid[j]]) << 32 | (j - a), static_cast<uint32_t>(j - a));
        std::sort(tmp.begin(), tmp.end());
        std::vector<uint32_t> w2(b - a), c2(b - a);
        for (uint64_t k = 0; k < tmp.size(); ++k) {
          w2[k] = cwid[a + tmp[k].second];
          c2[k] = cid[a + tmp[k].second];
        }
        std::copy(w2.begin(), w2.end(), cwid.begin() + static_cast<std::ptrdiff_t>(a));
        std::copy(c2.begin(), c2.end(), cid.begin() + static_cast<std::ptrdiff_t>(a));
      }
    });
  }
  std::vector<uint32_t>().swap(parent_of);
  std::vector<uint32_t>().swap(wid_of);
  if (child_order == 1) {
    parallel_chunks(n_nodes, nthreads, 1 << 14, [&](uint64_t v0, uint64_t v1, int) {
      std::vector<std::pair<uint64_t, uint32_t>> tmp;
      for (uint64_t v = v0; v < v1; ++v) {
        const uint64_t a = coff[v], b = coff[v + 1];
        if (b - a < 2) continue;
        tmp.clear();
        for (uint64_t j = a; j < b; ++j) tmp.emplace_back(mix64((v << 32) | cwid[j]), static_cast<uint32_t>(j - a));
        std::sort(tmp.begin(), tmp.end());
        std::vector<uint32_t> w2(b - a), c2(b - a);
        for (uint64_t k = 0; k < tmp.size(); ++k) {
          w2[k] = cwid[a + tmp[k].second];
          c2[k] = cid[a + tmp[k].second];
        }
        std::copy(w2.begin(), w2.end(), cwid.begin() + static_cast<std::ptrdiff_t>(a));
        std::copy(c2.begin(), c2.end(), cid.begin() + static_cast<std::ptrdiff_t>(a));
      }
    });
  }

  // A node with a '+' edge keeps it in slot 0, and a copy at the head of every other 64-B line
  // of its array, so that the '+' probe and the literal probe of a step read one line (one L2
  // request: tools/gather_bench pair).  (Round 1 measured copies per 128-B line
  // as 6% slower: then the kernel waited for the '+' load before issuing the literal one.)
  // A copy of the '+' edge at the head of every 64-B line of the array (layout.h plus_copy);
  // EMQX_PLUS_LINES=0 (A/B runs only): slot 0 alone
  static const bool plus_lines = [] {
    const char* x = getenv("EMQX_PLUS_LINES");
    return !(x && std::strcmp(x, "0") == 0);
  }();
  const uint32_t plus_mask = plus_lines ? ~(PLUS_LINE - 1u) : 0u;
  out.plus_mask = plus_mask;
  auto plus_slot = [&](uint64_t v, uint64_t cap, uint32_t i) -> bool {
    return has_plus[v] && plus_position(i, plus_copies(plus_mask, true, log2u(cap)));
  };

  // Bucketed placement of node v's literal edges (2-slot buckets, two candidate buckets,
  // random-walk eviction) for one seed; false when some word cannot be placed.  The '+'
  // slots stay free.  Afterwards every word outside its primary bucket flags that bucket.
  auto bucket_place = [&](uint64_t v, uint32_t sd, uint32_t cap, std::vector<uint32_t>& key_out,
                          std::vector<uint32_t>& child_out) -> bool {
    const uint32_t mk = cap - 1;
    const bool cp = plus_copies(plus_mask, has_plus[v], log2u(cap));
    key_out.assign(cap, WID_NONE);
    child_out.assign(cap, 0);
    for (uint32_t i = 0; i < cap; ++i)
      if (plus_slot(v, cap, i)) key_out[i] = WID_PLUS;
    uint32_t rng = 0x9E3779B9u ^ static_cast<uint32_t>(v) ^ (sd << 20);
    for (uint64_t j = coff[v]; j < coff[v + 1]; ++j) {
      if (cwid[j] == WID_PLUS) continue;
      uint32_t key = cwid[j], ch = cid[j];
      for (int kick = 0;; ++kick) {
        const uint32_t b1 = wide_slot(key, sd, mk, cp, false), b2 = wide_slot(key, sd, mk, cp, true);
        const uint32_t cand[4] = {b1, b1 + 1, b2, b2 + 1};
        bool placed = false;
        for (uint32_t c : cand)
          if (key_out[c] == WID_NONE) {
            key_out[c] = key;
            child_out[c] = ch;
            placed = true;
            break;
          }
        if (placed) break;
        if (kick > 500) return false;
        rng = rng * 1664525u + 1013904223u;
        const uint32_t victim = cand[(rng >> 16) & 3u];
        if (key_out[victim] == WID_PLUS) continue;
        std::swap(key, key_out[victim]);
        std::swap(ch, child_out[victim]);
      }
    }
    return true;
  };

  // ---- pass 3: hashing per node — perfect hash (seed search) or 2-slot buckets ---------
  std::vector<uint32_t> caplog(n_nodes, 0), seed(n_nodes, 0);
  std::vector<uint8_t> ph(n_nodes, 0);
  std::atomic<bool> failed{false};
  std::string fail_msg;
  std::mutex fail_mu;
  parallel_chunks(n_nodes, nthreads, 1 << 14, [&](uint64_t v0, uint64_t v1, int) {
  std::vector<uint32_t> slots_tmp, ck_key, ck_child;
  for (uint64_t v = v0; v < v1; ++v) {
    const uint32_t e = n_edges[v];
    if (!e) continue;
    const uint32_t n_lit = e - (has_plus[v] ? 1u : 0u);
    bool done = false;
    if (n_lit <= 32) {
      // smallest cap first: small nodes (plus + a literal or two) stay inside one 64-B line
      const uint64_t cap0 = next_pow2(std::max<uint64_t>(2, e));
      const uint64_t cap_max = next_pow2(std::max<uint64_t>(16, 8ull * e));
      for (uint64_t cap = cap0; cap <= cap_max && !done && log2u(cap) <= PH_MAX_CAPLOG; cap <<= 1) {
        const uint32_t mask = static_cast<uint32_t>(cap - 1);
        for (uint32_t sd = 0; sd < 256 && !done; ++sd) {
          slots_tmp.clear();
          bool ok = true;
          for (uint64_t j = coff[v]; j < coff[v + 1] && ok; ++j) {
            if (cwid[j] == WID_PLUS) continue;
            const uint32_t sl = lit_slot(cwid[j], sd, mask, plus_copies(plus_mask, has_plus[v], log2u(cap)));
            ok &= !plus_slot(v, cap, sl);
            for (uint32_t x : slots_tmp) ok &= (x != sl);
            slots_tmp.push_back(sl);
          }
          if (ok) {
            caplog[v] = log2u(cap);
            seed[v] = sd;
            ph[v] = 1;
            done = true;
          }
        }
      }
    }
    if (!done) {
      // 2-slot buckets at load <= 1/4 (EMQX_WIDE_SLACK=k, A/B runs only: load <= 1/k)
      static const uint64_t slack = [] {
        const char* x = getenv("EMQX_WIDE_SLACK");
        const long k = x ? std::atol(x) : 0;
        return static_cast<uint64_t>(k >= 2 && k <= 16 ? k : 4);
      }();
      // (an array holding '+' copies loses a quarter of its slots to them, and one candidate
      // slot of every other bucket: twice the room keeps later inserts in place)
      caplog[v] = log2u(next_pow2(slack * e + slack));
      bool ok = false;
      for (uint32_t sd = 0; sd < CUCKOO_SEEDS && !ok; ++sd) {
        ok = bucket_place(v, sd, 1u << caplog[v], ck_key, ck_child);
        if (ok) seed[v] = sd;
      }
      if (!ok) {
        std::lock_guard<std::mutex> g(fail_mu);
        fail_msg = "bucket placement failed for a node with " + std::to_string(e) + " edges";
        failed = true;
        return;
      }
    }
  }
  });
  if (failed) {
    if (err) *err = fail_msg;
    return false;
  }

  // ---- pass 4: layout — line-packed preorder ----------------------------------------
  // An L2 miss fetches a 128-B line (8 slots) while a probe uses one, so the layout packs
  // walks into lines: when a node is visited, the arrays of all its children are placed
  // right behind it, first-fit into the currently open line (an array of c <= 8 slots is
  // aligned to c, so it never straddles a line; larger arrays start on a line);
  // then the children are visited in order.  A chain of small nodes — the deep tail of
  // most filters — shares one line across several levels, so its walk misses once.
  std::vector<uint32_t> base(n_nodes, 0);
  uint64_t total_slots = 0;
  {
    constexpr uint64_t LINE = 128 / sizeof(EdgeSlot);
    constexpr uint32_t FULL = (1u << LINE) - 1u;
    uint64_t line = 0;       // open line (slot index, multiple of LINE)
    uint32_t used = FULL;    // its occupied slots (bit mask); FULL = no open line
    auto place = [&](uint32_t caplg) -> uint64_t {
      const uint64_t c = 1ull << caplg;
      if (c >= LINE) {
        const uint64_t at = (total_slots + LINE - 1) & ~(LINE - 1);
        total_slots = at + c;
        used = FULL;
        return at;
      }
      const uint32_t want = (1u << c) - 1u;
      for (uint32_t o = 0; o < LINE; o += static_cast<uint32_t>(c))
        if (!(used & (want << o))) {
          used |= want << o;
          return line + o;
        }
      line = (total_slots + LINE - 1) & ~(LINE - 1);
      total_slots = line + LINE;
      used = want;
      return line;
    };
    // EMQX_LAYOUT=bfs (A/B runs only): breadth-first by depth, larger arrays first
    static const bool bfs = [] {
      const char* v = getenv("EMQX_LAYOUT");
      return v && std::strcmp(v, "bfs") == 0;
    }();
    if (bfs) {
      std::vector<uint32_t> order(n_nodes);
      for (uint64_t v = 0; v < n_nodes; ++v) order[v] = static_cast<uint32_t>(v);
      std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        return depth[a] != depth[b] ? depth[a] < depth[b] : caplog[a] > caplog[b];
      });
      for (uint32_t v : order)
        if (n_edges[v]) base[v] = static_cast<uint32_t>(place(caplog[v]));
      if (total_slots + opts.slot_offset > MAX_SLOTS) {
        if (err) *err = "edge slot array exceeds 2^31 slots";
        return false;
      }
    }
    std::vector<uint32_t> stack;
    if (n_edges[0] && !bfs) {
      base[0] = static_cast<uint32_t>(place(caplog[0]));
      stack.push_back(0);
    }
    while (!stack.empty()) {
      const uint32_t v = stack.back();
      stack.pop_back();
      for (uint64_t j = coff[v]; j < coff[v + 1]; ++j)
        if (n_edges[cid[j]]) base[cid[j]] = static_cast<uint32_t>(place(caplog[cid[j]]));
      if (total_slots + opts.slot_offset > MAX_SLOTS) {
        if (err) *err = "edge slot array exceeds 2^31 slots";
        return false;
      }
      for (uint64_t j = coff[v + 1]; j-- > coff[v];)
        if (n_edges[cid[j]]) stack.push_back(cid[j]);
    }
  }
  // literal-edge filter of each node (stored in the slot that leads to it)
  std::vector<uint32_t> lf(n_nodes, 0), lf_flag(n_nodes, 0);
  parallel_chunks(n_nodes, nthreads, 1 << 16, [&](uint64_t v0, uint64_t v1, int) {
  for (uint64_t v = v0; v < v1; ++v) {
    uint32_t n_lit = 0, only = WID_NONE, bloom = 0;
    for (uint64_t j = coff[v]; j < coff[v + 1]; ++j) {
      if (cwid[j] == WID_PLUS) continue;
      ++n_lit;
      only = cwid[j];
      const uint32_t h = litf_hash(cwid[j]);
      bloom |= (1u << (h & 31u)) | (1u << ((h >> 5) & 31u));
    }
    if (n_lit == 0) {
      lf_flag[v] = META_LITF_NONE;
    } else if (n_lit == 1) {
      lf_flag[v] = META_LITF_EXACT;
      lf[v] = only;
    } else {
      lf[v] = n_lit <= LITF_BLOOM_MAX ? bloom : ~0u;
    }
  }
  });
  // A child with edges and exactly one filter id carries it in litf (META_XFID), so its
  // emission needs no fids[] reference; its literal filter moves to 8 bits of the meta: the
  // fingerprint of its only literal word, or an 8-bit Bloom mask.  (EMQX_XFID=0, A/B runs:
  // only children without literal edges, which lose no filter.)
  {
    static const bool xfid_off = [] {
      const char* v = getenv("EMQX_XFID");
      return v && std::strcmp(v, "0") == 0;
    }();
    parallel_chunks(n_nodes, nthreads, 1 << 16, [&](uint64_t v0, uint64_t v1, int) {
    for (uint64_t v = std::max<uint64_t>(v0, 1); v < v1; ++v) {
      if (!n_edges[v]) continue;
      const bool h = hash_fid[v] != FID_NONE, t = term_fid[v] != FID_NONE;
      if (h == t) continue;
      const bool none = (lf_flag[v] & META_LITF_NONE) != 0, exact = (lf_flag[v] & META_LITF_EXACT) != 0;
      if (!none && xfid_off) continue;
      uint32_t f8 = 0;
      if (exact) {
        f8 = litf_hash(lf[v]) >> 24;
      } else if (!none) {
        uint32_t n_lit = 0;
        for (uint64_t j = coff[v]; j < coff[v + 1]; ++j) {
          if (cwid[j] == WID_PLUS) continue;
          ++n_lit;
          f8 |= 1u << (litf_hash(cwid[j]) & 7u);
        }
        if (n_lit > LITF_BLOOM_MAX) f8 = 0xFFu;
      }
      lf_flag[v] |= META_XFID | (t ? META_XFID_TERM : 0u) | (f8 << META_F8_SHIFT);
      lf[v] = t ? term_fid[v] : hash_fid[v];
    }
    });
  }
  auto meta_of = [&](uint32_t v) -> uint32_t {
    uint32_t m = caplog[v] & META_CAPLOG2_MASK;
    if (n_edges[v]) m |= META_HAS_EDGES;
    if (has_plus[v]) m |= META_HAS_PLUS;
    if (hash_fid[v] != FID_NONE) m |= META_HAS_HASH;
    if (term_fid[v] != FID_NONE) m |= META_HAS_TERM;
    if (term_wild[v]) m |= META_TERM_WILD;
    m |= (ph[v] ? META_PH : 0u) | (seed[v] << META_SEED_SHIFT);
    m |= lf_flag[v];
    return m;
  };

  const uint64_t n_slots = std::max<uint64_t>(total_slots, 1);
  out.edges.assign(n_slots, EdgeSlot{WID_NONE, 0, 0, 0});
  out.fids.assign(2 * n_slots, FID_NONE);
  const uint32_t off0 = static_cast<uint32_t>(opts.slot_offset);
  if (opts.fid_loc) opts.fid_loc->assign(n_ids, FIDLOC_NONE);
  if (opts.slot_ids) opts.slot_ids->assign(2 * n_slots, WID_NONE);
  auto write_slot = [&](uint64_t at, uint32_t wid, uint32_t child) {
    EdgeSlot& r = out.edges[at];
    r.wid = wid;
    const bool leaf = n_edges[child] == 0;
    r.child_base = leaf ? hash_fid[child] : off0 + base[child];
    if (opts.fid_loc) {
      const uint64_t abs = opts.slot_offset + at;
      if (hash_id[child] != WID_NONE) (*opts.fid_loc)[hash_id[child]] = abs << 2 | FIDLOC_HASH;
      if (term_id[child] != WID_NONE) (*opts.fid_loc)[term_id[child]] = abs << 2 | FIDLOC_TERM;
    }
    r.meta = meta_of(child) | (r.meta & META_BUCKET_OVF);
    r.litf = leaf ? term_fid[child] : lf[child];
    out.fids[2 * at] = hash_fid[child];
    out.fids[2 * at + 1] = term_fid[child];
    if (opts.slot_ids) {
      (*opts.slot_ids)[2 * at] = hash_id[child];
      (*opts.slot_ids)[2 * at + 1] = term_id[child];
    }
  };
  // every node writes only its own array's slots and its children's ids: nodes in parallel
  parallel_chunks(n_nodes, nthreads, 1 << 14, [&](uint64_t v0, uint64_t v1, int) {
  std::vector<uint32_t> ck_key, ck_child;
  for (uint64_t v = v0; v < v1; ++v) {
    if (!n_edges[v]) continue;
    // '+' is pinned at slot 0, its copies at the other line heads (slot 0 written last: the
    // filter-id locations, fid_loc, name slot 0)
    for (uint64_t j = coff[v]; j < coff[v + 1]; ++j)
      if (cwid[j] == WID_PLUS)
        for (uint32_t i = (1u << caplog[v]); i-- > 0;)
          if (plus_slot(v, 1ull << caplog[v], i)) write_slot(base[v] + i, WID_PLUS, cid[j]);
    if (ph[v]) {
      const uint32_t mask = (1u << caplog[v]) - 1;
      for (uint64_t j = coff[v]; j < coff[v + 1]; ++j)
        if (cwid[j] != WID_PLUS)
          write_slot(base[v] + lit_slot(cwid[j], seed[v], mask, plus_copies(plus_mask, has_plus[v], caplog[v])), cwid[j],
                     cid[j]);
      continue;
    }
    // wide node: re-run the placement found in pass 3 (deterministic for its seed), then
    // flag every primary bucket that overflowed
    const uint32_t cap = 1u << caplog[v];
    const bool cp = plus_copies(plus_mask, has_plus[v], caplog[v]);
    bucket_place(v, seed[v], cap, ck_key, ck_child);
    for (uint32_t i = 0; i < cap; ++i)
      if (ck_key[i] != WID_NONE && ck_key[i] != WID_PLUS) write_slot(base[v] + i, ck_key[i], ck_child[i]);
    for (uint32_t i = 0; i < cap; ++i) {
      const uint32_t key = ck_key[i];
      if (key == WID_NONE || key == WID_PLUS) continue;
      const uint32_t b1 = wide_slot(key, seed[v], cap - 1, cp, false);
      if (i != b1 && i != b1 + 1) out.edges[base[v] + b1].meta |= META_BUCKET_OVF;
    }
  }
  });
  out.root_hash_fid = hash_fid[0];
  if (opts.fid_loc && hash_id[0] != WID_NONE) (*opts.fid_loc)[hash_id[0]] = FIDLOC_ROOT_HASH;
  out.root_base = off0 + base[0];
  out.slot_offset = opts.slot_offset;
  out.root_meta = meta_of(0);
  out.n_nodes = n_nodes;
  out.max_depth = max_depth;
  for (uint64_t v = 0; v < n_nodes; ++v) out.n_ph_nodes += ph[v];

  // ---- vocab device table ----------------------------------------------------------
  out.n_words = vb.n_words();
  if (opts.vocab_table) {
    vb.build_table();
    out.vocab = vb.table;
    out.vocab_mask = vb.mask;
    out.arena = vb.arena;
    if (out.arena.empty()) out.arena.push_back(0);
  }
  return true;
}

// Host self-check of a built table: every stored edge must be found by the device lookup
// rule (slot 0 for '+', perfect hash, or primary / flagged secondary bucket), every non-edge word
// must miss, and every literal filter must admit every word it summarises.
bool check_tables(const HostTables& t, std::string* err) {
  const uint64_t n = t.edges.size();
  std::vector<std::pair<uint32_t, uint32_t>> arrays;  // (base, meta) of every node with edges
  arrays.push_back({t.root_base, t.root_meta});
  for (uint64_t i = 0; i < n; ++i) {
    const EdgeSlot& s = t.edges[i];
    if (s.wid != WID_NONE && (s.meta & META_HAS_EDGES)) arrays.push_back({s.child_base, s.meta});
  }
  for (auto& [base, meta] : arrays) {
    if (!(meta & META_HAS_EDGES)) continue;
    const uint32_t caplog = meta & META_CAPLOG2_MASK;
    const uint32_t mask = (1u << caplog) - 1u;
    const bool ph = (meta & META_PH) != 0;
    uint32_t n_lit = 0;
    for (uint32_t i = 0; i <= mask; ++i) {
      const EdgeSlot& s = t.edges[base - t.slot_offset + i];
      if (s.wid == WID_NONE) continue;
      if (s.wid == WID_PLUS) {
        if (!plus_position(i, plus_copies(t.plus_mask, true, caplog)) || !(meta & META_HAS_PLUS)) {
          if (err) *err = "'+' edge outside its slots";
          return false;
        }
        continue;
      }
      ++n_lit;
      bool found;
      if (ph)
        found = lit_slot(s.wid, (meta >> META_SEED_SHIFT) & 255u, mask,
                         plus_copies(t.plus_mask, meta & META_HAS_PLUS, caplog)) == i;
      else {
        const uint32_t sd = (meta >> META_SEED_SHIFT) & 255u;
        const bool cp = plus_copies(t.plus_mask, meta & META_HAS_PLUS, caplog);
        const uint32_t b1 = wide_slot(s.wid, sd, mask, cp, false), b2 = wide_slot(s.wid, sd, mask, cp, true);
        found = i == b1 || i == b1 + 1 ||
                ((i == b2 || i == b2 + 1) && (t.edges[base - t.slot_offset + b1].meta & META_BUCKET_OVF));
      }
      if (!found) {
        if (err) *err = "edge not at its lookup slot";
        return false;
      }
    }
    if ((meta & META_HAS_PLUS) && t.edges[base - t.slot_offset].wid != WID_PLUS) {
      if (err) *err = "missing '+' edge";
      return false;
    }
    (void)n_lit;
  }
  // filter ids: a slot's pair agrees with its child's meta
  for (uint64_t i = 0; i < n; ++i) {
    const EdgeSlot& s = t.edges[i];
    if (s.wid == WID_NONE) continue;
    if ((t.fids[2 * i] != FID_NONE) != ((s.meta & META_HAS_HASH) != 0) ||
        (t.fids[2 * i + 1] != FID_NONE) != ((s.meta & META_HAS_TERM) != 0) ||
        (!(s.meta & META_HAS_EDGES) && (s.child_base != t.fids[2 * i] || s.litf != t.fids[2 * i + 1])) ||
        ((s.meta & META_HAS_EDGES) && (s.meta & META_XFID) &&
         s.litf != t.fids[2 * i + ((s.meta & META_XFID_TERM) ? 1 : 0)])) {
      if (err) *err = "filter ids disagree with the child's meta";
      return false;
    }
  }
  // literal filters: every literal child word of a node must pass the node's filter
  for (uint64_t i = 0; i < n; ++i) {
    const EdgeSlot& s = t.edges[i];
    if (s.wid == WID_NONE || !(s.meta & META_HAS_EDGES)) continue;
    const uint32_t mask = (1u << (s.meta & META_CAPLOG2_MASK)) - 1u;
    for (uint32_t j = 0; j <= mask; ++j) {
      const EdgeSlot& c = t.edges[s.child_base - t.slot_offset + j];
      if (c.wid == WID_NONE || c.wid == WID_PLUS) continue;
      if (!litf_may_contain(s.meta, s.litf, c.wid)) {
        if (err) *err = "literal filter rejects a present word";
        return false;
      }
    }
  }
  return true;
}

}  // namespace emqx
