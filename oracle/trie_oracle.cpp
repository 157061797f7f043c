// CPU restatement of EMQX's route lookup — TEST INFRASTRUCTURE ONLY (parity oracle and
// the CPU baseline timed by bench.py's cpu_baseline leg).  Never linked into the
// product library (emqx_amd/csrc); only tests/, __graft_entry__.smoke() and bench.py
// load it, through ctypes, as the checker / baseline.
//
// Restates (paths relative to /root/reference):
//   apps/emqx/src/emqx_topic.erl:153-164   tokens/words          -> split_words()
//   apps/emqx/src/emqx_topic.erl:53-62     wildcard/1            -> is_wild()
//   apps/emqx/src/emqx_topic.erl:184-195   join/1                -> join_words()
//   apps/emqx/src/emqx_trie.erl:192-233    make_keys/do_compact/make_prefixes -> make_keys()
//   apps/emqx/src/emqx_trie.erl:115-137    insert/delete (refcounted keys)     -> Trie::insert/erase
//   apps/emqx/src/emqx_trie.erl:256-270    lookup_topic/has_prefix             -> Trie::lookup/has_prefix
//   apps/emqx/src/emqx_trie.erl:272-334    do_match ($ rule), match_compact, match_no_compact
//   apps/emqx/src/emqx_router.erl:117-140  wildcard-only trie + match_routes = exact ∪ trie
//
// The ETS ordered_set {Key, Count} (emqx_trie.erl:56-77) is restated as a sorted array
// of {binary, 0|1} keys searched by binary search: the same O(log N) ordered-key probe
// per lookup, and like the reference every visited prefix is materialised by a fresh
// binary join (emqx_trie.erl:218-222).  Results are pinned against oracle/emqx_ref.py
// (itself pinned to the reference's KATs) in tests/test_oracle_cpp.py.
//
// Build: see oracle/Makefile  ->  oracle/_build/liboracle.so (gitignored).

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <vector>

namespace {

enum WordKind : uint8_t { W_BIN = 0, W_EMPTY = 1, W_PLUS = 2, W_HASH = 3 };

struct Word {
  std::string bin;
  uint8_t kind;
};

std::vector<Word> split_words(const char* p, size_t n) {
  std::vector<Word> out;
  size_t s = 0;
  for (size_t i = 0; i <= n; ++i) {
    if (i == n || p[i] == '/') {
      Word w;
      w.bin.assign(p + s, i - s);
      if (w.bin.empty()) w.kind = W_EMPTY;
      else if (w.bin == "+") w.kind = W_PLUS;
      else if (w.bin == "#") w.kind = W_HASH;
      else w.kind = W_BIN;
      out.push_back(std::move(w));
      s = i + 1;
    }
  }
  return out;
}

bool is_wild(const std::vector<Word>& ws) {
  for (auto& w : ws)
    if (w.kind == W_PLUS || w.kind == W_HASH) return true;
  return false;
}

// emqx_topic:join/1 — bin() of atoms is their text, so a plain '/'-join of the bins.
std::string join_strs(const std::vector<std::string>& parts) {
  std::string r;
  for (size_t i = 0; i < parts.size(); ++i) {
    if (i) r.push_back('/');
    r += parts[i];
  }
  return r;
}

// Prefix value: either the virtual root `empty` or a binary.
struct Prefix {
  bool root;
  std::string bin;
};

// emqx_trie.erl:218-222
Prefix trie_join(const Prefix& p, const std::string& w) {
  if (p.root) return Prefix{false, w};
  std::string r;
  r.reserve(p.bin.size() + 1 + w.size());
  r += p.bin;
  r.push_back('/');
  r += w;
  return Prefix{false, std::move(r)};
}

// emqx_trie.erl:208-216
std::vector<std::string> do_compact(const std::vector<Word>& ws) {
  std::vector<std::string> acc;
  Prefix seg{true, ""};
  for (auto& w : ws) {
    if (w.kind == W_PLUS || w.kind == W_HASH) {
      acc.push_back(trie_join(seg, w.bin).bin);
      seg = Prefix{true, ""};
    } else {
      seg = trie_join(seg, w.bin);
    }
  }
  if (!seg.root) acc.push_back(seg.bin);
  return acc;
}

struct Key {
  std::string bin;
  uint8_t tag;  // 0 = PREFIX, 1 = TOPIC (emqx_trie.erl:53-54)
  bool operator<(const Key& o) const {
    int c = bin.compare(o.bin);
    if (c != 0) return c < 0;
    return tag < o.tag;
  }
  bool operator==(const Key& o) const { return tag == o.tag && bin == o.bin; }
};

struct KeyHash {
  size_t operator()(const Key& k) const { return std::hash<std::string>()(k.bin) * 31 + k.tag; }
};

// emqx_trie.erl:192-194, 224-233
void make_keys(const std::string& topic, bool compact, std::vector<Key>& out) {
  out.clear();
  out.push_back(Key{topic, 1});
  auto ws = split_words(topic.data(), topic.size());
  std::vector<std::string> segs;
  if (compact) {
    segs = do_compact(ws);
  } else {
    for (auto& w : ws) segs.push_back(w.bin);
  }
  std::vector<std::string> prefix;
  std::vector<std::string> acc;
  for (size_t i = 0; i + 1 < segs.size(); ++i) {
    prefix.push_back(segs[i]);
    acc.push_back(join_strs(prefix));
  }
  std::reverse(acc.begin(), acc.end());
  for (auto& a : acc) out.push_back(Key{a, 0});
}

struct Trie {
  bool compact = true;
  // Mutable refcounted table while building; frozen into a sorted array for lookups.
  std::unordered_map<Key, int64_t, KeyHash> tab;
  std::vector<Key> sorted;
  bool frozen = false;

  void insert(const std::string& topic) {  // emqx_trie.erl:115-120
    std::vector<Key> ks;
    make_keys(topic, compact, ks);
    if (tab.count(ks[0])) return;
    for (auto& k : ks) tab[k] += 1;
    frozen = false;
  }
  void erase(const std::string& topic) {  // emqx_trie.erl:132-137, 244-252
    std::vector<Key> ks;
    make_keys(topic, compact, ks);
    if (!tab.count(ks[0])) return;
    for (auto& k : ks) {
      auto it = tab.find(k);
      if (it == tab.end()) continue;
      if (it->second > 1) it->second -= 1;
      else tab.erase(it);
    }
    frozen = false;
  }
  void freeze() {
    if (frozen) return;
    sorted.clear();
    sorted.reserve(tab.size());
    for (auto& kv : tab)
      if (kv.second > 0) sorted.push_back(kv.first);
    std::sort(sorted.begin(), sorted.end());
    frozen = true;
  }
  bool empty() const { return tab.empty(); }  // emqx_trie.erl:171

  bool has_key(const std::string& bin, uint8_t tag, uint64_t& lookups) const {
    ++lookups;
    Key k{bin, tag};
    auto it = std::lower_bound(sorted.begin(), sorted.end(), k);
    return it != sorted.end() && *it == k;
  }
  // emqx_trie.erl:259-263 (lookup_topic/2)
  void lookup_topic(const std::string& t, std::vector<std::string>& acc, uint64_t& lk) const {
    if (has_key(t, 1, lk)) acc.push_back(t);
  }
  // emqx_trie.erl:265-270
  bool has_prefix(const Prefix& p, uint64_t& lk) const {
    if (p.root) return true;
    return has_key(p.bin, 0, lk);
  }
  // 'match_#' emqx_trie.erl:332-334
  void match_hash(const Prefix& p, std::vector<std::string>& acc, uint64_t& lk) const {
    lookup_topic(trie_join(p, "#").bin, acc, lk);
  }
  // emqx_trie.erl:315-330
  void match_compact(const std::vector<Word>& ws, size_t i, const Prefix& p, bool wild,
                     std::vector<std::string>& acc, uint64_t& lk) const {
    if (i == ws.size()) {
      match_hash(p, acc, lk);
      if (wild && !p.root) lookup_topic(p.bin, acc, lk);
      return;
    }
    match_hash(p, acc, lk);
    match_compact(ws, i + 1, trie_join(p, ws[i].bin), wild, acc, lk);
    Prefix wp = trie_join(p, "+");
    if (i + 1 == ws.size() || has_prefix(wp, lk)) match_compact(ws, i + 1, wp, true, acc, lk);
  }
  // emqx_trie.erl:289-313
  void match_no_compact(const std::vector<Word>& ws, size_t i, const Prefix& p, bool wild,
                        std::vector<std::string>& acc, uint64_t& lk) const {
    if (i == ws.size()) {
      match_hash(p, acc, lk);
      if (wild && !p.root) lookup_topic(p.bin, acc, lk);
      return;
    }
    if (!has_prefix(p, lk)) return;
    match_hash(p, acc, lk);
    match_no_compact(ws, i + 1, trie_join(p, "+"), true, acc, lk);
    match_no_compact(ws, i + 1, trie_join(p, ws[i].bin), wild, acc, lk);
  }
  // emqx_trie.erl:148-162, 272-287
  void match(const char* t, size_t n, std::vector<std::string>& acc, uint64_t& lk) const {
    auto ws = split_words(t, n);
    if (is_wild(ws)) return;
    Prefix start{true, ""};
    size_t i0 = 0;
    if (ws[0].kind == W_BIN && ws[0].bin[0] == '$') {
      if (ws.size() == 1) lookup_topic(ws[0].bin, acc, lk);
      start = Prefix{false, ws[0].bin};
      i0 = 1;
    }
    if (compact) match_compact(ws, i0, start, false, acc, lk);
    else match_no_compact(ws, i0, start, false, acc, lk);
  }
};

struct Oracle {
  Trie trie;
  bool trie_all;  // true: every filter enters the trie (emqx_trie_SUITE style)
  std::unordered_map<std::string, uint32_t> ids;  // route table: filter -> id
  std::vector<uint8_t> live;
};

// Uncompacted level trie for the evals cost model (SURVEY §8 d).
struct LevelTrie {
  std::unordered_map<std::string, uint64_t> node_of;  // "parent_id\x01word" -> id
  uint64_t next = 1;
  static std::string key(uint64_t parent, const Word& w) {
    std::string k = std::to_string(parent);
    k.push_back('\x01');
    k.push_back(char('0' + w.kind));
    k += w.bin;
    return k;
  }
};

}  // namespace

extern "C" {

void* orc_create(int compact, int trie_all) {
  auto* o = new Oracle();
  o->trie.compact = compact != 0;
  o->trie_all = trie_all != 0;
  return o;
}

void orc_destroy(void* h) { delete static_cast<Oracle*>(h); }

// Adds filters with ids = insertion order (deduplicated: an existing filter keeps its id).
// ids_out[i] receives the id of filter i.  emqx_router.erl:110-124.
void orc_add(void* h, const uint8_t* bytes, const uint64_t* offs, uint64_t n, uint32_t* ids_out) {
  auto* o = static_cast<Oracle*>(h);
  for (uint64_t i = 0; i < n; ++i) {
    std::string f(reinterpret_cast<const char*>(bytes + offs[i]), offs[i + 1] - offs[i]);
    auto it = o->ids.find(f);
    if (it != o->ids.end()) {
      if (!o->live[it->second]) {
        o->live[it->second] = 1;
        auto ws = split_words(f.data(), f.size());
        if (o->trie_all || is_wild(ws)) o->trie.insert(f);
      }
      if (ids_out) ids_out[i] = it->second;
      continue;
    }
    uint32_t id = static_cast<uint32_t>(o->live.size());
    o->ids.emplace(f, id);
    o->live.push_back(1);
    auto ws = split_words(f.data(), f.size());
    if (o->trie_all || is_wild(ws)) o->trie.insert(f);
    if (ids_out) ids_out[i] = id;
  }
}

// emqx_router.erl:162-171 (delete of the last route removes the trie entry).
void orc_delete(void* h, const uint8_t* bytes, const uint64_t* offs, uint64_t n) {
  auto* o = static_cast<Oracle*>(h);
  for (uint64_t i = 0; i < n; ++i) {
    std::string f(reinterpret_cast<const char*>(bytes + offs[i]), offs[i + 1] - offs[i]);
    auto it = o->ids.find(f);
    if (it == o->ids.end() || !o->live[it->second]) continue;
    o->live[it->second] = 0;
    auto ws = split_words(f.data(), f.size());
    if (o->trie_all || is_wild(ws)) o->trie.erase(f);
  }
}

void orc_freeze(void* h) { static_cast<Oracle*>(h)->trie.freeze(); }

uint64_t orc_num_keys(void* h) { return static_cast<Oracle*>(h)->trie.sorted.size(); }

// mode 0: emqx_router:match_routes/1 ids (exact ∪ trie), emqx_router.erl:128-140
// mode 1: emqx_trie:match/1 ids, emqx_trie.erl:148-162
// Writes per-topic counts into counts[n] and, when ids != nullptr, the sorted ids of topic
// t at ids[t*stride ... t*stride+count) (count clipped to stride).  Returns total lookups.
uint64_t orc_match(void* h, const uint8_t* bytes, const uint64_t* offs, uint64_t n, int mode,
                   int nthreads, uint32_t* counts, uint32_t* ids, uint32_t stride) {
  auto* o = static_cast<Oracle*>(h);
  o->trie.freeze();
  if (nthreads < 1) nthreads = 1;
  std::atomic<uint64_t> total_lk{0};
  auto work = [&](uint64_t lo, uint64_t hi) {
    std::vector<std::string> acc;
    std::vector<uint32_t> out;
    uint64_t lk = 0;
    for (uint64_t t = lo; t < hi; ++t) {
      const char* p = reinterpret_cast<const char*>(bytes + offs[t]);
      size_t len = offs[t + 1] - offs[t];
      acc.clear();
      bool trie_empty = o->trie.empty();
      if (!(mode == 0 && trie_empty)) o->trie.match(p, len, acc, lk);
      out.clear();
      if (mode == 0) {
        // match_routes: lookup_routes(T) ++ lookup_routes(F) for F in trie matches
        auto it = o->ids.find(std::string(p, len));
        if (it != o->ids.end() && o->live[it->second]) out.push_back(it->second);
      }
      for (auto& f : acc) {
        auto it = o->ids.find(f);
        if (it != o->ids.end() && o->live[it->second]) out.push_back(it->second);
      }
      std::sort(out.begin(), out.end());
      out.erase(std::unique(out.begin(), out.end()), out.end());
      counts[t] = static_cast<uint32_t>(out.size());
      if (ids) {
        size_t m = std::min<size_t>(out.size(), stride);
        for (size_t k = 0; k < m; ++k) ids[t * stride + k] = out[k];
      }
    }
    total_lk += lk;
  };
  std::vector<std::thread> th;
  uint64_t chunk = (n + nthreads - 1) / nthreads;
  for (int k = 0; k < nthreads; ++k) {
    uint64_t lo = k * chunk, hi = std::min<uint64_t>(n, lo + chunk);
    if (lo >= hi) break;
    th.emplace_back(work, lo, hi);
  }
  for (auto& x : th) x.join();
  return total_lk.load();
}

// orc_match as a CSR (no per-topic stride): each thread matches a contiguous slice of the
// topics into its own id list; out_off[n+1] receives the offsets; the concatenated sorted ids
// stay in the returned result until orc_csr_copy / orc_csr_free.  *lookups = total lookups.
struct CsrResult {
  std::vector<std::vector<uint32_t>> parts;
  uint64_t total = 0;
};

void* orc_match_csr(void* h, const uint8_t* bytes, const uint64_t* offs, uint64_t n, int mode, int nthreads,
                    uint64_t* out_off, uint64_t* lookups) {
  auto* o = static_cast<Oracle*>(h);
  o->trie.freeze();
  if (nthreads < 1) nthreads = 1;
  auto* res = new CsrResult();
  std::vector<uint32_t> counts(n ? n : 1);
  const uint64_t chunk = (n + nthreads - 1) / std::max<uint64_t>(nthreads, 1);
  const int parts = n ? static_cast<int>((n + chunk - 1) / chunk) : 0;
  res->parts.resize(parts);
  std::atomic<uint64_t> total_lk{0};
  auto work = [&](int k) {
    const uint64_t lo = k * chunk, hi = std::min<uint64_t>(n, lo + chunk);
    std::vector<std::string> acc;
    std::vector<uint32_t> out;
    auto& dst = res->parts[k];
    uint64_t lk = 0;
    for (uint64_t t = lo; t < hi; ++t) {
      const char* p = reinterpret_cast<const char*>(bytes + offs[t]);
      size_t len = offs[t + 1] - offs[t];
      acc.clear();
      if (!(mode == 0 && o->trie.empty())) o->trie.match(p, len, acc, lk);
      out.clear();
      if (mode == 0) {
        auto it = o->ids.find(std::string(p, len));
        if (it != o->ids.end() && o->live[it->second]) out.push_back(it->second);
      }
      for (auto& f : acc) {
        auto it = o->ids.find(f);
        if (it != o->ids.end() && o->live[it->second]) out.push_back(it->second);
      }
      std::sort(out.begin(), out.end());
      out.erase(std::unique(out.begin(), out.end()), out.end());
      counts[t] = static_cast<uint32_t>(out.size());
      dst.insert(dst.end(), out.begin(), out.end());
    }
    total_lk += lk;
  };
  std::vector<std::thread> th;
  for (int k = 0; k < parts; ++k) th.emplace_back(work, k);
  for (auto& x : th) x.join();
  out_off[0] = 0;
  for (uint64_t t = 0; t < n; ++t) out_off[t + 1] = out_off[t] + counts[t];
  res->total = n ? out_off[n] : 0;
  if (lookups) *lookups = total_lk.load();
  return res;
}

void orc_csr_copy(void* r, uint32_t* dst) {
  auto* res = static_cast<CsrResult*>(r);
  for (auto& p : res->parts) {
    if (!p.empty()) std::memcpy(dst, p.data(), p.size() * sizeof(uint32_t));
    dst += p.size();
  }
}

void orc_csr_free(void* r) { delete static_cast<CsrResult*>(r); }

// evals(T) per SURVEY §8(d) over ALL live filters (exact and wildcard).
void orc_evals(void* h, const uint8_t* bytes, const uint64_t* offs, uint64_t n, uint64_t* out) {
  auto* o = static_cast<Oracle*>(h);
  LevelTrie lt;
  for (auto& kv : o->ids) {
    if (!o->live[kv.second]) continue;
    auto ws = split_words(kv.first.data(), kv.first.size());
    uint64_t node = 0;
    for (auto& w : ws) {
      auto k = LevelTrie::key(node, w);
      auto it = lt.node_of.find(k);
      if (it == lt.node_of.end()) it = lt.node_of.emplace(k, lt.next++).first;
      node = it->second;
    }
  }
  Word plus{"+", W_PLUS};
  for (uint64_t t = 0; t < n; ++t) {
    auto ws = split_words(reinterpret_cast<const char*>(bytes + offs[t]), offs[t + 1] - offs[t]);
    if (is_wild(ws)) { out[t] = 0; continue; }
    bool dollar = ws[0].kind == W_BIN && ws[0].bin[0] == '$';
    std::vector<uint64_t> fr{0}, nx;
    uint64_t total = 1;
    for (size_t i = 0; i < ws.size() && !fr.empty(); ++i) {
      nx.clear();
      for (auto nd : fr) {
        auto it = lt.node_of.find(LevelTrie::key(nd, ws[i]));
        if (it != lt.node_of.end()) nx.push_back(it->second);
        if (!(i == 0 && dollar)) {
          auto ip = lt.node_of.find(LevelTrie::key(nd, plus));
          if (ip != lt.node_of.end()) nx.push_back(ip->second);
        }
      }
      fr.swap(nx);
      total += fr.size();
    }
    out[t] = total;
  }
}

// emqx_topic:match/2 (emqx_topic.erl:68-87) on raw binaries.
int orc_topic_match(const uint8_t* name, uint64_t nlen, const uint8_t* filt, uint64_t flen) {
  if (nlen > 0 && name[0] == '$' && flen > 0 && (filt[0] == '+' || filt[0] == '#')) return 0;
  auto n = split_words(reinterpret_cast<const char*>(name), nlen);
  auto f = split_words(reinterpret_cast<const char*>(filt), flen);
  size_t i = 0;
  while (true) {
    if (i == n.size() && i == f.size()) return 1;
    if (i < n.size() && i < f.size() && n[i].kind == f[i].kind && n[i].bin == f[i].bin) { ++i; continue; }
    if (i < n.size() && i < f.size() && f[i].kind == W_PLUS) { ++i; continue; }
    if (f.size() - i == 1 && f[i].kind == W_HASH) return 1;
    return 0;
  }
}

}  // extern "C"
