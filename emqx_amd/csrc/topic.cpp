// emqx_topic:match/2 and wildcard/1 on the CPU (include/emqx_match.h).  Per-pair callers
// (authz rules, rule engine, bridges: SURVEY §2b) keep calling this on the CPU; it must agree
// with the device engine, which tests/test_abi_cpu.py checks against the reference KATs.
//
// apps/emqx/src/emqx_topic.erl:53-62 (wildcard/1), :68-87 (match/2), :153-164 (words).
#include <stdint.h>

#include <string.h>

#include <algorithm>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/emqx_match.h"
#include "tables.h"

namespace {

struct Level {
  const uint8_t* p;
  uint64_t n;
};

// next level starting at *pos; returns false when the string is exhausted
inline bool next_level(const uint8_t* s, uint64_t len, uint64_t* pos, bool* done, Level* out) {
  if (*done) return false;
  uint64_t i = *pos;
  while (i < len && s[i] != '/') ++i;
  out->p = s + *pos;
  out->n = i - *pos;
  if (i >= len) *done = true;
  *pos = i + 1;
  return true;
}

inline bool is_plus(const Level& l) { return l.n == 1 && l.p[0] == '+'; }
inline bool is_hash(const Level& l) { return l.n == 1 && l.p[0] == '#'; }
inline bool same(const Level& a, const Level& b) {
  if (a.n != b.n) return false;
  for (uint64_t i = 0; i < a.n; ++i)
    if (a.p[i] != b.p[i]) return false;
  return true;
}

}  // namespace

extern "C" int emqx_topic_wildcard(const uint8_t* t, uint64_t len) {
  uint64_t pos = 0;
  bool done = false;
  Level l;
  while (next_level(t, len, &pos, &done, &l))
    if (is_plus(l) || is_hash(l)) return 1;
  return 0;
}

extern "C" int emqx_topic_match(const uint8_t* name, uint64_t nlen, const uint8_t* filter, uint64_t flen) {
  // emqx_topic.erl:68-71: '$' names never match filters starting with '+' or '#'
  if (nlen > 0 && name[0] == '$' && flen > 0 && (filter[0] == '+' || filter[0] == '#')) return 0;
  uint64_t np = 0, fp = 0;
  bool nd = false, fd = false;
  Level n, f;
  bool hn = next_level(name, nlen, &np, &nd, &n);
  bool hf = next_level(filter, flen, &fp, &fd, &f);
  while (true) {
    if (!hn && !hf) return 1;                      // match([], [])
    if (hn && hf && (same(n, f) || is_plus(f))) {  // [H|T1],[H|T2]  /  [_|T1],['+'|T2]
      hn = next_level(name, nlen, &np, &nd, &n);
      hf = next_level(filter, flen, &fp, &fd, &f);
      continue;
    }
    if (hf && is_hash(f) && fd) return 1;          // match(_, ['#'])
    return 0;
  }
}

// Host-only builder self-check (no device needed): builds the level trie of the given
// filters and verifies its lookup invariants.  stats_out (optional, 4 entries): nodes,
// slots, words, perfect-hashed nodes.
extern "C" int emqx_shard_owner(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint32_t world,
                                uint32_t levels, int topics, uint32_t* owner_out) {
  if ((n && (!offsets || !owner_out)) || world == 0 || levels == 0) return EMQX_EINVAL;
  for (uint64_t i = 0; i < n; ++i) {
    if (offsets[i + 1] < offsets[i]) return EMQX_EINVAL;
    owner_out[i] = emqx::shard_owner(bytes + offsets[i], offsets[i + 1] - offsets[i], world, levels, topics != 0);
  }
  return EMQX_OK;
}

// Filter-sharded layout with two key spaces (layout.h shard_place_filter / shard_route_topic).
namespace {

// The level hashes a filter contributes to the plan: its key (space bit | 30-bit hash) and its
// next level (hash, SHARD_ABSENT, or SHARD_NONE for a wildcard).  false for root wildcards.
bool plan_key(const uint8_t* p, uint64_t len, uint32_t* key, uint32_t* hk, uint32_t* next) {
  uint64_t s1, e1, s2, e2, s3, e3;
  emqx::shard_level(p, len, 0, &s1, &e1);
  const bool has2 = emqx::shard_level(p, len, 1, &s2, &e2);
  if (!emqx::shard_is_wild(p, s1, e1)) {
    *hk = emqx::shard_level_hash(p, s1, e1);
    *key = *hk & emqx::SHARD_HASH_MASK;
    *next = !has2 ? emqx::SHARD_ABSENT : emqx::shard_is_wild(p, s2, e2) ? emqx::SHARD_NONE
                                                                        : emqx::shard_level_hash(p, s2, e2);
    return true;
  }
  if (p[s1] != '+' || !has2 || emqx::shard_is_wild(p, s2, e2)) return false;
  *hk = emqx::shard_level_hash(p, s2, e2);
  *key = emqx::SHARD_SPACE_P | (*hk & emqx::SHARD_HASH_MASK);
  const bool has3 = emqx::shard_level(p, len, 2, &s3, &e3);
  *next = !has3 ? emqx::SHARD_ABSENT : emqx::shard_is_wild(p, s3, e3) ? emqx::SHARD_NONE
                                                                      : emqx::shard_level_hash(p, s3, e3);
  return true;
}

}  // namespace

extern "C" int emqx_shard_plan(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint32_t world,
                               uint32_t max_piece_pm, uint32_t p_space, emqx_shard_split* out, uint32_t cap,
                               uint32_t* n_out) {
  if ((n && !offsets) || !n_out || world == 0 || world > 65535 || max_piece_pm == 0 || (cap && !out) ||
      p_space > EMQX_SHARD_P_REPLICATED)
    return EMQX_EINVAL;
  for (uint64_t i = 0; i < n; ++i)
    if (offsets[i + 1] < offsets[i]) return EMQX_EINVAL;
  // per key of each space: its filters, and those whose next level is a wildcard (they go to
  // every rank of a split key); root-wildcard filters are everywhere and count for no key
  struct KeyLoad {
    uint64_t all = 0, wild_next = 0;
  };
  std::unordered_map<uint32_t, KeyLoad> per_key;
  uint32_t key, hk, next;
  uint64_t n_p = 0;  // space P's filters
  for (uint64_t i = 0; i < n; ++i) {
    if (!plan_key(bytes + offsets[i], offsets[i + 1] - offsets[i], &key, &hk, &next)) continue;
    KeyLoad& k = per_key[key];
    ++k.all;
    k.wild_next += next == emqx::SHARD_NONE ? 1u : 0u;
    n_p += (key & emqx::SHARD_SPACE_P) ? 1u : 0u;
  }
  // space P replicated (layout.h SHARD_P_REPLICATED) when it holds at most a rank's share: its
  // keys then take no part in the plan
  const bool p_repl = world > 1 && (p_space == EMQX_SHARD_P_REPLICATED ||
                                    (p_space == EMQX_SHARD_P_AUTO && n_p * world <= n));
  if (p_repl)
    for (auto it = per_key.begin(); it != per_key.end();)
      it = (it->first & emqx::SHARD_SPACE_P) ? per_key.erase(it) : std::next(it);
  // Largest keys first onto the least-loaded ranks (LPT).  A key over max_piece_pm / 1000 of a
  // rank's share is split over the fewest consecutive ranks that bring each piece under it: its
  // wildcard-next filters go to all of them, its next-level words are placed one by one (the
  // largest first) on the least-loaded rank of that window.  Every key or next word down to
  // 1/4096 of a share is placed this way; the many smaller ones are left to the hash.
  const double share = static_cast<double>(n) / world;
  const double piece = share * max_piece_pm / 1000.0;
  const double small = std::max(2.0, share / 4096.0);
  std::vector<std::pair<uint32_t, KeyLoad>> keys;
  for (const auto& kv : per_key)
    if (static_cast<double>(kv.second.all) >= small) keys.push_back(kv);
  auto by_size = [](const std::pair<uint32_t, KeyLoad>& a, const std::pair<uint32_t, KeyLoad>& b) {
    return a.second.all != b.second.all ? a.second.all > b.second.all : a.first < b.first;
  };
  std::sort(keys.begin(), keys.end(), by_size);
  std::unordered_map<uint32_t, std::pair<uint32_t, uint32_t>> split;  // key -> (first rank, span)
  std::vector<uint32_t> span_of(keys.size(), 1);
  for (size_t q = 0; q < keys.size(); ++q) {
    uint32_t span = 1;
    while (span < world && static_cast<double>(keys[q].second.all) / span > piece) span *= 2;
    span_of[q] = std::min(span, world);
    if (span_of[q] > 1) split[keys[q].first] = {0, span_of[q]};
  }
  // next-level words of the split keys
  std::unordered_map<uint64_t, uint64_t> per_pair;  // key << 32 | pair hash -> filters
  if (!split.empty()) {
    for (uint64_t i = 0; i < n; ++i) {
      if (!plan_key(bytes + offsets[i], offsets[i + 1] - offsets[i], &key, &hk, &next)) continue;
      if (next == emqx::SHARD_NONE || next == emqx::SHARD_ABSENT || !split.count(key)) continue;
      ++per_pair[(uint64_t(key) << 32) | (emqx::mix32(next ^ hk) & emqx::SHARD_HASH_MASK)];
    }
  }
  std::unordered_map<uint32_t, std::vector<std::pair<uint32_t, uint64_t>>> pairs_of;
  for (const auto& kv : per_pair)
    if (static_cast<double>(kv.second) >= small)
      pairs_of[static_cast<uint32_t>(kv.first >> 32)].push_back({static_cast<uint32_t>(kv.first), kv.second});
  std::vector<double> load(world, 0.0);
  std::vector<emqx_shard_split> sp;
  for (size_t q = 0; q < keys.size(); ++q) {
    const uint32_t span = span_of[q];
    const double c = static_cast<double>(keys[q].second.all), g = static_cast<double>(keys[q].second.wild_next);
    uint32_t best = 0;
    double best_m = 0;
    for (uint32_t b = 0; b < world; ++b) {  // the window of `span` ranks whose busiest is least busy
      double m = 0;
      for (uint32_t k = 0; k < span; ++k) m = std::max(m, load[(b + k) % world]);
      if (b == 0 || m < best_m) {
        best = b;
        best_m = m;
      }
    }
    sp.push_back(emqx_shard_split{keys[q].first, best | (span << 16)});
    if (span == 1) {
      load[best] += c;
      continue;
    }
    for (uint32_t k = 0; k < span; ++k) load[(best + k) % world] += g;
    auto& pv = pairs_of[keys[q].first];
    std::sort(pv.begin(), pv.end(), [](const std::pair<uint32_t, uint64_t>& a, const std::pair<uint32_t, uint64_t>& b) {
      return a.second != b.second ? a.second > b.second : a.first < b.first;
    });
    double placed = g;
    for (const auto& pr : pv) {
      uint32_t r = best;
      for (uint32_t k = 1; k < span; ++k)
        if (load[(best + k) % world] < load[r]) r = (best + k) % world;
      load[r] += static_cast<double>(pr.second);
      placed += static_cast<double>(pr.second);
      sp.push_back(emqx_shard_split{emqx::SHARD_PAIR | (keys[q].first & emqx::SHARD_SPACE_P) | pr.first, r});
    }
    for (uint32_t k = 0; k < span; ++k) load[(best + k) % world] += (c - placed) / span;  // hashed rest
  }
  if (p_repl) sp.push_back(emqx_shard_split{emqx::SHARD_SPACE_P, emqx::SHARD_P_REPLICATED});
  std::sort(sp.begin(), sp.end(), [](const emqx_shard_split& a, const emqx_shard_split& b) { return a.key < b.key; });
  sp.erase(std::unique(sp.begin(), sp.end(),
                       [](const emqx_shard_split& a, const emqx_shard_split& b) { return a.key == b.key; }),
           sp.end());  // (a 30-bit collision: either entry gives a consistent placement)
  *n_out = static_cast<uint32_t>(sp.size());
  if (sp.size() > cap) return EMQX_EOVERFLOW;
  std::copy(sp.begin(), sp.end(), out);
  return EMQX_OK;
}

static_assert(sizeof(emqx_shard_split) == sizeof(emqx::ShardSplitE), "split layout");

extern "C" int emqx_shard_place(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint32_t world,
                                const emqx_shard_split* splits, uint32_t n_splits, uint32_t* first, uint32_t* span,
                                uint32_t* engine) {
  if ((n && (!offsets || !first || !span || !engine)) || world == 0 || (n_splits && !splits)) return EMQX_EINVAL;
  const auto* sp = reinterpret_cast<const emqx::ShardSplitE*>(splits);
  for (uint64_t i = 0; i < n; ++i) {
    if (offsets[i + 1] < offsets[i]) return EMQX_EINVAL;
    emqx::shard_place_filter(bytes + offsets[i], offsets[i + 1] - offsets[i], world, sp, n_splits, &first[i], &span[i],
                             &engine[i]);
  }
  return EMQX_OK;
}

extern "C" int emqx_shard_route(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint32_t world,
                                const emqx_shard_split* splits, uint32_t n_splits, uint32_t* req2) {
  if ((n && (!offsets || !req2)) || world == 0 || (n_splits && !splits)) return EMQX_EINVAL;
  const auto* sp = reinterpret_cast<const emqx::ShardSplitE*>(splits);
  for (uint64_t i = 0; i < n; ++i) {
    if (offsets[i + 1] < offsets[i]) return EMQX_EINVAL;
    emqx::shard_route_topic(bytes + offsets[i], offsets[i + 1] - offsets[i], world, sp, n_splits, req2 + 2 * i);
  }
  return EMQX_OK;
}

extern "C" int emqx_build_check(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint64_t* stats_out,
                                char* err, uint64_t err_cap) {
  emqx::FilterStore fs;
  for (uint64_t i = 0; i < n; ++i) {
    bool created = false;
    fs.insert(bytes + offsets[i], offsets[i + 1] - offsets[i], &created);
  }
  emqx::HostTables t;
  std::string e;
  bool ok = emqx::build_tables(fs, t, &e) && emqx::check_tables(t, &e);
  if (stats_out) {
    stats_out[0] = t.n_nodes;
    stats_out[1] = t.edges.size();
    stats_out[2] = t.n_words;
    stats_out[3] = t.n_ph_nodes;
  }
  if (!ok && err && err_cap) {
    strncpy(err, e.c_str(), err_cap - 1);
    err[err_cap - 1] = 0;
  }
  return ok ? EMQX_OK : EMQX_EINVAL;
}
