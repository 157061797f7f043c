// emqx_topic:match/2 and wildcard/1 on the CPU (include/emqx_match.h).  Per-pair callers
// (authz rules, rule engine, bridges: SURVEY §2b) keep calling this on the CPU; it must agree
// with the device engine, which tests/test_abi_cpu.py checks against the reference KATs.
//
// apps/emqx/src/emqx_topic.erl:53-62 (wildcard/1), :68-87 (match/2), :153-164 (words).
#include <stdint.h>

#include <string.h>

#include <string>

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
