// emqx_topic:match/2 and wildcard/1 on the CPU (include/emqx_match.h).  Per-pair callers
// (authz rules, rule engine, bridges: SURVEY §2b) keep calling this on the CPU; it must agree
// with the device engine, which tests/test_abi_cpu.py checks against the reference KATs.
//
// apps/emqx/src/emqx_topic.erl:53-62 (wildcard/1), :68-87 (match/2), :153-164 (words).
#include <stdint.h>

#include "../../include/emqx_match.h"

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
