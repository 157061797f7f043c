// ORACLE / CPU BASELINE (test infrastructure only — never linked into the product library).
//
// C++ restatement of the reference's retained-message lookup, the way the reference runs it:
//   * a wildcard filter is answered by mnesia:dirty_select(?TAB, MatchSpec) over a `set`
//     table, i.e. a scan of EVERY record, testing condition/1's pattern against the record's
//     token list and the expiry guard (apps/emqx_retainer/src/emqx_retainer_mnesia.erl:212-258)
//   * a plain filter is mnesia:dirty_read(?TAB, Tokens): one key lookup, then
//     Et =:= 0 orelse Et >= NowMs (:199-208)
// Used as bench.py's cpu_baseline for --workload R (kind "port") and, on small tables, as
// a second checker beside oracle/retain_ref.py.
#include <stdint.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

struct Tok {
  uint32_t off, len;
};

struct RetainScan {
  std::vector<uint8_t> bytes;
  std::vector<uint64_t> rec_tok;  // record i: tokens [rec_tok[i], rec_tok[i+1])
  std::vector<Tok> toks;
  std::vector<int64_t> expiry;
  std::unordered_map<std::string, uint32_t> key;
};

void split(const uint8_t* p, uint64_t n, std::vector<Tok>* out, uint32_t base) {
  uint64_t s = 0;
  for (uint64_t i = 0; i <= n; ++i) {
    if (i == n || p[i] == '/') {
      out->push_back(Tok{static_cast<uint32_t>(base + s), static_cast<uint32_t>(i - s)});
      s = i + 1;
    }
  }
}

}  // namespace

extern "C" {

void* orr_create(const uint8_t* bytes, const uint64_t* offs, uint64_t n, const int64_t* expiry) {
  auto* t = new RetainScan();
  t->bytes.assign(bytes + offs[0], bytes + offs[n]);
  t->rec_tok.push_back(0);
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t a = offs[i] - offs[0], b = offs[i + 1] - offs[0];
    split(t->bytes.data() + a, b - a, &t->toks, static_cast<uint32_t>(a));
    t->rec_tok.push_back(t->toks.size());
    t->expiry.push_back(expiry ? expiry[i] : 0);
    t->key.emplace(std::string(reinterpret_cast<const char*>(t->bytes.data() + a), b - a), static_cast<uint32_t>(i));
  }
  return t;
}

void orr_destroy(void* h) { delete static_cast<RetainScan*>(h); }

// dispatch/4 for every filter: counts[f] = topics selected, ids_sum[f] = sum of their ids
// (a checksum comparable with the device's CSR).  now < 0: no expiry guard.
void orr_select(void* h, const uint8_t* fb, const uint64_t* fo, uint64_t nf, int64_t now, int threads,
                uint32_t* counts, uint64_t* ids_sum) {
  const RetainScan& t = *static_cast<RetainScan*>(h);
  const uint64_t nrec = t.expiry.size();
  auto one = [&](uint64_t f) {
    const uint8_t* p = fb + fo[f];
    const uint64_t n = fo[f + 1] - fo[f];
    std::vector<Tok> ft;
    split(p, n, &ft, 0);
    bool wild = false;
    for (const Tok& k : ft) wild |= k.len == 1 && (p[k.off] == '+' || p[k.off] == '#');
    uint32_t c = 0;
    uint64_t sum = 0;
    if (!wild) {  // dirty_read on the token-list key
      auto it = t.key.find(std::string(reinterpret_cast<const char*>(p), n));
      if (it != t.key.end()) {
        const int64_t e = t.expiry[it->second];
        if (now < 0 || e == 0 || e >= now) {
          c = 1;
          sum = it->second;
        }
      }
    } else {
      // condition/1: '+' -> any; a final '#' dropped (the FIRST '#' removed) + open tail
      bool open = false;
      if (ft.back().len == 1 && p[ft.back().off] == '#') {
        open = true;
        for (uint64_t i = 0; i < ft.size(); ++i)
          if (ft[i].len == 1 && p[ft[i].off] == '#') {
            ft.erase(ft.begin() + i);
            break;
          }
      }
      for (uint64_t r = 0; r < nrec; ++r) {  // the full-table select
        const uint64_t a = t.rec_tok[r], b = t.rec_tok[r + 1];
        const uint64_t nt = b - a;
        if (nt < ft.size() || (!open && nt != ft.size())) continue;
        bool ok = true;
        for (uint64_t i = 0; i < ft.size() && ok; ++i) {
          const Tok& q = ft[i];
          if (q.len == 1 && p[q.off] == '+') continue;
          const Tok& s = t.toks[a + i];
          ok = s.len == q.len && std::memcmp(t.bytes.data() + s.off, p + q.off, q.len) == 0;
        }
        if (!ok) continue;
        const int64_t e = t.expiry[r];
        if (now < 0 || e == 0 || e > now) {
          ++c;
          sum += r;
        }
      }
    }
    counts[f] = c;
    ids_sum[f] = sum;
  };
  threads = std::max(1, threads);
  std::vector<std::thread> th;
  for (int k = 0; k < threads; ++k)
    th.emplace_back([&, k] {
      for (uint64_t f = k; f < nf; f += threads) one(f);
    });
  for (auto& x : th) x.join();
}

}  // extern "C"
