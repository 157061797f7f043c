// CPU restatement of the publish fan-out — TEST INFRASTRUCTURE ONLY (the CPU baseline of
// bench.py --workload E and a parity checker for its GPU fan-out).  Loaded through ctypes by
// bench.py's cpu_baseline leg and tests/; never linked into the product library.
//
// Restates (paths relative to /root/reference), given the match_routes/1 ids of each topic:
//   apps/emqx/src/emqx_broker.erl:244-272,500-524  route/aggre/do_dispatch: every plain
//       subscriber of every matched filter gets one delivery ({shard, I} buckets are a storage
//       split only, emqx_broker_helper.erl:81-86);
//   apps/emqx/src/emqx_shared_sub.erl:113-126,251-288  dispatch/pick: one member per $share
//       group of a matched filter; for hash_clientid / hash_topic the member is
//       lists:nth(1 + Key rem N, Members), Members in subscription order (ETS bag order,
//       :287-288), Key = the caller's erlang:phash2 value (not restated);
//       round_robin (:279-285) with the counter seeded 0 (SURVEY §8 d, config E): per (publisher,
//       group, filter) the first pick is member 1, each later one (Last + 1) rem N, in message
//       order; a one-member group is picked without touching the state (:265).
// Per topic it reports the delivery count and an order-free checksum of its deliveries
// (sum of mix(sub, filter | shared bit)), so a multiset comparison with the GPU's CSR needs no
// sort.  orf_churn applies subscribe / unsubscribe operations as the reference's tables take
// them (the CPU baseline of bench.py --workload S):
//   emqx_broker:do_subscribe/3 ets:insert(?SUBSCRIBER, {Topic, SubPid}) on a bag
//       (apps/emqx/src/emqx_broker.erl:146-164; an identical object is stored once);
//   emqx_broker:do_unsubscribe ets:delete_object(?SUBSCRIBER, {Topic, SubPid}) (:183-195);
//   emqx_shared_sub subscribe/unsubscribe: the {Group, Topic, SubPid} bag write / delete_object
//       (emqx_shared_sub.erl:308-322), members kept in insertion order.
// ETS takes writes to different keys concurrently (write_concurrency), so the ops are split by
// filter over the threads, each thread applying its filters' ops in order.
// Build: oracle/Makefile -> oracle/_build/liboracle.so.
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

constexpr uint32_t NO_GROUP = 0xFFFFFFFFu;
constexpr uint32_t SHARED_BIT = 0x80000000u;

struct Group {
  uint32_t id;
  std::vector<uint32_t> members;  // subscription order
};

struct RrKey {
  uint64_t fil_group;  // filter << 32 | group id
  uint32_t publisher;
  bool operator==(const RrKey& o) const { return fil_group == o.fil_group && publisher == o.publisher; }
};
struct RrHash {
  size_t operator()(const RrKey& k) const {
    uint64_t x = k.fil_group * 0x9E3779B97F4A7C15ULL ^ (uint64_t(k.publisher) * 0xC2B2AE3D27D4EB4FULL);
    return static_cast<size_t>(x ^ (x >> 29));
  }
};

struct Fanout {
  std::vector<std::vector<uint32_t>> plain;  // per filter id
  std::vector<std::vector<Group>> groups;    // per filter id, groups in first-subscription order
  std::unordered_map<RrKey, uint32_t, RrHash> rr;  // round_robin: the publisher's Last index (0-based)
};

inline uint64_t mix(uint32_t sub, uint32_t fil) {
  uint64_t x = (uint64_t(sub) << 32) | fil;
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

}  // namespace

extern "C" {

void* orf_create(const uint32_t* filt, const uint32_t* sub, const uint32_t* grp, uint64_t n) {
  auto* f = new Fanout();
  uint32_t nf = 0;
  for (uint64_t i = 0; i < n; ++i) nf = std::max(nf, filt[i] + 1);
  f->plain.resize(nf);
  f->groups.resize(nf);
  for (uint64_t i = 0; i < n; ++i) {
    if (grp[i] == NO_GROUP) {
      f->plain[filt[i]].push_back(sub[i]);
      continue;
    }
    auto& gs = f->groups[filt[i]];
    auto it = std::find_if(gs.begin(), gs.end(), [&](const Group& g) { return g.id == grp[i]; });
    if (it == gs.end()) {
      gs.push_back(Group{grp[i], {}});
      it = gs.end() - 1;
    }
    it->members.push_back(sub[i]);
  }
  return f;
}

void orf_destroy(void* h) { delete static_cast<Fanout*>(h); }

// Hash strategies: deliveries of each topic of a match CSR (moff[n+1], mids).  counts[t],
// sums[t] per topic; returns the total.
uint64_t orf_publish(void* h, const uint64_t* moff, const uint32_t* mids, uint64_t n, const uint32_t* keys,
                     int nthreads, uint32_t* counts, uint64_t* sums) {
  const Fanout* f = static_cast<const Fanout*>(h);
  if (nthreads < 1) nthreads = 1;
  std::atomic<uint64_t> total{0};
  auto work = [&](uint64_t lo, uint64_t hi) {
    uint64_t tot = 0;
    for (uint64_t t = lo; t < hi; ++t) {
      uint32_t c = 0;
      uint64_t s = 0;
      for (uint64_t j = moff[t]; j < moff[t + 1]; ++j) {
        const uint32_t fid = mids[j];
        if (fid >= f->plain.size()) continue;
        for (uint32_t sb : f->plain[fid]) {
          ++c;
          s += mix(sb, fid);
        }
        for (const Group& g : f->groups[fid]) {
          if (g.members.empty()) continue;
          ++c;
          s += mix(g.members[keys[t] % g.members.size()], fid | SHARED_BIT);
        }
      }
      counts[t] = c;
      sums[t] = s;
      tot += c;
    }
    total += tot;
  };
  std::vector<std::thread> th;
  const uint64_t chunk = (n + nthreads - 1) / nthreads;
  for (int k = 0; k < nthreads; ++k) {
    const uint64_t lo = k * chunk, hi = std::min<uint64_t>(n, lo + chunk);
    if (lo >= hi) break;
    th.emplace_back(work, lo, hi);
  }
  for (auto& x : th) x.join();
  return total.load();
}

// Hash strategies, deliveries listed: per topic of a match CSR its (subscriber, filter) pairs
// (filter | SHARED_BIT for a $share pick) at out_off[t] (exclusive prefix of the counts, which
// the caller sizes with orf_publish).  The per-topic order is route order, not sorted.
void orf_publish_list(void* h, const uint64_t* moff, const uint32_t* mids, uint64_t n, const uint32_t* keys,
                      int nthreads, const uint64_t* out_off, uint32_t* out_subs, uint32_t* out_fils) {
  const Fanout* f = static_cast<const Fanout*>(h);
  if (nthreads < 1) nthreads = 1;
  auto work = [&](uint64_t lo, uint64_t hi) {
    for (uint64_t t = lo; t < hi; ++t) {
      uint64_t at = out_off[t];
      for (uint64_t j = moff[t]; j < moff[t + 1]; ++j) {
        const uint32_t fid = mids[j];
        if (fid >= f->plain.size()) continue;
        for (uint32_t sb : f->plain[fid]) {
          out_subs[at] = sb;
          out_fils[at++] = fid;
        }
        for (const Group& g : f->groups[fid]) {
          if (g.members.empty()) continue;
          out_subs[at] = g.members[keys[t] % g.members.size()];
          out_fils[at++] = fid | SHARED_BIT;
        }
      }
    }
  };
  std::vector<std::thread> th;
  const uint64_t chunk = (n + nthreads - 1) / nthreads;
  for (int k = 0; k < nthreads; ++k) {
    const uint64_t lo = k * chunk, hi = std::min<uint64_t>(n, lo + chunk);
    if (lo >= hi) break;
    th.emplace_back(work, lo, hi);
  }
  for (auto& x : th) x.join();
}

// round_robin with the counter seeded 0, deliveries listed as orf_publish_list (route order per
// topic); keys[t] = the publishing process.  Message order is the batch order, so one thread; the
// state persists over calls (orf_rr_reset clears it).
void orf_publish_list_rr(void* h, const uint64_t* moff, const uint32_t* mids, uint64_t n, const uint32_t* keys,
                         const uint64_t* out_off, uint32_t* out_subs, uint32_t* out_fils) {
  Fanout* f = static_cast<Fanout*>(h);
  for (uint64_t t = 0; t < n; ++t) {
    uint64_t at = out_off[t];
    for (uint64_t j = moff[t]; j < moff[t + 1]; ++j) {
      const uint32_t fid = mids[j];
      if (fid >= f->plain.size()) continue;
      for (uint32_t sb : f->plain[fid]) {
        out_subs[at] = sb;
        out_fils[at++] = fid;
      }
      for (const Group& g : f->groups[fid]) {
        const uint32_t cnt = static_cast<uint32_t>(g.members.size());
        if (!cnt) continue;
        uint32_t idx = 0;
        if (cnt > 1) {
          const RrKey k{(uint64_t(fid) << 32) | g.id, keys[t]};
          auto it = f->rr.find(k);
          idx = it == f->rr.end() ? 0u : (it->second + 1) % cnt;
          f->rr[k] = idx;
        }
        out_subs[at] = g.members[idx];
        out_fils[at++] = fid | SHARED_BIT;
      }
    }
  }
}

void orf_rr_reset(void* h) { static_cast<Fanout*>(h)->rr.clear(); }

// Subscribe (add = 1) / unsubscribe (add = 0) operations, in order per filter.  Returns the
// operations that changed the table.
uint64_t orf_churn(void* h, const uint32_t* filt, const uint32_t* sub, const uint32_t* grp, const uint8_t* add,
                   uint64_t n, int nthreads) {
  Fanout* f = static_cast<Fanout*>(h);
  uint32_t nf = static_cast<uint32_t>(f->plain.size());
  for (uint64_t i = 0; i < n; ++i) nf = std::max(nf, filt[i] + 1);
  f->plain.resize(nf);
  f->groups.resize(nf);
  if (nthreads < 1) nthreads = 1;
  std::atomic<uint64_t> changed{0};
  auto work = [&](int k) {
    uint64_t ch = 0;
    for (uint64_t i = 0; i < n; ++i) {
      const uint32_t fid = filt[i];
      if (static_cast<int>(fid % static_cast<uint32_t>(nthreads)) != k) continue;
      std::vector<uint32_t>* v;
      if (grp[i] == NO_GROUP) {
        v = &f->plain[fid];
      } else {
        auto& gs = f->groups[fid];
        auto it = std::find_if(gs.begin(), gs.end(), [&](const Group& g) { return g.id == grp[i]; });
        if (it == gs.end()) {
          if (!add[i]) continue;
          gs.push_back(Group{grp[i], {}});
          it = gs.end() - 1;
        }
        v = &it->members;
      }
      auto pos = std::find(v->begin(), v->end(), sub[i]);
      if (add[i] && pos == v->end()) {
        v->push_back(sub[i]);
        ++ch;
      } else if (!add[i] && pos != v->end()) {
        v->erase(pos);  // keeps the others' order
        ++ch;
      }
    }
    changed += ch;
  };
  std::vector<std::thread> th;
  for (int k = 0; k < nthreads; ++k) th.emplace_back(work, k);
  for (auto& x : th) x.join();
  return changed.load();
}

// The same checksum of a GPU delivery CSR (off[n+1], subs, filters with the shared bit).
void orf_checksum(const uint64_t* off, const uint32_t* subs, const uint32_t* fils, uint64_t n, uint64_t* sums) {
  for (uint64_t t = 0; t < n; ++t) {
    uint64_t s = 0;
    for (uint64_t j = off[t]; j < off[t + 1]; ++j) s += mix(subs[j], fils[j]);
    sums[t] = s;
  }
}

}  // extern "C"
