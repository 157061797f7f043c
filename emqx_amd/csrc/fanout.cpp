// C ABI of the publish fan-out stage (include/emqx_match.h, emqx_subtab_* / emqx_fanout_* /
// emqx_publish_batch): host subscription store, device snapshot build, and the fan-out
// pipeline  entry_topic -> count -> scan -> offsets -> [one D2H of the total] -> write.
//
// Store semantics follow the reference's ETS tables:
//   plain subscriptions  ?SUBSCRIBER bag Topic -> SubPid (apps/emqx/src/emqx_broker.erl:146-158);
//                        the {shard, I} buckets of emqx_broker_helper:get_sub_shard/2
//                        (emqx_broker_helper.erl:81-86) only split storage, so the device
//                        array is the flattened union.
//   $share memberships   emqx_shared_subscription bag keyed by Group, selected per
//                        (Group, Topic) in insertion order (emqx_shared_sub.erl:288,300-314);
//                        the member order is what lists:nth/2 indexes in pick_subscriber/6.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "../../include/emqx_match.h"
#include "fanout.h"
#include "kernels.h"
#include "streams.h"

using namespace emqx;

namespace {

#define FO_TRY(expr)                \
  do {                              \
    hipError_t _e = (expr);         \
    if (_e != hipSuccess) return EMQX_EDEVICE; \
  } while (0)

inline uint64_t fo_mix64(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return x;
}

// Open-addressed set of u64 keys with tombstones (keys never take the two reserved values:
// filter ids and slots are < 2^31).
class U64Set {
 public:
  bool contains(uint64_t k) const {
    if (keys_.empty()) return false;
    const uint64_t mask = keys_.size() - 1;
    for (uint64_t i = fo_mix64(k) & mask;; i = (i + 1) & mask) {
      if (keys_[i] == EMPTY) return false;
      if (keys_[i] == k) return true;
    }
  }
  bool insert(uint64_t k) {  // true if newly inserted
    if (keys_.empty()) rehash(1024);
    else if ((used_ + 1) * 4 >= keys_.size() * 3)  // double, or just drop tombstones
      rehash((size_ + 1) * 2 >= keys_.size() ? keys_.size() * 2 : keys_.size());
    const uint64_t mask = keys_.size() - 1;
    uint64_t tomb = ~0ull;
    for (uint64_t i = fo_mix64(k) & mask;; i = (i + 1) & mask) {
      if (keys_[i] == k) return false;
      if (keys_[i] == TOMB && tomb == ~0ull) tomb = i;
      if (keys_[i] == EMPTY) {
        if (tomb != ~0ull) i = tomb; else ++used_;
        keys_[i] = k;
        ++size_;
        return true;
      }
    }
  }
  bool erase(uint64_t k) {
    if (keys_.empty()) return false;
    const uint64_t mask = keys_.size() - 1;
    for (uint64_t i = fo_mix64(k) & mask;; i = (i + 1) & mask) {
      if (keys_[i] == EMPTY) return false;
      if (keys_[i] == k) {
        keys_[i] = TOMB;
        --size_;
        return true;
      }
    }
  }
  uint64_t size() const { return size_; }

 private:
  static constexpr uint64_t EMPTY = ~0ull, TOMB = ~0ull - 1;
  void rehash(uint64_t cap) {
    std::vector<uint64_t> old;
    old.swap(keys_);
    keys_.assign(cap, EMPTY);
    used_ = size_ = 0;
    const uint64_t mask = cap - 1;
    for (uint64_t k : old) {
      if (k == EMPTY || k == TOMB) continue;
      uint64_t i = fo_mix64(k) & mask;
      while (keys_[i] != EMPTY) i = (i + 1) & mask;
      keys_[i] = k;
      ++used_;
      ++size_;
    }
  }
  std::vector<uint64_t> keys_;
  uint64_t used_ = 0, size_ = 0;  // used_ counts tombstones too
};

// u64 -> u32 map without deletion (group slots are persistent).
class U64Map {
 public:
  uint32_t find(uint64_t k) const {
    if (keys_.empty()) return SUB_NONE;
    const uint64_t mask = keys_.size() - 1;
    for (uint64_t i = fo_mix64(k) & mask;; i = (i + 1) & mask) {
      if (vals_[i] == SUB_NONE) return SUB_NONE;
      if (keys_[i] == k) return vals_[i];
    }
  }
  void insert_new(uint64_t k, uint32_t v) {
    if ((size_ + 1) * 4 >= keys_.size() * 3) grow();
    const uint64_t mask = keys_.size() - 1;
    uint64_t i = fo_mix64(k) & mask;
    while (vals_[i] != SUB_NONE) i = (i + 1) & mask;
    keys_[i] = k;
    vals_[i] = v;
    ++size_;
  }

 private:
  void grow() {
    const uint64_t cap = std::max<uint64_t>(1024, keys_.size() * 2);
    std::vector<uint64_t> ok;
    std::vector<uint32_t> ov;
    ok.swap(keys_);
    ov.swap(vals_);
    keys_.assign(cap, 0);
    vals_.assign(cap, SUB_NONE);
    size_ = 0;
    for (uint64_t i = 0; i < ok.size(); ++i)
      if (ov[i] != SUB_NONE) insert_new(ok[i], ov[i]);
  }
  std::vector<uint64_t> keys_;
  std::vector<uint32_t> vals_;
  uint64_t size_ = 0;
};

template <class T>
void fo_free(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

template <class T>
hipError_t fo_alloc(T*& p, uint64_t count) {
  fo_free(p);
  return hipMalloc(reinterpret_cast<void**>(&p), std::max<uint64_t>(count, 1) * sizeof(T));
}

template <class T>
hipError_t fo_ensure(T*& p, uint64_t& cap, uint64_t need) {
  if (need <= cap && p) return hipSuccess;
  uint64_t c = 1024;
  while (c < need) c <<= 1;
  hipError_t e = fo_alloc(p, c);
  cap = e == hipSuccess ? c : 0;
  return e;
}

struct Slot {
  uint32_t filter, group;
  std::vector<uint32_t> members;  // subscription order
  bool changed = false;
};

struct DevTables {
  FilterRec* recs = nullptr;
  uint32_t* plain = nullptr;
  GroupRec* groups = nullptr;
  uint32_t* members = nullptr;
  uint32_t n_recs = 0;
  uint64_t bytes = 0;
  void release() {
    fo_free(recs);
    fo_free(plain);
    fo_free(groups);
    fo_free(members);
  }
};

}  // namespace

// Per-stream scratch of the fan-out pipeline: calls on one stream run in order on the device,
// so they can share it; calls pipelined on different streams never do.
struct FoScratch {
  hipStream_t stream = nullptr;
  uint32_t* entry_topic = nullptr;
  uint64_t cap_entry_topic = 0;
  uint32_t* ecount = nullptr;
  uint64_t cap_ecount = 0;
  uint64_t* eoff = nullptr;
  uint64_t cap_eoff = 0;
  uint64_t* partials = nullptr;
  uint64_t cap_partials = 0;
  uint64_t* h_sum = nullptr;  // host-mapped call summary (synchronous calls)
  void release() {
    fo_free(entry_topic);
    fo_free(ecount);
    fo_free(eoff);
    fo_free(partials);
    if (h_sum) (void)hipHostFree(h_sum);
    h_sum = nullptr;
  }
};

struct emqx_subtab {
  int device = 0;
  std::mutex mu;  // serialises mutations, commits and fan-out calls
  // host store
  std::vector<std::vector<uint32_t>> plain;   // filter id -> plain subscribers
  U64Set plain_set;                            // (filter << 32) | sub
  U64Map slot_of;                              // (filter << 32) | group -> slot
  std::vector<Slot> slots;
  std::vector<std::vector<uint32_t>> fslots;   // filter id -> its slots (creation order)
  U64Set member_set;                           // (slot << 32) | sub
  uint64_t n_members = 0;
  // device
  DevTables dev;
  GroupState* state = nullptr;
  uint64_t state_cap = 0;
  uint64_t state_n = 0;                        // slots with device state
  uint64_t n_live_groups = 0;
  hipStream_t stream = nullptr;
  std::vector<std::unique_ptr<FoScratch>> scratch;  // one per stream that called
  uint64_t* h_total = nullptr;
  uint32_t seed = 0x2545F491u;
  // emqx_publish_batch staging
  uint8_t* d_tbytes = nullptr;
  uint64_t cap_tbytes = 0;
  uint64_t* d_toffs = nullptr;
  uint64_t cap_toffs = 0;
  uint64_t* d_moff = nullptr;
  uint64_t cap_moff = 0;
  uint32_t* d_mids = nullptr;
  uint64_t cap_mids = 0;
  uint32_t* d_keys = nullptr;
  uint64_t cap_keys = 0;
  uint64_t* d_ooff = nullptr;
  uint64_t cap_ooff = 0;
  uint32_t* d_osubs = nullptr;
  uint64_t cap_osubs = 0;
  uint32_t* d_ofil = nullptr;
  uint64_t cap_ofil = 0;

  ~emqx_subtab() {
    (void)hipSetDevice(device);
    dev.release();
    fo_free(state);
    for (auto& c : scratch) c->release();
    fo_free(d_tbytes);
    fo_free(d_toffs);
    fo_free(d_moff);
    fo_free(d_mids);
    fo_free(d_keys);
    fo_free(d_ooff);
    fo_free(d_osubs);
    fo_free(d_ofil);
    if (h_total) (void)hipHostFree(h_total);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

namespace {

bool ids_ok(const uint32_t* f, const uint32_t* s, uint64_t n) {
  if (n && (!f || !s)) return false;
  for (uint64_t i = 0; i < n; ++i)
    if (f[i] & FANOUT_SHARED_BIT || s[i] == SUB_NONE) return false;
  return true;
}

int commit_locked(emqx_subtab* s) {
  FO_TRY(hipSetDevice(s->device));
  // ---- host build -----------------------------------------------------------------
  const uint64_t nf = std::max(s->plain.size(), s->fslots.size());
  if (nf >= FANOUT_SHARED_BIT) return EMQX_EINVAL;
  std::vector<FilterRec> recs(nf);
  std::vector<uint32_t> plain, members;
  std::vector<GroupRec> groups;
  plain.reserve(s->plain_set.size());
  members.reserve(s->n_members);
  uint64_t live_groups = 0;
  for (uint64_t f = 0; f < nf; ++f) {
    FilterRec r{static_cast<uint32_t>(plain.size()), 0, static_cast<uint32_t>(groups.size()), 0};
    if (f < s->plain.size()) {
      const auto& v = s->plain[f];
      plain.insert(plain.end(), v.begin(), v.end());
      r.n_plain = static_cast<uint32_t>(v.size());
    }
    if (f < s->fslots.size()) {
      for (uint32_t sl : s->fslots[f]) {
        const Slot& slot = s->slots[sl];
        if (slot.members.empty()) continue;  // no members -> no {Group, node()} route
        groups.push_back(GroupRec{static_cast<uint32_t>(members.size()), static_cast<uint32_t>(slot.members.size()),
                                  sl, slot.group});
        members.insert(members.end(), slot.members.begin(), slot.members.end());
        ++live_groups;
      }
      r.n_groups = static_cast<uint32_t>(groups.size()) - r.group_begin;
    }
    recs[f] = r;
  }
  if (plain.size() >= (1ull << 32) || members.size() >= (1ull << 32) || groups.size() >= (1ull << 32))
    return EMQX_ENOMEM;

  // ---- pick state: keep counters, drop sticky picks of members that left ------------
  const uint64_t nslots = s->slots.size();
  std::vector<GroupState> st(nslots, GroupState{0, SUB_NONE});
  if (s->state_n) FO_TRY(hipMemcpy(st.data(), s->state, s->state_n * sizeof(GroupState), hipMemcpyDeviceToHost));
  for (uint64_t i = 0; i < nslots; ++i) {
    Slot& sl = s->slots[i];
    if (sl.changed && st[i].sticky != SUB_NONE && !s->member_set.contains((i << 32) | st[i].sticky))
      st[i].sticky = SUB_NONE;
    sl.changed = false;
  }

  // ---- upload (the old tables are released after the new ones are in place) ---------
  DevTables d;
  auto up = [&](auto*& p, const auto& v) -> hipError_t {
    hipError_t e = fo_alloc(p, v.size());
    if (e == hipSuccess && !v.empty()) e = hipMemcpy(p, v.data(), v.size() * sizeof(v[0]), hipMemcpyHostToDevice);
    return e;
  };
  if (up(d.recs, recs) != hipSuccess || up(d.plain, plain) != hipSuccess || up(d.groups, groups) != hipSuccess ||
      up(d.members, members) != hipSuccess) {
    d.release();
    return EMQX_ENOMEM;
  }
  d.n_recs = static_cast<uint32_t>(nf);
  d.bytes = recs.size() * sizeof(FilterRec) + plain.size() * 4 + groups.size() * sizeof(GroupRec) + members.size() * 4;
  if (nslots > s->state_cap) {
    GroupState* ns = nullptr;
    const uint64_t cap = std::max<uint64_t>(1024, nslots * 2);
    if (fo_alloc(ns, cap) != hipSuccess) {
      d.release();
      return EMQX_ENOMEM;
    }
    fo_free(s->state);
    s->state = ns;
    s->state_cap = cap;
  }
  if (nslots) FO_TRY(hipMemcpy(s->state, st.data(), nslots * sizeof(GroupState), hipMemcpyHostToDevice));
  s->state_n = nslots;
  s->dev.release();
  s->dev = d;
  s->n_live_groups = live_groups;
  return EMQX_OK;
}

// The fan-out pipeline on device buffers (s->mu held).
FoScratch* scratch_for(emqx_subtab* s, hipStream_t st) {
  for (auto& c : s->scratch)
    if (c->stream == st) return c.get();
  s->scratch.push_back(std::make_unique<FoScratch>());
  s->scratch.back()->stream = st;
  return s->scratch.back().get();
}

// Enqueue the fan-out of one match CSR on st, no host synchronisation; m_cap bounds the
// match entries (sizes the scratch); the summary goes to `summary` (FO_SUM_WORDS u64).
int enqueue_fanout(emqx_subtab* s, uint32_t strategy, const uint64_t* d_moff, const uint32_t* d_mids, uint64_t n,
                   uint64_t m_cap, const uint32_t* d_keys, uint64_t* d_out_off, uint32_t* d_out_subs,
                   uint32_t* d_out_fil, uint64_t cap, uint64_t* summary, hipStream_t st) {
  FoScratch* c = scratch_for(s, st);
  const bool hash = strategy == EMQX_SHARE_HASH_CLIENTID || strategy == EMQX_SHARE_HASH_TOPIC;
  if (hash) FO_TRY(fo_ensure(c->entry_topic, c->cap_entry_topic, m_cap));
  FO_TRY(fo_ensure(c->ecount, c->cap_ecount, m_cap));
  FO_TRY(fo_ensure(c->eoff, c->cap_eoff, m_cap + 1));
  FO_TRY(fo_ensure(c->partials, c->cap_partials, 2 * FO_BLOCKS));
  FanoutArgs a{};
  a.recs = s->dev.recs;
  a.n_recs = s->dev.n_recs;
  a.plain = s->dev.plain;
  a.groups = s->dev.groups;
  a.members = s->dev.members;
  a.state = s->state;
  a.moff = d_moff;
  a.mids = d_mids;
  a.n = n;
  a.keys = d_keys;
  a.strategy = strategy;
  s->seed = s->seed * 1664525u + 1013904223u;
  a.seed = s->seed;
  a.entry_topic = c->entry_topic;
  a.ecount = c->ecount;
  a.eoff = c->eoff;
  a.partials = c->partials;
  a.out_off = d_out_off;
  a.out_subs = d_out_subs;
  a.out_filters = d_out_fil;
  a.cap = d_out_subs ? cap : 0;
  a.summary = summary;
  FO_TRY(launch_fanout(a, m_cap, st));
  return EMQX_OK;
}

// Synchronous form: enqueue, drain, read the summary.  On overflow the write kernel wrote
// nothing (and consumed no pick state); *n_out is the capacity required.
int run_fanout(emqx_subtab* s, uint32_t strategy, const uint64_t* d_moff, const uint32_t* d_mids, uint64_t n,
               uint64_t m, const uint32_t* d_keys, uint64_t* d_out_off, uint32_t* d_out_subs, uint32_t* d_out_fil,
               uint64_t cap, uint64_t* n_out, hipStream_t st) {
  FoScratch* c = scratch_for(s, st);
  if (!c->h_sum)
    FO_TRY(hipHostMalloc(reinterpret_cast<void**>(&c->h_sum), FO_SUM_WORDS * sizeof(uint64_t), hipHostMallocDefault));
  uint64_t* d_sum = nullptr;
  FO_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&d_sum), c->h_sum, 0));
  int rc = enqueue_fanout(s, strategy, d_moff, d_mids, n, m, d_keys, d_out_off, d_out_subs, d_out_fil, cap, d_sum, st);
  if (rc != EMQX_OK) return rc;
  FO_TRY(hipStreamSynchronize(st));
  *n_out = c->h_sum[FO_SUM_TOTAL];
  if (c->h_sum[FO_SUM_FLAGS] & FO_SUM_F_OVERFLOW) return EMQX_EOVERFLOW;
  return EMQX_OK;
}

int ensure_stream(emqx_subtab* s) {
  if (!s->stream) {
    FO_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    FO_TRY(hipHostMalloc(reinterpret_cast<void**>(&s->h_total), 2 * sizeof(uint64_t), hipHostMallocDefault));
  }
  return EMQX_OK;
}

bool strategy_ok(uint32_t strategy, bool have_keys) {
  if (strategy > EMQX_SHARE_HASH_TOPIC) return false;
  if ((strategy == EMQX_SHARE_HASH_CLIENTID || strategy == EMQX_SHARE_HASH_TOPIC) && !have_keys) return false;
  return true;
}

}  // namespace

extern "C" {

int emqx_subtab_create(int32_t device, emqx_subtab** out) {
  if (!out) return EMQX_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return EMQX_EDEVICE;
  int dev = device;
  if (dev < 0) (void)hipGetDevice(&dev);
  if (dev >= ndev) return EMQX_EINVAL;
  FO_TRY(hipSetDevice(dev));
  auto* s = new (std::nothrow) emqx_subtab();
  if (!s) return EMQX_ENOMEM;
  s->device = dev;
  int rc = commit_locked(s);
  if (rc == EMQX_OK) rc = ensure_stream(s);
  if (rc != EMQX_OK) {
    delete s;
    return rc;
  }
  *out = s;
  return EMQX_OK;
}

int emqx_subtab_destroy(emqx_subtab* s) {
  if (!s) return EMQX_EINVAL;
  delete s;
  return EMQX_OK;
}

int emqx_subtab_add(emqx_subtab* s, const uint32_t* filter_ids, const uint32_t* sub_ids, const uint32_t* group_ids,
                    uint64_t n) {
  if (!s || !ids_ok(filter_ids, sub_ids, n)) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(s->mu);
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t f = filter_ids[i], sub = sub_ids[i];
    const uint32_t grp = group_ids ? group_ids[i] : EMQX_NO_GROUP;
    if (grp == EMQX_NO_GROUP) {
      if (s->plain_set.insert((uint64_t(f) << 32) | sub)) {
        if (f >= s->plain.size()) s->plain.resize(uint64_t(f) + 1);
        s->plain[f].push_back(sub);
      }
      continue;
    }
    const uint64_t key = (uint64_t(f) << 32) | grp;
    uint32_t sl = s->slot_of.find(key);
    if (sl == SUB_NONE) {
      if (s->slots.size() >= FANOUT_SHARED_BIT) return EMQX_ENOMEM;
      sl = static_cast<uint32_t>(s->slots.size());
      s->slots.push_back(Slot{f, grp, {}, false});
      s->slot_of.insert_new(key, sl);
      if (f >= s->fslots.size()) s->fslots.resize(uint64_t(f) + 1);
      s->fslots[f].push_back(sl);
    }
    if (s->member_set.insert((uint64_t(sl) << 32) | sub)) {
      s->slots[sl].members.push_back(sub);
      s->slots[sl].changed = true;
      ++s->n_members;
    }
  }
  return EMQX_OK;
}

int emqx_subtab_remove(emqx_subtab* s, const uint32_t* filter_ids, const uint32_t* sub_ids, const uint32_t* group_ids,
                       uint64_t n) {
  if (!s || !ids_ok(filter_ids, sub_ids, n)) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(s->mu);
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t f = filter_ids[i], sub = sub_ids[i];
    const uint32_t grp = group_ids ? group_ids[i] : EMQX_NO_GROUP;
    if (grp == EMQX_NO_GROUP) {
      if (s->plain_set.erase((uint64_t(f) << 32) | sub)) {
        auto& v = s->plain[f];
        auto it = std::find(v.begin(), v.end(), sub);
        *it = v.back();  // order of plain subscribers carries no meaning
        v.pop_back();
      }
      continue;
    }
    const uint32_t sl = s->slot_of.find((uint64_t(f) << 32) | grp);
    if (sl == SUB_NONE) continue;
    if (s->member_set.erase((uint64_t(sl) << 32) | sub)) {
      auto& v = s->slots[sl].members;
      v.erase(std::find(v.begin(), v.end(), sub));  // keeps the others' order (ETS bag)
      s->slots[sl].changed = true;
      --s->n_members;
    }
  }
  return EMQX_OK;
}

int emqx_subtab_commit(emqx_subtab* s) {
  if (!s) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(s->mu);
  return commit_locked(s);
}

int emqx_subtab_stats(emqx_subtab* s, uint64_t* counts4) {
  if (!s || !counts4) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(s->mu);
  counts4[0] = s->plain_set.size();
  counts4[1] = s->n_members;
  counts4[2] = s->n_live_groups;
  counts4[3] = s->dev.bytes;
  return EMQX_OK;
}

int emqx_fanout_batch_device(emqx_subtab* s, uint32_t strategy, const uint64_t* d_match_offsets,
                             const uint32_t* d_match_ids, uint64_t n, const uint32_t* d_pick_keys,
                             uint64_t* d_out_offsets, uint32_t* d_out_subs, uint32_t* d_out_filters, uint64_t cap,
                             uint64_t* n_out, void* stream) {
  if (!s || !n_out || !d_match_offsets || !d_out_offsets || !strategy_ok(strategy, d_pick_keys != nullptr))
    return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(s->mu);
  FO_TRY(hipSetDevice(s->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : s->stream;
  if (!stream) FO_TRY(after_null_stream(st));
  // the number of match entries: one small readback of the CSR bounds
  uint64_t bounds[2] = {0, 0};
  FO_TRY(hipMemcpyAsync(s->h_total, d_match_offsets, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  FO_TRY(hipMemcpyAsync(s->h_total + 1, d_match_offsets + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  FO_TRY(hipStreamSynchronize(st));
  bounds[0] = s->h_total[0];
  bounds[1] = s->h_total[1];
  if (bounds[1] < bounds[0]) return EMQX_EINVAL;
  if (bounds[1] - bounds[0] && !d_match_ids) return EMQX_EINVAL;
  return run_fanout(s, strategy, d_match_offsets, d_match_ids, n, bounds[1] - bounds[0], d_pick_keys,
                    d_out_offsets, d_out_subs, d_out_filters, cap, n_out, st);
}

int emqx_fanout_batch_device_async(emqx_subtab* s, uint32_t strategy, const uint64_t* d_match_offsets,
                                   const uint32_t* d_match_ids, uint64_t n, uint64_t match_cap,
                                   const uint32_t* d_pick_keys, uint64_t* d_out_offsets, uint32_t* d_out_subs,
                                   uint32_t* d_out_filters, uint64_t cap, uint64_t* summary, void* stream) {
  if (!s || !summary || !d_match_offsets || !d_match_ids || !d_out_offsets || !d_out_subs ||
      !strategy_ok(strategy, d_pick_keys != nullptr))
    return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(s->mu);
  FO_TRY(hipSetDevice(s->device));
  hipStream_t st = stream ? static_cast<hipStream_t>(stream) : s->stream;
  if (!stream) FO_TRY(after_null_stream(st));
  return enqueue_fanout(s, strategy, d_match_offsets, d_match_ids, n, match_cap, d_pick_keys, d_out_offsets,
                        d_out_subs, d_out_filters, cap, summary, st);
}

int emqx_publish_batch(emqx_engine* e, emqx_subtab* s, uint32_t strategy, const uint8_t* topic_bytes,
                       const uint64_t* topic_offsets, uint64_t n, const uint32_t* pick_keys, uint64_t* out_offsets,
                       uint32_t* out_subs, uint32_t* out_filters, uint64_t cap, uint64_t* n_out) {
  if (!e || !s || !n_out || !out_offsets || (n && !topic_offsets) || !strategy_ok(strategy, pick_keys != nullptr))
    return EMQX_EINVAL;
  for (uint64_t i = 0; i < n; ++i)
    if (topic_offsets[i + 1] < topic_offsets[i]) return EMQX_EINVAL;
  const uint64_t b0 = n ? topic_offsets[0] : 0, b1 = n ? topic_offsets[n] : 0;
  if (b1 > b0 && !topic_bytes) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(s->mu);
  FO_TRY(hipSetDevice(s->device));
  hipStream_t st = s->stream;
  // stage topics (rebased, padded) and keys
  FO_TRY(fo_ensure(s->d_tbytes, s->cap_tbytes, b1 - b0 + 16));
  FO_TRY(fo_ensure(s->d_toffs, s->cap_toffs, n + 1));
  FO_TRY(fo_ensure(s->d_moff, s->cap_moff, n + 1));
  FO_TRY(fo_ensure(s->d_ooff, s->cap_ooff, n + 1));
  std::vector<uint64_t> rebased(n + 1, 0);
  for (uint64_t i = 0; i <= n && n; ++i) rebased[i] = topic_offsets[i] - b0;
  if (b1 > b0) FO_TRY(hipMemcpyAsync(s->d_tbytes, topic_bytes + b0, b1 - b0, hipMemcpyHostToDevice, st));
  FO_TRY(hipMemcpyAsync(s->d_toffs, rebased.data(), (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  const uint32_t* d_keys = nullptr;
  if (pick_keys && n) {
    FO_TRY(fo_ensure(s->d_keys, s->cap_keys, n));
    FO_TRY(hipMemcpyAsync(s->d_keys, pick_keys, n * sizeof(uint32_t), hipMemcpyHostToDevice, st));
    d_keys = s->d_keys;
  }
  FO_TRY(hipStreamSynchronize(st));
  // match -> CSR in HBM (grow the id buffer once if needed)
  uint64_t m = 0;
  if (!s->d_mids) FO_TRY(fo_ensure(s->d_mids, s->cap_mids, 16 * n + 1024));
  int rc = emqx_match_batch_device(e, EMQX_MODE_ROUTES, s->d_tbytes, s->d_toffs, n, s->d_moff, s->d_mids,
                                   s->cap_mids, &m, st);
  if (rc == EMQX_EOVERFLOW) {
    FO_TRY(fo_ensure(s->d_mids, s->cap_mids, m));
    rc = emqx_match_batch_device(e, EMQX_MODE_ROUTES, s->d_tbytes, s->d_toffs, n, s->d_moff, s->d_mids,
                                 s->cap_mids, &m, st);
  }
  if (rc != EMQX_OK) return rc;
  // fan-out into the staging buffers; an overflow returns before the write kernel (no pick
  // state consumed), so the buffers grow once and the call repeats
  uint64_t total = 0;
  for (int attempt = 0; attempt < 2; ++attempt) {
    FO_TRY(fo_ensure(s->d_osubs, s->cap_osubs, 1));
    FO_TRY(fo_ensure(s->d_ofil, s->cap_ofil, s->cap_osubs));
    rc = run_fanout(s, strategy, s->d_moff, s->d_mids, n, m, d_keys, s->d_ooff, s->d_osubs, s->d_ofil,
                    s->cap_osubs, &total, st);
    if (rc != EMQX_EOVERFLOW) break;
    *n_out = total;
    if (total > cap) return EMQX_EOVERFLOW;
    FO_TRY(fo_ensure(s->d_osubs, s->cap_osubs, total));
  }
  if (rc != EMQX_OK) return rc;
  *n_out = total;
  if (total > cap) return EMQX_EOVERFLOW;
  FO_TRY(hipMemcpyAsync(out_offsets, s->d_ooff, (n + 1) * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  if (total && out_subs) FO_TRY(hipMemcpyAsync(out_subs, s->d_osubs, total * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  if (total && out_filters)
    FO_TRY(hipMemcpyAsync(out_filters, s->d_ofil, total * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
  FO_TRY(hipStreamSynchronize(st));
  return EMQX_OK;
}

}  // extern "C"
