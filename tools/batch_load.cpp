// Load generator for the cross-caller batcher (bench.py --workload L): `callers` concurrent
// single-topic callers in a closed loop — each submits one topic, waits for its ids, submits
// the next — as EMQX publisher processes call emqx_router:match_routes/1 once per PUBLISH
// (apps/emqx/src/emqx_broker.erl:213).  A few driver threads own the callers (caller c
// belongs to driver c mod D); the batcher's completion callback hands a finished caller back
// to its driver, which records the latency and resubmits its finished callers' next topics
// with one emqx_batcher_submit_many (as a NIF draining a scheduler's queue would).  Throughput and latency
// percentiles over the measured window go to out[] (12 entries).
//
// pub_load does the same through the publish batcher (emqx_pub_batcher_*: match + fan-out per
// message, as emqx_broker:publish/1 is called once per PUBLISH, emqx_broker.erl:203-214), with
// each caller's message key (the phash2 key of the hash strategies, or the caller's own
// publisher handle for round_robin / sticky).
//
// sub_load drives the commit coalescer (emqx_coalescer_*) the same way: each caller in a closed
// loop subscribes to a filter, waits until the commit carrying it has reached the device,
// unsubscribes, waits, ... (emqx_broker:subscribe/3 / unsubscribe/1 per call from each channel,
// emqx_broker.erl:124-195), or, with route_ops, adds a new topic's route and deletes it
// (emqx_router.erl:111-124 -> the trie).  It has its own globals, so a pub_load may run beside it
// (publishes during a subscribe storm).
//
// Built by __graft_entry__.build() into tools/_build/libbatchload.so; the emqx_batcher_*
// symbols resolve against libemqxmatch.so, which the caller has loaded (RTLD_GLOBAL).
#include <stdint.h>
#include <stdio.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "../include/emqx_match.h"

namespace {

using Clock = std::chrono::steady_clock;

struct Driver {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<uint32_t> done;  // callers whose result arrived
  bool waiting = false;
};

struct Load {
  std::vector<Driver> drv;
  std::vector<Clock::time_point> t_sub;  // per caller: submit time of its request in flight
  std::vector<int> status;
  uint32_t D = 1;
};

Load* g_load = nullptr;   // the batcher run in progress (one at a time)
Load* g_sload = nullptr;  // the coalescer run in progress (one at a time, beside a batcher run)

std::atomic<uint64_t> g_deliveries{0};

// ctx = caller index + 1
void on_result(void* ctx, int status, const uint32_t*, uint64_t) {
  Load* L = g_load;
  const uint32_t c = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(ctx) - 1);
  if (status != EMQX_OK) L->status[c] = status;
  Driver& d = L->drv[c % L->D];
  bool wake;
  {
    std::lock_guard<std::mutex> g(d.mu);
    d.done.push_back(c);
    wake = d.waiting;
  }
  if (wake) d.cv.notify_one();
}

// coalescer callbacks: the same hand-back as on_result, to g_sload's drivers
void on_change(void* ctx, int status) {
  Load* L = g_sload;
  const uint32_t c = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(ctx) - 1);
  if (status != EMQX_OK) L->status[c] = status;
  Driver& d = L->drv[c % L->D];
  bool wake;
  {
    std::lock_guard<std::mutex> g(d.mu);
    d.done.push_back(c);
    wake = d.waiting;
  }
  if (wake) d.cv.notify_one();
}

void on_publish(void* ctx, int status, const uint32_t*, const uint32_t*, uint64_t n) {
  g_deliveries.fetch_add(n, std::memory_order_relaxed);
  on_result(ctx, status, nullptr, n);
}

// The closed loop shared by both batchers: `submit_one(c, i)` / `submit_batch(cs, is)` hand the
// batcher caller c's next message i.
template <class One, class Many>
int run_load(uint64_t n, uint32_t callers, double warmup_ms, double duration_ms, Load& L, One submit_one,
             Many submit_many, std::vector<std::vector<float>>& lat, std::vector<uint64_t>& completed, double* secs) {
  std::atomic<uint64_t> next{0};
  const auto t_start = Clock::now();
  const auto t_meas = t_start + std::chrono::microseconds(static_cast<int64_t>(warmup_ms * 1e3));
  const auto t_end = t_meas + std::chrono::microseconds(static_cast<int64_t>(duration_ms * 1e3));
  std::atomic<int> err{EMQX_OK};
  std::vector<std::thread> th;
  for (uint32_t d = 0; d < L.D; ++d)
    th.emplace_back([&, d] {
      Driver& me = L.drv[d];
      uint64_t outstanding = 0;
      for (uint32_t c = d; c < callers; c += L.D, ++outstanding) {
        L.t_sub[c] = Clock::now();
        const int r = submit_one(c, next.fetch_add(1) % n);
        if (r != EMQX_OK) err = r;
      }
      std::vector<uint32_t> got, again;
      std::vector<uint64_t> idx;
      while (outstanding) {
        {
          std::unique_lock<std::mutex> lk(me.mu);
          me.waiting = true;
          me.cv.wait(lk, [&] { return !me.done.empty(); });
          me.waiting = false;
          got.swap(me.done);
        }
        const auto now = Clock::now();
        again.clear();
        for (uint32_t c : got) {
          --outstanding;
          if (now >= t_meas && L.t_sub[c] >= t_meas && now < t_end) {
            lat[d].push_back(std::chrono::duration<float, std::micro>(now - L.t_sub[c]).count());
            completed[d] += 1;
          }
          if (now < t_end && err.load() == EMQX_OK) again.push_back(c);
        }
        got.clear();
        if (!again.empty()) {  // the finished callers' next messages, under one batcher lock
          idx.clear();
          const auto ts = Clock::now();
          for (uint32_t c : again) {
            idx.push_back(next.fetch_add(1) % n);
            L.t_sub[c] = ts;
          }
          const int r = submit_many(again, idx);
          if (r != EMQX_OK) err = r;
          outstanding += again.size();
        }
      }
    });
  for (auto& x : th) x.join();
  *secs = std::chrono::duration<double>(std::min(Clock::now(), t_end) - t_meas).count();
  return err.load();
}

void summarize(Load& L, std::vector<std::vector<float>>& lat, std::vector<uint64_t>& completed, double secs,
               const uint64_t* ext, double* out) {
  std::vector<float> all;
  uint64_t done = 0;
  for (uint32_t d = 0; d < L.D; ++d) {
    all.insert(all.end(), lat[d].begin(), lat[d].end());
    done += completed[d];
  }
  std::sort(all.begin(), all.end());
  auto pct = [&](double q) -> double {
    if (all.empty()) return 0;
    return all[std::min<size_t>(all.size() - 1, static_cast<size_t>(q * all.size()))];
  };
  const uint64_t nb = ext[0], nt = ext[1];
  out[0] = static_cast<double>(done);
  out[1] = secs;
  out[2] = pct(0.50);
  out[3] = pct(0.90);
  out[4] = pct(0.99);
  out[5] = all.empty() ? 0 : all.back();
  out[6] = static_cast<double>(nb);
  out[7] = nb ? static_cast<double>(nt) / nb : 0;
  out[8] = static_cast<double>(ext[2]);          // most batches in flight
  out[9] = nb ? ext[3] / 1e3 / nb : 0;           // us per batch: completer waiting for the device
  out[10] = nb ? ext[4] / 1e3 / nb : 0;          // us per batch: callbacks
  out[11] = nb ? ext[5] / 1e3 / nb : 0;          // us per batch: submit
}

}  // namespace

// Publish batcher: out[0..11] as batch_load, out[12] = deliveries per message.
extern "C" int pub_load(emqx_engine* e, emqx_subtab* s, uint32_t strategy, const uint8_t* bytes, const uint64_t* offs,
                        const uint32_t* keys, uint64_t n, uint32_t callers, uint32_t max_batch, uint32_t max_wait_us,
                        double warmup_ms, double duration_ms, double* out) {
  if (!e || !s || !bytes || !offs || !n || !callers || !out) return EMQX_EINVAL;
  Load L;
  L.D = std::min<uint32_t>(callers, 8);
  L.drv = std::vector<Driver>(L.D);
  L.t_sub.resize(callers);
  L.status.assign(callers, EMQX_OK);
  g_load = &L;
  g_deliveries = 0;
  emqx_pub_batcher* b = nullptr;
  int rc = emqx_pub_batcher_create(e, s, strategy, max_batch, max_wait_us, on_publish, &b);
  if (rc != EMQX_OK) return rc;
  // round_robin / sticky: the key is the publisher, i.e. the caller; hash strategies: the
  // message's own phash2 key
  const bool per_caller = strategy == EMQX_SHARE_ROUND_ROBIN || strategy == EMQX_SHARE_STICKY;
  auto key_of = [&](uint32_t c, uint64_t i) -> uint32_t { return per_caller ? c : (keys ? keys[i] : 0u); };
  std::vector<std::vector<float>> lat(L.D);
  std::vector<uint64_t> completed(L.D, 0);
  double secs = 0;
  auto one = [&](uint32_t c, uint64_t i) {
    return emqx_pub_batcher_submit(b, bytes + offs[i], offs[i + 1] - offs[i], key_of(c, i),
                                   reinterpret_cast<void*>(static_cast<uintptr_t>(c) + 1));
  };
  thread_local std::vector<uint8_t> mb;
  thread_local std::vector<uint64_t> mo;
  thread_local std::vector<uint32_t> mk;
  thread_local std::vector<void*> mc;
  auto many = [&](const std::vector<uint32_t>& cs, const std::vector<uint64_t>& is) {
    mb.clear();
    mo.assign(1, 0);
    mk.clear();
    mc.clear();
    for (size_t j = 0; j < cs.size(); ++j) {
      const uint64_t i = is[j];
      mb.insert(mb.end(), bytes + offs[i], bytes + offs[i + 1]);
      mo.push_back(mb.size());
      mk.push_back(key_of(cs[j], i));
      mc.push_back(reinterpret_cast<void*>(static_cast<uintptr_t>(cs[j]) + 1));
    }
    return emqx_pub_batcher_submit_many(b, mb.data(), mo.data(), mk.data(), cs.size(), mc.data());
  };
  const uint64_t before = 0;
  int err = run_load(n, callers, warmup_ms, duration_ms, L, one, many, lat, completed, &secs);
  uint64_t ext[6] = {0, 0, 0, 0, 0, 0};
  emqx_pub_batcher_stats_ext(b, ext, 6);
  emqx_pub_batcher_destroy(b);
  g_load = nullptr;
  summarize(L, lat, completed, secs, ext, out);
  out[12] = ext[1] ? static_cast<double>(g_deliveries.load() - before) / ext[1] : 0;
  for (int st : L.status)
    if (st != EMQX_OK) return st;
  return err;
}

extern "C" int batch_load(emqx_engine* e, uint32_t mode, const uint8_t* bytes, const uint64_t* offs, uint64_t n,
                          uint32_t callers, uint32_t max_batch, uint32_t max_wait_us, double warmup_ms,
                          double duration_ms, double* out) {
  if (!e || !bytes || !offs || !n || !callers || !out) return EMQX_EINVAL;
  Load L;
  L.D = std::min<uint32_t>(callers, 8);
  L.drv = std::vector<Driver>(L.D);
  L.t_sub.resize(callers);
  L.status.assign(callers, EMQX_OK);
  g_load = &L;
  emqx_batcher* b = nullptr;
  int rc = emqx_batcher_create(e, mode, max_batch, max_wait_us, on_result, &b);
  if (rc != EMQX_OK) return rc;
  std::atomic<uint64_t> next{0};
  const auto t_start = Clock::now();
  const auto t_meas = t_start + std::chrono::microseconds(static_cast<int64_t>(warmup_ms * 1e3));
  const auto t_end = t_meas + std::chrono::microseconds(static_cast<int64_t>(duration_ms * 1e3));
  std::vector<std::vector<float>> lat(L.D);
  std::vector<uint64_t> completed(L.D, 0);
  std::atomic<int> err{EMQX_OK};
  auto submit = [&](uint32_t c) {
    const uint64_t i = next.fetch_add(1) % n;
    L.t_sub[c] = Clock::now();
    int r = emqx_batcher_submit(b, bytes + offs[i], offs[i + 1] - offs[i],
                                reinterpret_cast<void*>(static_cast<uintptr_t>(c) + 1));
    if (r != EMQX_OK) err = r;
  };
  std::vector<std::thread> th;
  for (uint32_t d = 0; d < L.D; ++d)
    th.emplace_back([&, d] {
      Driver& me = L.drv[d];
      uint64_t outstanding = 0;
      for (uint32_t c = d; c < callers; c += L.D, ++outstanding) submit(c);
      std::vector<uint32_t> got, again;
      std::vector<uint8_t> mb;
      std::vector<uint64_t> mo;
      std::vector<void*> mc;
      while (outstanding) {
        {
          std::unique_lock<std::mutex> lk(me.mu);
          me.waiting = true;
          me.cv.wait(lk, [&] { return !me.done.empty(); });
          me.waiting = false;
          got.swap(me.done);
        }
        const auto now = Clock::now();
        again.clear();
        for (uint32_t c : got) {
          --outstanding;
          if (now >= t_meas && L.t_sub[c] >= t_meas && now < t_end) {
            lat[d].push_back(std::chrono::duration<float, std::micro>(now - L.t_sub[c]).count());
            completed[d] += 1;
          }
          if (now < t_end && err.load() == EMQX_OK) again.push_back(c);
        }
        got.clear();
        if (!again.empty()) {  // the finished callers' next topics, under one batcher lock
          mb.clear();
          mo.assign(1, 0);
          mc.clear();
          const auto ts = Clock::now();
          for (uint32_t c : again) {
            const uint64_t i = next.fetch_add(1) % n;
            mb.insert(mb.end(), bytes + offs[i], bytes + offs[i + 1]);
            mo.push_back(mb.size());
            mc.push_back(reinterpret_cast<void*>(static_cast<uintptr_t>(c) + 1));
            L.t_sub[c] = ts;
          }
          const int r = emqx_batcher_submit_many(b, mb.data(), mo.data(), again.size(), mc.data());
          if (r != EMQX_OK) err = r;
          outstanding += again.size();
        }
      }
    });
  for (auto& x : th) x.join();
  const double secs = std::chrono::duration<double>(std::min(Clock::now(), t_end) - t_meas).count();
  uint64_t nb = 0, nt = 0, ext[6] = {0, 0, 0, 0, 0, 0};
  emqx_batcher_stats(b, &nb, &nt);
  emqx_batcher_stats_ext(b, ext, 6);
  emqx_batcher_destroy(b);
  g_load = nullptr;
  std::vector<float> all;
  uint64_t done = 0;
  for (uint32_t d = 0; d < L.D; ++d) {
    all.insert(all.end(), lat[d].begin(), lat[d].end());
    done += completed[d];
  }
  std::sort(all.begin(), all.end());
  auto pct = [&](double q) -> double {
    if (all.empty()) return 0;
    return all[std::min<size_t>(all.size() - 1, static_cast<size_t>(q * all.size()))];
  };
  out[0] = static_cast<double>(done);
  out[1] = secs;
  out[2] = pct(0.50);
  out[3] = pct(0.90);
  out[4] = pct(0.99);
  out[5] = all.empty() ? 0 : all.back();
  out[6] = static_cast<double>(nb);
  out[7] = nb ? static_cast<double>(nt) / nb : 0;
  out[8] = static_cast<double>(ext[2]);          // most batches in flight
  out[9] = nb ? ext[3] / 1e3 / nb : 0;           // us per batch: completer waiting for the device
  out[10] = nb ? ext[4] / 1e3 / nb : 0;          // us per batch: callbacks
  out[11] = nb ? ext[5] / 1e3 / nb : 0;          // us per batch: submit
  for (int s : L.status)
    if (s != EMQX_OK) return s;
  return err.load();
}

// Commit coalescer: `callers` closed-loop callers; caller c's ops alternate subscribe / unsubscribe
// of subscriber first_sub + c to a pseudo-random filter id < n_filters (route_ops = 0), or add /
// delete the route of a new filter "storm/<c>/<k>" (route_ops = 1).  out[0..11] as batch_load
// (batches = commits, messages per batch = changes per commit), out[12] = the coalescer's us per
// commit.
extern "C" int sub_load(emqx_engine* e, emqx_subtab* s, uint32_t callers, uint32_t n_filters, uint32_t first_sub,
                        int route_ops, uint32_t max_wait_us, double warmup_ms, double duration_ms, double* out) {
  if (!e || !s || !callers || (!route_ops && !n_filters) || !out) return EMQX_EINVAL;
  Load L;
  L.D = std::min<uint32_t>(callers, 8);
  L.drv = std::vector<Driver>(L.D);
  L.t_sub.resize(callers);
  L.status.assign(callers, EMQX_OK);
  g_sload = &L;
  emqx_coalescer* co = nullptr;
  int rc = emqx_coalescer_create(e, s, max_wait_us, on_change, &co);
  if (rc != EMQX_OK) return rc;
  std::vector<uint64_t> step(callers, 0);   // caller's op count
  std::vector<uint32_t> held(callers, 0);   // filter (or route id) of its live subscription
  auto one = [&](uint32_t c, uint64_t) -> int {
    void* ctx = reinterpret_cast<void*>(static_cast<uintptr_t>(c) + 1);
    const uint64_t k = step[c]++;
    const bool add = (k & 1) == 0;
    if (!route_ops) {
      if (add) {
        uint64_t x = (uint64_t(c) << 32) ^ (k * 0x9E3779B97F4A7C15ull);
        x ^= x >> 31;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 29;
        held[c] = static_cast<uint32_t>(x % n_filters);
      }
      const uint32_t sub = first_sub + c, f = held[c];
      return emqx_coalescer_subscribe(co, &f, &sub, nullptr, 1, add ? 1 : 0, ctx);
    }
    if (add) {
      char name[64];
      const int len = snprintf(name, sizeof(name), "storm/%u/%llu", c, static_cast<unsigned long long>(k));
      const uint64_t offs[2] = {0, static_cast<uint64_t>(len)};
      return emqx_coalescer_insert_filters(co, reinterpret_cast<const uint8_t*>(name), offs, 1, &held[c], ctx);
    }
    return emqx_coalescer_delete_filters(co, &held[c], 1, ctx);
  };
  // a driver's finished callers resubmit under one coalescer lock (subscription ops), as a NIF
  // draining a scheduler's queue would; route ops go one by one
  thread_local std::vector<uint32_t> mf, ms;
  thread_local std::vector<uint8_t> ma;
  thread_local std::vector<void*> mc;
  auto many = [&](const std::vector<uint32_t>& cs, const std::vector<uint64_t>& is) -> int {
    if (route_ops) {
      for (size_t j = 0; j < cs.size(); ++j) {
        const int r = one(cs[j], is[j]);
        if (r != EMQX_OK) return r;
      }
      return EMQX_OK;
    }
    mf.clear();
    ms.clear();
    ma.clear();
    mc.clear();
    for (uint32_t c : cs) {
      const uint64_t k = step[c]++;
      const bool add = (k & 1) == 0;
      if (add) {
        uint64_t x = (uint64_t(c) << 32) ^ (k * 0x9E3779B97F4A7C15ull);
        x ^= x >> 31;
        x *= 0xBF58476D1CE4E5B9ull;
        x ^= x >> 29;
        held[c] = static_cast<uint32_t>(x % n_filters);
      }
      mf.push_back(held[c]);
      ms.push_back(first_sub + c);
      ma.push_back(add ? 1 : 0);
      mc.push_back(reinterpret_cast<void*>(static_cast<uintptr_t>(c) + 1));
    }
    return emqx_coalescer_subscribe_many(co, mf.data(), ms.data(), nullptr, ma.data(), cs.size(), mc.data());
  };
  std::vector<std::vector<float>> lat(L.D);
  std::vector<uint64_t> completed(L.D, 0);
  double secs = 0;
  int err = run_load(1, callers, warmup_ms, duration_ms, L, one, many, lat, completed, &secs);
  emqx_coalescer_flush(co);
  uint64_t cs[6] = {0, 0, 0, 0, 0, 0};
  emqx_coalescer_stats(co, cs, 6);
  emqx_coalescer_destroy(co);
  g_sload = nullptr;
  const uint64_t ext[6] = {cs[0], cs[1], 0, 0, 0, 0};
  summarize(L, lat, completed, secs, ext, out);
  out[12] = cs[0] ? static_cast<double>(cs[3]) / cs[0] : 0;
  for (int st : L.status)
    if (st != EMQX_OK) return st;
  return err;
}
