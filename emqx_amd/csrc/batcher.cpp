// Cross-caller batchers (include/emqx_match.h, emqx_batcher_* and emqx_pub_batcher_*).
//
// emqx_router:match_routes/1 and emqx_broker:publish/1 are called once per PUBLISH by each
// publisher's own process (apps/emqx/src/emqx_broker.erl:203-214).  Many concurrent
// single-message calls are coalesced here into device batches: a caller's topic is copied
// straight into the pinned input buffer of the batch being filled (emqx_host_batch for matches,
// emqx_pub_batch for match + fan-out) and submit() returns at once.
//
// Two threads drive the batches, so that two are in flight while a third fills:
//   * the dispatcher submits a batch when it holds `max_batch` messages, or `max_wait_us` after
//     its first one, as long as fewer than two batches are in flight — or at once when nothing
//     is in flight (an idle device serves a lone PUBLISH without waiting);
//   * the completer waits for the oldest batch in flight and calls the callback for each of
//     its messages (results point into the batch's pinned output, valid during the call), then
//     frees the buffer.
// The Erlang NIF's callback enif_send()s the results to the waiting process, so the Erlang call
// shape stays synchronous while the GPU sees batches.  With every buffer busy, submit() blocks
// until one frees (backpressure instead of unbounded queues) and try_submit() returns
// EMQX_EBUSY instead, so that a NIF running on a normal scheduler never waits on the device.
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/emqx_match.h"

namespace {

using Clock = std::chrono::steady_clock;
constexpr int NBUF = 4;          // two in flight, one filling, one ready
constexpr int MAX_INFLIGHT = 2;

// Match batches: emqx_host_batch, results = filter ids per topic.
struct MatchPolicy {
  using HB = emqx_host_batch;
  emqx_engine* e = nullptr;
  uint32_t mode = EMQX_MODE_ROUTES;
  emqx_batch_cb cb = nullptr;
  int create(uint32_t max_batch, HB** out) const {
    // ~48 B per topic and 32 ids per topic to start with; both grow on demand
    return emqx_host_batch_create(e, max_batch, std::max<uint64_t>(48ull * max_batch, 1u << 16),
                                  std::max<uint64_t>(32ull * max_batch, 1u << 16), out);
  }
  static void destroy(HB* b) { emqx_host_batch_destroy(b); }
  static int reserve_bytes(HB* b, uint64_t bytes) { return emqx_host_batch_reserve(b, b->cap_topics, bytes, b->cap_ids); }
  static void put_key(HB*, uint64_t, uint32_t) {}
  int submit(HB* b) const { return emqx_host_batch_submit(b, mode); }
  int wait(HB* b) const {
    int rc = emqx_host_batch_wait(b);
    if (rc == EMQX_EOVERFLOW) {  // more ids than the buffer holds: grow it, rerun the batch
      rc = emqx_host_batch_reserve(b, b->cap_topics, b->cap_bytes, b->n_out + (b->n_out >> 1) + 1024);
      if (rc == EMQX_OK) rc = emqx_host_batch_submit(b, mode);
      if (rc == EMQX_OK) rc = emqx_host_batch_wait(b);
    }
    return rc;
  }
  void done(HB* b, uint64_t i, int rc, void* ctx) const {
    if (rc == EMQX_OK)
      cb(ctx, rc, b->out_ids + b->out_offsets[i], b->out_offsets[i + 1] - b->out_offsets[i]);
    else
      cb(ctx, rc, nullptr, 0);
  }
};

// Publish batches: emqx_pub_batch, results = deliveries (subscriber, filter) per message.
struct PublishPolicy {
  using HB = emqx_pub_batch;
  emqx_engine* e = nullptr;
  emqx_subtab* s = nullptr;
  uint32_t strategy = EMQX_SHARE_RANDOM;
  emqx_pub_cb cb = nullptr;
  int create(uint32_t max_batch, HB** out) const {
    return emqx_pub_batch_create(e, s, strategy, max_batch, std::max<uint64_t>(48ull * max_batch, 1u << 16),
                                 std::max<uint64_t>(64ull * max_batch, 1u << 16), out);
  }
  static void destroy(HB* b) { emqx_pub_batch_destroy(b); }
  static int reserve_bytes(HB* b, uint64_t bytes) { return emqx_pub_batch_reserve(b, b->cap_topics, bytes, b->cap_out); }
  static void put_key(HB* b, uint64_t i, uint32_t key) { b->keys[i] = key; }
  int submit(HB* b) const { return emqx_pub_batch_submit(b); }
  int wait(HB* b) const {
    int rc = emqx_pub_batch_wait(b);
    if (rc == EMQX_EOVERFLOW) {  // nothing delivered, no pick state used: grow and rerun
      rc = emqx_pub_batch_reserve(b, b->cap_topics, b->cap_bytes, b->n_out + (b->n_out >> 1) + 1024);
      if (rc == EMQX_OK) rc = emqx_pub_batch_submit(b);
      if (rc == EMQX_OK) rc = emqx_pub_batch_wait(b);
    }
    return rc;
  }
  void done(HB* b, uint64_t i, int rc, void* ctx) const {
    if (rc == EMQX_OK) {
      const uint64_t o = b->out_offsets[i];
      cb(ctx, rc, b->out_subs + o, b->out_filters + o, b->out_offsets[i + 1] - o);
    } else {
      cb(ctx, rc, nullptr, nullptr, 0);
    }
  }
};

template <class P>
struct BatcherCore {
  using HB = typename P::HB;
  struct Buf {
    HB* hb = nullptr;
    std::vector<void*> ctx;
    Clock::time_point t0;
    uint64_t bytes = 0;
  };

  P pol;
  uint32_t max_batch = 4096;
  uint32_t max_wait_us = 200;
  std::mutex mu;
  std::condition_variable cv;   // any state change
  Buf buf[NBUF];
  std::vector<int> free_;       // buffer indices
  int filling = -1;
  std::deque<int> ready, inflight;
  bool stop = false;
  bool dispatcher_done = false;
  std::thread dispatcher, completer;
  uint64_t n_batches = 0, n_topics = 0, max_inflight_seen = 0;
  uint64_t ns_wait = 0, ns_callbacks = 0, ns_submit = 0;  // completer waiting / in callbacks; dispatcher submitting

  int start() {
    for (int k = 0; k < NBUF; ++k) {
      int rc = pol.create(max_batch, &buf[k].hb);
      if (rc != EMQX_OK) {
        for (int j = 0; j < k; ++j) P::destroy(buf[j].hb);
        return rc;
      }
      buf[k].hb->topic_offsets[0] = 0;
      buf[k].hb->n = 0;
      free_.push_back(k);
    }
    dispatcher = std::thread([this] {
      dispatch_loop();
      std::lock_guard<std::mutex> g(mu);
      dispatcher_done = true;
      cv.notify_all();
    });
    completer = std::thread([this] { complete_loop(); });
    return EMQX_OK;
  }

  void shutdown() {
    {
      std::lock_guard<std::mutex> g(mu);
      stop = true;
    }
    cv.notify_all();
    if (dispatcher.joinable()) dispatcher.join();  // pending submissions are dispatched
    if (completer.joinable()) completer.join();    // and completed first
    for (int k = 0; k < NBUF; ++k) P::destroy(buf[k].hb);
  }

  bool filling_empty() const { return filling < 0 || buf[filling].ctx.empty(); }

  // Takes the filling buffer out of the filling state (caller holds mu).
  void seal() {
    if (filling >= 0 && !buf[filling].ctx.empty()) ready.push_back(filling);
    else if (filling >= 0) free_.push_back(filling);
    filling = -1;
  }

  void dispatch_loop() {
    std::unique_lock<std::mutex> lk(mu);
    while (true) {
      // a sealed batch, or the filling one once its deadline passed, and room in flight
      while (true) {
        // an idle device takes what is there at once (latency); a busy one lets the batch grow
        // to max_batch or until max_wait_us after its first message (throughput)
        if (ready.empty() && !filling_empty() &&
            (stop || inflight.empty() || Clock::now() >= buf[filling].t0 + std::chrono::microseconds(max_wait_us)))
          seal();
        if (!ready.empty() && static_cast<int>(inflight.size()) < MAX_INFLIGHT) break;
        if (stop && ready.empty() && filling_empty()) return;
        if (ready.empty() && !filling_empty() && static_cast<int>(inflight.size()) < MAX_INFLIGHT)
          cv.wait_until(lk, buf[filling].t0 + std::chrono::microseconds(max_wait_us));
        else
          cv.wait(lk);
      }
      const int k = ready.front();
      ready.pop_front();
      lk.unlock();
      const auto ts = Clock::now();
      int rc = pol.submit(buf[k].hb);
      const uint64_t dts = std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - ts).count();
      lk.lock();
      ns_submit += dts;
      if (rc != EMQX_OK) {  // report the failure to every caller of the batch
        lk.unlock();
        for (size_t i = 0; i < buf[k].ctx.size(); ++i) pol.done(buf[k].hb, i, rc, buf[k].ctx[i]);
        lk.lock();
        recycle(k);
        continue;
      }
      inflight.push_back(k);
      max_inflight_seen = std::max<uint64_t>(max_inflight_seen, inflight.size());
      cv.notify_all();
    }
  }

  void complete_loop() {
    std::unique_lock<std::mutex> lk(mu);
    while (true) {
      cv.wait(lk, [&] { return !inflight.empty() || (stop && ready.empty() && filling_empty() && dispatcher_done); });
      if (inflight.empty()) return;
      const int k = inflight.front();
      lk.unlock();
      HB* b = buf[k].hb;
      const auto tw = Clock::now();
      const int rc = pol.wait(b);
      const auto tc = Clock::now();
      const std::vector<void*>& ctx = buf[k].ctx;
      for (size_t i = 0; i < ctx.size(); ++i) pol.done(b, i, rc, ctx[i]);
      const auto te = Clock::now();
      lk.lock();
      ns_wait += std::chrono::duration_cast<std::chrono::nanoseconds>(tc - tw).count();
      ns_callbacks += std::chrono::duration_cast<std::chrono::nanoseconds>(te - tc).count();
      inflight.pop_front();
      n_batches += 1;
      n_topics += ctx.size();
      recycle(k);
    }
  }

  void recycle(int k) {  // caller holds mu
    buf[k].ctx.clear();
    buf[k].bytes = 0;
    buf[k].hb->n = 0;
    free_.push_back(k);
    cv.notify_all();
  }

  // One message into the filling buffer (the caller holds mu through lk).  may_wait = false:
  // EMQX_EBUSY instead of waiting for a buffer or growing one.
  int submit_locked(std::unique_lock<std::mutex>& lk, const uint8_t* topic, uint64_t len, uint32_t key, void* ctx,
                    bool may_wait) {
    while (true) {
      if (stop) return EMQX_EINVAL;
      if (filling < 0) {
        if (free_.empty()) {  // every buffer filling, sealed or in flight: wait for one
          if (!may_wait) return EMQX_EBUSY;
          cv.wait(lk);
          continue;
        }
        filling = free_.back();
        free_.pop_back();
        Buf& f = buf[filling];
        f.ctx.clear();
        f.bytes = 0;
        f.hb->n = 0;
        f.hb->topic_offsets[0] = 0;
      }
      Buf& f = buf[filling];
      HB* hb = f.hb;
      if (f.bytes + len > hb->cap_bytes) {
        if (f.ctx.empty()) {  // a topic larger than the buffer: grow it
          if (!may_wait) return EMQX_EBUSY;
          const int rc = P::reserve_bytes(hb, len + (len >> 1) + 64);
          if (rc != EMQX_OK) {  // give the (empty) buffer back: nothing is left filling
            free_.push_back(filling);
            filling = -1;
            cv.notify_all();
            return rc;
          }
        } else {
          seal();
          cv.notify_all();
          continue;
        }
      }
      if (len) std::memcpy(hb->topic_bytes + f.bytes, topic, len);
      P::put_key(hb, hb->n, key);
      f.bytes += len;
      hb->n += 1;
      hb->topic_offsets[hb->n] = f.bytes;
      f.ctx.push_back(ctx);
      if (f.ctx.size() == 1) f.t0 = Clock::now();
      if (f.ctx.size() >= max_batch) seal();
      if (f.ctx.size() == 1 || filling < 0) cv.notify_all();
      return EMQX_OK;
    }
  }

  int submit(const uint8_t* topic, uint64_t len, uint32_t key, void* ctx, bool may_wait) {
    if (len && !topic) return EMQX_EINVAL;
    std::unique_lock<std::mutex> lk(mu);
    return submit_locked(lk, topic, len, key, ctx, may_wait);
  }

  int submit_many(const uint8_t* bytes, const uint64_t* offsets, const uint32_t* keys, uint64_t n, void* const* ctxs) {
    if (n && (!offsets || !ctxs)) return EMQX_EINVAL;
    std::unique_lock<std::mutex> lk(mu);
    for (uint64_t i = 0; i < n; ++i) {
      const uint64_t len = offsets[i + 1] - offsets[i];
      if (len && !bytes) return EMQX_EINVAL;
      const int rc = submit_locked(lk, bytes + offsets[i], len, keys ? keys[i] : 0u, ctxs[i], true);
      if (rc != EMQX_OK) return rc;
    }
    return EMQX_OK;
  }

  void stats(uint64_t* out, uint32_t n) {
    std::lock_guard<std::mutex> g(mu);
    const uint64_t v[6] = {n_batches, n_topics, max_inflight_seen, ns_wait, ns_callbacks, ns_submit};
    for (uint32_t i = 0; i < n && i < 6; ++i) out[i] = v[i];
  }
};

}  // namespace

struct emqx_batcher : BatcherCore<MatchPolicy> {};
struct emqx_pub_batcher : BatcherCore<PublishPolicy> {};

extern "C" {

int emqx_batcher_create(emqx_engine* e, uint32_t mode, uint32_t max_batch, uint32_t max_wait_us, emqx_batch_cb cb,
                        emqx_batcher** out) {
  if (!e || !cb || !out || mode > EMQX_MODE_TRIE_WILDCARD || max_batch == 0) return EMQX_EINVAL;
  auto* b = new (std::nothrow) emqx_batcher();
  if (!b) return EMQX_ENOMEM;
  b->pol.e = e;
  b->pol.mode = mode;
  b->pol.cb = cb;
  b->max_batch = max_batch;
  b->max_wait_us = max_wait_us;
  const int rc = b->start();
  if (rc != EMQX_OK) {
    delete b;
    return rc;
  }
  *out = b;
  return EMQX_OK;
}

int emqx_batcher_submit(emqx_batcher* b, const uint8_t* topic, uint64_t len, void* ctx) {
  if (!b) return EMQX_EINVAL;
  return b->submit(topic, len, 0, ctx, true);
}

int emqx_batcher_try_submit(emqx_batcher* b, const uint8_t* topic, uint64_t len, void* ctx) {
  if (!b) return EMQX_EINVAL;
  return b->submit(topic, len, 0, ctx, false);
}

int emqx_batcher_submit_many(emqx_batcher* b, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                             void* const* ctxs) {
  if (!b) return EMQX_EINVAL;
  return b->submit_many(bytes, offsets, nullptr, n, ctxs);
}

int emqx_batcher_destroy(emqx_batcher* b) {
  if (!b) return EMQX_EINVAL;
  b->shutdown();
  delete b;
  return EMQX_OK;
}

int emqx_batcher_stats(emqx_batcher* b, uint64_t* n_batches, uint64_t* n_topics) {
  if (!b) return EMQX_EINVAL;
  uint64_t v[2];
  b->stats(v, 2);
  if (n_batches) *n_batches = v[0];
  if (n_topics) *n_topics = v[1];
  return EMQX_OK;
}

int emqx_batcher_stats_ext(emqx_batcher* b, uint64_t* out, uint32_t n) {
  if (!b || (n && !out)) return EMQX_EINVAL;
  b->stats(out, n);
  return EMQX_OK;
}

int emqx_pub_batcher_create(emqx_engine* e, emqx_subtab* s, uint32_t strategy, uint32_t max_batch,
                            uint32_t max_wait_us, emqx_pub_cb cb, emqx_pub_batcher** out) {
  if (!e || !s || !cb || !out || strategy > EMQX_SHARE_HASH_TOPIC || max_batch == 0) return EMQX_EINVAL;
  auto* b = new (std::nothrow) emqx_pub_batcher();
  if (!b) return EMQX_ENOMEM;
  b->pol.e = e;
  b->pol.s = s;
  b->pol.strategy = strategy;
  b->pol.cb = cb;
  b->max_batch = max_batch;
  b->max_wait_us = max_wait_us;
  const int rc = b->start();
  if (rc != EMQX_OK) {
    delete b;
    return rc;
  }
  *out = b;
  return EMQX_OK;
}

int emqx_pub_batcher_submit(emqx_pub_batcher* b, const uint8_t* topic, uint64_t len, uint32_t key, void* ctx) {
  if (!b) return EMQX_EINVAL;
  return b->submit(topic, len, key, ctx, true);
}

int emqx_pub_batcher_try_submit(emqx_pub_batcher* b, const uint8_t* topic, uint64_t len, uint32_t key, void* ctx) {
  if (!b) return EMQX_EINVAL;
  return b->submit(topic, len, key, ctx, false);
}

int emqx_pub_batcher_submit_many(emqx_pub_batcher* b, const uint8_t* bytes, const uint64_t* offsets,
                                 const uint32_t* keys, uint64_t n, void* const* ctxs) {
  if (!b) return EMQX_EINVAL;
  return b->submit_many(bytes, offsets, keys, n, ctxs);
}

int emqx_pub_batcher_destroy(emqx_pub_batcher* b) {
  if (!b) return EMQX_EINVAL;
  b->shutdown();
  delete b;
  return EMQX_OK;
}

int emqx_pub_batcher_stats_ext(emqx_pub_batcher* b, uint64_t* out, uint32_t n) {
  if (!b || (n && !out)) return EMQX_EINVAL;
  b->stats(out, n);
  return EMQX_OK;
}

}  // extern "C"
