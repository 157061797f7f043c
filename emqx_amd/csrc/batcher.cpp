// Cross-caller batcher (include/emqx_match.h, emqx_batcher_*).
//
// emqx_router:match_routes/1 is called once per PUBLISH by each publisher's own process
// (apps/emqx/src/emqx_broker.erl:213).  Many concurrent single-topic calls are coalesced here
// into device batches: a caller's topic is copied straight into the pinned input buffer of the
// batch being filled (emqx_host_batch, engine.cpp) and submit() returns at once.
//
// Two threads drive the batches, so that two are in flight while a third fills:
//   * the dispatcher submits a batch when it holds `max_batch` topics, or `max_wait_us` after
//     its first topic, as long as fewer than two batches are in flight — or at once when
//     nothing is in flight (an idle device serves a lone PUBLISH without waiting);
//   * the completer waits for the oldest batch in flight and calls cb(ctx, status, ids, n)
//     for each of its topics (ids point into the batch's pinned output, valid during the
//     call), then frees the buffer.
// The Erlang NIF's callback enif_send()s the ids to the waiting process, so the Erlang call
// shape stays synchronous while the GPU sees batches.  A full set of buffers blocks submit()
// until one frees (backpressure instead of unbounded queues).
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/emqx_match.h"

namespace {

using Clock = std::chrono::steady_clock;
constexpr int NBUF = 4;          // two in flight, one filling, one ready
constexpr int MAX_INFLIGHT = 2;

struct Buf {
  emqx_host_batch* hb = nullptr;
  std::vector<void*> ctx;
  Clock::time_point t0;
  uint64_t bytes = 0;
};

}  // namespace

struct emqx_batcher {
  emqx_engine* e = nullptr;
  uint32_t mode = EMQX_MODE_ROUTES;
  uint32_t max_batch = 4096;
  uint32_t max_wait_us = 200;
  emqx_batch_cb cb = nullptr;
  std::mutex mu;
  std::condition_variable cv;   // any state change
  Buf buf[NBUF];
  std::vector<int> free_;       // buffer indices
  int filling = -1;
  std::deque<int> ready, inflight;
  bool stop = false;
  std::thread dispatcher, completer;
  uint64_t n_batches = 0, n_topics = 0, max_inflight_seen = 0;
  uint64_t ns_wait = 0, ns_callbacks = 0, ns_submit = 0;  // completer waiting / in callbacks; dispatcher submitting

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
        // to max_batch or until max_wait_us after its first topic (throughput)
        if (ready.empty() && filling >= 0 && !buf[filling].ctx.empty() &&
            (stop || inflight.empty() || Clock::now() >= buf[filling].t0 + std::chrono::microseconds(max_wait_us)))
          seal();
        if (!ready.empty() && static_cast<int>(inflight.size()) < MAX_INFLIGHT) break;
        if (stop && ready.empty() && (filling < 0 || buf[filling].ctx.empty())) return;
        if (ready.empty() && filling >= 0 && !buf[filling].ctx.empty() &&
            static_cast<int>(inflight.size()) < MAX_INFLIGHT)
          cv.wait_until(lk, buf[filling].t0 + std::chrono::microseconds(max_wait_us));
        else
          cv.wait(lk);
      }
      const int k = ready.front();
      ready.pop_front();
      lk.unlock();
      const auto ts = Clock::now();
      int rc = emqx_host_batch_submit(buf[k].hb, mode);
      const uint64_t dts = std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now() - ts).count();
      lk.lock();
      ns_submit += dts;
      if (rc != EMQX_OK) {  // report the failure to every caller of the batch
        lk.unlock();
        for (void* c : buf[k].ctx) cb(c, rc, nullptr, 0);
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
      cv.wait(lk, [&] { return !inflight.empty() || (stop && ready.empty() && filling < 0 && dispatcher_done); });
      if (inflight.empty()) return;
      const int k = inflight.front();
      lk.unlock();
      emqx_host_batch* b = buf[k].hb;
      const auto tw = Clock::now();
      int rc = emqx_host_batch_wait(b);
      if (rc == EMQX_EOVERFLOW) {  // more ids than the buffer holds: grow it, rerun the batch
        rc = emqx_host_batch_reserve(b, b->cap_topics, b->cap_bytes, b->n_out + (b->n_out >> 1) + 1024);
        if (rc == EMQX_OK) rc = emqx_host_batch_submit(b, mode);
        if (rc == EMQX_OK) rc = emqx_host_batch_wait(b);
      }
      const auto tc = Clock::now();
      const std::vector<void*>& ctx = buf[k].ctx;
      for (size_t i = 0; i < ctx.size(); ++i) {
        if (rc == EMQX_OK)
          cb(ctx[i], rc, b->out_ids + b->out_offsets[i], b->out_offsets[i + 1] - b->out_offsets[i]);
        else
          cb(ctx[i], rc, nullptr, 0);
      }
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

  bool dispatcher_done = false;
};

extern "C" {

int emqx_batcher_create(emqx_engine* e, uint32_t mode, uint32_t max_batch, uint32_t max_wait_us, emqx_batch_cb cb,
                        emqx_batcher** out) {
  if (!e || !cb || !out || mode > EMQX_MODE_TRIE_WILDCARD || max_batch == 0) return EMQX_EINVAL;
  auto* b = new (std::nothrow) emqx_batcher();
  if (!b) return EMQX_ENOMEM;
  b->e = e;
  b->mode = mode;
  b->max_batch = max_batch;
  b->max_wait_us = max_wait_us;
  b->cb = cb;
  for (int k = 0; k < NBUF; ++k) {
    // ~48 B per topic and 32 ids per topic to start with; both grow on demand
    int rc = emqx_host_batch_create(e, max_batch, std::max<uint64_t>(48ull * max_batch, 1u << 16),
                                    std::max<uint64_t>(32ull * max_batch, 1u << 16), &b->buf[k].hb);
    if (rc != EMQX_OK) {
      for (int j = 0; j < k; ++j) emqx_host_batch_destroy(b->buf[j].hb);
      delete b;
      return rc;
    }
    b->buf[k].hb->topic_offsets[0] = 0;
    b->buf[k].hb->n = 0;
    b->free_.push_back(k);
  }
  b->dispatcher = std::thread([b] {
    b->dispatch_loop();
    std::lock_guard<std::mutex> g(b->mu);
    b->dispatcher_done = true;
    b->cv.notify_all();
  });
  b->completer = std::thread([b] { b->complete_loop(); });
  *out = b;
  return EMQX_OK;
}

}  // extern "C"

namespace {

// One topic into the filling buffer (the caller holds b->mu through lk).
int submit_locked(emqx_batcher* b, std::unique_lock<std::mutex>& lk, const uint8_t* topic, uint64_t len, void* ctx) {
  while (true) {
    if (b->stop) return EMQX_EINVAL;
    if (b->filling < 0) {
      if (b->free_.empty()) {  // every buffer filling, sealed or in flight: wait for one
        b->cv.wait(lk);
        continue;
      }
      b->filling = b->free_.back();
      b->free_.pop_back();
      Buf& f = b->buf[b->filling];
      f.ctx.clear();
      f.bytes = 0;
      f.hb->n = 0;
      f.hb->topic_offsets[0] = 0;
    }
    Buf& f = b->buf[b->filling];
    emqx_host_batch* hb = f.hb;
    if (f.bytes + len > hb->cap_bytes) {
      if (f.ctx.empty()) {  // a topic larger than the buffer: grow it
        int rc = emqx_host_batch_reserve(hb, hb->cap_topics, len + (len >> 1) + 64, hb->cap_ids);
        if (rc != EMQX_OK) return rc;
      } else {
        b->seal();
        b->cv.notify_all();
        continue;
      }
    }
    if (len) std::memcpy(hb->topic_bytes + f.bytes, topic, len);
    f.bytes += len;
    hb->n += 1;
    hb->topic_offsets[hb->n] = f.bytes;
    f.ctx.push_back(ctx);
    if (f.ctx.size() == 1) f.t0 = Clock::now();
    if (f.ctx.size() >= b->max_batch) b->seal();
    if (f.ctx.size() == 1 || b->filling < 0) b->cv.notify_all();
    return EMQX_OK;
  }
}

}  // namespace

extern "C" {

int emqx_batcher_submit(emqx_batcher* b, const uint8_t* topic, uint64_t len, void* ctx) {
  if (!b || (len && !topic)) return EMQX_EINVAL;
  std::unique_lock<std::mutex> lk(b->mu);
  return submit_locked(b, lk, topic, len, ctx);
}

int emqx_batcher_submit_many(emqx_batcher* b, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                             void* const* ctxs) {
  if (!b || (n && (!offsets || !ctxs))) return EMQX_EINVAL;
  std::unique_lock<std::mutex> lk(b->mu);
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t len = offsets[i + 1] - offsets[i];
    if (len && !bytes) return EMQX_EINVAL;
    const int rc = submit_locked(b, lk, bytes + offsets[i], len, ctxs[i]);
    if (rc != EMQX_OK) return rc;
  }
  return EMQX_OK;
}

int emqx_batcher_destroy(emqx_batcher* b) {
  if (!b) return EMQX_EINVAL;
  {
    std::lock_guard<std::mutex> g(b->mu);
    b->stop = true;
  }
  b->cv.notify_all();
  if (b->dispatcher.joinable()) b->dispatcher.join();  // pending submissions are dispatched
  if (b->completer.joinable()) b->completer.join();    // and completed first
  for (int k = 0; k < NBUF; ++k) emqx_host_batch_destroy(b->buf[k].hb);
  delete b;
  return EMQX_OK;
}

int emqx_batcher_stats(emqx_batcher* b, uint64_t* n_batches, uint64_t* n_topics) {
  if (!b) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(b->mu);
  if (n_batches) *n_batches = b->n_batches;
  if (n_topics) *n_topics = b->n_topics;
  return EMQX_OK;
}

int emqx_batcher_stats_ext(emqx_batcher* b, uint64_t* out, uint32_t n) {
  if (!b || (n && !out)) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(b->mu);
  const uint64_t v[6] = {b->n_batches, b->n_topics, b->max_inflight_seen, b->ns_wait, b->ns_callbacks, b->ns_submit};
  for (uint32_t i = 0; i < n && i < 6; ++i) out[i] = v[i];
  return EMQX_OK;
}

}  // extern "C"
