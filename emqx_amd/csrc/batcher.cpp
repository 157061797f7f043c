// Cross-caller batcher (include/emqx_match.h, emqx_batcher_*).
//
// emqx_router:match_routes/1 is called once per PUBLISH by each publisher's own process
// (apps/emqx/src/emqx_broker.erl:213).  Many concurrent single-topic calls are coalesced here
// into one device match: callers submit a topic and a context pointer and return at once; a
// worker thread gathers submissions until `max_batch` topics are queued or `max_wait_us` has
// passed since the oldest one, runs one emqx_match_batch over them and hands every caller its
// filter ids through the callback.  The Erlang NIF uses the callback to enif_send the result to
// the waiting process, so the Erlang call shape stays synchronous while the GPU sees batches.
#include <stdint.h>

#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/emqx_match.h"

namespace {

struct Req {
  std::string topic;
  void* ctx;
  std::chrono::steady_clock::time_point t;
};

}  // namespace

struct emqx_batcher {
  emqx_engine* e = nullptr;
  uint32_t mode = EMQX_MODE_ROUTES;
  uint32_t max_batch = 4096;
  uint32_t max_wait_us = 200;
  emqx_batch_cb cb = nullptr;
  std::mutex mu;
  std::condition_variable cv;
  std::deque<Req> q;
  bool stop = false;
  std::thread worker;
  uint64_t n_batches = 0, n_topics = 0;

  void run() {
    std::vector<Req> batch;
    std::vector<uint8_t> bytes;
    std::vector<uint64_t> offs;
    std::vector<uint64_t> out_off;
    std::vector<uint32_t> out_ids(1 << 16);
    while (true) {
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || !q.empty(); });
        if (q.empty() && stop) return;
        // wait for a full batch or the oldest request's deadline
        const auto deadline = q.front().t + std::chrono::microseconds(max_wait_us);
        cv.wait_until(lk, deadline, [&] { return stop || q.size() >= max_batch; });
        const size_t take = std::min<size_t>(q.size(), max_batch);
        batch.clear();
        for (size_t i = 0; i < take; ++i) {
          batch.push_back(std::move(q.front()));
          q.pop_front();
        }
      }
      if (batch.empty()) continue;
      bytes.clear();
      offs.assign(1, 0);
      for (auto& r : batch) {
        bytes.insert(bytes.end(), r.topic.begin(), r.topic.end());
        offs.push_back(bytes.size());
      }
      if (bytes.empty()) bytes.push_back(0);
      out_off.assign(batch.size() + 1, 0);
      uint64_t total = 0;
      int rc = emqx_match_batch(e, mode, bytes.data(), offs.data(), batch.size(), out_off.data(), out_ids.data(),
                                out_ids.size(), &total);
      if (rc == EMQX_EOVERFLOW) {
        out_ids.resize(total + 1024);
        rc = emqx_match_batch(e, mode, bytes.data(), offs.data(), batch.size(), out_off.data(), out_ids.data(),
                              out_ids.size(), &total);
      }
      for (size_t i = 0; i < batch.size(); ++i) {
        if (rc == EMQX_OK)
          cb(batch[i].ctx, rc, out_ids.data() + out_off[i], out_off[i + 1] - out_off[i]);
        else
          cb(batch[i].ctx, rc, nullptr, 0);
      }
      std::lock_guard<std::mutex> g(mu);
      n_batches += 1;
      n_topics += batch.size();
    }
  }
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
  b->worker = std::thread([b] { b->run(); });
  *out = b;
  return EMQX_OK;
}

int emqx_batcher_submit(emqx_batcher* b, const uint8_t* topic, uint64_t len, void* ctx) {
  if (!b || (len && !topic)) return EMQX_EINVAL;
  {
    std::lock_guard<std::mutex> g(b->mu);
    if (b->stop) return EMQX_EINVAL;
    b->q.push_back(Req{std::string(reinterpret_cast<const char*>(topic), len), ctx,
                       std::chrono::steady_clock::now()});
  }
  b->cv.notify_one();
  return EMQX_OK;
}

int emqx_batcher_destroy(emqx_batcher* b) {
  if (!b) return EMQX_EINVAL;
  {
    std::lock_guard<std::mutex> g(b->mu);
    b->stop = true;
  }
  b->cv.notify_all();
  if (b->worker.joinable()) b->worker.join();  // drains pending submissions first
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

}  // extern "C"
