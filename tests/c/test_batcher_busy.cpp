// CPU test of the cross-caller batchers (emqx_amd/csrc/batcher.cpp) against a fake device: the
// emqx_host_batch_* / emqx_pub_batch_* entry points are defined here, and a "device" gate holds
// every submitted batch until the test opens it.  Checks (tests/test_nif_protocol.py):
//   1. with every pinned buffer busy, emqx_batcher_try_submit returns EMQX_EBUSY at once (it
//      never waits: the NIF calls it from a normal BEAM scheduler), and so does
//      emqx_pub_batcher_try_submit;
//   2. the blocking submit waits until a buffer frees, then completes;
//   3. every accepted submission gets exactly one callback, with its own results;
//   4. a topic whose buffer cannot grow (reserve fails) returns the error, and destroy then
//      returns instead of hanging (the buffer was left filling with no topics).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "emqx_match.h"

namespace {

std::mutex g_mu;
std::condition_variable g_cv;
bool g_open = false;                 // the fake device completes batches only when open
std::atomic<int> g_submits{0};
constexpr uint64_t MAX_BYTES = 1u << 20;  // reserve beyond this fails (ENOMEM)

void gate_wait() {
  std::unique_lock<std::mutex> lk(g_mu);
  g_cv.wait(lk, [] { return g_open; });
}

void gate_set(bool open) {
  {
    std::lock_guard<std::mutex> g(g_mu);
    g_open = open;
  }
  g_cv.notify_all();
}

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      exit(1);                                                     \
    }                                                              \
  } while (0)

double ms_since(std::chrono::steady_clock::time_point t) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t).count();
}

}  // namespace

// ---- fake pinned match batches: topic i -> one id, its length ----
extern "C" {

int emqx_host_batch_create(emqx_engine*, uint64_t cap_topics, uint64_t cap_bytes, uint64_t cap_ids,
                           emqx_host_batch** out) {
  auto* b = static_cast<emqx_host_batch*>(calloc(1, sizeof(emqx_host_batch)));
  b->cap_topics = cap_topics;
  b->cap_bytes = cap_bytes;
  b->cap_ids = cap_ids;
  b->topic_bytes = static_cast<uint8_t*>(malloc(cap_bytes + 16));
  b->topic_offsets = static_cast<uint64_t*>(calloc(cap_topics + 1, 8));
  b->out_offsets = static_cast<uint64_t*>(calloc(cap_topics + 1, 8));
  b->out_ids = static_cast<uint32_t*>(calloc(cap_ids, 4));
  *out = b;
  return EMQX_OK;
}

int emqx_host_batch_destroy(emqx_host_batch* b) {
  free(b->topic_bytes);
  free(b->topic_offsets);
  free(b->out_offsets);
  free(b->out_ids);
  free(b);
  return EMQX_OK;
}

int emqx_host_batch_reserve(emqx_host_batch* b, uint64_t, uint64_t cap_bytes, uint64_t) {
  if (cap_bytes > MAX_BYTES) return EMQX_ENOMEM;
  if (cap_bytes > b->cap_bytes) {
    b->topic_bytes = static_cast<uint8_t*>(realloc(b->topic_bytes, cap_bytes + 16));
    b->cap_bytes = cap_bytes;
  }
  return EMQX_OK;
}

int emqx_host_batch_submit(emqx_host_batch*, uint32_t) {
  g_submits++;
  return EMQX_OK;
}

int emqx_host_batch_wait(emqx_host_batch* b) {
  gate_wait();
  for (uint64_t i = 0; i < b->n; ++i) {
    b->out_offsets[i] = i;
    b->out_ids[i] = static_cast<uint32_t>(b->topic_offsets[i + 1] - b->topic_offsets[i]);
  }
  b->out_offsets[b->n] = b->n;
  b->n_out = b->n;
  return EMQX_OK;
}

int emqx_host_batch_query(emqx_host_batch*) { return 1; }

// ---- fake pinned publish batches: message i -> one delivery (key, length) ----
int emqx_pub_batch_create(emqx_engine*, emqx_subtab*, uint32_t, uint64_t cap_topics, uint64_t cap_bytes,
                          uint64_t cap_out, emqx_pub_batch** out) {
  auto* b = static_cast<emqx_pub_batch*>(calloc(1, sizeof(emqx_pub_batch)));
  b->cap_topics = cap_topics;
  b->cap_bytes = cap_bytes;
  b->cap_out = cap_out;
  b->topic_bytes = static_cast<uint8_t*>(malloc(cap_bytes + 16));
  b->topic_offsets = static_cast<uint64_t*>(calloc(cap_topics + 1, 8));
  b->keys = static_cast<uint32_t*>(calloc(cap_topics, 4));
  b->out_offsets = static_cast<uint64_t*>(calloc(cap_topics + 1, 8));
  b->out_subs = static_cast<uint32_t*>(calloc(cap_out, 4));
  b->out_filters = static_cast<uint32_t*>(calloc(cap_out, 4));
  *out = b;
  return EMQX_OK;
}

int emqx_pub_batch_destroy(emqx_pub_batch* b) {
  free(b->topic_bytes);
  free(b->topic_offsets);
  free(b->keys);
  free(b->out_offsets);
  free(b->out_subs);
  free(b->out_filters);
  free(b);
  return EMQX_OK;
}

int emqx_pub_batch_reserve(emqx_pub_batch* b, uint64_t, uint64_t cap_bytes, uint64_t) {
  if (cap_bytes > MAX_BYTES) return EMQX_ENOMEM;
  if (cap_bytes > b->cap_bytes) {
    b->topic_bytes = static_cast<uint8_t*>(realloc(b->topic_bytes, cap_bytes + 16));
    b->cap_bytes = cap_bytes;
  }
  return EMQX_OK;
}

int emqx_pub_batch_submit(emqx_pub_batch*) {
  g_submits++;
  return EMQX_OK;
}

int emqx_pub_batch_wait(emqx_pub_batch* b) {
  gate_wait();
  for (uint64_t i = 0; i < b->n; ++i) {
    b->out_offsets[i] = i;
    b->out_subs[i] = b->keys[i];
    b->out_filters[i] = static_cast<uint32_t>(b->topic_offsets[i + 1] - b->topic_offsets[i]);
  }
  b->out_offsets[b->n] = b->n;
  b->n_out = b->n;
  return EMQX_OK;
}

int emqx_pub_batch_query(emqx_pub_batch*) { return 1; }

}  // extern "C"

namespace {

struct Result {
  std::atomic<int> calls{0};
  std::atomic<int> status{EMQX_OK};
  std::atomic<uint32_t> value{0};
};

Result g_res[64];

void match_cb(void* ctx, int status, const uint32_t* ids, uint64_t n) {
  Result& r = g_res[reinterpret_cast<uintptr_t>(ctx)];
  r.status = status;
  if (status == EMQX_OK && n == 1) r.value = ids[0];
  r.calls++;
}

void pub_cb(void* ctx, int status, const uint32_t* subs, const uint32_t* fils, uint64_t n) {
  Result& r = g_res[reinterpret_cast<uintptr_t>(ctx)];
  r.status = status;
  if (status == EMQX_OK && n == 1) r.value = subs[0] * 1000 + fils[0];
  r.calls++;
}

void reset() {
  for (auto& r : g_res) {
    r.calls = 0;
    r.status = EMQX_OK;
    r.value = 0;
  }
}

void wait_calls(int k, int want) {
  const auto t = std::chrono::steady_clock::now();
  while (g_res[k].calls.load() < want) {
    CHECK(ms_since(t) < 5000);
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
}

emqx_engine* const FAKE_ENGINE = reinterpret_cast<emqx_engine*>(0x1000);
emqx_subtab* const FAKE_SUBTAB = reinterpret_cast<emqx_subtab*>(0x2000);

void test_match_batcher() {
  reset();
  gate_set(false);
  emqx_batcher* b = nullptr;
  CHECK(emqx_batcher_create(FAKE_ENGINE, EMQX_MODE_ROUTES, 1, 0, match_cb, &b) == EMQX_OK);
  const char* topic = "a/b/c";
  int accepted = 0;
  int rc = EMQX_OK;
  for (int k = 1; k < 32; ++k) {
    const auto t = std::chrono::steady_clock::now();
    rc = emqx_batcher_try_submit(b, reinterpret_cast<const uint8_t*>(topic), 1 + k % 5,
                                 reinterpret_cast<void*>(static_cast<uintptr_t>(k)));
    CHECK(ms_since(t) < 50);  // never waits for the device
    if (rc == EMQX_EBUSY) break;
    CHECK(rc == EMQX_OK);
    ++accepted;
    std::this_thread::sleep_for(std::chrono::milliseconds(2));  // let the dispatcher take it
  }
  CHECK(rc == EMQX_EBUSY);
  CHECK(accepted == 4);  // two batches in flight, two sealed: every buffer busy
  for (int k = 1; k <= accepted; ++k) CHECK(g_res[k].calls.load() == 0);
  // a second try while still busy: EBUSY again, still at once, and no callback for it
  const auto t = std::chrono::steady_clock::now();
  CHECK(emqx_batcher_try_submit(b, reinterpret_cast<const uint8_t*>(topic), 3, reinterpret_cast<void*>(40)) ==
        EMQX_EBUSY);
  CHECK(ms_since(t) < 50);
  // the blocking submit waits for a buffer (the dirty-scheduler path)
  std::atomic<bool> returned{false};
  std::thread blocker([&] {
    CHECK(emqx_batcher_submit(b, reinterpret_cast<const uint8_t*>(topic), 5, reinterpret_cast<void*>(41)) ==
          EMQX_OK);
    returned = true;
  });
  std::this_thread::sleep_for(std::chrono::milliseconds(100));
  CHECK(!returned.load());
  gate_set(true);
  blocker.join();
  for (int k = 1; k <= accepted; ++k) {
    wait_calls(k, 1);
    CHECK(g_res[k].status.load() == EMQX_OK);
    CHECK(g_res[k].value.load() == static_cast<uint32_t>(1 + k % 5));
  }
  wait_calls(41, 1);
  CHECK(g_res[41].value.load() == 5);
  CHECK(g_res[40].calls.load() == 0);
  CHECK(emqx_batcher_destroy(b) == EMQX_OK);
  for (int k = 1; k <= 41; ++k) CHECK(g_res[k].calls.load() <= 1);
}

void test_pub_batcher() {
  reset();
  gate_set(false);
  emqx_pub_batcher* b = nullptr;
  CHECK(emqx_pub_batcher_create(FAKE_ENGINE, FAKE_SUBTAB, EMQX_SHARE_ROUND_ROBIN, 1, 0, pub_cb, &b) == EMQX_OK);
  const char* topic = "x/y";
  int accepted = 0, rc = EMQX_OK;
  for (int k = 1; k < 32; ++k) {
    const auto t = std::chrono::steady_clock::now();
    rc = emqx_pub_batcher_try_submit(b, reinterpret_cast<const uint8_t*>(topic), 3, 100 + k,
                                     reinterpret_cast<void*>(static_cast<uintptr_t>(k)));
    CHECK(ms_since(t) < 50);
    if (rc == EMQX_EBUSY) break;
    CHECK(rc == EMQX_OK);
    ++accepted;
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  }
  CHECK(rc == EMQX_EBUSY && accepted == 4);
  gate_set(true);
  for (int k = 1; k <= accepted; ++k) {
    wait_calls(k, 1);
    CHECK(g_res[k].value.load() == static_cast<uint32_t>((100 + k) * 1000 + 3));  // its own key and length
  }
  // submit_many with keys
  const uint8_t bytes[] = "ab" "cde";
  const uint64_t offs[] = {0, 2, 5};
  const uint32_t keys[] = {7, 9};
  void* ctxs[] = {reinterpret_cast<void*>(50), reinterpret_cast<void*>(51)};
  CHECK(emqx_pub_batcher_submit_many(b, bytes, offs, keys, 2, ctxs) == EMQX_OK);
  wait_calls(50, 1);
  wait_calls(51, 1);
  CHECK(g_res[50].value.load() == 7 * 1000 + 2 && g_res[51].value.load() == 9 * 1000 + 3);
  CHECK(emqx_pub_batcher_destroy(b) == EMQX_OK);
}

void test_reserve_failure_then_destroy() {
  reset();
  gate_set(true);
  emqx_batcher* b = nullptr;
  CHECK(emqx_batcher_create(FAKE_ENGINE, EMQX_MODE_ROUTES, 8, 100, match_cb, &b) == EMQX_OK);
  std::vector<uint8_t> huge(2 * MAX_BYTES, 'a');
  // non-blocking: growing a buffer is not done on a normal scheduler
  CHECK(emqx_batcher_try_submit(b, huge.data(), huge.size(), reinterpret_cast<void*>(1)) == EMQX_EBUSY);
  CHECK(emqx_batcher_submit(b, huge.data(), huge.size(), reinterpret_cast<void*>(1)) == EMQX_ENOMEM);
  // the batcher still works afterwards
  CHECK(emqx_batcher_submit(b, reinterpret_cast<const uint8_t*>("q"), 1, reinterpret_cast<void*>(2)) == EMQX_OK);
  wait_calls(2, 1);
  CHECK(g_res[2].value.load() == 1 && g_res[1].calls.load() == 0);
  alarm(10);  // a hang in destroy fails the test
  CHECK(emqx_batcher_destroy(b) == EMQX_OK);
  alarm(0);
}

}  // namespace

int main() {
  test_match_batcher();
  test_pub_batcher();
  test_reserve_failure_then_destroy();
  printf("ok\n");
  return 0;
}
