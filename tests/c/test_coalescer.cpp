// CPU test of the commit coalescer (emqx_amd/csrc/coalescer.cpp) against a fake engine and a
// fake subscription table: the emqx_insert_filters / emqx_delete_filters / emqx_commit and
// emqx_subtab_* entry points are defined here, and a gate holds every commit until the test
// opens it.  Checks (tests/test_nif_protocol.py):
//   1. a change is applied when its call returns (insert ids), its callback comes after the
//      commit that carries it, never before;
//   2. group commit: changes submitted while a commit runs all go into the next one;
//   3. route (engine) changes commit before subscription changes in a round;
//   4. flush waits for everything submitted before it; destroy commits and notifies the rest;
//   5. a failing commit reports its status to every change it carried, including a failure of
//      the subtable commit's device half (emqx_subtab_commit_wait), which the batch's callbacks
//      wait for.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "emqx_match.h"

#define CHECK(c)                                                            \
  do {                                                                      \
    if (!(c)) {                                                             \
      fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
      exit(1);                                                              \
    }                                                                       \
  } while (0)

namespace {

std::mutex g_mu;
std::condition_variable g_cv;
bool g_open = true;
std::vector<std::string> g_log;  // "E<ops>" engine commit, "S<ops>" subtab commit, in order
uint64_t g_eng_applied = 0, g_sub_applied = 0, g_eng_seen = 0, g_sub_seen = 0;
int g_fail = EMQX_OK;
int g_wait_fail = EMQX_OK;      // status of the subtable commit's device half
uint64_t g_waits = 0;           // emqx_subtab_commit_wait calls
uint32_t g_next_id = 100;

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

struct Done {
  std::atomic<int> calls{0};
  std::atomic<int> status{1};
  uint64_t commits_before = 0;  // commits logged when the callback ran
};

void on_done(void* ctx, int status) {
  auto* d = static_cast<Done*>(ctx);
  {
    std::lock_guard<std::mutex> g(g_mu);
    d->commits_before = g_log.size();
  }
  d->status = status;
  d->calls.fetch_add(1);
}

}  // namespace

extern "C" {

int emqx_insert_filters(emqx_engine*, const uint8_t*, const uint64_t*, uint64_t n, uint32_t* ids_out) {
  std::lock_guard<std::mutex> g(g_mu);
  for (uint64_t i = 0; i < n; ++i) ids_out[i] = g_next_id++;
  g_eng_applied += n;
  return EMQX_OK;
}
int emqx_delete_filters(emqx_engine*, const uint32_t* ids, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i)
    if (ids[i] >= 1000000) return EMQX_ENOTFOUND;
  std::lock_guard<std::mutex> g(g_mu);
  g_eng_applied += n;
  return EMQX_OK;
}
int emqx_commit(emqx_engine*) {
  uint64_t upto;
  {
    std::lock_guard<std::mutex> g(g_mu);  // the commit takes what is applied when it starts
    upto = g_eng_applied;
  }
  gate_wait();
  std::lock_guard<std::mutex> g(g_mu);
  g_log.push_back("E" + std::to_string(upto - g_eng_seen));
  g_eng_seen = upto;
  return g_fail;
}
int emqx_subtab_add(emqx_subtab*, const uint32_t*, const uint32_t*, const uint32_t*, uint64_t n) {
  std::lock_guard<std::mutex> g(g_mu);
  g_sub_applied += n;
  return EMQX_OK;
}
int emqx_subtab_remove(emqx_subtab*, const uint32_t*, const uint32_t*, const uint32_t*, uint64_t n) {
  std::lock_guard<std::mutex> g(g_mu);
  g_sub_applied += n;
  return EMQX_OK;
}
int emqx_subtab_set_alive(emqx_subtab*, const uint32_t*, uint64_t n, int) {
  std::lock_guard<std::mutex> g(g_mu);
  g_sub_applied += n;
  return EMQX_OK;
}
int emqx_subtab_commit(emqx_subtab*) {
  uint64_t upto;
  {
    std::lock_guard<std::mutex> g(g_mu);
    upto = g_sub_applied;
  }
  gate_wait();
  std::lock_guard<std::mutex> g(g_mu);
  g_log.push_back("S" + std::to_string(upto - g_sub_seen));
  g_sub_seen = upto;
  return g_fail;
}
int emqx_subtab_commit_wait(emqx_subtab*) {
  std::lock_guard<std::mutex> g(g_mu);
  ++g_waits;
  return g_wait_fail;
}

}  // extern "C"

int main() {
  emqx_engine* e = reinterpret_cast<emqx_engine*>(0x1);
  emqx_subtab* s = reinterpret_cast<emqx_subtab*>(0x2);
  emqx_coalescer* c = nullptr;
  CHECK(emqx_coalescer_create(e, s, 0, on_done, &c) == EMQX_OK);
  const uint8_t bytes[] = "a/b";
  const uint64_t offs[2] = {0, 3};
  uint32_t f = 7, sub = 9;

  // 1. one change: applied at return, callback after its commit
  Done d1;
  uint32_t id = 0;
  CHECK(emqx_coalescer_insert_filters(c, bytes, offs, 1, &id, &d1) == EMQX_OK);
  CHECK(id == 100);
  CHECK(emqx_coalescer_flush(c) == EMQX_OK);
  CHECK(d1.calls == 1 && d1.status == EMQX_OK && d1.commits_before >= 1);

  // 2. group commit: hold the first commit, submit 200 changes meanwhile -> one more commit
  gate_set(false);
  Done first;
  CHECK(emqx_coalescer_subscribe(c, &f, &sub, nullptr, 1, 1, &first) == EMQX_OK);
  std::this_thread::sleep_for(std::chrono::milliseconds(50));  // the worker is inside the commit
  std::vector<Done> many(200);
  std::vector<std::thread> th;
  for (int t = 0; t < 4; ++t)
    th.emplace_back([&, t] {
      for (int i = t; i < 200; i += 4) {
        uint32_t ff = 1000 + i, ss = i;
        CHECK(emqx_coalescer_subscribe(c, &ff, &ss, nullptr, 1, i & 1, &many[i]) == EMQX_OK);
      }
    });
  for (auto& x : th) x.join();
  size_t log_before;
  {
    std::lock_guard<std::mutex> g(g_mu);
    log_before = g_log.size();
  }
  for (auto& d : many) CHECK(d.calls == 0);  // nothing is reported before its commit
  gate_set(true);
  CHECK(emqx_coalescer_flush(c) == EMQX_OK);
  CHECK(first.calls == 1);
  for (auto& d : many) CHECK(d.calls == 1 && d.status == EMQX_OK);
  {
    std::lock_guard<std::mutex> g(g_mu);
    // the held commit carried 1 change, the next one all 200
    CHECK(g_log.size() == log_before + 2);
    CHECK(g_log[log_before] == "S1" && g_log[log_before + 1] == "S200");
  }

  // 2b. many callers' changes under one call: runs of adds and removes, every context called back
  //     after the one commit that carries them all
  {
    gate_set(false);
    Done hold;
    CHECK(emqx_coalescer_subscribe(c, &f, &sub, nullptr, 1, 1, &hold) == EMQX_OK);
    std::this_thread::sleep_for(std::chrono::milliseconds(50));
    std::vector<Done> ds(7);
    const uint32_t fs[7] = {1, 2, 3, 4, 5, 6, 7}, ss[7] = {1, 2, 3, 4, 5, 6, 7};
    const uint8_t adds[7] = {1, 1, 0, 0, 1, 0, 1};
    void* ctxs[7];
    for (int i = 0; i < 7; ++i) ctxs[i] = &ds[i];
    ctxs[3] = nullptr;  // a change nobody waits for
    CHECK(emqx_coalescer_subscribe_many(c, fs, ss, nullptr, adds, 7, ctxs) == EMQX_OK);
    size_t log_before;
    {
      std::lock_guard<std::mutex> g(g_mu);
      log_before = g_log.size();
    }
    gate_set(true);
    CHECK(emqx_coalescer_flush(c) == EMQX_OK);
    for (int i = 0; i < 7; ++i) CHECK(ds[i].calls == (i == 3 ? 0 : 1));
    std::lock_guard<std::mutex> g(g_mu);
    CHECK(g_log.size() == log_before + 2 && g_log[log_before + 1] == "S7");
  }

  // 3. a round with both kinds: engine first
  Done a, b;
  CHECK(emqx_coalescer_subscribe(c, &f, &sub, nullptr, 1, 1, &a) == EMQX_OK);
  CHECK(emqx_coalescer_insert_filters(c, bytes, offs, 1, &id, &b) == EMQX_OK);
  CHECK(emqx_coalescer_flush(c) == EMQX_OK);
  {
    std::lock_guard<std::mutex> g(g_mu);
    const size_t n = g_log.size();
    CHECK(g_log[n - 2][0] == 'E' && g_log[n - 1][0] == 'S');
  }

  // 4. a change that fails to apply is not queued; a failing commit reports to its changes
  uint32_t bad = 5000000;
  Done never;
  CHECK(emqx_coalescer_delete_filters(c, &bad, 1, &never) == EMQX_ENOTFOUND);
  g_fail = EMQX_EDEVICE;
  Done failed;
  CHECK(emqx_coalescer_subscribe(c, &f, &sub, nullptr, 1, 0, &failed) == EMQX_OK);
  CHECK(emqx_coalescer_flush(c) == EMQX_EDEVICE);
  CHECK(failed.calls == 1 && failed.status == EMQX_EDEVICE && never.calls == 0);
  g_fail = EMQX_OK;
  // 4b. the commit returned but its device half failed: the batch's callers get the error
  g_wait_fail = EMQX_EDEVICE;
  Done dev_failed;
  uint64_t waits0;
  {
    std::lock_guard<std::mutex> g(g_mu);
    waits0 = g_waits;
  }
  CHECK(emqx_coalescer_subscribe(c, &f, &sub, nullptr, 1, 1, &dev_failed) == EMQX_OK);
  CHECK(emqx_coalescer_flush(c) == EMQX_EDEVICE);
  CHECK(dev_failed.calls == 1 && dev_failed.status == EMQX_EDEVICE);
  {
    std::lock_guard<std::mutex> g(g_mu);
    CHECK(g_waits == waits0 + 1);
  }
  g_wait_fail = EMQX_OK;
  Done after;
  CHECK(emqx_coalescer_subscribe(c, &f, &sub, nullptr, 1, 1, &after) == EMQX_OK);
  CHECK(emqx_coalescer_flush(c) == EMQX_OK && after.status == EMQX_OK);

  // 5. destroy with changes pending: they are committed and notified
  gate_set(false);
  Done last[3];
  for (auto& d : last) CHECK(emqx_coalescer_subscribe(c, &f, &sub, nullptr, 1, 1, &d) == EMQX_OK);
  std::thread opener([] {
    std::this_thread::sleep_for(std::chrono::milliseconds(30));
    gate_set(true);
  });
  CHECK(emqx_coalescer_destroy(c) == EMQX_OK);
  opener.join();
  for (auto& d : last) CHECK(d.calls == 1 && d.status == EMQX_OK);
  printf("ok\n");
  return 0;
}
