// Commit coalescer (include/emqx_match.h, emqx_coalescer_*): route and subscription changes of
// many callers share one commit.
//
// The reference applies each change on its own: emqx_broker:subscribe/3 writes ?SUBSCRIBER per
// call (apps/emqx/src/emqx_broker.erl:146-164), a new topic's route is one mria transaction
// (emqx_router.erl:111-124 -> emqx_router_utils.erl:97-125), each visible to readers when it
// returns.  Here a change is applied to the host store at once (an insert returns its filter
// ids), and its caller is told when the commit that carries it has reached the device: a worker
// thread commits whenever changes are pending and it is idle (group commit: the changes that
// arrive during one commit make the next one), optionally waiting max_wait_us after the first
// pending change for more.  Engine (route) changes commit before subscription changes, so a
// subscription to a new topic never waits for a second round.
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "../../include/emqx_match.h"

namespace {
using Clock = std::chrono::steady_clock;
}

struct emqx_coalescer {
  emqx_engine* e = nullptr;
  emqx_subtab* s = nullptr;
  uint32_t max_wait_us = 0;
  emqx_done_cb cb = nullptr;
  std::mutex mu;
  std::condition_variable cv, cv_done;
  std::vector<void*> pending;  // contexts of applied changes waiting for a commit
  uint64_t pending_ops = 0;
  bool eng_dirty = false, sub_dirty = false;
  Clock::time_point first_at;
  uint64_t seq_submitted = 0, seq_done = 0;  // changes applied / changes committed (flush)
  bool stop = false;
  std::thread worker;
  // statistics
  uint64_t st_commits = 0, st_ops = 0, st_max_ops = 0, st_eng_commits = 0, st_sub_commits = 0;
  double st_commit_us = 0;
  int last_rc = EMQX_OK;
};

namespace {

void run(emqx_coalescer* c) {
  std::vector<void*> batch;
  std::unique_lock<std::mutex> lk(c->mu);
  for (;;) {
    c->cv.wait(lk, [&] { return c->stop || c->seq_submitted != c->seq_done; });
    if (c->seq_submitted == c->seq_done) break;  // stop, nothing pending
    if (c->max_wait_us && !c->stop)
      c->cv.wait_until(lk, c->first_at + std::chrono::microseconds(c->max_wait_us), [&] { return c->stop; });
    batch.swap(c->pending);
    const bool ed = c->eng_dirty, sd = c->sub_dirty;
    const uint64_t ops = c->pending_ops, seq = c->seq_submitted;
    c->eng_dirty = c->sub_dirty = false;
    c->pending_ops = 0;
    lk.unlock();
    const auto t0 = Clock::now();
    int rc = EMQX_OK;
    if (ed) rc = emqx_commit(c->e);
    // the callbacks say "committed": the subtable commit's device half (which emqx_subtab_commit
    // leaves in flight) is waited for first, so a device error reaches this batch's callers
    if (rc == EMQX_OK && sd) rc = emqx_subtab_commit(c->s);
    if (rc == EMQX_OK && sd) rc = emqx_subtab_commit_wait(c->s);
    const double us = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
    for (void* ctx : batch) c->cb(ctx, rc);
    batch.clear();
    lk.lock();
    c->seq_done = seq;
    c->last_rc = rc;
    ++c->st_commits;
    c->st_ops += ops;
    c->st_max_ops = std::max(c->st_max_ops, ops);
    c->st_eng_commits += ed;
    c->st_sub_commits += sd;
    c->st_commit_us += us;
    c->cv_done.notify_all();
  }
}

// Applies one change with `apply` under the coalescer's lock (so a commit that has taken its
// batch never misses a change whose context it carries) and queues its context.
template <class F>
int submit(emqx_coalescer* c, uint64_t n, bool engine, void* ctx, F apply) {
  std::lock_guard<std::mutex> g(c->mu);
  if (c->stop) return EMQX_EINVAL;
  const int rc = apply();
  if (rc != EMQX_OK) return rc;
  if (c->seq_submitted == c->seq_done) c->first_at = Clock::now();
  if (ctx) c->pending.push_back(ctx);
  c->pending_ops += n ? n : 1;
  (engine ? c->eng_dirty : c->sub_dirty) = true;
  ++c->seq_submitted;
  c->cv.notify_one();
  return EMQX_OK;
}

}  // namespace

extern "C" {

int emqx_coalescer_create(emqx_engine* e, emqx_subtab* s, uint32_t max_wait_us, emqx_done_cb cb,
                          emqx_coalescer** out) {
  if (!out || (!e && !s) || !cb) return EMQX_EINVAL;
  *out = nullptr;
  auto* c = new (std::nothrow) emqx_coalescer();
  if (!c) return EMQX_ENOMEM;
  c->e = e;
  c->s = s;
  c->max_wait_us = max_wait_us;
  c->cb = cb;
  try {
    c->worker = std::thread(run, c);
  } catch (...) {
    delete c;
    return EMQX_ENOMEM;
  }
  *out = c;
  return EMQX_OK;
}

int emqx_coalescer_insert_filters(emqx_coalescer* c, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                                  uint32_t* ids_out, void* ctx) {
  if (!c || !c->e) return EMQX_EINVAL;
  return submit(c, n, true, ctx, [&] { return emqx_insert_filters(c->e, bytes, offsets, n, ids_out); });
}

int emqx_coalescer_delete_filters(emqx_coalescer* c, const uint32_t* ids, uint64_t n, void* ctx) {
  if (!c || !c->e) return EMQX_EINVAL;
  return submit(c, n, true, ctx, [&] { return emqx_delete_filters(c->e, ids, n); });
}

int emqx_coalescer_subscribe(emqx_coalescer* c, const uint32_t* filter_ids, const uint32_t* sub_ids,
                             const uint32_t* group_ids, uint64_t n, int add, void* ctx) {
  if (!c || !c->s) return EMQX_EINVAL;
  return submit(c, n, false, ctx, [&] {
    return add ? emqx_subtab_add(c->s, filter_ids, sub_ids, group_ids, n)
               : emqx_subtab_remove(c->s, filter_ids, sub_ids, group_ids, n);
  });
}

int emqx_coalescer_subscribe_many(emqx_coalescer* c, const uint32_t* filter_ids, const uint32_t* sub_ids,
                                  const uint32_t* group_ids, const uint8_t* adds, uint64_t n, void* const* ctxs) {
  if (!c || !c->s || (n && (!filter_ids || !sub_ids || !adds))) return EMQX_EINVAL;
  if (n == 0) return EMQX_OK;
  std::lock_guard<std::mutex> g(c->mu);
  if (c->stop) return EMQX_EINVAL;
  // runs of the same kind, one table call each; all or nothing is not promised across runs, so
  // the contexts of the runs applied are queued before an error returns
  uint64_t i = 0;
  int rc = EMQX_OK;
  while (i < n && rc == EMQX_OK) {
    uint64_t j = i + 1;
    while (j < n && (adds[j] != 0) == (adds[i] != 0)) ++j;
    const uint32_t* gr = group_ids ? group_ids + i : nullptr;
    rc = adds[i] ? emqx_subtab_add(c->s, filter_ids + i, sub_ids + i, gr, j - i)
                 : emqx_subtab_remove(c->s, filter_ids + i, sub_ids + i, gr, j - i);
    if (rc != EMQX_OK) break;
    if (c->seq_submitted == c->seq_done) c->first_at = Clock::now();
    if (ctxs)
      for (uint64_t k = i; k < j; ++k)
        if (ctxs[k]) c->pending.push_back(ctxs[k]);
    c->pending_ops += j - i;
    c->sub_dirty = true;
    ++c->seq_submitted;
    i = j;
  }
  c->cv.notify_one();
  return rc;
}

int emqx_coalescer_set_alive(emqx_coalescer* c, const uint32_t* sub_ids, uint64_t n, int alive, void* ctx) {
  if (!c || !c->s) return EMQX_EINVAL;
  return submit(c, n, false, ctx, [&] { return emqx_subtab_set_alive(c->s, sub_ids, n, alive); });
}

int emqx_coalescer_flush(emqx_coalescer* c) {
  if (!c) return EMQX_EINVAL;
  std::unique_lock<std::mutex> lk(c->mu);
  const uint64_t target = c->seq_submitted;
  c->cv.notify_one();
  c->cv_done.wait(lk, [&] { return c->seq_done >= target; });
  return c->last_rc;
}

int emqx_coalescer_destroy(emqx_coalescer* c) {
  if (!c) return EMQX_EINVAL;
  {
    std::lock_guard<std::mutex> g(c->mu);
    c->stop = true;
    c->cv.notify_one();
  }
  if (c->worker.joinable()) c->worker.join();  // (commits and notifies what is pending first)
  delete c;
  return EMQX_OK;
}

int emqx_coalescer_stats(emqx_coalescer* c, uint64_t* out, uint32_t n) {
  if (!c || (n && !out)) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(c->mu);
  const uint64_t v[6] = {c->st_commits, c->st_ops, c->st_max_ops, static_cast<uint64_t>(c->st_commit_us),
                         c->st_eng_commits, c->st_sub_commits};
  for (uint32_t i = 0; i < n && i < 6; ++i) out[i] = v[i];
  return EMQX_OK;
}

}  // extern "C"
