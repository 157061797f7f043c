// C ABI implementation (include/emqx_match.h): filter store, full commits with an RCU-style
// snapshot swap, incremental commits patched into the committed table (live_trie.cpp),
// per-call workspaces, and the match pipeline
//   fast kernel -> deep kernel -> group reduce -> scatter -> summary (one sync per call).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/emqx_match.h"
#include "kernels.h"
#include "streams.h"
#include "tables.h"

using namespace emqx;

namespace {

#define HIP_TRY(expr)                    \
  do {                                   \
    hipError_t _e = (expr);              \
    if (_e != hipSuccess) {              \
      set_last_error(hipGetErrorString(_e)); \
      return EMQX_EDEVICE;               \
    }                                    \
  } while (0)

thread_local std::string g_last_error;
void set_last_error(const char* s) { g_last_error = s ? s : ""; }

template <class T>
void dfree(T*& p) {
  if (p) (void)hipFree(p);
  p = nullptr;
}

template <class T>
hipError_t dalloc(T*& p, uint64_t count) {
  dfree(p);
  return hipMalloc(reinterpret_cast<void**>(&p), std::max<uint64_t>(count, 1) * sizeof(T));
}

// Device buffers of one full build, with headroom for incremental commits: a spare slot
// region behind the built slots (new nodes and relocated arrays), vocab slots to fill, arena
// bytes to append.  Shared by every snapshot published from that build; freed (after draining
// the device: an async call may still read it) when the last one goes.
struct DeviceTables {
  int device = 0;
  EdgeSlot* edges = nullptr;  // cap_slots
  uint32_t* fids = nullptr;   // 2 * cap_slots
  VocabSlot* vocab = nullptr;
  uint8_t* arena = nullptr;
  uint64_t cap_slots = 0, n_vocab = 0, cap_arena = 0;
  uint64_t bytes() const {
    return cap_slots * (sizeof(EdgeSlot) + 2 * sizeof(uint32_t)) + n_vocab * sizeof(VocabSlot) + cap_arena;
  }
  ~DeviceTables() {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    (void)hipDeviceSynchronize();
    dfree(edges);
    dfree(fids);
    dfree(vocab);
    dfree(arena);
    (void)hipSetDevice(cur);
  }
};

struct Snapshot {
  std::shared_ptr<DeviceTables> dt;
  TableView tv{};
  uint64_t n_nodes = 0, n_slots = 0, n_words = 0, bytes = 0;
  uint32_t max_depth = 0;
};

// Writer-side state of incremental commits (under emqx_engine::writer): the host image of
// the committed table, patched per commit (tables.h LiveTrie), and the device buffers the
// commit writes through.
struct LiveState {
  bool valid = false;
  std::shared_ptr<DeviceTables> dt;
  std::unique_ptr<VocabState> vocab;
  std::unique_ptr<LiveTrie> lt;
  uint64_t inserted = 0;        // filters placed by incremental commits since the full build
  uint64_t base_live = 0;       // live filters at the full build
  hipStream_t stream = nullptr; // commit stream (uploads + patch kernels; synchronised alone)
  SlotPatch* d_patch = nullptr;
  uint64_t cap_patch = 0;
  std::vector<SlotPatch> patches;
  int device = 0;
  ~LiveState() {
    (void)hipSetDevice(device);
    if (d_patch) (void)hipFree(d_patch);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

struct Workspace {
  int device = 0;
  hipStream_t stream = nullptr;
  hipStream_t last_stream = nullptr;  // stream of the last call enqueued with this workspace
  hipEvent_t ev0 = nullptr, ev1 = nullptr, evk = nullptr;
  uint64_t cap_n = 0, cap_tiles = 0, cap_slab = 0;
  uint32_t slab_per_tile = 256;
  uint32_t* counts = nullptr;
  uint32_t* deferred = nullptr;
  uint32_t* deep_rank = nullptr;
  uint64_t* slab = nullptr;
  uint32_t* tile_fill = nullptr;
  uint64_t* tile_defer = nullptr;
  uint2* spill = nullptr;
  uint64_t* diag = nullptr;
  uint32_t spill_cap = 2048;  // items per tile
  uint32_t* ctrl = nullptr;         // CTRL_WORDS words (one memset per call)
  uint64_t* tile_sum = nullptr;
  uint2* tile_stats = nullptr;
  uint64_t* group_sum = nullptr;
  uint2* group_stats = nullptr;
  hipEvent_t done = nullptr;        // end of the last call enqueued with this workspace
  std::shared_ptr<Snapshot> inflight;  // table of the last async call (kept alive for it)
  uint32_t* deep_wids = nullptr;
  uint4* deep_stack = nullptr;
  uint32_t deep_stack_cap = 1u << 14;
  uint64_t* deep_slab = nullptr;
  uint32_t deep_slab_cap = 1u << 20;
  uint64_t* h_rb = nullptr;         // pinned call summary (SUM_WORDS), written by summary_kernel
  bool deep_ready = false;
  // walk order (order_kernels.hip): prefix keys, sorted positions, the reordered batch
  bool ordered = false;             // the last call enqueued walked in prefix-key order
  hipEvent_t evo = nullptr;         // start of its reordering
  uint64_t ord_cap_n = 0, ord_cap_bytes = 0, ord_temp_bytes = 0;
  uint64_t* ord_keys = nullptr;
  uint64_t* ord_keys_out = nullptr;
  uint32_t* ord_idx = nullptr;
  uint32_t* ord_perm = nullptr;
  uint32_t* ord_lens = nullptr;
  uint32_t* ord_corig = nullptr;
  uint64_t* ord_noffs = nullptr;
  uint64_t* ord_partials = nullptr;
  uint8_t* ord_bytes = nullptr;
  uint8_t* ord_temp = nullptr;

  ~Workspace() {
    (void)hipSetDevice(device);
    dfree(counts); dfree(deferred); dfree(deep_rank); dfree(slab); dfree(tile_fill);
    dfree(tile_defer); dfree(spill); dfree(diag); dfree(ctrl); dfree(tile_sum); dfree(tile_stats);
    dfree(group_sum); dfree(group_stats);
    dfree(deep_wids); dfree(deep_stack); dfree(deep_slab);
    dfree(ord_keys); dfree(ord_keys_out); dfree(ord_idx); dfree(ord_perm); dfree(ord_lens); dfree(ord_corig);
    dfree(ord_noffs); dfree(ord_partials); dfree(ord_bytes); dfree(ord_temp);
    if (h_rb) (void)hipHostFree(h_rb);
    if (ev0) (void)hipEventDestroy(ev0);
    if (ev1) (void)hipEventDestroy(ev1);
    if (evk) (void)hipEventDestroy(evk);
    if (evo) (void)hipEventDestroy(evo);
    if (done) (void)hipEventDestroy(done);
    if (stream) (void)hipStreamDestroy(stream);
  }
};

uint64_t round_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

}  // namespace

struct emqx_engine {
  int device = 0;
  std::mutex writer;
  FilterStore store;
  uint64_t epoch = 0;
  double last_build_ms = 0;
  std::mutex snap_mu;
  std::shared_ptr<Snapshot> snap;
  std::mutex ws_mu;
  std::vector<std::unique_ptr<Workspace>> all_ws;
  std::vector<Workspace*> free_ws;
  std::atomic<uint64_t> last_evals{0}, last_deferred{0}, last_max_stack{0};
  std::atomic<double> last_match_ms{0};
  std::atomic<double> last_kernel_ms{0};
  std::atomic<int> forced_variant{-1};
  std::atomic<bool> diag_on{false};
  std::atomic<uint32_t> diag_stop{0};  // emqx_set_tuning("diag_stop", 1): diag calls skip the walk
  uint4* timeline = nullptr;          // emqx_set_tuning("timeline", tiles): per-tile wall clocks of
  uint64_t timeline_cap = 0;          // the fast kernel (diag calls), read by emqx_diag_timeline
  std::atomic<uint32_t> slab_hint{256};  // largest slab per tile any workspace needed
  // incremental commits (under `writer`)
  LiveState ls;
  std::vector<uint32_t> dirty;  // ids inserted / deleted since the last commit
  bool incremental = true;      // emqx_set_tuning("incremental", 0|1)
  int64_t delta_max = -1;       // emqx_set_tuning("delta_max", n): filters placed by incremental
                                // commits before a full rebuild (-1: until the spare region is full)
  uint64_t last_commit_kind = 0;
  uint64_t last_relocations = 0, last_in_place = 0, last_patches = 0, last_new_slots = 0;
  double last_host_ms = 0;      // host part (LiveTrie::commit) of the last incremental commit
  uint64_t last_extents = 0, last_vocab_slots = 0;  // its new-slot extents and new vocab slots
  double last_upload_ms = 0;    // from the end of the host part to the end of the uploads + patches
  std::mutex hb_mu;             // pinned host batches of emqx_match_batch (pool)
  std::vector<emqx_host_batch*> hb_free;
  int commit_threads = std::max(1u, std::min(8u, std::thread::hardware_concurrency()));
  // walk order (emqx_set_tuning): "order" -1 auto (deep tables, batches of >= ORDER_MIN_N
  // topics) / 0 off / 1 on; "order_level_bits" key bits per level (0: 4 for deep tables, else
  // 8); "order_sort_bits" top key bits sorted on; "order_deal" XCD-contiguous tile ranges
  std::atomic<int> order{-1};
  std::atomic<int> order_level_bits{0};
  std::atomic<int> order_sort_bits{64};
  std::atomic<int> order_deal{1};
  std::atomic<uint64_t> last_ordered{0};
  std::atomic<uint64_t> order_bpt{48};  // reordered-batch bytes per topic to provision (learnt)
  std::atomic<double> last_order_ms{0};
  std::atomic<bool> small_batch{true};  // emqx_set_tuning("small_batch", 0|1): the one-launch path
};

namespace {

constexpr int EMQX_NEED_FULL = 1;  // internal: the incremental path cannot take this commit

void publish(emqx_engine* e, std::shared_ptr<Snapshot> s) {
  std::lock_guard<std::mutex> g(e->snap_mu);
  e->snap = std::move(s);  // the old snapshot goes when its last reader returns
}

// Full rebuild: every live filter into a fresh trie, uploaded into new device tables with a
// spare region for incremental commits; the old tables stay alive until their last reader
// returns.  The host keeps the build's image for incremental commits (LiveTrie::adopt).
int full_commit(emqx_engine* e) {
  auto vs = std::make_unique<VocabState>();
  std::vector<uint64_t> loc;
  std::vector<uint32_t> slot_ids;
  BuildOpts o;
  o.vocab = vs.get();
  o.fid_loc = &loc;
  o.slot_ids = &slot_ids;
  o.threads = e->commit_threads;
  HostTables ht;
  std::string err;
  if (!build_tables(e->store, o, ht, &err)) {
    set_last_error(err.c_str());
    return EMQX_ENOMEM;
  }
  const uint64_t n_slots = ht.edges.size();
  const uint64_t spare = std::min<uint64_t>(std::max<uint64_t>(1u << 20, n_slots / 2), MAX_SLOTS - n_slots);
  auto dt = std::make_shared<DeviceTables>();
  dt->device = e->device;
  dt->cap_slots = n_slots + spare;
  dt->n_vocab = ht.vocab.size();
  dt->cap_arena = ht.arena.size() + std::max<uint64_t>(1u << 20, ht.arena.size() / 4) + 16;
  HIP_TRY(dalloc(dt->edges, dt->cap_slots));
  HIP_TRY(dalloc(dt->fids, 2 * dt->cap_slots));
  HIP_TRY(dalloc(dt->vocab, dt->n_vocab));
  HIP_TRY(dalloc(dt->arena, dt->cap_arena));
  HIP_TRY(hipMemcpy(dt->edges, ht.edges.data(), n_slots * sizeof(EdgeSlot), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dt->fids, ht.fids.data(), ht.fids.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dt->vocab, ht.vocab.data(), ht.vocab.size() * sizeof(VocabSlot), hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(dt->arena, ht.arena.data(), ht.arena.size(), hipMemcpyHostToDevice));
  // a copy from pageable memory may return before its DMA lands, and the match streams do not
  // follow the null stream: the tables are on the device before the snapshot is published
  HIP_TRY(hipStreamSynchronize(nullptr));

  auto s = std::make_shared<Snapshot>();
  s->dt = dt;
  s->tv.edges = dt->edges;
  s->tv.fids = dt->fids;
  s->tv.vocab = dt->vocab;
  s->tv.arena = dt->arena;
  s->tv.vocab_mask = ht.vocab_mask;
  s->tv.root_base = ht.root_base;
  s->tv.root_meta = ht.root_meta;
  s->tv.root_hash_fid = ht.root_hash_fid;
  s->tv.plus_mask = ht.plus_mask;
  s->n_nodes = ht.n_nodes;
  s->n_slots = n_slots;
  s->n_words = ht.n_words;
  s->max_depth = ht.max_depth;
  s->bytes = dt->bytes();

  LiveState& d = e->ls;
  d.device = e->device;
  d.dt = dt;
  d.vocab = std::move(vs);
  if (!d.lt) d.lt = std::make_unique<LiveTrie>();
  d.lt->adopt(ht, loc, slot_ids, spare, d.vocab.get());
  d.valid = true;
  d.inserted = 0;
  d.base_live = e->store.n_live;
  e->dirty.clear();
  publish(e, std::move(s));
  e->last_commit_kind = 0;
  return EMQX_OK;
}

// Incremental commit: the filters inserted / deleted since the last commit are patched into
// the committed table (LiveTrie::apply), then the device gets the new spare-region slots and
// the rewritten existing slots on the commit stream, which alone is synchronised.  A walk that
// overlaps the commit sees each filter of it present or absent.  EMQX_NEED_FULL when the spare
// region, the vocab or the arena headroom runs out, e->delta_max is reached, or (delta_max
// unset) the filters placed since the full build reach half of the filters it held.
int live_commit(emqx_engine* e) {
  LiveState& d = e->ls;
  LiveTrie& lt = *d.lt;
  const FilterStore& fs = e->store;
  std::vector<uint32_t> ids(e->dirty);
  sort_unique_u32(ids);
  uint64_t creates = 0;
  for (uint32_t id : ids)
    if (fs.live[id] && (id >= lt.loc.size() || lt.loc[id] == FIDLOC_NONE)) ++creates;
  if (e->delta_max >= 0) {
    if (d.inserted + creates > static_cast<uint64_t>(e->delta_max)) return EMQX_NEED_FULL;
  } else if (creates && 2 * (d.inserted + creates) > d.base_live) {
    // default policy: once the table has grown by half since its build (and at the first
    // filters of an empty build), a fresh line-packed, perfect-hashed build serves it better
    return EMQX_NEED_FULL;
  }

  const uint64_t nw0 = d.vocab->n_words(), arena0 = d.vocab->arena.size();
  auto th0 = std::chrono::steady_clock::now();
  if (!lt.commit(fs, ids, e->commit_threads)) return EMQX_NEED_FULL;  // spare region exhausted: the
                                                                     // host image is rebuilt too
  e->last_host_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th0).count();
  std::vector<uint32_t> vdirty;
  if (!d.vocab->insert_table(nw0, &vdirty) || d.vocab->arena.size() + 16 > d.dt->cap_arena) return EMQX_NEED_FULL;
  lt.patches(d.patches);
  e->last_extents = lt.ranges.size();
  e->last_vocab_slots = vdirty.size();
  const auto tu0 = std::chrono::steady_clock::now();

  HIP_TRY(hipSetDevice(e->device));
  if (!d.stream) HIP_TRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  hipStream_t st = d.stream;
  for (const auto& r : lt.ranges) {  // the commit's new slots, extent by extent
    const uint64_t a0 = r.first, a1 = r.second;
    HIP_TRY(hipMemcpyAsync(d.dt->edges + a0, lt.edges.data() + a0, (a1 - a0) * sizeof(EdgeSlot),
                           hipMemcpyHostToDevice, st));
    HIP_TRY(hipMemcpyAsync(d.dt->fids + 2 * a0, lt.fids.data() + 2 * a0, 2 * (a1 - a0) * sizeof(uint32_t),
                           hipMemcpyHostToDevice, st));
  }
  if (d.vocab->arena.size() > arena0)
    HIP_TRY(hipMemcpyAsync(d.dt->arena + arena0, d.vocab->arena.data() + arena0, d.vocab->arena.size() - arena0,
                           hipMemcpyHostToDevice, st));
  for (uint32_t v : vdirty)
    HIP_TRY(hipMemcpyAsync(d.dt->vocab + v, &d.vocab->table[v], sizeof(VocabSlot), hipMemcpyHostToDevice, st));
  const uint64_t np = d.patches.size();
  if (np) {
    if (np > d.cap_patch) {
      HIP_TRY(hipStreamSynchronize(st));
      d.cap_patch = round_pow2(np);
      HIP_TRY(dalloc(d.d_patch, d.cap_patch));
    }
    HIP_TRY(hipMemcpyAsync(d.d_patch, d.patches.data(), np * sizeof(SlotPatch), hipMemcpyHostToDevice, st));
    HIP_TRY(launch_slot_patches(d.dt->edges, d.dt->fids, d.d_patch, static_cast<uint32_t>(np), st));
  }
  HIP_TRY(hipStreamSynchronize(st));
  e->last_upload_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tu0).count();

  std::shared_ptr<Snapshot> cur;
  {
    std::lock_guard<std::mutex> g(e->snap_mu);
    cur = e->snap;
  }
  auto s = std::make_shared<Snapshot>(*cur);
  s->tv.root_base = lt.root_base;
  s->tv.root_meta = lt.root_meta;
  s->tv.root_hash_fid = lt.root_hash_fid;
  s->n_nodes = lt.n_nodes;
  s->n_slots = lt.used;
  s->n_words = d.vocab->n_words();
  s->max_depth = lt.max_depth;
  d.inserted += creates;
  e->last_relocations = lt.relocations;
  e->last_in_place = lt.in_place;
  e->last_patches = np;
  e->last_new_slots = lt.new_slots();
  e->dirty.clear();
  publish(e, std::move(s));
  e->last_commit_kind = 1;
  return EMQX_OK;
}

int commit_locked(emqx_engine* e) {
  auto t0 = std::chrono::steady_clock::now();
  int rc = EMQX_NEED_FULL;
  if (e->incremental && e->ls.valid && e->snap) rc = live_commit(e);
  if (rc == EMQX_NEED_FULL) rc = full_commit(e);
  if (rc != EMQX_OK) return rc;
  e->epoch += 1;
  e->last_build_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return EMQX_OK;
}

// A free workspace for a call on stream `want` (null: the workspace's own stream).  Prefers
// one last used on that stream, then one whose last call has drained; otherwise a new one, so
// calls pipelined on different streams never wait for each other's workspace.
Workspace* acquire_ws(emqx_engine* e, hipStream_t want = nullptr) {
  std::lock_guard<std::mutex> g(e->ws_mu);
  auto& f = e->free_ws;
  auto take = [&](size_t i) {
    Workspace* w = f[i];
    f.erase(f.begin() + static_cast<std::ptrdiff_t>(i));
    w->slab_per_tile = std::max(w->slab_per_tile, e->slab_hint.load());
    return w;
  };
  if (!f.empty() && !want) return take(f.size() - 1);
  for (size_t i = f.size(); i-- > 0;)
    if (f[i]->last_stream == want || !f[i]->last_stream) return take(i);
  if (f.size() >= 8)  // many streams: reuse a drained workspace rather than grow the pool
    for (size_t i = f.size(); i-- > 0;)
      if (!f[i]->done || hipEventQuery(f[i]->done) == hipSuccess) return take(i);
  auto w = std::make_unique<Workspace>();
  w->device = e->device;
  w->slab_per_tile = std::max(w->slab_per_tile, e->slab_hint.load());
  Workspace* p = w.get();
  e->all_ws.push_back(std::move(w));
  return p;
}

void release_ws(emqx_engine* e, Workspace* w) {
  std::lock_guard<std::mutex> g(e->ws_mu);
  e->free_ws.push_back(w);
}

int ensure_ws(Workspace* w, uint64_t n) {
  if (!w->stream) {
    HIP_TRY(hipStreamCreateWithFlags(&w->stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreate(&w->ev0));
    HIP_TRY(hipEventCreate(&w->ev1));
    HIP_TRY(hipEventCreate(&w->evk));
    HIP_TRY(hipEventCreate(&w->evo));
    HIP_TRY(hipEventCreateWithFlags(&w->done, hipEventDisableTiming));
    HIP_TRY(hipHostMalloc(reinterpret_cast<void**>(&w->h_rb), SUM_WORDS * sizeof(uint64_t), hipHostMallocDefault));
    HIP_TRY(dalloc(w->ctrl, CTRL_WORDS));
    HIP_TRY(dalloc(w->diag, DIAG_WORDS));
    HIP_TRY(hipMemset(w->diag, 0, DIAG_WORDS * sizeof(uint64_t)));
  }
  if (!w->deep_ready) {
    HIP_TRY(dalloc(w->deep_wids, uint64_t(DEEP_WAVES) * DEEP_MAX_LEVELS));
    HIP_TRY(dalloc(w->deep_stack, uint64_t(DEEP_WAVES) * w->deep_stack_cap));
    HIP_TRY(dalloc(w->deep_slab, w->deep_slab_cap));
    w->deep_ready = true;
  }
  if (n > w->cap_n) {
    const uint64_t cap = round_pow2(std::max<uint64_t>(n, 1024));
    HIP_TRY(dalloc(w->counts, cap));
    HIP_TRY(dalloc(w->deferred, cap));
    HIP_TRY(dalloc(w->deep_rank, cap));
    w->cap_n = cap;
  }
  const uint64_t ntiles = (n + TILE_TOPICS - 1) / TILE_TOPICS;
  if (ntiles > w->cap_tiles || w->cap_tiles == 0) {
    const uint64_t cap = round_pow2(std::max<uint64_t>(ntiles, 64));
    HIP_TRY(dalloc(w->tile_fill, cap));
    HIP_TRY(dalloc(w->tile_defer, cap));
    HIP_TRY(dalloc(w->tile_sum, cap));
    HIP_TRY(dalloc(w->tile_stats, cap));
    HIP_TRY(dalloc(w->group_sum, cap / GROUP_TILES + 1));
    HIP_TRY(dalloc(w->group_stats, cap / GROUP_TILES + 1));
    HIP_TRY(dalloc(w->spill, cap * w->spill_cap));
    w->cap_tiles = cap;
  }
  const uint64_t need_slab = std::max<uint64_t>(ntiles, 1) * w->slab_per_tile;
  if (need_slab > w->cap_slab) {
    const uint64_t cap = need_slab;
    HIP_TRY(dalloc(w->slab, cap));
    w->cap_slab = cap;
  }
  return EMQX_OK;
}

constexpr uint64_t ORDER_MIN_N = 65536;

bool use_order(const emqx_engine* e, const Snapshot& snap, uint64_t n) {
  if (n > 0xFFFFFFFFull) return false;  // batch positions are 32-bit
  const int o = e->order.load();
  if (o >= 0) return o > 0 && n > 0;
  return snap.max_depth > 12 && n >= ORDER_MIN_N;
}

// Walk-order buffers for n topics; the reordered bytes buffer keeps `cap_bytes` (grown by
// run_match when a call reports CTRL_ERR_ORDER_CAP).
int ensure_order(emqx_engine* e, Workspace* w, uint64_t n, uint32_t sort_bits) {
  if (n > w->ord_cap_n) {
    const uint64_t cap = round_pow2(std::max<uint64_t>(n, 1024));
    HIP_TRY(dalloc(w->ord_keys, cap));
    HIP_TRY(dalloc(w->ord_keys_out, cap));
    HIP_TRY(dalloc(w->ord_idx, cap));
    HIP_TRY(dalloc(w->ord_perm, cap));
    HIP_TRY(dalloc(w->ord_lens, cap));
    HIP_TRY(dalloc(w->ord_corig, cap));
    HIP_TRY(dalloc(w->ord_noffs, cap + 1));
    HIP_TRY(dalloc(w->ord_partials, scan_partials(cap)));
    w->ord_cap_n = cap;
  }
  const uint64_t tb = order_sort_temp_bytes(n, sort_bits);
  if (!w->ord_temp || tb > w->ord_temp_bytes) {
    HIP_TRY(dalloc(w->ord_temp, tb));
    w->ord_temp_bytes = tb;
  }
  const uint64_t want = e->order_bpt.load() * n + 4096;
  if (!w->ord_bytes || w->ord_cap_bytes < want) {
    const uint64_t cap = std::max<uint64_t>(w->ord_cap_bytes, want);
    HIP_TRY(dalloc(w->ord_bytes, cap + 16));
    w->ord_cap_bytes = cap;
  }
  return EMQX_OK;
}

// Fast-kernel variant: EMQX_FAST_VARIANT overrides (A/B runs); otherwise deep tables get
// the 2K-item stack and everything else the 384-item stack, one item per lane (26 waves/CU).
FastVariant pick_variant(const emqx_engine* e, const Snapshot& snap) {
  static const int env_forced = [] {
    const char* v = getenv("EMQX_FAST_VARIANT");
    return v ? atoi(v) : -1;
  }();
  const int fv = e->forced_variant.load();
  const int forced = fv >= 0 ? fv : env_forced;
  if (forced >= 0 && forced < FAST_NVARIANTS) return static_cast<FastVariant>(forced);
  // shallow tables: FAST_K1_S384's walk in one-wave workgroups (round 5: the waves share
  // nothing, and single-wave groups let the dispatcher refill a CU wave by wave; config B 0.5591
  // against 0.5668 ms for 4-wave groups, profiles/r5_b1_ab_block_waves.json)
  return snap.max_depth > 12 ? FAST_K1_S512W : FAST_K1_S384B1;
}

// Enqueue one match call on stream s (no host synchronisation): memset of the control
// words, fast kernel, deep kernel, tile scan (+ summary into `summary`), scatter.  A call on
// a workspace last used from another stream first waits for that call to drain.
// The MatchArgs of one call on workspace w (the batched and the small-batch launches).
MatchArgs match_args(emqx_engine* e, const Snapshot& snap, Workspace* w, uint32_t mode, const uint8_t* d_tbytes,
                     const uint64_t* d_toffs, uint64_t n, uint64_t* d_out_off, uint32_t* d_out_ids, uint64_t cap,
                     uint64_t* summary) {
  MatchArgs a{};
  a.tv = snap.tv;
  a.tbytes = d_tbytes;
  a.toffs = d_toffs;
  a.n = n;
  a.mode = mode;
  a.slab_cap = w->slab_per_tile;
  a.counts = w->counts;
  a.slab = w->slab;
  a.tile_fill = w->tile_fill;
  a.tile_defer = w->tile_defer;
  a.spill = w->spill;
  a.diag = e->diag_on.load() ? w->diag : nullptr;
  a.diag_stop = a.diag ? e->diag_stop.load() : 0u;
  a.timeline = a.diag && e->timeline && (n + TILE_TOPICS - 1) / TILE_TOPICS <= e->timeline_cap ? e->timeline : nullptr;
  a.spill_cap = w->spill_cap;
  a.ctrl = w->ctrl;
  a.deferred = w->deferred;
  a.deep_wids = w->deep_wids;
  a.deep_stack = w->deep_stack;
  a.deep_stack_cap = w->deep_stack_cap;
  a.deep_waves = DEEP_WAVES;
  a.deep_slab = w->deep_slab;
  a.deep_slab_cap = w->deep_slab_cap;
  a.tile_sum = w->tile_sum;
  a.tile_stats = w->tile_stats;
  a.group_sum = w->group_sum;
  a.group_stats = w->group_stats;
  a.ngroups = static_cast<uint32_t>((n + TILE_TOPICS * GROUP_TILES - 1) / (TILE_TOPICS * GROUP_TILES));
  a.deep_rank = w->deep_rank;
  a.out_off = d_out_off;
  a.out_ids = d_out_ids;
  a.out_cap = d_out_ids ? cap : 0;
  a.summary = summary;
  return a;
}

int enqueue_match(emqx_engine* e, const Snapshot& snap, Workspace* w, uint32_t mode, const uint8_t* d_tbytes,
                  const uint64_t* d_toffs, uint64_t n, uint64_t* d_out_off, uint32_t* d_out_ids, uint64_t cap,
                  uint64_t* summary, hipStream_t s) {
  int rc = ensure_ws(w, n);
  if (rc != EMQX_OK) return rc;
  MatchArgs a = match_args(e, snap, w, mode, d_tbytes, d_toffs, n, d_out_off, d_out_ids, cap, summary);
  const bool ordered = use_order(e, snap, n);
  const uint32_t sort_bits = static_cast<uint32_t>(std::min(64, std::max(1, e->order_sort_bits.load())));
  if (ordered) {
    rc = ensure_order(e, w, n, sort_bits);
    if (rc != EMQX_OK) return rc;
  }

  HIP_TRY(hipStreamWaitEvent(s, w->done, 0));
  w->last_stream = s;
  HIP_TRY(hipMemsetAsync(w->ctrl, 0, CTRL_WORDS * sizeof(uint32_t), s));
  w->ordered = ordered;
  if (ordered) {
    HIP_TRY(hipEventRecord(w->evo, s));
    OrderArgs o{};
    o.tbytes = d_tbytes;
    o.toffs = d_toffs;
    o.n = n;
    const int lb = e->order_level_bits.load();
    o.level_bits = static_cast<uint32_t>(lb > 0 ? std::min(lb, 32) : (snap.max_depth > 12 ? 4 : 8));
    o.sort_bits = sort_bits;
    o.keys = w->ord_keys;
    o.keys_out = w->ord_keys_out;
    o.idx = w->ord_idx;
    o.perm = w->ord_perm;
    o.lens = w->ord_lens;
    o.noffs = w->ord_noffs;
    o.partials = w->ord_partials;
    o.obytes = w->ord_bytes;
    o.cap_bytes = w->ord_cap_bytes;
    o.temp = w->ord_temp;
    o.temp_bytes = w->ord_temp_bytes;
    o.ctrl = w->ctrl;
    HIP_TRY(launch_order(o, s));
    a.tbytes = w->ord_bytes;
    a.toffs = w->ord_noffs;
    a.perm = w->ord_perm;
    a.deal = e->order_deal.load() ? 1u : 0u;
    a.corig = w->ord_corig;
    a.partials = w->ord_partials;
  }
  HIP_TRY(hipEventRecord(w->ev0, s));
  HIP_TRY(launch_match_fast(a, pick_variant(e, snap), s));
  HIP_TRY(hipEventRecord(w->evk, s));
  HIP_TRY(launch_match_deep(a, s));
  HIP_TRY(launch_assemble(a, s));
  HIP_TRY(hipEventRecord(w->ev1, s));
  HIP_TRY(hipEventRecord(w->done, s));
  return EMQX_OK;
}

// The pipeline on device buffers, synchronous: enqueue, drain, read the summary, rerun with
// larger scratch areas if one overflowed (learnt once per workspace).
int run_match(emqx_engine* e, const Snapshot& snap, Workspace* w, uint32_t mode, const uint8_t* d_tbytes,
              const uint64_t* d_toffs, uint64_t n, uint64_t* d_out_off, uint32_t* d_out_ids, uint64_t cap,
              uint64_t* n_out, hipStream_t s) {
  uint64_t* sum_dev = nullptr;
  HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&sum_dev), w->h_rb, 0));
  for (int attempt = 0; attempt < 8; ++attempt) {
    int rc = enqueue_match(e, snap, w, mode, d_tbytes, d_toffs, n, d_out_off, d_out_ids, cap, sum_dev, s);
    if (rc != EMQX_OK) return rc;
    HIP_TRY(hipStreamSynchronize(s));
    const uint64_t* sm = w->h_rb;
    const uint64_t flags = sm[SUM_FLAGS];
    const uint32_t err = static_cast<uint32_t>(sm[SUM_ERROR]);
    if (flags & SUM_F_ERROR) {
      set_last_error("topic longer than 65535 bytes on the deep path");
      return EMQX_EINVAL;
    }
    if (flags & SUM_F_RETRY) {
      if (sm[SUM_NEED_SLAB] > w->slab_per_tile) {
        // the learnt need plus 1/8, in whole 512-entry (4 KiB) blocks: a power of two would
        // nearly double the slab on a '#'-rich table (config D: 16 GB instead of ~9 GB per
        // workspace), and every stream in flight holds its own
        const uint64_t need = sm[SUM_NEED_SLAB];
        w->slab_per_tile = static_cast<uint32_t>(((need + need / 8) + 511) / 512 * 512);
        uint32_t h = e->slab_hint.load();  // later workspaces start at the learnt size
        while (h < w->slab_per_tile && !e->slab_hint.compare_exchange_weak(h, w->slab_per_tile)) {
        }
      }
      if (err & CTRL_ERR_DEEP_SLAB) {
        w->deep_slab_cap = static_cast<uint32_t>(std::min<uint64_t>(round_pow2(sm[SUM_DEEP_FILL] + uint64_t(DEEP_WAVES) * DEEP_CHUNK + 1), 1u << 30));
        HIP_TRY(dalloc(w->deep_slab, w->deep_slab_cap));
      }
      if (err & CTRL_ERR_ORDER_CAP) {  // the batch's byte count, read once, sizes the reordered copy
        uint64_t nb = 0;
        HIP_TRY(hipMemcpy(&nb, d_toffs + n, sizeof(uint64_t), hipMemcpyDeviceToHost));
        uint64_t nb0 = 0;
        HIP_TRY(hipMemcpy(&nb0, d_toffs, sizeof(uint64_t), hipMemcpyDeviceToHost));
        const uint64_t need = nb - nb0;
        w->ord_cap_bytes = need + need / 8 + 4096;
        HIP_TRY(dalloc(w->ord_bytes, w->ord_cap_bytes + 16));
        const uint64_t bpt = (need + need / 8) / std::max<uint64_t>(n, 1) + 1;  // later workspaces start there
        uint64_t h = e->order_bpt.load();
        while (h < bpt && !e->order_bpt.compare_exchange_weak(h, bpt)) {
        }
      }
      if (err & CTRL_ERR_TOO_DEEP) {
        if (w->deep_stack_cap >= (1u << 22)) {
          set_last_error("topic frontier exceeds the deep path's stack");
          return EMQX_ETOODEEP;
        }
        w->deep_stack_cap <<= 2;
        HIP_TRY(dalloc(w->deep_stack, uint64_t(DEEP_WAVES) * w->deep_stack_cap));
      }
      continue;
    }
    float kms = 0, ms = 0;
    if (hipEventElapsedTime(&kms, w->ev0, w->evk) == hipSuccess) e->last_kernel_ms.store(kms);
    (void)hipEventElapsedTime(&ms, w->ev0, w->ev1);
    float oms = 0;
    if (w->ordered && hipEventElapsedTime(&oms, w->evo, w->ev0) == hipSuccess) ms += oms;
    e->last_match_ms.store(ms);  // the call: reordering (if any) + match pipeline
    e->last_order_ms.store(w->ordered ? oms : 0.0);
    e->last_ordered.store(w->ordered ? 1 : 0);
    e->last_deferred.store(sm[SUM_DEFERRED]);
    e->last_evals.store(sm[SUM_EVALS]);
    e->last_max_stack.store(sm[SUM_MAXSTACK]);
    *n_out = sm[SUM_TOTAL];
    return (flags & SUM_F_OVERFLOW) ? EMQX_EOVERFLOW : EMQX_OK;
  }
  set_last_error("match did not converge");
  return EMQX_EDEVICE;
}

std::shared_ptr<Snapshot> current(emqx_engine* e) {
  std::lock_guard<std::mutex> g(e->snap_mu);
  return e->snap;
}

// A batch the one-launch small path takes (kernels.h SmallArgs): at most SMALL_MAX_N topics of a
// table within the shallow variant's depth, no walk order, no diagnostic counters.
bool small_ok(const emqx_engine* e, const Snapshot& snap, uint64_t n) {
  return e->small_batch.load() && n > 0 && n <= SMALL_MAX_N && snap.max_depth <= 12 && !e->diag_on.load() &&
         !use_order(e, snap, n);
}

// Enqueue a small batch as one kernel on s: inputs read from host-mapped pinned memory (copied to
// d_tbytes / d_toffs on the way), the match CSR into d_out_off / d_out_ids, the summary into
// host-mapped `summary`; then the CSR into host-mapped h_out_off / h_out_ids (match only), or the
// fan-out f straight into its pinned buffers.
int enqueue_small(emqx_engine* e, const Snapshot& snap, Workspace* w, uint32_t mode, const uint8_t* h_tbytes,
                  const uint64_t* h_toffs, uint64_t n, uint64_t nbytes, uint8_t* d_tbytes, uint64_t* d_toffs,
                  uint64_t* d_out_off, uint32_t* d_out_ids, uint64_t cap, uint64_t* summary, uint64_t* h_out_off,
                  uint32_t* h_out_ids, uint64_t h_cap, const SmallFanout* f, hipStream_t s) {
  // the workspace sized for SMALL_WAVES tiles whatever n: the kernel's tiles are ceil(n / 16)
  // topics wide, so a batch of a few topics still spans up to 16 slab tiles
  int rc = ensure_ws(w, SMALL_MAX_N);
  if (rc != EMQX_OK) return rc;
  SmallArgs sa{};
  sa.m = match_args(e, snap, w, mode, d_tbytes, d_toffs, n, d_out_off, d_out_ids, cap, summary);
  sa.m.diag = nullptr;
  sa.h_tbytes = h_tbytes;
  sa.h_toffs = h_toffs;
  sa.nbytes = nbytes;
  sa.tt = static_cast<uint32_t>((n + SMALL_WAVES - 1) / SMALL_WAVES);
  sa.slab_tiles = static_cast<uint32_t>(std::min<uint64_t>(w->cap_slab / w->slab_per_tile, w->cap_tiles));
  sa.h_out_off = h_out_off;
  sa.h_out_ids = h_out_ids;
  sa.h_cap = h_cap;
  // the phase clock: a timeline of >= SMALL_CLK_WORDS / 2 tiles with diag off (tools/small_clock.py)
  sa.clk = e->timeline && e->timeline_cap * 2 >= SMALL_CLK_WORDS ? reinterpret_cast<uint64_t*>(e->timeline) : nullptr;
  if (f) {
    sa.has_fanout = 1;
    sa.f = *f;
  }
  HIP_TRY(hipStreamWaitEvent(s, w->done, 0));
  w->last_stream = s;
  w->ordered = false;
  HIP_TRY(launch_small_batch(sa, s));
  HIP_TRY(hipEventRecord(w->done, s));
  return EMQX_OK;
}

// Device side of a pinned host batch (include/emqx_match.h, emqx_host_batch_*).
struct HostBatchPriv {
  emqx_engine* e = nullptr;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  uint8_t* d_tbytes = nullptr;
  uint64_t* d_toffs = nullptr;
  uint64_t* d_out_off = nullptr;
  uint32_t* d_out_ids = nullptr;
  uint64_t* summary = nullptr;  // pinned, SUM_WORDS
  std::shared_ptr<Snapshot> snap;
  std::shared_ptr<Snapshot> pin;  // set by emqx_match_batch: every chunk of one call reads one table version
  uint32_t mode = 0;
  bool pending = false;
  uint64_t evals = 0, deferred = 0, max_stack = 0;  // of the last call
};

template <class T>
hipError_t halloc(T*& p, uint64_t count) {
  if (p) (void)hipHostFree(p);
  p = nullptr;
  return hipHostMalloc(reinterpret_cast<void**>(&p), std::max<uint64_t>(count, 1) * sizeof(T), hipHostMallocDefault);
}

int hb_alloc(emqx_host_batch* b, uint64_t cap_topics, uint64_t cap_bytes, uint64_t cap_ids, bool keep_inputs) {
  auto* p = static_cast<HostBatchPriv*>(b->priv);
  HIP_TRY(hipSetDevice(p->e->device));
  if (cap_topics > b->cap_topics) {
    uint64_t* t = nullptr;
    HIP_TRY(halloc(t, cap_topics + 1));
    if (keep_inputs && b->topic_offsets) std::memcpy(t, b->topic_offsets, (b->cap_topics + 1) * sizeof(uint64_t));
    if (b->topic_offsets) (void)hipHostFree(b->topic_offsets);
    b->topic_offsets = t;
    HIP_TRY(halloc(b->out_offsets, cap_topics + 1));
    HIP_TRY(dalloc(p->d_toffs, cap_topics + 1));
    HIP_TRY(dalloc(p->d_out_off, cap_topics + 1));
    b->cap_topics = cap_topics;
  }
  if (cap_bytes > b->cap_bytes) {
    uint8_t* t = nullptr;
    HIP_TRY(halloc(t, cap_bytes + 16));
    if (keep_inputs && b->topic_bytes) std::memcpy(t, b->topic_bytes, b->cap_bytes);
    if (b->topic_bytes) (void)hipHostFree(b->topic_bytes);
    b->topic_bytes = t;
    HIP_TRY(dalloc(p->d_tbytes, cap_bytes + 16));
    b->cap_bytes = cap_bytes;
  }
  if (cap_ids > b->cap_ids) {
    HIP_TRY(halloc(b->out_ids, cap_ids));
    HIP_TRY(dalloc(p->d_out_ids, cap_ids));
    b->cap_ids = cap_ids;
  }
  return EMQX_OK;
}

// Enqueue: inputs to HBM (DMA from pinned memory), the match pipeline, the CSR back into the
// pinned outputs; one event at the end.
int hb_enqueue(emqx_host_batch* b) {
  auto* p = static_cast<HostBatchPriv*>(b->priv);
  emqx_engine* e = p->e;
  const uint64_t n = b->n, nbytes = n ? b->topic_offsets[n] : 0;
  hipStream_t s = p->stream;
  uint64_t* sum_dev = nullptr;
  HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&sum_dev), p->summary, 0));
  p->snap = p->pin ? p->pin : current(e);
  if (small_ok(e, *p->snap, n)) {  // one launch: the batch read from and the CSR written to pinned memory
    const uint8_t* h_tb = nullptr;
    const uint64_t* h_to = nullptr;
    uint64_t* h_off = nullptr;
    uint32_t* h_ids = nullptr;
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(const_cast<uint8_t**>(&h_tb)), b->topic_bytes, 0));
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(const_cast<uint64_t**>(&h_to)), b->topic_offsets, 0));
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_off), b->out_offsets, 0));
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_ids), b->out_ids, 0));
    Workspace* w = acquire_ws(e, s);
    int rc = enqueue_small(e, *p->snap, w, p->mode, h_tb, h_to, n, nbytes, p->d_tbytes, p->d_toffs, p->d_out_off,
                           p->d_out_ids, b->cap_ids, sum_dev, h_off, h_ids, b->cap_ids, nullptr, s);
    if (rc == EMQX_OK) w->inflight = p->snap;
    release_ws(e, w);
    if (rc != EMQX_OK) return rc;
    HIP_TRY(hipEventRecord(p->done, s));
    p->pending = true;
    return EMQX_OK;
  }
  if (nbytes) HIP_TRY(hipMemcpyAsync(p->d_tbytes, b->topic_bytes, nbytes, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(p->d_toffs, b->topic_offsets, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, s));
  Workspace* w = acquire_ws(e, s);
  int rc = ensure_ws(w, n);
  if (rc == EMQX_OK)
    rc = enqueue_match(e, *p->snap, w, p->mode, p->d_tbytes, p->d_toffs, n, p->d_out_off, p->d_out_ids, b->cap_ids,
                       sum_dev, s);
  if (rc == EMQX_OK) w->inflight = p->snap;
  release_ws(e, w);
  if (rc != EMQX_OK) return rc;
  uint64_t *h_off = nullptr;
  uint32_t* h_ids = nullptr;
  HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_off), b->out_offsets, 0));
  HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_ids), b->out_ids, 0));
  HIP_TRY(launch_csr_to_host(p->d_out_off, n, p->d_out_ids, b->cap_ids, h_off, h_ids, s));
  HIP_TRY(hipEventRecord(p->done, s));
  p->pending = true;
  return EMQX_OK;
}

int hb_wait(emqx_host_batch* b) {
  auto* p = static_cast<HostBatchPriv*>(b->priv);
  if (!p->pending) return EMQX_EINVAL;
  HIP_TRY(hipSetDevice(p->e->device));
  p->pending = false;
  HIP_TRY(hipEventSynchronize(p->done));
  uint64_t flags = p->summary[SUM_FLAGS];
  uint64_t total = p->summary[SUM_TOTAL];
  if (flags & SUM_F_RETRY) {  // a scratch area overflowed: the synchronous path grows it and reruns
    Workspace* w = acquire_ws(p->e, p->stream);
    int rc = ensure_ws(w, b->n);
    if (rc == EMQX_OK)
      rc = run_match(p->e, *p->snap, w, p->mode, p->d_tbytes, p->d_toffs, b->n, p->d_out_off, p->d_out_ids,
                     b->cap_ids, &total, p->stream);
    release_ws(p->e, w);
    if (rc != EMQX_OK && rc != EMQX_EOVERFLOW) return rc;
    uint64_t *h_off = nullptr;
    uint32_t* h_ids = nullptr;
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_off), b->out_offsets, 0));
    HIP_TRY(hipHostGetDevicePointer(reinterpret_cast<void**>(&h_ids), b->out_ids, 0));
    HIP_TRY(launch_csr_to_host(p->d_out_off, b->n, p->d_out_ids, b->cap_ids, h_off, h_ids, p->stream));
    HIP_TRY(hipStreamSynchronize(p->stream));
    flags = total > b->cap_ids ? SUM_F_OVERFLOW : 0;
  } else if (flags & SUM_F_ERROR) {
    set_last_error("topic longer than 65535 bytes on the deep path");
    return EMQX_EINVAL;
  }
  p->snap.reset();
  b->n_out = total;
  if (!(flags & SUM_F_RETRY)) {  // (run_match already recorded a rerun's numbers)
    p->evals = p->summary[SUM_EVALS];
    p->deferred = p->summary[SUM_DEFERRED];
    p->max_stack = p->summary[SUM_MAXSTACK];
    p->e->last_evals.store(p->evals);
    p->e->last_deferred.store(p->deferred);
    p->e->last_max_stack.store(p->max_stack);
  } else {
    p->evals = p->e->last_evals.load();
    p->deferred = p->e->last_deferred.load();
    p->max_stack = p->e->last_max_stack.load();
  }
  return (flags & SUM_F_OVERFLOW) ? EMQX_EOVERFLOW : EMQX_OK;
}

}  // namespace

int emqx::engine_small_batch(emqx_engine* e, uint32_t mode, const uint8_t* h_tbytes, const uint64_t* h_toffs,
                             uint64_t n, uint64_t nbytes, uint8_t* d_tbytes, uint64_t* d_toffs, uint64_t* d_out_off,
                             uint32_t* d_out_ids, uint64_t cap, uint64_t* h_summary, const SmallFanout& f,
                             hipStream_t s) {
  auto snap = current(e);
  if (!small_ok(e, *snap, n)) return SMALL_NOT_TAKEN;
  HIP_TRY(hipSetDevice(e->device));
  Workspace* w = acquire_ws(e, s);
  int rc = enqueue_small(e, *snap, w, mode, h_tbytes, h_toffs, n, nbytes, d_tbytes, d_toffs, d_out_off, d_out_ids,
                         cap, h_summary, nullptr, nullptr, 0, &f, s);
  if (rc == EMQX_OK) w->inflight = snap;
  release_ws(e, w);
  return rc;
}

namespace {

bool offsets_ok(const uint64_t* offs, uint64_t n) {
  if (!offs) return n == 0;
  for (uint64_t i = 0; i < n; ++i)
    if (offs[i + 1] < offs[i]) return false;
  return true;
}

}  // namespace

extern "C" {

int emqx_engine_create(const emqx_engine_opts* opts, emqx_engine** out) {
  if (!out) return EMQX_EINVAL;
  *out = nullptr;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
    set_last_error("no HIP device");
    return EMQX_EDEVICE;
  }
  int dev = 0;
  if (opts && opts->device >= 0) dev = opts->device;
  else (void)hipGetDevice(&dev);
  if (dev >= ndev) return EMQX_EINVAL;
  HIP_TRY(hipSetDevice(dev));
  auto* e = new (std::nothrow) emqx_engine();
  if (!e) return EMQX_ENOMEM;
  e->device = dev;
  int rc = commit_locked(e);  // empty snapshot
  if (rc != EMQX_OK) {
    delete e;
    return rc;
  }
  e->epoch = 0;
  *out = e;
  return EMQX_OK;
}

int emqx_engine_destroy(emqx_engine* e) {
  if (!e) return EMQX_EINVAL;
  (void)hipSetDevice(e->device);
  for (emqx_host_batch* b : e->hb_free) emqx_host_batch_destroy(b);
  e->hb_free.clear();
  dfree(e->timeline);
  delete e;
  return EMQX_OK;
}

int emqx_insert_filters(emqx_engine* e, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                        uint32_t* ids_out) {
  if (!e || (n && (!offsets || (!bytes && offsets[n] != offsets[0])))) return EMQX_EINVAL;
  if (!offsets_ok(offsets, n)) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(e->writer);
  for (uint64_t i = 0; i < n; ++i) {
    bool created = false;
    const uint32_t id = e->store.insert(bytes + offsets[i], offsets[i + 1] - offsets[i], &created);
    e->dirty.push_back(id);
    if (ids_out) ids_out[i] = id;
  }
  return EMQX_OK;
}

int emqx_insert_filters_ext(emqx_engine* e, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                            const uint32_t* ext_ids, uint32_t* ids_out) {
  if (!e || !ext_ids || (n && (!offsets || (!bytes && offsets[n] != offsets[0])))) return EMQX_EINVAL;
  if (!offsets_ok(offsets, n)) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(e->writer);
  for (uint64_t i = 0; i < n; ++i) {
    bool created = false;
    const uint32_t id = e->store.insert(bytes + offsets[i], offsets[i + 1] - offsets[i], &created);
    if (e->store.ext[id] != ext_ids[i]) e->ls.valid = false;  // a changed report id: rebuild
    e->store.ext[id] = ext_ids[i];
    e->dirty.push_back(id);
    if (ids_out) ids_out[i] = id;
  }
  return EMQX_OK;
}

int emqx_delete_filters(emqx_engine* e, const uint32_t* ids, uint64_t n) {
  if (!e || (n && !ids)) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(e->writer);
  for (uint64_t i = 0; i < n; ++i)  // all or nothing: an unknown id leaves the store unchanged
    if (ids[i] >= e->store.n_ids()) return EMQX_ENOTFOUND;
  for (uint64_t i = 0; i < n; ++i) {
    if (e->store.live[ids[i]]) {
      e->store.live[ids[i]] = 0;
      e->store.n_live -= 1;
      e->dirty.push_back(ids[i]);
    }
  }
  return EMQX_OK;
}

int emqx_lookup_filter(emqx_engine* e, const uint8_t* bytes, uint64_t len, uint32_t* id_out) {
  if (!e || !id_out || (len && !bytes)) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(e->writer);
  const uint32_t id = e->store.find(bytes, len);
  if (id == WID_NONE || !e->store.live[id]) return EMQX_ENOTFOUND;
  *id_out = id;
  return EMQX_OK;
}

int emqx_filter_name(emqx_engine* e, uint32_t id, uint8_t* buf, uint64_t cap, uint64_t* len_out) {
  if (!e || !len_out) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(e->writer);
  if (id >= e->store.n_ids()) return EMQX_ENOTFOUND;
  const uint64_t len = e->store.off[id + 1] - e->store.off[id];
  *len_out = len;
  if (buf && cap) std::memcpy(buf, e->store.bytes.data() + e->store.off[id], std::min(len, cap));
  return EMQX_OK;
}

int emqx_commit(emqx_engine* e) {
  if (!e) return EMQX_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  std::lock_guard<std::mutex> g(e->writer);
  return commit_locked(e);
}

int emqx_match_batch_device(emqx_engine* e, uint32_t mode, const uint8_t* d_topic_bytes,
                            const uint64_t* d_topic_offsets, uint64_t n, uint64_t* d_out_offsets,
                            uint32_t* d_out_ids, uint64_t cap, uint64_t* n_out, void* stream) {
  if (!e || !n_out || mode > EMQX_MODE_TRIE_WILDCARD) return EMQX_EINVAL;
  if (n && (!d_topic_bytes || !d_topic_offsets)) return EMQX_EINVAL;
  if (!d_out_offsets) return EMQX_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  auto snap = current(e);
  Workspace* w = acquire_ws(e, static_cast<hipStream_t>(stream));
  int rc = ensure_ws(w, n);
  if (rc == EMQX_OK) {
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : w->stream;
    if (!stream && after_null_stream(s) != hipSuccess) rc = EMQX_EDEVICE;
    if (rc == EMQX_OK)
      rc = run_match(e, *snap, w, mode, d_topic_bytes, d_topic_offsets, n, d_out_offsets, d_out_ids, cap, n_out, s);
  }
  release_ws(e, w);
  return rc;
}

int emqx_match_batch_device_async(emqx_engine* e, uint32_t mode, const uint8_t* d_topic_bytes,
                                  const uint64_t* d_topic_offsets, uint64_t n, uint64_t* d_out_offsets,
                                  uint32_t* d_out_ids, uint64_t cap, uint64_t* summary, void* stream) {
  if (!e || !summary || mode > EMQX_MODE_TRIE_WILDCARD) return EMQX_EINVAL;
  if (n && (!d_topic_bytes || !d_topic_offsets)) return EMQX_EINVAL;
  if (!d_out_offsets) return EMQX_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  auto snap = current(e);
  Workspace* w = acquire_ws(e, static_cast<hipStream_t>(stream));
  int rc = ensure_ws(w, n);
  if (rc == EMQX_OK) {
    hipStream_t s = stream ? static_cast<hipStream_t>(stream) : w->stream;
    if (!stream && after_null_stream(s) != hipSuccess) rc = EMQX_EDEVICE;
    if (rc == EMQX_OK)
      rc = enqueue_match(e, *snap, w, mode, d_topic_bytes, d_topic_offsets, n, d_out_offsets, d_out_ids, cap,
                       summary, s);
    w->inflight = snap;  // released when the workspace is next used (its stream has moved on)
  }
  release_ws(e, w);
  return rc;
}

int emqx_host_batch_create(emqx_engine* e, uint64_t cap_topics, uint64_t cap_bytes, uint64_t cap_ids,
                           emqx_host_batch** out) {
  if (!e || !out) return EMQX_EINVAL;
  *out = nullptr;
  auto* b = new (std::nothrow) emqx_host_batch();
  auto* p = new (std::nothrow) HostBatchPriv();
  if (!b || !p) {
    delete b;
    delete p;
    return EMQX_ENOMEM;
  }
  std::memset(b, 0, sizeof(*b));
  b->priv = p;
  p->e = e;
  int rc = EMQX_OK;
  if (hipSetDevice(e->device) != hipSuccess || hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&p->done, hipEventDisableTiming) != hipSuccess || halloc(p->summary, SUM_WORDS) != hipSuccess)
    rc = EMQX_EDEVICE;
  if (rc == EMQX_OK)
    rc = hb_alloc(b, std::max<uint64_t>(cap_topics, 1), std::max<uint64_t>(cap_bytes, 64), std::max<uint64_t>(cap_ids, 64),
                  false);
  if (rc != EMQX_OK) {
    emqx_host_batch_destroy(b);
    return rc;
  }
  *out = b;
  return EMQX_OK;
}

int emqx_host_batch_destroy(emqx_host_batch* b) {
  if (!b) return EMQX_EINVAL;
  auto* p = static_cast<HostBatchPriv*>(b->priv);
  (void)hipSetDevice(p->e->device);
  if (p->stream) (void)hipStreamSynchronize(p->stream);
  if (b->topic_bytes) (void)hipHostFree(b->topic_bytes);
  if (b->topic_offsets) (void)hipHostFree(b->topic_offsets);
  if (b->out_offsets) (void)hipHostFree(b->out_offsets);
  if (b->out_ids) (void)hipHostFree(b->out_ids);
  if (p->summary) (void)hipHostFree(p->summary);
  dfree(p->d_tbytes);
  dfree(p->d_toffs);
  dfree(p->d_out_off);
  dfree(p->d_out_ids);
  if (p->done) (void)hipEventDestroy(p->done);
  if (p->stream) (void)hipStreamDestroy(p->stream);
  delete p;
  delete b;
  return EMQX_OK;
}

int emqx_host_batch_reserve(emqx_host_batch* b, uint64_t cap_topics, uint64_t cap_bytes, uint64_t cap_ids) {
  if (!b || static_cast<HostBatchPriv*>(b->priv)->pending) return EMQX_EINVAL;
  return hb_alloc(b, cap_topics, cap_bytes, cap_ids, true);
}

int emqx_host_batch_submit(emqx_host_batch* b, uint32_t mode) {
  if (!b || mode > EMQX_MODE_TRIE_WILDCARD) return EMQX_EINVAL;
  auto* p = static_cast<HostBatchPriv*>(b->priv);
  if (p->pending || b->n > b->cap_topics) return EMQX_EINVAL;
  const uint64_t* o = b->topic_offsets;
  if (o[0] != 0 || o[b->n] > b->cap_bytes || !offsets_ok(o, b->n)) return EMQX_EINVAL;
  HIP_TRY(hipSetDevice(p->e->device));
  p->mode = mode;
  return hb_enqueue(b);
}

int emqx_host_batch_wait(emqx_host_batch* b) {
  if (!b) return EMQX_EINVAL;
  return hb_wait(b);
}

int emqx_host_batch_query(emqx_host_batch* b) {
  if (!b) return EMQX_EINVAL;
  auto* p = static_cast<HostBatchPriv*>(b->priv);
  return !p->pending || hipEventQuery(p->done) == hipSuccess ? 1 : 0;
}

// Host buffers of any kind: chunks of the batch flow through two pinned host batches of the
// engine's pool — while one chunk is on the device, the previous chunk's results are copied
// out and the next chunk is packed.
int emqx_match_batch(emqx_engine* e, uint32_t mode, const uint8_t* topic_bytes, const uint64_t* topic_offsets,
                     uint64_t n, uint64_t* out_offsets, uint32_t* out_ids, uint64_t cap, uint64_t* n_out) {
  if (!e || !n_out || !out_offsets || mode > EMQX_MODE_TRIE_WILDCARD) return EMQX_EINVAL;
  if (n && !topic_offsets) return EMQX_EINVAL;
  if (!offsets_ok(topic_offsets, n)) return EMQX_EINVAL;
  const uint64_t b0 = n ? topic_offsets[0] : 0, b1 = n ? topic_offsets[n] : 0;
  if (b1 > b0 && !topic_bytes) return EMQX_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  constexpr uint64_t CH_TOPICS = 1u << 18, CH_BYTES = 16u << 20, CH_IDS = 8u << 20;
  emqx_host_batch* hb[2] = {nullptr, nullptr};
  {
    std::lock_guard<std::mutex> g(e->hb_mu);
    for (int k = 0; k < 2 && !e->hb_free.empty(); ++k) {
      hb[k] = e->hb_free.back();
      e->hb_free.pop_back();
    }
  }
  int rc = EMQX_OK;
  for (int k = 0; k < 2 && rc == EMQX_OK; ++k)
    if (!hb[k]) rc = emqx_host_batch_create(e, CH_TOPICS, CH_BYTES, CH_IDS, &hb[k]);
  // one table version for the whole call: a commit landing between two chunks (or before a
  // chunk's rerun) must not mix versions within one result
  const std::shared_ptr<Snapshot> pin = current(e);
  for (int k = 0; k < 2; ++k)
    if (hb[k]) static_cast<HostBatchPriv*>(hb[k]->priv)->pin = pin;
  uint64_t chunk_lo[2] = {0, 0}, total = 0, next = 0, evals = 0, deferred = 0, max_stack = 0;
  bool inflight[2] = {false, false}, overflow = false;
  // pack topics [next, ...) into hb[k] (rebased offsets)
  auto pack = [&](int k) -> int {
    emqx_host_batch* b = hb[k];
    const uint64_t lo = next;
    uint64_t hi = lo;
    const uint64_t base = topic_offsets[lo];
    while (hi < n && hi - lo < b->cap_topics && topic_offsets[hi + 1] - base <= b->cap_bytes) ++hi;
    if (hi == lo) {  // one topic larger than the chunk buffer
      int r = emqx_host_batch_reserve(b, b->cap_topics, topic_offsets[lo + 1] - base + 16, b->cap_ids);
      if (r != EMQX_OK) return r;
      hi = lo + 1;
    }
    const uint64_t nb = topic_offsets[hi] - base;
    if (nb) std::memcpy(b->topic_bytes, topic_bytes + base, nb);
    for (uint64_t i = lo; i <= hi; ++i) b->topic_offsets[i - lo] = topic_offsets[i] - base;
    b->n = hi - lo;
    chunk_lo[k] = lo;
    next = hi;
    return emqx_host_batch_submit(b, mode);
  };
  // results of hb[k] into the caller's arrays (offsets rebased to the running total)
  auto drain = [&](int k) -> int {
    emqx_host_batch* b = hb[k];
    int r = emqx_host_batch_wait(b);
    // more ids than the chunk's buffer: grow it to the reported need and rerun the chunk (same
    // pinned snapshot, so the need cannot move; the loop only guards against that anyway)
    for (int tries = 0; r == EMQX_EOVERFLOW && tries < 4; ++tries) {
      r = emqx_host_batch_reserve(b, b->cap_topics, b->cap_bytes, b->n_out + (b->n_out >> 2) + 1024);
      if (r == EMQX_OK) r = emqx_host_batch_submit(b, mode);
      if (r == EMQX_OK) r = emqx_host_batch_wait(b);
    }
    if (r != EMQX_OK) return r;
    const auto* p = static_cast<const HostBatchPriv*>(b->priv);
    evals += p->evals;
    deferred += p->deferred;
    max_stack = std::max(max_stack, p->max_stack);
    const uint64_t lo = chunk_lo[k], m = b->n_out;
    for (uint64_t i = 0; i < b->n; ++i) out_offsets[lo + i] = total + b->out_offsets[i];
    if (!overflow && out_ids && total + m <= cap) {
      if (m) std::memcpy(out_ids + total, b->out_ids, m * sizeof(uint32_t));
    } else if (m) {
      overflow = true;
    }
    total += m;
    return EMQX_OK;
  };
  int k = 0;
  if (rc == EMQX_OK && n == 0) {
    out_offsets[0] = 0;
  } else {
    while (rc == EMQX_OK && (next < n || inflight[0] || inflight[1])) {
      if (inflight[k]) {
        rc = drain(k);
        inflight[k] = false;
      }
      if (rc == EMQX_OK && next < n) {
        rc = pack(k);
        inflight[k] = rc == EMQX_OK;
      }
      k ^= 1;
    }
  }
  for (int j = 0; j < 2; ++j)  // drain what an error left in flight before the batches go back
    if (inflight[j]) (void)emqx_host_batch_wait(hb[j]);
  out_offsets[n] = total;
  *n_out = total;
  e->last_evals.store(evals);  // the whole call's numbers, over its chunks
  e->last_deferred.store(deferred);
  e->last_max_stack.store(max_stack);
  for (int j = 0; j < 2; ++j)
    if (hb[j]) static_cast<HostBatchPriv*>(hb[j]->priv)->pin.reset();
  {
    std::lock_guard<std::mutex> g(e->hb_mu);
    for (int j = 0; j < 2; ++j)
      if (hb[j]) e->hb_free.push_back(hb[j]);
  }
  if (rc == EMQX_OK && (overflow || total > cap)) rc = EMQX_EOVERFLOW;
  return rc;
}

int emqx_stats_get(emqx_engine* e, emqx_stats* dst) {
  if (!e || !dst || (dst->size && dst->size < sizeof(uint64_t))) return EMQX_EINVAL;
  const uint64_t want = dst->size ? std::min<uint64_t>(dst->size, sizeof(emqx_stats)) : sizeof(emqx_stats);
  emqx_stats full;
  emqx_stats* out = &full;
  std::memset(out, 0, sizeof(*out));
  {
    std::lock_guard<std::mutex> g(e->writer);
    out->n_filters = e->store.n_live;
    out->n_ids = e->store.n_ids();
    out->epoch = e->epoch;
    out->last_build_ms = e->last_build_ms;
    out->delta_filters = e->ls.inserted;
    out->last_commit_kind = e->last_commit_kind;
  }
  auto s = current(e);
  if (s) {
    out->n_nodes = s->n_nodes;
    out->n_slots = s->n_slots;
    out->n_words = s->n_words;
    out->table_bytes = s->bytes;
    out->max_depth = s->max_depth;
  }
  out->last_ordered = e->last_ordered.load();
  out->last_order_ms = e->last_order_ms.load();
  out->last_evals = e->last_evals.load();
  out->last_deferred = e->last_deferred.load();
  out->last_max_stack = e->last_max_stack.load();
  out->last_match_ms = e->last_match_ms.load();
  out->last_kernel_ms = e->last_kernel_ms.load();
  out->size = want;
  std::memcpy(dst, out, want);
  return EMQX_OK;
}

const char* emqx_strerror(int code) {
  switch (code) {
    case EMQX_OK: return "ok";
    case EMQX_EINVAL: return "invalid argument";
    case EMQX_ENOMEM: return "out of memory";
    case EMQX_EDEVICE: return g_last_error.empty() ? "device error" : g_last_error.c_str();
    case EMQX_EOVERFLOW: return "output capacity too small";
    case EMQX_ENOTFOUND: return "not found";
    case EMQX_ETOODEEP: return "topic frontier too deep";
    case EMQX_EBUSY: return "busy: every batch buffer is in use";
    default: return "unknown error";
  }
}

int emqx_set_tuning(emqx_engine* e, const char* key, int64_t value) {
  if (!e || !key) return EMQX_EINVAL;
  if (std::strcmp(key, "fast_variant") == 0) {
    if (value < -1 || value >= FAST_NVARIANTS) return EMQX_EINVAL;
    e->forced_variant.store(static_cast<int>(value));
    return EMQX_OK;
  }
  if (std::strcmp(key, "diag") == 0) {
    e->diag_on.store(value != 0);
    return EMQX_OK;
  }
  if (std::strcmp(key, "diag_stop") == 0) {
    e->diag_stop.store(static_cast<uint32_t>(value));
    return EMQX_OK;
  }
  if (std::strcmp(key, "timeline") == 0) {  // tiles to record (0: off); diag calls only
    if (value < 0) return EMQX_EINVAL;
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipDeviceSynchronize());
    dfree(e->timeline);
    e->timeline_cap = 0;
    if (value) {
      HIP_TRY(dalloc(e->timeline, static_cast<uint64_t>(value)));
      HIP_TRY(hipMemset(e->timeline, 0, static_cast<uint64_t>(value) * sizeof(uint4)));
      e->timeline_cap = static_cast<uint64_t>(value);
    }
    return EMQX_OK;
  }
  if (std::strcmp(key, "small_batch") == 0) {  // host batches of <= SMALL_MAX_N topics in one launch
    e->small_batch.store(value != 0);
    return EMQX_OK;
  }
  if (std::strcmp(key, "incremental") == 0) {
    std::lock_guard<std::mutex> g(e->writer);
    e->incremental = value != 0;
    return EMQX_OK;
  }
  if (std::strcmp(key, "commit_threads") == 0) {
    if (value < 1 || value > 256) return EMQX_EINVAL;
    std::lock_guard<std::mutex> g(e->writer);
    e->commit_threads = static_cast<int>(value);
    return EMQX_OK;
  }
  if (std::strcmp(key, "order") == 0) {
    if (value < -1 || value > 1) return EMQX_EINVAL;
    e->order.store(static_cast<int>(value));
    return EMQX_OK;
  }
  if (std::strcmp(key, "order_level_bits") == 0) {
    if (value < 0 || value > 32) return EMQX_EINVAL;
    e->order_level_bits.store(static_cast<int>(value));
    return EMQX_OK;
  }
  if (std::strcmp(key, "order_sort_bits") == 0) {
    if (value < 1 || value > 64) return EMQX_EINVAL;
    e->order_sort_bits.store(static_cast<int>(value));
    return EMQX_OK;
  }
  if (std::strcmp(key, "order_deal") == 0) {
    e->order_deal.store(value != 0);
    return EMQX_OK;
  }
  if (std::strcmp(key, "delta_max") == 0) {
    std::lock_guard<std::mutex> g(e->writer);
    e->delta_max = value;
    return EMQX_OK;
  }
  return EMQX_ENOTFOUND;
}

uint64_t emqx_permute_scratch_bytes(uint64_t n) { return permute_scratch_bytes(n); }

uint64_t emqx_owner_sort_scratch_bytes(uint64_t n, uint32_t world) { return owner_sort_scratch_bytes(n, world); }

int emqx_owner_sort_device(const uint32_t* d_owner, uint64_t n, uint32_t world, uint32_t* d_perm, void* d_scratch,
                           void* stream) {
  if (world == 0 || (n && (!d_owner || !d_perm || !d_scratch)) || n > 0xFFFFFFFFull) return EMQX_EINVAL;
  HIP_TRY(launch_owner_sort(d_owner, n, world, d_perm, d_scratch, static_cast<hipStream_t>(stream)));
  return EMQX_OK;
}

int emqx_batch_permute_device(const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n, const uint32_t* d_perm,
                              uint8_t* d_out_bytes, uint64_t* d_out_offsets, void* d_scratch, void* stream) {
  if (!d_out_offsets || !d_scratch || (n && (!d_bytes || !d_offsets || !d_perm || !d_out_bytes))) return EMQX_EINVAL;
  HIP_TRY(launch_batch_permute(d_bytes, d_offsets, n, d_perm, d_out_bytes, d_out_offsets, d_scratch,
                               static_cast<hipStream_t>(stream)));
  return EMQX_OK;
}

int emqx_csr_unpermute_device(const uint32_t* d_counts, const uint32_t* d_ids, uint64_t n, const uint32_t* d_perm,
                              uint64_t* d_out_offsets, uint32_t* d_out_ids, void* d_scratch, void* stream) {
  if (!d_out_offsets || !d_scratch || (n && (!d_counts || !d_perm))) return EMQX_EINVAL;
  HIP_TRY(launch_csr_unpermute(d_counts, d_ids, n, d_perm, d_out_offsets, d_out_ids, d_scratch,
                               static_cast<hipStream_t>(stream)));
  return EMQX_OK;
}

int emqx_shard_owner_device(const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n, uint32_t world,
                            uint32_t levels, uint32_t* d_owner, void* stream) {
  if ((n && (!d_bytes || !d_offsets || !d_owner)) || world == 0 || levels == 0) return EMQX_EINVAL;
  HIP_TRY(launch_shard_owner(d_bytes, d_offsets, n, world, levels, d_owner, static_cast<hipStream_t>(stream)));
  return EMQX_OK;
}

int emqx_shard_route_device(const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n, uint32_t world,
                            const emqx_shard_split* d_splits, uint32_t n_splits, uint32_t* d_req2, void* stream) {
  if ((n && (!d_bytes || !d_offsets || !d_req2)) || world == 0 || (n_splits && !d_splits)) return EMQX_EINVAL;
  HIP_TRY(launch_shard_route(d_bytes, d_offsets, n, world, reinterpret_cast<const ShardSplitE*>(d_splits), n_splits,
                             d_req2, static_cast<hipStream_t>(stream)));
  return EMQX_OK;
}

int emqx_commit_stats(emqx_engine* e, uint64_t* out, uint32_t n) {
  if (!e || (n && !out)) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(e->writer);
  const LiveTrie* lt = e->ls.lt.get();
  uint64_t host_us = static_cast<uint64_t>(e->last_host_ms * 1e3);
  const uint64_t v[12] = {e->last_commit_kind, e->last_relocations, e->last_in_place, e->last_patches,
                          e->last_new_slots, lt ? lt->used : 0, lt ? lt->cap : 0, lt ? lt->garbage : 0, host_us,
                          e->last_extents, e->last_vocab_slots, static_cast<uint64_t>(e->last_upload_ms * 1e3)};
  for (uint32_t i = 0; i < n && i < 12; ++i) out[i] = v[i];
  return EMQX_OK;
}

int emqx_diag_read(emqx_engine* e, uint64_t* out, uint32_t n, int reset) {
  if (!e || !out) return EMQX_EINVAL;
  HIP_TRY(hipSetDevice(e->device));
  std::vector<uint64_t> acc(DIAG_WORDS, 0), tmp(DIAG_WORDS);
  std::lock_guard<std::mutex> g(e->ws_mu);
  for (auto& w : e->all_ws) {
    if (!w->diag) continue;
    HIP_TRY(hipMemcpy(tmp.data(), w->diag, DIAG_WORDS * sizeof(uint64_t), hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < DIAG_WORDS; ++i) acc[i] += tmp[i];
    if (reset) HIP_TRY(hipMemset(w->diag, 0, DIAG_WORDS * sizeof(uint64_t)));
  }
  for (uint32_t i = 0; i < n && i < DIAG_WORDS; ++i) out[i] = acc[i];
  return EMQX_OK;
}

int emqx_diag_timeline(emqx_engine* e, uint32_t* out, uint64_t cap_tiles, uint64_t* n_tiles) {
  if (!e || !n_tiles || (cap_tiles && !out)) return EMQX_EINVAL;
  *n_tiles = e->timeline_cap;
  if (!e->timeline || !cap_tiles) return EMQX_OK;
  HIP_TRY(hipSetDevice(e->device));
  HIP_TRY(hipDeviceSynchronize());
  HIP_TRY(hipMemcpy(out, e->timeline, std::min(cap_tiles, e->timeline_cap) * sizeof(uint4), hipMemcpyDeviceToHost));
  return EMQX_OK;
}

const char* emqx_version(void) { return "emqx-match-mi355x 0.1.0 (gfx950)"; }

}  // extern "C"
