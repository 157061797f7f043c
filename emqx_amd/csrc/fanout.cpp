// C ABI of the publish fan-out stage (include/emqx_match.h, emqx_subtab_* / emqx_fanout_* /
// emqx_pub_batch_* / emqx_publish_batch): host subscription store, device tables patched in
// place per commit, the per-publisher $share pick state, and the fan-out pipeline
//   entry_topic -> count -> scan -> write (+ offsets) [-> resolve] -> finish   (one stream, no host sync)
//
// Store semantics follow the reference's ETS tables:
//   plain subscriptions  ?SUBSCRIBER bag Topic -> SubPid (apps/emqx/src/emqx_broker.erl:146-158);
//                        the {shard, I} buckets of emqx_broker_helper:get_sub_shard/2
//                        (emqx_broker_helper.erl:81-86) only split storage, so the device
//                        array is the flattened union.
//   $share memberships   emqx_shared_subscription bag keyed by Group, selected per
//                        (Group, Topic) in insertion order (emqx_shared_sub.erl:287-288,308-322);
//                        the member order is what lists:nth/2 indexes in pick_subscriber/6.
//
// Commits cost what changed: the host keeps an image of every device array;
// a subscribe appends to its filter's plain list in place (or moves the list to the end of the
// arena with twice the room), an unsubscribe moves the list's last entry into the hole; a
// $share membership change rewrites that group's member list and its 16-B group record.  The
// commit uploads the touched words and records only, ordered after the fan-outs in flight and
// before the next ones by events (no fan-out reads a table while a commit writes it).  A full
// rebuild (compaction) runs only when moved-away extents outweigh the live ones.
#include <hip/hip_runtime.h>

#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/emqx_match.h"
#include "fanout.h"
#include "kernels.h"
#include "streams.h"
#include "workpool.h"

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

// Open-addressed map u64 -> u32 with tombstones (keys never take the two reserved values:
// filter ids and slots are < 2^31).  Key and value share one 16-B entry, so a probe that misses
// the caches costs one line, and prefetch() lets a batch start the next ops' lines early.
class U64Map {
 public:
  uint32_t find(uint64_t k) const {
    if (e_.empty()) return SUB_NONE;
    const uint64_t mask = e_.size() - 1;
    for (uint64_t i = fo_mix64(k) & mask;; i = (i + 1) & mask) {
      if (e_[i].k == EMPTY) return SUB_NONE;
      if (e_[i].k == k) return e_[i].v;
    }
  }
  // true if newly inserted (an existing key keeps its value)
  bool insert(uint64_t k, uint32_t v) {
    if (e_.empty()) rehash(1024);
    else if ((used_ + 1) * 4 >= e_.size() * 3)  // double, or just drop tombstones
      rehash((size_ + 1) * 2 >= e_.size() ? e_.size() * 2 : e_.size());
    const uint64_t mask = e_.size() - 1;
    uint64_t tomb = ~0ull;
    for (uint64_t i = fo_mix64(k) & mask;; i = (i + 1) & mask) {
      if (e_[i].k == k) return false;
      if (e_[i].k == TOMB && tomb == ~0ull) tomb = i;
      if (e_[i].k == EMPTY) {
        if (tomb != ~0ull) i = tomb; else ++used_;
        e_[i].k = k;
        e_[i].v = v;
        ++size_;
        return true;
      }
    }
  }
  void assign(uint64_t k, uint32_t v) {  // k present
    const uint64_t mask = e_.size() - 1;
    for (uint64_t i = fo_mix64(k) & mask;; i = (i + 1) & mask)
      if (e_[i].k == k) {
        e_[i].v = v;
        return;
      }
  }
  bool erase(uint64_t k) {
    if (e_.empty()) return false;
    const uint64_t mask = e_.size() - 1;
    for (uint64_t i = fo_mix64(k) & mask;; i = (i + 1) & mask) {
      if (e_[i].k == EMPTY) return false;
      if (e_[i].k == k) {
        e_[i].k = TOMB;
        --size_;
        return true;
      }
    }
  }
  void prefetch(uint64_t k) const {
    if (!e_.empty()) __builtin_prefetch(&e_[fo_mix64(k) & (e_.size() - 1)], 1);
  }
  bool contains(uint64_t k) const { return find(k) != SUB_NONE; }
  uint64_t size() const { return size_; }

 private:
  static constexpr uint64_t EMPTY = ~0ull, TOMB = ~0ull - 1;
  struct Ent {
    uint64_t k;
    uint32_t v, pad;
  };
  void rehash(uint64_t cap) {
    std::vector<Ent> old;
    old.swap(e_);
    e_.assign(cap, Ent{EMPTY, 0, 0});
    used_ = size_ = 0;
    const uint64_t mask = cap - 1;
    for (const Ent& x : old) {
      if (x.k == EMPTY || x.k == TOMB) continue;
      uint64_t i = fo_mix64(x.k) & mask;
      while (e_[i].k != EMPTY) i = (i + 1) & mask;
      e_[i] = Ent{x.k, x.v, 0};
      ++used_;
      ++size_;
    }
  }
  std::vector<Ent> e_;
  uint64_t used_ = 0, size_ = 0;  // used_ counts tombstones too
};

// The plain positions, sharded by filter: a batch's plain ops run on one thread per shard
// (their filters' lists and map entries are the shard's alone).
constexpr uint32_t PP_SHARDS = 16;
inline uint32_t pp_shard(uint32_t f) { return (f * 0x9E3779B1u) >> 28; }

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

template <class T>
void fo_hfree(T*& p) {
  if (p) (void)hipHostFree(p);
  p = nullptr;
}

template <class T>
hipError_t fo_halloc(T*& p, uint64_t count) {
  fo_hfree(p);
  return hipHostMalloc(reinterpret_cast<void**>(&p), std::max<uint64_t>(count, 1) * sizeof(T), hipHostMallocDefault);
}

template <class T>
T* mapped(T* h) {
  void* d = nullptr;
  return hipHostGetDevicePointer(&d, h, 0) == hipSuccess ? static_cast<T*>(d) : nullptr;
}

struct Slot {
  uint32_t filter, group;
  std::vector<uint32_t> members;  // subscription order
  uint32_t mbegin = 0, mcap = 0;  // the member list's extent in the members arena
  uint32_t live_idx = SUB_NONE;   // index in its filter's group list (SUB_NONE: no members)
  bool dirty = false;
};

// One device array with its capacity (elements).
template <class T>
struct DevArr {
  T* p = nullptr;
  uint64_t cap = 0;
};

constexpr uint64_t PS_INIT_CAP = 1ull << 20;
constexpr uint64_t RANGE_COPY_MIN = 256;  // dirty ranges at least this long are copied, not patched

}  // namespace

// Per-stream scratch of the fan-out pipeline: calls on one stream run in order on the device,
// so they can share it; calls pipelined on different streams never do.
struct FoScratch {
  hipStream_t stream = nullptr;
  uint32_t* entry_topic = nullptr;
  uint64_t cap_entry_topic = 0;
  uint64_t* csum = nullptr;      // chunk offsets: per-chunk deliveries and picks, block sums
  uint64_t* gchunk = nullptr;
  uint64_t cap_chunks = 0;
  uint64_t* partials = nullptr;
  // round_robin / sticky: the pick list, its sorted copy and the sort's scratch, per state entry
  // the run info of the resolve
  uint32_t* pk = nullptr;       // 4 arrays of pk_cap: keys, vals, sorted keys, sorted vals
  uint64_t pk_cap = 0;
  uint8_t* sort_temp = nullptr;
  uint64_t sort_temp_bytes = 0;
  uint32_t* run_ent = nullptr;  // per run id (pk_cap)
  uint32_t* run_cnt = nullptr;  // per run id (pk_cap): picks per run (small path)
  uint32_t* run_named = nullptr;  // [FO_BLOCKS] per probe block: runs named
  unsigned long long* multi = nullptr;  // [FO_MULTI_CAP] (small path)
  unsigned long long* seg = nullptr;
  uint32_t* seg_from = nullptr;
  unsigned long long* tag = nullptr;  // per state entry (ps_cap): stamp << 32 | run id
  uint64_t cap_tag = 0;
  uint32_t stamp = 0;
  unsigned long long* ctl = nullptr;
  uint64_t* h_sum = nullptr;  // host-mapped call summary (synchronous calls)
  unsigned long long* h_seen = nullptr;  // host-mapped [2]: picks and runs of this stream's last call
  uint64_t rerun_picks = 0;   // a rerun after FO_SUM_F_PICKS: the flagged call's own picks ...
  bool rerun_large = false;   // ... and the large resolve path for it
  hipEvent_t done = nullptr;  // end of the last fan-out enqueued on this stream
  bool used = false;
  void release() {
    fo_free(entry_topic);
    fo_free(csum);
    fo_free(gchunk);
    fo_free(partials);
    fo_free(pk);
    fo_free(sort_temp);
    fo_free(run_ent);
    fo_free(run_cnt);
    fo_free(run_named);
    fo_free(multi);
    fo_free(seg);
    fo_free(seg_from);
    fo_free(tag);
    fo_free(ctl);
    fo_hfree(h_sum);
    fo_hfree(h_seen);
    if (done) (void)hipEventDestroy(done);
    done = nullptr;
  }
};

struct PubBatchPriv;

struct emqx_subtab {
  int device = 0;
  std::mutex mu;   // serialises mutations, the host half of commits, and fan-out enqueues
  std::mutex cmu;  // one commit at a time (held while it drains the previous device half, which s->mu is not)
  uint8_t* h_stage = nullptr;  // pinned staging of a commit's uploads (one commit at a time)
  // fault injection (emqx_subtab_set_tuning, tests): the next k drains report a device error,
  // the next k full commits throw std::bad_alloc
  uint32_t inject_drain_error = 0, inject_bad_alloc = 0;
  uint64_t stage_cap = 0;
  // ---- host store, and the image of every device array ----
  std::vector<FilterRec> recs;                // per filter id
  std::vector<uint32_t> pcap, gcap;           // capacities of the filter's plain / group extents
  std::vector<uint32_t> plain;                // plain arena
  std::vector<GroupRec> groups;               // group-record arena
  std::vector<uint32_t> members;              // member arena
  uint64_t garbage = 0;                       // words of extents moved away from
  U64Map plain_pos[PP_SHARDS];                // (filter << 32 | sub) -> index in the plain list,
                                              // by pp_shard(filter)
  std::vector<uint8_t> plocal;                // batch ops: the filter's list is in its thread's arena
  U64Map slot_of;                             // (filter << 32 | group) -> slot
  std::vector<Slot> slots;
  std::vector<std::vector<uint32_t>> fslots;  // filter id -> its slots (creation order)
  U64Map member_set;                          // (slot << 32 | sub) -> 1
  uint64_t n_members = 0, n_live_groups = 0;
  // ---- changes since the last commit ----
  std::vector<std::pair<uint64_t, uint64_t>> dirty_plain;  // (first word, words)
  std::vector<uint32_t> dirty_recs, dirty_slots, dirty_glists;
  std::vector<uint8_t> rec_flag, glist_flag;  // per filter: listed in dirty_recs / dirty_glists
  uint64_t plain_count() const {
    uint64_t n = 0;
    for (const U64Map& m : plain_pos) n += m.size();
    return n;
  }
  std::vector<uint32_t> alive;                // liveness bitmap image (bit per subscriber id)
  std::vector<uint32_t> dirty_alive;          // words of it changed since the last commit
  bool need_full = true;
  uint64_t ops_pending = 0;                   // mutations since the last commit
  bool bulk = false;                          // so many that the next commit rebuilds: no dirt kept
  // ---- device ----
  DevArr<DevRec> d_recs;
  DevArr<uint32_t> d_fcnt;  // fo_cnt_word of each device record (written with it, on the device)
  DevArr<uint32_t> d_plain, d_members;
  DevArr<GroupRec> d_groups;
  DevArr<uint32_t> d_alive;
  uint32_t dev_n_recs = 0, dev_n_alive = 0;
  hipStream_t stream = nullptr;       // commits and table maintenance
  hipEvent_t commit_ev = nullptr;     // end of the last commit: later fan-outs wait for it
  bool commit_pending = false;
  bool commit_inflight = false;       // (s->cmu) the last commit's device half not yet waited for
  std::vector<void*> retired_prev;    // (s->cmu) device arrays it replaced: freed once it is done
  hipEvent_t state_ev = nullptr;      // end of the last round_robin / sticky resolve (or re-pick):
  bool state_pending = false;         // the next one waits for it, so state updates follow call order
  std::vector<WordPatch> wpatch;
  std::vector<RecPatch> rpatch;
  DevArr<WordPatch> d_wpatch;
  DevArr<RecPatch> d_rpatch;
  // pick state per (group slot, publisher)
  uint64_t* ps_keys = nullptr;
  uint32_t* ps_vals = nullptr;
  unsigned long long* ps_count = nullptr;
  unsigned long long* ps_tombs = nullptr;
  uint64_t ps_cap = 0;
  bool ps_force_grow = false;               // a call found no room for a key: grow before the next
  unsigned long long* h_ps_seen = nullptr;  // host-mapped [4]: live keys, tombstones, picks and run
                                            // ids of the last finished call
  std::vector<uint32_t> pending_forget;     // publishers to drop (emqx_subtab_forget_publishers)
  DevArr<uint32_t> d_forget;                // the last flushed list, from pinned staging h_forget
  uint32_t* h_forget = nullptr;
  hipEvent_t forget_ev = nullptr;           // end of the last flush's pass
  bool forget_pending = false;
  std::vector<std::unique_ptr<FoScratch>> scratch;  // one per stream that called
  uint64_t* h_total = nullptr;
  uint32_t seed = 0x2545F491u;
  uint32_t rr_first0 = 0;  // emqx_subtab_set_tuning "rr_seed0"
  // commit statistics (emqx_subtab_commit_stats)
  uint64_t st_commits = 0, st_full = 0, st_words = 0, st_records = 0, st_moves = 0, st_last_kind = 0;
  double st_host_us = 0, st_total_us = 0;
  // pinned publish batches of emqx_publish_batch (pool)
  std::mutex pb_mu;
  std::vector<emqx_pub_batch*> pb_free;

  ~emqx_subtab();
};

namespace {

bool ids_ok(const uint32_t* f, const uint32_t* s, uint64_t n) {
  if (n && (!f || !s)) return false;
  for (uint64_t i = 0; i < n; ++i)
    if (f[i] >= FANOUT_ID_LIMIT || s[i] == SUB_NONE) return false;
  return true;
}

// Sets subscriber `sub`'s liveness bit in the image (dirty words go out with the next commit).
void set_alive_bit(emqx_subtab* s, uint32_t sub, bool on) {
  const uint64_t w = sub >> 5;
  if (w >= s->alive.size()) {
    if (!on) return;
    s->alive.resize(std::max<uint64_t>(w + 1, s->alive.size() + s->alive.size() / 2), 0u);
  }
  const uint32_t bit = 1u << (sub & 31u), old = s->alive[w];
  const uint32_t nv = on ? old | bit : old & ~bit;
  if (nv == old) return;
  s->alive[w] = nv;
  s->dirty_alive.push_back(static_cast<uint32_t>(w));
}

void ensure_filter(emqx_subtab* s, uint32_t f) {
  if (f < s->recs.size()) return;
  const uint64_t n = uint64_t(f) + 1;
  s->recs.resize(n, FilterRec{0, 0, 0, 0});
  s->pcap.resize(n, 0);
  s->gcap.resize(n, 0);
  s->rec_flag.resize(n, 0);
  s->glist_flag.resize(n, 0);
  s->plocal.resize(n, 0);
  if (s->fslots.size() < n) s->fslots.resize(n);
}

// A bulk load (more mutations before a commit than a quarter of the table, at least 64K) is
// cheaper as one full upload than as patches: past that point no dirt is recorded.
uint64_t bulk_threshold(const emqx_subtab* s) {
  return std::max<uint64_t>(1u << 16, (s->plain_count() + s->n_members) / 4);
}

void go_bulk(emqx_subtab* s) {
  s->bulk = true;
  std::vector<std::pair<uint64_t, uint64_t>>().swap(s->dirty_plain);
  std::vector<uint32_t>().swap(s->dirty_recs);
  std::vector<uint32_t>().swap(s->dirty_slots);
  std::vector<uint32_t>().swap(s->dirty_glists);
}

void note_op(emqx_subtab* s) {
  if (s->bulk || ++s->ops_pending <= bulk_threshold(s)) return;
  go_bulk(s);
}

void mark_rec(emqx_subtab* s, uint32_t f) {
  if (s->bulk) return;
  if (!s->rec_flag[f]) {
    s->rec_flag[f] = 1;
    s->dirty_recs.push_back(f);
  }
}

void mark_glist(emqx_subtab* s, uint32_t f) {
  if (s->bulk) return;
  if (!s->glist_flag[f]) {
    s->glist_flag[f] = 1;
    s->dirty_glists.push_back(f);
  }
}

void mark_slot(emqx_subtab* s, uint32_t sl) {
  if (s->bulk) return;
  if (!s->slots[sl].dirty) {
    s->slots[sl].dirty = true;
    s->dirty_slots.push_back(sl);
  }
}

uint32_t grow_cap(uint64_t n, uint32_t min_cap) {
  return static_cast<uint32_t>(std::max<uint64_t>(min_cap, n + (n >> 1) + 1));
}

void plain_add(emqx_subtab* s, uint32_t f, uint32_t sub) {
  const uint64_t key = (uint64_t(f) << 32) | sub;
  ensure_filter(s, f);
  FilterRec& r = s->recs[f];
  if (!s->plain_pos[pp_shard(f)].insert(key, r.n_plain)) return;  // ETS bag: a pair is stored once
  if (r.n_plain == s->pcap[f]) {  // the extent is full: move the list to the arena's end
    const uint64_t nb = s->plain.size();
    const uint32_t cap = std::max<uint32_t>(4, 2 * r.n_plain);
    s->plain.resize(nb + cap);
    std::copy(s->plain.begin() + r.plain_begin, s->plain.begin() + r.plain_begin + r.n_plain, s->plain.begin() + nb);
    if (r.n_plain && !s->bulk) s->dirty_plain.emplace_back(nb, r.n_plain);
    s->garbage += s->pcap[f];
    r.plain_begin = static_cast<uint32_t>(nb);
    s->pcap[f] = cap;
    ++s->st_moves;
  }
  const uint64_t w = uint64_t(r.plain_begin) + r.n_plain;
  s->plain[w] = sub;
  if (!s->bulk) s->dirty_plain.emplace_back(w, 1);
  r.n_plain += 1;
  mark_rec(s, f);
  note_op(s);
}

void plain_remove(emqx_subtab* s, uint32_t f, uint32_t sub) {
  const uint64_t key = (uint64_t(f) << 32) | sub;
  U64Map& pp = s->plain_pos[pp_shard(f)];
  const uint32_t pos = pp.find(key);
  if (pos == SUB_NONE) return;
  pp.erase(key);
  FilterRec& r = s->recs[f];
  const uint32_t last = r.n_plain - 1;
  if (pos != last) {  // the last subscriber fills the hole (plain order carries no meaning)
    const uint32_t moved = s->plain[uint64_t(r.plain_begin) + last];
    s->plain[uint64_t(r.plain_begin) + pos] = moved;
    pp.assign((uint64_t(f) << 32) | moved, pos);
    if (!s->bulk) s->dirty_plain.emplace_back(uint64_t(r.plain_begin) + pos, 1);
  }
  r.n_plain = last;
  mark_rec(s, f);
  note_op(s);
}

// The device form of filter f's record (fanout.h FO_INLINE): a short plain list and no
// groups inline, otherwise the image's record.
DevRec dev_rec(const emqx_subtab* s, uint32_t f) {
  const FilterRec& r = s->recs[f];
  if (r.n_groups == 0 && r.n_plain >= 1 && r.n_plain <= FO_INLINE) {
    const uint32_t* p = s->plain.data() + r.plain_begin;
    uint32_t v[FO_INLINE] = {};
    for (uint32_t i = 0; i < r.n_plain; ++i) v[i] = p[i];
    return DevRec{make_uint4(v[0], r.n_plain | FO_INLINE_BIT, v[1], v[2]), make_uint4(v[3], v[4], v[5], v[6])};
  }
  return DevRec{make_uint4(r.plain_begin, r.n_plain, r.group_begin, r.n_groups), make_uint4(0, 0, 0, 0)};
}

// EMQX_SUBTAB_PROF=1: per add/remove call and per commit, where the host time goes, on stderr
// (experiments)
static bool subtab_prof() {
  static const bool on = [] {
    const char* e = std::getenv("EMQX_SUBTAB_PROF");
    return e && *e == '1';
  }();
  return on;
}
static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// ---- batched plain ops on several threads --------------------------------------------------
// A batch of plain subscribes or unsubscribes runs one thread per filter shard (pp_shard): a
// shard's filters, their records, extents and map entries belong to its thread alone, and a
// list that outgrows its extent moves into the thread's own arena, appended to the shared one
// after the batch (its filters' extents rebased then).  Ops on one filter keep their order, so
// the result equals the serial loop's.  The random lines of the next ops are prefetched.
constexpr uint64_t PAR_MIN = 4096;  // smaller batches stay on the caller's thread

unsigned par_threads() {
  static const unsigned t = [] {
    unsigned n = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0) n = static_cast<unsigned>(CPU_COUNT(&cs));
    if (const char* e = std::getenv("EMQX_SUBTAB_THREADS")) n = static_cast<unsigned>(std::max(1, std::atoi(e)));
    return std::max(1u, std::min(n, PP_SHARDS));
  }();
  return t;
}

// (WorkPool: workpool.h; spawning 16 threads per batch cost more than the batch's work)

struct PlainLocal {
  std::vector<uint32_t> arena;                        // lists moved in this batch
  std::vector<std::pair<uint64_t, uint64_t>> dirty;  // touched words of the shared arena
  std::vector<uint32_t> recs;                         // records newly dirty
  std::vector<uint32_t> moved;                        // filters whose list is in `arena`
  uint64_t garbage = 0, moves = 0, ops = 0;
};

void plain_batch_shard(emqx_subtab* s, const uint32_t* fs, const uint32_t* subs, const uint32_t* idx, uint64_t cnt,
                       bool add, PlainLocal& L) {
  const bool bulk = s->bulk;
  uint32_t* const shared = s->plain.data();
  const uint64_t nrec = s->recs.size();
  // two-stage prefetch: 16 ops ahead the op's map entry, record and per-filter flags (each its
  // own random line); 4 ahead, from the record fetched by then, the list word it will write
  // (add) or move (remove)
  constexpr uint64_t AHEAD = 16, AHEAD2 = 4;
  for (uint64_t j = 0; j < cnt; ++j) {
    if (j + AHEAD < cnt) {
      const uint64_t q2 = idx[j + AHEAD];
      const uint32_t f2 = fs[q2];
      if (f2 < nrec) {
        s->plain_pos[pp_shard(f2)].prefetch((uint64_t(f2) << 32) | subs[q2]);
        __builtin_prefetch(&s->recs[f2], 1);
        __builtin_prefetch(&s->pcap[f2], 1);
        __builtin_prefetch(&s->plocal[f2], 1);
        __builtin_prefetch(&s->rec_flag[f2], 1);
      }
    }
    if (j + AHEAD2 < cnt) {
      const uint32_t f3 = fs[idx[j + AHEAD2]];
      if (f3 < nrec && !s->plocal[f3]) {
        const FilterRec& r3 = s->recs[f3];
        const uint64_t w3 = uint64_t(r3.plain_begin) + r3.n_plain - (add || r3.n_plain == 0 ? 0u : 1u);
        if (w3 < s->plain.size()) __builtin_prefetch(shared + w3, 1);
      }
    }
    const uint64_t q = idx[j];
    const uint32_t f = fs[q], sub = subs[q];
    if (f >= nrec) continue;  // an unsubscribe from a filter never seen
    U64Map& pp = s->plain_pos[pp_shard(f)];
    FilterRec& r = s->recs[f];
    const uint64_t key = (uint64_t(f) << 32) | sub;
    if (add) {
      if (!pp.insert(key, r.n_plain)) continue;  // ETS bag: a pair is stored once
      if (r.n_plain == s->pcap[f]) {             // full: into this thread's arena, twice the room
        const uint32_t cap = std::max<uint32_t>(4, 2 * r.n_plain);
        const uint64_t nb = L.arena.size();
        L.arena.resize(nb + cap);
        const uint32_t* from = (s->plocal[f] ? L.arena.data() : shared) + r.plain_begin;
        std::copy(from, from + r.n_plain, L.arena.data() + nb);
        L.garbage += s->pcap[f];
        if (!s->plocal[f]) {
          s->plocal[f] = 1;
          L.moved.push_back(f);
        }
        r.plain_begin = static_cast<uint32_t>(nb);
        s->pcap[f] = cap;
        ++L.moves;
      }
      (s->plocal[f] ? L.arena.data() : shared)[uint64_t(r.plain_begin) + r.n_plain] = sub;
      if (!bulk && !s->plocal[f]) L.dirty.emplace_back(uint64_t(r.plain_begin) + r.n_plain, 1);
      r.n_plain += 1;
    } else {
      const uint32_t pos = pp.find(key);
      if (pos == SUB_NONE) continue;
      pp.erase(key);
      const uint32_t last = r.n_plain - 1;
      if (pos != last) {  // the last subscriber fills the hole
        uint32_t* l = (s->plocal[f] ? L.arena.data() : shared) + r.plain_begin;
        const uint32_t moved = l[last];
        l[pos] = moved;
        pp.assign((uint64_t(f) << 32) | moved, pos);
        if (!bulk && !s->plocal[f]) L.dirty.emplace_back(uint64_t(r.plain_begin) + pos, 1);
      }
      r.n_plain = last;
    }
    ++L.ops;
    if (!bulk && !s->rec_flag[f]) {
      s->rec_flag[f] = 1;
      L.recs.push_back(f);
    }
  }
}

// n plain subscribes (add) or unsubscribes, s->mu held.
void plain_batch(emqx_subtab* s, const uint32_t* fs, const uint32_t* subs, uint64_t n, bool add) {
  const double p0 = subtab_prof() ? now_us() : 0;
  if (add) {
    uint32_t fmax = 0;
    for (uint64_t i = 0; i < n; ++i) fmax = std::max(fmax, fs[i]);
    ensure_filter(s, fmax);
    for (uint64_t i = 0; i < n; ++i) set_alive_bit(s, subs[i], true);  // a subscribing process is alive
  }
  if (!s->bulk && s->ops_pending + n > bulk_threshold(s)) go_bulk(s);
  // the ops by shard, in order within each
  uint64_t start[PP_SHARDS + 1] = {};
  for (uint64_t i = 0; i < n; ++i) ++start[pp_shard(fs[i]) + 1];
  for (uint32_t k = 0; k < PP_SHARDS; ++k) start[k + 1] += start[k];
  std::vector<uint32_t> idx(n);
  {
    uint64_t pos[PP_SHARDS];
    std::copy(start, start + PP_SHARDS, pos);
    for (uint64_t i = 0; i < n; ++i) idx[pos[pp_shard(fs[i])]++] = static_cast<uint32_t>(i);
  }
  std::vector<PlainLocal> loc(PP_SHARDS);
  std::atomic<uint32_t> next{0};
  const std::function<void()> work = [&] {
    for (uint32_t k; (k = next.fetch_add(1)) < PP_SHARDS;)
      plain_batch_shard(s, fs, subs, idx.data() + start[k], start[k + 1] - start[k], add, loc[k]);
  };
  // every thread (the ops are cache misses, not compute: more threads, more misses in flight)
  const double p1 = subtab_prof() ? now_us() : 0;
  WorkPool::get().run(work, par_threads());
  const double p2 = subtab_prof() ? now_us() : 0;
  // merge, shard by shard: moved lists appended to the shared arena
  for (PlainLocal& L : loc) {
    if (!L.arena.empty()) {
      const uint64_t base = s->plain.size();
      s->plain.insert(s->plain.end(), L.arena.begin(), L.arena.end());
      for (uint32_t f : L.moved) {
        FilterRec& r = s->recs[f];
        r.plain_begin = static_cast<uint32_t>(r.plain_begin + base);
        s->plocal[f] = 0;
        if (!s->bulk && r.n_plain) s->dirty_plain.emplace_back(r.plain_begin, r.n_plain);
      }
    }
    if (!s->bulk) {
      s->dirty_plain.insert(s->dirty_plain.end(), L.dirty.begin(), L.dirty.end());
      s->dirty_recs.insert(s->dirty_recs.end(), L.recs.begin(), L.recs.end());
    }
    s->garbage += L.garbage;
    s->st_moves += L.moves;
    s->ops_pending += L.ops;
  }
  if (subtab_prof())
    std::fprintf(stderr, "SUBTAB_PROF plain_batch %s prep_us %.1f run_us %.1f merge_us %.1f\n", add ? "add" : "remove",
                 p1 - p0, p2 - p1, now_us() - p2);
}

// ---- device side of a commit ----------------------------------------------------------------

// Orders the commit stream after every fan-out in flight.
int barrier_after_fanouts(emqx_subtab* s) {
  for (auto& c : s->scratch)
    if (c->used) FO_TRY(hipStreamWaitEvent(s->stream, c->done, 0));
  return EMQX_OK;
}

// Grows a device array to hold `need` elements, keeping its first `keep` elements.
template <class T>
int dev_reserve(emqx_subtab* s, DevArr<T>& a, uint64_t need, uint64_t keep, std::vector<void*>& retired) {
  if (need <= a.cap && a.p) return EMQX_OK;
  const uint64_t cap = std::max<uint64_t>(need + need / 2, 1u << 16);
  T* p = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&p), cap * sizeof(T)) != hipSuccess) return EMQX_ENOMEM;
  if (keep && a.p) FO_TRY(hipMemcpyAsync(p, a.p, keep * sizeof(T), hipMemcpyDeviceToDevice, s->stream));
  if (cap > keep) FO_TRY(hipMemsetAsync(p + keep, 0, (cap - keep) * sizeof(T), s->stream));
  if (a.p) retired.push_back(a.p);
  a.p = p;
  a.cap = cap;
  return EMQX_OK;
}

// Rebuilds the image compactly (every extent with a quarter of slack) and marks it all dirty.
void compact_image(emqx_subtab* s) {
  const uint64_t nf = s->recs.size();
  std::vector<uint32_t> plain;
  std::vector<GroupRec> groups;
  std::vector<uint32_t> members;
  plain.reserve(s->plain_count() + s->plain_count() / 4 + 4 * nf);
  members.reserve(s->n_members + s->n_members / 4);
  s->n_live_groups = 0;
  for (uint64_t f = 0; f < nf; ++f) {
    FilterRec& r = s->recs[f];
    const uint32_t pb = static_cast<uint32_t>(plain.size());
    const uint32_t pc = r.n_plain ? r.n_plain + (r.n_plain >> 2) + 1 : 0;
    plain.insert(plain.end(), s->plain.begin() + r.plain_begin, s->plain.begin() + r.plain_begin + r.n_plain);
    plain.resize(uint64_t(pb) + pc, 0);
    r.plain_begin = pb;
    s->pcap[f] = pc;
    const uint32_t gb = static_cast<uint32_t>(groups.size());
    uint32_t ng = 0;
    for (uint32_t sl : s->fslots[f]) {
      Slot& S = s->slots[sl];
      S.dirty = false;
      S.live_idx = SUB_NONE;
      const uint32_t nm = static_cast<uint32_t>(S.members.size());
      S.mbegin = static_cast<uint32_t>(members.size());
      S.mcap = nm ? nm + (nm >> 2) + 1 : 0;
      members.insert(members.end(), S.members.begin(), S.members.end());
      members.resize(uint64_t(S.mbegin) + S.mcap, 0);
      if (!nm) continue;
      S.live_idx = ng++;
      groups.push_back(GroupRec{S.mbegin, nm, sl, S.group});
    }
    const uint32_t gc = ng ? ng + (ng >> 2) + 1 : 0;
    groups.resize(uint64_t(gb) + gc, GroupRec{0, 0, 0, 0});
    r.group_begin = gb;
    r.n_groups = ng;
    s->gcap[f] = gc;
    s->n_live_groups += ng;
  }
  s->plain.swap(plain);
  s->groups.swap(groups);
  s->members.swap(members);
  s->garbage = 0;
  s->dirty_plain.clear();
  s->dirty_recs.clear();
  s->dirty_slots.clear();
  s->dirty_glists.clear();
  std::fill(s->rec_flag.begin(), s->rec_flag.end(), 0);
  std::fill(s->glist_flag.begin(), s->glist_flag.end(), 0);
}

// Full commit: the compacted image uploaded into fresh device arrays.
int full_commit(emqx_subtab* s) {
  if (s->inject_bad_alloc) {
    --s->inject_bad_alloc;
    throw std::bad_alloc();
  }
  compact_image(s);
  // the old plain positions are indices into the lists, which compaction keeps: nothing to redo
  DevArr<DevRec> recs;
  DevArr<uint32_t> plain, members;
  DevArr<GroupRec> groups;
  auto up = [&](auto& d, const auto& v) -> int {
    d.cap = std::max<uint64_t>(v.size() + v.size() / 2, 1u << 16);
    if (hipMalloc(reinterpret_cast<void**>(&d.p), d.cap * sizeof(v[0])) != hipSuccess) return EMQX_ENOMEM;
    FO_TRY(hipMemsetAsync(d.p, 0, d.cap * sizeof(v[0]), s->stream));
    if (!v.empty()) FO_TRY(hipMemcpyAsync(d.p, v.data(), v.size() * sizeof(v[0]), hipMemcpyHostToDevice, s->stream));
    return EMQX_OK;
  };
  DevArr<uint32_t> alive;
  std::vector<DevRec> drecs(s->recs.size());  // the device form (inline short lists)
  for (uint64_t f = 0; f < drecs.size(); ++f) drecs[f] = dev_rec(s, static_cast<uint32_t>(f));
  int rc = up(recs, drecs);
  DevArr<uint32_t> fcnt;
  if (rc == EMQX_OK) {
    fcnt.cap = recs.cap;
    if (hipMalloc(reinterpret_cast<void**>(&fcnt.p), fcnt.cap * sizeof(uint32_t)) != hipSuccess) rc = EMQX_ENOMEM;
    if (rc == EMQX_OK && hipMemsetAsync(fcnt.p, 0, fcnt.cap * sizeof(uint32_t), s->stream) != hipSuccess)
      rc = EMQX_EDEVICE;
    if (rc == EMQX_OK && launch_fcnt_from_recs(recs.p, drecs.size(), fcnt.p, s->stream) != hipSuccess)
      rc = EMQX_EDEVICE;
  }
  if (rc == EMQX_OK) rc = up(plain, s->plain);
  if (rc == EMQX_OK) rc = up(groups, s->groups);
  if (rc == EMQX_OK) rc = up(members, s->members);
  if (rc == EMQX_OK) rc = up(alive, s->alive);
  if (rc == EMQX_OK && hipStreamSynchronize(s->stream) != hipSuccess) rc = EMQX_EDEVICE;
  if (rc != EMQX_OK) {
    fo_free(recs.p);
    fo_free(fcnt.p);
    fo_free(plain.p);
    fo_free(groups.p);
    fo_free(members.p);
    fo_free(alive.p);
    return rc;
  }
  fo_free(s->d_recs.p);
  fo_free(s->d_fcnt.p);
  fo_free(s->d_plain.p);
  fo_free(s->d_groups.p);
  fo_free(s->d_members.p);
  fo_free(s->d_alive.p);
  s->d_recs = recs;
  s->d_fcnt = fcnt;
  s->d_plain = plain;
  s->d_groups = groups;
  s->d_members = members;
  s->d_alive = alive;
  s->dev_n_recs = static_cast<uint32_t>(s->recs.size());
  s->dev_n_alive = static_cast<uint32_t>(s->alive.size());
  s->dirty_alive.clear();
  s->st_words += s->plain.size() + s->members.size();
  s->st_records += s->recs.size() + s->groups.size();
  s->need_full = false;
  ++s->st_full;
  s->st_last_kind = 0;
  return EMQX_OK;
}

// Incremental commit: member lists and group lists of the changed slots / filters are
// rewritten in the image (moved to the arena's end when they outgrow their extent); then the
// touched words and records go to the device.
int live_commit(emqx_subtab* s, std::vector<void*>& retired) {
  const auto t0 = std::chrono::steady_clock::now();
  double pt[8] = {};
  int np = 0;
  auto mark = [&] {
    if (subtab_prof() && np < 8) pt[np++] = now_us();
  };
  mark();
  std::vector<std::pair<uint64_t, uint64_t>> member_ranges;
  std::vector<uint64_t> group_idx;
  const std::vector<uint32_t>& ds = s->dirty_slots;
  for (size_t di = 0; di < ds.size(); ++di) {
    // the slot 8 ahead, its member list, image extent and filter record 4 ahead (random lines)
    if (di + 8 < ds.size()) __builtin_prefetch(&s->slots[ds[di + 8]], 1);
    if (di + 4 < ds.size()) {
      const Slot& S4 = s->slots[ds[di + 4]];
      __builtin_prefetch(S4.members.data());
      if (uint64_t(S4.mbegin) < s->members.size()) __builtin_prefetch(s->members.data() + S4.mbegin, 1);
      __builtin_prefetch(&s->recs[S4.filter]);
    }
    const uint32_t sl = ds[di];
    Slot& S = s->slots[sl];
    S.dirty = false;
    const uint32_t nm = static_cast<uint32_t>(S.members.size());
    if (nm > S.mcap) {
      s->garbage += S.mcap;
      S.mbegin = static_cast<uint32_t>(s->members.size());
      S.mcap = grow_cap(nm, 4);
      s->members.resize(uint64_t(S.mbegin) + S.mcap, 0);
      ++s->st_moves;
    }
    std::copy(S.members.begin(), S.members.end(), s->members.begin() + S.mbegin);
    if (nm) member_ranges.emplace_back(S.mbegin, nm);
    const bool was_live = S.live_idx != SUB_NONE;
    if (was_live != (nm > 0)) {
      mark_glist(s, S.filter);
    } else if (nm) {
      const uint64_t gi = uint64_t(s->recs[S.filter].group_begin) + S.live_idx;
      s->groups[gi] = GroupRec{S.mbegin, nm, sl, S.group};
      group_idx.push_back(gi);
    }
  }
  for (uint32_t f : s->dirty_glists) {
    s->glist_flag[f] = 0;
    uint32_t ng = 0;
    for (uint32_t sl : s->fslots[f]) ng += s->slots[sl].members.empty() ? 0u : 1u;
    FilterRec& r = s->recs[f];
    s->n_live_groups = s->n_live_groups - r.n_groups + ng;
    if (ng > s->gcap[f]) {
      s->garbage += s->gcap[f];
      r.group_begin = static_cast<uint32_t>(s->groups.size());
      s->gcap[f] = grow_cap(ng, 2);
      s->groups.resize(uint64_t(r.group_begin) + s->gcap[f], GroupRec{0, 0, 0, 0});
      ++s->st_moves;
    }
    uint32_t k = 0;
    for (uint32_t sl : s->fslots[f]) {
      Slot& S = s->slots[sl];
      S.live_idx = SUB_NONE;
      if (S.members.empty()) continue;
      S.live_idx = k;
      s->groups[uint64_t(r.group_begin) + k] = GroupRec{S.mbegin, static_cast<uint32_t>(S.members.size()), sl, S.group};
      group_idx.push_back(uint64_t(r.group_begin) + k);
      ++k;
    }
    r.n_groups = ng;
    mark_rec(s, f);
  }
  if (s->plain.size() >= (1ull << 32) || s->members.size() >= (1ull << 32) || s->groups.size() >= (1ull << 32))
    return EMQX_ENOMEM;
  mark();  // 1: slots and group lists

  // ---- patches ----
  s->wpatch.clear();
  s->rpatch.clear();
  std::vector<std::pair<uint64_t, uint64_t>> copies_plain, copies_members;
  auto words = [&](const std::vector<std::pair<uint64_t, uint64_t>>& ranges, const std::vector<uint32_t>& img,
                   std::vector<std::pair<uint64_t, uint64_t>>& copies) {
    for (size_t i = 0; i < ranges.size(); ++i) {
      if (i + 16 < ranges.size()) __builtin_prefetch(img.data() + ranges[i + 16].first);  // random words
      const auto& rg = ranges[i];
      if (rg.second >= RANGE_COPY_MIN) {
        copies.push_back(rg);
        continue;
      }
      for (uint64_t w = rg.first; w < rg.first + rg.second; ++w)
        s->wpatch.push_back(WordPatch{static_cast<uint32_t>(w), static_cast<uint32_t>(w >> 32), img[w], 0});
    }
  };
  if (s->dirty_plain.size() >= PAR_MIN && par_threads() > 1) {
    // many touched plain words: the patches are built on the pool, a slice of ranges per
    // thread (counted, then written at their place)
    const auto& R = s->dirty_plain;
    const unsigned T = par_threads();
    std::vector<uint64_t> cnt(T + 1, 0);
    std::vector<std::vector<std::pair<uint64_t, uint64_t>>> cp(T);
    auto slice = [&](unsigned t, size_t* b, size_t* e) {
      *b = R.size() * t / T;
      *e = R.size() * (t + 1) / T;
    };
    std::atomic<unsigned> next{0};
    const std::function<void()> count = [&] {
      for (unsigned t; (t = next.fetch_add(1)) < T;) {
        size_t b, e;
        slice(t, &b, &e);
        uint64_t c = 0;
        for (size_t i = b; i < e; ++i)
          if (R[i].second < RANGE_COPY_MIN) c += R[i].second;
          else cp[t].push_back(R[i]);
        cnt[t + 1] = c;
      }
    };
    WorkPool::get().run(count, T);
    for (unsigned t = 0; t < T; ++t) cnt[t + 1] += cnt[t];
    s->wpatch.resize(cnt[T]);
    next = 0;
    const uint32_t* img = s->plain.data();
    WordPatch* out = s->wpatch.data();
    const std::function<void()> fill = [&] {
      for (unsigned t; (t = next.fetch_add(1)) < T;) {
        size_t b, e;
        slice(t, &b, &e);
        uint64_t o = cnt[t];
        for (size_t i = b; i < e; ++i) {
          if (i + 16 < e) __builtin_prefetch(img + R[i + 16].first);
          if (R[i].second >= RANGE_COPY_MIN) continue;
          for (uint64_t w = R[i].first; w < R[i].first + R[i].second; ++w)
            out[o++] = WordPatch{static_cast<uint32_t>(w), static_cast<uint32_t>(w >> 32), img[w], 0};
        }
      }
    };
    WorkPool::get().run(fill, T);
    for (auto& c : cp) copies_plain.insert(copies_plain.end(), c.begin(), c.end());
  } else {
    words(s->dirty_plain, s->plain, copies_plain);
  }
  const uint64_t n_plain_w = s->wpatch.size();
  mark();  // 2: plain words
  words(member_ranges, s->members, copies_members);
  const uint64_t n_member_w = s->wpatch.size() - n_plain_w;
  std::sort(s->dirty_alive.begin(), s->dirty_alive.end());
  s->dirty_alive.erase(std::unique(s->dirty_alive.begin(), s->dirty_alive.end()), s->dirty_alive.end());
  for (uint32_t w : s->dirty_alive) s->wpatch.push_back(WordPatch{w, 0u, s->alive[w], 0});
  const uint64_t n_alive_w = s->dirty_alive.size();
  mark();  // 3: member and alive words
  std::sort(group_idx.begin(), group_idx.end());
  group_idx.erase(std::unique(group_idx.begin(), group_idx.end()), group_idx.end());
  for (size_t k = 0; k < group_idx.size(); ++k) {
    if (k + 8 < group_idx.size()) __builtin_prefetch(&s->groups[group_idx[k + 8]]);
    const uint64_t gi = group_idx[k];
    const GroupRec& g = s->groups[gi];
    s->rpatch.push_back(RecPatch{static_cast<uint32_t>(gi), {0, 0, 0}, make_uint4(g.member_begin, g.n_members, g.slot, g.group_id),
                                 make_uint4(0, 0, 0, 0)});
  }
  const uint64_t n_group_p = s->rpatch.size();
  mark();  // 4: group records
  {  // two-stage prefetch: the record 16 ahead, its plain list (inline candidates) 8 ahead;
     // a long list on the pool, a slice per thread
    const std::vector<uint32_t>& dr = s->dirty_recs;
    const uint64_t r0 = s->rpatch.size();
    s->rpatch.resize(r0 + dr.size());
    RecPatch* out = s->rpatch.data() + r0;
    auto part = [&](size_t b, size_t e) {
      for (size_t i = b; i < e; ++i) {
        if (i + 16 < e) __builtin_prefetch(&s->recs[dr[i + 16]]);
        if (i + 8 < e) {
          const FilterRec& r8 = s->recs[dr[i + 8]];
          if (r8.n_plain && r8.n_plain <= FO_INLINE) __builtin_prefetch(s->plain.data() + r8.plain_begin);
        }
        const uint32_t f = dr[i];
        s->rec_flag[f] = 0;
        const DevRec d = dev_rec(s, f);
        out[i] = RecPatch{f, {0, 0, 0}, d.head, d.ext};
      }
    };
    const unsigned T = dr.size() >= PAR_MIN ? par_threads() : 1u;
    if (T > 1) {
      std::atomic<unsigned> next{0};
      const std::function<void()> run = [&] {
        for (unsigned t; (t = next.fetch_add(1)) < T;) part(dr.size() * t / T, dr.size() * (t + 1) / T);
      };
      WorkPool::get().run(run, T);
    } else {
      part(0, dr.size());
    }
  }
  const uint64_t n_rec_p = s->rpatch.size() - n_group_p;
  const auto t1 = std::chrono::steady_clock::now();
  mark();  // 5: filter records

  // ---- device: after the fan-outs in flight, before the next ones ----
  // Everything the device reads comes from pinned staging (a snapshot of the image taken here),
  // so the commit's copies and patch kernels run after s->mu is released; later fan-outs wait for
  // commit_ev; arrays a growth replaced are freed once it has passed (commit_finish).
  uint64_t cw = 0;
  for (const auto& c : copies_plain) cw += c.second;
  for (const auto& c : copies_members) cw += c.second;
  const uint64_t wp_bytes = s->wpatch.size() * sizeof(WordPatch), rp_bytes = s->rpatch.size() * sizeof(RecPatch);
  const uint64_t stage = cw * 4 + wp_bytes + rp_bytes;
  int rc = barrier_after_fanouts(s);
  if (rc == EMQX_OK && stage > s->stage_cap) {
    fo_hfree(s->h_stage);
    const uint64_t cap = std::max<uint64_t>(stage + stage / 2, 1u << 20);
    if (fo_halloc(s->h_stage, cap) != hipSuccess) rc = EMQX_ENOMEM;
    s->stage_cap = rc == EMQX_OK ? cap : 0;
  }
  if (rc == EMQX_OK) rc = dev_reserve(s, s->d_recs, s->recs.size(), s->dev_n_recs, retired);
  if (rc == EMQX_OK) rc = dev_reserve(s, s->d_fcnt, s->recs.size(), s->dev_n_recs, retired);
  if (rc == EMQX_OK) rc = dev_reserve(s, s->d_plain, s->plain.size(), s->d_plain.cap, retired);
  if (rc == EMQX_OK) rc = dev_reserve(s, s->d_members, s->members.size(), s->d_members.cap, retired);
  if (rc == EMQX_OK) rc = dev_reserve(s, s->d_groups, s->groups.size(), s->d_groups.cap, retired);
  if (rc == EMQX_OK) rc = dev_reserve(s, s->d_alive, s->alive.size(), s->dev_n_alive, retired);
  uint8_t* h = s->h_stage;
  auto up = [&](void* dst, const void* src, uint64_t bytes) {
    if (rc != EMQX_OK || !bytes) return;
    std::memcpy(h, src, bytes);
    if (hipMemcpyAsync(dst, h, bytes, hipMemcpyHostToDevice, s->stream) != hipSuccess) rc = EMQX_EDEVICE;
    h += bytes;
  };
  for (const auto& c : copies_plain) up(s->d_plain.p + c.first, s->plain.data() + c.first, c.second * 4);
  for (const auto& c : copies_members) up(s->d_members.p + c.first, s->members.data() + c.first, c.second * 4);
  if (rc == EMQX_OK && !s->wpatch.empty() && fo_ensure(s->d_wpatch.p, s->d_wpatch.cap, s->wpatch.size()) != hipSuccess)
    rc = EMQX_ENOMEM;
  up(s->d_wpatch.p, s->wpatch.data(), wp_bytes);
  if (rc == EMQX_OK && !s->rpatch.empty() && fo_ensure(s->d_rpatch.p, s->d_rpatch.cap, s->rpatch.size()) != hipSuccess)
    rc = EMQX_ENOMEM;
  up(s->d_rpatch.p, s->rpatch.data(), rp_bytes);
  if (rc == EMQX_OK &&
      launch_subtab_patches(s->d_plain.p, s->d_members.p, s->d_alive.p, s->d_wpatch.p, n_plain_w, n_member_w,
                            n_alive_w, s->d_groups.p, s->d_recs.p, s->d_fcnt.p, s->d_rpatch.p, n_group_p, n_rec_p,
                            s->stream) != hipSuccess)
    rc = EMQX_EDEVICE;
  if (rc != EMQX_OK) {
    s->need_full = true;  // the device copy is in an unknown state: the next commit rebuilds it
    return rc;
  }
  s->dev_n_recs = static_cast<uint32_t>(s->recs.size());
  s->dev_n_alive = static_cast<uint32_t>(s->alive.size());
  s->dirty_alive.clear();
  s->dirty_plain.clear();
  s->dirty_recs.clear();
  s->dirty_slots.clear();
  s->dirty_glists.clear();
  s->st_words += n_plain_w + n_member_w + n_alive_w + cw;
  s->st_records += n_group_p + n_rec_p;
  s->st_host_us = std::chrono::duration<double, std::micro>(t1 - t0).count();
  s->st_last_kind = 1;
  mark();  // 6: staging and uploads
  if (subtab_prof() && np == 7)
    std::fprintf(stderr,
                 "SUBTAB_PROF commit slots_us %.1f plain_us %.1f members_alive_us %.1f groups_us %.1f recs_us %.1f "
                 "upload_us %.1f alive %llu slots_recs %llu\n",
                 pt[1] - pt[0], pt[2] - pt[1], pt[3] - pt[2], pt[4] - pt[3], pt[5] - pt[4], pt[6] - pt[5],
                 (unsigned long long)n_alive_w, (unsigned long long)n_rec_p);
  return EMQX_OK;
}

// The host half of a commit (s->mu held): the image's changes into device operations enqueued
// on s->stream, ending with commit_ev.  `retired`: device arrays to free after commit_ev.
int commit_enqueue(emqx_subtab* s, std::vector<void*>& retired) {
  FO_TRY(hipSetDevice(s->device));
  if (s->recs.size() >= FANOUT_ID_LIMIT) return EMQX_EINVAL;
  const uint64_t live = s->plain_count() + s->n_members + s->recs.size();
  int rc;
  if (s->need_full || s->bulk || s->garbage > std::max<uint64_t>(1u << 20, live)) {
    int b = barrier_after_fanouts(s);
    rc = b != EMQX_OK ? b : full_commit(s);  // (synchronous: bulk loads and compactions)
  } else {
    rc = live_commit(s, retired);
  }
  if (rc != EMQX_OK) return rc;
  s->ops_pending = 0;
  s->bulk = false;
  FO_TRY(hipEventRecord(s->commit_ev, s->stream));
  s->commit_pending = true;
  ++s->st_commits;
  return EMQX_OK;
}

// The previous commit's device half (s->cmu held): waited for, and the arrays it replaced
// freed.  Its staging is then free for the next host half.
int commit_drain(emqx_subtab* s) {
  int rc = EMQX_OK;
  if (s->commit_inflight && hipEventSynchronize(s->commit_ev) != hipSuccess) rc = EMQX_EDEVICE;
  if (s->inject_drain_error) {
    --s->inject_drain_error;
    rc = EMQX_EDEVICE;
  }
  s->commit_inflight = false;
  for (void* p : s->retired_prev) (void)hipFree(p);
  s->retired_prev.clear();
  return rc;
}

// A whole commit (s->cmu held, s->mu not): the previous commit's device half is drained first
// (outside s->mu), then the host half runs under s->mu and the call returns without waiting for
// its own device half: every fan-out enqueued after the return waits for commit_ev on the
// device, so the changes are visible to it all the same, and the caller's next changes (the next
// subscribe round, the coalescer's next batch) are prepared while the device applies these.  A
// device error of a commit is reported by the next one (which then rebuilds the tables).
int commit_now(emqx_subtab* s) {
  const auto t0 = std::chrono::steady_clock::now();
  int rc = commit_drain(s);
  std::vector<void*> retired;
  {
    std::lock_guard<std::mutex> g(s->mu);
    if (rc == EMQX_OK) rc = commit_enqueue(s, retired);
    if (rc != EMQX_OK) s->need_full = true;
    s->st_total_us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  }
  s->retired_prev = std::move(retired);
  s->commit_inflight = rc == EMQX_OK;
  return rc;
}

// ---- pick state -----------------------------------------------------------------------------

int ps_alloc(uint64_t cap, uint64_t*& keys, uint32_t*& vals, hipStream_t st) {
  keys = nullptr;
  vals = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&keys), cap * sizeof(uint64_t)) != hipSuccess) return EMQX_ENOMEM;
  if (hipMalloc(reinterpret_cast<void**>(&vals), cap * sizeof(uint32_t)) != hipSuccess) {
    (void)hipFree(keys);
    keys = nullptr;
    return EMQX_ENOMEM;
  }
  FO_TRY(hipMemsetAsync(keys, 0xFF, cap * sizeof(uint64_t), st));  // PS_EMPTY
  FO_TRY(hipMemsetAsync(vals, 0xFF, cap * sizeof(uint32_t), st));  // PS_NOVAL
  return EMQX_OK;
}

// The table exists and will stay at most half full (live keys and tombstones as of the last
// finished call, plus `incoming` new keys) — otherwise it is rehashed, dropping the tombstones,
// into a table of at least four times the live keys; that waits for the fan-outs in flight.
int ps_ready(emqx_subtab* s, uint64_t incoming) {
  if (!s->ps_keys) {
    uint64_t cap = PS_INIT_CAP;
    while (cap < 4 * incoming) cap <<= 1;
    FO_TRY(hipMemsetAsync(s->ps_count, 0, sizeof(unsigned long long), s->stream));
    FO_TRY(hipMemsetAsync(s->ps_tombs, 0, sizeof(unsigned long long), s->stream));
    int rc = ps_alloc(cap, s->ps_keys, s->ps_vals, s->stream);
    if (rc != EMQX_OK) return rc;
    FO_TRY(hipStreamSynchronize(s->stream));
    s->ps_cap = cap;
    return EMQX_OK;
  }
  const uint64_t live = s->h_ps_seen[0], tombs = s->h_ps_seen[1];
  if (!s->ps_force_grow && (live + tombs + incoming) * 2 <= s->ps_cap) return EMQX_OK;
  int rc = barrier_after_fanouts(s);
  if (rc != EMQX_OK) return rc;
  if (s->state_pending) FO_TRY(hipStreamWaitEvent(s->stream, s->state_ev, 0));
  uint64_t cap = PS_INIT_CAP;
  while (cap < 4 * (live + incoming)) cap <<= 1;
  if (s->ps_force_grow) cap = std::max(cap, 2 * s->ps_cap);
  uint64_t* keys;
  uint32_t* vals;
  rc = ps_alloc(cap, keys, vals, s->stream);
  if (rc != EMQX_OK) return rc;
  FO_TRY(hipMemsetAsync(s->ps_count, 0, sizeof(unsigned long long), s->stream));
  FO_TRY(hipMemsetAsync(s->ps_tombs, 0, sizeof(unsigned long long), s->stream));
  FO_TRY(launch_ps_rehash(s->ps_keys, s->ps_vals, s->ps_cap, keys, vals, cap - 1, s->ps_count, s->stream));
  FO_TRY(hipStreamSynchronize(s->stream));
  fo_free(s->ps_keys);
  fo_free(s->ps_vals);
  s->ps_keys = keys;
  s->ps_vals = vals;
  s->ps_cap = cap;
  s->ps_force_grow = false;
  FO_TRY(hipMemcpy(s->h_ps_seen, s->ps_count, sizeof(unsigned long long), hipMemcpyDeviceToHost));
  s->h_ps_seen[1] = 0;
  return EMQX_OK;
}

// Applies the queued forget_publishers calls on stream st (before a stateful call's write
// kernel inserts keys of those publishers' possible successors): one pass over the table.
int flush_forgets(emqx_subtab* s, hipStream_t st) {
  if (s->pending_forget.empty() || !s->ps_keys) {
    s->pending_forget.clear();
    return EMQX_OK;
  }
  std::vector<uint32_t>& p = s->pending_forget;
  std::sort(p.begin(), p.end());
  p.erase(std::unique(p.begin(), p.end()), p.end());
  // the previous pass has read its list (pinned staging and device copy) before they are reused
  if (s->forget_pending) FO_TRY(hipEventSynchronize(s->forget_ev));
  if (s->d_forget.cap < p.size()) {
    FO_TRY(fo_ensure(s->d_forget.p, s->d_forget.cap, p.size()));
    FO_TRY(fo_halloc(s->h_forget, s->d_forget.cap));
  }
  std::memcpy(s->h_forget, p.data(), p.size() * 4);
  FO_TRY(hipMemcpyAsync(s->d_forget.p, s->h_forget, p.size() * 4, hipMemcpyHostToDevice, st));
  // resolves in flight on other streams write ps_vals of entries this pass may tombstone: after them
  if (s->state_pending) FO_TRY(hipStreamWaitEvent(st, s->state_ev, 0));
  FO_TRY(launch_ps_forget(s->ps_keys, s->ps_cap, s->d_forget.p, p.size(), s->ps_count, s->ps_tombs, st));
  FO_TRY(hipEventRecord(s->forget_ev, st));
  s->forget_pending = true;
  p.clear();
  return EMQX_OK;
}

// ---- the fan-out pipeline ---------------------------------------------------------------------

FoScratch* scratch_for(emqx_subtab* s, hipStream_t st) {
  for (auto& c : s->scratch)
    if (c->stream == st) return c.get();
  auto c = std::make_unique<FoScratch>();
  c->stream = st;
  if (hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess) return nullptr;
  s->scratch.push_back(std::move(c));
  return s->scratch.back().get();
}

// Sizes the stateful scratch of c for m_cap entries and the learnt number of picks.
int stateful_scratch(emqx_subtab* s, FoScratch* c, uint64_t m_cap, uint64_t cap) {
  // the pick list: the last finished call's picks with a margin (a call with more is flagged,
  // writes no ids and is rerun after this grows); never more than the delivery capacity
  const uint64_t seen = std::max<uint64_t>(s->h_ps_seen[2], c->rerun_picks);
  uint64_t want = std::max<uint64_t>(c->pk_cap, std::max<uint64_t>(1u << 16, seen + seen / 2 + 4096));
  want = std::min<uint64_t>(want, std::max<uint64_t>(cap + 1, 1u << 16));
  if (want > c->pk_cap || !c->pk) {
    FO_TRY(fo_alloc(c->pk, 4 * want));
    FO_TRY(fo_alloc(c->run_ent, want));
    FO_TRY(fo_alloc(c->run_cnt, want));
    FO_TRY(fo_alloc(c->seg, want));
    FO_TRY(fo_alloc(c->seg_from, want));
    c->pk_cap = want;
    const uint64_t tb = fanout_sort_temp_bytes(want);
    if (tb > c->sort_temp_bytes || !c->sort_temp) {
      FO_TRY(fo_alloc(c->sort_temp, tb));
      c->sort_temp_bytes = tb;
    }
  }
  if (c->cap_tag != s->ps_cap) {  // (a new table: the stream's earlier calls have drained)
    FO_TRY(fo_alloc(c->tag, s->ps_cap));
    FO_TRY(hipMemsetAsync(c->tag, 0, s->ps_cap * sizeof(unsigned long long), c->stream));
    c->cap_tag = s->ps_cap;
    c->stamp = 0;
  }
  if (!c->multi) FO_TRY(fo_alloc(c->multi, FO_MULTI_CAP));
  if (!c->run_named) FO_TRY(fo_alloc(c->run_named, FO_BLOCKS));
  if (++c->stamp == 0) {  // stamps wrapped: no tag may look current
    FO_TRY(hipMemsetAsync(c->tag, 0, s->ps_cap * sizeof(unsigned long long), c->stream));
    c->stamp = 1;
  }
  return EMQX_OK;
}

// Enqueue the fan-out of one match CSR on st, no host synchronisation (s->mu held); m_cap
// bounds the match entries (sizes the scratch; a longer CSR is refused on the device, as is
// one whose match summary `msum` reports a problem); the summary goes to `summary`
// (FO_SUM_WORDS u64).  round_robin / sticky: the resolve waits for the table's previous one, so
// the per-publisher state advances call after call in the order the calls were enqueued.
int enqueue_fanout(emqx_subtab* s, uint32_t strategy, const uint64_t* d_moff, const uint32_t* d_mids, uint64_t n,
                   uint64_t m_cap, const uint32_t* d_keys, uint64_t* d_out_off, uint32_t* d_out_subs,
                   uint32_t* d_out_fil, uint64_t cap, uint64_t* summary, hipStream_t st, const uint64_t* msum) {
  FoScratch* c = scratch_for(s, st);
  if (!c) return EMQX_EDEVICE;
  const bool stateful = fo_stateful(strategy);
  if (!d_out_subs) cap = 0;
  if (stateful && cap >= (1ull << 32)) return EMQX_EINVAL;  // pick positions are 32-bit
  if (stateful) {
    const uint64_t pk_guess = std::max<uint64_t>(c->pk_cap, std::max<uint64_t>(1u << 16, s->h_ps_seen[2] * 2));
    int rc = ps_ready(s, std::min<uint64_t>(pk_guess, std::max<uint64_t>(cap, 1u << 16)));
    if (rc == EMQX_OK) rc = stateful_scratch(s, c, m_cap, cap);
    if (rc == EMQX_OK) rc = flush_forgets(s, st);
    if (rc != EMQX_OK) return rc;
  }
  FO_TRY(fo_ensure(c->entry_topic, c->cap_entry_topic, std::max<uint64_t>(m_cap, 1)));
  {
    const uint64_t chunks = m_cap / FO_WCHUNK + 2;
    if (chunks > c->cap_chunks || !c->csum) {
      FO_TRY(fo_alloc(c->csum, chunks));
      FO_TRY(fo_alloc(c->gchunk, chunks));
      c->cap_chunks = chunks;
    }
    if (!c->partials) FO_TRY(fo_alloc(c->partials, 4 * FO_BLOCKS));
  }
  if (!c->ctl) FO_TRY(fo_alloc(c->ctl, FO_CTL_WORDS));
  if (!c->h_seen) {
    FO_TRY(fo_halloc(c->h_seen, 2));
    c->h_seen[0] = c->h_seen[1] = 0;
  }
  if (s->commit_pending) FO_TRY(hipStreamWaitEvent(st, s->commit_ev, 0));
  // (c->ctl is zeroed by the call's first kernel, fanout_entry_topic)
  FanoutArgs a{};
  a.recs = s->d_recs.p;
  a.fcnt = s->d_fcnt.p;
  a.n_recs = s->dev_n_recs;
  a.plain = s->d_plain.p;
  a.groups = s->d_groups.p;
  a.members = s->d_members.p;
  a.alive = s->d_alive.p;
  a.n_alive_words = s->dev_n_alive;
  a.ps_keys = s->ps_keys;
  a.ps_vals = s->ps_vals;
  a.ps_count = s->ps_count;
  a.ps_tombs = s->ps_tombs;
  a.ps_mask = s->ps_cap ? s->ps_cap - 1 : 0;
  if (stateful) {
    a.pk_keys = c->pk;
    a.pk_vals = c->pk + c->pk_cap;
    a.pk_skeys = c->pk + 2 * c->pk_cap;
    a.pk_svals = c->pk + 3 * c->pk_cap;
    a.pk_cap = c->pk_cap;
    a.tag = c->tag;
    a.stamp = c->stamp;
    a.run_ent = c->run_ent;
    a.run_named = c->run_named;
    a.seg = c->seg;
    a.seg_from = c->seg_from;
    // the small resolve path (no sort) unless the last finished call had many picks per run:
    // picks - runs bounds the picks of multi-pick runs by half
    const uint64_t S_last = s->h_ps_seen[2], R_last = s->h_ps_seen[3];
    if (!c->rerun_large && S_last < R_last + FO_MULTI_CAP / 2) {
      a.run_cnt = c->run_cnt;
      a.multi = c->multi;
      FO_TRY(hipMemsetAsync(c->run_cnt, 0, c->pk_cap * sizeof(uint32_t), st));
    }
  }
  a.ctl = c->ctl;
  a.ps_seen = mapped(s->h_ps_seen);
  a.call_seen = mapped(c->h_seen);
  c->rerun_picks = 0;  // (consumed by this call's sizing)
  c->rerun_large = false;
  a.moff = d_moff;
  a.mids = d_mids;
  a.n = n;
  a.m_cap = m_cap;
  a.msum = msum;
  a.keys = d_keys;
  a.strategy = strategy;
  s->seed = s->seed * 1664525u + 1013904223u;
  a.seed = s->seed;
  a.rr_first0 = s->rr_first0;
  a.entry_topic = c->entry_topic;
  a.csum = c->csum;
  a.gchunk = c->gchunk;
  a.partials = c->partials;
  a.out_off = d_out_off;
  a.out_subs = d_out_subs;
  a.out_filters = d_out_fil;
  a.cap = cap;
  a.summary = summary;
  FO_TRY(launch_fanout(a, m_cap, st));
  if (stateful) {
    if (s->state_pending) FO_TRY(hipStreamWaitEvent(st, s->state_ev, 0));
    FO_TRY(launch_fanout_resolve(a, c->sort_temp, c->sort_temp_bytes, st));
    FO_TRY(hipEventRecord(s->state_ev, st));
    s->state_pending = true;
  }
  FO_TRY(hipEventRecord(c->done, st));
  c->used = true;
  return EMQX_OK;
}

// After a call on stream st flagged FO_SUM_F_RERUN: what to grow before it runs again.  The
// sizes come from the flagged call's own counts (its scratch's h_seen, written by its finish
// kernel), not from the shared h_ps_seen, which a smaller call on another stream may have
// overwritten since: the rerun sizes its pick list from them and takes the large resolve path
// (FO_SUM_F_PICKS is raised for a list too short and for too many multi-pick picks alike).
void note_rerun(emqx_subtab* s, hipStream_t st, uint64_t flags) {
  if (flags & FO_SUM_F_STATE_FULL) s->ps_force_grow = true;
  if (flags & FO_SUM_F_PICKS) {
    FoScratch* c = scratch_for(s, st);
    if (c && c->h_seen) {
      c->rerun_picks = c->h_seen[0];
      c->rerun_large = true;
    }
  }
}

// Synchronous form: enqueue, drain, read the summary.  On overflow the write kernel wrote
// nothing (and consumed no pick state); *n_out is the capacity required.  A call flagged for a
// rerun (state table or pick scratch too small: nothing consumed) grows them and runs again.
int run_fanout(emqx_subtab* s, uint32_t strategy, const uint64_t* d_moff, const uint32_t* d_mids, uint64_t n,
               uint64_t m, const uint32_t* d_keys, uint64_t* d_out_off, uint32_t* d_out_subs, uint32_t* d_out_fil,
               uint64_t cap, uint64_t* n_out, hipStream_t st) {
  FoScratch* c = scratch_for(s, st);
  if (!c) return EMQX_EDEVICE;
  if (!c->h_sum) FO_TRY(fo_halloc(c->h_sum, FO_SUM_WORDS));
  for (int attempt = 0;; ++attempt) {
    int rc = enqueue_fanout(s, strategy, d_moff, d_mids, n, m, d_keys, d_out_off, d_out_subs, d_out_fil, cap,
                            mapped(c->h_sum), st, nullptr);
    if (rc != EMQX_OK) return rc;
    FO_TRY(hipStreamSynchronize(st));
    *n_out = c->h_sum[FO_SUM_TOTAL];
    const uint64_t fl = c->h_sum[FO_SUM_FLAGS];
    if (fl & FO_SUM_F_MATCH) return EMQX_EINVAL;
    if (fl & FO_SUM_F_OVERFLOW) return EMQX_EOVERFLOW;
    if (!(fl & FO_SUM_F_RERUN)) return EMQX_OK;
    if (attempt >= 3) return EMQX_ENOMEM;
    note_rerun(s, st, fl);
  }
}

int ensure_stream(emqx_subtab* s) {
  if (!s->stream) {
    FO_TRY(hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking));
    FO_TRY(hipEventCreateWithFlags(&s->commit_ev, hipEventDisableTiming));
    FO_TRY(hipEventCreateWithFlags(&s->state_ev, hipEventDisableTiming));
    FO_TRY(hipEventCreateWithFlags(&s->forget_ev, hipEventDisableTiming));
    FO_TRY(fo_halloc(s->h_total, 2));
    FO_TRY(fo_halloc(s->h_ps_seen, 4));
    s->h_ps_seen[0] = s->h_ps_seen[1] = s->h_ps_seen[2] = s->h_ps_seen[3] = 0;
    FO_TRY(fo_alloc(s->ps_count, 1));  // (read by every call's finish kernel)
    FO_TRY(fo_alloc(s->ps_tombs, 1));
    FO_TRY(hipMemset(s->ps_count, 0, sizeof(unsigned long long)));
    FO_TRY(hipMemset(s->ps_tombs, 0, sizeof(unsigned long long)));
  }
  return EMQX_OK;
}

bool strategy_ok(uint32_t strategy, bool have_keys) {
  if (strategy > EMQX_SHARE_HASH_TOPIC) return false;
  if ((strategy == EMQX_SHARE_HASH_CLIENTID || strategy == EMQX_SHARE_HASH_TOPIC) && !have_keys) return false;
  return true;
}

}  // namespace

// ---- pinned publish batches -------------------------------------------------------------------

struct PubBatchPriv {
  emqx_engine* e = nullptr;
  emqx_subtab* s = nullptr;
  uint32_t strategy = 0;
  bool use_keys = true;
  hipStream_t stream = nullptr;
  hipEvent_t done = nullptr;
  uint8_t* d_tbytes = nullptr;
  uint64_t* d_toffs = nullptr;
  uint32_t* d_keys = nullptr;
  uint64_t* d_moff = nullptr;
  uint32_t* d_mids = nullptr;
  uint64_t cap_mids = 0;
  uint64_t* d_ooff = nullptr;
  uint32_t* d_osubs = nullptr;
  uint32_t* d_ofil = nullptr;
  uint64_t* d_msum = nullptr;  // match summary (8 words) then fan-out summary (4 words)
  uint64_t* h_sums = nullptr;  // pinned copy of both
  uint4* d_erec = nullptr;     // one-launch small path: per match entry its record and topic
  uint32_t* d_etop = nullptr;
  uint64_t mids_per_topic = 16;  // learnt match ids per topic (sizes d_mids)
  uint64_t limit = ~0ull;        // deliveries the submission may write (<= cap_out): a call that
                                 // needs more writes no ids and consumes no pick state
  bool pending = false;
};

emqx_subtab::~emqx_subtab() {
  (void)hipSetDevice(device);
  if (stream) (void)hipStreamSynchronize(stream);
  for (void* p : retired_prev) (void)hipFree(p);
  for (auto& c : scratch)
    if (c->used) (void)hipEventSynchronize(c->done);
  for (emqx_pub_batch* b : pb_free) emqx_pub_batch_destroy(b);
  fo_free(d_recs.p);
  fo_free(d_fcnt.p);
  fo_free(d_plain.p);
  fo_free(d_groups.p);
  fo_free(d_members.p);
  fo_free(d_wpatch.p);
  fo_free(d_rpatch.p);
  fo_free(d_alive.p);
  fo_free(d_forget.p);
  fo_free(ps_keys);
  fo_free(ps_vals);
  fo_free(ps_count);
  fo_free(ps_tombs);
  for (auto& c : scratch) c->release();
  fo_hfree(h_total);
  fo_hfree(h_ps_seen);
  fo_hfree(h_stage);
  if (commit_ev) (void)hipEventDestroy(commit_ev);
  if (state_ev) (void)hipEventDestroy(state_ev);
  if (forget_ev) (void)hipEventDestroy(forget_ev);
  fo_hfree(h_forget);
  if (stream) (void)hipStreamDestroy(stream);
}

namespace {

constexpr uint64_t PB_MSUM_WORDS = 8;

int pb_alloc(emqx_pub_batch* b, uint64_t cap_topics, uint64_t cap_bytes, uint64_t cap_out, bool keep_inputs) {
  auto* p = static_cast<PubBatchPriv*>(b->priv);
  FO_TRY(hipSetDevice(p->s->device));
  if (cap_topics > b->cap_topics) {
    uint64_t* t = nullptr;
    uint32_t* k = nullptr;
    FO_TRY(fo_halloc(t, cap_topics + 1));
    FO_TRY(fo_halloc(k, cap_topics));
    if (keep_inputs && b->topic_offsets) {
      std::memcpy(t, b->topic_offsets, (b->cap_topics + 1) * sizeof(uint64_t));
      std::memcpy(k, b->keys, b->cap_topics * sizeof(uint32_t));
    }
    fo_hfree(b->topic_offsets);
    fo_hfree(b->keys);
    b->topic_offsets = t;
    b->keys = k;
    FO_TRY(fo_halloc(b->out_offsets, cap_topics + 1));
    FO_TRY(fo_alloc(p->d_toffs, cap_topics + 1));
    FO_TRY(fo_alloc(p->d_keys, cap_topics));
    FO_TRY(fo_alloc(p->d_moff, cap_topics + 1));
    FO_TRY(fo_alloc(p->d_ooff, cap_topics + 1));
    b->cap_topics = cap_topics;
  }
  if (cap_bytes > b->cap_bytes) {
    uint8_t* t = nullptr;
    FO_TRY(fo_halloc(t, cap_bytes + 16));
    if (keep_inputs && b->topic_bytes) std::memcpy(t, b->topic_bytes, b->cap_bytes);
    fo_hfree(b->topic_bytes);
    b->topic_bytes = t;
    FO_TRY(fo_alloc(p->d_tbytes, cap_bytes + 16));
    b->cap_bytes = cap_bytes;
  }
  if (cap_out > b->cap_out) {
    FO_TRY(fo_halloc(b->out_subs, cap_out));
    FO_TRY(fo_halloc(b->out_filters, cap_out));
    FO_TRY(fo_alloc(p->d_osubs, cap_out));
    FO_TRY(fo_alloc(p->d_ofil, cap_out));
    b->cap_out = cap_out;
  }
  return EMQX_OK;
}

// After the match ids of the batch are in HBM: fan-out, the delivery CSR into the pinned
// outputs, both summaries into pinned memory (s->mu is taken here).
// fanout_words_only: copy back only the fan-out summary (the one-launch path's fallback, whose
// match summary the small kernel already wrote into the mapped h_sums: d_msum's match words
// are an older call's).
int pb_enqueue_fanout(emqx_pub_batch* b, uint64_t m_cap, const uint64_t* msum, bool fanout_words_only = false) {
  auto* p = static_cast<PubBatchPriv*>(b->priv);
  emqx_subtab* s = p->s;
  uint64_t* fsum = p->d_msum + PB_MSUM_WORDS;
  const uint64_t cap = std::min(b->cap_out, p->limit);
  {
    std::lock_guard<std::mutex> g(s->mu);
    int rc = enqueue_fanout(s, p->strategy, p->d_moff, p->d_mids, b->n, m_cap, p->use_keys ? p->d_keys : nullptr,
                            p->d_ooff, p->d_osubs, p->d_ofil, cap, fsum, p->stream, msum);
    if (rc != EMQX_OK) return rc;
  }
  FO_TRY(launch_fanout_to_host(p->d_ooff, b->n, p->d_osubs, p->d_ofil, fsum, cap, mapped(b->out_offsets),
                               mapped(b->out_subs), mapped(b->out_filters), p->stream));
  const uint64_t skip = fanout_words_only ? PB_MSUM_WORDS : 0;
  FO_TRY(hipMemcpyAsync(p->h_sums + skip, p->d_msum + skip, (PB_MSUM_WORDS + FO_SUM_WORDS - skip) * sizeof(uint64_t),
                        hipMemcpyDeviceToHost, p->stream));
  return EMQX_OK;
}

// The one-launch small path (kernels.h SmallArgs): match and stateless fan-out in one kernel that
// reads the pinned inputs and writes the pinned outputs and both summaries itself.  Returns
// SMALL_NOT_TAKEN (nothing enqueued) when the batch or the strategy does not qualify.
int pb_enqueue_small(emqx_pub_batch* b, uint64_t nbytes) {
  auto* p = static_cast<PubBatchPriv*>(b->priv);
  emqx_subtab* s = p->s;
  if (fo_stateful(p->strategy) || b->n == 0 || b->n > SMALL_MAX_N) return SMALL_NOT_TAKEN;
  hipStream_t st = p->stream;
  if (!p->d_erec) {
    FO_TRY(fo_alloc(p->d_erec, SMALL_FO_MAX_ENTRIES));
    FO_TRY(fo_alloc(p->d_etop, SMALL_FO_MAX_ENTRIES));
  }
  const uint64_t want = p->mids_per_topic * b->n + 1024;
  if (want > p->cap_mids) {
    p->cap_mids = want + want / 4;
    FO_TRY(fo_alloc(p->d_mids, p->cap_mids));
  }
  std::lock_guard<std::mutex> g(s->mu);
  FoScratch* c = scratch_for(s, st);  // (its done event orders later commits after this fan-out)
  if (!c) return EMQX_EDEVICE;
  if (s->commit_pending) FO_TRY(hipStreamWaitEvent(st, s->commit_ev, 0));
  SmallFanout f{};
  f.recs = reinterpret_cast<const uint4*>(s->d_recs.p);
  f.n_recs = s->dev_n_recs;
  f.plain = s->d_plain.p;
  f.groups = reinterpret_cast<const uint4*>(s->d_groups.p);
  f.members = s->d_members.p;
  f.strategy = p->strategy;
  s->seed = s->seed * 1664525u + 1013904223u;
  f.seed = s->seed;
  f.h_keys = p->use_keys ? mapped(b->keys) : nullptr;
  f.d_keys = p->d_keys;
  f.erec = p->d_erec;
  f.etop = p->d_etop;
  f.ps_count = s->ps_count;
  f.h_off = mapped(b->out_offsets);
  f.h_subs = mapped(b->out_subs);
  f.h_fil = mapped(b->out_filters);
  f.cap = std::min(b->cap_out, p->limit);
  f.h_sum = mapped(p->h_sums) + PB_MSUM_WORDS;
  int rc = engine_small_batch(p->e, EMQX_MODE_ROUTES, mapped(b->topic_bytes), mapped(b->topic_offsets), b->n, nbytes,
                              p->d_tbytes, p->d_toffs, p->d_moff, p->d_mids, p->cap_mids, mapped(p->h_sums), f, st);
  if (rc != EMQX_OK) return rc;
  FO_TRY(hipEventRecord(c->done, st));
  c->used = true;
  return EMQX_OK;
}

int pb_enqueue(emqx_pub_batch* b) {
  auto* p = static_cast<PubBatchPriv*>(b->priv);
  const uint64_t n = b->n, nbytes = n ? b->topic_offsets[n] : 0;
  hipStream_t st = p->stream;
  {
    const int rc = pb_enqueue_small(b, nbytes);
    if (rc == EMQX_OK) {
      FO_TRY(hipEventRecord(p->done, st));
      p->pending = true;
      return EMQX_OK;
    }
    if (rc != SMALL_NOT_TAKEN) return rc;
  }
  if (nbytes) FO_TRY(hipMemcpyAsync(p->d_tbytes, b->topic_bytes, nbytes, hipMemcpyHostToDevice, st));
  FO_TRY(hipMemcpyAsync(p->d_toffs, b->topic_offsets, (n + 1) * sizeof(uint64_t), hipMemcpyHostToDevice, st));
  if (p->use_keys && n) FO_TRY(hipMemcpyAsync(p->d_keys, b->keys, n * sizeof(uint32_t), hipMemcpyHostToDevice, st));
  const uint64_t want = p->mids_per_topic * n + 1024;
  if (want > p->cap_mids) {
    p->cap_mids = want + want / 4;
    FO_TRY(fo_alloc(p->d_mids, p->cap_mids));
  }
  int rc = emqx_match_batch_device_async(p->e, EMQX_MODE_ROUTES, p->d_tbytes, p->d_toffs, n, p->d_moff, p->d_mids,
                                         p->cap_mids, p->d_msum, st);
  if (rc != EMQX_OK) return rc;
  rc = pb_enqueue_fanout(b, p->cap_mids, p->d_msum);
  if (rc != EMQX_OK) return rc;
  FO_TRY(hipEventRecord(p->done, st));
  p->pending = true;
  return EMQX_OK;
}

int pb_wait(emqx_pub_batch* b) {
  auto* p = static_cast<PubBatchPriv*>(b->priv);
  if (!p->pending) return EMQX_EINVAL;
  FO_TRY(hipSetDevice(p->s->device));
  p->pending = false;
  FO_TRY(hipEventSynchronize(p->done));
  const uint64_t* ms = p->h_sums;
  const uint64_t* fs = p->h_sums + PB_MSUM_WORDS;
  if (ms[0] != 0) {
    // the match did not complete in the batch's buffers (its scratch learnt a larger size, or
    // more ids than d_mids holds): rerun it synchronously, then the fan-out (which read nothing)
    if (ms[0] & 4) return EMQX_EINVAL;  // a topic over 65535 bytes
    uint64_t m = 0;
    if (ms[1] + 1024 > p->cap_mids) {
      p->cap_mids = ms[1] + ms[1] / 4 + 1024;
      FO_TRY(fo_alloc(p->d_mids, p->cap_mids));
    }
    int rc = emqx_match_batch_device(p->e, EMQX_MODE_ROUTES, p->d_tbytes, p->d_toffs, b->n, p->d_moff, p->d_mids,
                                     p->cap_mids, &m, p->stream);
    if (rc == EMQX_EOVERFLOW) {
      p->cap_mids = m + m / 4 + 1024;
      FO_TRY(fo_alloc(p->d_mids, p->cap_mids));
      rc = emqx_match_batch_device(p->e, EMQX_MODE_ROUTES, p->d_tbytes, p->d_toffs, b->n, p->d_moff, p->d_mids,
                                   p->cap_mids, &m, p->stream);
    }
    if (rc != EMQX_OK) return rc;
    rc = pb_enqueue_fanout(b, p->cap_mids, nullptr);
    if (rc != EMQX_OK) return rc;
    FO_TRY(hipStreamSynchronize(p->stream));
    p->mids_per_topic = std::max<uint64_t>(p->mids_per_topic, m / std::max<uint64_t>(b->n, 1) + 1);
  } else if (b->n) {
    p->mids_per_topic = std::max<uint64_t>(4, (ms[1] + ms[1] / 4) / b->n + 1);
  }
  if (fs[FO_SUM_FLAGS] & FO_SUM_F_SMALL) {  // the one-launch path's fan-out did not fit: batched kernels
    int rc = pb_enqueue_fanout(b, p->cap_mids, nullptr, true);
    if (rc != EMQX_OK) return rc;
    FO_TRY(hipStreamSynchronize(p->stream));
  }
  // round_robin / sticky state table or pick scratch too small: nothing was consumed; grow, rerun
  for (int attempt = 0; (fs[FO_SUM_FLAGS] & FO_SUM_F_RERUN) && !(fs[FO_SUM_FLAGS] & ~FO_SUM_F_RERUN); ++attempt) {
    if (attempt >= 3) return EMQX_ENOMEM;
    {
      std::lock_guard<std::mutex> g(p->s->mu);
      note_rerun(p->s, p->stream, fs[FO_SUM_FLAGS]);
    }
    int rc = pb_enqueue_fanout(b, p->cap_mids, nullptr);
    if (rc != EMQX_OK) return rc;
    FO_TRY(hipStreamSynchronize(p->stream));
  }
  b->n_out = fs[FO_SUM_TOTAL];
  if (fs[FO_SUM_FLAGS] & FO_SUM_F_MATCH) return EMQX_EDEVICE;
  if (fs[FO_SUM_FLAGS] & FO_SUM_F_OVERFLOW) return EMQX_EOVERFLOW;
  return EMQX_OK;
}

}  // namespace

namespace {

// Entry points that grow host tables: an allocation failure (here or on a pool worker) becomes
// EMQX_ENOMEM instead of an exception through the C ABI (which would end the hosting VM); the
// image may hold part of the call's ops, so the next commit rebuilds the device tables.
template <class F>
int subtab_guarded(emqx_subtab* s, F f) {
  int rc;
  try {
    return f();
  } catch (const std::bad_alloc&) {
    rc = EMQX_ENOMEM;
  } catch (...) {
    rc = EMQX_EDEVICE;
  }
  try {
    std::lock_guard<std::mutex> g(s->mu);
    s->need_full = true;
  } catch (...) {
  }
  return rc;
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
  int rc = ensure_stream(s);
  if (rc == EMQX_OK) {
    std::lock_guard<std::mutex> g(s->cmu);
    rc = commit_now(s);
  }
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

// The serial ops: a plain op's map entry and record, a $share op's (filter, group) slot 16 ops
// ahead and its membership line 8 ops ahead are prefetched (the maps are too large for the
// caches; each op was one or two dependent misses).
void prefetch_op(const emqx_subtab* s, const uint32_t* fs, const uint32_t* subs, const uint32_t* gs,
                 const uint32_t* idx, uint64_t j, uint64_t nl) {
  if (j + 16 < nl) {
    const uint64_t i = idx ? idx[j + 16] : j + 16;
    if (gs && gs[i] != EMQX_NO_GROUP) {
      s->slot_of.prefetch((uint64_t(fs[i]) << 32) | gs[i]);
    } else if (fs[i] < s->recs.size()) {  // a plain op: its map entry and record
      s->plain_pos[pp_shard(fs[i])].prefetch((uint64_t(fs[i]) << 32) | subs[i]);
      __builtin_prefetch(&s->recs[fs[i]]);
    }
  }
  if (j + 8 < nl) {
    const uint64_t i = idx ? idx[j + 8] : j + 8;
    if (gs && gs[i] != EMQX_NO_GROUP) {
      const uint32_t sl = s->slot_of.find((uint64_t(fs[i]) << 32) | gs[i]);
      if (sl != SUB_NONE) {
        s->member_set.prefetch((uint64_t(sl) << 32) | subs[i]);
        __builtin_prefetch(&s->slots[sl]);
      }
    }
  }
}

// A long batch: its plain ops go through plain_batch (threads), and *rest_out = the indices of
// its $share ops, which the caller applies serially after them (plain lists and group
// memberships are separate structures, so the split changes no result).  False: a short batch.
bool plain_parallel(emqx_subtab* s, const uint32_t* fs, const uint32_t* subs, const uint32_t* group_ids,
                    uint64_t n, bool add, std::vector<uint32_t>* rest_out) {
  if (n < PAR_MIN || par_threads() < 2) return false;
  rest_out->clear();
  if (!group_ids) {
    plain_batch(s, fs, subs, n, add);
    return true;
  }
  std::vector<uint32_t> pf, ps;
  pf.reserve(n);
  ps.reserve(n);
  for (uint64_t i = 0; i < n; ++i) {
    if (group_ids[i] == EMQX_NO_GROUP) {
      pf.push_back(fs[i]);
      ps.push_back(subs[i]);
    } else {
      rest_out->push_back(static_cast<uint32_t>(i));
    }
  }
  if (!pf.empty()) plain_batch(s, pf.data(), ps.data(), pf.size(), add);
  return true;
}

static int subtab_add_impl(emqx_subtab* s, const uint32_t* filter_ids, const uint32_t* sub_ids, const uint32_t* group_ids,
                    uint64_t n) {
  if (!s || !ids_ok(filter_ids, sub_ids, n)) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(s->mu);
  std::vector<uint32_t> rest;
  const double t0 = subtab_prof() ? now_us() : 0;
  const bool split = plain_parallel(s, filter_ids, sub_ids, group_ids, n, true, &rest);
  const double t1 = subtab_prof() ? now_us() : 0;
  const uint64_t nl = split ? rest.size() : n;
  struct Report {
    double t0, t1;
    uint64_t n, nl;
    const char* what;
    ~Report() {
      if (subtab_prof())
        std::fprintf(stderr, "SUBTAB_PROF %s n %llu plain_us %.1f serial %llu serial_us %.1f\n", what,
                     (unsigned long long)n, t1 - t0, (unsigned long long)nl, now_us() - t1);
    }
  } report{t0, t1, n, nl, "add"};
  for (uint64_t j = 0; j < nl; ++j) {
    prefetch_op(s, filter_ids, sub_ids, group_ids, split ? rest.data() : nullptr, j, nl);
    const uint64_t i = split ? rest[j] : j;
    const uint32_t f = filter_ids[i], sub = sub_ids[i];
    const uint32_t grp = group_ids ? group_ids[i] : EMQX_NO_GROUP;
    set_alive_bit(s, sub, true);  // a subscribing process is alive
    if (grp == EMQX_NO_GROUP) {
      plain_add(s, f, sub);
      continue;
    }
    ensure_filter(s, f);
    const uint64_t key = (uint64_t(f) << 32) | grp;
    uint32_t sl = s->slot_of.find(key);
    if (sl == SUB_NONE) {
      if (s->slots.size() >= FANOUT_SHARED_BIT) return EMQX_ENOMEM;
      sl = static_cast<uint32_t>(s->slots.size());
      s->slots.push_back(Slot{f, grp, {}, 0, 0, SUB_NONE, false});
      s->slot_of.insert(key, sl);
      s->fslots[f].push_back(sl);
    }
    if (s->member_set.insert((uint64_t(sl) << 32) | sub, 1)) {
      s->slots[sl].members.push_back(sub);
      ++s->n_members;
      mark_slot(s, sl);
      note_op(s);
    }
  }
  return EMQX_OK;
}

static int subtab_remove_impl(emqx_subtab* s, const uint32_t* filter_ids, const uint32_t* sub_ids, const uint32_t* group_ids,
                       uint64_t n) {
  if (!s || !ids_ok(filter_ids, sub_ids, n)) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(s->mu);
  std::vector<uint32_t> rest;
  const double t0 = subtab_prof() ? now_us() : 0;
  const bool split = plain_parallel(s, filter_ids, sub_ids, group_ids, n, false, &rest);
  const double t1 = subtab_prof() ? now_us() : 0;
  const uint64_t nl = split ? rest.size() : n;
  struct Report {
    double t0, t1;
    uint64_t n, nl;
    const char* what;
    ~Report() {
      if (subtab_prof())
        std::fprintf(stderr, "SUBTAB_PROF %s n %llu plain_us %.1f serial %llu serial_us %.1f\n", what,
                     (unsigned long long)n, t1 - t0, (unsigned long long)nl, now_us() - t1);
    }
  } report{t0, t1, n, nl, "remove"};
  for (uint64_t j = 0; j < nl; ++j) {
    prefetch_op(s, filter_ids, sub_ids, group_ids, split ? rest.data() : nullptr, j, nl);
    const uint64_t i = split ? rest[j] : j;
    const uint32_t f = filter_ids[i], sub = sub_ids[i];
    const uint32_t grp = group_ids ? group_ids[i] : EMQX_NO_GROUP;
    if (f >= s->recs.size()) continue;
    if (grp == EMQX_NO_GROUP) {
      plain_remove(s, f, sub);
      continue;
    }
    const uint32_t sl = s->slot_of.find((uint64_t(f) << 32) | grp);
    if (sl == SUB_NONE) continue;
    if (s->member_set.erase((uint64_t(sl) << 32) | sub)) {
      auto& v = s->slots[sl].members;
      v.erase(std::find(v.begin(), v.end(), sub));  // keeps the others' order (ETS bag)
      --s->n_members;
      mark_slot(s, sl);
      note_op(s);
    }
  }
  return EMQX_OK;
}

int emqx_subtab_commit(emqx_subtab* s) {
  if (!s) return EMQX_EINVAL;
  return subtab_guarded(s, [&] {
    std::lock_guard<std::mutex> g(s->cmu);
    return commit_now(s);
  });
}

int emqx_subtab_commit_wait(emqx_subtab* s) {
  if (!s) return EMQX_EINVAL;
  // (guarded: the rebuild below allocates host vectors of every record, the path most likely
  // to throw, and the coalescer calls this on every batch)
  return subtab_guarded(s, [&] {
    std::lock_guard<std::mutex> g(s->cmu);
    if (hipSetDevice(s->device) != hipSuccess) return static_cast<int>(EMQX_EDEVICE);
    int rc = commit_drain(s);
    if (rc == EMQX_OK) return static_cast<int>(EMQX_OK);
    // the device half failed: its tables are in an unknown state, so they are rebuilt from the
    // host image now (a full commit), and the error goes to the callers of the failed commit
    {
      std::lock_guard<std::mutex> m(s->mu);
      s->need_full = true;
    }
    if (commit_now(s) == EMQX_OK) (void)commit_drain(s);
    return rc;
  });
}

int emqx_subtab_set_tuning(emqx_subtab* s, const char* key, int64_t value) {
  if (!s || !key || value < 0) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(s->cmu);
  if (!std::strcmp(key, "inject_drain_error")) {
    s->inject_drain_error = static_cast<uint32_t>(value);
  } else if (!std::strcmp(key, "inject_bad_alloc")) {
    s->inject_bad_alloc = static_cast<uint32_t>(value);
  } else if (!std::strcmp(key, "rr_seed0")) {  // round_robin's first pick: member 0 (SURVEY §8 d)
    s->rr_first0 = value ? 1u : 0u;
  } else {
    return EMQX_ENOTFOUND;
  }
  return EMQX_OK;
}

int emqx_subtab_stats(emqx_subtab* s, uint64_t* counts4) {
  if (!s || !counts4) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(s->mu);
  counts4[0] = s->plain_count();
  counts4[1] = s->n_members;
  counts4[2] = s->n_live_groups;
  counts4[3] = s->d_recs.cap * sizeof(DevRec) + s->d_plain.cap * 4 + s->d_groups.cap * sizeof(GroupRec) +
               s->d_members.cap * 4 + s->ps_cap * 12 + s->d_fcnt.cap * sizeof(uint32_t);
  return EMQX_OK;
}

int emqx_subtab_commit_stats(emqx_subtab* s, uint64_t* out, uint32_t n) {
  if (!s || (n && !out)) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(s->mu);
  const uint64_t v[9] = {s->st_last_kind, s->st_commits, s->st_full, s->st_words, s->st_records, s->st_moves,
                         s->garbage, static_cast<uint64_t>(s->st_host_us), static_cast<uint64_t>(s->st_total_us)};
  for (uint32_t i = 0; i < n && i < 9; ++i) out[i] = v[i];
  return EMQX_OK;
}

static int subtab_forget_publishers_impl(emqx_subtab* s, const uint32_t* publishers, uint64_t n) {
  if (!s || (n && !publishers)) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(s->mu);
  if (!s->ps_keys) return EMQX_OK;  // no state kept yet
  // queued: the next stateful fan-out or re-pick applies every queued publisher in one pass
  s->pending_forget.insert(s->pending_forget.end(), publishers, publishers + n);
  return EMQX_OK;
}

static int subtab_set_alive_impl(emqx_subtab* s, const uint32_t* sub_ids, uint64_t n, int alive) {
  if (!s || (n && !sub_ids)) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(s->mu);
  for (uint64_t i = 0; i < n; ++i)
    if (sub_ids[i] != SUB_NONE) set_alive_bit(s, sub_ids[i], alive != 0);
  return EMQX_OK;
}

int emqx_share_repick(emqx_subtab* s, uint32_t strategy, uint64_t n, const uint32_t* filter_ids,
                      const uint32_t* group_ids, const uint32_t* keys, const uint64_t* failed_offsets,
                      const uint32_t* failed_subs, uint32_t* out_subs, uint32_t* out_kind) {
  if (!s || strategy > EMQX_SHARE_HASH_TOPIC || (n && (!filter_ids || !group_ids || !failed_offsets || !out_subs ||
                                                       !out_kind)))
    return EMQX_EINVAL;
  if ((strategy == EMQX_SHARE_HASH_CLIENTID || strategy == EMQX_SHARE_HASH_TOPIC) && n && !keys) return EMQX_EINVAL;
  if (n == 0) return EMQX_OK;
  if (failed_offsets[0] != 0) return EMQX_EINVAL;
  for (uint64_t i = 0; i < n; ++i)
    if (failed_offsets[i + 1] < failed_offsets[i]) return EMQX_EINVAL;
  const uint64_t nf = failed_offsets[n];
  if (nf && !failed_subs) return EMQX_EINVAL;
  std::lock_guard<std::mutex> g(s->mu);
  FO_TRY(hipSetDevice(s->device));
  hipStream_t st = s->stream;
  int rc = ps_ready(s, n);
  if (rc == EMQX_OK) rc = flush_forgets(s, st);
  if (rc != EMQX_OK) return rc;
  // one device block: the requests, the failed lists, the outputs, a flag word
  const uint64_t bytes = 12 * n + 8 * (n + 1) + 4 * nf + 8 * n + 64;
  uint8_t* h = nullptr;
  uint8_t* d = nullptr;
  if (fo_halloc(h, bytes) != hipSuccess) return EMQX_ENOMEM;
  if (fo_alloc(d, bytes) != hipSuccess) {
    fo_hfree(h);
    return EMQX_ENOMEM;
  }
  auto place = [&](uint64_t& off, uint64_t sz) {
    const uint64_t o = off;
    off = (off + sz + 7) & ~7ull;
    return o;
  };
  uint64_t off = 0;
  const uint64_t o_f = place(off, 4 * n), o_g = place(off, 4 * n), o_k = place(off, 4 * n);
  const uint64_t o_fo = place(off, 8 * (n + 1)), o_fs = place(off, 4 * nf), o_os = place(off, 4 * n);
  const uint64_t o_ok = place(off, 4 * n), o_ctl = place(off, 8);
  std::memcpy(h + o_f, filter_ids, 4 * n);
  std::memcpy(h + o_g, group_ids, 4 * n);
  if (keys) std::memcpy(h + o_k, keys, 4 * n);
  else std::memset(h + o_k, 0, 4 * n);
  std::memcpy(h + o_fo, failed_offsets, 8 * (n + 1));
  if (nf) std::memcpy(h + o_fs, failed_subs, 4 * nf);
  std::memset(h + o_ctl, 0, 8);
  RepickArgs a{};
  a.recs = s->d_recs.p;
  a.n_recs = s->dev_n_recs;
  a.groups = s->d_groups.p;
  a.members = s->d_members.p;
  a.alive = s->d_alive.p;
  a.n_alive_words = s->dev_n_alive;
  a.ps_keys = s->ps_keys;
  a.ps_vals = s->ps_vals;
  a.ps_count = s->ps_count;
  a.ps_mask = s->ps_cap - 1;
  a.strategy = strategy;
  s->seed = s->seed * 1664525u + 1013904223u;
  a.seed = s->seed;
  a.rr_first0 = s->rr_first0;
  a.n = n;
  a.filter_ids = reinterpret_cast<const uint32_t*>(d + o_f);
  a.group_ids = reinterpret_cast<const uint32_t*>(d + o_g);
  a.keys = reinterpret_cast<const uint32_t*>(d + o_k);
  a.failed_off = reinterpret_cast<const uint64_t*>(d + o_fo);
  a.failed = reinterpret_cast<const uint32_t*>(d + o_fs);
  a.out_subs = reinterpret_cast<uint32_t*>(d + o_os);
  a.out_kind = reinterpret_cast<uint32_t*>(d + o_ok);
  a.ctl = reinterpret_cast<unsigned long long*>(d + o_ctl);
  // after the last commit and the last stateful resolve; the next stateful call waits for this
  rc = EMQX_OK;
  if ((s->commit_pending && hipStreamWaitEvent(st, s->commit_ev, 0) != hipSuccess) ||
      (s->state_pending && hipStreamWaitEvent(st, s->state_ev, 0) != hipSuccess) ||
      hipMemcpyAsync(d, h, off, hipMemcpyHostToDevice, st) != hipSuccess || launch_share_repick(a, st) != hipSuccess ||
      hipMemcpyAsync(h + o_os, d + o_os, off - o_os, hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipEventRecord(s->state_ev, st) != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
    rc = EMQX_EDEVICE;
  s->state_pending = true;
  if (rc == EMQX_OK) {
    std::memcpy(out_subs, h + o_os, 4 * n);
    std::memcpy(out_kind, h + o_ok, 4 * n);
    uint64_t fl;
    std::memcpy(&fl, h + o_ctl, 8);
    if (fl & FO_SUM_F_STATE_FULL) s->ps_force_grow = true;  // (those picks were made without state)
  }
  fo_free(d);
  fo_hfree(h);
  return rc;
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
  FO_TRY(hipMemcpyAsync(s->h_total, d_match_offsets, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  FO_TRY(hipMemcpyAsync(s->h_total + 1, d_match_offsets + n, sizeof(uint64_t), hipMemcpyDeviceToHost, st));
  FO_TRY(hipStreamSynchronize(st));
  const uint64_t b0 = s->h_total[0], b1 = s->h_total[1];
  if (b1 < b0) return EMQX_EINVAL;
  if (b1 - b0 && !d_match_ids) return EMQX_EINVAL;
  return run_fanout(s, strategy, d_match_offsets, d_match_ids, n, b1 - b0, d_pick_keys, d_out_offsets, d_out_subs,
                    d_out_filters, cap, n_out, st);
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
                        d_out_subs, d_out_filters, cap, summary, st, nullptr);
}

int emqx_pub_batch_create(emqx_engine* e, emqx_subtab* s, uint32_t strategy, uint64_t cap_topics, uint64_t cap_bytes,
                          uint64_t cap_out, emqx_pub_batch** out) {
  if (!e || !s || !out || strategy > EMQX_SHARE_HASH_TOPIC) return EMQX_EINVAL;
  *out = nullptr;
  auto* b = new (std::nothrow) emqx_pub_batch();
  auto* p = new (std::nothrow) PubBatchPriv();
  if (!b || !p) {
    delete b;
    delete p;
    return EMQX_ENOMEM;
  }
  std::memset(b, 0, sizeof(*b));
  b->priv = p;
  p->e = e;
  p->s = s;
  p->strategy = strategy;
  p->use_keys = strategy != EMQX_SHARE_RANDOM;
  int rc = EMQX_OK;
  if (hipSetDevice(s->device) != hipSuccess || hipStreamCreateWithFlags(&p->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&p->done, hipEventDisableTiming) != hipSuccess ||
      fo_alloc(p->d_msum, PB_MSUM_WORDS + FO_SUM_WORDS) != hipSuccess ||
      fo_halloc(p->h_sums, PB_MSUM_WORDS + FO_SUM_WORDS) != hipSuccess)
    rc = EMQX_EDEVICE;
  if (rc == EMQX_OK)
    rc = pb_alloc(b, std::max<uint64_t>(cap_topics, 1), std::max<uint64_t>(cap_bytes, 64),
                  std::max<uint64_t>(cap_out, 64), false);
  if (rc != EMQX_OK) {
    emqx_pub_batch_destroy(b);
    return rc;
  }
  b->topic_offsets[0] = 0;
  *out = b;
  return EMQX_OK;
}

int emqx_pub_batch_destroy(emqx_pub_batch* b) {
  if (!b) return EMQX_EINVAL;
  auto* p = static_cast<PubBatchPriv*>(b->priv);
  (void)hipSetDevice(p->s->device);
  if (p->stream) (void)hipStreamSynchronize(p->stream);
  fo_hfree(b->topic_bytes);
  fo_hfree(b->topic_offsets);
  fo_hfree(b->keys);
  fo_hfree(b->out_offsets);
  fo_hfree(b->out_subs);
  fo_hfree(b->out_filters);
  fo_hfree(p->h_sums);
  fo_free(p->d_tbytes);
  fo_free(p->d_toffs);
  fo_free(p->d_keys);
  fo_free(p->d_moff);
  fo_free(p->d_mids);
  fo_free(p->d_ooff);
  fo_free(p->d_osubs);
  fo_free(p->d_ofil);
  fo_free(p->d_msum);
  fo_free(p->d_erec);
  fo_free(p->d_etop);
  {  // the subtab keeps a scratch per stream: it goes with the stream
    std::lock_guard<std::mutex> g(p->s->mu);
    auto& v = p->s->scratch;
    for (size_t i = 0; i < v.size(); ++i)
      if (v[i]->stream == p->stream) {
        v[i]->release();
        v.erase(v.begin() + static_cast<std::ptrdiff_t>(i));
        break;
      }
  }
  if (p->done) (void)hipEventDestroy(p->done);
  if (p->stream) (void)hipStreamDestroy(p->stream);
  delete p;
  delete b;
  return EMQX_OK;
}

int emqx_pub_batch_reserve(emqx_pub_batch* b, uint64_t cap_topics, uint64_t cap_bytes, uint64_t cap_out) {
  if (!b || static_cast<PubBatchPriv*>(b->priv)->pending) return EMQX_EINVAL;
  return pb_alloc(b, cap_topics, cap_bytes, cap_out, true);
}

int emqx_pub_batch_submit(emqx_pub_batch* b) {
  if (!b) return EMQX_EINVAL;
  auto* p = static_cast<PubBatchPriv*>(b->priv);
  if (p->pending || b->n > b->cap_topics) return EMQX_EINVAL;
  const uint64_t* o = b->topic_offsets;
  if (o[0] != 0 || o[b->n] > b->cap_bytes) return EMQX_EINVAL;
  for (uint64_t i = 0; i < b->n; ++i)
    if (o[i + 1] < o[i]) return EMQX_EINVAL;
  if (fo_stateful(p->strategy) && b->cap_out >= (1ull << 32)) return EMQX_EINVAL;
  FO_TRY(hipSetDevice(p->s->device));
  return pb_enqueue(b);
}

int emqx_pub_batch_wait(emqx_pub_batch* b) {
  if (!b) return EMQX_EINVAL;
  return pb_wait(b);
}

int emqx_pub_batch_query(emqx_pub_batch* b) {
  if (!b) return EMQX_EINVAL;
  auto* p = static_cast<PubBatchPriv*>(b->priv);
  return !p->pending || hipEventQuery(p->done) == hipSuccess ? 1 : 0;
}

// Host buffers of any kind: one pinned publish batch of the table's pool, grown to the call.
int emqx_publish_batch(emqx_engine* e, emqx_subtab* s, uint32_t strategy, const uint8_t* topic_bytes,
                       const uint64_t* topic_offsets, uint64_t n, const uint32_t* pick_keys, uint64_t* out_offsets,
                       uint32_t* out_subs, uint32_t* out_filters, uint64_t cap, uint64_t* n_out) {
  if (!e || !s || !n_out || !out_offsets || (n && !topic_offsets) || !strategy_ok(strategy, pick_keys != nullptr))
    return EMQX_EINVAL;
  for (uint64_t i = 0; i < n; ++i)
    if (topic_offsets[i + 1] < topic_offsets[i]) return EMQX_EINVAL;
  const uint64_t b0 = n ? topic_offsets[0] : 0, b1 = n ? topic_offsets[n] : 0;
  if (b1 > b0 && !topic_bytes) return EMQX_EINVAL;
  if (fo_stateful(strategy) && cap >= (1ull << 32)) cap = (1ull << 32) - 1;
  FO_TRY(hipSetDevice(s->device));
  emqx_pub_batch* b = nullptr;
  {
    std::lock_guard<std::mutex> g(s->pb_mu);
    for (size_t i = 0; i < s->pb_free.size(); ++i)
      if (static_cast<PubBatchPriv*>(s->pb_free[i]->priv)->strategy == strategy &&
          static_cast<PubBatchPriv*>(s->pb_free[i]->priv)->e == e) {
        b = s->pb_free[i];
        s->pb_free.erase(s->pb_free.begin() + static_cast<std::ptrdiff_t>(i));
        break;
      }
  }
  int rc = EMQX_OK;
  if (!b) rc = emqx_pub_batch_create(e, s, strategy, n, b1 - b0, std::min<uint64_t>(cap, 64 * n + 64), &b);
  if (rc == EMQX_OK) rc = emqx_pub_batch_reserve(b, n, b1 - b0, std::min<uint64_t>(cap, std::max<uint64_t>(b->cap_out, 64)));
  if (rc == EMQX_OK) {
    if (b1 > b0) std::memcpy(b->topic_bytes, topic_bytes + b0, b1 - b0);
    for (uint64_t i = 0; i <= n; ++i) b->topic_offsets[i] = n ? topic_offsets[i] - b0 : 0;
    if (pick_keys && n) std::memcpy(b->keys, pick_keys, n * sizeof(uint32_t));
    else if (n) std::memset(b->keys, 0, n * sizeof(uint32_t));
    b->n = n;
    auto* p = static_cast<PubBatchPriv*>(b->priv);
    p->limit = cap;  // a result the caller cannot take is not made (no pick state consumed)
    rc = emqx_pub_batch_submit(b);
    if (rc == EMQX_OK) rc = emqx_pub_batch_wait(b);
    if (rc == EMQX_EOVERFLOW && b->n_out <= cap) {  // nothing was written and no pick state used
      rc = emqx_pub_batch_reserve(b, n, b1 - b0, b->n_out);
      if (rc == EMQX_OK) rc = emqx_pub_batch_submit(b);
      if (rc == EMQX_OK) rc = emqx_pub_batch_wait(b);
    }
    p->limit = ~0ull;
    *n_out = b->n_out;
    if (rc == EMQX_OK) {
      std::memcpy(out_offsets, b->out_offsets, (n + 1) * sizeof(uint64_t));
      if (b->n_out > cap) {
        rc = EMQX_EOVERFLOW;
      } else {
        if (out_subs && b->n_out) std::memcpy(out_subs, b->out_subs, b->n_out * sizeof(uint32_t));
        if (out_filters && b->n_out) std::memcpy(out_filters, b->out_filters, b->n_out * sizeof(uint32_t));
      }
    } else if (rc == EMQX_EOVERFLOW) {
      std::memcpy(out_offsets, b->out_offsets, (n + 1) * sizeof(uint64_t));
    }
  }
  if (b) {
    std::lock_guard<std::mutex> g(s->pb_mu);
    s->pb_free.push_back(b);
  }
  return rc;
}

int emqx_subtab_add(emqx_subtab* s, const uint32_t* filter_ids, const uint32_t* sub_ids, const uint32_t* group_ids,
                    uint64_t n) {
  if (!s) return EMQX_EINVAL;
  return subtab_guarded(s, [&] { return subtab_add_impl(s, filter_ids, sub_ids, group_ids, n); });
}

int emqx_subtab_remove(emqx_subtab* s, const uint32_t* filter_ids, const uint32_t* sub_ids, const uint32_t* group_ids,
                       uint64_t n) {
  if (!s) return EMQX_EINVAL;
  return subtab_guarded(s, [&] { return subtab_remove_impl(s, filter_ids, sub_ids, group_ids, n); });
}

int emqx_subtab_set_alive(emqx_subtab* s, const uint32_t* sub_ids, uint64_t n, int alive) {
  if (!s) return EMQX_EINVAL;
  return subtab_guarded(s, [&] { return subtab_set_alive_impl(s, sub_ids, n, alive); });
}

int emqx_subtab_forget_publishers(emqx_subtab* s, const uint32_t* publishers, uint64_t n) {
  if (!s) return EMQX_EINVAL;
  return subtab_guarded(s, [&] { return subtab_forget_publishers_impl(s, publishers, n); });
}

}  // extern "C"
