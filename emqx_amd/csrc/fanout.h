// Device layout and launch interface of the publish fan-out stage (fanout_kernels.hip,
// fanout.cpp).  See DESIGN.md §3.3.
//
// Reference: after emqx_router:match_routes/1, emqx_broker:publish/1 aggregates the routes
// (aggre/1, apps/emqx/src/emqx_broker.erl:261-272) and routes each one:
//   {Filter, node()}  -> dispatch/2 -> every local subscriber of Filter, with the {shard, I}
//                        buckets of big filters expanded (emqx_broker.erl:500-524)
//   {Filter, Group}   -> emqx_shared_sub:dispatch/3 -> ONE member of the group, picked by the
//                        configured strategy (apps/emqx/src/emqx_shared_sub.erl:234-288)
// Here both become one flattened CSR of deliveries per published topic.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.h"

namespace emqx {

constexpr uint32_t SUB_NONE = 0xFFFFFFFFu;
constexpr uint32_t FANOUT_SHARED_BIT = 0x80000000u;  // set in out_filters[] for $share picks
constexpr uint32_t FANOUT_RETRY_BIT = 0x40000000u;   // ... of type retry (do_pick/6's {retry, Sub})
constexpr uint32_t FANOUT_ID_LIMIT = 0x40000000u;    // filter ids stay below the flag bits

// Per filter id (16 B, one load per matched filter).  The plain list and the group list are
// extents of their arenas with room to grow in place (incremental commits, fanout.cpp).
struct FilterRec {
  uint32_t plain_begin;  // first entry in plain[]
  uint32_t n_plain;      // plain (non-shared) subscribers
  uint32_t group_begin;  // first entry in groups[]
  uint32_t n_groups;     // $share groups with >= 1 member
};
// The device copy of a record is 32 B (two per 64-B line): head = the record, ext unused; for a
// filter with 1..FO_INLINE plain subscribers and no $share group the list itself,
// head {s0, n_plain | FO_INLINE_BIT, s1, s2}, ext {s3, s4, s5, s6}, so its deliveries cost no
// second random line (the host image keeps the arena form; fanout.cpp dev_rec).  Round 5 widened
// it from 16 B and three subscribers: at Poisson(4.5) subscribers per filter (config E) the
// inline share of match entries went from 34 % to 91 %.
struct alignas(32) DevRec {
  uint4 head;
  uint4 ext;
};
constexpr uint32_t FO_INLINE = 7;
constexpr uint32_t FO_INLINE_HEAD = 3;  // inline subscribers held in head (x, z, w); the rest in ext
constexpr uint32_t FO_INLINE_BIT = 0x80000000u;
// Inline subscriber r < FO_INLINE_HEAD from the head.
__host__ __device__ inline uint32_t fo_inline_head(uint4 h, uint32_t r) { return r == 0 ? h.x : (r == 1 ? h.z : h.w); }
// Address of inline subscriber r >= FO_INLINE_HEAD of filter f (in the record's own 32 B).
__host__ __device__ inline const uint32_t* fo_inline_ext(const DevRec* recs, uint32_t f, uint32_t r) {
  return reinterpret_cast<const uint32_t*>(&recs[f].ext) + (r - FO_INLINE_HEAD);
}
__host__ __device__ inline uint32_t fo_rec_plain(uint4 r) { return r.y & ~FO_INLINE_BIT; }
__host__ __device__ inline uint32_t fo_rec_groups(uint4 r) { return (r.y & FO_INLINE_BIT) ? 0u : r.w; }

// The count pass's dense per-filter word (4 B, maintained on the device from each record it
// writes): deliveries (n_plain + n_groups) in bits 0..23 and $share groups in bits 24..31, each
// saturated; a saturated word sends the count pass to the record's head.  Sixteen per 64-B line where
// the device records fit two, so the count pass's random reads mostly hit in L2.
constexpr uint32_t FO_CNT_DELIV_MAX = 0xFFFFFFu, FO_CNT_GROUPS_MAX = 0xFFu;
__host__ __device__ inline uint32_t fo_cnt_word(uint4 r) {
  const uint32_t d = fo_rec_plain(r) + fo_rec_groups(r), g = fo_rec_groups(r);
  return (d >= FO_CNT_DELIV_MAX || g >= FO_CNT_GROUPS_MAX) ? 0xFFFFFFFFu : (d | (g << 24));
}

// Per ($share group, filter) with members (16 B).
struct GroupRec {
  uint32_t member_begin;  // first entry in members[] (subscription order)
  uint32_t n_members;
  uint32_t slot;          // persistent slot id of (filter, group): the pick-state key's high half
  uint32_t group_id;      // caller's group id
};

// Pick state of round_robin / sticky, per (group slot, publisher): the reference keeps it in
// the publishing process's dictionary under {shared_sub_round_robin | shared_sub_sticky, Group,
// Topic} (emqx_shared_sub.erl:234-247,279-285).  Open-addressed table, key = slot << 32 |
// publisher, value = the last round-robin index or the sticky subscriber (PS_NOVAL: none yet).
constexpr uint64_t PS_EMPTY = ~0ull;
constexpr uint64_t PS_TOMB = ~0ull - 1;
constexpr uint32_t PS_NOVAL = 0xFFFFFFFFu;
constexpr uint32_t PS_MAX_PROBES = 64;
// Per-call control words of one scratch (memset per call).
constexpr uint32_t FO_CTL_PICKS = 0;  // round_robin / sticky picks of the call (the pick list's length)
constexpr uint32_t FO_CTL_FLAGS = 1;  // FO_SUM_F_* bits raised by the kernels
constexpr uint32_t FO_CTL_SPARE = 2;
constexpr uint32_t FO_CTL_MULTI = 3;  // small path: picks of runs with more than one pick
constexpr uint32_t FO_CTL_WORDS = 4;
// Small resolve path: at most this many picks in runs of more than one pick (sorted in LDS).
constexpr uint32_t FO_MULTI_CAP = 4096;

// Liveness of subscribers: erlang:is_process_alive/1 (emqx_shared_sub.erl:386-393), one bit per
// subscriber id; a sticky pick stays while its subscriber is alive, member or not.
__host__ __device__ inline bool fo_alive(const uint32_t* alive, uint32_t n_words, uint32_t sub) {
  return sub != SUB_NONE && (sub >> 5) < n_words && ((alive[sub >> 5] >> (sub & 31u)) & 1u);
}

struct FanoutArgs {
  const DevRec* recs;
  const uint32_t* fcnt;      // [n_recs] fo_cnt_word of each record (the count pass's dense copy)
  uint32_t n_recs;           // filter ids >= n_recs have no subscribers
  const uint32_t* plain;
  const GroupRec* groups;
  const uint32_t* members;
  const uint32_t* alive;     // [n_alive_words] liveness bitmap
  uint32_t n_alive_words;
  // pick state (round_robin / sticky)
  uint64_t* ps_keys;         // [ps_mask + 1]
  uint32_t* ps_vals;         // [ps_mask + 1]
  unsigned long long* ps_count;  // live keys (device)
  unsigned long long* ps_tombs;  // tombstones (device)
  uint64_t ps_mask;
  // the call's pick list (round_robin / sticky): one (run, output position) pair per $share pick,
  // written in output order, then stably sorted by run.  A run is the call's picks of one
  // (group slot, publisher) state entry, named by the list index of its first pick to be probed
  // (so ids are < picks <= pk_cap - 1, few key bits), and pk_cap - 1 pads the list past the
  // call's picks.
  uint32_t* pk_keys;         // [pk_cap] run id (written by the probe)
  uint32_t* pk_vals;         // [pk_cap] output position
  uint32_t* pk_skeys;        // [pk_cap] sorted keys (large path); before: the pick's group record
  uint32_t* pk_svals;        // [pk_cap] their positions (large path); before: the pick's publisher,
                             // then (probe) its state entry
  uint64_t pk_cap;
  unsigned long long* tag;   // [ps_mask + 1] per state entry: call stamp << 32 | its run id in that call
  uint32_t stamp;            // this call's stamp (never 0)
  uint32_t* run_ent;         // [pk_cap] run id -> state entry
  unsigned long long* seg;   // [pk_cap] per run: first list index | first pick << 32
  uint32_t* seg_from;        // [pk_cap] sticky: list index from which the run's pick is constant
  uint32_t* run_cnt;         // small path ([pk_cap], zeroed per call): picks per run; null: large path
  uint32_t* run_named;       // [FO_BLOCKS] runs named per block of the probe kernel
  unsigned long long* multi; // small path [FO_MULTI_CAP]: run << 32 | list index of multi-pick runs' picks
  unsigned long long* ctl;   // [FO_CTL_WORDS]
  unsigned long long* ps_seen;  // host-mapped [4]: live keys, tombstones, picks, runs of the last finished call
  unsigned long long* call_seen;  // host-mapped [2] of the calling stream's scratch: this call's picks, runs
                                  // (the shared ps_seen holds whichever call finished last)
  // the match CSR
  const uint64_t* moff;      // match CSR offsets [n+1]
  const uint32_t* mids;      // match CSR filter ids [moff[n] - moff[0]]
  uint64_t n;                // topics
  uint64_t m_cap;            // entries the scratch holds (a larger CSR is refused, not read)
  const uint64_t* msum;      // the match call's summary (device) or null: flags != 0 -> no fan-out
  const uint32_t* keys;      // per topic: phash2 key (hash strategies) / publisher (rr, sticky), or null
  uint32_t strategy;         // EMQX_SHARE_*
  uint32_t seed;             // per-call seed of random picks
  uint32_t rr_first0;        // round_robin's first pick of a state entry is member 0 (SURVEY §8 d's
                             // "counter seeded 0"), not rand:uniform(N) (emqx_subtab "rr_seed0")
  uint32_t* entry_topic;     // [m] scratch: entry -> topic
  uint64_t* csum;            // [m_cap / FO_WCHUNK + 2] deliveries per chunk of FO_WCHUNK entries
  uint64_t* gchunk;          // [m_cap / FO_WCHUNK + 2] $share picks per chunk (round_robin / sticky)
  uint64_t* partials;        // [4 * FO_BLOCKS] block sums and bases (deliveries, then picks)
  uint64_t* out_off;         // [n+1]
  uint32_t* out_subs;        // [cap]
  uint32_t* out_filters;     // [cap] or null
  uint64_t cap;              // capacity of out_subs / out_filters
  uint64_t* summary;         // [FO_SUM_WORDS] device or host-mapped
};

// Chunks of the fixed-grid count/scan kernels (the entry count is only known on the device):
// FO_BLOCKS blocks, each a whole number of FO_WCHUNK-entry chunks (the write kernel's unit).
constexpr uint32_t FO_BLOCKS = 1024;
constexpr uint32_t FO_WCHUNK = 256;
// Call summary words: flags, deliveries, match entries, live pick-state keys.
constexpr uint32_t FO_SUM_FLAGS = 0, FO_SUM_TOTAL = 1, FO_SUM_ENTRIES = 2, FO_SUM_STATE = 3, FO_SUM_WORDS = 4;
constexpr uint64_t FO_SUM_F_OVERFLOW = 1;    // more deliveries than cap: offsets only, no ids written
constexpr uint64_t FO_SUM_F_MATCH = 2;       // the match call flagged an error/overflow: nothing read
constexpr uint64_t FO_SUM_F_STATE_FULL = 4;  // a pick found no room in the pick-state table: no pick
                                             // state consumed, $share outputs not final (rerun)
constexpr uint64_t FO_SUM_F_PICKS = 8;       // more round_robin / sticky picks than the pick list
                                             // holds: no ids written (rerun; the list grows)
constexpr uint64_t FO_SUM_F_RERUN = FO_SUM_F_STATE_FULL | FO_SUM_F_PICKS;

constexpr uint64_t FO_SUM_F_SMALL = 16;      // the one-launch small-batch path could not take the
                                             // fan-out (too many entries): run the regular kernels
// Counter-based random pick of EMQX_SHARE_RANDOM: entry i of the call, group record gidx.
__host__ __device__ inline uint32_t fo_rand(uint32_t seed, uint64_t i, uint32_t salt) {
  return mix32(seed ^ mix32(static_cast<uint32_t>(i) * 0x9E3779B1u ^ static_cast<uint32_t>(i >> 32) ^ salt));
}
// Member index of a stateless pick among n >= 2 members (emqx_shared_sub.erl:251-288): the
// caller's phash2 key for hash_clientid / hash_topic (1 + Key rem Count, 1-based there),
// fo_rand for random.  strategy: EMQX_SHARE_* (3, 4 hash; else random).
__host__ __device__ inline uint32_t fo_stateless_index(uint32_t strategy, uint32_t key, uint32_t seed, uint64_t entry,
                                                       uint32_t gidx, uint32_t n) {
  return (strategy == 3u || strategy == 4u) ? key % n : fo_rand(seed, entry, gidx + 0x632BE5ABu) % n;
}

// True for the strategies whose picks depend on state kept per publisher.
__host__ __device__ inline bool fo_stateful(uint32_t strategy) { return strategy == 1u || strategy == 2u; }
// True for the strategies that read the per-topic key.
__host__ __device__ inline bool fo_needs_topic(uint32_t strategy) { return strategy != 0u; }

// The whole fan-out of one batch, enqueued on s; m_cap bounds the match entries.  Stateful
// strategies: launch_fanout enqueues the count / scan / write kernels, the caller orders the
// stream after the subtable's last resolve, then launch_fanout_resolve sorts the pick list and
// makes the picks (sort_temp: fanout_sort_temp_bytes(pk_cap) bytes).
hipError_t launch_fanout(const FanoutArgs& a, uint64_t m_cap, hipStream_t s);
uint64_t fanout_sort_temp_bytes(uint64_t pk_cap);
hipError_t launch_fanout_resolve(const FanoutArgs& a, void* sort_temp, uint64_t sort_temp_bytes, hipStream_t s);

// emqx_shared_sub:dispatch/4's retry after a failed delivery (emqx_shared_sub.erl:118-130):
// pick/6 -> do_pick/6 with FailedSubs, in request order, one wave.
struct RepickArgs {
  const DevRec* recs;
  uint32_t n_recs;
  const GroupRec* groups;
  const uint32_t* members;
  const uint32_t* alive;
  uint32_t n_alive_words;
  uint64_t* ps_keys;
  uint32_t* ps_vals;
  unsigned long long* ps_count;
  uint64_t ps_mask;
  uint32_t strategy;
  uint32_t seed;
  uint32_t rr_first0;            // as FanoutArgs
  uint64_t n;
  const uint32_t* filter_ids;   // [n]
  const uint32_t* group_ids;    // [n]
  const uint32_t* keys;         // [n]
  const uint64_t* failed_off;   // [n + 1]
  const uint32_t* failed;       // [failed_off[n]]
  uint32_t* out_subs;           // [n]
  uint32_t* out_kind;           // [n] EMQX_PICK_*
  unsigned long long* ctl;      // [1]: FO_SUM_F_STATE_FULL when a state entry found no room
};
hipError_t launch_share_repick(const RepickArgs& a, hipStream_t s);

// One device record (a 16-B group record, or a 32-B DevRec as value + ext) / one u32 word
// written into a device table by an incremental commit.
struct RecPatch {
  uint32_t index;
  uint32_t pad[3];
  uint4 value;
  uint4 ext;
};
struct WordPatch {
  uint32_t index_lo, index_hi;  // element index (u64)
  uint32_t value;
  uint32_t pad;
};
// Word patches go to plain[] (the first n_plain_w), members[] (the next n_member_w), then the
// liveness bitmap alive[] (n_alive_w).
hipError_t launch_subtab_patches(uint32_t* plain, uint32_t* members, uint32_t* alive, const WordPatch* wp,
                                 uint64_t n_plain_w, uint64_t n_member_w, uint64_t n_alive_w, GroupRec* groups,
                                 DevRec* recs, uint32_t* fcnt, const RecPatch* rp, uint64_t n_group_p,
                                 uint64_t n_rec_p, hipStream_t s);
// fcnt[i] = fo_cnt_word(recs[i].head) for i < n (a full upload).
hipError_t launch_fcnt_from_recs(const DevRec* recs, uint64_t n, uint32_t* fcnt, hipStream_t s);

// Pick-state table maintenance: rehash into a larger table; drop the keys of the given
// publishers (sorted, unique).
hipError_t launch_ps_rehash(const uint64_t* old_keys, const uint32_t* old_vals, uint64_t old_cap, uint64_t* keys,
                            uint32_t* vals, uint64_t mask, unsigned long long* count, hipStream_t s);
hipError_t launch_ps_forget(uint64_t* keys, uint64_t cap, const uint32_t* pubs, uint64_t n_pubs,
                            unsigned long long* count, unsigned long long* tombs, hipStream_t s);

// Copies a delivery CSR into host-mapped pinned memory (the pinned publish batches): offsets
// always, ids when the call's total (summary) fits cap.
hipError_t launch_fanout_to_host(const uint64_t* d_off, uint64_t n, const uint32_t* d_subs, const uint32_t* d_fil,
                                 const uint64_t* d_summary, uint64_t cap, uint64_t* h_off, uint32_t* h_subs,
                                 uint32_t* h_fil, hipStream_t s);

}  // namespace emqx
