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

namespace emqx {

constexpr uint32_t SUB_NONE = 0xFFFFFFFFu;
constexpr uint32_t FANOUT_SHARED_BIT = 0x80000000u;  // set in out_filters[] for $share picks

// Per filter id (16 B, one load per matched filter).  The plain list and the group list are
// extents of their arenas with room to grow in place (incremental commits, fanout.cpp).
struct FilterRec {
  uint32_t plain_begin;  // first entry in plain[]
  uint32_t n_plain;      // plain (non-shared) subscribers
  uint32_t group_begin;  // first entry in groups[]
  uint32_t n_groups;     // $share groups with >= 1 member
};

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
constexpr uint32_t FO_CTL_TOUCHED = 0;  // state-table entries this call deferred picks to
constexpr uint32_t FO_CTL_FLAGS = 1;    // FO_SUM_F_* bits raised by the write kernel
constexpr uint32_t FO_CTL_WORDS = 2;

struct FanoutArgs {
  const FilterRec* recs;
  uint32_t n_recs;           // filter ids >= n_recs have no subscribers
  const uint32_t* plain;
  const GroupRec* groups;
  const uint32_t* members;
  // pick state (round_robin / sticky)
  uint64_t* ps_keys;         // [ps_mask + 1]
  uint32_t* ps_vals;         // [ps_mask + 1]
  unsigned long long* ps_count;  // live keys (device)
  uint64_t ps_mask;
  unsigned long long* heads; // [ps_mask + 1] per-call chains: stamp << 32 | first output position
  uint32_t stamp;            // this call's stamp (never 0)
  uint32_t* next;            // [cap] chain links, by output position
  uint32_t* touched;         // [ps_mask + 1] state entries with a chain in this call
  unsigned long long* ctl;   // [FO_CTL_WORDS]
  unsigned long long* ps_seen;  // host-mapped: ps_count as of the last finished call (growth check)
  // the match CSR
  const uint64_t* moff;      // match CSR offsets [n+1]
  const uint32_t* mids;      // match CSR filter ids [moff[n] - moff[0]]
  uint64_t n;                // topics
  uint64_t m_cap;            // entries the scratch holds (a larger CSR is refused, not read)
  const uint64_t* msum;      // the match call's summary (device) or null: flags != 0 -> no fan-out
  const uint32_t* keys;      // per topic: phash2 key (hash strategies) / publisher (rr, sticky), or null
  uint32_t strategy;         // EMQX_SHARE_*
  uint32_t seed;             // per-call seed of random picks
  uint32_t* entry_topic;     // [m] scratch (strategies that read per-topic keys)
  uint32_t* ecount;          // [m] scratch
  uint64_t* eoff;            // [m+1] scratch: per-entry output offsets
  uint64_t* partials;        // [2 * FO_BLOCKS] scratch: chunk sums, chunk bases
  uint64_t* out_off;         // [n+1]
  uint32_t* out_subs;        // [cap]
  uint32_t* out_filters;     // [cap] or null
  uint64_t cap;              // capacity of out_subs / out_filters
  uint64_t* summary;         // [FO_SUM_WORDS] device or host-mapped
};

// Chunks of the fixed-grid count/scan kernels (the entry count is only known on the device).
constexpr uint32_t FO_BLOCKS = 1024;
// Call summary words: flags, deliveries, match entries, live pick-state keys.
constexpr uint32_t FO_SUM_FLAGS = 0, FO_SUM_TOTAL = 1, FO_SUM_ENTRIES = 2, FO_SUM_STATE = 3, FO_SUM_WORDS = 4;
constexpr uint64_t FO_SUM_F_OVERFLOW = 1;    // more deliveries than cap: nothing written
constexpr uint64_t FO_SUM_F_MATCH = 2;       // the match call flagged an error/overflow: nothing read
constexpr uint64_t FO_SUM_F_STATE_FULL = 4;  // a pick found no room in the pick-state table

// True for the strategies whose picks depend on state kept per publisher.
__host__ __device__ inline bool fo_stateful(uint32_t strategy) { return strategy == 1u || strategy == 2u; }
// True for the strategies that read the per-topic key.
__host__ __device__ inline bool fo_needs_topic(uint32_t strategy) { return strategy != 0u; }

// The whole fan-out of one batch, enqueued on s; m_cap bounds the match entries.
hipError_t launch_fanout(const FanoutArgs& a, uint64_t m_cap, hipStream_t s);

// One 16-B record / one u32 word written into a device table by an incremental commit.
struct RecPatch {
  uint32_t index;
  uint32_t pad[3];
  uint4 value;
};
struct WordPatch {
  uint32_t index_lo, index_hi;  // element index (u64)
  uint32_t value;
  uint32_t pad;
};
hipError_t launch_subtab_patches(uint32_t* plain, uint32_t* members, const WordPatch* wp, uint64_t n_plain_w,
                                 uint64_t n_member_w, GroupRec* groups, FilterRec* recs, const RecPatch* rp,
                                 uint64_t n_group_p, uint64_t n_rec_p, hipStream_t s);

// Pick-state table maintenance: rehash into a larger table; drop the keys of the given
// publishers (sorted, unique).
hipError_t launch_ps_rehash(const uint64_t* old_keys, const uint32_t* old_vals, uint64_t old_cap, uint64_t* keys,
                            uint32_t* vals, uint64_t mask, unsigned long long* count, hipStream_t s);
hipError_t launch_ps_forget(uint64_t* keys, uint64_t cap, const uint32_t* pubs, uint64_t n_pubs,
                            unsigned long long* count, hipStream_t s);

// Copies a delivery CSR into host-mapped pinned memory (the pinned publish batches): offsets
// always, ids when the call's total (summary) fits cap.
hipError_t launch_fanout_to_host(const uint64_t* d_off, uint64_t n, const uint32_t* d_subs, const uint32_t* d_fil,
                                 const uint64_t* d_summary, uint64_t cap, uint64_t* h_off, uint32_t* h_subs,
                                 uint32_t* h_fil, hipStream_t s);

}  // namespace emqx
