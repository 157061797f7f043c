// Device layout and launch interface of the publish fan-out stage (fanout_kernels.hip,
// fanout.cpp).  See DESIGN.md §3.2.
//
// Reference: after emqx_router:match_routes/1, emqx_broker:publish/1 aggregates the routes
// (aggre/1, apps/emqx/src/emqx_broker.erl:261-272) and routes each one:
//   {Filter, node()}  -> dispatch/2 -> every local subscriber of Filter, with the {shard, I}
//                        buckets of big filters expanded (emqx_broker.erl:500-524)
//   {Filter, Group}   -> emqx_shared_sub:dispatch/3 -> ONE member of the group, picked by the
//                        configured strategy (apps/emqx/src/emqx_shared_sub.erl:251-288)
// Here both become one flattened CSR of deliveries per published topic.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace emqx {

constexpr uint32_t SUB_NONE = 0xFFFFFFFFu;
constexpr uint32_t FANOUT_SHARED_BIT = 0x80000000u;  // set in out_filters[] for $share picks

// Per filter id (16 B, one load per matched filter).
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
  uint32_t slot;          // persistent state slot (round-robin counter, sticky member)
  uint32_t group_id;      // caller's group id
};

// Mutable pick state per persistent group slot.
struct GroupState {
  uint32_t rr;      // round_robin: picks made so far
  uint32_t sticky;  // sticky: the member subscriber id, SUB_NONE = none yet
};

struct FanoutArgs {
  const FilterRec* recs;
  uint32_t n_recs;           // filter ids >= n_recs have no subscribers
  const uint32_t* plain;
  const GroupRec* groups;
  const uint32_t* members;
  GroupState* state;
  const uint64_t* moff;      // match CSR offsets [n+1]
  const uint32_t* mids;      // match CSR filter ids [moff[n]]
  uint64_t n;                // topics
  const uint32_t* keys;      // per topic pick key (erlang:phash2 of ClientId / topic), or null
  uint32_t strategy;         // EMQX_SHARE_*
  uint32_t seed;             // per-call seed of the 'random' strategy
  uint32_t* entry_topic;     // [m] scratch (hash strategies)
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
// Call summary words.
constexpr uint32_t FO_SUM_FLAGS = 0, FO_SUM_TOTAL = 1, FO_SUM_ENTRIES = 2, FO_SUM_WORDS = 4;
constexpr uint64_t FO_SUM_F_OVERFLOW = 1;

// The whole fan-out of one batch, enqueued on s; m_cap bounds the match entries.
hipError_t launch_fanout(const FanoutArgs& a, uint64_t m_cap, hipStream_t s);

}  // namespace emqx
