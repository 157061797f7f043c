// Launch interface of the HIP kernels (match_kernels.hip), used by engine.cpp.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.h"

namespace emqx {

// ctrl[] words (zeroed before every call)
enum Ctrl : uint32_t {
  CTRL_DEFERRED = 0,    // number of topics handed to the deep path
  CTRL_NEED_SLAB = 1,   // max entries any tile needed (> slab_cap => rerun)
  CTRL_ERROR = 2,       // error bits (CTRL_ERR_*)
  CTRL_DEEP_FILL = 3,   // entries the deep path emitted
  CTRL_DEEP_EVALS = 4,  // node visits of the deep path
  CTRL_WORDS = 8
};
constexpr uint32_t GROUP_TILES = 256;  // tiles per group sum (two-level output offsets)
constexpr uint32_t CTRL_ERR_TOO_LONG = 1u;   // deferred topic longer than 65535 bytes
constexpr uint32_t CTRL_ERR_TOO_DEEP = 2u;   // deep-path frontier exceeded its stack
constexpr uint32_t CTRL_ERR_DEEP_SLAB = 4u;  // deep-path slab overflow
constexpr uint32_t CTRL_ERR_ORDER_CAP = 8u;  // walk order: the reordered topic bytes exceed their buffer

constexpr int TILE_TOPICS = 64;

// Diagnostic counters (emqx_set_tuning("diag", 1); read with emqx_diag_read).
enum Diag : uint32_t {
  DIAG_STEPS = 0,        // frontier steps (wave iterations)
  DIAG_ITEMS = 1,        // items popped
  DIAG_LIT_PROBES = 2,   // literal lookups started
  DIAG_LIT_HITS = 3,     // literal lookups that found the child
  DIAG_LIT_EXTRA = 4,    // extra slot loads beyond the first (linear probing)
  DIAG_PLUS_PROBES = 5,  // '+' slot loads
  DIAG_PLUS_HITS = 6,
  DIAG_EMITS = 7,        // filter ids emitted
  DIAG_SPILLS = 8,       // stack spills to HBM
  DIAG_TICKS_A = 9,      // wall-clock ticks (100 MHz) in phase A (tokenize + intern), summed over waves
  DIAG_TICKS_B = 10,     // ... in phase B (frontier walk)
  DIAG_WAVES = 11,       // waves (tiles) counted
  DIAG_LEVEL0 = 12,      // items popped at topic level 0..7 (12..19; 19 = level >= 7)
  DIAG_SMALL = 20,       // items whose node array has <= 8 slots (one 128-B line)
  DIAG_WIDE = 21,        // items whose node array is larger
  DIAG_NCOUNT = 22,
  DIAG_WORDS = 32
};        // topics per wave (one per lane during tokenizing)
constexpr uint32_t DEEP_MAX_LEVELS = 65536;

// Call summary written by tile_scan_kernel (u64 words), read by the host after the stream
// drains (sync calls) or by the caller of the async entry point.
enum Summary : uint32_t {
  SUM_FLAGS = 0,      // SUM_F_* bits; 0 = the call's output is complete
  SUM_TOTAL = 1,      // matched filter ids over the batch (= out_offsets[n])
  SUM_EVALS = 2,      // node visits (fast + deep path)
  SUM_MAXSTACK = 3,   // max frontier stack depth of any tile
  SUM_DEFERRED = 4,   // topics handed to the deep path
  SUM_NEED_SLAB = 5,  // max slab entries any tile needed
  SUM_DEEP_FILL = 6,  // deep-path slab entries
  SUM_ERROR = 7,      // CTRL_ERR_* bits
  SUM_WORDS = 8
};
constexpr uint64_t SUM_F_RETRY = 1;     // a scratch area overflowed: rerun with larger buffers
constexpr uint64_t SUM_F_OVERFLOW = 2;  // total > out_cap: out_ids truncated
constexpr uint64_t SUM_F_ERROR = 4;     // a topic the engine cannot match (see SUM_ERROR)

struct MatchArgs {
  TableView tv;
  const uint8_t* tbytes;
  const uint64_t* toffs;
  uint64_t n;
  uint32_t mode;
  uint32_t slab_cap;       // entries per tile
  uint32_t* counts;        // [n]
  uint64_t* slab;          // [ntiles * slab_cap]  (topic_local << 32) | fid
  uint32_t* tile_fill;     // [ntiles]
  uint64_t* tile_defer;    // [ntiles]
  uint32_t* ctrl;          // [CTRL_WORDS]
  uint32_t* deferred;      // [n]
  uint64_t* diag;          // optional [DIAG_WORDS] counters (nullptr = off)
  uint4* timeline;         // optional (diag on): per tile {start lo, start hi, phase-A end, end}
                           // in 100 MHz wall-clock ticks (end / A-end relative to start), CU id
  uint32_t diag_stop;      // diag kernels only: 1 = skip the walk after phase A (counter passes
                           // that split the kernel's misses by phase; the output is then wrong)
  uint2* spill;            // [ntiles * spill_cap] HBM overflow of the per-wave LDS stack
  uint32_t spill_cap;
  // deep path
  uint32_t* deep_wids;     // [deep_waves * DEEP_MAX_LEVELS]
  uint4* deep_stack;       // [deep_waves * deep_stack_cap]
  uint32_t deep_stack_cap;
  uint32_t deep_waves;
  uint64_t* deep_slab;     // [deep_slab_cap]  (deferred_slot << 32) | fid
  uint32_t deep_slab_cap;
  // output assembly
  uint64_t* tile_sum;      // [ntiles] filter ids per tile (fast path + deep path's atomics)
  uint2* tile_stats;       // [ntiles] {node visits, max stack depth}
  uint64_t* group_sum;     // [ngroups] filter ids per GROUP_TILES tiles
  uint2* group_stats;      // [ngroups] {node visits, max stack depth}
  uint32_t ngroups;
  uint32_t* deep_rank;     // [n] per deferred slot: ids placed so far
  uint64_t* out_off;       // [n + 1] CSR offsets (caller's)
  uint32_t* out_ids;       // [out_cap] CSR ids (caller's)
  uint64_t out_cap;
  uint64_t* summary;       // [SUM_WORDS] (device or host-pinned memory)
  // walk order (order_kernels.hip): the batch is walked in prefix-key order
  const uint32_t* perm;    // [n] batch position -> caller's topic index (nullptr: identity);
                           // tbytes/toffs are then the reordered batch and out_off is in the
                           // caller's order, filled by the scan of the counts put back
  uint32_t deal;           // fast kernel: logical tiles dealt to XCDs in contiguous ranges
  uint32_t* corig;         // [n] counts in the caller's order (perm set)
  uint64_t* partials;      // [scan_partials(n)] scan scratch (perm set)
};

// Small batches in ONE launch (the host batcher's and the publish batcher's calls, a few dozen to
// a few hundred topics: DESIGN §3.5).  One block of SMALL_WAVES waves copies the batch from
// pinned host memory into HBM, walks it in SMALL_WAVES tiles of ceil(n / SMALL_WAVES) topics
// (fast_tile, the batched kernel's walk), runs the deep path over deferred topics, scans and
// scatters the CSR, and either streams it into pinned host memory (match) or fans it out
// (stateless $share strategies) straight into the pinned delivery buffers — no copy engine, no
// second launch.  Anything that does not fit is flagged and rerun on the batched path.
constexpr uint32_t SMALL_WAVES = 16;
constexpr uint64_t SMALL_MAX_N = uint64_t(SMALL_WAVES) * TILE_TOPICS;  // 1024 topics
constexpr uint32_t SMALL_FO_MAX_ENTRIES = 16384;                     // match entries the fan-out takes

struct SmallFanout {
  const uint4* recs;        // DevRec per filter id (fanout.h; two uint4: head, ext with inline lists)
  uint32_t n_recs;
  const uint32_t* plain;
  const uint4* groups;      // GroupRec
  const uint32_t* members;
  uint32_t strategy;        // stateless: EMQX_SHARE_RANDOM / HASH_CLIENTID / HASH_TOPIC
  uint32_t seed;
  const uint32_t* h_keys;   // host-mapped per-topic keys, or null
  uint32_t* d_keys;         // their HBM copy (the batched fan-out of a rerun reads it)
  uint4* erec;              // [SMALL_FO_MAX_ENTRIES] scratch: each entry's record
  uint32_t* etop;           // [SMALL_FO_MAX_ENTRIES] scratch: each entry's topic
  const unsigned long long* ps_count;  // pick-state keys (the summary's state word), or null
  uint64_t* h_off;          // host-mapped delivery CSR: offsets [n + 1]
  uint32_t* h_subs;         // [cap]
  uint32_t* h_fil;          // [cap] filter id | FANOUT_SHARED_BIT for $share picks
  uint64_t cap;
  uint64_t* h_sum;          // host-mapped fan-out summary [FO_SUM_WORDS]
};

struct SmallArgs {
  MatchArgs m;              // tbytes / toffs: the HBM copy; out_off / out_ids: the CSR in HBM;
                            // summary: host-mapped; perm / diag off
  const uint8_t* h_tbytes;  // host-mapped batch: bytes [0, nbytes), offsets [n + 1] (from 0)
  const uint64_t* h_toffs;
  uint64_t nbytes;
  uint32_t tt;              // topics per tile: ceil(n / SMALL_WAVES)
  uint32_t slab_tiles;      // tiles the workspace's slab holds (>= the batch's tiles: checked at launch)
  uint32_t has_fanout;
  uint64_t* h_out_off;      // match only: the CSR into host-mapped buffers (null: not copied)
  uint32_t* h_out_ids;
  uint64_t h_cap;
  uint64_t* clk;            // optional (emqx_set_tuning "timeline" >= SMALL_CLK_WORDS / 2 tiles, diag off):
                            // per-phase wall-clock ticks accumulated over launches (SMALL_CLK_*)
  SmallFanout f;
};
// small-batch phase clock words (100 MHz ticks summed over launches; the last word counts them)
enum : uint32_t {
  SMALL_CLK_COPY = 0, SMALL_CLK_WALK, SMALL_CLK_DEEP, SMALL_CLK_SCAN, SMALL_CLK_SCATTER, SMALL_CLK_OUT,
  SMALL_CLK_FO_PASS1, SMALL_CLK_FO_PASS2, SMALL_CLK_LAUNCHES, SMALL_CLK_WORDS = 10
};
hipError_t launch_small_batch(const SmallArgs& a, hipStream_t s);
}  // namespace emqx
struct emqx_engine;
namespace emqx {
// engine.cpp, for the publish batches (fanout.cpp): a small batch's match and stateless fan-out
// as one launch on s.  SMALL_NOT_TAKEN (> 0): the batch does not qualify and nothing was
// enqueued (the caller runs the batched pipeline).
constexpr int SMALL_NOT_TAKEN = 1;
int engine_small_batch(emqx_engine* e, uint32_t mode, const uint8_t* h_tbytes, const uint64_t* h_toffs, uint64_t n,
                       uint64_t nbytes, uint8_t* d_tbytes, uint64_t* d_toffs, uint64_t* d_out_off, uint32_t* d_out_ids,
                       uint64_t cap, uint64_t* h_summary, const SmallFanout& f, hipStream_t s);

// Deep path: waves of match_deep_kernel, slab entries each wave reserves per atomic, and the
// padding value of a reserved entry left unused.
constexpr uint32_t DEEP_WAVES = 512;
constexpr uint32_t DEEP_CHUNK = 256;
constexpr uint64_t DEEP_PAD = ~0ull;

// Fast-kernel variants: K items per lane per step, LDS stack / word-id capacity per wave.
enum FastVariant {
  FAST_K1_S1K = 0,   // 4 waves/block, stack 1024, K=1
  FAST_K2_S1K = 1,   // 4 waves/block, stack 1024, K=2
  FAST_K2_S2K = 2,   // 2 waves/block, stack 2048, K=2 (deep tables)
  FAST_K2_S768 = 3,  // 4 waves/block, stack 768, K=2 (shallow tables, more waves per CU)
  FAST_K4_S2K = 4,   // 2 waves/block, stack 2048, K=4
  FAST_K1_S256 = 5,  // 4 waves/block, stack 256 (+HBM spill), 640 word ids: 32 waves/CU
  FAST_K2_S512 = 6,  // 4 waves/block, stack 512 (+HBM spill), 640 word ids
  FAST_K1_S384 = 7,  // 4 waves/block, stack 384 (+HBM spill), 640 word ids
  FAST_K2_S512W = 8, // 4 waves/block, stack 512 (+HBM spill), 512 word ids: 24 waves/CU
  FAST_K1_S768W = 9, // 4 waves/block, stack 768, 1024 word ids, K=1 (deep tables: 15 waves/CU)
  FAST_K1_S512W = 10,// 4 waves/block, stack 512 (+HBM spill), 1024 word ids, K=1: 18 waves/CU
  FAST_K1_S384R = 11,// FAST_K1_S384 with the root's edge array staged in LDS (an A/B of round 5)
  FAST_K1_S384P = 12,// FAST_K1_S384 as two kernels: phase A, then the walk (an A/B of round 5)
  FAST_K1_S384N = 13,// FAST_K1_S384 with the next word id read after the probe loads return (the
                     // order before round 5's hoist; kept for the A/B harness)
  FAST_K1_S384W7 = 14,// 4 waves/block, stack 384, 448 word ids, K=1: 21.5 KiB per block, compiled for 7 waves/SIMD
  FAST_K1_S384B2 = 15,// FAST_K1_S384 in blocks of 2 waves (finer dispatch at the grid's tail; an A/B)
  FAST_K1_S384B1 = 16,// ... in blocks of one wave (the default for tables up to 12 levels deep)
  FAST_K1_S512WB1 = 17,// FAST_K1_S512W in blocks of one wave
  FAST_NVARIANTS = 18
};

hipError_t launch_match_fast(const MatchArgs& a, FastVariant v, hipStream_t s);
hipError_t launch_match_deep(const MatchArgs& a, hipStream_t s);
// group sums -> per-tile offsets + ids (fast path), the deep path's ids, then out_off[n]
// and the call summary
hipError_t launch_assemble(const MatchArgs& a, hipStream_t s);
// host batches: the CSR of a finished call (device) into pinned host buffers, sized on the device
hipError_t launch_csr_to_host(const uint64_t* d_off, uint64_t n, const uint32_t* d_ids, uint64_t cap,
                               uint64_t* h_off, uint32_t* h_ids, hipStream_t s);
// filter-sharded tables: owner rank of every topic of a device batch
hipError_t launch_shard_owner(const uint8_t* tbytes, const uint64_t* toffs, uint64_t n, uint32_t world,
                              uint32_t levels, uint32_t* owner, hipStream_t s);
hipError_t launch_shard_route(const uint8_t* tbytes, const uint64_t* toffs, uint64_t n, uint32_t world,
                              const ShardSplitE* splits, uint32_t n_splits, uint32_t* req2, hipStream_t s);
// incremental commits (live_trie.cpp): whole-slot rewrites of the committed table, ids first
hipError_t launch_slot_patches(EdgeSlot* edges, uint32_t* fids, const SlotPatch* patches, uint32_t n,
                               hipStream_t s);
// Walk order: prefix keys, radix sort, reordered topic bytes (order_kernels.hip).
struct OrderArgs {
  const uint8_t* tbytes;    // caller's batch
  const uint64_t* toffs;
  uint64_t n;
  uint32_t level_bits;      // key bits per level (first level highest)
  uint32_t sort_bits;       // top key bits the radix sort orders by (1..64)
  uint64_t* keys;           // [n]
  uint64_t* keys_out;       // [n]
  uint32_t* idx;            // [n]
  uint32_t* perm;           // [n] out: batch position -> caller's topic index
  uint32_t* lens;           // [n]
  uint64_t* noffs;          // [n + 1] out: offsets of the reordered batch
  uint64_t* partials;       // [scan_partials(n)]
  uint8_t* obytes;          // [cap_bytes] out: reordered topic bytes
  uint64_t cap_bytes;
  void* temp;               // radix sort scratch
  uint64_t temp_bytes;
  uint32_t* ctrl;           // CTRL_ERR_ORDER_CAP when the bytes exceed cap_bytes
};
uint64_t order_sort_temp_bytes(uint64_t n, uint32_t sort_bits);
hipError_t launch_order(const OrderArgs& o, hipStream_t s);
// after the walk: corig[perm[p]] = counts[p]
hipError_t launch_order_counts(const uint32_t* counts, const uint32_t* perm, uint64_t n, uint32_t* corig,
                               hipStream_t s);
// Batches regrouped by a permutation and their CSR put back (emqx_batch_permute_device,
// emqx_csr_unpermute_device).
uint64_t permute_scratch_bytes(uint64_t n);
hipError_t launch_batch_permute(const uint8_t* tbytes, const uint64_t* toffs, uint64_t n, const uint32_t* perm,
                                uint8_t* obytes, uint64_t* ooffs, void* scratch, hipStream_t s);
hipError_t launch_csr_unpermute(const uint32_t* counts, const uint32_t* ids, uint64_t n, const uint32_t* perm,
                                uint64_t* out_off, uint32_t* out_ids, void* scratch, hipStream_t s);
uint64_t owner_sort_scratch_bytes(uint64_t n, uint32_t world);
hipError_t launch_owner_sort(const uint32_t* owner, uint64_t n, uint32_t world, uint32_t* perm, void* scratch,
                             hipStream_t s);
// counts[n] -> offsets[n+1] (exclusive); partials: scratch of >= scan_partials(n) u64
// (fan-out's entry scan).
uint64_t scan_partials(uint64_t n);
hipError_t launch_scan(const uint32_t* counts, uint64_t n, uint64_t* offsets, uint64_t* partials,
                       hipStream_t s);

}  // namespace emqx
