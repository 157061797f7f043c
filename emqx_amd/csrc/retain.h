// Device layout and launch interface of the retained-message index (retain_kernels.hip,
// retain.cpp).  See DESIGN.md §3.4.
//
// Reference: the mnesia retainer keeps one record per retained topic, keyed by its token list
// (apps/emqx_retainer/src/emqx_retainer_mnesia.erl:74-98), and answers a wildcard
// subscription with a full-table match-spec select (match_messages/1, :212-215, condition/1
// :225-231).  Here the stored topics form a level trie over interned words (no wildcards in
// it: they are published topics) and a FILTER walks it — the inverse of the route lookup:
//   literal word -> one hashed child lookup;  '+' -> every child (one range item), or, when
//                   a literal follows the '+' run, one slice of that literal's level postings;
//   final '#'    -> the node's whole subtree, which is ONE contiguous range of topic ranks,
//                   because ranks are numbered in depth-first preorder.
// So a walk emits rank ranges, and the output stage copies rank -> topic id for the live
// (unexpired) ranks of each range: coalesced streaming reads, no per-topic pointer chasing.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.h"

namespace emqx {

constexpr uint32_t RNODE_TERM = 0x80000000u;  // RNode.ncld: the node is a stored topic (rank lo)

// One trie node (16 B).  Children are contiguous node ids [cbeg, cbeg + ncld) (BFS order);
// the subtree's stored topics are ranks [lo, hi) (DFS preorder: the node's own topic first).
struct alignas(16) RNode {
  uint32_t cbeg;
  uint32_t ncld;  // | RNODE_TERM
  uint32_t lo;
  uint32_t hi;
};

// Literal-edge lookup: (parent name, wid) -> child name in 64-B buckets of REDGE_BUCKET
// edges, bucket = hash & edge_mask, load <= 3/8 (a bucket overflows ~1 % of the time:
// REDGE_OVF in its first key's word id sends the lookup on to the next bucket).  A node's
// NAME is its postings index (RNAME_ROOT for the root), so a lookup needs no node load first,
// and its hit is a postings index again: the child's fields are posts[child].  A lookup
// reads the bucket's keys and child names (48 B) in one round trip, hit or miss.
constexpr uint32_t REDGE_BUCKET = 4;
constexpr uint32_t REDGE_OVF = 1u << 31;  // on key[0].wid (word ids < 2^31)
constexpr uint32_t RNAME_ROOT = 0xFFFFFFF0u;
struct alignas(64) REdgeBucket {
  uint2 key[REDGE_BUCKET];      // {parent name, wid}; parent WID_NONE = empty
  uint32_t child[REDGE_BUCKET]; // child names
  uint32_t pad[4];
};
EMQX_HD uint32_t redge_slot0(uint32_t parent, uint32_t wid) {
  return mix32(parent * 0x9E3779B1u ^ mix32(wid + 0x7F4A7C15u));
}

// Level postings: every node at depth d reached by word w, sorted by its first rank `lo`
// (same-depth subtrees are disjoint, so `lo` orders them and a subtree of v is the slice with
// lo in [v.lo, v.hi)).  A run of '+' levels followed by a literal w is answered from the
// postings of (depth after the run, w) inside the current node's rank interval — a binary
// search instead of visiting every child (and grandchild) the '+' run spans.
struct alignas(16) RPostKey {
  uint32_t depth;  // WID_NONE = empty slot
  uint32_t wid;
  uint32_t off;    // first entry in posts[]
  uint32_t len;
};
EMQX_HD uint32_t rpost_slot0(uint32_t depth, uint32_t wid) { return mix32(wid * 0x9E3779B1u + depth * 0x85EBCA77u); }

// Sorted-key search tree (S-tree) of one key array: level 0 = the keys, level k = every
// 16^k-th key, each level 64-B aligned.  A lower bound inside a slice [L, H) of level 0 (keys
// sorted within the slice) starts at the lowest level where the slice lies in one 16-key block
// and goes down one level per step, each step one 64-B line read as four 16-B loads issued
// together: ~6 round trips instead of the ~20 dependent loads of a binary search.
constexpr uint32_t RST_MAX = 9;  // levels at most
constexpr uint32_t RST_SH = 4;
constexpr uint32_t RST_FAN = 1u << RST_SH;
struct RSTree {
  const uint32_t* keys;  // all levels; level k has n_k = ceil(n / 16^k) keys and takes
                         // rst_level_words(n_k) words (its start is computed, not stored:
                         // a dynamically indexed offset table costs the walk registers)
  uint32_t n;            // level-0 keys
  uint32_t levels;
};
EMQX_HD uint32_t rst_level_words(uint32_t nk) { return ((nk + RST_FAN - 1) & ~(RST_FAN - 1)) + RST_FAN; }

// Two-level binary searches (RSEARCH_FENCED): every RFENCE-th key of posts[] / dterm[] in a
// small fence array, searched first; the final search stays inside one block.
constexpr uint32_t RFENCE = 32;
enum RSearch : uint32_t { RSEARCH_FENCED = 0, RSEARCH_STREE = 1 };

struct RetainView {
  const REdgeBucket* edges;
  uint32_t edge_mask;         // buckets - 1
  uint32_t root_ncld, root_lo, root_hi;  // the root's RNode fields (the root has no postings entry)
  const VocabSlot* vocab;
  const uint8_t* arena;
  uint32_t vocab_mask;
  const uint32_t* rank_id;    // [n_ranks] topic id of each rank
  const int64_t* rank_exp;    // [n_ranks] expiry (ms, 0 = never)
  const RPostKey* pkeys;      // (depth, wid) -> postings slice
  uint32_t pkey_mask;
  const uint4* posts;         // {lo, node, ncld, hi} per node but the root, grouped by (depth, wid):
                              // the index of a node's entry is its name (REdgeBucket);
                              // a postings visit reads its node's fields from the (coalesced) slice
  const uint32_t* dterm_off;  // [max_depth + 2] per depth: first entry in dterm
  const uint32_t* dterm;      // ranks of the stored topics, grouped by depth (levels), ascending
  const uint16_t* rank_depth; // [n_ranks] levels of each stored topic (capped at 65535)
  RSTree pst;                 // over posts[].x: the postings searches
  RSTree dst;                 // over dterm[]: the per-depth rank-list searches
  const uint32_t* pfence;     // posts[RFENCE * b].x: two-level binary searches (RSEARCH_FENCED)
  const uint32_t* dfence;     // dterm[RFENCE * b]
  uint32_t max_depth;
  uint32_t n_nodes;           // 0: empty table
  uint32_t has_expiring;      // some rank has a nonzero expiry
};


// Work item of the walk (uint4): x = first postings entry (node name), y = count, z = level |
// RITEM_POST (else the item is the root), w = filter lane in the tile (first round) or global
// filter id (spilled items)
constexpr uint32_t RITEM_POST = 1u << 31;
constexpr uint32_t RITEM_LEVEL = RITEM_POST - 1;

// Range emitted by the walk: filter f's matches include ranks [lo, hi), or, RRANGE_INDIRECT,
// the ranks dterm[lo .. hi) (a filter ending in a '+' run: the stored topics of that many
// levels inside a subtree, a contiguous slice of the per-depth rank list).
constexpr uint32_t RRANGE_STRICT = 1;    // expiry guard expiry > now (match spec); else >= now (read)
constexpr uint32_t RRANGE_INDIRECT = 2;
constexpr uint32_t RRANGE_MIND_SHIFT = 8;  // flags >> 8: only ranks of at least this many levels
                                           // (a '+' run then '#': the subtree minus shallow topics)
struct RRange {
  uint32_t f;
  uint32_t lo;
  uint32_t hi;
  uint32_t flags;  // RRANGE_*
};

// ctrl words of one call (zeroed per call).  Words that many waves update or poll sit on 64-B
// lines of their own: same-address (and same-line) traffic from thousands of waves is served
// one request at a time at one memory channel (~25 ns each), so it is spread or kept rare.
enum RCtrl : uint32_t {
  RC_RANGES = 0,    // small range record slots reserved (with RC_BIG may exceed range_cap: rerun)
  RC_BIG = 16,      // big range records, stored from the top of ranges[] down
  RC_TILE = 32,     // first-round tiles taken beyond the first a.waves (queue mode: all tiles)
  RC_STACK = 48,    // a wave's stack overflowed (rerun with a larger stack)
  RC_ROUNDS = 49,   // spill rounds that had work
  RC_SPILLED = 50,  // items those rounds took in
  RC_SPILLFAIL = 51,  // waves whose spill found no room (they finish their stacks themselves)
  RC_SPILLMAX = 52,   // the most pieces one wave's spill asked for
  // per-wave totals, added when a wave ends on line (wave % RC_STAT_LINES) of 16 words:
  // [RC_STAT + 16 l + 0] node visits, [.. + 1] range records written (RC_RANGES counts reserved
  // slots: waves reserve RRES at a time, the unused ones stay zeroed = empty records),
  // [.. + 2] pieces shared, [.. + 3] sharing events (queue mode)
  RC_STAT = 64,
  RC_STAT_LINES = 16,
  RC_QABORT = 320,  // queue mode: a waiting wave gave up (poll limit); the host reruns in spill mode
  RC_SPILL = 384,   // items spilled by the walk (a u64 over words RC_SPILL, RC_SPILL + 1); RC_SPILL +
                    // 2 (k + 1): by spill round k (each round its own u64, all zeroed with the rest at
                    // the call's start; 64-bit so that failed reservations' overshoot cannot wrap)
  RC_WORDS = 480
};
constexpr uint32_t RC_MAX_ROUNDS = (RC_WORDS - RC_SPILL) / 2 - 2;  // budgeted spill rounds per call at most

// Queue mode: the control words of one shard (RetainArgs.qctl + shard * QS_STRIDE; all zero when
// a call starts, zeroed again by the call's last kernel)
enum QCtrl : uint32_t {
  QS_HEAD = 0,   // tickets taken by waves waiting for shared work (slot = ticket)
  QS_TAIL = 1,   // slots reserved by waves sharing work (read with QS_HEAD as one u64)
  QS_TILES = 2,  // tile tickets taken (tile s + shards * ticket)
  QS_DONE = 3,   // the shard's walk is over (set by the wave whose retire ended it; read with
                 // QS_TILES as one u64)
  QS_PEND = 4,   // units held (a tile being walked, or about to be taken) + pieces not yet walked
  QS_FAIL = 5,   // ~(first slot of a reservation past the shard's end), atomicMax; 0: none
};
constexpr uint32_t QS_STRIDE = 1088;  // words between shards' control lines (4352 B)
constexpr uint32_t QS_MAX_SHARDS = 1024;

struct RetainArgs {
  RetainView rv;
  const uint8_t* fbytes;   // filters, packed
  const uint64_t* foffs;   // [n + 1]
  uint64_t n;
  int64_t now_ms;          // < 0: no expiry guard (match_delete_messages)
  uint32_t strict_all;     // RRANGE_STRICT for every filter (match spec calls), else wildcard ones only
  uint32_t* wids;          // [foffs[n] - foffs[0] + n] scratch: word ids, filter f at foffs[f] - foffs[0] + f
  uint4* stack;            // [waves * stack_cap] per-wave work stacks (range items)
  uint32_t stack_cap;
  uint32_t waves;
  uint32_t tile_filters;   // filters per wave tile of the first round (1..64)
  uint32_t search;         // RSearch
  uint64_t* prof;          // RETAIN_PROF builds: per-phase walk cycles (null otherwise)
  uint32_t ablate;         // RETAIN_PROF builds: output-stage ablation bits (EMQX_RETAIN_ABLATE)
  uint32_t step_budget;    // wave steps before the rest of a stack spills (~0u: no budget)
  uint4* spill_out;        // [spill_cap] items left when the budget ran out
  uint32_t spill_cap;
  uint32_t spill_word;     // ctrl word (even: the low half of a u64) counting the items this launch
                           // spills (RC_SPILL + 2 * round)
  uint4* queue;            // [queue_cap] shared work (queue mode), all zero when a call starts;
                           // shard s has slots [s * cap/S, (s + 1) * cap/S)
  uint32_t queue_cap;
  uint32_t* qctl;          // [qshards * QS_STRIDE] the shards' control words
  uint32_t qshards;
  uint32_t qpiece;         // nodes per shared piece (queue mode)
  uint32_t qcheck;         // steps between a busy wave's looks at the waiting count (power of 2)
  uint32_t ownmap;         // 1: a step's lane -> item map from a ballot of item starts (else a binary
                           // search of the prefix per lane; tuning key "lane_map")
  uint32_t qpoll_limit;    // polls before a waiting wave gives up (RC_QABORT; a safety valve)
  uint32_t qmaxwait;       // waves waiting on tickets of one shard at most (more return)
  uint32_t qsleep;         // s_sleep(16) (1024 clocks) per poll of a waiting wave
  uint32_t qroam;          // other shards a wave visits once its own shard's walk is over
  uint32_t ntiles;         // tiles of the call (queue mode's termination count)
  uint64_t wdesc_n;        // entries of wdesc (foffs[n] - foffs[0] + 2n + 1)
  uint4* wdesc;            // [foffs[n] - foffs[0] + 2n] per-level step descriptors of the spill
                           // rounds, filter f's level l at foffs[f] - foffs[0] + 2f + l, levels
                           // 0..nlev: {word, end of the '+' run from l, the word after it
                           // (WID_HASH: none), nlev | wildcard flag << 31}
  RRange* ranges;          // [range_cap]
  uint32_t range_cap;
  uint32_t* ctrl;          // [RC_WORDS]
  uint32_t* rcount;        // [range_cap] live ranks per range
  uint64_t* rlive;         // [5 * range_cap] live-rank masks of checked records (count pass -> write
                           // pass): small record r at [r], big record j = range_cap-1-br at
                           // [range_cap + 4j, +4)
  uint32_t* fcount;        // [n] live matches per filter
  uint32_t* fcursor;       // [n] write cursor per filter
  uint64_t* out_off;       // [n + 1]
  uint32_t* out_ids;       // [out_cap]
  uint64_t out_cap;
};

// tokenize + intern every filter, then walk the trie: ranges[], ctrl
hipError_t launch_retain_walk(const RetainArgs& a, hipStream_t s);
// one rebalanced round over the items a previous round spilled: their count is read on the
// device (ctrl[in_word]), dealt `per_wave` to a wave over at most a.waves waves; an empty
// round exits at once, so a call enqueues its rounds without waiting for the host
hipError_t launch_retain_walk_spill(const RetainArgs& a, const uint4* in, uint32_t in_word, uint32_t per_wave,
                                    hipStream_t s);
// the walk with work sharing instead of spill rounds: waves take tiles, then shared pieces from
// a ticket queue; a busy wave that sees waiting waves shares the bottom half of its stack
// (as qpiece-node pieces); every wave exits when no work is held or queued (ctrl[RC_QPEND])
hipError_t launch_retain_walk_queue(const RetainArgs& a, hipStream_t s);
// live ranks per range -> rcount, fcount (the range count is read on the device)
hipError_t launch_retain_count(const RetainArgs& a, hipStream_t s);
// ids of the live ranks -> out_ids at out_off[f] + cursor; nothing when out_off[n] > out_cap
hipError_t launch_retain_write(const RetainArgs& a, hipStream_t s);

}  // namespace emqx
