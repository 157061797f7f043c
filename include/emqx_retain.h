/*
 * emqx_retain.h — C ABI of the retained-message index (libemqxmatch.so), SURVEY §8 f4.
 *
 * The "inverse" lookup of the mnesia retainer backend: a subscription filter -> the stored
 * retained topics it matches.  Paths are relative to the reference checkout
 * (xiongzhenhai-zh/emqx, EMQX 5.0.0-beta.3):
 *
 *   emqx_retainer_mnesia:store_retained/2     apps/emqx_retainer/src/emqx_retainer_mnesia.erl:74-98
 *       -> emqx_retain_store (+ emqx_retain_commit: batched rebuild, snapshot swap)
 *   emqx_retainer_mnesia:delete_message/2     emqx_retainer_mnesia.erl:117-128
 *       -> emqx_retain_lookup + emqx_retain_delete (exact topic); a wildcard topic
 *          (match_delete_messages/1, :217-223) -> emqx_retain_match_batch(now_ms = -1)
 *          + emqx_retain_delete of the returned ids
 *   emqx_retainer_mnesia:clear_expired/1      emqx_retainer_mnesia.erl:106-115
 *       -> emqx_retain_expired + emqx_retain_delete
 *   emqx_retainer:dispatch/4 -> read_message/2 (plain filter, :199-208) or match_messages/3
 *       (wildcard filter, :212-215 + make_match_spec/1 :233-245)
 *       -> emqx_retain_match_batch: one call for a batch of filters (a subscribe storm),
 *          each filter answered as dispatch/4 would (plain: expiry == 0 || expiry >= now;
 *          wildcard: expiry == 0 || expiry > now; no '$' rule — the match spec has none).
 *   emqx_retainer_mnesia:size/1               emqx_retainer_mnesia.erl:164-165
 *       -> emqx_retain_stats(...).n_live
 *
 * Ordering: the reference sorts a wildcard answer by message timestamp (sort_retained/1,
 * qlc:sort in make_cursor/1); the index returns each filter's topic ids as a set (order
 * unspecified) and the caller, who holds the messages, orders them.  Cursor batching
 * (max_read_number) is likewise a caller-side slice of that list.
 *
 * Conventions as in emqx_match.h: int status, EMQX_* codes, packed byte buffers + uint64
 * offsets[n+1], CSR results.  One writer (store/delete/commit) at a time; any number of
 * concurrent emqx_retain_match_batch callers read an immutable snapshot.
 */
#ifndef EMQX_RETAIN_H
#define EMQX_RETAIN_H

#include <stdint.h>

#include "emqx_match.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct emqx_retain emqx_retain;

/* Versioned by size, as emqx_stats: set `size` = sizeof(emqx_retain_stats) before the call. */
typedef struct emqx_retain_stats {
  uint64_t size;             /* in: sizeof(emqx_retain_stats) of the caller; out: bytes written */
  uint64_t n_ids;            /* topic ids ever assigned                                     */
  uint64_t n_live;           /* retained topics stored (emqx_retainer_mnesia:size/1)        */
  uint64_t n_nodes;          /* trie nodes of the committed snapshot                        */
  uint64_t n_words;          /* interned words                                              */
  uint64_t table_bytes;      /* device bytes of the committed snapshot                      */
  uint64_t epoch;            /* commits so far                                              */
  uint64_t last_ranges;      /* rank ranges the last match emitted                          */
  uint64_t last_visits;      /* trie nodes the last match visited                           */
  uint64_t last_total;       /* topic ids the last match returned                           */
  double last_build_ms;      /* host build + upload time of the last commit                 */
  double last_match_ms;      /* device time of the last match call (hipEvent)               */
  double last_walk_ms;       /* ... of its walk (first round and spill rounds)              */
  uint64_t last_spill_rounds; /* walk rounds after the first (work left by waves over budget) */
  uint64_t last_spilled;     /* work items handed to those rounds                           */
  uint64_t last_spill_full;  /* waves whose spill found the buffer full (walked on themselves)  */
  uint64_t last_shares;      /* queue mode: times a busy wave shared work (last_spilled: pieces) */
  uint64_t queue_aborts;     /* queue-mode calls rerun in spill mode (a waiting wave gave up; 0) */
} emqx_retain_stats;

int emqx_retain_create(int32_t device, emqx_retain** out);
int emqx_retain_destroy(emqx_retain* r);

/* Stores n topics (no '+'/'#' level: EMQX_EINVAL, nothing stored).  expiry_ms[i] is the
 * message's expiry time in ms (0 = never; emqx_retainer:get_expiry_time/1); NULL = all 0.
 * Re-storing a topic keeps its id and replaces its expiry.  ids_out (may be NULL) gets ids. */
int emqx_retain_store(emqx_retain* r, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                      const int64_t* expiry_ms, uint32_t* ids_out);
/* Deletes topics by id (unknown / already deleted ids are ignored). */
int emqx_retain_delete(emqx_retain* r, const uint32_t* ids, uint64_t n);
/* Id of a stored (live) topic, EMQX_ENOTFOUND otherwise. */
int emqx_retain_lookup(emqx_retain* r, const uint8_t* bytes, uint64_t len, uint32_t* id_out);
/* Bytes of topic `id` (cap bytes copied); *len_out = its length. */
int emqx_retain_topic(emqx_retain* r, uint32_t id, uint8_t* buf, uint64_t cap, uint64_t* len_out);
/* Ids of live topics whose expiry is nonzero and < now_ms (clear_expired/1); *n_out = count,
 * at most cap written (EMQX_EOVERFLOW if more: *n_out = the count needed). */
int emqx_retain_expired(emqx_retain* r, int64_t now_ms, uint32_t* ids_out, uint64_t cap, uint64_t* n_out);
/* Publishes every store/delete since the last commit (snapshot swap). */
int emqx_retain_commit(emqx_retain* r);

/* dispatch/4 for a batch of filters against the committed snapshot.  now_ms < 0: no expiry
 * guard (match_delete_messages/1).  out_offsets[n+1], out_ids[out_offsets[n]] (topic ids);
 * EMQX_EOVERFLOW when out_cap is too small (*n_out = the capacity needed, offsets valid). */
int emqx_retain_match_batch(emqx_retain* r, const uint8_t* filter_bytes, const uint64_t* filter_offsets,
                            uint64_t n, int64_t now_ms, uint64_t* out_offsets, uint32_t* out_ids,
                            uint64_t out_cap, uint64_t* n_out);
/* match_messages/3 and page_read/4 semantics (emqx_retainer_mnesia.erl:136-158,210-215,233-246):
 * the match spec's strict guard (Et =:= 0 orelse Et > Now) for every filter, plain ones
 * included — where emqx_retain_match_batch follows dispatch/4 (emqx_retainer.erl:119-131):
 * read_message/2's Et >= Now for a plain filter, the match spec for a wildcard one. */
int emqx_retain_match_spec_batch(emqx_retain* r, const uint8_t* filter_bytes, const uint64_t* filter_offsets,
                                 uint64_t n, int64_t now_ms, uint64_t* out_offsets, uint32_t* out_ids,
                                 uint64_t out_cap, uint64_t* n_out);
/* Same, with every buffer in device memory of the index's device, on `stream` (0 = the
 * index's own, ordered after the work already enqueued on the device's null stream).
 * Synchronizes the stream before returning. */
int emqx_retain_match_batch_device(emqx_retain* r, const uint8_t* d_filter_bytes,
                                   const uint64_t* d_filter_offsets, uint64_t n, int64_t now_ms,
                                   uint64_t* d_out_offsets, uint32_t* d_out_ids, uint64_t out_cap,
                                   uint64_t* n_out, void* stream);

/* Walk tuning (experiments and tests; results never depend on it).  Keys: "tile" (filters
 * per wave tile of the first round, 1..64, default 16 with the work-sharing walk, 10 with the
 * spill rounds), "step_budget" (wave steps before a
 * stack spills to the next round, 0 = never, default 24), "spill_budget" (the same for the
 * budgeted spill rounds, 0 = step_budget, default 64), "spill_per_wave" (spilled pieces
 * per wave of a round, default 4), "spill_rounds" (budgeted rounds per call, then one without
 * a budget, default 4, at most 46), "spill_cap" (spill-buffer items a round may use, 64..4M,
 * default 4M; tests), "search" (0: two-level binary searches of the postings and rank lists,
 * 1: 16-ary search trees, default), "walk_waves" (persistent waves of the first round, default
 * 8192), "spill_waves" (waves of a spill round at most, default 4096), "balance" (1: the
 * work-sharing walk, default: waves out of tiles wait on tickets of a queue of shared pieces and
 * busy waves share the bottom of their stacks, no rounds; 0: the spill rounds above),
 * "queue_piece" (nodes per shared piece, 64..1M, default 256), "queue_check" (steps between a
 * busy wave's looks at the waiting count, a power of 2 up to 1024, default 8), "queue_cap"
 * (queue slots a call may use, 64..4M, default 4M; tests), "lane_map" (1: a walk step maps
 * lanes to items by a ballot of the items' first lanes, default; 0: a binary search per lane,
 * the round-5 A/B).  EMQX_RETAIN_TILE / _STEP_BUDGET / _SPILL_BUDGET / _SPILL_PER_WAVE / _SPILL_ROUNDS /
 * _SEARCH / _WALK_WAVES / _SPILL_WAVES / _BALANCE / _QUEUE_PIECE / _QUEUE_CHECK / _LANE_MAP give the initial values at create.  EMQX_ENOTFOUND for unknown keys. */
int emqx_retain_set_tuning(emqx_retain* r, const char* key, int64_t value);
int emqx_retain_stats_get(emqx_retain* r, emqx_retain_stats* out);

#ifdef __cplusplus
}
#endif

#endif /* EMQX_RETAIN_H */
