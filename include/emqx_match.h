/*
 * emqx_match.h — C ABI of the MI355X-native EMQX route-lookup engine (libemqxmatch.so).
 *
 * This is the drop-in boundary for EMQX's publish-side route lookup.  A thin Erlang NIF
 * (emqx_amd/csrc/nif/emqx_match_nif.c) binds these entry points so
 * that the Erlang call shapes stay unchanged.  Paths are relative to the reference
 * checkout (xiongzhenhai-zh/emqx, EMQX 5.0.0-beta.3):
 *
 *   emqx_trie:insert/1, emqx_trie:delete/1   apps/emqx/src/emqx_trie.erl:106-137
 *       -> emqx_insert_filters / emqx_delete_filters (+ emqx_commit: batched rebuild,
 *          epoch swap; the reference applies each mutation in a mria transaction,
 *          apps/emqx/src/emqx_router_utils.erl:33-70,97-125)
 *   emqx_trie:match/1                        apps/emqx/src/emqx_trie.erl:139-162
 *       -> emqx_match_batch(mode = EMQX_MODE_TRIE)
 *   emqx_router:match_trie/1 (private)       apps/emqx/src/emqx_router.erl:136-140
 *       -> emqx_match_batch(mode = EMQX_MODE_TRIE_WILDCARD)
 *   emqx_router:match_routes/1               apps/emqx/src/emqx_router.erl:127-133
 *       -> emqx_match_batch(mode = EMQX_MODE_ROUTES): filter ids whose routes the
 *          reference returns; the NIF maps ids to the #route{} records it keeps.
 *   emqx_trie:empty/0                        apps/emqx/src/emqx_trie.erl:164-171
 *       -> emqx_stats(...).n_filters == 0
 *   emqx_topic:match/2                       apps/emqx/src/emqx_topic.erl:65-87
 *       -> emqx_topic_match (CPU; per-pair callers such as authz stay on the CPU)
 *
 * Conventions: plain C, no exceptions cross the ABI, every entry point returns an int
 * status (EMQX_OK = 0, negative = error) unless documented otherwise.  Topic/filter
 * batches are packed byte buffers plus uint64 offsets[n+1] (item i = bytes[offsets[i] ..
 * offsets[i+1])).  Match results are CSR: out_offsets[n+1] and out_ids[out_offsets[n]].
 *
 * Threading: any number of threads may call emqx_match_batch* concurrently; each call
 * reads the committed table.  Mutations (insert/delete/commit) must come from one writer at a
 * time (the reference serialises route mutations per topic through router_pool,
 * apps/emqx/src/emqx_router.erl:184-188); see emqx_commit for what a concurrent match sees.
 *
 * Ownership: the caller owns every buffer it passes for the duration of the call; the
 * engine owns device tables, staging and workspaces, all released by
 * emqx_engine_destroy.
 */
#ifndef EMQX_MATCH_H
#define EMQX_MATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes -------------------------------------------------------------- */
#define EMQX_OK 0
#define EMQX_EINVAL -1        /* bad argument (null handle, bad mode, bad offsets)          */
#define EMQX_ENOMEM -2        /* host or device allocation failed                            */
#define EMQX_EDEVICE -3       /* HIP runtime / kernel error (no device, launch failure)      */
#define EMQX_EOVERFLOW -4     /* out_ids too small: *n_out holds the required capacity       */
#define EMQX_ENOTFOUND -5     /* unknown filter id / name                                     */
#define EMQX_ETOODEEP -6      /* a topic exceeded the engine's frontier capacity             */
#define EMQX_EBUSY -7         /* *_try_submit: every batch buffer is busy; nothing was queued */

/* ---- match modes --------------------------------------------------------------- */
#define EMQX_MODE_ROUTES 0          /* emqx_router:match_routes/1 — exact ∪ wildcard    */
#define EMQX_MODE_TRIE 1            /* emqx_trie:match/1, trie holding every inserted
                                       filter (emqx_trie_SUITE usage)                  */
#define EMQX_MODE_TRIE_WILDCARD 2   /* emqx_router:match_trie/1 — wildcard filters only */

typedef struct emqx_engine emqx_engine; /* opaque */

typedef struct emqx_engine_opts {
  int32_t device;        /* HIP device ordinal (-1: current device)                        */
  uint32_t flags;        /* reserved, must be 0                                             */
} emqx_engine_opts;

/* Versioned by size: the caller sets `size` to sizeof(emqx_stats) as it was compiled; the
 * engine writes at most that many bytes (fields are only ever appended) and sets `size` to
 * the bytes it wrote, so a caller built against an older, shorter struct stays safe. */
typedef struct emqx_stats {
  uint64_t size;             /* in: sizeof(emqx_stats) of the caller; out: bytes written      */
  uint64_t n_filters;        /* live filters                                                 */
  uint64_t n_ids;            /* ids ever assigned (ids are never reused)                    */
  uint64_t n_nodes;          /* level-trie nodes in the committed snapshot (root included)  */
  uint64_t n_slots;          /* edge-array slots                                             */
  uint64_t n_words;          /* interned literal words                                       */
  uint64_t table_bytes;      /* device bytes held by the committed snapshot                  */
  uint64_t epoch;            /* number of commits                                            */
  uint64_t last_evals;       /* node visits (SURVEY §8 d) of the last match call             */
  uint64_t last_deferred;    /* topics that took the deep-topic path in the last call        */
  uint64_t last_max_stack;   /* deepest per-wave work stack of the last call (items)         */
  double last_build_ms;      /* host build time of the last commit                           */
  double last_match_ms;      /* device time of the last match call (hipEvent)                */
  double last_kernel_ms;     /* device time of its fused match kernel alone (hipEvent)       */
  uint64_t delta_filters;    /* filters placed by incremental commits since the last full build */
  uint64_t last_commit_kind; /* 0 = full rebuild, 1 = incremental (patched in place)          */
  uint64_t max_depth;        /* levels of the deepest filter in the committed snapshot       */
  uint64_t last_ordered;     /* 1 if the last synchronous match call walked its batch in
                              * prefix-key order (emqx_set_tuning "order"; the CSR is in the
                              * caller's order either way)                                   */
  double last_order_ms;      /* device time of that call's reordering (keys, sort, gather)   */
} emqx_stats;

/* Lifecycle. */
int emqx_engine_create(const emqx_engine_opts* opts, emqx_engine** out);
int emqx_engine_destroy(emqx_engine* e);

/* Mutations (applied to the device snapshot by emqx_commit).
 * insert: ids_out[i] = id of filter i; an already-live filter keeps its id (emqx_trie:insert/2
 *         is idempotent, emqx_trie.erl:115-120); a deleted filter re-inserted gets its old id. */
int emqx_insert_filters(emqx_engine* e, const uint8_t* bytes, const uint64_t* offsets,
                        uint64_t n, uint32_t* ids_out);
/* As emqx_insert_filters, but matches report ext_ids[i] for filter i instead of the engine's
 * own id (filter-sharded tables report global ids; a NIF may report its route-table keys).
 * Deletion and lookup keep using the engine's ids (ids_out). */
int emqx_insert_filters_ext(emqx_engine* e, const uint8_t* bytes, const uint64_t* offsets,
                            uint64_t n, const uint32_t* ext_ids, uint32_t* ids_out);
int emqx_delete_filters(emqx_engine* e, const uint32_t* ids, uint64_t n);
int emqx_lookup_filter(emqx_engine* e, const uint8_t* bytes, uint64_t len, uint32_t* id_out);
/* Copies the bytes of filter `id` into buf (cap bytes); *len_out = its length. */
int emqx_filter_name(emqx_engine* e, uint32_t id, uint8_t* buf, uint64_t cap, uint64_t* len_out);
/* Publishes every insert/delete since the last commit.  Incremental by default, at a cost
 * proportional to the changes: a deleted / re-inserted filter flips a flag of its slot, a new
 * filter's missing tail is added to the committed table in place (new nodes in a spare region,
 * whole-slot rewrites of existing slots); a match call that overlaps the commit sees each
 * changed filter present or absent, as concurrent ETS readers see a mria commit.  A full
 * rebuild (fresh tables, epoch swap: in-flight matches keep the old tables) runs when the
 * spare region is used up (emqx_set_tuning "delta_max": at most that many filters placed
 * incrementally; "incremental" = 0 forces full rebuilds). */
int emqx_commit(emqx_engine* e);
/* Details of the last commit: out[0..11] = kind (0 full, 1 incremental), node relocations,
 * edges placed in place, slots rewritten in place, new slots, spare-region cursor, spare-region
 * capacity (slots), slots of superseded arrays, host microseconds of the last incremental
 * commit's table patching, its new-slot extents, its new vocab slots, microseconds of its
 * uploads and device patches.  n < 12 returns the first n. */
int emqx_commit_stats(emqx_engine* e, uint64_t* out, uint32_t n);

/* Batched match, host buffers (any host memory).  out_offsets has n+1 entries.  On
 * EMQX_EOVERFLOW *n_out is the capacity required and out_ids holds no complete result.
 * Internally the batch is cut into chunks that flow through two pinned host batches, so the
 * copies into and out of pinned memory overlap the device work of the other chunk. */
int emqx_match_batch(emqx_engine* e, uint32_t mode, const uint8_t* topic_bytes,
                     const uint64_t* topic_offsets, uint64_t n, uint64_t* out_offsets,
                     uint32_t* out_ids, uint64_t cap, uint64_t* n_out);

/* Batched match, DEVICE buffers already resident in HBM (d_* pointers), ordered on the
 * given hipStream_t (NULL: the engine's own stream, which first waits for the work already
 * enqueued on the device's null stream, where such a caller produced its inputs; the same
 * holds for every device entry point below that takes NULL).  Same contract as above, except that on
 * EMQX_EOVERFLOW d_out_offsets are complete and d_out_ids holds the first cap ids; *n_out is
 * a host pointer.  Returns after the results are complete on `stream`. */
int emqx_match_batch_device(emqx_engine* e, uint32_t mode, const uint8_t* d_topic_bytes,
                            const uint64_t* d_topic_offsets, uint64_t n,
                            uint64_t* d_out_offsets, uint32_t* d_out_ids, uint64_t cap,
                            uint64_t* n_out, void* stream);

/* Asynchronous emqx_match_batch_device for pipelined callers (a batcher double-buffering
 * device batches): enqueues the call on `stream` and returns at once.  `summary` (>= 8
 * uint64_t, device or host-pinned memory) receives, when the stream reaches it:
 *   [0] flags: 0 = complete; 1 = a scratch area overflowed (redo the batch with
 *       emqx_match_batch_device, which grows it once for the engine); 2 = more than cap ids
 *       (d_out_offsets complete, d_out_ids truncated); 4 = a topic over 65535 bytes;
 *   [1] total ids; [2] trie node visits; [3] max frontier depth; [4] deep-path topics.
 * The table snapshot the call reads stays alive until the call has drained. */
int emqx_match_batch_device_async(emqx_engine* e, uint32_t mode, const uint8_t* d_topic_bytes,
                                  const uint64_t* d_topic_offsets, uint64_t n,
                                  uint64_t* d_out_offsets, uint32_t* d_out_ids, uint64_t cap,
                                  uint64_t* summary, void* stream);

int emqx_stats_get(emqx_engine* e, emqx_stats* out);

/* ---- pinned host batches (the NIF's batch buffers) --------------------------------
 * A host batch owns pinned (page-locked, device-mapped) input and output buffers and its own
 * stream.  The caller packs topics straight into topic_bytes / topic_offsets (offsets[0] = 0,
 * n topics), submits, and reads the CSR from out_offsets / out_ids after wait — no pageable
 * copy anywhere: the inputs go to HBM by DMA, the match runs, and one kernel streams the
 * finished CSR into the pinned outputs.  Several batches may be in flight at once (the
 * batcher keeps two).  wait(): EMQX_OK, EMQX_EOVERFLOW (n_out = ids needed: reserve and
 * submit again) or an error. */
typedef struct emqx_host_batch {
  uint8_t* topic_bytes;     /* pinned, cap_bytes                                             */
  uint64_t* topic_offsets;  /* pinned, cap_topics + 1                                       */
  uint64_t cap_topics, cap_bytes;
  uint64_t n;               /* topics packed (set by the caller)                             */
  uint64_t* out_offsets;    /* pinned, cap_topics + 1 (valid after wait)                     */
  uint32_t* out_ids;        /* pinned, cap_ids                                               */
  uint64_t cap_ids;
  uint64_t n_out;           /* ids of the last call (after wait)                             */
  void* priv;
} emqx_host_batch;
int emqx_host_batch_create(emqx_engine* e, uint64_t cap_topics, uint64_t cap_bytes, uint64_t cap_ids,
                           emqx_host_batch** out);
int emqx_host_batch_destroy(emqx_host_batch* b);
/* Grows the buffers (contents of the inputs kept); not while a call is in flight. */
int emqx_host_batch_reserve(emqx_host_batch* b, uint64_t cap_topics, uint64_t cap_bytes, uint64_t cap_ids);
int emqx_host_batch_submit(emqx_host_batch* b, uint32_t mode);
int emqx_host_batch_wait(emqx_host_batch* b);
/* 1 when the batch's call has completed (wait will not block), 0 while in flight. */
int emqx_host_batch_query(emqx_host_batch* b);

/* Cross-caller batcher: coalesces concurrent single-topic matches (emqx_router:match_routes/1
 * is called once per PUBLISH from each publisher process, apps/emqx/src/emqx_broker.erl:213)
 * into one device batch.  submit() returns at once; a worker thread runs a batch when
 * max_batch topics are queued or max_wait_us after the oldest submission, then calls
 * cb(ctx, status, ids, n) once per submission from that thread (ids valid during the call).
 * destroy() drains pending submissions.  The NIF's cb enif_send()s the ids to the caller.
 * submit() blocks while every pinned buffer is filling, sealed or in flight (backpressure);
 * try_submit() never waits: it returns EMQX_EBUSY instead (nothing queued, cb not called), and
 * likewise when the topic would need a larger pinned buffer.  A NIF on a normal scheduler uses
 * try_submit and moves to a dirty scheduler only on EMQX_EBUSY. */
typedef struct emqx_batcher emqx_batcher;
typedef void (*emqx_batch_cb)(void* ctx, int status, const uint32_t* ids, uint64_t n);
int emqx_batcher_create(emqx_engine* e, uint32_t mode, uint32_t max_batch, uint32_t max_wait_us,
                        emqx_batch_cb cb, emqx_batcher** out);
int emqx_batcher_submit(emqx_batcher* b, const uint8_t* topic, uint64_t len, void* ctx);
int emqx_batcher_try_submit(emqx_batcher* b, const uint8_t* topic, uint64_t len, void* ctx);
/* n submissions at once (topic i = bytes[offsets[i] .. offsets[i+1]), context ctxs[i]): one
 * lock for the lot, e.g. a NIF draining a scheduler's queue of match_routes/1 calls. */
int emqx_batcher_submit_many(emqx_batcher* b, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                             void* const* ctxs);
int emqx_batcher_destroy(emqx_batcher* b);
int emqx_batcher_stats(emqx_batcher* b, uint64_t* n_batches, uint64_t* n_topics);
/* out[0..5] = batches, topics, most batches in flight at once, ns the completer spent waiting
 * for the device, ns it spent in callbacks, ns the dispatcher spent submitting. */
int emqx_batcher_stats_ext(emqx_batcher* b, uint64_t* out, uint32_t n);

/* ---- publish fan-out ------------------------------------------------------------
 * A subscription table maps the filter ids reported by a match (engine ids, or the ext ids of
 * emqx_insert_filters_ext) to subscribers.  It replaces the broker's ETS tables
 *   ?SUBSCRIBER  Topic -> SubPid | {shard, I}      apps/emqx/src/emqx_broker.erl:96-108,146-158
 *   emqx_shared_subscription {Group, Topic, SubPid} apps/emqx/src/emqx_shared_sub.erl:78-91,300-314
 * and the dispatch that follows match_routes/1 in emqx_broker:publish/1:
 *   route/2 + aggre/1 + do_dispatch/2,3            apps/emqx/src/emqx_broker.erl:244-272,500-524
 *   emqx_shared_sub:dispatch/3, pick/6, do_pick/6  apps/emqx/src/emqx_shared_sub.erl:113-126,251-288
 * Subscriber ids and group ids are the caller's uint32 handles (the NIF maps pids and group
 * names to them).  Filter ids must be < 2^30.  A delivery is (subscriber id, filter id); the
 * filter id has EMQX_FANOUT_SHARED_BIT set when the delivery is a $share pick ({share, To, ...}
 * in publish_result(), emqx_types.erl:201-206), and also EMQX_FANOUT_RETRY_BIT when do_pick/6
 * made it as {retry, Sub} (the message then goes out without an ack request,
 * emqx_shared_sub.erl:152-155,251-263; only a sticky re-pick whose dead subscriber is the
 * group's only member does this in a fan-out).
 *
 * Per-message keys (pick_keys / d_pick_keys / emqx_pub_batch.keys), by strategy:
 *   hash_clientid / hash_topic: the caller's erlang:phash2(ClientId) / phash2(Topic) (required);
 *   round_robin / sticky: the PUBLISHER of the message (a collision-free uint32 handle of the
 *     dispatching process): the reference keeps this state in the publishing
 *     process's dictionary under {shared_sub_round_robin | shared_sub_sticky, Group, Topic}
 *     (emqx_shared_sub.erl:234-247,279-285), so the device keeps it per (group slot, publisher).
 *     NULL = one publisher.  Picks of one publisher in one call are made in message order, and
 *     the state updates of concurrent calls are made one call after the other, in the order
 *     the calls were made (a publisher that waits for each publish, as emqx_broker:publish/1
 *     does, sees its messages picked in order);
 *   random: ignored. */
#define EMQX_NO_GROUP 0xFFFFFFFFu
#define EMQX_FANOUT_SHARED_BIT 0x80000000u
#define EMQX_FANOUT_RETRY_BIT 0x40000000u

/* broker.shared_subscription_strategy (emqx_shared_sub.erl:60-65) */
#define EMQX_SHARE_RANDOM 0          /* rand:uniform(N)                                         */
#define EMQX_SHARE_ROUND_ROBIN 1     /* per publisher: rand:uniform(N) - 1 first, then +1 rem N  */
#define EMQX_SHARE_STICKY 2          /* per publisher: first pick random, kept while alive       */
#define EMQX_SHARE_HASH_CLIENTID 3   /* 1 + Key rem N, Key = erlang:phash2(ClientId)             */
#define EMQX_SHARE_HASH_TOPIC 4      /* 1 + Key rem N, Key = erlang:phash2(Topic)                */

typedef struct emqx_subtab emqx_subtab; /* opaque */

int emqx_subtab_create(int32_t device, emqx_subtab** out);
/* Destroy the table's emqx_pub_batch / emqx_pub_batcher objects first. */
int emqx_subtab_destroy(emqx_subtab* s);
/* emqx_broker:subscribe/3 (emqx_broker.erl:124-163): subscriber sub_ids[i] subscribes to
 * filter_ids[i], plainly (group_ids NULL or EMQX_NO_GROUP) or in $share group group_ids[i].
 * Idempotent: re-subscribing keeps the member's place in its group (ETS bag semantics). */
int emqx_subtab_add(emqx_subtab* s, const uint32_t* filter_ids, const uint32_t* sub_ids,
                    const uint32_t* group_ids, uint64_t n);
/* emqx_broker:unsubscribe/1 (emqx_broker.erl:169-195); absent pairs are ignored. */
int emqx_subtab_remove(emqx_subtab* s, const uint32_t* filter_ids, const uint32_t* sub_ids,
                       const uint32_t* group_ids, uint64_t n);
/* Liveness of subscriber processes (erlang:is_process_alive/1 and the ?ALIVE_SUBS table of
 * remote pids, emqx_shared_sub.erl:365-393): alive = 0 when a subscriber's process went down
 * (the channel-down hook, before its subscriptions are cleaned up, as cleanup_down/1 does);
 * emqx_subtab_add marks its subscribers alive.  sticky keeps its stored subscriber while it is
 * alive, whether or not it is still a member (pick/6, :234-240), and re-picks among the other
 * members once it is not.  Published by the next commit. */
int emqx_subtab_set_alive(emqx_subtab* s, const uint32_t* sub_ids, uint64_t n, int alive);
/* Publishes the mutations to the device at a cost proportional to them: the touched list
 * words and 16-B records are patched in place (a list that outgrows its extent moves to the
 * arena's end with room to grow); a full rebuild compacts the arenas only when moved-away
 * extents outweigh the live ones.  Ordered after the fan-outs in flight and before later
 * ones (device events): the call returns once the changes are enqueued (the previous commit's
 * device half is waited for first), and every fan-out / publish / re-pick called after it sees
 * them.  A device error of a commit's device half is returned by the next commit, or by
 * emqx_subtab_commit_wait. */
int emqx_subtab_commit(emqx_subtab* s);
/* Waits for the last commit's device half and returns its status.  On a device error the
 * tables are rebuilt from the host image at once (a full commit) and the error is returned, so
 * it reaches the callers of the failed commit (the commit coalescer calls this before it runs a
 * batch's callbacks). */
int emqx_subtab_commit_wait(emqx_subtab* s);
/* Fault injection for tests: "inject_drain_error" = the next `value` waits for a commit's
 * device half report EMQX_EDEVICE; "inject_bad_alloc" = the next `value` full commits fail
 * their host allocations (the call returns EMQX_ENOMEM).  "rr_seed0" = 1: round_robin's first pick
 * of a (group, publisher) state entry is the first member instead of rand:uniform(N) (SURVEY §8 d's
 * config E: "round_robin with counter seeded 0"; deterministic, so checked pick by pick).
 * EMQX_ENOTFOUND for unknown keys. */
int emqx_subtab_set_tuning(emqx_subtab* s, const char* key, int64_t value);
/* counts[0..3] = live plain subscriptions, live shared memberships, groups with members,
 * device bytes */
int emqx_subtab_stats(emqx_subtab* s, uint64_t* counts4);
/* out[0..8] = last commit kind (0 full, 1 incremental), commits, full commits, words written,
 * 16-B records written, extents moved, garbage words, host us of the last incremental commit's
 * image update, us of the last commit in total. */
int emqx_subtab_commit_stats(emqx_subtab* s, uint64_t* out, uint32_t n);
/* Drops the round_robin / sticky state of the given publishers (their processes ended: the
 * reference's state dies with the process dictionary).  Queued on the host and applied on the
 * device before the table's next stateful fan-out or re-pick (one pass for many publishers). */
int emqx_subtab_forget_publishers(emqx_subtab* s, const uint32_t* publishers, uint64_t n);

/* emqx_shared_sub:dispatch/4's retry after a failed delivery (shared_dispatch_ack_enabled:
 * a nack, a timeout or the subscriber going down, emqx_shared_sub.erl:118-130,165-189): request i
 * picks again for (filter_ids[i], group_ids[i]) with FailedSubs = failed_subs[failed_offsets[i]
 * .. failed_offsets[i+1]) (host buffers), as pick/6 -> do_pick/6 do (:234-263): Subs = All --
 * FailedSubs in member order; none left -> {retry, pick over All}; one -> it (the strategy is
 * not consulted); else the strategy over Subs (round_robin: (Last + 1) rem length(Subs), the
 * publisher's state advanced again; hash: 1 + Key rem length(Subs); random).  sticky keeps
 * its stored subscriber while it is alive and not failed, else re-picks at random among All
 * -- [Sub0 | FailedSubs] and stores the pick.  keys[i]: as the fan-out's per-message key (the
 * publisher for round_robin / sticky, phash2 for the hash strategies).  out_subs[i] = the pick,
 * out_kind[i] = EMQX_PICK_FRESH / EMQX_PICK_RETRY, or EMQX_PICK_NONE when the group has no
 * member ({error, no_subscribers}).  Requests are made in order, after the fan-outs already
 * enqueued on the table; the call returns when they are done. */
#define EMQX_PICK_NONE 0
#define EMQX_PICK_FRESH 1
#define EMQX_PICK_RETRY 2
int emqx_share_repick(emqx_subtab* s, uint32_t strategy, uint64_t n, const uint32_t* filter_ids,
                      const uint32_t* group_ids, const uint32_t* keys, const uint64_t* failed_offsets,
                      const uint32_t* failed_subs, uint32_t* out_subs, uint32_t* out_kind);

/* Fan-out of a match CSR already in HBM (d_match_offsets[n+1], d_match_ids): per-topic CSR of
 * deliveries d_out_offsets[n+1], d_out_subs[], d_out_filters[] (optional, may be NULL).
 * d_pick_keys[n] (device): per-message keys as above.  On EMQX_EOVERFLOW d_out_offsets are
 * complete, nothing is written to the id arrays, no pick state is consumed, and *n_out is the
 * capacity required. */
int emqx_fanout_batch_device(emqx_subtab* s, uint32_t strategy, const uint64_t* d_match_offsets,
                             const uint32_t* d_match_ids, uint64_t n, const uint32_t* d_pick_keys,
                             uint64_t* d_out_offsets, uint32_t* d_out_subs, uint32_t* d_out_filters,
                             uint64_t cap, uint64_t* n_out, void* stream);
/* Asynchronous form of emqx_fanout_batch_device for pipelined callers: the whole fan-out is
 * enqueued on `stream` with no host synchronisation (the entry count is read on the device).
 * match_cap bounds the match entries (the match call's id capacity; sizes the scratch): a CSR
 * with more entries (a match call that overflowed its ids) is not read.  summary[4] (device or
 * host-mapped memory) receives {flags, deliveries, match entries, live pick-state keys} when the
 * call completes; flags bit 0: more deliveries than cap (offsets complete, nothing written to
 * the id arrays, no $share pick state consumed); bit 1: the CSR was refused (nothing read); bit 2: a
 * round_robin / sticky pick found no room for its state, bit 3: more round_robin / sticky picks
 * than the table's pick scratch holds: in both cases no pick state was consumed and the $share
 * deliveries are not final: redo the batch with emqx_fanout_batch_device, which grows the
 * state table / the scratch (once) and reruns. */
int emqx_fanout_batch_device_async(emqx_subtab* s, uint32_t strategy, const uint64_t* d_match_offsets,
                                   const uint32_t* d_match_ids, uint64_t n, uint64_t match_cap,
                                   const uint32_t* d_pick_keys, uint64_t* d_out_offsets, uint32_t* d_out_subs,
                                   uint32_t* d_out_filters, uint64_t cap, uint64_t* summary, void* stream);
/* emqx_broker:publish/1's lookup + fan-out for a batch of topics (host buffers): match
 * (mode EMQX_MODE_ROUTES) and fan-out run back to back on the device; the match CSR never
 * leaves HBM.  pick_keys[n] (host) as above.  Runs through a pinned publish batch of the
 * table's pool (no pageable staging, one host synchronisation).  On EMQX_EOVERFLOW out_offsets
 * are complete, *n_out is the capacity required and no pick state was consumed. */
int emqx_publish_batch(emqx_engine* e, emqx_subtab* s, uint32_t strategy, const uint8_t* topic_bytes,
                       const uint64_t* topic_offsets, uint64_t n, const uint32_t* pick_keys,
                       uint64_t* out_offsets, uint32_t* out_subs, uint32_t* out_filters, uint64_t cap,
                       uint64_t* n_out);

/* ---- commit coalescer -------------------------------------------------------------
 * The per-call boundary for route and subscription changes.  The reference applies each one on
 * its own: emqx_broker:subscribe/3 / unsubscribe/1 write ?SUBSCRIBER per call
 * (emqx_broker.erl:124-195), emqx_shared_sub's handlers per call (emqx_shared_sub.erl:308-322),
 * a topic's first / last subscriber adds / deletes its route in one mria transaction
 * (emqx_router.erl:111-124 -> emqx_router_utils.erl:97-125).  Through a coalescer, a change is
 * applied to the host store when the call returns (insert_filters writes ids_out), and
 * cb(ctx, status) runs from the coalescer's thread once the commit that carries it has reached
 * the device (ctx NULL: no callback).  The thread commits whenever changes are pending and it is
 * idle — the changes that arrive during one commit make the next one — waiting max_wait_us
 * after the first pending change when max_wait_us > 0.  Route changes commit before
 * subscription changes in each round.  flush() returns when everything submitted before it is
 * committed (the last commit's status); destroy() commits and notifies what is pending.
 * stats out[0..5]: commits, changes, most changes in one commit, us spent committing, engine
 * commits, subscription-table commits.  e or s may be NULL (then its calls return EINVAL). */
typedef struct emqx_coalescer emqx_coalescer;
typedef void (*emqx_done_cb)(void* ctx, int status);
int emqx_coalescer_create(emqx_engine* e, emqx_subtab* s, uint32_t max_wait_us, emqx_done_cb cb,
                          emqx_coalescer** out);
int emqx_coalescer_insert_filters(emqx_coalescer* c, const uint8_t* bytes, const uint64_t* offsets, uint64_t n,
                                  uint32_t* ids_out, void* ctx);
int emqx_coalescer_delete_filters(emqx_coalescer* c, const uint32_t* ids, uint64_t n, void* ctx);
int emqx_coalescer_subscribe(emqx_coalescer* c, const uint32_t* filter_ids, const uint32_t* sub_ids,
                             const uint32_t* group_ids, uint64_t n, int add, void* ctx);
/* n changes of n callers under one lock (a NIF draining a scheduler's queue of SUBSCRIBEs):
 * change i subscribes (adds[i] != 0) or unsubscribes, and ctxs[i] (or NULL) is called back. */
int emqx_coalescer_subscribe_many(emqx_coalescer* c, const uint32_t* filter_ids, const uint32_t* sub_ids,
                                  const uint32_t* group_ids, const uint8_t* adds, uint64_t n, void* const* ctxs);
int emqx_coalescer_set_alive(emqx_coalescer* c, const uint32_t* sub_ids, uint64_t n, int alive, void* ctx);
int emqx_coalescer_flush(emqx_coalescer* c);
int emqx_coalescer_destroy(emqx_coalescer* c);
int emqx_coalescer_stats(emqx_coalescer* c, uint64_t* out, uint32_t n);

/* ---- pinned publish batches (the NIF's publish buffers) ---------------------------
 * The publish counterpart of emqx_host_batch: pinned inputs (topics, per-message keys) and
 * pinned outputs (the delivery CSR).  submit() enqueues, on the batch's own stream with no host
 * synchronisation: inputs to HBM, the match (EMQX_MODE_ROUTES), the fan-out of its CSR in HBM,
 * and the delivery CSR streamed into the pinned outputs.  wait(): EMQX_OK, EMQX_EOVERFLOW
 * (n_out = deliveries needed: reserve and submit again; nothing was delivered and no pick state
 * consumed) or an error. */
typedef struct emqx_pub_batch {
  uint8_t* topic_bytes;     /* pinned, cap_bytes                                             */
  uint64_t* topic_offsets;  /* pinned, cap_topics + 1 (offsets[0] = 0)                      */
  uint32_t* keys;           /* pinned, cap_topics: per-message keys (see above)             */
  uint64_t cap_topics, cap_bytes;
  uint64_t n;               /* messages packed (set by the caller)                          */
  uint64_t* out_offsets;    /* pinned, cap_topics + 1 (valid after wait)                    */
  uint32_t* out_subs;       /* pinned, cap_out: subscriber ids                              */
  uint32_t* out_filters;    /* pinned, cap_out: filter ids | EMQX_FANOUT_SHARED_BIT         */
  uint64_t cap_out;
  uint64_t n_out;           /* deliveries of the last call (after wait)                     */
  void* priv;
} emqx_pub_batch;
int emqx_pub_batch_create(emqx_engine* e, emqx_subtab* s, uint32_t strategy, uint64_t cap_topics,
                          uint64_t cap_bytes, uint64_t cap_out, emqx_pub_batch** out);
int emqx_pub_batch_destroy(emqx_pub_batch* b);
int emqx_pub_batch_reserve(emqx_pub_batch* b, uint64_t cap_topics, uint64_t cap_bytes, uint64_t cap_out);
int emqx_pub_batch_submit(emqx_pub_batch* b);
int emqx_pub_batch_wait(emqx_pub_batch* b);
int emqx_pub_batch_query(emqx_pub_batch* b);

/* Cross-caller publish batcher: the emqx_batcher counterpart for emqx_broker:publish/1, which
 * each publisher process calls once per PUBLISH (emqx_channel.erl:608-617 -> emqx_broker.erl:
 * 203-214).  Concurrent single-message submissions are packed into the pinned publish batch
 * being filled; batches run match + fan-out with two in flight; a completion thread calls
 * cb(ctx, status, subs, filters, n) per message (arrays valid during the call).  Same
 * submit / try_submit contract as emqx_batcher. */
typedef struct emqx_pub_batcher emqx_pub_batcher;
typedef void (*emqx_pub_cb)(void* ctx, int status, const uint32_t* subs, const uint32_t* filters, uint64_t n);
int emqx_pub_batcher_create(emqx_engine* e, emqx_subtab* s, uint32_t strategy, uint32_t max_batch,
                            uint32_t max_wait_us, emqx_pub_cb cb, emqx_pub_batcher** out);
int emqx_pub_batcher_submit(emqx_pub_batcher* b, const uint8_t* topic, uint64_t len, uint32_t key, void* ctx);
int emqx_pub_batcher_try_submit(emqx_pub_batcher* b, const uint8_t* topic, uint64_t len, uint32_t key,
                                void* ctx);
int emqx_pub_batcher_submit_many(emqx_pub_batcher* b, const uint8_t* bytes, const uint64_t* offsets,
                                 const uint32_t* keys, uint64_t n, void* const* ctxs);
int emqx_pub_batcher_destroy(emqx_pub_batcher* b);
/* out[0..5] as emqx_batcher_stats_ext. */
int emqx_pub_batcher_stats_ext(emqx_pub_batcher* b, uint64_t* out, uint32_t n);

/* Filter-sharded tables (emqx_amd/dist.py): owner_out[i] = the rank that holds filter / topic i
 * in a world of `world` ranks — a hash of its first `levels` levels.  Filters (topics = 0): a
 * '+' or '#' among those levels, or fewer levels, gives EMQX_SHARD_ALL (replicated on every
 * rank).  Every filter that can match a topic lives on the topic's owner rank, so each topic is
 * matched on one rank only.  Topics (topics = 1): a wildcard key level sends the topic to rank
 * 0.  CPU form (any host memory) and device form (a topic batch in HBM, on `stream`). */
#define EMQX_SHARD_ALL 0xFFFFFFFFu
int emqx_shard_owner(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint32_t world, uint32_t levels,
                     int topics, uint32_t* owner_out);
int emqx_shard_owner_device(const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n, uint32_t world,
                            uint32_t levels, uint32_t* d_owner, void* stream);
/* Filter-sharded layout with two key spaces (emqx_amd/dist.py): the tables past
 * one GPU.  A topic l1/l2/l3/... is matched by root-wildcard filters ('#', '+', '+/#',
 * '+/+/...', replicated on every rank), by filters with a literal first level (space L, placed by
 * l1) and by filters '+/x/...' (space P, placed by x = the second level).  A key with many filters
 * (emqx_shard_plan: more than max_piece_pm / 1000 of a rank's share) is split over `span`
 * consecutive ranks by the next level; its filters whose next level is '+' / '#' live on all of
 * them.  Each rank holds two engines: "A" (space L + root-wildcard) and "B" (space P).
 * p_space: EMQX_SHARD_P_SHARDED as above; EMQX_SHARD_P_REPLICATED: space P lives on every rank
 * with the root wildcards (engine A) and a topic makes one request, to its L-space rank;
 * EMQX_SHARD_P_AUTO: replicated when space P holds at most n / world filters.  The choice is
 * recorded in the plan (entry {0x80000000, 0x0000FFFF}), so place and route follow it.
 *   emqx_shard_plan   the hot keys of a filter set (sorted; EMQX_EOVERFLOW: *n_out = needed)
 *   emqx_shard_place  filters: ranks [first, first + span) (mod world) of engine A (0) or B (1)
 *   emqx_shard_route  topics: req2[2i] = rank * 2 of its engine-A request, req2[2i + 1] = rank * 2
 *                     + 1 of its engine-B request or EMQX_SHARD_NONE ('$' topics and one-level
 *                     topics make no B request; a wildcard topic makes one request, to the first
 *                     rank of its byte-identical filter).  Every filter that can match the topic
 *                     lives, once, on one of the two: the two answers concatenate.
 *   emqx_shard_route_device  the same for a topic batch in HBM, on `stream`. */
#define EMQX_SHARD_NONE 0xFFFFFFFFu
typedef struct emqx_shard_split {
  uint32_t key;   /* space bit (0x80000000 = space P) | 31-bit level hash                       */
  uint32_t info;  /* first rank | span << 16                                                    */
} emqx_shard_split;
#define EMQX_SHARD_P_AUTO 0u
#define EMQX_SHARD_P_SHARDED 1u
#define EMQX_SHARD_P_REPLICATED 2u
int emqx_shard_plan(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint32_t world, uint32_t max_piece_pm,
                    uint32_t p_space, emqx_shard_split* out, uint32_t cap, uint32_t* n_out);
int emqx_shard_place(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint32_t world,
                     const emqx_shard_split* splits, uint32_t n_splits, uint32_t* first, uint32_t* span,
                     uint32_t* engine);
int emqx_shard_route(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint32_t world,
                     const emqx_shard_split* splits, uint32_t n_splits, uint32_t* req2);
int emqx_shard_route_device(const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n, uint32_t world,
                            const emqx_shard_split* d_splits, uint32_t n_splits, uint32_t* d_req2, void* stream);
/* Device batches regrouped for the filter-sharded layout (and their results put back), on
 * `stream`, no host synchronisation.  d_perm[p] (< n, a permutation) names the batch topic at
 * position p of the regrouped batch.
 *   emqx_batch_permute_device: topic d_perm[p] of (d_bytes, d_offsets) -> topic p of
 *     (d_out_bytes, d_out_offsets[n+1], starting at 0); d_out_bytes holds the batch's bytes.
 *   emqx_csr_unpermute_device: per-topic results of the regrouped batch (d_counts[n] in
 *     position order, d_ids topic after topic) -> the CSR in batch order (d_out_offsets[n+1],
 *     d_out_ids).
 * d_scratch: device memory of emqx_permute_scratch_bytes(n) bytes. */
uint64_t emqx_permute_scratch_bytes(uint64_t n);
/* d_perm = the batch's topics stably sorted by owner rank (d_owner[n] < world, from
 * emqx_shard_owner_device): the regrouping emqx_batch_permute_device takes.  d_scratch:
 * emqx_owner_sort_scratch_bytes(n, world) bytes. */
uint64_t emqx_owner_sort_scratch_bytes(uint64_t n, uint32_t world);
int emqx_owner_sort_device(const uint32_t* d_owner, uint64_t n, uint32_t world, uint32_t* d_perm, void* d_scratch,
                           void* stream);
int emqx_batch_permute_device(const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n, const uint32_t* d_perm,
                              uint8_t* d_out_bytes, uint64_t* d_out_offsets, void* d_scratch, void* stream);
int emqx_csr_unpermute_device(const uint32_t* d_counts, const uint32_t* d_ids, uint64_t n, const uint32_t* d_perm,
                              uint64_t* d_out_offsets, uint32_t* d_out_ids, void* d_scratch, void* stream);

/* One rank's filter-sharded match step on the device (emqx_amd/dist.py ShardedMatcher.match_all;
 * DESIGN.md §6), split at the exchanges the caller makes with its collectives (all_to_all over
 * RCCL): each call enqueues on `stream` and returns, nothing waits for the device, and the
 * step's scratch (learnt, grown with the batch) stays on the step.  One step at a time per
 * object; world <= EMQX_SHARD_MAX_WORLD; a batch holds fewer than 2^31 topics.
 * A rank matches on EMQX_SHARD_ENGINES engine slots: 0 = A (its space-L and root-wildcard
 * filters), 1 = B (its space-P filters), 2 = AB (both in one table).  A topic whose two
 * emqx_shard_route requests name the same rank, or that makes only one, asks slot 2 of that
 * rank once; otherwise slot 0 of its A rank and slot 1 of its B rank (at world 1 every request
 * is a slot-2 request).
 *   send    routes each topic, folds its requests onto the slots, sorts them by destination
 *           (stable) and packs one chunk per destination rank into d_send (send_cap >=
 *           emqx_shard_send_cap(n, batch bytes, world) bytes), chunk r first at the sum of the
 *           sizes before it:
 *             [u32 n0, n1, n2, 0, bytes0, bytes1, bytes2, 0][offsets of the n0 slot-0 requests,
 *             + 1][slot 1, + 1][slot 2, + 1] pad 16 [slot-0 topic bytes][slot 1][slot 2] pad 16
 *           d_meta[7 * world] (i64, device): per destination the chunk bytes (-1: over send_cap),
 *           n0, n1, n2, bytes0, bytes1, bytes2 — what the destination passes to recv.
 *   recv    meta_in[7 * world] (host) = the meta the sources sent this rank, d_chunks[world]
 *           (host array of device pointers) their chunks — the rank's own chunk where send
 *           packed it, so it never needs to cross a link -> one batch per slot (every source's
 *           slot-e requests in source order, offsets from 0): d_bytes[3], d_offsets[3] (host
 *           arrays of device pointers; a slot no source asks may have a NULL byte buffer).  A
 *           slot whose requests all come from one source is not copied: d_bytes[e] is replaced
 *           by the address of that source's byte region (match the slot batch there).
 *   answer  the three engines' CSRs over those batches (d_offsets[3], d_ids[3]; d_summaries[3]
 *           their emqx_match_batch_device_async summaries, entries or the array NULL) -> one
 *           answer chunk per source in d_answer (u32 words, chunk s first at the sum of the sizes
 *           before it; room for 8 * world + requests + ids):
 *             [n0, n1, n2, ids0, ids1, ids2, 0, 0][per request of slot 0, 1, 2: the end of its
 *             ids in the chunk's id region (u32, inclusive prefix)][ids 0][ids 1][ids 2]
 *           except that the chunk for self_rank (this rank's own requests; UINT32_MAX: none)
 *           carries no ids: merge reads them in place from d_ids, which must stay unchanged
 *           until it has run.  d_ans_meta[3 * world] (i64, device): per source the chunk's
 *           words, a flag (1 when an engine call did not complete, its summary flags: then no
 *           ids were copied and the caller redoes that match and the answer before the
 *           exchange), and the answer's ids.
 *   merge   ans_meta_in[3 * world] (host) = what the destinations sent, d_chunks[world] their
 *           answer chunks (host array of device pointers; this rank's own in place) ->
 *           the CSR of the batch given to send, in batch order (d_out_offsets[n + 1], d_out_ids:
 *           each topic's engine-A ids, then its engine-B ids; one slot-2 answer otherwise).
 * device < 0 creates the step in host mode: every pointer above is host memory, the calls run on
 * the caller's thread and ignore `stream` (the kernels' per-item bodies as loops; the CPU tests'
 * rehearsal of the protocol).  With one request a topic (world 1, or a plan that replicates
 * space P) the sort runs over n requests and every request is a slot-2 request. */
#define EMQX_SHARD_MAX_WORLD 64
#define EMQX_SHARD_ENGINES 3
typedef struct emqx_shard_step emqx_shard_step;
int emqx_shard_step_create(int device, uint32_t world, const emqx_shard_split* splits, uint32_t n_splits,
                           emqx_shard_step** out);
int emqx_shard_step_destroy(emqx_shard_step* st);
uint64_t emqx_shard_send_cap(uint64_t n, uint64_t batch_bytes, uint32_t world);
int emqx_shard_step_send(emqx_shard_step* st, const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n,
                         uint8_t* d_send, uint64_t send_cap, int64_t* d_meta, void* stream);
int emqx_shard_step_recv(emqx_shard_step* st, const uint8_t* const* d_chunks, const int64_t* meta_in,
                         uint8_t** d_bytes, uint64_t* const* d_offsets, void* stream);
int emqx_shard_step_answer(emqx_shard_step* st, const uint64_t* const* d_offsets, const uint32_t* const* d_ids,
                           const uint64_t* const* d_summaries, uint32_t self_rank, uint32_t* d_answer,
                           int64_t* d_ans_meta, void* stream);
int emqx_shard_step_merge(emqx_shard_step* st, const uint32_t* const* d_chunks, const int64_t* ans_meta_in,
                          uint64_t* d_out_offsets, uint32_t* d_out_ids, void* stream);

/* The step in fixed-capacity form: no size exchange and no host read between the calls, so a
 * caller can enqueue steps back to back (dist.py match_stream).  The ranks agree beforehand on
 * a request-chunk size and an answer-chunk size (each rank's chunks sit at those capacities,
 * exchanged with equal splits); a step that does not fit anywhere is flagged, the same on every
 * rank, and its result is invalid: the caller redoes it with the calls above (and learns larger
 * capacities).  One step at a time per object, as above; the calls of one step in this order.
 *   send_fixed    as send, chunk r at r * chunk_bytes of d_send (world * chunk_bytes bytes;
 *                 chunk_bytes a multiple of 16).  A chunk over chunk_bytes empties every chunk
 *                 and sets flag bit 1 in their header word 3.  d_meta as send's (device).
 *   recv_fixed    d_chunks[world] the received chunks (host array of device pointers; the own
 *                 one where send_fixed packed it) -> one fixed-size batch per slot: cap_requests[e]
 *                 topics (host array), d_offsets[e] cap_requests[e] + 1 offsets (the slot's
 *                 requests, then empty padding topics at the end of its bytes), bytes into d_bytes[e]
 *                 (cap_bytes[e] bytes).  d_bytes NULL (world 1 only): every slot is matched in place,
 *                 with its offsets from the start of d_chunks[0] (match the slot batches with bytes
 *                 = d_chunks[0]).  A flagged chunk, or a slot over its capacity, flags the step and
 *                 empties every batch.  The engines then match cap_requests[e] topics per slot.
 *   answer_fixed  as answer, chunk s at s * chunk_words of d_answer (world * chunk_words u32
 *                 words), header word 7 = the step's flag; an engine call that did not complete (its
 *                 summary) or a chunk over chunk_words flags the step, and a flagged step sends
 *                 header-only chunks.
 *   merge_fixed   d_chunks[world] the answer chunks -> the CSR as merge's (d_out_ids: room for
 *                 every answer chunk's ids and this rank's own engine ids); *d_flag (u32, device or
 *                 mapped host memory) = the step's flag ORed over every rank's chunk: 0 = valid. */
int emqx_shard_step_send_fixed(emqx_shard_step* st, const uint8_t* d_bytes, const uint64_t* d_offsets, uint64_t n,
                               uint8_t* d_send, uint64_t chunk_bytes, int64_t* d_meta, void* stream);
int emqx_shard_step_recv_fixed(emqx_shard_step* st, const uint8_t* const* d_chunks, const uint64_t* cap_requests,
                               const uint64_t* cap_bytes, uint8_t* const* d_bytes, uint64_t* const* d_offsets,
                               void* stream);
int emqx_shard_step_answer_fixed(emqx_shard_step* st, const uint64_t* const* d_offsets, const uint32_t* const* d_ids,
                                 const uint64_t* const* d_summaries, uint32_t self_rank, uint32_t* d_answer,
                                 uint64_t chunk_words, void* stream);
int emqx_shard_step_merge_fixed(emqx_shard_step* st, const uint32_t* const* d_chunks, uint64_t* d_out_offsets,
                                uint32_t* d_out_ids, uint32_t* d_flag, void* stream);

/* emqx_topic:match/2 on raw binaries (emqx_topic.erl:68-87): 1 = match, 0 = no match. */
int emqx_topic_match(const uint8_t* name, uint64_t name_len, const uint8_t* filter,
                     uint64_t filter_len);
/* emqx_topic:wildcard/1 (emqx_topic.erl:53-62): 1 if some level is exactly '+' or '#'. */
int emqx_topic_wildcard(const uint8_t* topic, uint64_t len);

/* Tuning hook (benchmarks / A-B runs).  Keys: "fast_variant" (-1 = automatic, otherwise a
 * fixed kernel variant, see emqx_amd/csrc/kernels.h), "diag" (1 = accumulate the kernel's
 * diagnostic counters), "incremental" (0 = every commit rebuilds), "delta_max" (filters placed
 * incrementally before a rebuild, -1 = default policy), "commit_threads" (host threads of an
 * incremental commit, default min(8, cores)), "timeline" (tiles of emqx_diag_timeline to record,
 * 0 = off), "small_batch" (1 = default: host / publish batches of at most 1024 topics run as one
 * kernel launch that reads the pinned inputs and writes the pinned outputs itself; 0 = the
 * batched pipeline).  EMQX_ENOTFOUND for unknown keys. */
int emqx_set_tuning(emqx_engine* e, const char* key, int64_t value);
/* Reads (and optionally resets) the accumulated diagnostic counters (DIAG_* order). */
int emqx_diag_read(emqx_engine* e, uint64_t* out, uint32_t n, int reset);
/* Per-tile timeline of the fast kernel's last "diag" call (emqx_set_tuning "timeline" = tiles to
 * record): 4 uint32 per tile {start (100 MHz ticks, low), start high, phase-A ticks | CU id << 20,
 * end - start ticks}; *n_tiles = the recorded capacity.  With "diag" off and a timeline of at
 * least 5 tiles, the one-launch small-batch kernel instead accumulates its per-phase wall clocks
 * there: 10 uint64 {copy-in, walk, deep, scan, scatter, output, fan-out pass 1, pass 2 (100 MHz
 * ticks summed over launches), launches, unused} (emqx_amd/csrc/kernels.h SMALL_CLK_*). */
int emqx_diag_timeline(emqx_engine* e, uint32_t* out, uint64_t cap_tiles, uint64_t* n_tiles);

/* Host-only self-check of the table builder (no device needed): builds the level trie of
 * the given filters and verifies its lookup invariants.  stats_out (4 entries, optional):
 * nodes, slots, interned words, perfect-hashed nodes.  err receives the failure reason. */
int emqx_build_check(const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint64_t* stats_out,
                     char* err, uint64_t err_cap);

/* Host-only self-check of incremental commits (no device): a filter store + the table builder
 * + the in-place patcher the engine uses, and a host walk of the patched table by the kernels'
 * lookup and emission rules.  spare_slots: the spare region (0 = default); threads: commit
 * threads (as the engine's "commit_threads" tuning key); commit(full = 1)
 * rebuilds; stats8 as emqx_commit_stats.  match supports EMQX_MODE_ROUTES / _TRIE_WILDCARD on
 * non-wildcard topics.  check verifies the lookup invariants of every reachable node. */
typedef struct emqx_htrie emqx_htrie;
int emqx_htrie_create(uint64_t spare_slots, int threads, emqx_htrie** out);
int emqx_htrie_destroy(emqx_htrie* h);
int emqx_htrie_insert(emqx_htrie* h, const uint8_t* bytes, const uint64_t* offsets, uint64_t n, uint32_t* ids_out);
int emqx_htrie_delete(emqx_htrie* h, const uint32_t* ids, uint64_t n);
int emqx_htrie_commit(emqx_htrie* h, int full, uint64_t* stats8);
int emqx_htrie_match(emqx_htrie* h, uint32_t mode, const uint8_t* topic_bytes, const uint64_t* topic_offsets,
                     uint64_t n, uint64_t* out_offsets, uint32_t* out_ids, uint64_t cap, uint64_t* n_out);
int emqx_htrie_check(emqx_htrie* h, char* err, uint64_t err_cap);
/* Diagnostic (tools/walk_sim.py): an L2 model of the fast kernel's walk over this image.
 * params[8]: XCDs, L2 bytes per XCD, line bytes, ways, resident tiles per XCD, phase-A ticks,
 * slab writes (1: allocate in L2, 0: streamed past it), what-if layout flags.
 * out[n_out]: topics, tiles, items, 16-B loads, L2 accesses, misses, vocab loads, vocab
 * misses, items with both probes, ... of them in different lines, chain items, their misses,
 * misses by item level 0..7+, items by level 0..7+, wide items, their misses, steps, '+' probe
 * misses, literal probe misses, emissions, '+' loads, perfect-hash loads, wide-bucket loads,
 * hits by item level 0..7+. */
int emqx_htrie_walk_sim(emqx_htrie* h, const uint8_t* topic_bytes, const uint64_t* topic_offsets, uint64_t n,
                        const uint64_t* params, uint64_t* out, uint32_t n_out);

const char* emqx_strerror(int code);
/* Library version string. */
const char* emqx_version(void);

#ifdef __cplusplus
}
#endif

#endif /* EMQX_MATCH_H */
