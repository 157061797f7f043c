/*
 * emqx_match_nif.c — thin Erlang NIF over the engine's C ABI (include/emqx_match.h).
 *
 * This is the reference-side binding: EMQX's Erlang modules keep their call shapes and call
 * these NIFs (see INTEGRATION.md for the Erlang stubs and the edits to emqx_trie.erl,
 * emqx_router.erl and emqx_broker.erl).  Built only where OTP's erl_nif.h exists
 * (`make -C emqx_amd/csrc/nif ERL_INCLUDE=...`); this image has no Erlang/OTP,
 * so the C ABI underneath is what the repo's tests exercise directly.
 *
 * Scheduling: every call that can wait on the device runs on a DIRTY CPU scheduler.  The
 * per-PUBLISH calls (emqx_router:match_routes/1, apps/emqx/src/emqx_router.erl:127-133, and the
 * fan-out of emqx_broker:publish/1, emqx_broker.erl:203-214, both called from each publisher
 * process) go through the cross-caller batchers: match_async/3 and publish_async/4 copy the
 * topic into the pinned batch being filled and return at once; the engine's completion thread
 * enif_send()s {Ref, Result} to the caller when its batch completes, so many publisher
 * processes share one kernel launch.  These two run on a normal scheduler and never wait:
 * they use the batchers' try_submit, and only when every pinned buffer is busy do they
 * reschedule themselves (enif_schedule_nif) onto a dirty CPU scheduler, where the blocking
 * submit applies the backpressure.
 *
 * Errors: {error, Atom} with Atom in einval | enomem | device_error | overflow | not_found |
 * too_deep; non-binary topics raise badarg (the reference's `when is_binary(Topic)` guards).
 */
#include <erl_nif.h>
#include <stdlib.h>
#include <string.h>

#include "../../../include/emqx_match.h"
#include "../../../include/emqx_retain.h"
#include "grow_retry.h"

static ErlNifResourceType* RES_ENGINE;
static ErlNifResourceType* RES_SUBTAB;
static ErlNifResourceType* RES_BATCHER;
static ErlNifResourceType* RES_PUB_BATCHER;
static ErlNifResourceType* RES_RETAIN;
static ErlNifResourceType* RES_COALESCER;

typedef struct { emqx_engine* e; } engine_res;
typedef struct { emqx_subtab* s; } subtab_res;
typedef struct { emqx_batcher* b; engine_res* owner; } batcher_res;
typedef struct { emqx_pub_batcher* b; engine_res* eng; subtab_res* tab; } pub_batcher_res;
typedef struct { emqx_retain* r; } retain_res;
typedef struct { emqx_coalescer* c; engine_res* eng; subtab_res* tab; } coalescer_res;

static ERL_NIF_TERM ATOM_OK, ATOM_ERROR, ATOM_TRUE, ATOM_FALSE, ATOM_EINVAL, ATOM_ENOMEM, ATOM_DEVICE,
    ATOM_OVERFLOW, ATOM_NOTFOUND, ATOM_TOODEEP, ATOM_BUSY, ATOM_UNKNOWN, ATOM_FRESH, ATOM_RETRY;

static ERL_NIF_TERM err_term(ErlNifEnv* env, int rc) {
  ERL_NIF_TERM a;
  switch (rc) {
    case EMQX_EINVAL: a = ATOM_EINVAL; break;
    case EMQX_ENOMEM: a = ATOM_ENOMEM; break;
    case EMQX_EDEVICE: a = ATOM_DEVICE; break;
    case EMQX_EOVERFLOW: a = ATOM_OVERFLOW; break;
    case EMQX_ENOTFOUND: a = ATOM_NOTFOUND; break;
    case EMQX_ETOODEEP: a = ATOM_TOODEEP; break;
    case EMQX_EBUSY: a = ATOM_BUSY; break;
    default: a = ATOM_UNKNOWN; break;
  }
  return enif_make_tuple2(env, ATOM_ERROR, a);
}

static void engine_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  engine_res* r = (engine_res*)obj;
  if (r->e) emqx_engine_destroy(r->e);
  r->e = NULL;
}

static void subtab_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  subtab_res* r = (subtab_res*)obj;
  if (r->s) emqx_subtab_destroy(r->s);
  r->s = NULL;
}

static void batcher_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  batcher_res* r = (batcher_res*)obj;
  if (r->b) emqx_batcher_destroy(r->b); /* drains pending submissions */
  r->b = NULL;
  if (r->owner) enif_release_resource(r->owner);
  r->owner = NULL;
}

static void pub_batcher_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  pub_batcher_res* r = (pub_batcher_res*)obj;
  if (r->b) emqx_pub_batcher_destroy(r->b); /* drains pending submissions */
  r->b = NULL;
  if (r->tab) enif_release_resource(r->tab);
  if (r->eng) enif_release_resource(r->eng);
  r->tab = NULL;
  r->eng = NULL;
}

static void coalescer_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  coalescer_res* r = (coalescer_res*)obj;
  if (r->c) emqx_coalescer_destroy(r->c); /* commits and notifies what is pending */
  r->c = NULL;
  if (r->tab) enif_release_resource(r->tab);
  if (r->eng) enif_release_resource(r->eng);
  r->tab = NULL;
  r->eng = NULL;
}

static void retain_dtor(ErlNifEnv* env, void* obj) {
  (void)env;
  retain_res* r = (retain_res*)obj;
  if (r->r) emqx_retain_destroy(r->r);
  r->r = NULL;
}

/* Packs a list of binaries into one buffer + offsets (malloc'd; caller frees).  Returns 1, 0
 * for a bad argument, -1 when out of memory (nothing to free in either failure). */
static int pack_binaries(ErlNifEnv* env, ERL_NIF_TERM list, uint8_t** bytes, uint64_t** offs, unsigned* n_out) {
  unsigned n;
  if (!enif_get_list_length(env, list, &n)) return 0;
  *offs = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
  if (!*offs) return -1;
  size_t total = 0;
  ERL_NIF_TERM head, tail = list;
  ErlNifBinary bin;
  for (unsigned i = 0; i < n; ++i) {
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_inspect_binary(env, head, &bin)) {
      free(*offs);
      return 0;
    }
    total += bin.size;
  }
  *bytes = (uint8_t*)malloc(total ? total : 1);
  if (!*bytes) {
    free(*offs);
    return -1;
  }
  (*offs)[0] = 0;
  tail = list;
  for (unsigned i = 0; i < n; ++i) {
    enif_get_list_cell(env, tail, &head, &tail);
    enif_inspect_binary(env, head, &bin);
    memcpy(*bytes + (*offs)[i], bin.data, bin.size);
    (*offs)[i + 1] = (*offs)[i] + bin.size;
  }
  *n_out = n;
  return 1;
}

/* A delivery's filter id and its kind: false (plain), true ($share pick) or retry (a $share
 * pick made as do_pick/6's {retry, Sub}: sent without an ack request). */
static uint32_t filter_of(uint32_t fl) { return fl & ~(EMQX_FANOUT_SHARED_BIT | EMQX_FANOUT_RETRY_BIT); }
static ERL_NIF_TERM shared_term(uint32_t fl) {
  if (!(fl & EMQX_FANOUT_SHARED_BIT)) return ATOM_FALSE;
  return (fl & EMQX_FANOUT_RETRY_BIT) ? ATOM_RETRY : ATOM_TRUE;
}

static ERL_NIF_TERM u32_list(ErlNifEnv* env, const uint32_t* v, uint64_t n) {
  ERL_NIF_TERM l = enif_make_list(env, 0);
  for (uint64_t i = n; i > 0; --i) l = enif_make_list_cell(env, enif_make_uint(env, v[i - 1]), l);
  return l;
}

/* new_engine(Device) -> {ok, Ref} | {error, Reason} */
static ERL_NIF_TERM nif_new_engine(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  int dev;
  (void)argc;
  if (!enif_get_int(env, argv[0], &dev)) return enif_make_badarg(env);
  emqx_engine_opts o = {dev, 0};
  engine_res* r = (engine_res*)enif_alloc_resource(RES_ENGINE, sizeof(engine_res));
  int rc = emqx_engine_create(&o, &r->e);
  if (rc != EMQX_OK) {
    r->e = NULL;
    enif_release_resource(r);
    return err_term(env, rc);
  }
  ERL_NIF_TERM t = enif_make_resource(env, r);
  enif_release_resource(r);
  return enif_make_tuple2(env, ATOM_OK, t);
}

/* insert(Eng, [Filter]) -> {ok, [Id]}  (emqx_trie:insert/1, emqx_router:do_add_route/2) */
static ERL_NIF_TERM nif_insert(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  engine_res* r;
  uint8_t* bytes;
  uint64_t* offs;
  unsigned n;
  int pk = 0;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_ENGINE, (void**)&r) || (pk = pack_binaries(env, argv[1], &bytes, &offs, &n)) != 1)
    return pk < 0 ? err_term(env, EMQX_ENOMEM) : enif_make_badarg(env);
  uint32_t* ids = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  if (!ids) {
    free(bytes);
    free(offs);
    return err_term(env, EMQX_ENOMEM);
  }
  int rc = emqx_insert_filters(r->e, bytes, offs, n, ids);
  ERL_NIF_TERM out = rc == EMQX_OK ? enif_make_tuple2(env, ATOM_OK, u32_list(env, ids, n)) : err_term(env, rc);
  free(ids);
  free(bytes);
  free(offs);
  return out;
}

/* delete(Eng, [Id]) -> ok  (emqx_trie:delete/1) */
static ERL_NIF_TERM nif_delete(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  engine_res* r;
  unsigned n;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_ENGINE, (void**)&r) || !enif_get_list_length(env, argv[1], &n))
    return enif_make_badarg(env);
  uint32_t* ids = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  if (!ids) return err_term(env, EMQX_ENOMEM);
  ERL_NIF_TERM head, tail = argv[1];
  for (unsigned i = 0; i < n; ++i) {
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_get_uint(env, head, &ids[i])) {
      free(ids);
      return enif_make_badarg(env);
    }
  }
  int rc = emqx_delete_filters(r->e, ids, n);
  free(ids);
  return rc == EMQX_OK ? ATOM_OK : err_term(env, rc);
}

/* commit(Eng) -> ok  (rebuild + epoch swap; dirty CPU, seconds at 10M filters) */
static ERL_NIF_TERM nif_commit(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  engine_res* r;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_ENGINE, (void**)&r)) return enif_make_badarg(env);
  int rc = emqx_commit(r->e);
  return rc == EMQX_OK ? ATOM_OK : err_term(env, rc);
}

/* empty(Eng) -> boolean()  (emqx_trie:empty/0) */
static ERL_NIF_TERM nif_empty(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  engine_res* r;
  emqx_stats st;
  (void)argc;
  st.size = sizeof(st);
  if (!enif_get_resource(env, argv[0], RES_ENGINE, (void**)&r)) return enif_make_badarg(env);
  if (emqx_stats_get(r->e, &st) != EMQX_OK) return enif_make_badarg(env);
  return st.n_filters == 0 ? ATOM_TRUE : ATOM_FALSE;
}

/* emqx_match_batch as an emqx_sized_call (grow_retry.h) */
typedef struct {
  emqx_engine* e;
  unsigned mode;
  const uint8_t* bytes;
  const uint64_t* offs;
  unsigned n;
  uint64_t* out_off;
} match_call;

static int call_match(void* ctx, void* buf, uint64_t cap, uint64_t* need) {
  match_call* c = (match_call*)ctx;
  return emqx_match_batch(c->e, c->mode, c->bytes, c->offs, c->n, c->out_off, (uint32_t*)buf, cap, need);
}

/* match_batch(Eng, Mode, [Topic]) -> {ok, [[Id]]}  (batched emqx_trie:match/1 and
 * emqx_router:match_routes/1; dirty CPU) */
static ERL_NIF_TERM nif_match_batch(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  engine_res* r;
  unsigned mode, n;
  uint8_t* bytes;
  uint64_t* offs;
  int pk = 0;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_ENGINE, (void**)&r) || !enif_get_uint(env, argv[1], &mode) || (pk = pack_binaries(env, argv[2], &bytes, &offs, &n)) != 1)
    return pk < 0 ? err_term(env, EMQX_ENOMEM) : enif_make_badarg(env);
  uint64_t* out_off = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
  if (!out_off) {
    free(bytes);
    free(offs);
    return err_term(env, EMQX_ENOMEM);
  }
  match_call mc = {r->e, mode, bytes, offs, n, out_off};
  void* buf = NULL;
  uint64_t cap = 0, total = 0;
  int rc = emqx_call_growing(call_match, &mc, sizeof(uint32_t), 16 * (uint64_t)n + 64, &buf, &cap, &total);
  const uint32_t* ids = (const uint32_t*)buf;
  ERL_NIF_TERM out;
  if (rc == EMQX_OK) {
    ERL_NIF_TERM l = enif_make_list(env, 0);
    for (unsigned i = n; i > 0; --i)
      l = enif_make_list_cell(env, u32_list(env, ids + out_off[i - 1], out_off[i] - out_off[i - 1]), l);
    out = enif_make_tuple2(env, ATOM_OK, l);
  } else {
    out = err_term(env, rc);
  }
  free(buf);
  free(out_off);
  free(bytes);
  free(offs);
  return out;
}

/* ---- cross-caller batcher ------------------------------------------------------ */
typedef struct {
  ErlNifPid pid;
  ErlNifEnv* env;
  ERL_NIF_TERM ref;
} waiter;

static void batch_done(void* ctx, int status, const uint32_t* ids, uint64_t n) {
  waiter* w = (waiter*)ctx;
  ERL_NIF_TERM res = status == EMQX_OK ? enif_make_tuple2(w->env, ATOM_OK, u32_list(w->env, ids, n))
                                       : err_term(w->env, status);
  enif_send(NULL, &w->pid, w->env, enif_make_tuple2(w->env, w->ref, res));
  enif_free_env(w->env);
  enif_free(w);
}

/* new_batcher(Eng, Mode, MaxBatch, MaxWaitUs) -> {ok, Ref} */
static ERL_NIF_TERM nif_new_batcher(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  engine_res* r;
  unsigned mode, max_batch, max_wait;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_ENGINE, (void**)&r) || !enif_get_uint(env, argv[1], &mode) ||
      !enif_get_uint(env, argv[2], &max_batch) || !enif_get_uint(env, argv[3], &max_wait))
    return enif_make_badarg(env);
  batcher_res* b = (batcher_res*)enif_alloc_resource(RES_BATCHER, sizeof(batcher_res));
  b->owner = NULL;
  int rc = emqx_batcher_create(r->e, mode, max_batch, max_wait, batch_done, &b->b);
  if (rc != EMQX_OK) {
    b->b = NULL;
    enif_release_resource(b);
    return err_term(env, rc);
  }
  enif_keep_resource(r); /* the engine outlives its batcher */
  b->owner = r;
  ERL_NIF_TERM t = enif_make_resource(env, b);
  enif_release_resource(b);
  return enif_make_tuple2(env, ATOM_OK, t);
}

/* match_async(Batcher, Topic, Ref) -> ok; the caller then receives {Ref, {ok, [Id]}}.
 * Normal scheduler: the topic goes into the batch being filled (a memcpy under the batcher's
 * lock); with every pinned buffer busy the call continues on a dirty scheduler. */
static ERL_NIF_TERM match_async_submit(ErlNifEnv* env, const ERL_NIF_TERM argv[], int may_wait, int* busy) {
  batcher_res* b;
  ErlNifBinary bin;
  if (!enif_get_resource(env, argv[0], RES_BATCHER, (void**)&b) || !enif_inspect_binary(env, argv[1], &bin))
    return enif_make_badarg(env);
  *busy = 0;
  waiter* w = (waiter*)enif_alloc(sizeof(waiter));
  enif_self(env, &w->pid);
  w->env = enif_alloc_env();
  w->ref = enif_make_copy(w->env, argv[2]);
  int rc = may_wait ? emqx_batcher_submit(b->b, bin.data, bin.size, w)
                    : emqx_batcher_try_submit(b->b, bin.data, bin.size, w);
  if (rc != EMQX_OK) {
    enif_free_env(w->env);
    enif_free(w);
    *busy = rc == EMQX_EBUSY && !may_wait;
    return *busy ? ATOM_ERROR : err_term(env, rc);
  }
  return ATOM_OK;
}

static ERL_NIF_TERM nif_match_async_dirty(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  int busy = 0;
  return match_async_submit(env, argv, 1, &busy);
}

static ERL_NIF_TERM nif_match_async(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  int busy = 0;
  ERL_NIF_TERM r = match_async_submit(env, argv, 0, &busy);
  if (busy) /* EMQX_EBUSY: wait for a buffer on a dirty scheduler, not here */
    return enif_schedule_nif(env, "match_async", ERL_NIF_DIRTY_JOB_CPU_BOUND, nif_match_async_dirty, argc, argv);
  return r;
}

/* ---- fan-out ------------------------------------------------------------------- */
/* new_subtab(Device) -> {ok, Ref} */
static ERL_NIF_TERM nif_new_subtab(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  int dev;
  (void)argc;
  if (!enif_get_int(env, argv[0], &dev)) return enif_make_badarg(env);
  subtab_res* r = (subtab_res*)enif_alloc_resource(RES_SUBTAB, sizeof(subtab_res));
  int rc = emqx_subtab_create(dev, &r->s);
  if (rc != EMQX_OK) {
    r->s = NULL;
    enif_release_resource(r);
    return err_term(env, rc);
  }
  ERL_NIF_TERM t = enif_make_resource(env, r);
  enif_release_resource(r);
  return enif_make_tuple2(env, ATOM_OK, t);
}

/* ---- route and subscription changes through the commit coalescer -------------------------
 * One SUBSCRIBE is one ETS write in the reference (emqx_broker.erl:146-164), a new topic's route
 * one mria transaction (emqx_router.erl:111-124); here every change of every caller is applied at
 * once and committed with the others that arrive meanwhile (emqx_coalescer, group commit), and
 * the caller gets {Ref, ok | {error, Reason}} when the commit carrying it has reached the device. */
static void change_done(void* ctx, int status) {
  waiter* w = (waiter*)ctx;
  enif_send(NULL, &w->pid, w->env, enif_make_tuple2(w->env, w->ref, status == EMQX_OK ? ATOM_OK : err_term(w->env, status)));
  enif_free_env(w->env);
  enif_free(w);
}

static waiter* new_waiter(ErlNifEnv* env, ERL_NIF_TERM ref) {
  waiter* w = (waiter*)enif_alloc(sizeof(waiter));
  if (!w) return NULL;
  enif_self(env, &w->pid);
  w->env = enif_alloc_env();
  w->ref = enif_make_copy(w->env, ref);
  return w;
}

static void drop_waiter(waiter* w) {
  enif_free_env(w->env);
  enif_free(w);
}

/* new_coalescer(Eng, Subtab, MaxWaitUs) -> {ok, Ref} */
static ERL_NIF_TERM nif_new_coalescer(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  engine_res* er;
  subtab_res* sr;
  unsigned max_wait;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_ENGINE, (void**)&er) ||
      !enif_get_resource(env, argv[1], RES_SUBTAB, (void**)&sr) || !enif_get_uint(env, argv[2], &max_wait))
    return enif_make_badarg(env);
  coalescer_res* c = (coalescer_res*)enif_alloc_resource(RES_COALESCER, sizeof(coalescer_res));
  c->eng = NULL;
  c->tab = NULL;
  int rc = emqx_coalescer_create(er->e, sr->s, max_wait, change_done, &c->c);
  if (rc != EMQX_OK) {
    c->c = NULL;
    enif_release_resource(c);
    return err_term(env, rc);
  }
  enif_keep_resource(er); /* the engine and the table outlive their coalescer */
  enif_keep_resource(sr);
  c->eng = er;
  c->tab = sr;
  ERL_NIF_TERM t = enif_make_resource(env, c);
  enif_release_resource(c);
  return enif_make_tuple2(env, ATOM_OK, t);
}

/* subscribe_async(Coal, [{FilterId, SubId, GroupId | none}], Add :: boolean(), Ref) -> ok; then
 * {Ref, ok | {error, Reason}} once committed (emqx_broker:subscribe/3 and unsubscribe/1,
 * emqx_broker.erl:124-195; emqx_shared_sub's subscribe / unsubscribe, emqx_shared_sub.erl:308-322) */
static ERL_NIF_TERM nif_subscribe_async(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  coalescer_res* r;
  unsigned n;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_COALESCER, (void**)&r) || !enif_get_list_length(env, argv[1], &n))
    return enif_make_badarg(env);
  uint32_t* f = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1) * 3);
  if (!f) return err_term(env, EMQX_ENOMEM);
  uint32_t *s = f + n, *g = f + 2 * n;
  ERL_NIF_TERM head, tail = argv[1];
  for (unsigned i = 0; i < n; ++i) {
    const ERL_NIF_TERM* tup;
    int arity;
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_get_tuple(env, head, &arity, &tup) || arity != 3 ||
        !enif_get_uint(env, tup[0], &f[i]) || !enif_get_uint(env, tup[1], &s[i])) {
      free(f);
      return enif_make_badarg(env);
    }
    if (!enif_get_uint(env, tup[2], &g[i])) g[i] = EMQX_NO_GROUP; /* 'none' */
  }
  waiter* w = new_waiter(env, argv[3]);
  if (!w) {
    free(f);
    return err_term(env, EMQX_ENOMEM);
  }
  int rc = emqx_coalescer_subscribe(r->c, f, s, g, n, enif_is_identical(argv[2], ATOM_TRUE), w);
  free(f);
  if (rc != EMQX_OK) drop_waiter(w);
  return rc == EMQX_OK ? ATOM_OK : err_term(env, rc);
}

/* route_add_async(Coal, [Filter], Ref) -> {ok, [Id]}; then {Ref, ok | {error, Reason}} once the
 * filters are in the committed trie (emqx_trie:insert/1 via emqx_router_utils:insert_trie_route/2,
 * emqx_router_utils.erl:33-50,97-125) */
static ERL_NIF_TERM nif_route_add_async(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  coalescer_res* r;
  uint8_t* bytes;
  uint64_t* offs;
  unsigned n;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_COALESCER, (void**)&r)) return enif_make_badarg(env);
  int pk = pack_binaries(env, argv[1], &bytes, &offs, &n);
  if (pk < 0) return err_term(env, EMQX_ENOMEM);
  if (!pk) return enif_make_badarg(env);
  uint32_t* ids = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  waiter* w = ids ? new_waiter(env, argv[2]) : NULL;
  int rc = w ? emqx_coalescer_insert_filters(r->c, bytes, offs, n, ids, w) : EMQX_ENOMEM;
  if (rc != EMQX_OK && w) drop_waiter(w);
  ERL_NIF_TERM out = rc == EMQX_OK ? enif_make_tuple2(env, ATOM_OK, u32_list(env, ids, n)) : err_term(env, rc);
  free(ids);
  free(bytes);
  free(offs);
  return out;
}

/* route_delete_async(Coal, [Id], Ref) -> ok; then {Ref, ok | {error, Reason}} (emqx_trie:delete/1
 * via delete_trie_route/2, emqx_router_utils.erl:52-70) */
static ERL_NIF_TERM nif_route_delete_async(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  coalescer_res* r;
  unsigned n;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_COALESCER, (void**)&r) || !enif_get_list_length(env, argv[1], &n))
    return enif_make_badarg(env);
  uint32_t* ids = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  if (!ids) return err_term(env, EMQX_ENOMEM);
  ERL_NIF_TERM head, tail = argv[1];
  for (unsigned i = 0; i < n; ++i) {
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_get_uint(env, head, &ids[i])) {
      free(ids);
      return enif_make_badarg(env);
    }
  }
  waiter* w = new_waiter(env, argv[2]);
  int rc = w ? emqx_coalescer_delete_filters(r->c, ids, n, w) : EMQX_ENOMEM;
  if (rc != EMQX_OK && w) drop_waiter(w);
  free(ids);
  return rc == EMQX_OK ? ATOM_OK : err_term(env, rc);
}

/* emqx_publish_batch as an emqx_sized_call: subscriber ids in buf[0, cap), filter ids in
 * buf[cap, 2 cap) */
typedef struct {
  emqx_engine* e;
  emqx_subtab* s;
  unsigned strategy;
  const uint8_t* bytes;
  const uint64_t* offs;
  unsigned n;
  const uint32_t* keys;
  uint64_t* out_off;
} publish_call;

static int call_publish(void* ctx, void* buf, uint64_t cap, uint64_t* need) {
  publish_call* c = (publish_call*)ctx;
  uint32_t* subs = (uint32_t*)buf;
  return emqx_publish_batch(c->e, c->s, c->strategy, c->bytes, c->offs, c->n, c->keys, c->out_off, subs, subs + cap,
                            cap, need);
}

/* publish_batch(Eng, Subtab, Strategy, [{Topic, Key}]) ->
 *   {ok, [[{SubId, FilterId, Shared :: boolean() | retry}]]}
 * Key = erlang:phash2(ClientId) or erlang:phash2(Topic) computed by the caller (hash
 * strategies); the publisher's handle, erlang:phash2(self()), for round_robin / sticky, whose
 * state the reference keeps in the publishing process's dictionary
 * (emqx_shared_sub.erl:234-247,279-285); ignored for random.  Dirty CPU. */
static ERL_NIF_TERM nif_publish_batch(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  engine_res* er;
  subtab_res* sr;
  unsigned strategy, n;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_ENGINE, (void**)&er) ||
      !enif_get_resource(env, argv[1], RES_SUBTAB, (void**)&sr) || !enif_get_uint(env, argv[2], &strategy) ||
      !enif_get_list_length(env, argv[3], &n))
    return enif_make_badarg(env);
  uint64_t* offs = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
  uint32_t* keys = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  ErlNifBinary* bins = (ErlNifBinary*)malloc(sizeof(ErlNifBinary) * (n ? n : 1));
  if (!offs || !keys || !bins) {
    free(offs);
    free(keys);
    free(bins);
    return err_term(env, EMQX_ENOMEM);
  }
  ERL_NIF_TERM head, tail = argv[3];
  offs[0] = 0;
  for (unsigned i = 0; i < n; ++i) {
    const ERL_NIF_TERM* tup;
    int arity;
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_get_tuple(env, head, &arity, &tup) || arity != 2 ||
        !enif_inspect_binary(env, tup[0], &bins[i]) || !enif_get_uint(env, tup[1], &keys[i])) {
      free(offs);
      free(keys);
      free(bins);
      return enif_make_badarg(env);
    }
    offs[i + 1] = offs[i] + bins[i].size;
  }
  uint8_t* bytes = (uint8_t*)malloc(offs[n] ? offs[n] : 1);
  uint64_t* out_off = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
  if (!bytes || !out_off) {
    free(bytes);
    free(out_off);
    free(offs);
    free(keys);
    free(bins);
    return err_term(env, EMQX_ENOMEM);
  }
  for (unsigned i = 0; i < n; ++i) memcpy(bytes + offs[i], bins[i].data, bins[i].size);
  /* deliveries: subscriber ids then filter ids, `cap` each (8 bytes per delivery); a topic
   * with more subscribers than the first guess overflows and is retried at the size the
   * engine reports (emqx_broker:publish/1 delivers to every subscriber, emqx_broker.erl:500-524) */
  publish_call pc = {er->e, sr->s, strategy, bytes, offs, n, keys, out_off};
  void* buf = NULL;
  uint64_t cap = 0, total = 0;
  int rc = emqx_call_growing(call_publish, &pc, 2 * sizeof(uint32_t), 64 * (uint64_t)n + 64, &buf, &cap, &total);
  ERL_NIF_TERM out;
  if (rc == EMQX_OK) {
    const uint32_t* subs = (const uint32_t*)buf;
    ERL_NIF_TERM rows = enif_make_list(env, 0);
    for (unsigned i = n; i > 0; --i) {
      ERL_NIF_TERM row = enif_make_list(env, 0);
      for (uint64_t j = out_off[i]; j > out_off[i - 1]; --j) {
        const uint32_t fl = subs[cap + j - 1];
        ERL_NIF_TERM d = enif_make_tuple3(env, enif_make_uint(env, subs[j - 1]), enif_make_uint(env, filter_of(fl)),
                                          shared_term(fl));
        row = enif_make_list_cell(env, d, row);
      }
      rows = enif_make_list_cell(env, row, rows);
    }
    out = enif_make_tuple2(env, ATOM_OK, rows);
  } else {
    out = err_term(env, rc);
  }
  free(buf);
  free(out_off);
  free(bytes);
  free(bins);
  free(keys);
  free(offs);
  return out;
}

/* ---- publish fan-out batcher ------------------------------------------------------- */
static ERL_NIF_TERM deliveries(ErlNifEnv* env, const uint32_t* subs, const uint32_t* fils, uint64_t n) {
  ERL_NIF_TERM row = enif_make_list(env, 0);
  for (uint64_t j = n; j > 0; --j) {
    const uint32_t fl = fils[j - 1];
    row = enif_make_list_cell(
        env, enif_make_tuple3(env, enif_make_uint(env, subs[j - 1]), enif_make_uint(env, filter_of(fl)), shared_term(fl)),
        row);
  }
  return row;
}

static void publish_done(void* ctx, int status, const uint32_t* subs, const uint32_t* fils, uint64_t n) {
  waiter* w = (waiter*)ctx;
  ERL_NIF_TERM res = status == EMQX_OK ? enif_make_tuple2(w->env, ATOM_OK, deliveries(w->env, subs, fils, n))
                                       : err_term(w->env, status);
  enif_send(NULL, &w->pid, w->env, enif_make_tuple2(w->env, w->ref, res));
  enif_free_env(w->env);
  enif_free(w);
}

/* new_pub_batcher(Eng, Subtab, Strategy, MaxBatch, MaxWaitUs) -> {ok, Ref} */
static ERL_NIF_TERM nif_new_pub_batcher(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  engine_res* er;
  subtab_res* sr;
  unsigned strategy, max_batch, max_wait;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_ENGINE, (void**)&er) ||
      !enif_get_resource(env, argv[1], RES_SUBTAB, (void**)&sr) || !enif_get_uint(env, argv[2], &strategy) ||
      !enif_get_uint(env, argv[3], &max_batch) || !enif_get_uint(env, argv[4], &max_wait))
    return enif_make_badarg(env);
  pub_batcher_res* b = (pub_batcher_res*)enif_alloc_resource(RES_PUB_BATCHER, sizeof(pub_batcher_res));
  b->eng = NULL;
  b->tab = NULL;
  int rc = emqx_pub_batcher_create(er->e, sr->s, strategy, max_batch, max_wait, publish_done, &b->b);
  if (rc != EMQX_OK) {
    b->b = NULL;
    enif_release_resource(b);
    return err_term(env, rc);
  }
  enif_keep_resource(er); /* the engine and the table outlive their batcher */
  enif_keep_resource(sr);
  b->eng = er;
  b->tab = sr;
  ERL_NIF_TERM t = enif_make_resource(env, b);
  enif_release_resource(b);
  return enif_make_tuple2(env, ATOM_OK, t);
}

/* publish_async(PubBatcher, Topic, Key, Ref) -> ok; the caller then receives
 * {Ref, {ok, [{SubId, FilterId, Shared}]}} (Key as in publish_batch/4).  Normal scheduler,
 * continued on a dirty one only when every pinned buffer is busy. */
static ERL_NIF_TERM publish_async_submit(ErlNifEnv* env, const ERL_NIF_TERM argv[], int may_wait, int* busy) {
  pub_batcher_res* b;
  ErlNifBinary bin;
  unsigned key;
  if (!enif_get_resource(env, argv[0], RES_PUB_BATCHER, (void**)&b) || !enif_inspect_binary(env, argv[1], &bin) ||
      !enif_get_uint(env, argv[2], &key))
    return enif_make_badarg(env);
  *busy = 0;
  waiter* w = (waiter*)enif_alloc(sizeof(waiter));
  enif_self(env, &w->pid);
  w->env = enif_alloc_env();
  w->ref = enif_make_copy(w->env, argv[3]);
  int rc = may_wait ? emqx_pub_batcher_submit(b->b, bin.data, bin.size, key, w)
                    : emqx_pub_batcher_try_submit(b->b, bin.data, bin.size, key, w);
  if (rc != EMQX_OK) {
    enif_free_env(w->env);
    enif_free(w);
    *busy = rc == EMQX_EBUSY && !may_wait;
    return *busy ? ATOM_ERROR : err_term(env, rc);
  }
  return ATOM_OK;
}

static ERL_NIF_TERM nif_publish_async_dirty(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  (void)argc;
  int busy = 0;
  return publish_async_submit(env, argv, 1, &busy);
}

static ERL_NIF_TERM nif_publish_async(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  int busy = 0;
  ERL_NIF_TERM r = publish_async_submit(env, argv, 0, &busy);
  if (busy)
    return enif_schedule_nif(env, "publish_async", ERL_NIF_DIRTY_JOB_CPU_BOUND, nif_publish_async_dirty, argc, argv);
  return r;
}

/* forget_publishers(Subtab, [Key]) -> ok: the round_robin / sticky state of publishers whose
 * processes ended (their process dictionaries are gone in the reference) */
static ERL_NIF_TERM nif_forget_publishers(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  subtab_res* r;
  unsigned n;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_SUBTAB, (void**)&r) || !enif_get_list_length(env, argv[1], &n))
    return enif_make_badarg(env);
  uint32_t* keys = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  if (!keys) return err_term(env, EMQX_ENOMEM);
  ERL_NIF_TERM head, tail = argv[1];
  for (unsigned i = 0; i < n; ++i) {
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_get_uint(env, head, &keys[i])) {
      free(keys);
      return enif_make_badarg(env);
    }
  }
  int rc = emqx_subtab_forget_publishers(r->s, keys, n);
  free(keys);
  return rc == EMQX_OK ? ATOM_OK : err_term(env, rc);
}

/* subscriber_down(Coal, [SubId]) -> ok: the subscribers' processes ended (the 'DOWN' that
 * emqx_shared_sub monitors, emqx_shared_sub.erl:347-350): a sticky pick leaves them from the next
 * commit on, which the coalescer runs at once when idle; their subscriptions are removed by the
 * caller's cleanup as cleanup_down/1 does (:369-376).  Does not wait for the commit. */
static ERL_NIF_TERM nif_subscriber_down(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  coalescer_res* r;
  unsigned n;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_COALESCER, (void**)&r) || !enif_get_list_length(env, argv[1], &n))
    return enif_make_badarg(env);
  uint32_t* ids = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  if (!ids) return err_term(env, EMQX_ENOMEM);
  ERL_NIF_TERM head, tail = argv[1];
  for (unsigned i = 0; i < n; ++i) {
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_get_uint(env, head, &ids[i])) {
      free(ids);
      return enif_make_badarg(env);
    }
  }
  int rc = emqx_coalescer_set_alive(r->c, ids, n, 0, NULL);
  free(ids);
  return rc == EMQX_OK ? ATOM_OK : err_term(env, rc);
}

/* share_repick(Subtab, Strategy, FilterId, GroupId, Key, [FailedSubId]) ->
 *   {fresh, SubId} | {retry, SubId} | false
 * emqx_shared_sub:dispatch/4's next pick after a nack / timeout / 'DOWN' of the delivery to
 * SubId (shared_dispatch_ack_enabled, emqx_shared_sub.erl:118-130,165-189): do_pick/6 over
 * All -- FailedSubs with the publisher's round_robin / sticky state (Key as in
 * publish_batch/4).  Dirty CPU: it waits for the device. */
static ERL_NIF_TERM nif_share_repick(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  subtab_res* r;
  unsigned strategy, fid, gid, key, n;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_SUBTAB, (void**)&r) || !enif_get_uint(env, argv[1], &strategy) ||
      !enif_get_uint(env, argv[2], &fid) || !enif_get_uint(env, argv[3], &gid) || !enif_get_uint(env, argv[4], &key) ||
      !enif_get_list_length(env, argv[5], &n))
    return enif_make_badarg(env);
  uint32_t* failed = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  if (!failed) return err_term(env, EMQX_ENOMEM);
  ERL_NIF_TERM head, tail = argv[5];
  for (unsigned i = 0; i < n; ++i) {
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_get_uint(env, head, &failed[i])) {
      free(failed);
      return enif_make_badarg(env);
    }
  }
  const uint32_t f = fid, g = gid, k = key;
  const uint64_t off[2] = {0, n};
  uint32_t sub = 0, kind = EMQX_PICK_NONE;
  int rc = emqx_share_repick(r->s, strategy, 1, &f, &g, &k, off, failed, &sub, &kind);
  free(failed);
  if (rc != EMQX_OK) return err_term(env, rc);
  if (kind == EMQX_PICK_NONE) return ATOM_FALSE;
  return enif_make_tuple2(env, kind == EMQX_PICK_RETRY ? ATOM_RETRY : ATOM_FRESH, enif_make_uint(env, sub));
}

/* ---- retained-message index (include/emqx_retain.h) ------------------------------------
 * The mnesia retainer backend keeps its #retained{} records; the device index answers which
 * stored topics a subscription filter selects (emqx_retainer_mnesia.erl:199-245). */

/* new_retain(Device) -> {ok, Ref}  (emqx_retainer_mnesia:create_resource/1, :47-72) */
static ERL_NIF_TERM nif_new_retain(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  int dev;
  (void)argc;
  if (!enif_get_int(env, argv[0], &dev)) return enif_make_badarg(env);
  retain_res* r = (retain_res*)enif_alloc_resource(RES_RETAIN, sizeof(retain_res));
  int rc = emqx_retain_create(dev, &r->r);
  if (rc != EMQX_OK) {
    r->r = NULL;
    enif_release_resource(r);
    return err_term(env, rc);
  }
  ERL_NIF_TERM t = enif_make_resource(env, r);
  enif_release_resource(r);
  return enif_make_tuple2(env, ATOM_OK, t);
}

/* retain_store(Idx, [Topic], [ExpiryMs]) -> {ok, [Id]}  (store_retained/2, :74-98; ExpiryMs 0 =
 * never, emqx_retainer:get_expiry_time/1) */
static ERL_NIF_TERM nif_retain_store(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  retain_res* r;
  uint8_t* bytes;
  uint64_t* offs;
  unsigned n, ne;
  int pk = 0;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_RETAIN, (void**)&r) || !enif_get_list_length(env, argv[2], &ne) || (pk = pack_binaries(env, argv[1], &bytes, &offs, &n)) != 1)
    return pk < 0 ? err_term(env, EMQX_ENOMEM) : enif_make_badarg(env);
  if (ne != n) {
    free(bytes);
    free(offs);
    return enif_make_badarg(env);
  }
  int64_t* exp = (int64_t*)malloc(sizeof(int64_t) * (n ? n : 1));
  uint32_t* ids = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  if (!exp || !ids) {
    free(exp);
    free(ids);
    free(bytes);
    free(offs);
    return err_term(env, EMQX_ENOMEM);
  }
  ERL_NIF_TERM head, tail = argv[2];
  int ok = 1;
  for (unsigned i = 0; i < n && ok; ++i) {
    ErlNifSInt64 v;
    ok = enif_get_list_cell(env, tail, &head, &tail) && enif_get_int64(env, head, &v);
    exp[i] = (int64_t)v;
  }
  ERL_NIF_TERM out;
  if (!ok) {
    out = enif_make_badarg(env);
  } else {
    int rc = emqx_retain_store(r->r, bytes, offs, n, exp, ids);
    out = rc == EMQX_OK ? enif_make_tuple2(env, ATOM_OK, u32_list(env, ids, n)) : err_term(env, rc);
  }
  free(ids);
  free(exp);
  free(bytes);
  free(offs);
  return out;
}

/* retain_delete(Idx, [Id]) -> ok  (delete_message/2, :117-128; clear_expired/1, :106-115) */
static ERL_NIF_TERM nif_retain_delete(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  retain_res* r;
  unsigned n;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_RETAIN, (void**)&r) || !enif_get_list_length(env, argv[1], &n))
    return enif_make_badarg(env);
  uint32_t* ids = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
  if (!ids) return err_term(env, EMQX_ENOMEM);
  ERL_NIF_TERM head, tail = argv[1];
  for (unsigned i = 0; i < n; ++i) {
    if (!enif_get_list_cell(env, tail, &head, &tail) || !enif_get_uint(env, head, &ids[i])) {
      free(ids);
      return enif_make_badarg(env);
    }
  }
  int rc = emqx_retain_delete(r->r, ids, n);
  free(ids);
  return rc == EMQX_OK ? ATOM_OK : err_term(env, rc);
}

/* retain_commit(Idx) -> ok  (the end of the mria write that made the store visible) */
static ERL_NIF_TERM nif_retain_commit(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  retain_res* r;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_RETAIN, (void**)&r)) return enif_make_badarg(env);
  int rc = emqx_retain_commit(r->r);
  return rc == EMQX_OK ? ATOM_OK : err_term(env, rc);
}

/* emqx_retain_match_batch as an emqx_sized_call (grow_retry.h) */
typedef struct {
  emqx_retain* r;
  const uint8_t* bytes;
  const uint64_t* offs;
  unsigned n;
  int64_t now;
  uint64_t* out_off;
} retain_call;

static int call_retain(void* ctx, void* buf, uint64_t cap, uint64_t* need) {
  retain_call* c = (retain_call*)ctx;
  return emqx_retain_match_batch(c->r, c->bytes, c->offs, c->n, c->now, c->out_off, (uint32_t*)buf, cap, need);
}

/* retain_match(Idx, [Filter], NowMs) -> {ok, [[Id]]}  (emqx_retainer:dispatch/4 ->
 * read_message/2 or match_messages/3, emqx_retainer.erl:119-131, emqx_retainer_mnesia.erl:
 * 199-245; NowMs < 0: no expiry guard, match_delete_messages/1) */
static ERL_NIF_TERM nif_retain_match(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  retain_res* r;
  uint8_t* bytes;
  uint64_t* offs;
  unsigned n;
  ErlNifSInt64 now;
  int pk = 0;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_RETAIN, (void**)&r) || !enif_get_int64(env, argv[2], &now) || (pk = pack_binaries(env, argv[1], &bytes, &offs, &n)) != 1)
    return pk < 0 ? err_term(env, EMQX_ENOMEM) : enif_make_badarg(env);
  uint64_t* out_off = (uint64_t*)malloc(sizeof(uint64_t) * (n + 1));
  if (!out_off) {
    free(bytes);
    free(offs);
    return err_term(env, EMQX_ENOMEM);
  }
  retain_call rc_ = {r->r, bytes, offs, n, (int64_t)now, out_off};
  void* buf = NULL;
  uint64_t cap = 0, total = 0;
  int rc = emqx_call_growing(call_retain, &rc_, sizeof(uint32_t), 64 * (uint64_t)n + 64, &buf, &cap, &total);
  ERL_NIF_TERM out;
  if (rc == EMQX_OK) {
    const uint32_t* ids = (const uint32_t*)buf;
    ERL_NIF_TERM l = enif_make_list(env, 0);
    for (unsigned i = n; i > 0; --i)
      l = enif_make_list_cell(env, u32_list(env, ids + out_off[i - 1], out_off[i] - out_off[i - 1]), l);
    out = enif_make_tuple2(env, ATOM_OK, l);
  } else {
    out = err_term(env, rc);
  }
  free(buf);
  free(out_off);
  free(bytes);
  free(offs);
  return out;
}

/* retain_lookup(Idx, Topic) -> {ok, Id} | {error, not_found}  (read_message/2's key read) */
static ERL_NIF_TERM nif_retain_lookup(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  retain_res* r;
  ErlNifBinary bin;
  uint32_t id;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_RETAIN, (void**)&r) || !enif_inspect_binary(env, argv[1], &bin))
    return enif_make_badarg(env);
  int rc = emqx_retain_lookup(r->r, bin.data, bin.size, &id);
  return rc == EMQX_OK ? enif_make_tuple2(env, ATOM_OK, enif_make_uint(env, id)) : err_term(env, rc);
}

/* emqx_retain_expired as an emqx_sized_call */
typedef struct {
  emqx_retain* r;
  int64_t now;
} expired_call;

static int call_expired(void* ctx, void* buf, uint64_t cap, uint64_t* need) {
  expired_call* c = (expired_call*)ctx;
  return emqx_retain_expired(c->r, c->now, (uint32_t*)buf, cap, need);
}

/* retain_expired(Idx, NowMs) -> {ok, [Id]}  (clear_expired/1's select, :106-115) */
static ERL_NIF_TERM nif_retain_expired(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  retain_res* r;
  ErlNifSInt64 now;
  (void)argc;
  if (!enif_get_resource(env, argv[0], RES_RETAIN, (void**)&r) || !enif_get_int64(env, argv[1], &now))
    return enif_make_badarg(env);
  expired_call c = {r->r, (int64_t)now};
  void* buf = NULL;
  uint64_t cap = 0, total = 0;
  int rc = emqx_call_growing(call_expired, &c, sizeof(uint32_t), 1024, &buf, &cap, &total);
  ERL_NIF_TERM out = rc == EMQX_OK ? enif_make_tuple2(env, ATOM_OK, u32_list(env, (const uint32_t*)buf, total))
                                   : err_term(env, rc);
  free(buf);
  return out;
}

/* retain_size(Idx) -> non_neg_integer()  (size/1, :164-165) */
static ERL_NIF_TERM nif_retain_size(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  retain_res* r;
  emqx_retain_stats st;
  (void)argc;
  st.size = sizeof(st);
  if (!enif_get_resource(env, argv[0], RES_RETAIN, (void**)&r)) return enif_make_badarg(env);
  int rc = emqx_retain_stats_get(r->r, &st);
  return rc == EMQX_OK ? enif_make_uint64(env, (ErlNifUInt64)st.n_live) : err_term(env, rc);
}

/* topic_match(Name, Filter) -> boolean()  (emqx_topic:match/2 on binaries; normal scheduler) */
static ERL_NIF_TERM nif_topic_match(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]) {
  ErlNifBinary a, b;
  (void)argc;
  if (!enif_inspect_binary(env, argv[0], &a) || !enif_inspect_binary(env, argv[1], &b)) return enif_make_badarg(env);
  return emqx_topic_match(a.data, a.size, b.data, b.size) ? ATOM_TRUE : ATOM_FALSE;
}

static int load(ErlNifEnv* env, void** priv, ERL_NIF_TERM info) {
  (void)priv;
  (void)info;
  const ErlNifResourceFlags fl = ERL_NIF_RT_CREATE | ERL_NIF_RT_TAKEOVER;
  RES_ENGINE = enif_open_resource_type(env, NULL, "emqx_match_engine", engine_dtor, fl, NULL);
  RES_SUBTAB = enif_open_resource_type(env, NULL, "emqx_match_subtab", subtab_dtor, fl, NULL);
  RES_BATCHER = enif_open_resource_type(env, NULL, "emqx_match_batcher", batcher_dtor, fl, NULL);
  RES_PUB_BATCHER = enif_open_resource_type(env, NULL, "emqx_match_pub_batcher", pub_batcher_dtor, fl, NULL);
  RES_RETAIN = enif_open_resource_type(env, NULL, "emqx_match_retain", retain_dtor, fl, NULL);
  RES_COALESCER = enif_open_resource_type(env, NULL, "emqx_match_coalescer", coalescer_dtor, fl, NULL);
  ATOM_OK = enif_make_atom(env, "ok");
  ATOM_ERROR = enif_make_atom(env, "error");
  ATOM_TRUE = enif_make_atom(env, "true");
  ATOM_FALSE = enif_make_atom(env, "false");
  ATOM_EINVAL = enif_make_atom(env, "einval");
  ATOM_ENOMEM = enif_make_atom(env, "enomem");
  ATOM_DEVICE = enif_make_atom(env, "device_error");
  ATOM_OVERFLOW = enif_make_atom(env, "overflow");
  ATOM_NOTFOUND = enif_make_atom(env, "not_found");
  ATOM_TOODEEP = enif_make_atom(env, "too_deep");
  ATOM_BUSY = enif_make_atom(env, "busy");
  ATOM_UNKNOWN = enif_make_atom(env, "unknown");
  ATOM_FRESH = enif_make_atom(env, "fresh");
  ATOM_RETRY = enif_make_atom(env, "retry");
  return RES_ENGINE && RES_SUBTAB && RES_BATCHER && RES_PUB_BATCHER && RES_RETAIN && RES_COALESCER ? 0 : 1;
}

/* Flags: DIRTY for every call that can wait on the device or on a lock held across device
 * work (empty/1 reads the filter count under the writer lock a commit holds); 0 (normal
 * scheduler) only for calls that never wait: topic_match/2 (a CPU predicate), match_async/3 and publish_async/4 (try_submit; a busy batcher moves the call to a
 * dirty scheduler with enif_schedule_nif). */
static ErlNifFunc nif_funcs[] = {
    {"new_engine", 1, nif_new_engine, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"insert", 2, nif_insert, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"delete", 2, nif_delete, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"commit", 1, nif_commit, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"empty", 1, nif_empty, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"match_batch", 3, nif_match_batch, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"new_batcher", 4, nif_new_batcher, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"match_async", 3, nif_match_async, 0},
    {"new_subtab", 1, nif_new_subtab, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"new_coalescer", 3, nif_new_coalescer, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"subscribe_async", 4, nif_subscribe_async, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"route_add_async", 3, nif_route_add_async, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"route_delete_async", 3, nif_route_delete_async, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"publish_batch", 4, nif_publish_batch, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"new_pub_batcher", 5, nif_new_pub_batcher, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"publish_async", 4, nif_publish_async, 0},
    {"forget_publishers", 2, nif_forget_publishers, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"subscriber_down", 2, nif_subscriber_down, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"share_repick", 6, nif_share_repick, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"topic_match", 2, nif_topic_match, 0},
    {"new_retain", 1, nif_new_retain, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"retain_store", 3, nif_retain_store, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"retain_delete", 2, nif_retain_delete, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"retain_commit", 1, nif_retain_commit, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"retain_match", 3, nif_retain_match, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"retain_lookup", 2, nif_retain_lookup, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"retain_expired", 2, nif_retain_expired, ERL_NIF_DIRTY_JOB_CPU_BOUND},
    {"retain_size", 1, nif_retain_size, ERL_NIF_DIRTY_JOB_CPU_BOUND},
};

ERL_NIF_INIT(emqx_match_nif, nif_funcs, load, NULL, NULL, NULL)
