/* Declarations of the erl_nif API subset emqx_amd/csrc/nif/emqx_match_nif.c uses, written from
 * the public erl_nif reference (OTP 24 "erl_nif" man page), for a -fsyntax-only type check of
 * the NIF in this image, which has no Erlang/OTP (tests/test_nif_protocol.py).  Nothing is
 * linked or run against it; a real build uses OTP's own erl_nif.h (emqx_amd/csrc/nif/Makefile). */
#ifndef EMQX_TEST_ERL_NIF_DECLS_H
#define EMQX_TEST_ERL_NIF_DECLS_H
#include <stddef.h>

typedef unsigned long ERL_NIF_TERM;
typedef long ErlNifSInt64;
typedef unsigned long ErlNifUInt64;
typedef struct enif_environment_t ErlNifEnv;
typedef struct enif_resource_type_t ErlNifResourceType;
typedef struct { ERL_NIF_TERM pid; } ErlNifPid;
typedef struct {
  size_t size;
  unsigned char* data;
  void* ref_bin;
  void* __spare__[2];
} ErlNifBinary;
typedef void ErlNifResourceDtor(ErlNifEnv*, void*);
typedef enum { ERL_NIF_RT_CREATE = 1, ERL_NIF_RT_TAKEOVER = 2 } ErlNifResourceFlags;
typedef struct {
  const char* name;
  unsigned arity;
  ERL_NIF_TERM (*fptr)(ErlNifEnv* env, int argc, const ERL_NIF_TERM argv[]);
  unsigned flags;
} ErlNifFunc;
#define ERL_NIF_DIRTY_JOB_CPU_BOUND 1

int enif_get_resource(ErlNifEnv*, ERL_NIF_TERM, ErlNifResourceType*, void**);
int enif_get_int(ErlNifEnv*, ERL_NIF_TERM, int*);
int enif_get_uint(ErlNifEnv*, ERL_NIF_TERM, unsigned*);
int enif_get_int64(ErlNifEnv*, ERL_NIF_TERM, ErlNifSInt64*);
int enif_get_list_length(ErlNifEnv*, ERL_NIF_TERM, unsigned*);
int enif_get_list_cell(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM*, ERL_NIF_TERM*);
int enif_get_tuple(ErlNifEnv*, ERL_NIF_TERM, int*, const ERL_NIF_TERM**);
int enif_inspect_binary(ErlNifEnv*, ERL_NIF_TERM, ErlNifBinary*);
int enif_is_identical(ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_list(ErlNifEnv*, unsigned, ...);
ERL_NIF_TERM enif_make_list_cell(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_tuple2(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_tuple3(ErlNifEnv*, ERL_NIF_TERM, ERL_NIF_TERM, ERL_NIF_TERM);
ERL_NIF_TERM enif_make_uint(ErlNifEnv*, unsigned);
ERL_NIF_TERM enif_make_uint64(ErlNifEnv*, ErlNifUInt64);
ERL_NIF_TERM enif_schedule_nif(ErlNifEnv*, const char*, int,
                               ERL_NIF_TERM (*)(ErlNifEnv*, int, const ERL_NIF_TERM[]), int, const ERL_NIF_TERM[]);
ERL_NIF_TERM enif_make_atom(ErlNifEnv*, const char*);
ERL_NIF_TERM enif_make_badarg(ErlNifEnv*);
ERL_NIF_TERM enif_make_resource(ErlNifEnv*, void*);
ERL_NIF_TERM enif_make_copy(ErlNifEnv*, ERL_NIF_TERM);
void* enif_alloc_resource(ErlNifResourceType*, size_t);
void enif_release_resource(void*);
void enif_keep_resource(void*);
ErlNifResourceType* enif_open_resource_type(ErlNifEnv*, const char*, const char*, ErlNifResourceDtor*,
                                            ErlNifResourceFlags, ErlNifResourceFlags*);
int enif_send(ErlNifEnv*, const ErlNifPid*, ErlNifEnv*, ERL_NIF_TERM);
ErlNifPid* enif_self(ErlNifEnv*, ErlNifPid*);
ErlNifEnv* enif_alloc_env(void);
void enif_free_env(ErlNifEnv*);
void* enif_alloc(size_t);
void enif_free(void*);

#define ERL_NIF_INIT(NAME, FUNCS, LOAD, RELOAD, UPGRADE, UNLOAD)                    \
  static int (*erl_nif_load_fn_)(ErlNifEnv*, void**, ERL_NIF_TERM) = LOAD;         \
  const ErlNifFunc* nif_init_funcs_(void) { return FUNCS; }                        \
  void* nif_init_load_(void) { return (void*)erl_nif_load_fn_; }
#endif
