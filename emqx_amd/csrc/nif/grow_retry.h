/*
 * grow_retry.h — the NIF's output-capacity protocol, in plain C (no erl_nif.h), so the CPU
 * tests can drive it without OTP (tests/c/test_grow_retry.c).
 *
 * Engine calls that return variable-size results (emqx_match_batch, emqx_publish_batch) take a
 * capacity and return EMQX_EOVERFLOW with the capacity they need.  The result can grow between
 * two calls (a commit in between; a round-robin or sticky $share pick moving), so the caller
 * grows its buffer to what was reported (plus slack) and tries again, a bounded number of times.
 * One topic fanned out to 10K subscribers (emqx_broker.erl:500-524 delivers to every one) is the
 * case the first guess (64 deliveries per topic) misses.
 */
#ifndef EMQX_GROW_RETRY_H
#define EMQX_GROW_RETRY_H

#include <stdint.h>
#include <stdlib.h>

#include "../../../include/emqx_match.h"

/* One attempt: fill `buf` (capacity `cap` elements) and set *need to the element count of the
 * full result (set on success and on EMQX_EOVERFLOW). */
typedef int (*emqx_sized_call)(void* ctx, void* buf, uint64_t cap, uint64_t* need);

#define EMQX_GROW_ATTEMPTS 4

/* Calls `call` with a malloc'd buffer of `cap` elements of `elem` bytes, growing it on
 * EMQX_EOVERFLOW.  On EMQX_OK, *buf_out (caller frees) holds *n_out elements and has room
 * for *cap_out.  On any other status the buffer is freed and *buf_out is NULL. */
static int emqx_call_growing(emqx_sized_call call, void* ctx, size_t elem, uint64_t cap, void** buf_out,
                             uint64_t* cap_out, uint64_t* n_out) {
  void* buf = NULL;
  int rc = EMQX_EOVERFLOW;
  uint64_t need = 0;
  *buf_out = NULL;
  for (int attempt = 0; attempt < EMQX_GROW_ATTEMPTS && rc == EMQX_EOVERFLOW; ++attempt) {
    free(buf);
    buf = malloc(elem * (cap ? cap : 1));
    if (!buf) return EMQX_ENOMEM;
    need = 0;
    rc = call(ctx, buf, cap, &need);
    if (rc == EMQX_EOVERFLOW) {
      if (need <= cap) {  /* an engine that reports no larger need: give up rather than spin */
        rc = EMQX_EDEVICE;
        break;
      }
      cap = need + need / 8 + 64;
    }
  }
  if (rc != EMQX_OK) {
    free(buf);
    return rc;
  }
  *buf_out = buf;
  *cap_out = cap;
  *n_out = need;
  return EMQX_OK;
}

#endif /* EMQX_GROW_RETRY_H */
