/* CPU test of the NIF's output-capacity protocol (emqx_amd/csrc/nif/grow_retry.h), driven by
 * a stand-in for emqx_publish_batch: one PUBLISH whose topic has 10K subscribers, a result that
 * grows between attempts (a commit in between), and an engine that keeps overflowing.
 * Built and run by tests/test_nif_protocol.py with gcc; exit status 0 = pass. */
#include <stdio.h>
#include <string.h>

#include "grow_retry.h"

typedef struct {
  uint64_t result[8];  /* the full result size at each attempt */
  int calls;
} fake;

/* emqx_publish_batch's contract: deliveries (sub, filter) pairs into two arrays of `cap` each
 * (elem = 8 bytes), EMQX_EOVERFLOW + needed count when they do not fit. */
static int fake_publish(void* ctx, void* buf, uint64_t cap, uint64_t* need) {
  fake* f = (fake*)ctx;
  const uint64_t n = f->result[f->calls < 8 ? f->calls : 7];
  f->calls += 1;
  *need = n;
  if (n > cap) return EMQX_EOVERFLOW;
  uint32_t* subs = (uint32_t*)buf;
  uint32_t* fil = subs + cap;
  for (uint64_t i = 0; i < n; ++i) {
    subs[i] = (uint32_t)i;
    fil[i] = 7;
  }
  return EMQX_OK;
}

#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      fprintf(stderr, "%s:%d: %s\n", __FILE__, __LINE__, #c); \
      return 1;                                               \
    }                                                         \
  } while (0)

int main(void) {
  void* buf;
  uint64_t cap, n;
  /* one topic, 10K subscribers: the 64/topic first guess overflows once */
  fake a = {{10000, 10000}, 0};
  CHECK(emqx_call_growing(fake_publish, &a, 8, 64 + 64, &buf, &cap, &n) == EMQX_OK);
  CHECK(a.calls == 2 && n == 10000 && cap >= 10000);
  const uint32_t* s = (const uint32_t*)buf;
  CHECK(s[0] == 0 && s[9999] == 9999 && s[cap + 9999] == 7);
  free(buf);
  /* the result grows between attempts (subscribers added by a commit): a third attempt */
  fake b = {{10000, 12000, 12000}, 0};
  CHECK(emqx_call_growing(fake_publish, &b, 8, 128, &buf, &cap, &n) == EMQX_OK);
  CHECK(b.calls == 3 && n == 12000);
  free(buf);
  /* first guess large enough: one call */
  fake c = {{5}, 0};
  CHECK(emqx_call_growing(fake_publish, &c, 8, 128, &buf, &cap, &n) == EMQX_OK);
  CHECK(c.calls == 1 && n == 5);
  free(buf);
  /* keeps growing every time: bounded attempts, then the overflow is reported */
  fake d = {{200, 400, 800, 1600, 3200, 6400, 12800, 25600}, 0};
  CHECK(emqx_call_growing(fake_publish, &d, 8, 128, &buf, &cap, &n) == EMQX_EOVERFLOW);
  CHECK(d.calls == EMQX_GROW_ATTEMPTS && buf == NULL);
  /* an engine that reports overflow without a larger need: no spinning */
  fake e = {{0}, 0};
  e.result[0] = 100;
  CHECK(emqx_call_growing(fake_publish, &e, 8, 100, &buf, &cap, &n) == EMQX_OK);
  printf("ok\n");
  return 0;
}
