// Exhaustive host check of llm_inference_amd/csrc/glibc_math.h against the
// host libm (tests/test_glibc_math.py builds and runs it): every float bit
// pattern through expf and tanhf, the same source the device compiles.
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>

#include "../../llm_inference_amd/csrc/glibc_math.h"

struct Job {
  uint64_t lo, hi, bad_exp, bad_tanh, first_exp, first_tanh;
};

static int same(float a, float b) {
  uint32_t x, y;
  memcpy(&x, &a, 4);
  memcpy(&y, &b, 4);
  return x == y || (isnan(a) && isnan(b));
}

static void* run(void* p) {
  Job* j = (Job*)p;
  j->first_exp = j->first_tanh = ~0ull;
  for (uint64_t u = j->lo; u < j->hi; u++) {
    float x;
    uint32_t b = (uint32_t)u;
    memcpy(&x, &b, 4);
    if (!same(llmi_glibc::expf(x), ::expf(x))) {
      if (!j->bad_exp++) j->first_exp = u;
    }
    if (!same(llmi_glibc::tanhf(x), ::tanhf(x))) {
      if (!j->bad_tanh++) j->first_tanh = u;
    }
  }
  return NULL;
}

int main(int argc, char** argv) {
  const int T = argc > 1 ? atoi(argv[1]) : 8;
  const uint64_t N = 1ull << 32, step = (N + T - 1) / T;
  Job jobs[64];
  pthread_t th[64];
  for (int t = 0; t < T; t++) {
    jobs[t] = Job{t * step, (t + 1) * step < N ? (t + 1) * step : N, 0, 0, 0, 0};
    pthread_create(&th[t], NULL, run, &jobs[t]);
  }
  uint64_t be = 0, bt = 0;
  for (int t = 0; t < T; t++) {
    pthread_join(th[t], NULL);
    be += jobs[t].bad_exp;
    bt += jobs[t].bad_tanh;
    if (jobs[t].bad_exp && be == jobs[t].bad_exp) printf("first expf mismatch at 0x%08llx\n", (unsigned long long)jobs[t].first_exp);
    if (jobs[t].bad_tanh && bt == jobs[t].bad_tanh) printf("first tanhf mismatch at 0x%08llx\n", (unsigned long long)jobs[t].first_tanh);
  }
  printf("expf mismatches %llu, tanhf mismatches %llu (of 2^32)\n", (unsigned long long)be, (unsigned long long)bt);
  return (be || bt) ? 1 : 0;
}
