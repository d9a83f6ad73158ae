// Op-level A/B of the prefill attention kernels (MFMA vs vector) on random q / K / V
// (development tool: hipcc -std=c++17 -I llm_inference_amd/csrc scripts/dev/pattn_check.cpp -L llm_inference_amd -lllmi)
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include "session_kernels.h"
using namespace llmi;
static uint16_t f2h(float f) { _Float16 h = (_Float16)f; uint16_t u; memcpy(&u, &h, 2); return u; }
int main(int argc, char** argv) {
  const int HD = argc > 1 ? atoi(argv[1]) : 256, NH = argc > 2 ? atoi(argv[2]) : 4, NKV = argc > 3 ? atoi(argv[3]) : 1;
  const int T = argc > 4 ? atoi(argv[4]) : 40, pos0 = argc > 5 ? atoi(argv[5]) : 0, max_ctx = 1024;
  std::mt19937 rng(1);
  std::normal_distribution<float> nd(0.f, 1.f);
  std::vector<uint16_t> q((size_t)T * NH * HD), kc((size_t)NKV * max_ctx * HD), vc(kc.size());
  for (auto& x : q) x = f2h(nd(rng) * 0.1f);
  const int mode = argc > 6 ? atoi(argv[6]) : 0;  // 1: K = 0 (uniform softmax: isolates P V)
  for (auto& x : kc) x = mode == 1 ? 0 : f2h(nd(rng));
  for (size_t i = 0; i < vc.size(); i++)  // 2: V[key][d] = key / 64, 3: V[key][d] = d / 256 (K = 0 in both)
    vc[i] = mode == 2 ? f2h((float)((i / HD) % max_ctx) / 64) : mode == 3 ? f2h((float)(i % HD) / 256) : f2h(nd(rng));
  if (mode >= 2) for (auto& x : kc) x = 0;
  uint16_t *dq, *dk, *dv;
  XBlock *o1, *o2;
  const int xs = NH * HD / 32;
  hipMalloc(&dq, q.size() * 2); hipMalloc(&dk, kc.size() * 2); hipMalloc(&dv, vc.size() * 2);
  hipMalloc(&o1, (size_t)T * xs * sizeof(XBlock)); hipMalloc(&o2, (size_t)T * xs * sizeof(XBlock));
  hipMemcpy(dq, q.data(), q.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dk, kc.data(), kc.size() * 2, hipMemcpyHostToDevice);
  hipMemcpy(dv, vc.data(), vc.size() * 2, hipMemcpyHostToDevice);
  PrefillAttn a;
  a.q = dq; a.k_cache = dk; a.v_cache = dv; a.n_head = NH; a.n_head_kv = NKV; a.head_dim = HD;
  a.max_ctx = max_ctx; a.pos0 = pos0; a.xstride = xs;
  a.xq = o1; setenv("LLMI_PREFILL_ATTN_V1", "1", 1); launch_prefill_attn(a, T, 0);
  a.xq = o2; unsetenv("LLMI_PREFILL_ATTN_V1"); launch_prefill_attn(a, T, 0);
  hipDeviceSynchronize();
  std::vector<XBlock> h1((size_t)T * xs), h2(h1.size());
  hipMemcpy(h1.data(), o1, h1.size() * sizeof(XBlock), hipMemcpyDeviceToHost);
  hipMemcpy(h2.data(), o2, h2.size() * sizeof(XBlock), hipMemcpyDeviceToHost);
  double worst = 0; int wt = -1, wb = -1;
  for (int t = 0; t < T; t++)
    for (int b = 0; b < xs; b++) {
      const XBlock &x1 = h1[(size_t)t * xs + b], &x2 = h2[(size_t)t * xs + b];
      const int8_t* q1 = reinterpret_cast<const int8_t*>(&x1);
      const int8_t* q2 = reinterpret_cast<const int8_t*>(&x2);
      for (int i = 0; i < 32; i++) {
        const double e = std::fabs(q1[i] * (double)x1.d - q2[i] * (double)x2.d);
        if (e > worst) { worst = e; wt = t; wb = b; }
      }
    }
  printf("HD %d NH %d NKV %d T %d pos0 %d: max |vector - mfma| = %.4g (token %d block %d)\n", HD, NH, NKV, T, pos0, worst, wt, wb);
  if (wt >= 0) {
    const XBlock &x1 = h1[(size_t)wt * xs + wb], &x2 = h2[(size_t)wt * xs + wb];
    const int8_t* q1 = reinterpret_cast<const int8_t*>(&x1);
    const int8_t* q2 = reinterpret_cast<const int8_t*>(&x2);
    for (int i = 0; i < 32; i++) printf("%6.3f/%6.3f%s", q1[i] * x1.d, q2[i] * x2.d, i % 8 == 7 ? "\n" : " ");
  }
  return worst > 0.05;
}
