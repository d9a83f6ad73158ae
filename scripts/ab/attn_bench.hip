// attn_bench.hip -- A/B timing of the fast attention launch (development tool).
// The current k_attn.hip is compiled as namespace llmi, a reference copy as
// namespace llmi_old (-Dllmi=llmi_old); both are timed on the same inputs,
// 200 launches captured in one hipGraph.
#include "../../llm_inference_amd/csrc/attn.h"

#include <algorithm>
#include <vector>

namespace llmi_old {
struct AttnArgs;
struct QKVArgs;
void launch_attention(const AttnArgs& a, bool exact, hipStream_t s, const QKVArgs* fused);
}  // namespace llmi_old

using namespace llmi;
#ifdef LLMI_ATTN_TRACE
namespace llmi {
void attn_set_trace(unsigned long long* p);
}
#endif

__global__ void fill_h(uint16_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15;
    p[i] = f2h(((h & 0xFFFF) / 65536.0f - 0.5f) * 0.5f);
  }
}
__global__ void fill_f(float* p, size_t n, uint32_t seed, float scale, float bias) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 15;
    p[i] = ((h & 0xFFFF) / 65536.0f - 0.5f) * scale + bias;
  }
}

template <typename T>
T* dm(size_t n) {
  T* p;
  LLMI_HIP(hipMalloc(&p, n * sizeof(T) + 256));
  LLMI_HIP(hipMemset(p, 0, n * sizeof(T) + 256));
  return p;
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  hipStream_t s;
  LLMI_HIP(hipStreamCreate(&s));
  const int n_kv = 4, G = 2, HD = 256, n_head = n_kv * G, max_ctx = 4096;
  const size_t kvn = (size_t)n_kv * max_ctx * HD;
  std::vector<uint16_t*> kc, vc;
  const int layers = 34;  // distinct caches so launches read HBM, as in decode
  for (int l = 0; l < layers; l++) {
    kc.push_back(dm<uint16_t>(kvn));
    vc.push_back(dm<uint16_t>(kvn));
    hipLaunchKernelGGL(fill_h, dim3(1024), dim3(256), 0, s, kc[l], kvn, 1u + l);
    hipLaunchKernelGGL(fill_h, dim3(1024), dim3(256), 0, s, vc[l], kvn, 100u + l);
  }
  const int qkv_n = (n_head + 2 * n_kv) * HD;
  float* qkv = dm<float>(qkv_n);
  hipLaunchKernelGGL(fill_f, dim3(64), dim3(256), 0, s, qkv, (size_t)qkv_n, 7u, 2.0f, 0.0f);
  float* nw = dm<float>(HD);
  hipLaunchKernelGGL(fill_f, dim3(4), dim3(256), 0, s, nw, (size_t)HD, 9u, 0.2f, 1.0f);
  float* cs = dm<float>((size_t)max_ctx * HD);
  hipLaunchKernelGGL(fill_f, dim3(256), dim3(256), 0, s, cs, (size_t)max_ctx * HD, 11u, 1.0f, 0.0f);
  float* q = dm<float>(n_head * HD);
  float* part = dm<float>((size_t)n_head * ATTN_NSPLIT * (HD + 2));
  float* out = dm<float>(n_head * HD);
  unsigned* ticket = dm<unsigned>(n_kv);
  XBlock* q8 = dm<XBlock>(n_head * HD / 32 + 1);
  int* dpos = dm<int>(1);
  hipEvent_t e0, e1;
  LLMI_HIP(hipEventCreate(&e0));
  LLMI_HIP(hipEventCreate(&e1));
  for (int pos : {100, 700, 2000, 4000}) {
    LLMI_HIP(hipMemcpy(dpos, &pos, 4, hipMemcpyHostToDevice));
    for (int ver = 0; ver < 2; ver++) {
      auto launch = [&](int l) {
        QKVArgs qa{qkv, n_head * HD, (n_head + n_kv) * HD, n_head, n_kv, HD, nw, nw, cs, 0.0625f, 1e-6, q,
                   kc[l], vc[l], max_ctx, dpos};
        AttnArgs a{q, kc[l], vc[l], n_head, n_kv, HD, max_ctx, dpos, part, out, ticket, q8};
        if (ver == 0)
          launch_attention(a, false, s, &qa);
        else
          llmi_old::launch_attention(reinterpret_cast<const llmi_old::AttnArgs&>(a), false, s,
                                     reinterpret_cast<const llmi_old::QKVArgs*>(&qa));
      };
      for (int l = 0; l < layers; l++) launch(l);
      LLMI_HIP(hipStreamSynchronize(s));
      hipGraph_t g;
      hipGraphExec_t ge;
      LLMI_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
      for (int i = 0; i < reps; i++) launch(i % layers);
      LLMI_HIP(hipStreamEndCapture(s, &g));
      LLMI_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      LLMI_HIP(hipGraphLaunch(ge, s));
      LLMI_HIP(hipStreamSynchronize(s));
      LLMI_HIP(hipEventRecord(e0, s));
      LLMI_HIP(hipGraphLaunch(ge, s));
      LLMI_HIP(hipEventRecord(e1, s));
      LLMI_HIP(hipEventSynchronize(e1));
      float ms = 0;
      LLMI_HIP(hipEventElapsedTime(&ms, e0, e1));
      printf("pos %5d  %-8s %7.2f us/launch\n", pos, ver == 0 ? "current" : "old", ms * 1000.0 / reps);
      fflush(stdout);
      (void)hipGraphExecDestroy(ge);
      (void)hipGraphDestroy(g);
    }
  }
#ifdef LLMI_ATTN_TRACE
  // phase trace of one launch per position (current version), 100 MHz ticks
  unsigned long long* tr = dm<unsigned long long>((size_t)n_kv * ATTN_NSPLIT * 8);
  std::vector<unsigned long long> h((size_t)n_kv * ATTN_NSPLIT * 8);
  for (int pos : {700, 4000}) {
    LLMI_HIP(hipMemcpy(dpos, &pos, 4, hipMemcpyHostToDevice));
    LLMI_HIP(hipMemset(tr, 0, h.size() * 8));
    attn_set_trace(tr);
    QKVArgs qa{qkv, n_head * HD, (n_head + n_kv) * HD, n_head, n_kv, HD, nw, nw, cs, 0.0625f, 1e-6, q,
               kc[3], vc[3], max_ctx, dpos};
    AttnArgs a{q, kc[3], vc[3], n_head, n_kv, HD, max_ctx, dpos, part, out, ticket, q8};
    launch_attention(a, false, s, &qa);
    LLMI_HIP(hipStreamSynchronize(s));
    attn_set_trace(nullptr);
    LLMI_HIP(hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long t0 = ~0ull;
    for (size_t b = 0; b < h.size() / 8; b++) t0 = std::min(t0, h[b * 8]);
    printf("pos %d: per work-group phase times in us from the first work-group start\n", pos);
    printf("  wg(hkv,c)  start  prolog  tile1  loopend ticket merged  ml_in  v_done\n");
    for (size_t b = 0; b < h.size() / 8; b++) {
      if ((b % ATTN_NSPLIT) > 12 && (b % ATTN_NSPLIT) != ATTN_NSPLIT - 1 && !h[b * 8 + 5]) continue;
      printf("  (%d,%2d)", (int)(b / ATTN_NSPLIT), (int)(b % ATTN_NSPLIT));
      for (int ph = 0; ph < 8; ph++)
        printf(" %7.2f", h[b * 8 + ph] ? (h[b * 8 + ph] - t0) / 100.0 : -1.0);
      printf("\n");
    }
  }
#endif
  printf("done\n");
  return 0;
}
