// kq_sweep.hip -- microbenchmark of the K-quant (kq layout) decode GEMVs of the
// 4B Q4_K_M layer (development tool, not part of the product): Q4_K gate_up
// (GELU role) and Q6_K / Q4_K down (QUANT role), row-major vs slab-major, next
// to the Q4_0 table entries.  Every timed launch reads a different copy of the
// weight (copies x bytes > the MALL), as in a real decode step.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude \
//        scripts/kq_sweep.hip -o scripts/kq_sweep
// run:   scripts/kq_sweep [reps]
#include "../llm_inference_amd/csrc/k_layer.hip"

#include <algorithm>
#include <cstring>
#include <vector>

using namespace llmi;

namespace {

__global__ void fill_kernel(uint32_t* p, size_t n, uint32_t seed, uint32_t mask, uint32_t add) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    p[i] = (h & mask) + add;
  }
}

struct KW {  // one kq weight copy (or Q4_0 when type == T_Q4_0)
  DevWeight w;
  size_t bytes;
};

KW alloc_w(uint32_t type, int rows, int cols, int slab, hipStream_t s, uint32_t seed) {
  KW k;
  DevWeight& w = k.w;
  w.type = type;
  w.rows = rows;
  w.cols = cols;
  w.slab = slab;
  const size_t nsub = (size_t)rows * (cols / 32), nsb = nsub / 8;
  LLMI_HIP(hipMalloc(&w.qs, nsub * 16 + 64));
  LLMI_HIP(hipMalloc((void**)&w.d, nsub * 2 + 64));
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, s, (uint32_t*)w.qs, nsub * 4, seed, ~0u, 0u);
  // small positive f16 scales (two per word)
  hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, s, (uint32_t*)w.d, nsub / 2, seed + 1, 0x00FF00FFu,
                     type == T_Q4_0 ? 0x20002000u : 0x01010101u);
  k.bytes = nsub * 18;
  if (type != T_Q4_0) {
    w.kq = 1;
    LLMI_HIP(hipMalloc(&w.kdd, nsb * 4 + 64));
    hipLaunchKernelGGL(fill_kernel, dim3(256), dim3(256), 0, s, w.kdd, nsb, seed + 2, 0x00FF00FFu, 0x20002000u);
    k.bytes = nsub * 18 + nsb * 4;
    if (type == T_Q6_K) {
      LLMI_HIP(hipMalloc(&w.kqh, nsub * 8 + 64));
      hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, s, (uint32_t*)w.kqh, nsub * 2, seed + 3, ~0u, 0u);
      k.bytes += nsub * 8;
    }
  }
  return k;
}

float* dmalloc_f(size_t n) {
  float* p;
  LLMI_HIP(hipMalloc(&p, n * 4 + 256));
  LLMI_HIP(hipMemset(p, 0, n * 4 + 256));
  return p;
}

}  // namespace

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 200;
  LLMI_HIP(hipSetDevice(0));
  hipStream_t s;
  LLMI_HIP(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  LLMI_HIP(hipEventCreate(&e0));
  LLMI_HIP(hipEventCreate(&e1));
  float* y = dmalloc_f(32768);
  float* r0 = dmalloc_f(32768);
  float* r1 = dmalloc_f(32768);
  float* wn = dmalloc_f(32768);
  float* hid = dmalloc_f(32768);
  float* out = dmalloc_f(32768);

  // time one kernel variant over `copies` weight copies of (type, rows, cols, slab)
  auto sweep = [&](const char* label, uint32_t type, int rows, int cols, int slab, int role, auto kern,
                   int rows_per_wg, int threads) {
    std::vector<KW> ws;
    size_t one = 0;
    {
      KW k = alloc_w(type, rows, cols, slab, s, 1u);
      one = k.bytes;
      ws.push_back(k);
    }
    const int copies = (int)std::max<size_t>(2, (size_t)(1536ull << 20) / one + 1);
    for (int c = 1; c < copies; c++) ws.push_back(alloc_w(type, rows, cols, slab, s, 1u + 7u * c));
    LLMI_HIP(hipStreamSynchronize(s));
    const int nb = cols / 32;
    LayerGemv a{};
    a.y = y;
    a.resid_in = r0;
    a.resid_out = r1;
    a.w_post = wn;
    a.w_next = wn;
    a.eps = 1e-6f;
    if (role == LAYER_GELU) a.hid = hid;
    else a.out = out;
    a.rows = rows;
    a.nb = nb;
    a.magic = div_magic(nb);
    a.n = cols;
    a.slab = slab;
    const bool pro = role == LAYER_PRO || role == LAYER_GELU;
    const size_t lds = (size_t)nb * sizeof(XBlock) + 16 + (pro ? (size_t)cols * 4 : 0);
    auto launch = [&](const KW& k) {
      LayerGemv b = a;
      b.qs = (const uint4*)k.w.qs;
      b.wd = k.w.d;
      b.kdd = k.w.kdd;
      b.kqh = k.w.kqh;
      hipLaunchKernelGGL(kern, dim3((rows + rows_per_wg - 1) / rows_per_wg), dim3(threads), lds, s, b);
    };
    for (int i = 0; i < copies; i++) launch(ws[i]);
    LLMI_HIP(hipGetLastError());
    LLMI_HIP(hipStreamSynchronize(s));
    hipGraph_t g;
    hipGraphExec_t ge;
    LLMI_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < reps; i++) launch(ws[i % copies]);
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
    (void)hipGraphExecDestroy(ge);
    (void)hipGraphDestroy(g);
    const double us = ms * 1000.0 / reps;
    printf("%-44s %8.2f us  %7.1f GB/s\n", label, us, one / (us * 1e-6) / 1e9);
    fflush(stdout);
    for (auto& k : ws) {
      (void)hipFree(k.w.qs);
      (void)hipFree(k.w.d);
      if (k.w.kdd) (void)hipFree(k.w.kdd);
      if (k.w.kqh) (void)hipFree(k.w.kqh);
    }
  };
  constexpr int G = LAYER_GELU, Q = LAYER_QUANT;
  // 4B gate_up: 20480 x 2560 (GELU role)
  sweep("q4_0 gate_up slab R8 NW10 P10 PE7 (table)", T_Q4_0, 20480, 2560, 1, G,
        gemv_q4_0_layer<8, 10, 10, 4, G, false, false, 7>, 80, 640);
  sweep("q4_k gate_up row R8 NW10 P10 PE7 (old)", T_Q4_K, 20480, 2560, 0, G,
        gemv_q4_0_layer<8, 10, 10, 4, G, false, false, 7, false, WT_Q4_K>, 80, 640);
  sweep("q4_k gate_up slab R8 NW10 P10 PE7", T_Q4_K, 20480, 2560, 1, G,
        gemv_q4_0_layer<8, 10, 10, 4, G, false, false, 7, false, WT_Q4_K>, 80, 640);
  sweep("q4_k gate_up slab R8 NW10 P10 PE5", T_Q4_K, 20480, 2560, 1, G,
        gemv_q4_0_layer<8, 10, 10, 4, G, false, false, 5, false, WT_Q4_K>, 80, 640);
  sweep("q4_k gate_up slab R8 NW10 P10 PE9", T_Q4_K, 20480, 2560, 1, G,
        gemv_q4_0_layer<8, 10, 10, 4, G, false, false, 9, false, WT_Q4_K>, 80, 640);
  sweep("q4_k gate_up slab R8 NW10 P10 early", T_Q4_K, 20480, 2560, 1, G,
        gemv_q4_0_layer<8, 10, 10, 4, G, false, true, 0, false, WT_Q4_K>, 80, 640);
  sweep("q4_k gate_up slab R8 NW8 P10 E5 PE7", T_Q4_K, 20480, 2560, 1, G,
        gemv_q4_0_layer<8, 8, 10, 5, G, false, false, 7, false, WT_Q4_K>, 64, 512);
  sweep("q4_k gate_up slab R4 NW16 P5 E3 PE3", T_Q4_K, 20480, 2560, 1, G,
        gemv_q4_0_layer<4, 16, 5, 3, G, false, false, 3, false, WT_Q4_K>, 64, 1024);
  sweep("q4_k gate_up row R4 NW16 P5 E3 PE3", T_Q4_K, 20480, 2560, 0, G,
        gemv_q4_0_layer<4, 16, 5, 3, G, false, false, 3, false, WT_Q4_K>, 64, 1024);
  // 4B down: 2560 x 10240 (QUANT role)
  sweep("q4_0 down row R1 NW10 P5 PE3 (table)", T_Q4_0, 2560, 10240, 0, Q,
        gemv_q4_0_layer<1, 10, 5, 2, Q, false, false, 3>, 10, 640);
  sweep("q6_k down row R1 NW10 P5 PE3 (table)", T_Q6_K, 2560, 10240, 0, Q,
        gemv_q4_0_layer<1, 10, 5, 2, Q, false, false, 3, false, WT_Q6_K>, 10, 640);
  sweep("q4_k down row R1 NW10 P5 PE3 (table)", T_Q4_K, 2560, 10240, 0, Q,
        gemv_q4_0_layer<1, 10, 5, 2, Q, false, false, 3, false, WT_Q4_K>, 10, 640);
  sweep("q6_k down row R1 NW10 P5 PE2", T_Q6_K, 2560, 10240, 0, Q,
        gemv_q4_0_layer<1, 10, 5, 2, Q, false, false, 2, false, WT_Q6_K>, 10, 640);
  sweep("q6_k down row R1 NW10 P5 PE4", T_Q6_K, 2560, 10240, 0, Q,
        gemv_q4_0_layer<1, 10, 5, 2, Q, false, false, 4, false, WT_Q6_K>, 10, 640);
  sweep("q6_k down row R1 NW10 P5 early", T_Q6_K, 2560, 10240, 0, Q,
        gemv_q4_0_layer<1, 10, 5, 2, Q, false, true, 0, false, WT_Q6_K>, 10, 640);
  sweep("q6_k down row R2 NW5 P10 E4 PE6", T_Q6_K, 2560, 10240, 0, Q,
        gemv_q4_0_layer<2, 5, 10, 4, Q, false, false, 6, false, WT_Q6_K>, 10, 320);
  sweep("q6_k down row R1 NW8 P5 E3 PE3", T_Q6_K, 2560, 10240, 0, Q,
        gemv_q4_0_layer<1, 8, 5, 3, Q, false, false, 3, false, WT_Q6_K>, 8, 512);
  sweep("q6_k down row R1 NW4 P5 E5 PE3", T_Q6_K, 2560, 10240, 0, Q,
        gemv_q4_0_layer<1, 4, 5, 5, Q, false, false, 3, false, WT_Q6_K>, 4, 256);
  printf("done\n");
  return 0;
}
