// f16_sweep.hip -- logits (F16) GEMV variants on the Gemma-3 table shapes
// (development tool).  Launches captured in a hipGraph, each launch on a
// different weight copy so it streams from HBM.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude \
//        scripts/f16_sweep.hip -o scripts/f16_sweep
#include "../llm_inference_amd/csrc/k_gemv.hip"

#include <algorithm>
#include <vector>

using namespace llmi;

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  LLMI_HIP(hipSetDevice(0));
  hipStream_t s;
  LLMI_HIP(hipStreamCreate(&s));
  struct Shape { const char* name; int rows, cols; };
  const Shape shapes[] = {{"4b.logits", 262208, 2560}, {"4b.logits/8", 32776, 2560},
                          {"27b.logits", 262208, 5376}, {"27b.logits/8", 32776, 5376}, {"1b.logits", 262144, 1152}};
  hipEvent_t e0, e1;
  LLMI_HIP(hipEventCreate(&e0));
  LLMI_HIP(hipEventCreate(&e1));
  for (const Shape& sh : shapes) {
    const size_t wbytes = (size_t)sh.rows * sh.cols * 2;
    const int copies = (int)std::max<size_t>(2, (size_t)(1536ull << 20) / wbytes + 1);
    std::vector<uint16_t*> ws(copies);
    for (auto& p : ws) {
      LLMI_HIP(hipMalloc(&p, wbytes + 256));
      LLMI_HIP(hipMemset(p, 0x11, wbytes + 256));
    }
    uint16_t* x;
    LLMI_HIP(hipMalloc(&x, sh.cols * 2 + 256));
    LLMI_HIP(hipMemset(x, 0x22, sh.cols * 2 + 256));
    float* out;
    LLMI_HIP(hipMalloc(&out, (size_t)sh.rows * 4 + 256));
    unsigned long long* key;
    LLMI_HIP(hipMalloc(&key, 64));
    auto timeit = [&](const char* label, auto&& launch) {
      for (int i = 0; i < copies; i++) launch(ws[i % copies]);
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
      printf("%-14s %-40s %9.2f us  %7.1f GB/s\n", sh.name, label, us, wbytes / (us * 1e-6) / 1e9);
      fflush(stdout);
    };
    DevWeight w;
    w.type = T_F16;
    w.rows = sh.rows;
    w.cols = sh.cols;
    ActBuf act{};
    act.x16 = x;
    timeit("launch_gemv (product dispatch)", [&](uint16_t* p) {
      w.qs = p;
      launch_gemv(w, act, out, GEMV_FAST, s, key);
    });
    for (int wv : {2048, 4096, 8192}) {
      char lab[64];
      snprintf(lab, sizeof lab, "pipe, %d waves", wv);
      const int hp = sh.cols / 256;
      timeit(lab, [&](uint16_t* p) {
        const dim3 grid((std::min(sh.rows, wv) + 3) / 4);
        if (sh.cols == 2560) hipLaunchKernelGGL((gemv_f16_rows_pipe<5, 0>), grid, dim3(256), 0, s, (const uint4*)p, sh.rows, (const uint4*)x, out, key);
        if (sh.cols == 5376) hipLaunchKernelGGL((gemv_f16_rows_pipe<10, 32>), grid, dim3(256), 0, s, (const uint4*)p, sh.rows, (const uint4*)x, out, key);
        if (sh.cols == 1152) hipLaunchKernelGGL((gemv_f16_rows_pipe<2, 16>), grid, dim3(256), 0, s, (const uint4*)p, sh.rows, (const uint4*)x, out, key);
      });
    }
    if (sh.cols == 2560)
      timeit("old fast_rows<5> 8192 waves", [&](uint16_t* p) {
        hipLaunchKernelGGL(gemv_f16_fast_rows<5>, dim3(2048), dim3(256), 0, s, (const uint4*)p, sh.rows, (const uint4*)x, out, key);
      });
    for (auto p : ws) (void)hipFree(p);
    (void)hipFree(x);
    (void)hipFree(out);
    (void)hipFree(key);
  }
  printf("done\n");
  return 0;
}
