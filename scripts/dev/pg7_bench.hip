// Development micro-benchmark of the prefill GEMMs (k_prefill.hip compiled in): the 4B Q4_0 projection shapes at
// T = 512 tokens, random weights / f16 activations, every GEMM v7 geometry (LLMI_PG7) and v6 (LLMI_PG6) and the
// int8 v5 on Q8_0 blocks, 20 launches each timed by events; prints us per launch and TFLOP/s.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -I llm_inference_amd/csrc \
//         scripts/dev/pg7_bench.hip -o scripts/dev/pg7_bench
//   scripts/dev/pg7_bench [geometry ...]   (128x128 ... for v7, v6 or v6:<LLMI_PG6_GEO> for v6, v5)
#include "../../llm_inference_amd/csrc/k_prefill.hip"

namespace llmi {
void dev_free(void* p) { (void)hipFree(p); }
void* dev_alloc(size_t b) {
  void* p = nullptr;
  (void)hipMalloc(&p, b);
  return p;
}
}  // namespace llmi

#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

using namespace llmi;

int main(int argc, char** argv) {
  struct Shape { const char* name; int rows, cols; } shapes[] = {
      {"qkv", 4096, 2560}, {"o", 2560, 2048}, {"gate_up", 20480, 2560}, {"down", 2560, 10240}};
  const int T = 512;
  std::vector<std::string> geos;
  for (int i = 1; i < argc; i++) geos.push_back(argv[i]);
  if (geos.empty()) geos = {"128x128", "128x64", "64x128", "256x128", "128x256", "v6", "v5"};
  std::mt19937 g(7);
  hipStream_t s;
  LLMI_HIP(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  LLMI_HIP(hipEventCreate(&e0));
  LLMI_HIP(hipEventCreate(&e1));
  for (const auto& sh : shapes) {
    const int nb = sh.cols / 32;
    DevWeight w;
    w.type = T_Q4_0;
    w.rows = sh.rows;
    w.cols = sh.cols;
    std::vector<uint8_t> q((size_t)sh.rows * nb * 16);
    std::vector<uint16_t> d((size_t)sh.rows * nb);
    for (auto& b : q) b = (uint8_t)g();
    for (auto& x : d) x = 0x2000 + (g() & 0x3FF);
    LLMI_HIP(hipMalloc(&w.qs, q.size()));
    LLMI_HIP(hipMalloc(&w.d, d.size() * 2));
    LLMI_HIP(hipMemcpy(w.qs, q.data(), q.size(), hipMemcpyHostToDevice));
    LLMI_HIP(hipMemcpy(w.d, d.data(), d.size() * 2, hipMemcpyHostToDevice));
    std::vector<uint16_t> x((size_t)T * sh.cols);
    for (auto& v : x) v = 0x3000 + (g() & 0x7FF) | ((g() & 1) << 15);
    uint16_t* dx;
    LLMI_HIP(hipMalloc(&dx, x.size() * 2));
    LLMI_HIP(hipMemcpy(dx, x.data(), x.size() * 2, hipMemcpyHostToDevice));
    std::vector<XBlock> xb((size_t)T * nb);
    for (auto& b : xb) {
      uint8_t* p = reinterpret_cast<uint8_t*>(&b);
      for (int i = 0; i < 32; i++) p[i] = (uint8_t)g();
      b.d = 0.01f;
      b.nsum8 = 0;
    }
    XBlock* dxb;
    LLMI_HIP(hipMalloc(&dxb, xb.size() * sizeof(XBlock)));
    LLMI_HIP(hipMemcpy(dxb, xb.data(), xb.size() * sizeof(XBlock), hipMemcpyHostToDevice));
    float* out;
    LLMI_HIP(hipMalloc(&out, (size_t)T * sh.rows * 4));
    for (const auto& geo : geos) {
      unsetenv("LLMI_PG6");
      unsetenv("LLMI_PG7");
      unsetenv("LLMI_PG6_GEO");
      if (geo.rfind("v6", 0) == 0) {  // v6 or v6:<LLMI_PG6_GEO>
        setenv("LLMI_PG6", "1", 1);
        if (geo.size() > 3) setenv("LLMI_PG6_GEO", geo.c_str() + 3, 1);
      } else if (geo != "v5") {
        setenv("LLMI_PG7", geo.c_str(), 1);
      }
      auto run = [&]() {
        if (geo == "v5") launch_prefill_gemm(w, dxb, nb, T, out, sh.rows, s);
        else launch_prefill_gemm16(w, dx, sh.cols, T, out, sh.rows, nullptr, s);
      };
      run();
      LLMI_HIP(hipStreamSynchronize(s));
      LLMI_HIP(hipEventRecord(e0, s));
      for (int i = 0; i < 20; i++) run();
      LLMI_HIP(hipEventRecord(e1, s));
      LLMI_HIP(hipEventSynchronize(e1));
      float ms;
      LLMI_HIP(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / 20, fl = 2.0 * sh.rows * (double)sh.cols * T;
      std::printf("%-8s %-9s %8.2f us  %7.1f TFLOP/s\n", sh.name, geo.c_str(), us, fl / us * 1e-6);
    }
    LLMI_HIP(hipFree(w.qs));
    LLMI_HIP(hipFree(w.d));
    LLMI_HIP(hipFree(dx));
    LLMI_HIP(hipFree(dxb));
    LLMI_HIP(hipFree(out));
  }
  return 0;
}
