// gemv_sweep.hip -- standalone microbenchmark of the Q4_0 decode GEMV variants
// (development tool, not part of the product).  Every timed launch reads a
// different copy of the weight (copies x bytes > the 256 MB MALL), so each
// launch streams from HBM as in a real decode step.
//
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude \
//        scripts/gemv_sweep.hip -o scripts/gemv_sweep
// run:   scripts/gemv_sweep [reps]
#include "../llm_inference_amd/csrc/k_gemv.hip"
#include "../llm_inference_amd/csrc/k_layer.hip"

#include <algorithm>
#include <cstring>
#include <vector>

using namespace llmi;
#ifdef LLMI_LAYER_TRACE
namespace llmi {
void layer_set_trace(unsigned long long* p);
}
#endif

namespace {

__global__ void fill_kernel(uint32_t* p, size_t n, uint32_t seed) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    h ^= h >> 15;
    p[i] = h;
  }
}
__global__ void fill_scales(uint16_t* p, size_t n) {  // small positive f16 scales
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = 0x2000 + (uint16_t)(i & 0xFF);
}

// pure streaming read of the same bytes (qs + d), 16 B per lane per load,
// P loads in flight: the achievable-bandwidth reference for this layout
template <int P>
__global__ __launch_bounds__(256) void stream_kernel(const uint4* __restrict__ q, size_t n16, float* out) {
  uint32_t acc = 0;
  const size_t stride = (size_t)gridDim.x * 256 * P;
  for (size_t base = blockIdx.x * (size_t)256 * P + threadIdx.x; base < n16; base += stride) {
    uint4 v[P];
#pragma unroll
    for (int p = 0; p < P; p++) {
      const size_t i = base + (size_t)p * 256;
      v[p] = i < n16 ? ld_nt(q + i) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int p = 0; p < P; p++) acc ^= v[p].x ^ v[p].y ^ v[p].z ^ v[p].w;
  }
  if (acc == 0x12345678u) out[0] = 1.0f;
}

__global__ void empty_kernel(float* out) {
  if (threadIdx.x == 1023) out[0] = 1.0f;
}

// default-policy (allocating) read of a weight's qs and d: warms the MALL
__global__ __launch_bounds__(256) void prefetch_kernel(const uint4* __restrict__ q, size_t n16,
                                                       const uint4* __restrict__ d, size_t nd16, float* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)256 + threadIdx.x; i < n16 + nd16; i += (size_t)gridDim.x * 256) {
    const uint4 v = i < n16 ? q[i] : d[i - n16];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = 1.0f;
}

struct Shape {
  const char* name;
  int rows, cols;
};

DevWeight alloc_q4(int rows, int cols) {
  DevWeight w;
  w.type = T_Q4_0;
  w.rows = rows;
  w.cols = cols;
  const size_t nblk = (size_t)rows * (cols / 32);
  w.bytes = nblk * 18;
  LLMI_HIP(hipMalloc(&w.qs, nblk * 16 + 64));
  LLMI_HIP(hipMalloc((void**)&w.d, nblk * 2 + 64));
  return w;
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
  const char* only = argc > 2 ? argv[2] : nullptr;  // substring filter on shape names
  LLMI_HIP(hipSetDevice(0));
  hipStream_t s;
  LLMI_HIP(hipStreamCreate(&s));
  const Shape shapes[] = {{"4b.qkv", 4096, 2560}, {"4b.o", 2560, 2048}, {"4b.gate_up", 20480, 2560},
                          {"4b.down", 2560, 10240}, {"1b.gate_up", 13824, 1152}, {"1b.down", 1152, 6912}, {"27b.qkv", 8192, 5376}, {"27b.o", 5376, 4096},
                          {"27b.gate_up", 43008, 5376}, {"27b.down", 5376, 21504}};
  hipEvent_t e0, e1;
  LLMI_HIP(hipEventCreate(&e0));
  LLMI_HIP(hipEventCreate(&e1));
  for (const Shape& sh : shapes) {
    if (only && !strstr(sh.name, only)) continue;
    const size_t wbytes = (size_t)sh.rows * (sh.cols / 32) * 18;
    int copies = (int)std::max<size_t>(2, (size_t)(1536ull << 20) / wbytes + 1);
    // LLMI_SWEEP_COPIES=1: every launch re-reads the same (cache-resident) copy
    if (const char* e = getenv("LLMI_SWEEP_COPIES")) copies = std::max(1, atoi(e));
    std::vector<DevWeight> ws(copies);
    for (int c = 0; c < copies; c++) {
      ws[c] = alloc_q4(sh.rows, sh.cols);
      const size_t nblk = (size_t)sh.rows * (sh.cols / 32);
      hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, s, (uint32_t*)ws[c].qs, nblk * 4, (uint32_t)c);
      hipLaunchKernelGGL(fill_scales, dim3(1024), dim3(256), 0, s, ws[c].d, nblk);
    }
    const int nb = sh.cols / 32;
    XBlock* xb;
    LLMI_HIP(hipMalloc(&xb, (size_t)(nb + 1) * sizeof(XBlock)));
    hipLaunchKernelGGL(fill_kernel, dim3(64), dim3(256), 0, s, (uint32_t*)xb, (size_t)(nb + 1) * 12, 7u);
    float* out = dmalloc_f(sh.rows);
    float* y = dmalloc_f(sh.cols);
    float* r0 = dmalloc_f(sh.cols);
    float* r1 = dmalloc_f(sh.cols);
    float* wn = dmalloc_f(sh.cols);
    float* hid = dmalloc_f(sh.rows);
    XBlock* hq;
    LLMI_HIP(hipMalloc(&hq, (size_t)(sh.rows / 32 + 1) * sizeof(XBlock)));
    LLMI_HIP(hipStreamSynchronize(s));
    ActBuf act{};
    act.q8.xb = xb;
    act.q8.nb = nb;

    // reps launches captured into one hipGraph (device-side cost per launch,
    // including the kernel boundary, without the host launch rate)
    auto timeit = [&](const char* label, auto&& launch) {
      for (int i = 0; i < copies; i++) launch(ws[i % copies]);
      LLMI_HIP(hipStreamSynchronize(s));
      if (getenv("LLMI_SWEEP_EAGER")) {  // for rocprofv3 --pmc: plain launches, no graph
        for (int i = 0; i < 8; i++) launch(ws[i % copies]);
        LLMI_HIP(hipStreamSynchronize(s));
        printf("%-12s %-34s (eager)\n", sh.name, label);
        return;
      }
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
      printf("%-12s %-34s %8.2f us  %7.1f GB/s\n", sh.name, label, us, wbytes / (us * 1e-6) / 1e9);
      fflush(stdout);
    };
    // the layout a table entry reads (the sweep's weights are random: only
    // the addressing differs)
    auto lw = [&](const DevWeight& w, int role) {
      DevWeight x = w;
      x.slab = layer_gemv_slab(w, role);
      return x;
    };
    timeit("empty kernel (1 WG)", [&](const DevWeight&) { hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s, out); });
    timeit("empty kernel (256 WG)", [&](const DevWeight&) { hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(256), 0, s, out); });
    timeit("stream<8> (qs only, 2048 WG)", [&](const DevWeight& w) {
      hipLaunchKernelGGL(stream_kernel<8>, dim3(2048), dim3(256), 0, s, (const uint4*)w.qs,
                         (size_t)sh.rows * nb, out);
    });
    timeit("stream<4> (qs only, 1024 WG)", [&](const DevWeight& w) {
      hipLaunchKernelGGL(stream_kernel<4>, dim3(1024), dim3(256), 0, s, (const uint4*)w.qs,
                         (size_t)sh.rows * nb, out);
    });
    timeit("gemv_q4_0_fast (k_gemv)", [&](const DevWeight& w) { launch_gemv(w, act, out, GEMV_FAST, s); });
    LayerGemv plain;
    plain.xg = xb;
    plain.out = out;
    DevWeight probe = ws[0];
    if (layer_gemv_supported(probe, LAYER_PLAIN))
      timeit("layer plain", [&](const DevWeight& w) { launch_layer_gemv(lw(w, LAYER_PLAIN), plain, LAYER_PLAIN, s); });
    if (layer_gemv_supported(probe, LAYER_PLAIN))
  timeit("layer plain, same weight (cache-hot)", [&](const DevWeight&) { launch_layer_gemv(lw(ws[0], LAYER_PLAIN), plain, LAYER_PLAIN, s); });
    LayerGemv pro;
    pro.y = y;
    pro.resid_in = r0;
    pro.resid_out = r1;
    pro.w_post = wn;
    pro.w_next = wn;
    pro.eps = 1e-6;
    pro.out = out;
    if (layer_gemv_supported(probe, LAYER_PRO))
      timeit("layer pro", [&](const DevWeight& w) { launch_layer_gemv(lw(w, LAYER_PRO), pro, LAYER_PRO, s); });
    LayerGemv gl = pro;
    gl.out = nullptr;
    gl.hid = hid;
    if (layer_gemv_supported(probe, LAYER_GELU))
      timeit("layer pro+gelu", [&](const DevWeight& w) { launch_layer_gemv(lw(w, LAYER_GELU), gl, LAYER_GELU, s); });
    LayerGemv qz;
    qz.y = y;
    qz.out = out;
    if (layer_gemv_supported(probe, LAYER_QUANT))
      timeit("layer quant", [&](const DevWeight& w) { launch_layer_gemv(lw(w, LAYER_QUANT), qz, LAYER_QUANT, s); });
    // MALL experiment: a default-policy prefetch of the same weight right
    // before the GEMV (as a forked graph branch would do during attention)
    {
      auto pre = [&](const DevWeight& w) {
        hipLaunchKernelGGL(prefetch_kernel, dim3(512), dim3(256), 0, s, (const uint4*)w.qs, (size_t)sh.rows * nb,
                           (const uint4*)w.d, (size_t)sh.rows * nb * 2 / 16, out);
      };
      timeit("prefetch only", pre);
      if (layer_gemv_supported(probe, LAYER_PLAIN))
        timeit("prefetch + layer plain", [&](const DevWeight& w) { pre(w); launch_layer_gemv(lw(w, LAYER_PLAIN), plain, LAYER_PLAIN, s); });
      if (layer_gemv_supported(probe, LAYER_GELU))
        timeit("prefetch + layer gelu", [&](const DevWeight& w) { pre(w); launch_layer_gemv(lw(w, LAYER_GELU), gl, LAYER_GELU, s); });
      if (layer_gemv_supported(probe, LAYER_QUANT))
        timeit("prefetch + layer quant", [&](const DevWeight& w) { pre(w); launch_layer_gemv(lw(w, LAYER_QUANT), qz, LAYER_QUANT, s); });
    }
#ifdef LLMI_LAYER_TRACE
    // phase trace of one launch per role (100 MHz ticks, from the first WG start)
    {
      unsigned long long* tr;
      const size_t nslot = 4096 * 8;
      LLMI_HIP(hipMalloc(&tr, nslot * 8));
      std::vector<unsigned long long> h(nslot);
      auto trace = [&](const char* label, auto&& launch) {
        if (!layer_gemv_supported(probe, 0)) {}
        LLMI_HIP(hipMemset(tr, 0, nslot * 8));
        LLMI_HIP(hipStreamSynchronize(s));
        layer_set_trace(tr);
        for (int i = 0; i < 24; i++) launch(ws[i % copies]);  // the last of a back-to-back run is kept
        LLMI_HIP(hipStreamSynchronize(s));
        layer_set_trace(nullptr);
        LLMI_HIP(hipMemcpy(h.data(), tr, nslot * 8, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull, tend = 0;
        int nwg = 0;
        double ph[8] = {0};
        int cnt[8] = {0};
        for (size_t b = 0; b < nslot / 8; b++) {
          if (!h[b * 8]) continue;
          nwg++;
          t0 = std::min(t0, h[b * 8]);
        }
        for (size_t b = 0; b < nslot / 8; b++) {
          if (!h[b * 8]) continue;
          for (int k = 0; k < 7; k++)
            if (h[b * 8 + k]) { ph[k] += (h[b * 8 + k] - t0) / 100.0; cnt[k]++; }
          tend = std::max(tend, h[b * 8 + 6]);
        }
        printf("%-12s trace %-18s wgs=%d span=%.2f us  mean phase times (us):", sh.name, label, nwg, (tend - t0) / 100.0);
        for (int k = 0; k < 7; k++) printf(" p%d=%.2f", k, cnt[k] ? ph[k] / cnt[k] : -1.0);
        printf("\n");
      };
      if (layer_gemv_supported(probe, LAYER_PLAIN)) trace("plain", [&](const DevWeight& w) { launch_layer_gemv(lw(w, LAYER_PLAIN), plain, LAYER_PLAIN, s); });
      if (layer_gemv_supported(probe, LAYER_PRO)) trace("pro", [&](const DevWeight& w) { launch_layer_gemv(lw(w, LAYER_PRO), pro, LAYER_PRO, s); });
      if (layer_gemv_supported(probe, LAYER_GELU)) trace("gelu", [&](const DevWeight& w) { launch_layer_gemv(lw(w, LAYER_GELU), gl, LAYER_GELU, s); });
      if (layer_gemv_supported(probe, LAYER_QUANT)) trace("quant", [&](const DevWeight& w) { launch_layer_gemv(lw(w, LAYER_QUANT), qz, LAYER_QUANT, s); });
      (void)hipFree(tr);
    }
#endif
    // geometry variants of the plain kernel
    const uint32_t mg = div_magic(nb);
    auto geo = [&](const char* label, auto kern, int rows_per_wg, int threads) {
      LayerGemv a = plain;
      a.wd = nullptr;
      timeit(label, [&](const DevWeight& w) {
        a.qs = (const uint4*)w.qs;
        a.wd = w.d;
        a.rows = w.rows;
        a.nb = nb;
        a.magic = mg;
        hipLaunchKernelGGL(kern, dim3((w.rows + rows_per_wg - 1) / rows_per_wg), dim3(threads),
                           (size_t)nb * sizeof(XBlock) + 16, s, a);
      });
    };
    if (nb % 64 == 0) {
      geo("plain R1 NW4 P1", gemv_q4_0_layer<1, 4, 1, 4, 0, true, true>, 4, 256);
      geo("plain R1 NW8 P1", gemv_q4_0_layer<1, 8, 1, 4, 0, true, true>, 8, 512);
    }
    if ((4 * nb) % 64 == 0) {
      geo("plain R4 NW4 P5", gemv_q4_0_layer<4, 4, 5, 4, 0, true, true>, 16, 256);
      geo("plain R4 NW2 P5", gemv_q4_0_layer<4, 2, 5, 4, 0, true, true>, 8, 128);
      geo("plain R4 NW1 P5", gemv_q4_0_layer<4, 1, 5, 4, 0, true, true>, 4, 64);
      geo("plain R4 NW8 P5", gemv_q4_0_layer<4, 8, 5, 4, 0, true, true>, 32, 512);
    }
    geo("plain R8 NW4 P5", gemv_q4_0_layer<8, 4, 5, 4, 0, true, true>, 32, 256);
    geo("plain R2 NW4 P5", gemv_q4_0_layer<2, 4, 5, 4, 0, true, true>, 8, 256);
    // role variants: (args, role LDS) with explicit geometry
    auto geo_role = [&](const char* label, auto kern, int rows_per_wg, int threads, LayerGemv a, bool pro_lds) {
      if (sh.rows % rows_per_wg) return;
      timeit(label, [&](const DevWeight& w) {
        a.qs = (const uint4*)w.qs;
        a.wd = w.d;
        a.rows = w.rows;
        a.nb = nb;
        a.magic = mg;
        a.n = sh.cols;
        const size_t lds = (size_t)nb * sizeof(XBlock) + 16 + (pro_lds ? (size_t)sh.cols * 4 : 0);
        hipLaunchKernelGGL(kern, dim3((w.rows + rows_per_wg - 1) / rows_per_wg), dim3(threads), lds, s, a);
      });
    };
    // slab-major layout variants (addressing only: the sweep's weights are random)
    if (nb % 8 == 0) {
      LayerGemv ps = plain, gs = gl, qs2 = qz;
      ps.slab = gs.slab = qs2.slab = 1;
      if (nb == 168) {
        geo_role("SLAB plain R8 NW4 P7 M", gemv_q4_0_layer<8, 4, 7, 4, 0, true, true>, 32, 256, ps, false);
        geo_role("SLAB plain R4 NW8 P6 M", gemv_q4_0_layer<4, 8, 6, 2, 0, true, true>, 32, 512, ps, false);
        geo_role("SLAB gelu R8 NW8 P7 E11 M", gemv_q4_0_layer<8, 8, 7, 11, 2, true, false>, 64, 512, gs, true);
        geo_role("SLAB gelu R8 NW8 P4 E11 M", gemv_q4_0_layer<8, 8, 4, 11, 2, true, false>, 64, 512, gs, true);
      }
      if (nb == 672) {
        geo_role("SLAB quant R1 NW8 P6 E6 M late", gemv_q4_0_layer<1, 8, 6, 6, 3, true, false>, 8, 512, qs2, false);
        geo_role("SLAB plain R1 NW8 P6 M", gemv_q4_0_layer<1, 8, 6, 4, 0, true, true>, 8, 512, ps, false);
        geo_role("SLAB plain R2 NW4 P5", gemv_q4_0_layer<2, 4, 5, 4, 0, true, true>, 8, 256, ps, false);
      }
      if (nb == 80) {
        geo_role("SLAB plain R4 NW4 P5 (4b table)", gemv_q4_0_layer<4, 4, 5, 1, 0, false, true>, 16, 256, ps, false);
        geo_role("SLAB plain R8 NW4 P5", gemv_q4_0_layer<8, 4, 5, 4, 0, true, true>, 32, 256, ps, false);
      }
      if (nb == 320) {
        geo_role("SLAB quant R1 NW10 P5 (4b table)", gemv_q4_0_layer<1, 10, 5, 2, 3, false, true>, 10, 640, qs2, false);
        geo_role("SLAB plain R1 NW4 P5 M", gemv_q4_0_layer<1, 4, 5, 4, 0, true, true>, 4, 256, ps, false);
      }
    }
    if (nb == 80) {  // 4B gate_up / qkv (x 2560)
      LayerGemv gs = gl, ps = pro;
      gs.slab = ps.slab = 1;
      geo_role("gelu R5 NW16 P7 E3 (table, flat)", gemv_q4_0_layer<5, 16, 7, 3, 2, false, false>, 80, 1024, gl, true);
      geo_role("gelu R8 NW10 P10 E4", gemv_q4_0_layer<8, 10, 10, 4, 2, false, false>, 80, 640, gl, true);
      geo_role("gelu R8 NW10 P10 E4 early", gemv_q4_0_layer<8, 10, 10, 4, 2, false, true>, 80, 640, gl, true);
      geo_role("gelu R8 NW8 P10 E5", gemv_q4_0_layer<8, 8, 10, 5, 2, false, false>, 64, 512, gl, true);
      geo_role("gelu R4 NW16 P5 E3", gemv_q4_0_layer<4, 16, 5, 3, 2, false, false>, 64, 1024, gl, true);
      geo_role("gelu R8 NW5 P10 E8", gemv_q4_0_layer<8, 5, 10, 8, 2, false, false>, 40, 320, gl, true);
      geo_role("SLAB gelu R8 NW10 P10 E4", gemv_q4_0_layer<8, 10, 10, 4, 2, false, false>, 80, 640, gs, true);
      geo_role("SLAB gelu R8 NW10 P10 E4 PE1", gemv_q4_0_layer<8, 10, 10, 4, 2, false, false, 1>, 80, 640, gs, true);
      geo_role("SLAB gelu R8 NW10 P10 E4 PE2", gemv_q4_0_layer<8, 10, 10, 4, 2, false, false, 2>, 80, 640, gs, true);
      geo_role("SLAB gelu R8 NW10 P10 E4 PE3", gemv_q4_0_layer<8, 10, 10, 4, 2, false, false, 3>, 80, 640, gs, true);
      geo_role("SLAB gelu R8 NW10 P10 E4 PE5", gemv_q4_0_layer<8, 10, 10, 4, 2, false, false, 5>, 80, 640, gs, true);
      geo_role("SLAB gelu R8 NW10 P10 E4 PE7", gemv_q4_0_layer<8, 10, 10, 4, 2, false, false, 7>, 80, 640, gs, true);
      geo_role("SLAB gelu R8 NW10 P10 E4 PE6", gemv_q4_0_layer<8, 10, 10, 4, 2, false, false, 6>, 80, 640, gs, true);
      geo_role("SLAB gelu R8 NW10 P10 E4 PE8", gemv_q4_0_layer<8, 10, 10, 4, 2, false, false, 8>, 80, 640, gs, true);
      geo_role("SLAB gelu R4 NW8 P5 E5 (H16) PE3", gemv_q4_0_layer<4, 8, 5, 5, 2, false, false, 3>, 32, 512, gs, true);
      geo_role("SLAB gelu R4 NW8 P5 E5 (H16) PE4", gemv_q4_0_layer<4, 8, 5, 5, 2, false, false, 4>, 32, 512, gs, true);
      geo_role("SLAB gelu R8 NW8 P10 E5 PE7", gemv_q4_0_layer<8, 8, 10, 5, 2, false, false, 7>, 64, 512, gs, true);
      geo_role("SLAB gelu R8 NW5 P10 E8 PE7", gemv_q4_0_layer<8, 5, 10, 8, 2, false, false, 7>, 40, 320, gs, true);
      geo_role("SLAB gelu R4 NW16 P5 E3 PE3", gemv_q4_0_layer<4, 16, 5, 3, 2, false, false, 3>, 64, 1024, gs, true);
      geo_role("SLAB gelu R8 NW10 P10 E4 PE9", gemv_q4_0_layer<8, 10, 10, 4, 2, false, false, 9>, 80, 640, gs, true);
      geo_role("SLAB gelu R8 NW10 P10 E4 early", gemv_q4_0_layer<8, 10, 10, 4, 2, false, true>, 80, 640, gs, true);
      geo_role("SLAB gelu R8 NW10 P10 E4 again", gemv_q4_0_layer<8, 10, 10, 4, 2, false, false>, 80, 640, gs, true);
      geo_role("SLAB gelu R4 NW4 P5 E10 (H8)", gemv_q4_0_layer<4, 4, 5, 10, 2, false, false>, 16, 256, gs, true);
      geo_role("SLAB gelu R4 NW4 P5 E10 (H8) early", gemv_q4_0_layer<4, 4, 5, 10, 2, false, true>, 16, 256, gs, true);
      geo_role("SLAB gelu R8 NW4 P10 E10 (H16)", gemv_q4_0_layer<8, 4, 10, 10, 2, false, false>, 32, 256, gs, true);
      geo_role("SLAB gelu R8 NW4 P10 E10 (H16) early", gemv_q4_0_layer<8, 4, 10, 10, 2, false, true>, 32, 256, gs, true);
      geo_role("SLAB gelu R4 NW8 P5 E5 (H16)", gemv_q4_0_layer<4, 8, 5, 5, 2, false, false>, 32, 512, gs, true);
      geo_role("SLAB plain R8 NW10 P10", gemv_q4_0_layer<8, 10, 10, 1, 0, false, true>, 80, 640, [&] { LayerGemv g = plain; g.slab = 1; return g; }(), false);
      geo_role("SLAB gelu R8 NW10 P10 H1", gemv_q4_0_layer<8, 10, 10, 1, 5, false, true>, 80, 704, gs, true);
      geo_role("SLAB gelu R8 NW10 P10 H2", gemv_q4_0_layer<8, 10, 10, 2, 5, false, true>, 80, 768, gs, true);
      geo_role("gelu R8 NW10 P10 H2", gemv_q4_0_layer<8, 10, 10, 2, 5, false, true>, 80, 768, gl, true);
      geo_role("SLAB gelu R8 NW5 P10 H2", gemv_q4_0_layer<8, 5, 10, 2, 5, false, true>, 40, 448, gs, true);
      geo_role("pro R4 NW4 P5 H1", gemv_q4_0_layer<4, 4, 5, 1, 4, false, true>, 16, 320, pro, true);
      geo_role("pro R4 NW4 P5 H2", gemv_q4_0_layer<4, 4, 5, 2, 4, false, true>, 16, 384, pro, true);
      geo_role("pro R8 NW4 P10 H2", gemv_q4_0_layer<8, 4, 10, 2, 4, false, true>, 32, 384, pro, true);
      geo_role("SLAB gelu R8 NW8 P10 E5", gemv_q4_0_layer<8, 8, 10, 5, 2, false, false>, 64, 512, gs, true);
      geo_role("SLAB gelu R4 NW16 P5 E3", gemv_q4_0_layer<4, 16, 5, 3, 2, false, false>, 64, 1024, gs, true);
      geo_role("pro R4 NW4 P5 E10 (table)", gemv_q4_0_layer<4, 4, 5, 10, 1, false, true>, 16, 256, pro, true);
      geo_role("pro R4 NW4 P5 E10 late", gemv_q4_0_layer<4, 4, 5, 10, 1, false, false>, 16, 256, pro, true);
      geo_role("pro R4 NW4 P5 E10 PE2", gemv_q4_0_layer<4, 4, 5, 10, 1, false, false, 2>, 16, 256, pro, true);
      geo_role("pro R4 NW4 P5 E10 PE3", gemv_q4_0_layer<4, 4, 5, 10, 1, false, false, 3>, 16, 256, pro, true);
      geo_role("pro R4 NW4 P5 E10 PE4", gemv_q4_0_layer<4, 4, 5, 10, 1, false, false, 4>, 16, 256, pro, true);
      geo_role("pro R8 NW2 P10 E20", gemv_q4_0_layer<8, 2, 10, 20, 1, false, true>, 16, 128, pro, true);
      geo_role("pro R2 NW8 P3 E5", gemv_q4_0_layer<2, 8, 3, 5, 1, false, true>, 16, 512, pro, true);
      geo_role("pro R4 NW8 P5 E5", gemv_q4_0_layer<4, 8, 5, 5, 1, false, true>, 32, 512, pro, true);
      geo_role("SLAB pro R4 NW4 P5 E10", gemv_q4_0_layer<4, 4, 5, 10, 1, false, true>, 16, 256, ps, true);
      geo_role("SLAB pro R8 NW2 P10 E20", gemv_q4_0_layer<8, 2, 10, 20, 1, false, true>, 16, 128, ps, true);
    }
    if (nb == 36) {  // 1B gate_up (x 1152)
      geo_role("1b gelu R6 NW9 P4 E2 (table, flat)", gemv_q4_0_layer<6, 9, 4, 2, 2, false, false>, 54, 576, gl, true);
      geo_role("1b gelu R8 NW8 P5 E3", gemv_q4_0_layer<8, 8, 5, 3, 2, false, false>, 64, 512, gl, true);
      geo_role("1b gelu R8 NW8 P5 E3 PE2", gemv_q4_0_layer<8, 8, 5, 3, 2, false, false, 2>, 64, 512, gl, true);
      geo_role("1b gelu R8 NW8 P5 E3 PE3", gemv_q4_0_layer<8, 8, 5, 3, 2, false, false, 3>, 64, 512, gl, true);
      geo_role("1b gelu R8 NW8 P5 E3 PE4", gemv_q4_0_layer<8, 8, 5, 3, 2, false, false, 4>, 64, 512, gl, true);
      geo_role("1b gelu R6 NW9 P4 E2 again", gemv_q4_0_layer<6, 9, 4, 2, 2, false, false>, 54, 576, gl, true);
    }
    if (nb == 216) {  // 1B down (x 6912)
      geo_role("1b quant R2 NW2 P7 E7 (table)", gemv_q4_0_layer<2, 2, 7, 7, 3, false, true>, 4, 128, qz, false);
      geo_role("1b quant R2 NW2 P7 E7 late", gemv_q4_0_layer<2, 2, 7, 7, 3, false, false>, 4, 128, qz, false);
      geo_role("1b quant R2 NW2 P7 E7 PE3", gemv_q4_0_layer<2, 2, 7, 7, 3, false, false, 3>, 4, 128, qz, false);
      geo_role("1b quant R2 NW2 P7 E7 PE5", gemv_q4_0_layer<2, 2, 7, 7, 3, false, false, 5>, 4, 128, qz, false);
      geo_role("1b quant R1 NW4 P4 E4", gemv_q4_0_layer<1, 4, 4, 4, 3, false, true>, 4, 256, qz, false);
      geo_role("1b quant R1 NW4 P4 E4 PE2", gemv_q4_0_layer<1, 4, 4, 4, 3, false, false, 2>, 4, 256, qz, false);
      geo_role("1b quant R2 NW2 P7 E7 (table) b", gemv_q4_0_layer<2, 2, 7, 7, 3, false, true>, 4, 128, qz, false);
    }
    if (nb == 320) {  // 4B down (x 10240)
      geo_role("quant R1 NW10 P5 E2 (table)", gemv_q4_0_layer<1, 10, 5, 2, 3, false, true>, 10, 640, qz, false);
      geo_role("quant R1 NW10 P5 E2 late", gemv_q4_0_layer<1, 10, 5, 2, 3, false, false>, 10, 640, qz, false);
      geo_role("quant R1 NW10 P5 E2 PE1", gemv_q4_0_layer<1, 10, 5, 2, 3, false, false, 1>, 10, 640, qz, false);
      geo_role("quant R1 NW10 P5 E2 PE2", gemv_q4_0_layer<1, 10, 5, 2, 3, false, false, 2>, 10, 640, qz, false);
      geo_role("quant R1 NW10 P5 E2 PE3", gemv_q4_0_layer<1, 10, 5, 2, 3, false, false, 3>, 10, 640, qz, false);
      geo_role("quant R1 NW10 P5 E2 PE4", gemv_q4_0_layer<1, 10, 5, 2, 3, false, false, 4>, 10, 640, qz, false);
      geo_role("quant R1 NW4 P5 E5", gemv_q4_0_layer<1, 4, 5, 5, 3, false, true>, 4, 256, qz, false);
      geo_role("quant R1 NW4 P5 E5 PE3", gemv_q4_0_layer<1, 4, 5, 5, 3, false, false, 3>, 4, 256, qz, false);
      geo_role("quant R1 NW8 P5 E3 PE3", gemv_q4_0_layer<1, 8, 5, 3, 3, false, false, 3>, 8, 512, qz, false);
      geo_role("quant R1 NW5 P5 E4 PE3", gemv_q4_0_layer<1, 5, 5, 4, 3, false, false, 3>, 5, 320, qz, false);
      geo_role("quant R2 NW5 P10 E4 PE6", gemv_q4_0_layer<2, 5, 10, 4, 3, false, false, 6>, 10, 320, qz, false);
      geo_role("quant R1 NW10 P5 E2 PE3 b", gemv_q4_0_layer<1, 10, 5, 2, 3, false, false, 3>, 10, 640, qz, false);
      geo_role("quant R1 NW10 P5 E2 (table) b", gemv_q4_0_layer<1, 10, 5, 2, 3, false, true>, 10, 640, qz, false);
      geo_role("quant R1 NW8 P5 E3", gemv_q4_0_layer<1, 8, 5, 3, 3, false, true>, 8, 512, qz, false);
      geo_role("quant R2 NW5 P10 E4", gemv_q4_0_layer<2, 5, 10, 4, 3, false, true>, 10, 320, qz, false);
      geo_role("quant R2 NW8 P10 E3", gemv_q4_0_layer<2, 8, 10, 3, 3, false, true>, 16, 512, qz, false);
      geo_role("quant R1 NW16 P5 E2", gemv_q4_0_layer<1, 16, 5, 2, 3, false, true>, 16, 1024, qz, false);
    }
    if (nb == 168) {  // 27B PRO (qkv) variants
      LayerGemv ps = pro;
      ps.slab = 1;
      geo_role("pro R4 NW8 P6 E11 M (table)", gemv_q4_0_layer<4, 8, 6, 11, 1, true, true>, 32, 512, pro, true);
      geo_role("pro R4 NW8 P6 E11 M late", gemv_q4_0_layer<4, 8, 6, 11, 1, true, false>, 32, 512, pro, true);
      geo_role("SLAB pro R4 NW8 P6 E11 M", gemv_q4_0_layer<4, 8, 6, 11, 1, true, true>, 32, 512, ps, true);
      geo_role("SLAB pro R4 NW8 P6 H4 M", gemv_q4_0_layer<4, 8, 6, 4, 4, true, true>, 32, 768, ps, true);
      geo_role("SLAB gelu R8 NW8 P4 H4 M", gemv_q4_0_layer<8, 8, 4, 4, 5, true, true>, 64, 768, [&] { LayerGemv g = gl; g.slab = 1; return g; }(), true);
      geo_role("SLAB gelu R8 NW8 P4 H7 M", gemv_q4_0_layer<8, 8, 4, 7, 5, true, true>, 64, 960, [&] { LayerGemv g = gl; g.slab = 1; return g; }(), true);
      geo_role("SLAB pro R8 NW4 P7 E21 M", gemv_q4_0_layer<8, 4, 7, 21, 1, true, true>, 32, 256, ps, true);
      geo_role("SLAB pro R8 NW8 P4 E11 M", gemv_q4_0_layer<8, 8, 4, 11, 1, true, true>, 64, 512, ps, true);
      geo_role("SLAB pro R8 NW8 P4 E11 M late", gemv_q4_0_layer<8, 8, 4, 11, 1, true, false>, 64, 512, ps, true);
      geo_role("SLAB pro R8 NW4 P4 E21 M", gemv_q4_0_layer<8, 4, 4, 21, 1, true, true>, 32, 256, ps, true);
      geo_role("SLAB gelu R8 NW8 P4 E11 M early", gemv_q4_0_layer<8, 8, 4, 11, 2, true, true>, 64, 512, [&] { LayerGemv g = gl; g.slab = 1; return g; }(), true);
      geo_role("SLAB gelu R8 NW4 P4 E21 M", gemv_q4_0_layer<8, 4, 4, 21, 2, true, false>, 32, 256, [&] { LayerGemv g = gl; g.slab = 1; return g; }(), true);
      geo_role("SLAB plain R8 NW4 P4 M", gemv_q4_0_layer<8, 4, 4, 2, 0, true, true>, 32, 256, [&] { LayerGemv g = plain; g.slab = 1; return g; }(), false);
    }
    if (nb == 128) {  // 27B o (x 4096)
      LayerGemv ps = plain;
      ps.slab = 1;
      geo_role("plain R1 NW8 P2 E1 (table)", gemv_q4_0_layer<1, 8, 2, 1, 0, false, true>, 8, 512, plain, false);
      geo_role("plain R1 NW4 P2 E2", gemv_q4_0_layer<1, 4, 2, 2, 0, false, true>, 4, 256, plain, false);
      geo_role("plain R2 NW4 P4 E2", gemv_q4_0_layer<2, 4, 4, 2, 0, false, true>, 8, 256, plain, false);
      geo_role("plain R4 NW4 P8 E2", gemv_q4_0_layer<4, 4, 8, 2, 0, false, true>, 16, 256, plain, false);
      geo_role("SLAB plain R4 NW4 P8 E2", gemv_q4_0_layer<4, 4, 8, 2, 0, false, true>, 16, 256, ps, false);
      geo_role("SLAB plain R8 NW4 P8 M", gemv_q4_0_layer<8, 4, 8, 2, 0, true, true>, 32, 256, ps, false);
      geo_role("SLAB plain R8 NW2 P8 M", gemv_q4_0_layer<8, 2, 8, 3, 0, true, true>, 16, 128, ps, false);
    }
    if (nb == 168) {  // 27B gate_up / qkv (x 5376)
      geo_role("gelu R8 NW8 P7 E11 M (table)", gemv_q4_0_layer<8, 8, 7, 11, 2, true, false>, 64, 512, gl, true);
      geo_role("gelu R8 NW8 P7 E11 M early", gemv_q4_0_layer<8, 8, 7, 11, 2, true, true>, 64, 512, gl, true);
      geo_role("gelu R4 NW8 P6 E11 M", gemv_q4_0_layer<4, 8, 6, 11, 2, true, false>, 32, 512, gl, true);
      geo_role("gelu R8 NW4 P7 E21 M", gemv_q4_0_layer<8, 4, 7, 21, 2, true, false>, 32, 256, gl, true);
      geo_role("gelu R8 NW8 P4 E11 M", gemv_q4_0_layer<8, 8, 4, 11, 2, true, false>, 64, 512, gl, true);
      geo_role("gelu R8 NW8 P11 E11 M", gemv_q4_0_layer<8, 8, 11, 11, 2, true, false>, 64, 512, gl, true);
      geo_role("gelu R16 NW8 P7 E11 M", gemv_q4_0_layer<16, 8, 7, 11, 2, true, false>, 128, 512, gl, true);
      geo_role("plain R8 NW8 P7 M", gemv_q4_0_layer<8, 8, 7, 2, 0, true, true>, 64, 512, plain, false);
      geo_role("plain R4 NW8 P6 M", gemv_q4_0_layer<4, 8, 6, 2, 0, true, true>, 32, 512, plain, false);
      geo_role("plain R2 NW8 P6 M", gemv_q4_0_layer<2, 8, 6, 2, 0, true, true>, 16, 512, plain, false);
      geo_role("plain R8 NW4 P7 M", gemv_q4_0_layer<8, 4, 7, 4, 0, true, true>, 32, 256, plain, false);
    }
    if (nb == 672) {  // 27B down (x 21504)
      geo_role("quant R1 NW8 P6 E6 M (table)", gemv_q4_0_layer<1, 8, 6, 6, 3, true, true>, 8, 512, qz, false);
      geo_role("quant R1 NW8 P6 E6 M late", gemv_q4_0_layer<1, 8, 6, 6, 3, true, false>, 8, 512, qz, false);
      geo_role("quant R2 NW8 P6 E6 M", gemv_q4_0_layer<2, 8, 6, 6, 3, true, true>, 16, 512, qz, false);
      geo_role("quant R1 NW4 P6 E11 M", gemv_q4_0_layer<1, 4, 6, 11, 3, true, true>, 4, 256, qz, false);
      geo_role("quant R1 NW8 P11 E6 M", gemv_q4_0_layer<1, 8, 11, 6, 3, true, true>, 8, 512, qz, false);
      geo_role("quant R1 NW16 P6 E3 M", gemv_q4_0_layer<1, 16, 6, 3, 3, true, true>, 16, 1024, qz, false);
      geo_role("plain R1 NW8 P6 M", gemv_q4_0_layer<1, 8, 6, 4, 0, true, true>, 8, 512, plain, false);
      geo_role("plain R2 NW8 P6 M", gemv_q4_0_layer<2, 8, 6, 8, 0, true, true>, 16, 512, plain, false);
    }
    for (auto& w : ws) {
      (void)hipFree(w.qs);
      (void)hipFree(w.d);
    }
    (void)hipFree(xb);
    (void)hipFree(out);
    (void)hipFree(y);
    (void)hipFree(r0);
    (void)hipFree(r1);
    (void)hipFree(wn);
    (void)hipFree(hid);
    (void)hipFree(hq);
  }
  printf("done\n");
  return 0;
}
