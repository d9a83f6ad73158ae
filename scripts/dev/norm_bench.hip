// Development timing of the one-work-group norm launches (k_session.hip) in exact and fast form, linked against
// the in-tree libllmi.so: launch_residual_norm with the decode loop's final-norm outputs (xn + screening blocks).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I llm_inference_amd/csrc scripts/dev/norm_bench.hip \
//        -L llm_inference_amd -lllmi -Wl,-rpath,'$ORIGIN/../../llm_inference_amd' -o scripts/dev/norm_bench
#include <cstdio>
#include <random>
#include <vector>

#include "session_kernels.h"
#include "spec_chain.h"

using namespace llmi;

static float* rnd(int n, std::mt19937& g) {
  std::normal_distribution<float> N(0.0f, 1.0f);
  std::vector<float> h(n);
  for (auto& x : h) x = N(g);
  float* d;
  LLMI_HIP(hipMalloc(&d, n * 4 + 64));
  LLMI_HIP(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

__device__ unsigned long long g_ph[8];
#define PH(i) do { if (threadIdx.x == 0) g_ph[i] = __builtin_amdgcn_s_memtime(); } while (0)
// xl_chain_spec_fast<NW, NT> with phase stamps (development copy of spec_chain.h)
template <int NW, int NT>
__device__ float spec_fast_traced(const float* s, int n) {
  constexpr int K = 2 * NW, R = 6;
  constexpr bool ALL = NT == NW * 64;
  __shared__ double s_seg[K];
  __shared__ float s_e[K * 32];
  __shared__ int s_base[K];
  __shared__ float s_res;
  const int t = threadIdx.x, lane = t & 63;
  const bool act = ALL || t < NW * 64;
  const int k = min(t >> 5, K - 1), c = lane & 31, L = n / K, L4 = L / 4;
  PH(0);
  if (act) {
    const float4* s4 = reinterpret_cast<const float4*>(s + k * L);
    float4 v[R];
#pragma unroll
    for (int r = 0; r < R; r++) v[r] = s4[min(c + 32 * r, L4 - 1)];
    double p0 = 0.0, p1 = 0.0;
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (c + 32 * r < L4) {
        const double x = v[r].x, y = v[r].y, z = v[r].z, w = v[r].w;
        p0 = fma(x, x, fma(y, y, p0));
        p1 = fma(z, z, fma(w, w, p1));
      }
    }
    double p = p0 + p1;
    p += dpp_d<DPP_QUAD_1032>(p);
    p += dpp_d<DPP_QUAD_2301>(p);
    p += dpp_d<DPP_ROW_MIRROR>(p);
    p += dpp_d<DPP_ROW_HALF_MIRROR>(p);
    p += __shfl_xor(p, 16);
    if (c == 0) s_seg[k] = p;
  }
  PH(1);
  __syncthreads();
  PH(2);
  if (act) {
    double pre = 0.0;
#pragma unroll
    for (int j = 0; j < K - 1; j++)
      if (j < k) pre += s_seg[j];
    const int base = k == 0 ? 0 : max(0, (int)__float_as_uint((float)pre) - 16);
    const float x0 = k == 0 ? 0.0f : __uint_as_float((uint32_t)(base + c));
    PH(3);
    const float e = xl_chain(s + k * L, L, x0);
    PH(4);
    s_e[k * 32 + c] = e;
    if (c == 0) s_base[k] = base;
  }
  __syncthreads();
  PH(5);
  if (t < 64) {
    const float res = xl_spec_walk<K>(s, L, s_e, s_base, nullptr);
    if (t == 0) s_res = res;
  }
  PH(6);
  __syncthreads();
  PH(7);
  return s_res;
}
__device__ unsigned long long g_cyc[4];
__device__ float g_res[4];
template <int V>
__global__ __launch_bounds__(1024) void chain_kernel(const float* x, int n) {
  extern __shared__ float s_h[];
  for (int i = threadIdx.x; i < n; i += 1024) s_h[i] = x[i];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  float r;
  if (V == 0) r = xl_chain_spec_fast<4, 1024>(s_h, n);
  else if (V == 2) r = spec_fast_traced<4, 1024>(s_h, n);
  else {
    __shared__ float s_r;
    if (threadIdx.x == 0) {
      float sum = 0.0f;
      for (int i = 0; i < n; i++) sum = fmaf(s_h[i], s_h[i], sum);
      s_r = sum;
    }
    __syncthreads();
    r = s_r;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { g_cyc[V] = t1 - t0; g_res[V] = r; }
}

int main() {
  std::mt19937 g(3);
  const int n = 2560;
  float *y = rnd(n, g), *r = rnd(n, g), *wp = rnd(n, g), *wn = rnd(n, g), *xn = rnd(n, g);
  ScreenX* scr;
  unsigned* mk;
  LLMI_HIP(hipMalloc(&scr, (n / 32 + 1) * sizeof(ScreenX)));
  LLMI_HIP(hipMalloc(&mk, 64));
  for (int variant = 0; variant < 4; variant++) {
    const bool exact = variant & 1, with_scr = variant & 2;
    NormOut o;
    o.xn = xn;
    if (with_scr) {
      o.scr = scr;
      o.scr_mkey = mk;
    }
    hipEvent_t e0, e1;
    LLMI_HIP(hipEventCreate(&e0));
    LLMI_HIP(hipEventCreate(&e1));
    for (int i = 0; i < 3; i++) launch_residual_norm(y, wp, r, wn, o, n, 1e-6, exact, 0);
    LLMI_HIP(hipDeviceSynchronize());
    LLMI_HIP(hipEventRecord(e0, 0));
    for (int i = 0; i < 50; i++) launch_residual_norm(y, wp, r, wn, o, n, 1e-6, exact, 0);
    LLMI_HIP(hipEventRecord(e1, 0));
    LLMI_HIP(hipEventSynchronize(e1));
    float ms = 0;
    LLMI_HIP(hipEventElapsedTime(&ms, e0, e1));
    std::printf("residual_norm %-5s %-14s %8.2f us/launch\n", exact ? "exact" : "fast", with_scr ? "xn + screening" : "xn",
                ms * 1000.0 / 50);
  }
  hipLaunchKernelGGL(chain_kernel<0>, dim3(1), dim3(1024), n * 4, 0, y, n);
  hipLaunchKernelGGL(chain_kernel<1>, dim3(1), dim3(1024), n * 4, 0, y, n);
  hipLaunchKernelGGL(chain_kernel<2>, dim3(1), dim3(1024), n * 4, 0, y, n);
  LLMI_HIP(hipDeviceSynchronize());
  unsigned long long ph[8];
  LLMI_HIP(hipMemcpyFromSymbol(ph, HIP_SYMBOL(g_ph), sizeof ph));
  std::printf("spec_fast<4, 1024> phases (cycles from start):");
  for (int i = 1; i < 8; i++) std::printf(" %d:%llu", i, ph[i] - ph[0]);
  std::printf("\n");
  unsigned long long c[4];
  float rr[4];
  LLMI_HIP(hipMemcpyFromSymbol(c, HIP_SYMBOL(g_cyc), sizeof c));
  LLMI_HIP(hipMemcpyFromSymbol(rr, HIP_SYMBOL(g_res), sizeof rr));
  std::printf("chain 2560 in a 1024-thread block: spec_fast<4, 1024> %llu cycles, one thread %llu cycles (%s)\n", c[0], c[1],
              rr[0] == rr[1] ? "same bits" : "DIFFERENT");
  return 0;
}
