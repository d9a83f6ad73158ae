// Development: dependent-chain latency of the exact accumulator's instruction pairs on one wave (s_memtime cycles
// per step): v_fma_mix_f32 + v_cvt_f16_f32, and alternatives.
// build: hipcc --offload-arch=gfx950 -O3 scripts/dev/lat_check.hip -o scripts/dev/lat_check
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void chain_mix(unsigned* out, float e, unsigned v0, long long* cyc) {
  uint32_t acc = threadIdx.x, v = v0 + threadIdx.x;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 1024; i++) {
    asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]\n\tv_cvt_f16_f32_e32 %0, %0" : "+v"(acc) : "v"(v), "v"(e));
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void chain_fma(unsigned* out, float e, unsigned v0, long long* cyc) {
  float acc = threadIdx.x, v = (float)v0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 1024; i++) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(v), "v"(e));
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = __float_as_uint(acc);
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void chain_cvt(unsigned* out, float e, unsigned v0, long long* cyc) {
  uint32_t acc = threadIdx.x;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 1024; i++) asm volatile("v_cvt_f32_f16_e32 %0, %0\n\tv_cvt_f16_f32_e32 %0, %0" : "+v"(acc));
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}
__global__ void chain_mixlo(unsigned* out, float e, unsigned v0, long long* cyc) {
  uint32_t acc = threadIdx.x, v = v0 + threadIdx.x;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 1024; i++) asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(acc) : "v"(v), "v"(e));
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

__device__ __forceinline__ void mad8(uint32_t& acc, const uint32_t* v, const float* e) {
  asm volatile(
      "v_fma_mix_f32 %0, %1, %9, %0 op_sel_hi:[1,0,1]\n\tv_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %2, %10, %0 op_sel_hi:[1,0,1]\n\tv_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %3, %11, %0 op_sel_hi:[1,0,1]\n\tv_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %4, %12, %0 op_sel_hi:[1,0,1]\n\tv_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %5, %13, %0 op_sel_hi:[1,0,1]\n\tv_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %6, %14, %0 op_sel_hi:[1,0,1]\n\tv_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %7, %15, %0 op_sel_hi:[1,0,1]\n\tv_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %8, %16, %0 op_sel_hi:[1,0,1]\n\tv_cvt_f16_f32_e32 %0, %0"
      : "+v"(acc)
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]), "v"(e[0]), "v"(e[1]),
        "v"(e[2]), "v"(e[3]), "v"(e[4]), "v"(e[5]), "v"(e[6]), "v"(e[7]));
}
// the accumulate kernel's fast-path loop alone: per 32-key batch a broadcast s_up read, 8 float4 e reads from LDS,
// 4 x mad8 on register V values; 19 batches (600 keys), timed on wave 0
__global__ __launch_bounds__(320) void batch_loop(unsigned* out, long long* cyc, int nb, int nwaves_work) {
  __shared__ __attribute__((aligned(16))) float s_e[1024];
  __shared__ uint32_t s_up[32];
  const int t = threadIdx.x;
  for (int i = t; i < 1024; i += 320) s_e[i] = 0.5f + i * 1e-4f;
  if (t < 32) s_up[t] = 0;
  __syncthreads();
  uint32_t va[32];
  for (int u = 0; u < 32; u++) va[u] = 0x3c00u + u + t;
  uint32_t v16 = t;
  const long long t0 = __builtin_amdgcn_s_memtime();
  if ((t >> 6) < nwaves_work) {
    for (int j0 = 0; j0 < nb * 32; j0 += 32) {
      const uint32_t up = __builtin_amdgcn_readfirstlane(s_up[j0 >> 5]);
      float e[32];
#pragma unroll
      for (int u4 = 0; u4 < 8; u4++) {
        const float4 q = reinterpret_cast<const float4*>(s_e + j0)[u4];
        e[4 * u4] = q.x; e[4 * u4 + 1] = q.y; e[4 * u4 + 2] = q.z; e[4 * u4 + 3] = q.w;
      }
      if (up == 0) {
        uint32_t acc = v16;
#pragma unroll
        for (int u = 0; u < 32; u += 8) mad8(acc, va + u, e + u);
        v16 = acc & 0xFFFF;
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[t] = v16;
  if (t == 0) cyc[0] = t1 - t0;
}

int main() {
  unsigned* o;
  long long* c;
  hipMalloc(&o, 512 * 4);
  hipMalloc(&c, 8);
  auto run = [&](const char* n, void (*k)(unsigned*, float, unsigned, long long*)) {
    long long h = 0;
    for (int r = 0; r < 3; r++) {
      hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o, 0.5f, 0x3c00u, c);
      hipDeviceSynchronize();
    }
    hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    std::printf("%-28s %6.1f cycles per step\n", n, h / 1024.0);
  };
  run("fma_mix + cvt_f16 (pair)", chain_mix);
  run("fma_mix alone", chain_mixlo);
  run("cvt_f32_f16 + cvt_f16_f32", chain_cvt);
  run("v_fma_f32", chain_fma);
  for (int nw : {1, 5}) {
    long long h = 0;
    for (int r = 0; r < 3; r++) {
      hipLaunchKernelGGL(batch_loop, dim3(1), dim3(320), 0, 0, o, c, 19, nw);
      hipDeviceSynchronize();
    }
    hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    std::printf("batch loop, %d working waves: %6.1f cycles per batch of 32 keys\n", nw, h / 19.0);
  }
  return 0;
}
