// O^T = V^T P^T with V^T from ds_read_b64_tr_b16 and P^T from registers in the 32x32 D layout
// (development tool): V[key][d] = key, P[key][q] = key <= 19 -> every output should be 190
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef __fp16 fp16x4 __attribute__((__vector_size__(4 * sizeof(__fp16))));
__global__ void k(float* out, int variant) {
  __shared__ _Float16 s[32 * 32];
  for (int i = threadIdx.x; i < 32 * 32; i += 64)
    s[i] = variant == 4 ? __builtin_bit_cast(_Float16, (short)((i / 32) * 100 + i % 32)) : (_Float16)(float)(i / 32);
  __syncthreads();
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5, lg = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  f16x8 pb[2];
  for (int reg = 0; reg < 16; reg++) {
    const int key = variant != 1 ? (reg & 3) + 8 * (reg >> 2) + 4 * h : 8 * h + (reg & 7) + 16 * (reg >> 3);
    pb[reg >> 3][reg & 7] = (_Float16)(key <= 19 ? 1.0f : 0.0f);
  }
  v16f o = {};
  for (int kk = 0; kk < 2; kk++) {
    f16x4 vv[2];
    for (int e = 0; e < 2; e++) {
      const int key = variant != 1 ? 16 * kk + 4 * (lg >> 1) + 8 * e + tq : 16 * kk + 8 * (lg >> 1) + 4 * e + tq;
      const int col = 16 * (lg & 1) + 4 * tp;
      vv[e] = __builtin_bit_cast(f16x4, __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) fp16x4*)(s + key * 32 + col)));
    }
    f16x8 vf = __builtin_shufflevector(vv[0], vv[1], 0, 1, 2, 3, 4, 5, 6, 7);
    if (variant == 2)  // A built in registers with variant 0's key order (no LDS)
      for (int j = 0; j < 8; j++) vf[j] = (_Float16)(float)(16 * kk + 4 * h + 8 * (j >> 2) + (j & 3));
    if (variant == 3) {  // print what tr16 delivered to lane 0 / 32
      for (int j = 0; j < 8; j++) out[2048 + kk * 512 + lane * 8 + j] = (float)vf[j];
    }
    if (variant == 4)
      for (int j = 0; j < 8; j++) out[2048 + kk * 512 + lane * 8 + j] = (float)__builtin_bit_cast(short, vf[j]);
    o = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pb[kk], o, 0, 0, 0);
  }
  for (int reg = 0; reg < 16; reg++) out[lane * 16 + reg] = o[reg];
}
int main() {
  float* d;
  hipMalloc(&d, 4096 * 4);
  for (int v = 0; v < 5; v++) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, v);
    static float hbuf[4096];
    hipMemcpy(hbuf, d, 4096 * 4, hipMemcpyDeviceToHost);
    if (v >= 3) {
      for (int l : {0, 1, 16, 32, 33}) {
        printf("tr16 A lane %d kk0: ", l);
        for (int j = 0; j < 8; j++) printf("%g ", hbuf[2048 + l * 8 + j]);
        printf(" kk1: ");
        for (int j = 0; j < 8; j++) printf("%g ", hbuf[2048 + 512 + l * 8 + j]);
        printf("\n");
      }
    }
    printf("variant %d: lane 0: ", v);
    for (int i = 0; i < 16; i++) printf("%g ", hbuf[i]);
    printf("\n   lane 33: ");
    for (int i = 0; i < 16; i++) printf("%g ", hbuf[33 * 16 + i]);
    printf("\n");
  }
  return 0;
}
