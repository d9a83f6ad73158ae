#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
__global__ void k(short* out, int mode) {
  __shared__ short s[32 * 32];
  for (int i = threadIdx.x; i < 32 * 32; i += 64) s[i] = (short)((i / 32) * 100 + i % 32);
  __syncthreads();
  const int lane = threadIdx.x, lg = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;
  const int key = mode == 0 ? 4 * (lg >> 1) + tq : 4 * (lg >> 1) + (lane & 3);
  const int col = mode == 0 ? 16 * (lg & 1) + 4 * tp : 16 * (lg & 1) + 4 * ((lane >> 2) & 3);
  v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(s + key * 32 + col));
  for (int e = 0; e < 4; e++) out[lane * 4 + e] = r[e];
}
int main() {
  short* d;
  hipMalloc(&d, 512);
  for (int m = 0; m < 2; m++) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, m);
    short h[256];
    hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    printf("mode %d\n", m);
    for (int l = 0; l < 20; l++) printf("lane %2d: %4d %4d %4d %4d%s", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3], l % 4 == 3 ? "\n" : " | ");
  }
  return 0;
}
