// What ds_read_b64_tr_b16 returns per lane on gfx950 (development tool): LDS holds a [16 rows][64 cols]
// u16 image with value row * 100 + col; lane 4q+p of each 16-lane group addresses row q, cols 4p..4p+3
// of a block whose first column is 16 * (group & 1), first row 4 * (group >> 1).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short v4s __attribute__((ext_vector_type(4)));
__global__ void k(short* out, int stride) {
  __shared__ short s[16 * 64];
  for (int i = threadIdx.x; i < 16 * 64; i += 64) s[i] = (short)((i / stride) * 100 + i % stride);
  __syncthreads();
  const int lane = threadIdx.x, g = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  const int row = 4 * (g >> 1) + q, col = 16 * (g & 1) + 4 * p;
  v4s r = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4s*)(s + row * stride + col));
  for (int e = 0; e < 4; e++) out[lane * 4 + e] = r[e];
}
int main() {
  short* d;
  hipMalloc(&d, 256 * 2);
  for (int stride : {64, 32}) {
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, stride);
  short h[256];
  printf("row stride %d elements\n", stride);
  hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
  for (int l = 0; l < 64; l++) printf("lane %2d: %4d %4d %4d %4d%s", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3], l % 4 == 3 ? "\n" : " | ");
  }
  return 0;
}
