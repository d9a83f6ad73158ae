// Checks the lane maps of __builtin_amdgcn_mfma_i32_32x32x32_i8 on gfx950 with
// asymmetric integer data (development tool for k_prefill.hip).
// Assumed: lane l (r = l & 31, h = l >> 5) holds A[r][16h + j] and B[16h + j][r],
// j = 0..15 (bytes of two 64-bit halves); D: col = l & 31,
// row = (reg & 3) + 8 (reg >> 2) + 4 (l >> 5).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef long v2l __attribute__((ext_vector_type(2)));

__global__ void k(const signed char* A, const signed char* B, int* D) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  signed char a[16], b[16];
  for (int j = 0; j < 16; j++) {
    a[j] = A[r * 32 + 16 * h + j];     // A[row r][k]
    b[j] = B[(16 * h + j) * 32 + r];   // B[k][col r]
  }
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  v16i c = {};
  v16i d = __builtin_amdgcn_mfma_i32_32x32x32_i8(av, bv, c, 0, 0, 0);
  for (int reg = 0; reg < 16; reg++) {
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h, col = r;
    D[row * 32 + col] = d[reg];
  }
}

int main() {
  signed char hA[1024], hB[1024];
  for (int i = 0; i < 32; i++)
    for (int kk = 0; kk < 32; kk++) {
      hA[i * 32 + kk] = (signed char)((i * 7 + kk * 3) % 17 - 8);
      hB[kk * 32 + i] = (signed char)((i * 5 + kk * 11 + 3) % 23 - 11);
    }
  signed char *dA, *dB;
  int* dD;
  hipMalloc(&dA, 1024);
  hipMalloc(&dB, 1024);
  hipMalloc(&dD, 4096);
  hipMemcpy(dA, hA, 1024, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, 1024, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
  int hD[1024];
  hipMemcpy(hD, dD, 4096, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 32; i++)
    for (int j = 0; j < 32; j++) {
      int s = 0;
      for (int kk = 0; kk < 32; kk++) s += hA[i * 32 + kk] * hB[kk * 32 + j];
      if (s != hD[i * 32 + j]) bad++;
    }
  printf("mfma_i32_32x32x32_i8 lane map: %s (%d mismatches)\n", bad ? "WRONG" : "OK", bad);
  return bad ? 1 : 0;
}
