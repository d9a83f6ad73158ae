// realloc_repro.hip -- plain-HIP probe of DESIGN.md section 7's "memory read wrong on its first use" signature
// (round 5, causes 2 and 4: a reallocated block read wrong once, right afterwards).  Hypothesis under test: a
// stale line in one XCD's L2 (the 8 XCDs' L2s are not coherent with each other) survives a rewrite of the
// memory that does not pass through that L2 -- a DMA copy (hipMemcpyAsync H2D) or another XCD's kernel -- and the
// next kernel on that XCD reads the old bytes.
//
// Per trial: a buffer (1 MiB: resident in every XCD's 4 MiB L2) is filled with pattern A and read by every XCD
// (work-groups dealt round-robin over the XCDs, each WG reading the whole buffer: the lines land in all 8 L2s);
// then it is rewritten with pattern B by one of
//   0: hipMemcpyAsync host -> device on the stream (DMA)
//   1: hipMemcpy host -> device (synchronous, null stream)
//   2: a kernel whose work-groups run on one XCD only (blockIdx 0 of a 1-WG grid)
//   3: hipFree + hipMalloc (same size) + hipMemcpyAsync H2D
// and read again by every XCD, twice: mismatching words of the first and the second read are counted per XCD.
//
//   hipcc --offload-arch=gfx950 -O2 -o scripts/dev/realloc_repro scripts/dev/realloc_repro.hip
//   scripts/dev/realloc_repro [trials]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

constexpr int kWords = 1 << 18;  // 1 MiB
constexpr int kXcd = 8;

__device__ __forceinline__ uint32_t pat(uint32_t i, uint32_t seed) { return (i * 2654435761u) ^ seed; }

// every work-group reads the whole buffer; WG b runs on XCD b % 8 (round-robin dealing); counts mismatches
__global__ void read_all(const uint32_t* __restrict__ buf, uint32_t seed, unsigned long long* bad) {
  unsigned n = 0;
  for (int i = threadIdx.x; i < kWords; i += blockDim.x) n += buf[i] != pat(i, seed) ? 1u : 0u;
  for (int o = 32; o >= 1; o >>= 1) n += __shfl_xor(n, o);
  if ((threadIdx.x & 63) == 0 && n) atomicAdd(bad + (blockIdx.x % kXcd), (unsigned long long)n);
}

__global__ void write_all(uint32_t* buf, uint32_t seed) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kWords; i += gridDim.x * blockDim.x) buf[i] = pat(i, seed);
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? std::atoi(argv[1]) : 20;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned long long* bad;
  CK(hipMalloc(&bad, 2 * kXcd * sizeof(unsigned long long)));
  std::vector<uint32_t> host(kWords);
  const char* names[] = {"memcpyAsync H2D", "memcpy H2D (sync)", "kernel on one XCD", "free+malloc+memcpyAsync"};
  for (int mode = 0; mode < 4; mode++) {
    unsigned long long tot[2] = {0, 0}, first_trial = 0;
    for (int tr = 0; tr < trials; tr++) {
      uint32_t* buf;
      CK(hipMalloc(&buf, kWords * 4));
      const uint32_t sa = 0x1234567u + tr * 77u, sb = 0xABCDEF1u + tr * 131u;
      hipLaunchKernelGGL(write_all, dim3(64), dim3(256), 0, s, buf, sa);
      CK(hipMemsetAsync(bad, 0, 2 * kXcd * sizeof(unsigned long long), s));
      hipLaunchKernelGGL(read_all, dim3(64), dim3(256), 0, s, buf, sa, bad);  // lines of A in every L2
      hipLaunchKernelGGL(read_all, dim3(64), dim3(256), 0, s, buf, sa, bad);
      CK(hipStreamSynchronize(s));
      for (int i = 0; i < kWords; i++) host[i] = (i * 2654435761u) ^ sb;
      if (mode == 0) {
        CK(hipMemcpyAsync(buf, host.data(), kWords * 4, hipMemcpyHostToDevice, s));
      } else if (mode == 1) {
        CK(hipMemcpy(buf, host.data(), kWords * 4, hipMemcpyHostToDevice));
      } else if (mode == 2) {
        hipLaunchKernelGGL(write_all, dim3(1), dim3(1024), 0, s, buf, sb);
      } else {
        CK(hipStreamSynchronize(s));
        CK(hipFree(buf));
        CK(hipMalloc(&buf, kWords * 4));
        CK(hipMemcpyAsync(buf, host.data(), kWords * 4, hipMemcpyHostToDevice, s));
      }
      CK(hipMemsetAsync(bad, 0, 2 * kXcd * sizeof(unsigned long long), s));
      hipLaunchKernelGGL(read_all, dim3(64), dim3(256), 0, s, buf, sb, bad);
      hipLaunchKernelGGL(read_all, dim3(64), dim3(256), 0, s, buf, sb, bad + kXcd);
      CK(hipStreamSynchronize(s));
      unsigned long long h[2 * kXcd];
      CK(hipMemcpy(h, bad, sizeof(h), hipMemcpyDeviceToHost));
      for (int x = 0; x < kXcd; x++) {
        tot[0] += h[x];
        tot[1] += h[kXcd + x];
      }
      if (h[0] + h[1] + h[2] + h[3] + h[4] + h[5] + h[6] + h[7] && !first_trial) first_trial = tr + 1;
      CK(hipFree(buf));
    }
    std::printf("%-26s trials %d: mismatching words, first read after the rewrite %llu, second read %llu%s\n",
                names[mode], trials, tot[0], tot[1], first_trial ? " (STALE READS)" : "");
  }
  return 0;
}
