// graph_wrap_repro.cpp -- development: does rocprofv3 --kernel-trace abort a
// plain HIP program that replays a captured hipGraph the way the session's
// token loop does (one small input kernel, one graph of ~100 kernel nodes, a
// stream sync; repeated until the AQL queue has wrapped several times)?
// Nothing of libllmi is used.
//
// build: hipcc --offload-arch=gfx950 -O2 scripts/dev/graph_wrap_repro.cpp -o scripts/dev/graph_wrap_repro
// run:   scripts/dev/graph_wrap_repro [nodes] [replays] [sync_every]   (sync_every 0: one sync at the end)
//        rocprofv3 --kernel-trace --stats -d gpurun_out/repro -o run -- scripts/dev/graph_wrap_repro [nodes] [replays]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

__global__ void set_input(int* d, int v) {
  if (threadIdx.x == 0) d[0] = v;
}
__global__ void step(int* d, int k) {  // a dependent chain, like the layers
  if (blockIdx.x == 0 && threadIdx.x == 0) d[1 + (k & 63)] += d[0];
}

int main(int argc, char** argv) {
  const int nodes = argc > 1 ? std::atoi(argv[1]) : 108;
  const int replays = argc > 2 ? std::atoi(argv[2]) : 400;
  const int sync_every = argc > 3 ? std::atoi(argv[3]) : 1;
  int* d = nullptr;
  CK(hipMalloc(&d, 4096));
  CK(hipMemset(d, 0, 4096));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < nodes; k++) hipLaunchKernelGGL(step, dim3(256), dim3(256), 0, s, d, k);
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int r = 0; r < replays; r++) {
    hipLaunchKernelGGL(set_input, dim3(1), dim3(64), 0, s, d, r);
    CK(hipGetLastError());
    CK(hipGraphLaunch(ge, s));
    if (sync_every > 0 && (r + 1) % sync_every == 0) CK(hipStreamSynchronize(s));
    if (r % 50 == 0) std::printf("replay %d ok (%d kernel packets so far)\n", r, (r + 1) * (nodes + 1));
  }
  CK(hipStreamSynchronize(s));
  int h[2];
  CK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  std::printf("done: %d replays x %d nodes, d[0] = %d\n", replays, nodes, h[0]);
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipFree(d));
  return 0;
}
