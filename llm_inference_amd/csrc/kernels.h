// kernels.h -- host-side launchers for the gfx950 decode kernels.
// All launchers are asynchronous on `s` and capture-safe (no allocation, no
// synchronization), so the session can record them into one hipGraph.
#pragma once

#include "common.h"

namespace llmi {

// ---- device weight layouts (repacked once at upload) -------
// Q4_0 : qs [rows][nb][16] B (16-B aligned), d [rows][nb] f16
// Q8_0 : qs [rows][nb][32] B (16-B aligned), d [rows][nb] f16
// F16  : [rows][cols] f16 (cols % 8 == 0 for the vector kernels)
// Q4_K / Q6_K / Q5_0 / BF16 : the GGUF block bytes, unchanged
// Q4_K / Q6_K, kq (fused fast path, to_kq_layout): 32-element sub-blocks u
//   qs  [rows][nsub][16] B  nibbles in the Q4_0 order (byte i: elements i, 16 + i)
//   d   [rows][nsub] u16    Q4_K: 6-bit scale | 6-bit min << 8; Q6_K: int8 scales of elements 0-15 | 16-31 << 8
//   kdd [rows][nsb] u32     Q4_K: f16 d | f16 dmin << 16; Q6_K: f16 d
//   kqh [rows][nsub] 8 B    Q6_K: the high 2 bits, word w of elements 4w + b (b = byte) at bits 8b + 2w
//                           (first dword: elements 0-15, second: 16-31)
struct DevWeight {
  uint32_t type = 0;
  int rows = 0, cols = 0;
  void* qs = nullptr;      // quants (or raw blocks / f16 / bf16 data)
  uint16_t* d = nullptr;   // per-block scales (Q4_0/Q8_0 only; kq: per sub-block scale words)
  size_t bytes = 0;        // algorithmic bytes (GGUF size of the tensor)
  int slab = 0;            // Q4_0 only: 1 = slab-major blocks (to_slab_layout; layer kernels only)
  int kq = 0;              // Q4_K / Q6_K: 1 = the kq layout above (layer kernels only)
  uint32_t* kdd = nullptr;
  uint2* kqh = nullptr;
};

// Activation prepared for a weight type (device scratch):
//   Q8_0 : Q8Act {qs[nb][32], d[nb], nsum8[nb]}
//   Q8_K : raw 292-B blocks (ops.h:98-102)
//   F16  : x rounded to f16 (ops.cpp:542-551)
struct ActBuf {
  Q8Act q8{};
  uint8_t* q8k = nullptr;
  uint16_t* x16 = nullptr;
  const float* xf = nullptr;  // raw f32 x (Q5_0 / BF16 consume it directly)
};

enum GemvMode { GEMV_EXACT = 0, GEMV_FAST = 1 };

// Kernel timing hook (bench): when set, the next instrumented launch on this
// thread records start/stop through hipExtLaunchKernel -- the events are
// signalled by the kernel's own dispatch, so the elapsed time is the kernel's
// duration as rocprofv3 reports it (no launch gap) -- and clears the hook.
struct KernelTiming {
  hipEvent_t start = nullptr, stop = nullptr;
};
KernelTiming& kernel_timing();

// quantizers (bit-exact with ops.cpp:116-178)
void launch_quantize_q8_0(const float* x, int n, Q8Act out, hipStream_t s);
void launch_quantize_q8_k(const float* x, int n, uint8_t* out, hipStream_t s);
void launch_round_f16(const float* x, int n, uint16_t* out, hipStream_t s);

// o[rows] = W x.  For F16 with amax_key != nullptr the kernel also folds a
// first-index argmax over the outputs into *amax_key (must be pre-zeroed).
void launch_gemv(const DevWeight& w, const ActBuf& x, float* o, GemvMode mode, hipStream_t s,
                 unsigned long long* amax_key = nullptr);

// elementwise / norms
// o = rms_norm(x) [* w if w]  per row of n, n_rows rows; exact = serial FMA sum
void launch_rms_norm(const float* x, const float* w, float* o, int n, int n_rows, double eps, bool exact,
                     hipStream_t s);
void launch_softmax(float* x, int n, hipStream_t s);
// NEOX rope on t[n_rows][head_dim] (row r uses table row r / rows_per_pos):
// cs = [n_pos][n_rot/2][2] (cos, sin) precomputed on the host with glibc
void launch_rope(float* t, int n_rows, int head_dim, int n_rot, const float* cs, int rows_per_pos, hipStream_t s);
void launch_scale(float* t, int n, float sc, hipStream_t s);
void launch_vec_scale_f16(uint16_t* y, int n, float v, hipStream_t s);
void launch_vec_mad_f16(uint16_t* y, const uint16_t* x, int n, float v, hipStream_t s);
void launch_gelu_mul(const float* g, const float* u, float* o, int n, hipStream_t s);
void launch_dequantize_rows(uint32_t type, const uint8_t* blocks, size_t row_bytes, const int32_t* row_ids,
                            int n_ids, int n_cols, float scale, float* o, hipStream_t s);

}  // namespace llmi
