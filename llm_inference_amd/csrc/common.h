// common.h -- shared device/host helpers for the gfx950 decode kernels.
//
// Numerics contract: this library is compiled with -ffp-contract=off; every
// fused multiply-add that the reference's pinned build contracts is written as
// an explicit fmaf() (see oracle/llmi_oracle.c for the CPU statement of the
// same arithmetic).  Kernels named *_exact reproduce the reference's AVX2
// operation order bit-for-bit; *_fast kernels reassociate reductions across a
// wavefront and are checked to a stated tolerance.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>

#include "glibc_math.h"

namespace llmi {

constexpr int WAVE = 64;

// ggml tensor type ids (reference gguf.h:30-46)
enum : uint32_t { T_F32 = 0, T_F16 = 1, T_Q4_0 = 2, T_Q5_0 = 6, T_Q8_0 = 8, T_Q4_K = 12, T_Q6_K = 14, T_BF16 = 30 };

struct hip_error : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define LLMI_HIP(call)                                                                           \
  do {                                                                                           \
    hipError_t e_ = (call);                                                                      \
    if (e_ != hipSuccess)                                                                        \
      throw ::llmi::hip_error(std::string(#call) + ": " + hipGetErrorString(e_) + " @" __FILE__); \
  } while (0)

// ---------------------------------------------------------------------------
// fp16 conversions.  The reference uses ggml's software conversions
// (gguf.cpp:40-95): exact IEEE binary16<->binary32, round-to-nearest-even,
// NaN -> 0x7E00.  gfx950's v_cvt_f16_f32 / v_cvt_f32_f16 give the same bits
// for every non-NaN input (checked by tests/test_hip_ops.py against the
// reference's 65536-entry table and its RNE edge cases); the ggml form is kept
// for the NaN-exact path.
// ---------------------------------------------------------------------------
__device__ __forceinline__ float h2f(uint16_t h) {
  return (float)__builtin_bit_cast(_Float16, h);
}
__device__ __forceinline__ uint16_t f2h(float f) {
  return __builtin_bit_cast(uint16_t, (_Float16)f);
}
__device__ __forceinline__ uint16_t f2h_ggml(float f) {  // gguf.cpp:68-95
  float base = (fabsf(f) * 0x1.0p+112f) * 0x1.0p-110f;
  const uint32_t w = __float_as_uint(f);
  const uint32_t shl1_w = w + w;
  const uint32_t sign = w & 0x80000000u;
  uint32_t bias = shl1_w & 0xFF000000u;
  if (bias < 0x71000000u) bias = 0x71000000u;
  base = __uint_as_float((bias >> 1) + 0x07800000u) + base;
  const uint32_t bits = __float_as_uint(base);
  const uint32_t nonsign = ((bits >> 13) & 0x00007C00u) + (bits & 0x00000FFFu);
  return (uint16_t)((sign >> 16) | (shl1_w > 0xFF000000u ? 0x7E00u : nonsign));
}

// nearest_int with the product fused into the magic add, exactly as the
// reference's compiler emits it (ops.cpp:107-113,135-136: vfmadd132ss).
__device__ __forceinline__ int nearest_int_fma(float a, float b) {
  return (int)(__float_as_uint(fmaf(a, b, 12582912.f)) & 0x007fffffu) - 0x00400000;
}

// GELU(tanh)(x) * u (model.cpp:892-899; no contraction in the reference's
// build of this expression).  EXACT: glibc's own tanhf (glibc_math.h),
// bit-exact with the reference for the same gate/up inputs; fast: the device
// libm's tanhf (ulp-level differences; glibc's correctly-rounded divisions
// cost the fused gate_up epilogue 0.6 us per launch, A/B in DESIGN.md)
template <bool EXACT = false>
__device__ __forceinline__ float gelu_mul1(float x, float u) {
  const float c = __uint_as_float(0x3F4C4229u);  // sqrtf((float)(2.0 / M_PI)) = 0.79788452f
  const float inner = x + ((0.044715f * x) * x) * x;
  return ((0.5f * x) * (1.0f + (EXACT ? llmi_glibc::tanhf(c * inner) : tanhf(c * inner)))) * u;
}

__device__ __forceinline__ int sdot4(int a, int b, int c) { return __builtin_amdgcn_sdot4(a, b, c, false); }

// streamed-once weight loads: non-temporal 16-B global loads (MI355X_MICROARCH
// 'nt-weights': once-read decode weights should not displace L2 lines)
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ld_nt(const uint4* p) {
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ int4 ld_nt(const int4* p) {
  const u32x4_t v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(p));
  return make_int4((int)v.x, (int)v.y, (int)v.z, (int)v.w);
}

__device__ __forceinline__ uint16_t ld_nt16(const uint16_t* p) { return __builtin_nontemporal_load(p); }

// Buffer (SRD) loads: a 32-bit per-lane offset + a wave-uniform SGPR offset
// instead of a 64-bit address per load (fewer VGPRs for long load chains),
// and loads past `bytes` return 0.  The descriptor inputs are made provably
// wave-uniform (readfirstlane) so it lives in SGPRs (guide T8/T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(bytes);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), 0, (int)n,
                                           0x00020000);
}
#ifndef LLMI_WEIGHT_POLICY
#define LLMI_WEIGHT_POLICY 2
#endif
constexpr int BUF_NT = LLMI_WEIGHT_POLICY;  // cache-policy bits of streamed weights: 2 = non-temporal (streamed once)
__device__ __forceinline__ float4 buf_ldf4(__amdgpu_buffer_rsrc_t r, int voff) {  // default policy (re-read data)
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
  return make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
}
__device__ __forceinline__ uint4 buf_ld16(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, BUF_NT);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint16_t buf_ld2(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  return __builtin_amdgcn_raw_buffer_load_b16(r, voff, soff, BUF_NT);
}

// Cross-work-group hand-off primitives.  Counter form (MI355X_MICROARCH
// hand-off table, first row; the split attention's partials): the producer
// stores every handed-off byte write-through (sc1), drains (vmcnt(0)) and one
// lane adds to an agent-scope counter; the consumer learns it from the counter
// and reads the bytes with sc1 loads only.  Granule form: below.
constexpr int BUF_SC1 = 16;  // cache-policy bit: sc1 (bypasses L1; producers' sc1 stores write through)
__device__ __forceinline__ uint4 buf_ld16_sc1(__amdgpu_buffer_rsrc_t r, int voff) {
  const u32x4_t v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, BUF_SC1);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void st_sc1(float* p, float v) {  // write-through store (cross-CU hand-off)
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_sc1(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_sc1(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Data-tagged granules (MI355X_MICROARCH hand-off price list, handoff-1to1;
// cdna_hip_programming.md Guideline 16 R2): each 32-bit word travels as ONE
// 8-byte write-through store {value, tag}; the consumer re-loads it (sc1)
// until the tag is this launch's, so a hand-off costs one store + one load --
// no drain, no counter, no flag.  Tags never repeat for a buffer (the
// launch count + 1, the count advanced once per launch by the launch itself:
// block_count / block_count_done below), and the buffers start zeroed (count
// 0 -> tag 1).
constexpr int BLOCK_SPIN_LIMIT = 1 << 21;  // ~0.1-0.3 s of polls: a wait that never ends is a bug
// a wait that took longer than this (wall clock, 100 MHz ticks) adds 1 to err[1]: how often a hand-off stalls,
// reported by the session (llmi_session_info.block_slow_waits).  Product builds count the merge's ticket wait
// (one thread per merging work-group); the granule loads count only in LLMI_SLOW_WAITS diagnostic builds
// (once per wave) -- any count there reshuffled the attention block's registers and cost it 0.5 %
constexpr uint64_t BLOCK_SLOW_TICKS = 2000;  // 20 us
__device__ __forceinline__ void count_slow_wait(bool slow, int* err) {
  const unsigned long long m = __ballot(slow);
  if (m && (int)(threadIdx.x & 63) == __ffsll((long long)m) - 1)
    __hip_atomic_fetch_add(err + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_granule(uint2* g, uint32_t v, uint32_t tag) {
  st_sc1(reinterpret_cast<uint64_t*>(g), ((uint64_t)tag << 32) | v);
}
// N (1, 2 or 4) consecutive granules at g[off..] (g wave-uniform) -> values;
// bounded: on timeout *err = 1 and the values are garbage (results invalid,
// but the grid drains)
template <int N>
__device__ __forceinline__ void ld_granules(uint32_t (&v)[N], const uint2* g, int off, uint32_t tag, int* err) {
  const __amdgpu_buffer_rsrc_t r = buf_rsrc(g, 1u << 30);
  int n = 0;
#ifdef LLMI_SLOW_WAITS
  uint64_t t0 = 0;
#endif
  for (;;) {
    bool ok;
    if constexpr (N == 4) {
      const uint4 a = buf_ld16_sc1(r, off * 8), b = buf_ld16_sc1(r, off * 8 + 16);
      v[0] = a.x; v[1] = a.z; v[2] = b.x; v[3] = b.z;
      ok = (a.y == tag) & (a.w == tag) & (b.y == tag) & (b.w == tag);
    } else if constexpr (N == 2) {
      const uint4 a = buf_ld16_sc1(r, off * 8);
      v[0] = a.x; v[1] = a.z;
      ok = (a.y == tag) & (a.w == tag);
    } else {
      const uint64_t a = ld_sc1(reinterpret_cast<const uint64_t*>(g + off));
      v[0] = (uint32_t)a;
      ok = (uint32_t)(a >> 32) == tag;
    }
    if (ok) break;
#ifdef LLMI_SLOW_WAITS
    if (n == 0) t0 = wall_clock64();
#endif
    if (++n >= BLOCK_SPIN_LIMIT) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");  // re-load every time
  }
#ifdef LLMI_SLOW_WAITS  // diagnostic builds only: any count here reshuffles the attention block's registers (-0.5 %)
  count_slow_wait(n > 0 && wall_clock64() - t0 > BLOCK_SLOW_TICKS, err);
#endif
}

// The attention block's tag advance (BlockSync::epoch / done / done_n): a counted work-group's thread 0 adds one
// to *done once all of the work-group's waves are past their last use of the tag (block_count, relaxed: the
// tag loads were consumed before; the return is left in flight) and checks the return at its end
// (block_count_done): the add that completes the count resets *done and advances *epoch for the next launch
__device__ __forceinline__ unsigned block_count(unsigned* done) {
  return __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void block_count_done(unsigned old, unsigned n, unsigned* done, unsigned* epoch) {
  if (old == n - 1u) {
    __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_fetch_add(epoch, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// development trace of the block kernels (builds with -DLLMI_BLOCK_TRACE
// only: the runtime test alone costs the layer bodies ~100 VGPRs): phase
// clock of work-group blockIdx.x
#ifdef LLMI_BLOCK_TRACE
#define BLK_MARK(bs, ph)                                                                              \
  do {                                                                                               \
    if ((bs).trace && threadIdx.x == 0) (bs).trace[(size_t)blockIdx.x * 8 + (ph)] = wall_clock64(); \
  } while (0)
#else
#define BLK_MARK(bs, ph) \
  do {                   \
  } while (0)
#endif

// Q4_0 nibbles of 4 packed bytes: low = elements 0..15, high = 16..31 (ops.cpp:334-340)
__device__ __forceinline__ int nib_lo(uint32_t w) { return (int)(w & 0x0F0F0F0Fu); }
__device__ __forceinline__ int nib_hi(uint32_t w) { return (int)((w >> 4) & 0x0F0F0F0Fu); }

// ---------------------------------------------------------------------------
// wave-level reductions (64 lanes) on DPP lane swizzles + readlane, no LDS
// round trips.  Fixed order: quad butterflies, row mirror, row half-mirror
// (every lane of a 16-lane row then holds the row total, bit-identical since
// a+b == b+a), then the four row totals combined as (r0+r1)+(r2+r3).
// Deterministic run to run; call from wave-uniform control flow.
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(dpp_i<CTRL>(__float_as_int(v)));
}
constexpr int DPP_QUAD_1032 = 0xB1, DPP_QUAD_2301 = 0x4E, DPP_ROW_MIRROR = 0x140, DPP_ROW_HALF_MIRROR = 0x141;

__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<DPP_QUAD_1032>(v);
  v += dpp_f<DPP_QUAD_2301>(v);
  v += dpp_f<DPP_ROW_MIRROR>(v);
  v += dpp_f<DPP_ROW_HALF_MIRROR>(v);
  return v;
}
__device__ __forceinline__ float row16_max(float v) {
  v = fmaxf(v, dpp_f<DPP_QUAD_1032>(v));
  v = fmaxf(v, dpp_f<DPP_QUAD_2301>(v));
  v = fmaxf(v, dpp_f<DPP_ROW_MIRROR>(v));
  v = fmaxf(v, dpp_f<DPP_ROW_HALF_MIRROR>(v));
  return v;
}
__device__ __forceinline__ int row16_isum(int v) {
  v += dpp_i<DPP_QUAD_1032>(v);
  v += dpp_i<DPP_QUAD_2301>(v);
  v += dpp_i<DPP_ROW_MIRROR>(v);
  v += dpp_i<DPP_ROW_HALF_MIRROR>(v);
  return v;
}
__device__ __forceinline__ float lane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float wave_sum(float v) {
  v = row16_sum(v);
  return (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
}
__device__ __forceinline__ float wave_max(float v) {
  v = row16_max(v);
  return fmaxf(fmaxf(lane_f(v, 0), lane_f(v, 16)), fmaxf(lane_f(v, 32), lane_f(v, 48)));
}
// 32-lane (half-wave) reductions: each half gets its own total
__device__ __forceinline__ float half_max(float v) {
  v = row16_max(v);
  const float lo = fmaxf(lane_f(v, 0), lane_f(v, 16)), hi = fmaxf(lane_f(v, 32), lane_f(v, 48));
  return (threadIdx.x & 32) ? hi : lo;
}
__device__ __forceinline__ float half_sum(float v) {
  v = row16_sum(v);
  const float lo = lane_f(v, 0) + lane_f(v, 16), hi = lane_f(v, 32) + lane_f(v, 48);
  return (threadIdx.x & 32) ? hi : lo;
}
__device__ __forceinline__ int half_isum(int v) {
  v = row16_isum(v);
  const int lo = __builtin_amdgcn_readlane(v, 0) + __builtin_amdgcn_readlane(v, 16);
  const int hi = __builtin_amdgcn_readlane(v, 32) + __builtin_amdgcn_readlane(v, 48);
  return (threadIdx.x & 32) ? hi : lo;
}

// orderable key for argmax with "first maximal index wins" (std::max_element,
// reference main.cpp:193-194): larger value first, then smaller index.
__device__ __forceinline__ unsigned long long argmax_key(float v, uint32_t idx) {
  uint32_t u = __float_as_uint(v);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((unsigned long long)u << 32) | (0xFFFFFFFFu - idx);
}
__host__ __device__ inline uint32_t argmax_key_index(unsigned long long k) {
  return 0xFFFFFFFFu - (uint32_t)(k & 0xFFFFFFFFull);
}

// One Q8_0 activation block in device layout (BlockQ8_0 of ops.h:89-92,
// restated for 16-B loads): 48 bytes =
//   q[32] int8 | d f32 (= f16(amax/127) widened: exactly the value the
//   reference multiplies with, ops.cpp:380-381) | nsum8 = -8 * sum(q) (the Q4_0
//   zero-point term, so sum((nib-8)*q) = dot4(nib, q) + nsum8) | pad
struct XBlock {
  int4 lo;  // q[0..15]
  int4 hi;  // q[16..31]
  float d;
  int nsum8;
  int pad0, pad1;
};
static_assert(sizeof(XBlock) == 48, "XBlock layout");

struct Q8Act {
  XBlock* xb = nullptr;
  int nb = 0;
};

// quantize_row_q8_0 (ops.cpp:116-139) of one 32-element block held by 32
// consecutive lanes (element = lane & 31), bit-exact: amax (order-free),
// d = amax/127 (IEEE), id = 1/d from the UNROUNDED d, q = nearest_int(fma(x,
// id, 1.5*2^23)), stored scale = f16(d).  Every lane of the 32-lane group must
// execute this (lane swizzles), and the group is a half-wave (lanes 0-31 or
// 32-63); `ok` masks the stores.
struct Q8Lane {  // one element's share of a half-wave's Q8_0 block
  int q;          // its quant
  float d;        // the block's f16-rounded scale
  int nsum8;      // -8 x the block's quant sum
};
__device__ __forceinline__ Q8Lane q8_block_lane(float v) {
  const float amax = half_max(fabsf(v));  // max and integer sum: order-free, exact
  const float dd = amax / 127.0f;
  const float id = dd != 0.0f ? 1.0f / dd : 0.0f;
  const int q = nearest_int_fma(v, id);
  return Q8Lane{q, h2f(f2h_ggml(dd)), -8 * half_isum(q)};
}
__device__ __forceinline__ void q8_block_store(float v, bool ok, XBlock* blk, int e) {
  const Q8Lane b = q8_block_lane(v);
  if (ok) {
    reinterpret_cast<int8_t*>(blk)[e] = (int8_t)b.q;
    if (e == 0) {
      blk->d = b.d;
      blk->nsum8 = b.nsum8;
    }
  }
}

// The same quantization of one block by ONE thread (no cross-lane traffic):
// used where a whole vector is staged in LDS and each thread owns a block.
// Bit-identical to q8_block_store (max and integer sums are order-free).
__device__ __forceinline__ void q8_block_from_regs(const float (&v)[32], XBlock* __restrict__ blk) {
  float amax = 0.0f;
#pragma unroll
  for (int k = 0; k < 32; k++) amax = fmaxf(amax, fabsf(v[k]));
  const float dd = amax / 127.0f;
  const float id = dd != 0.0f ? 1.0f / dd : 0.0f;
  int s = 0;
  uint32_t w[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint32_t pk = 0;
#pragma unroll
    for (int e = 0; e < 4; e++) {
      const int q = nearest_int_fma(v[4 * k + e], id);
      s += q;
      pk |= (uint32_t)(q & 0xFF) << (8 * e);
    }
    w[k] = pk;
  }
  blk->lo = make_int4((int)w[0], (int)w[1], (int)w[2], (int)w[3]);
  blk->hi = make_int4((int)w[4], (int)w[5], (int)w[6], (int)w[7]);
  blk->d = h2f(f2h_ggml(dd));
  blk->nsum8 = -8 * s;
}
__device__ __forceinline__ void q8_block_serial(const float* __restrict__ x32, XBlock* __restrict__ blk) {
  float v[32];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const float4 f = reinterpret_cast<const float4*>(x32)[k];
    v[4 * k] = f.x; v[4 * k + 1] = f.y; v[4 * k + 2] = f.z; v[4 * k + 3] = f.w;
  }
  q8_block_from_regs(v, blk);
}

// The same quantization with a block spread over the 4 lanes of a DPP quad
// (lane & 3 = sub owns elements 8 sub .. 8 sub + 7): quad max / integer sum
// by two DPP steps each.  Bit-identical to q8_block_store (order-free max
// and integer sums).  All 4 lanes of every quad must execute it.
__device__ __forceinline__ void q8_block_quad(const float (&v)[8], int sub, XBlock* __restrict__ blk) {
  float amax = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; k++) amax = fmaxf(amax, fabsf(v[k]));
  amax = fmaxf(amax, dpp_f<DPP_QUAD_1032>(amax));
  amax = fmaxf(amax, dpp_f<DPP_QUAD_2301>(amax));
  const float dd = amax / 127.0f;
  const float id = dd != 0.0f ? 1.0f / dd : 0.0f;
  int s = 0;
  uint32_t w0 = 0, w1 = 0;
#pragma unroll
  for (int e = 0; e < 4; e++) {
    const int q0 = nearest_int_fma(v[e], id), q1 = nearest_int_fma(v[4 + e], id);
    s += q0 + q1;
    w0 |= (uint32_t)(q0 & 0xFF) << (8 * e);
    w1 |= (uint32_t)(q1 & 0xFF) << (8 * e);
  }
  s += dpp_i<DPP_QUAD_1032>(s);
  s += dpp_i<DPP_QUAD_2301>(s);
  reinterpret_cast<uint2*>(blk)[sub] = make_uint2(w0, w1);  // q[8 sub .. 8 sub + 7]
  if (sub == 0) {
    blk->d = h2f(f2h_ggml(dd));
    blk->nsum8 = -8 * s;
  }
}

// quantize_row_q8_k (ops.cpp:142-178) of one 256-element super-block held by a
// half-wave (lanes 0-31 or 32-63), each DPP quad one 32-element block (lane
// & 3 = sub owns elements 8 sub .. 8 sub + 7 of block (lane >> 2) & 7), into
// 8 XBlocks in the K-quant convention: q = the Q8_K quants, d = the
// super-block's d (the same in its 8 blocks), nsum8 = sum of the block's q
// (the reference's bsums of its two 16-groups).  max: the signed value of the
// first element with the largest |x| (strict > scan), as quantize_q8_k_kernel.
// Every lane of the half-wave must execute it.
__device__ __forceinline__ void q8k_block_quad(const float (&v)[8], int sub, XBlock* __restrict__ blk) {
  const int e0 = ((int)(threadIdx.x >> 2) & 7) * 32 + sub * 8;
  // the super-block's max |x| (DPP within each 16-lane row, one swizzle across the two rows), then the first
  // element attaining it and its sign as the min of (index << 1 | sign) -- the reference's first maximal |x|
  float ax = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; k++) ax = fmaxf(ax, fabsf(v[k]));
  ax = row16_max(ax);
  ax = fmaxf(ax, __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(ax), 0x401F)));  // lane ^ 16
  int key = 0x7FFFFFFF;
#pragma unroll
  for (int k = 7; k >= 0; k--)
    if (fabsf(v[k]) == ax) key = ((e0 + k) << 1) | (v[k] < 0.0f ? 1 : 0);
  key = min(key, dpp_i<DPP_QUAD_1032>(key));
  key = min(key, dpp_i<DPP_QUAD_2301>(key));
  key = min(key, dpp_i<DPP_ROW_MIRROR>(key));
  key = min(key, dpp_i<DPP_ROW_HALF_MIRROR>(key));
  key = min(key, __builtin_amdgcn_ds_swizzle(key, 0x401F));
  const float sv = (key & 1) ? -ax : ax;
  uint32_t w0 = 0, w1 = 0;
  int s = 0;
  float d = 0.0f;
  if (ax != 0.0f) {  // ops.cpp:158-163: an all-zero super-block stays 0
    const float iscale = -127.f / sv;
    d = 1.0f / iscale;
#pragma unroll
    for (int e = 0; e < 4; e++) {
      int q0 = nearest_int_fma(iscale, v[e]), q1 = nearest_int_fma(iscale, v[4 + e]);
      q0 = q0 < -128 ? -128 : (q0 > 127 ? 127 : q0);
      q1 = q1 < -128 ? -128 : (q1 > 127 ? 127 : q1);
      s += q0 + q1;
      w0 |= (uint32_t)(q0 & 0xFF) << (8 * e);
      w1 |= (uint32_t)(q1 & 0xFF) << (8 * e);
    }
  }
  s += dpp_i<DPP_QUAD_1032>(s);
  s += dpp_i<DPP_QUAD_2301>(s);
  reinterpret_cast<uint2*>(blk)[sub] = make_uint2(w0, w1);
  if (sub == 0) {
    blk->d = d;
    blk->nsum8 = s;
  }
}

// f / nb by multiply-high for the small f of one wave's chunk; nb == 1 has
// no 32-bit magic and is encoded as 0
__host__ __device__ inline uint32_t div_magic(uint32_t nb) { return nb == 1 ? 0u : (uint32_t)((1ull << 32) / nb + 1); }
__device__ __forceinline__ int div_by_magic(int f, uint32_t magic) {  // branch-free
  return (int)(__umulhi((uint32_t)f, magic) + ((uint32_t)f & (magic ? 0u : 0xFFFFFFFFu)));
}

}  // namespace llmi
