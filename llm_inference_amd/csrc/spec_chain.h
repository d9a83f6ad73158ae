// spec_chain.h -- the reference's serial sum of squares (rms_norm, ops.cpp:28-43) and its speculative
// parallel form, shared by the exact-order engine (k_exact.hip) and the exact-mode norm launches (k_session.hip).
#pragma once

#include "common.h"

namespace llmi {

// The reference's serial sum of squares (ops.cpp:33-36, contracted to fma by its build) over s[0..n) in LDS.
// Every lane of the calling wave runs the same chain (broadcast reads); the reads of the next 32 values are
// issued before the current 32 are consumed, so the chain is the fma latency alone (~8 cycles a step on
// gfx950, scripts/dev/xl_bench).
__device__ __forceinline__ float xl_chain(const float* s, int n, float sum = 0.0f) {
  const float4* s4 = reinterpret_cast<const float4*>(s);
  const int n4 = n >> 2, nfull = n4 & ~7;
  float4 a[8], b[8];
  if (nfull > 0) {
#pragma unroll
    for (int k = 0; k < 8; k++) a[k] = s4[k];
  }
  for (int i = 0; i < nfull; i += 16) {
    const bool more = i + 8 < nfull;
    if (more) {
#pragma unroll
      for (int k = 0; k < 8; k++) b[k] = s4[i + 8 + k];
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
      sum = fmaf(a[k].x, a[k].x, sum);
      sum = fmaf(a[k].y, a[k].y, sum);
      sum = fmaf(a[k].z, a[k].z, sum);
      sum = fmaf(a[k].w, a[k].w, sum);
    }
    if (!more) break;
    if (i + 16 < nfull) {
#pragma unroll
      for (int k = 0; k < 8; k++) a[k] = s4[i + 16 + k];
    }
#pragma unroll
    for (int k = 0; k < 8; k++) {
      sum = fmaf(b[k].x, b[k].x, sum);
      sum = fmaf(b[k].y, b[k].y, sum);
      sum = fmaf(b[k].z, b[k].z, sum);
      sum = fmaf(b[k].w, b[k].w, sum);
    }
  }
  for (int i = nfull * 4; i < n; i++) sum = fmaf(s[i], s[i], sum);
  return sum;
}

// f64 DPP step (both halves moved by the same row-local control)
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const int lo = dpp_i<CTRL>(__double2loint(v)), hi = dpp_i<CTRL>(__double2hiint(v));
  return __hiloint2double(hi, lo);
}

constexpr int DPP_ROW_SHL4 = 0x104;  // lane i reads lane i + 4 of its 16-lane row

// The boundary walk of the speculative chains (wave 0): the true start of segment k is the chain value after
// segment k - 1; if it is one of the segment's 32 candidates (s_base[k] + c) its end value is that candidate's
// (s_e[k * 32 + c]), otherwise the segment is recomputed serially from it.  The walk over hits is unrolled with
// the end values in registers; the first miss leaves it for a rolled loop with one serial chain in the code
// (round 5: one inlined chain per boundary, 2 x 15 per launch in the 16-segment form, bloated the GEMV kernels)
template <int K>
__device__ __forceinline__ float xl_spec_walk(const float* s, int L, const float* s_e, const int* s_base,
                                              unsigned* fallbacks) {
  const int lane = threadIdx.x & 63;
  float ev[K];
#pragma unroll
  for (int kk = 0; kk < K; kk++) ev[kk] = s_e[kk * 32 + (lane & 31)];
  int bs[K];
#pragma unroll
  for (int kk = 0; kk < K; kk++) bs[kk] = s_base[kk];
  float cur = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(ev[0])));
  int miss = K;
#pragma unroll
  for (int kk = 1; kk < K; kk++) {
    if (miss == K) {
      const int i = __builtin_amdgcn_readfirstlane((int)__float_as_uint(cur) - bs[kk]);
      if (i >= 0 && i < 32) cur = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ev[kk]), i));
      else miss = kk;
    }
  }
#pragma unroll 1
  for (int kk = miss; kk < K; kk++) {  // (rare) from the first miss on: serial where the start is not a candidate
    const int i = __builtin_amdgcn_readfirstlane((int)__float_as_uint(cur) - s_base[kk]);
    if (kk > miss && i >= 0 && i < 32) {
      cur = s_e[kk * 32 + i];
    } else {
      cur = xl_chain(s + kk * L, L, cur);
      if (fallbacks && lane == 0) atomicAdd(fallbacks, 1u);
    }
  }
  return cur;
}

// xl_chain_spec with its fixed costs cut (round 5: 6.4K cycles per 2560-term chain of which the chain is ~2.6K,
// scripts/dev/xl_bench): the segment's f64 sum of squares from float4 loads issued together (not one dependent
// load per step) and reduced on DPP within each 16-lane row plus one cross-row shuffle (not five ds_bpermute
// steps), and every wave walking the boundaries itself (no result broadcast).  n % (8 NW) == 0, n / (8 NW) <= 192
// float4s per segment.  Bit-identical to xl_chain (the sums only place the candidate window).
// NT: the block's threads.  Beyond NW waves (the 1024-thread norm launches) only the first NW waves speculate
// and wave 0 walks, the rest meet the barriers and read the result (16 waves all speculating over 32 segments
// shared each SIMD four ways: 12.4K cycles per chain, scripts/dev/norm_bench).
template <int NW, int NT = NW * 64>
__device__ __forceinline__ float xl_chain_spec_fast(const float* s, int n) {
  constexpr int K = 2 * NW, R = 6;
  constexpr bool ALL = NT == NW * 64;
  __shared__ double s_seg[K];
  __shared__ float s_e[K * 32];
  __shared__ int s_base[K];
  __shared__ float s_res;
  const int t = threadIdx.x, lane = t & 63;
  const bool act = ALL || t < NW * 64;
  const int k = min(t >> 5, K - 1), c = lane & 31, L = n / K, L4 = L / 4;
  float e = 0.0f;
  int base = 0;
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
  __syncthreads();
  if (act) {
    double pre = 0.0;
#pragma unroll
    for (int j = 0; j < K - 1; j++)
      if (j < k) pre += s_seg[j];
    base = k == 0 ? 0 : max(0, (int)__float_as_uint((float)pre) - 16);
    const float x0 = k == 0 ? 0.0f : __uint_as_float((uint32_t)(base + c));
    e = xl_chain(s + k * L, L, x0);
    s_e[k * 32 + c] = e;
    if (c == 0) s_base[k] = base;
  }
  __syncthreads();
  if constexpr (ALL) {
    const float res = xl_spec_walk<K>(s, L, s_e, s_base, nullptr);
    __syncthreads();  // the LDS words are reused by the next call
    return res;
  } else {
    if (t < 64) {
      const float res = xl_spec_walk<K>(s, L, s_e, s_base, nullptr);
      if (t == 0) s_res = res;
    }
    __syncthreads();
    const float res = s_res;
    __syncthreads();  // the LDS words are reused by the next call
    return res;
  }
}

}  // namespace llmi
