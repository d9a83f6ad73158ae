// k_exact.hip -- the exact-order engine's Q4_0 GEMVs (exact.h): the
// reference's operation order (ops.cpp:364-399 mat_vec_mul_q4_0, ops.cpp:28-43
// rms_norm, ops.cpp:116-139 quantize_row_q8_0, model.cpp:843-924 residual /
// norm / GELU) with the weights streamed like the fast path's layer GEMVs.
#include <cstdlib>
#include <stdexcept>

#include "exact.h"
#include "glibc_math.h"
#include "spec_chain.h"

namespace llmi {

namespace {

constexpr int XL_P = 8;   // groups (4 blocks each) per chunk of loads

#ifdef XL_TRACE  // development (scripts/dev/xl_bench.hip): per-work-group phase clocks of the last launch
__device__ unsigned long long g_xl_trace[8192 * 8];
#define XL_MARK(ph)                                                                                          \
  do {                                                                                                       \
    const unsigned xl_b_ = blockIdx.y * gridDim.x + blockIdx.x;                                              \
    if (threadIdx.x == 0 && xl_b_ < 8192) g_xl_trace[xl_b_ * 8 + (ph)] = __builtin_amdgcn_s_memtime();      \
  } while (0)
#else
#define XL_MARK(ph) \
  do {              \
  } while (0)
#endif

__device__ __forceinline__ float xl_rms_scale(float sum, int n, double eps) {  // ops.cpp:37-38
  return 1.0f / sqrtf((float)((double)(sum / (float)n) + eps));
}

// The same serial chain, its latency divided by speculation (every work-group thread calls it; the result is
// bit-identical to xl_chain).  The n terms split into K = 2 NW segments of L; half-wave k runs segment k's chain
// from 32 candidate start values at once -- the floats from 16 below to 15 above fl(P_k), P_k the f64 sum of the
// earlier segments' squares (within ~2^-50 of exact, while the float chain's accumulated rounding stays within a
// few ulps: |s - fl(P)| < 16 ulps at ~97.5 % of the boundaries of a 2560-term chain in a CPU simulation of random
// vectors, scripts/dev/spec_chain.c).  Wave 0 then walks the boundaries: the true start of segment k is the chain
// value after segment k - 1; if it is one of the candidates its end value is that lane's, otherwise the segment
// is recomputed serially from it.  Either way every step is the reference's fma on the reference's value.
template <int NW>
__device__ __forceinline__ float xl_chain_spec(const float* s, int n, unsigned* fallbacks = nullptr) {
  constexpr int K = 2 * NW;
  __shared__ double s_seg[K];
  __shared__ float s_e[K * 32];
  __shared__ int s_base[K];
  __shared__ float s_res;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int k = t >> 5, c = lane & 31, L = n / K;
  double p = 0.0;
  for (int i = c; i < L; i += 32) {
    const double v = (double)s[k * L + i];
    p = fma(v, v, p);
  }
#pragma unroll
  for (int m = 16; m >= 1; m >>= 1) p += __shfl_xor(p, m);
  if (c == 0) s_seg[k] = p;
  __syncthreads();
  double pre = 0.0;
  for (int j = 0; j < k; j++) pre += s_seg[j];
  const int base = k == 0 ? 0 : max(0, (int)__float_as_uint((float)pre) - 16);
  const float x0 = k == 0 ? 0.0f : __uint_as_float((uint32_t)(base + c));
  const float e = xl_chain(s + k * L, L, x0);
  s_e[k * 32 + c] = e;
  if (c == 0) s_base[k] = base;
  __syncthreads();
  if (wave == 0) s_res = xl_spec_walk<K>(s, L, s_e, s_base, fallbacks);
  __syncthreads();
  return s_res;
}

// xl_chain for two start values at once over the same terms: two independent dependency chains interleaved, so
// each step's latency is paid once for both (the same fma on the same value as xl_chain, per chain)
__device__ __forceinline__ void xl_chain2(const float* s, int n, float& sa, float& sb) {
  const float4* s4 = reinterpret_cast<const float4*>(s);
  const int n4 = n >> 2;
  float4 a[8], b[8];
  auto ld = [&](float4 (&d)[8], int i) {
#pragma unroll
    for (int k = 0; k < 8; k++) d[k] = s4[min(i + k, n4 - 1)];
  };
  auto eat = [&](const float4 (&d)[8], int i) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      if (i + k >= n4) break;  // wave-uniform
      sa = fmaf(d[k].x, d[k].x, sa);
      sb = fmaf(d[k].x, d[k].x, sb);
      sa = fmaf(d[k].y, d[k].y, sa);
      sb = fmaf(d[k].y, d[k].y, sb);
      sa = fmaf(d[k].z, d[k].z, sa);
      sb = fmaf(d[k].z, d[k].z, sb);
      sa = fmaf(d[k].w, d[k].w, sa);
      sb = fmaf(d[k].w, d[k].w, sb);
    }
  };
  ld(a, 0);
  for (int i = 0; i < n4; i += 16) {
    ld(b, i + 8);
    eat(a, i);
    if (i + 8 >= n4) break;
    ld(a, i + 16);
    eat(b, i + 8);
  }
}

// xl_chain_spec with twice the segments: K = 4 NW segments of n / K terms, a quarter-wave per segment whose lane c
// runs the chains from the candidates base + c and base + 16 + c at once (xl_chain2) -- the same 32-candidate
// window around fl(P_k) as xl_chain_spec, each chain half as long, the two chains of a lane sharing each step's
// latency (round 5: the exact engine's norm chains, 6.6K -> see DESIGN.md section 4.4).  Bit-identical to
// xl_chain: every step is the reference's fma on the reference's value; a boundary whose true start is not a
// candidate runs its segment serially.
template <int NW>
__device__ __forceinline__ float xl_chain_spec2(const float* s, int n, unsigned* fallbacks = nullptr) {
  constexpr int K = 4 * NW;
  __shared__ double s_seg[K];
  __shared__ float s_e[K * 32];
  __shared__ int s_base[K];
  __shared__ float s_res;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int k = t >> 4, c = lane & 15, L = n / K;
  double p = 0.0;
  if (L <= 64) {  // (the attention rows: every load issued before the sums; a 16-lane row on DPP)
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; r++) v[r] = s[k * L + min(c + 16 * r, L - 1)];
#pragma unroll
    for (int r = 0; r < 4; r++)
      if (c + 16 * r < L) p = fma((double)v[r], (double)v[r], p);
    p += dpp_d<DPP_QUAD_1032>(p);
    p += dpp_d<DPP_QUAD_2301>(p);
    p += dpp_d<DPP_ROW_MIRROR>(p);
    p += dpp_d<DPP_ROW_HALF_MIRROR>(p);
  } else {
    for (int i = c; i < L; i += 16) {
      const double v = (double)s[k * L + i];
      p = fma(v, v, p);
    }
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) p += __shfl_xor(p, m);
  }
  if (c == 0) s_seg[k] = p;
  __syncthreads();
  double pre = 0.0;
  for (int j = 0; j < k; j++) pre += s_seg[j];
  const int base = k == 0 ? 0 : max(0, (int)__float_as_uint((float)pre) - 16);
  float ea = k == 0 ? 0.0f : __uint_as_float((uint32_t)(base + c));
  float eb = k == 0 ? 0.0f : __uint_as_float((uint32_t)(base + 16 + c));
  xl_chain2(s + k * L, L, ea, eb);
  s_e[k * 32 + c] = ea;
  s_e[k * 32 + 16 + c] = eb;
  if (c == 0) s_base[k] = base;
  __syncthreads();
  if (wave == 0) s_res = xl_spec_walk<K>(s, L, s_e, s_base, fallbacks);
  __syncthreads();
  return s_res;
}

// the serial chain by the calling work-group: speculative where n splits into 4 NW segments of whole float4s
template <int NW>
__device__ __forceinline__ float xl_sumsq(const float* s, int n, float* s_out) {
  // (xl_chain_spec2 here: 14.40 / 19.94 us for the 4B qkv / gate_up launches vs 13.37 / 18.95 with xl_chain_spec,
  // scripts/dev/xl_bench -- its halved chain is paid back in the 16-segment prefix and walk)
  if (n % (8 * NW) == 0 && n / (8 * NW) <= 192) return xl_chain_spec_fast<NW>(s, n);
  if (n % (8 * NW) == 0) return xl_chain_spec<NW>(s, n);
  if ((threadIdx.x >> 6) == 0) {
    const float v = xl_chain(s, n);
    if ((threadIdx.x & 63) == 0) *s_out = v;
  }
  __syncthreads();
  return *s_out;
}

// The activation of one XL lane: per block b and slot jj, {q[4jj..4jj+3], q[16+4jj..16+4jj+3], -8 sum of the
// first four, -8 sum of the second four} (the Q4_0 zero point folded into the integer dot's accumulator input)
__device__ __forceinline__ int4 xe_entry(const XBlock& xb, int jj) {
  const int lo = reinterpret_cast<const int*>(&xb.lo)[jj], hi = reinterpret_cast<const int*>(&xb.hi)[jj];
  return make_int4(lo, hi, -8 * sdot4(lo, 0x01010101, 0), -8 * sdot4(hi, 0x01010101, 0));
}

struct XlChunk {
  uint4 q[XL_P];
  uint2 d[XL_P];
};

__device__ __forceinline__ void xl_load(XlChunk& c, __amdgpu_buffer_rsrc_t rq, __amdgpu_buffer_rsrc_t rd, int voq,
                                        int vod, int sq, int sd, int g0, int ng) {
#pragma unroll
  for (int p = 0; p < XL_P; p++) {
    const int g = g0 + p;
    const bool in = g < ng;  // groups past the row's end: out of the descriptor's range (0, no traffic)
    c.q[p] = buf_ld16(rq, in ? voq + g * sq : (1 << 30), 0);
    typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
    const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(rd, in ? vod + g * sd : (1 << 30), 0, BUF_NT);
    c.d[p] = make_uint2(v.x, v.y);
  }
}

// one block: the reference's two accumulator updates of slots jj and jj + 4 (ops.cpp:380-395:
// d = f16(w.d) * f16(x.d), acc = fma(d, (float)isum, acc))
__device__ __forceinline__ void xl_block(uint32_t w, uint32_t dw16, const int4 x, float xd, float& lo, float& hi) {
  const int il = sdot4((int)(w & 0x0F0F0F0Fu), x.x, x.z);
  const int ih = sdot4((int)((w >> 4) & 0x0F0F0F0Fu), x.y, x.w);
  const float d = h2f((uint16_t)dw16) * xd;
  lo = fmaf(d, (float)il, lo);
  hi = fmaf(d, (float)ih, hi);
}

__device__ __forceinline__ void xl_eat(const XlChunk& c, int g0, int ng, int jj, const int4* s_xe, const float4* s_xd4,
                                       float& lo, float& hi) {
#pragma unroll
  for (int p = 0; p < XL_P; p++) {
    const int g = g0 + p;
    if (g >= ng) break;  // wave-uniform: the chain skips what the row does not have (no +0 step)
    const float4 xd = s_xd4[g];
    const int4* xe = s_xe + (size_t)g * 16 + jj;
    xl_block(c.q[p].x, c.d[p].x & 0xFFFFu, xe[0], xd.x, lo, hi);
    xl_block(c.q[p].y, c.d[p].x >> 16, xe[4], xd.y, lo, hi);
    xl_block(c.q[p].z, c.d[p].y & 0xFFFFu, xe[8], xd.z, lo, hi);
    xl_block(c.q[p].w, c.d[p].y >> 16, xe[12], xd.w, lo, hi);
  }
}

// one slot per lane (LPR 8): slot jj of the low (sh 0) or high (sh 4) nibbles -- the reference's accumulator jj or
// jj + 4 -- over the row's blocks in order
__device__ __forceinline__ void xl_eat1(const XlChunk& c, int g0, int ng, int jj, int sh, const int4* s_xe,
                                        const float4* s_xd4, float& acc) {
#pragma unroll
  for (int p = 0; p < XL_P; p++) {
    const int g = g0 + p;
    if (g >= ng) break;  // wave-uniform: the chain skips what the row does not have (no +0 step)
    const float4 xd = s_xd4[g];
    const int4* xe = s_xe + (size_t)g * 16 + jj;
    const uint32_t w4[4] = {c.q[p].x, c.q[p].y, c.q[p].z, c.q[p].w};
    const uint32_t d16[4] = {c.d[p].x & 0xFFFFu, c.d[p].x >> 16, c.d[p].y & 0xFFFFu, c.d[p].y >> 16};
    const float xdv[4] = {xd.x, xd.y, xd.z, xd.w};
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const int4 x = xe[4 * b];
      const int is = sdot4((int)((w4[b] >> sh) & 0x0F0F0F0Fu), sh ? x.y : x.x, sh ? x.w : x.z);
      acc = fmaf(h2f((uint16_t)d16[b]) * xdv[b], (float)is, acc);
    }
  }
}

// XL_K4: PRE / GELU float4 of each operand per thread (n <= 4 XL_K4 T); NCH: chunks of XL_P groups in flight;
// LPR: lanes per row -- 4 (lane jj holds the reference's accumulators jj and jj + 4) or 8 (PLAIN: one accumulator
// per lane, twice the waves over the same rows: more of the weight stream in flight for the long down rows)
// SPR (PRE only, 0: off): SPR rows per work-group with the rows' dots split over all lanes and the chains run
// after them (as exact_plain_split_kernel): the qkv launch's 64 work-groups of 64 rows left 192 CUs idle in
// its GEMV phase
template <int NW, int ROLE, int XL_K4, int NCH, int LPR = 4, int SPR = 0>
__global__ __launch_bounds__(NW * 64) void exact_gemv_kernel(const uint4* __restrict__ wq, const uint2* __restrict__ wd,
                                                             int rows, int nb, XlArgs a) {
  extern __shared__ int4 s_dyn[];
  int4* s_xe = s_dyn;                                                // [nb][4]
  float* s_xd = reinterpret_cast<float*>(s_dyn + (size_t)nb * 4);    // [nb]
  float* s_a = s_xd + nb;                                            // PRE: [n] y, then the XBlocks
  float* s_b = s_a + a.n;                                            // PRE: [n] h
  __shared__ float s_scale[2];
  __shared__ float s_rows[NW * 16];
  static_assert(LPR == 4 || (LPR == 8 && ROLE == XL_PLAIN), "8 lanes per row: the PLAIN role");
  constexpr int T = NW * 64, RPW = 64 / LPR;  // rows per wave
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int rl = lane / LPR, jl = lane % LPR, jj = jl & 3;
  const int row = (blockIdx.x * NW + wave) * RPW + rl;
  const int ng = nb >> 2;
  // weight stream: issued first, the activation prologue runs while it is in flight
  const __amdgpu_buffer_rsrc_t rq = buf_rsrc(wq, (uint32_t)((size_t)ng * rows * 64));
  const __amdgpu_buffer_rsrc_t rd = buf_rsrc(wd, (uint32_t)((size_t)ng * rows * 8));
  const bool row_ok = row < rows;
  const int voq = row_ok ? (row * 4 + jj) * 16 : (1 << 30), vod = row_ok ? row * 8 : (1 << 30);
  const int sq = rows * 64, sd = rows * 8;
  XL_MARK(0);
  // the weight stream is issued right AFTER the activation operands' first loads: loads return in issue order, so
  // operands issued behind 32 KB per wave of weights waited for them (round 5: the operands-in-LDS phase of the
  // PRE / GELU roles 3.2-3.9K cycles; scripts/dev/xl_bench)
  static_assert(SPR == 0 || (ROLE == XL_PRE && NW == 4 && SPR * 8 % 64 == 0 && (SPR & (SPR - 1)) == 0), "SPR: PRE");
  constexpr int SIPL = SPR ? (SPR * 4 * (XL_K4 * T / 32) + T - 1) / T : 1;  // split items per lane (ng <= XL_K4 T / 32)
  XlChunk ck[SPR ? 1 : NCH];
  uint4 sq4[SIPL];
  uint2 sd2[SIPL];
  const int srow0 = blockIdx.x * (SPR ? SPR : 1);
  auto issue_w = [&]() {
    if constexpr (SPR > 0) {  // item i = t + T m: slot jj = i % 4, row R = (i / 4) % SPR, group g = i / (4 SPR)
#pragma unroll
      for (int m = 0; m < SIPL; m++) {
        const int i = t + T * m, jj4 = i & 3, R = (i >> 2) & (SPR - 1), g = i / (4 * SPR);
        const bool in = g < ng;
        sq4[m] = buf_ld16(rq, in ? ((g * rows + srow0 + R) * 4 + jj4) * 16 : (1 << 30), 0);
        typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
        const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(rd, in && jj4 == 0 ? (g * rows + srow0 + R) * 8 : (1 << 30), 0, BUF_NT);
        sd2[m] = make_uint2(v.x, v.y);
      }
    } else {
#pragma unroll
      for (int k = 0; k < NCH; k++) xl_load(ck[k], rq, rd, voq, vod, sq, sd, k * XL_P, ng);
    }
  };

  // ---- the activation: XE entries + scales in LDS.  Every global operand a thread needs is loaded in one
  // batch before any is used (a load per loop trip would pay one memory latency per trip) ----
  if constexpr (ROLE == XL_PLAIN) {
    const uint4* xg = reinterpret_cast<const uint4*>(a.xb);  // 3 uint4 per XBlock
    for (int b0 = 0; b0 < nb; b0 += 4 * T) {
      uint4 lo[4], hi[4];
      float d[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int b = min(b0 + k * T + t, nb - 1);
        lo[k] = xg[3 * b];
        hi[k] = xg[3 * b + 1];
        d[k] = __uint_as_float(xg[3 * b + 2].x);
      }
      if (b0 == 0) issue_w();
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int b = b0 + k * T + t;
        if (b < nb) {
          const uint32_t l4[4] = {lo[k].x, lo[k].y, lo[k].z, lo[k].w}, h4[4] = {hi[k].x, hi[k].y, hi[k].z, hi[k].w};
#pragma unroll
          for (int j = 0; j < 4; j++)
            s_xe[b * 4 + j] = make_int4((int)l4[j], (int)h4[j], -8 * sdot4((int)l4[j], 0x01010101, 0),
                                        -8 * sdot4((int)h4[j], 0x01010101, 0));
          s_xd[b] = d[k];
        }
      }
    }
  } else {
    const int n = a.n, n4 = n >> 2;
    XBlock* s_xb = reinterpret_cast<XBlock*>(s_a);
    float4* s_a4 = reinterpret_cast<float4*>(s_a);
    float4* s_b4 = reinterpret_cast<float4*>(s_b);
    if constexpr (ROLE == XL_QUANT) {
      const float4* y4 = reinterpret_cast<const float4*>(a.y);
      for (int i0 = 0; i0 < n4; i0 += 8 * T) {
        float4 v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = y4[min(i0 + k * T + t, n4 - 1)];
        if (i0 == 0) issue_w();
#pragma unroll
        for (int k = 0; k < 8; k++)
          if (i0 + k * T + t < n4) s_b4[i0 + k * T + t] = v[k];
      }
      __syncthreads();
      // quantize_row_q8_0 (ops.cpp:116-139): a DPP quad per block, then the XE entries
      for (int q0 = 0; q0 < nb * 4; q0 += T) {
        const int qi = q0 + t, b = qi >> 2, sub = qi & 3;
        if (b < nb) {  // whole quads (the quad's DPP steps stay inside it)
          float v[8];
#pragma unroll
          for (int k = 0; k < 8; k++) v[k] = s_b[b * 32 + sub * 8 + k];
          q8_block_quad(v, sub, s_xb + b);
        }
      }
      __syncthreads();
      for (int i = t; i < nb * 4; i += T) {
        s_xe[i] = xe_entry(s_xb[i >> 2], i & 3);
        if ((i & 3) == 0) s_xd[i >> 2] = s_xb[i >> 2].d;
      }
    } else {
      // thread t owns float4 i = t + k T (k < XL_K4) of every operand
      const float4* y4 = reinterpret_cast<const float4*>(a.y);
      const float4* r4 = reinterpret_cast<const float4*>(a.resid_in);
      const float4* wp4 = reinterpret_cast<const float4*>(a.w_post);
      const float4* wn4 = reinterpret_cast<const float4*>(a.w_next);
      float4 yv[XL_K4], hv[XL_K4], wv[XL_K4], nv[XL_K4];
#pragma unroll
      for (int k = 0; k < XL_K4; k++) {
        const int i = min(k * T + t, n4 - 1);
        hv[k] = r4[i];
        if (a.y) {
          yv[k] = y4[i];
          wv[k] = wp4[i];
        }
        nv[k] = wn4[i];
      }
      issue_w();
      auto own = [&](int k) { return k * T + t < n4; };
      if (a.y) {
#pragma unroll
        for (int k = 0; k < XL_K4; k++)
          if (own(k)) s_a4[k * T + t] = yv[k];
        __syncthreads();
        XL_MARK(1);
        const float sc1 = xl_rms_scale(xl_sumsq<NW>(s_a, n, &s_scale[0]), n, a.eps);
        XL_MARK(2);
#pragma unroll
        for (int k = 0; k < XL_K4; k++) {  // model.cpp:843-858: the post norm, then the residual add
          hv[k].x = hv[k].x + (sc1 * yv[k].x) * wv[k].x;
          hv[k].y = hv[k].y + (sc1 * yv[k].y) * wv[k].y;
          hv[k].z = hv[k].z + (sc1 * yv[k].z) * wv[k].z;
          hv[k].w = hv[k].w + (sc1 * yv[k].w) * wv[k].w;
        }
      }
#pragma unroll
      for (int k = 0; k < XL_K4; k++)
        if (own(k)) {
          s_b4[k * T + t] = hv[k];
          if (blockIdx.x == 0 && (a.y || a.resid_out != a.resid_in))
            reinterpret_cast<float4*>(a.resid_out)[k * T + t] = hv[k];
        }
      __syncthreads();
      XL_MARK(3);
      const float sc2 = xl_rms_scale(xl_sumsq<NW>(s_b, n, &s_scale[1]), n, a.eps);
      XL_MARK(4);
      // run_norm: (scale * x) * w (model.cpp:352-357), then quantize_row_q8_0 (ops.cpp:116-139) straight from the
      // registers: 8 consecutive lanes hold a block's 32 elements (a float4 each; blocks never straddle a k
      // round: n4 and T are multiples of 8), amax over the octet and the per-slot quant sums (order-free,
      // exact), the XE entries written by the octet's lanes 0-3 with the high words from lanes 4-7 (round 5:
      // two LDS passes and two barriers fewer than staging x and the XBlocks in LDS)
#pragma unroll
      for (int k = 0; k < XL_K4; k++) {
        const bool ok = own(k);  // (whole octets)
        const float4 x = make_float4((sc2 * hv[k].x) * nv[k].x, (sc2 * hv[k].y) * nv[k].y,
                                     (sc2 * hv[k].z) * nv[k].z, (sc2 * hv[k].w) * nv[k].w);
        if (ok && blockIdx.x == 0 && a.xn_out) reinterpret_cast<float4*>(a.xn_out)[k * T + t] = x;
        float amax = ok ? fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))) : 0.0f;
        amax = fmaxf(amax, dpp_f<DPP_QUAD_1032>(amax));  // (max: exact in any order; the octet on DPP)
        amax = fmaxf(amax, dpp_f<DPP_QUAD_2301>(amax));
        amax = fmaxf(amax, dpp_f<DPP_ROW_HALF_MIRROR>(amax));
        const float dd = amax / 127.0f;
        const float id = dd != 0.0f ? 1.0f / dd : 0.0f;
        const int q0 = nearest_int_fma(x.x, id), q1 = nearest_int_fma(x.y, id), q2 = nearest_int_fma(x.z, id),
                  q3 = nearest_int_fma(x.w, id);
        const uint32_t w = (uint32_t)(q0 & 0xFF) | ((uint32_t)(q1 & 0xFF) << 8) | ((uint32_t)(q2 & 0xFF) << 16) |
                           ((uint32_t)(q3 & 0xFF) << 24);
        const int sum = q0 + q1 + q2 + q3;
        const uint32_t wh = (uint32_t)dpp_i<DPP_ROW_SHL4>((int)w);  // octet lanes 4-7: elements 16-31 of the block
        const int sumh = dpp_i<DPP_ROW_SHL4>(sum);
        const int i4 = k * T + t, b = i4 >> 3, sl = i4 & 7;
        if (ok && sl < 4) s_xe[b * 4 + sl] = make_int4((int)w, (int)wh, -8 * sum, -8 * sumh);
        if (ok && sl == 0) s_xd[b] = h2f(f2h_ggml(dd));
      }
    }
  }
  __syncthreads();

  XL_MARK(5);
  if constexpr (SPR > 0) {  // ---- split rows: every (row, block, slot) dot by all lanes, then the chains ----
    constexpr int NBMAX = XL_K4 * T / 8;  // blocks per row: n <= 4 XL_K4 T
    __shared__ __attribute__((aligned(16))) float s_p[SPR * 8 * (NBMAX + 4)];
    __shared__ __attribute__((aligned(16))) float s_d[SPR * (NBMAX + 4)];
    const int ld = nb + 4;  // (conflict-free float4 rows: ld % 64 == 20 for nb = 80)
    const float4* s_xd4c = reinterpret_cast<const float4*>(s_xd);
#pragma unroll
    for (int m = 0; m < SIPL; m++) {
      const int i = t + T * m, jj4 = i & 3, R = (i >> 2) & (SPR - 1), g = i / (4 * SPR);
      if (g < ng) {
        const uint32_t w4[4] = {sq4[m].x, sq4[m].y, sq4[m].z, sq4[m].w};
        float4 pl, ph;
        float* plv = reinterpret_cast<float*>(&pl);
        float* phv = reinterpret_cast<float*>(&ph);
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int4 x = s_xe[(4 * g + u) * 4 + jj4];
          plv[u] = (float)sdot4((int)(w4[u] & 0x0F0F0F0Fu), x.x, x.z);
          phv[u] = (float)sdot4((int)((w4[u] >> 4) & 0x0F0F0F0Fu), x.y, x.w);
        }
        *reinterpret_cast<float4*>(s_p + (R * 8 + jj4) * ld + 4 * g) = pl;
        *reinterpret_cast<float4*>(s_p + (R * 8 + jj4 + 4) * ld + 4 * g) = ph;
        if (jj4 == 0) {
          const float4 xd = s_xd4c[g];
          *reinterpret_cast<float4*>(s_d + R * ld + 4 * g) =
              make_float4(h2f((uint16_t)(sd2[m].x & 0xFFFFu)) * xd.x, h2f((uint16_t)(sd2[m].x >> 16)) * xd.y,
                          h2f((uint16_t)(sd2[m].y & 0xFFFFu)) * xd.z, h2f((uint16_t)(sd2[m].y >> 16)) * xd.w);
        }
      }
    }
    __syncthreads();
    if (t < SPR * 8) {  // chain t: accumulator t % 8 of row t / 8, block order (ops.cpp:380-395)
      const float4* p4 = reinterpret_cast<const float4*>(s_p + t * ld);
      const float4* d4 = reinterpret_cast<const float4*>(s_d + (t >> 3) * ld);
      float acc = 0.0f;
#pragma unroll 4
      for (int b4 = 0; b4 < nb / 4; b4++) {
        const float4 p = p4[b4], d = d4[b4];
        acc = fmaf(d.x, p.x, acc);
        acc = fmaf(d.y, p.y, acc);
        acc = fmaf(d.z, p.z, acc);
        acc = fmaf(d.w, p.w, acc);
      }
      // hsum_float_8 (ops.cpp:324-330): ((a0 + a4) + (a2 + a6)) + ((a1 + a5) + (a3 + a7))
      const float t4 = acc + dpp_f<DPP_ROW_SHL4>(acc);
      const float u = t4 + dpp_f<DPP_QUAD_2301>(t4);
      const float r = u + dpp_f<DPP_QUAD_1032>(u);
      const int orow = srow0 + (t >> 3);
      if ((t & 7) == 0 && orow < rows) a.out[orow] = r;
    }
    XL_MARK(6);
    return;
  }
  // ---- the rows: every block in order, NCH chunks in flight ----
  float lo = 0.0f, hi = 0.0f;
  const float4* s_xd4 = reinterpret_cast<const float4*>(s_xd);
  for (int g0 = 0; g0 < ng; g0 += NCH * XL_P) {
#pragma unroll
    for (int k = 0; k < NCH; k++) {
      const int gk = g0 + k * XL_P;
      if (gk >= ng) break;
      if constexpr (LPR == 4) xl_eat(ck[k], gk, ng, jj, s_xe, s_xd4, lo, hi);
      else xl_eat1(ck[k], gk, ng, jj, jl & 4, s_xe, s_xd4, lo);
      if (gk + NCH * XL_P < ng) xl_load(ck[k], rq, rd, voq, vod, sq, sd, gk + NCH * XL_P, ng);
    }
  }
  // hsum_float_8 (ops.cpp:324-330): ((a0 + a4) + (a2 + a6)) + ((a1 + a5) + (a3 + a7)); lane jj holds a_jj, a_jj+4
  // (LPR 8: lane jl < 4 holds a_jl, lane jl + 4 holds a_jl+4)
  const float t4 = LPR == 4 ? lo + hi : lo + __shfl_xor(lo, 4);
  const float u = t4 + dpp_f<DPP_QUAD_2301>(t4);  // jj 0: t0 + t2, jj 1: t1 + t3
  const float r = u + dpp_f<DPP_QUAD_1032>(u);    // jj 0: (t0 + t2) + (t1 + t3)
  XL_MARK(6);
  if constexpr (ROLE == XL_GELU) {
    if (jj == 0) s_rows[wave * 16 + rl] = r;
    __syncthreads();
    // rows [64 u, 64 u + 32) gate, [64 u + 32, 64 u + 64) up of units 32 u .. 32 u + 31 (model.cpp:892-899)
    if (t < 32) {
      const float gv = gelu_mul1<true>(s_rows[t], s_rows[32 + t]);
      a.hid[blockIdx.x * 32 + t] = gv;
      q8_block_store(gv, true, a.hq + blockIdx.x, t);
    }
  } else {
    if (jl == 0 && row_ok) a.out[row] = r;
  }
}

// The PLAIN role split into the parallel part and the chains (round 5: down 16.9 us on 160 single-wave
// work-groups, each lane's 320-block loop one wave's VALU work on one SIMD of the CU).  Every accumulator update
// is acc = fma(d_b, (float)isum_b, acc) in block order (ops.cpp:380-395); d_b and the integer dots isum_b depend
// on nothing before them.  So a work-group of 4 waves owns 8 rows: per chunk of XS_CB blocks all 256 lanes compute
// the dots (sdot4 of the row's nibbles with the XE entries, exact integers, stored as floats) and the products
// d_b = f16(w.d) * x.d into LDS, then wave 0 -- lane R * 8 + k the accumulator k of row R -- runs the chains over
// the chunk: one LDS read per four steps, one fma per step.  Bit-identical to exact_gemv_kernel<.., XL_PLAIN>:
// the same values in the same fma chain, combined in the same order (hsum_float_8).
constexpr int XS_ROWS = 8, XS_CB = 160, XS_LD = XS_CB + 4;  // rows per WG, blocks per chunk, LDS row stride
constexpr int XS_IPL = XS_ROWS * (XS_CB / 4) * 4 / 256;      // items (group, row, slot) per lane per chunk

__global__ __launch_bounds__(256) void exact_plain_split_kernel(const uint4* __restrict__ wq, const uint2* __restrict__ wd,
                                                                int rows, int nb, XlArgs a) {
  extern __shared__ int4 s_dyn[];
  int4* s_xe = s_dyn;                                              // [nb][4]
  float* s_xd = reinterpret_cast<float*>(s_dyn + (size_t)nb * 4);  // [nb]
  __shared__ __attribute__((aligned(16))) float s_p[XS_ROWS * 8 * XS_LD];  // (float)isum per accumulator and block
  __shared__ __attribute__((aligned(16))) float s_d[XS_ROWS * XS_LD];      // d per row and block
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int row0 = blockIdx.x * XS_ROWS, ng = nb >> 2;
  const __amdgpu_buffer_rsrc_t rq = buf_rsrc(wq, (uint32_t)((size_t)ng * rows * 64));
  const __amdgpu_buffer_rsrc_t rd = buf_rsrc(wd, (uint32_t)((size_t)ng * rows * 8));
  XL_MARK(0);
  // item m of this lane in a chunk: local group gl, row R, slot jj (32 consecutive lanes: one group's 8 rows x 4
  // slots, 512 contiguous bytes of the XL stream)
  uint4 qa[XS_IPL], qb[XS_IPL];  // two chunks' weights in flight: the next chunk's issued before this one is used
  uint2 da[XS_IPL], db[XS_IPL];
  auto issue = [&](uint4 (&q)[XS_IPL], uint2 (&dq)[XS_IPL], int c0) {
#pragma unroll
    for (int m = 0; m < XS_IPL; m++) {
      const int i = t + 256 * m, jj = i & 3, R = (i >> 2) & 7, g = (c0 >> 2) + (i >> 5);
      const bool in = g < ng;
      q[m] = buf_ld16(rq, in ? ((g * rows + row0 + R) * 4 + jj) * 16 : (1 << 30), 0);
      typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
      const u32x2_t v = __builtin_amdgcn_raw_buffer_load_b64(rd, in && jj == 0 ? (g * rows + row0 + R) * 8 : (1 << 30), 0, BUF_NT);
      dq[m] = make_uint2(v.x, v.y);
    }
  };
  {  // the activation's XE entries (as exact_gemv_kernel's PLAIN role), the first chunk's weights issued behind
     // the activation's loads
    const uint4* xg = reinterpret_cast<const uint4*>(a.xb);
    for (int b0 = 0; b0 < nb; b0 += 4 * 256) {
      uint4 lo[4], hi[4];
      float d[4];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int b = min(b0 + k * 256 + t, nb - 1);
        lo[k] = xg[3 * b];
        hi[k] = xg[3 * b + 1];
        d[k] = __uint_as_float(xg[3 * b + 2].x);
      }
      if (b0 == 0) issue(qa, da, 0);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        const int b = b0 + k * 256 + t;
        if (b < nb) {
          const uint32_t l4[4] = {lo[k].x, lo[k].y, lo[k].z, lo[k].w}, h4[4] = {hi[k].x, hi[k].y, hi[k].z, hi[k].w};
#pragma unroll
          for (int j = 0; j < 4; j++)
            s_xe[b * 4 + j] = make_int4((int)l4[j], (int)h4[j], -8 * sdot4((int)l4[j], 0x01010101, 0),
                                        -8 * sdot4((int)h4[j], 0x01010101, 0));
          s_xd[b] = d[k];
        }
      }
    }
  }
  __syncthreads();
  XL_MARK(1);
  float acc = 0.0f;  // wave 0: accumulator k = lane & 7 of row lane >> 3
  const float4* s_xd4 = reinterpret_cast<const float4*>(s_xd);
  auto chunk = [&](const uint4 (&q)[XS_IPL], const uint2 (&dq)[XS_IPL], int c0) {
    // the dots and products of this chunk
#pragma unroll
    for (int m = 0; m < XS_IPL; m++) {
      const int i = t + 256 * m, jj = i & 3, R = (i >> 2) & 7, gl = i >> 5, g = (c0 >> 2) + gl;
      if (g < ng) {
        const uint32_t w4[4] = {q[m].x, q[m].y, q[m].z, q[m].w};
        float4 pl, ph;
        float* plv = reinterpret_cast<float*>(&pl);
        float* phv = reinterpret_cast<float*>(&ph);
#pragma unroll
        for (int u = 0; u < 4; u++) {
          const int4 x = s_xe[(4 * g + u) * 4 + jj];
          plv[u] = (float)sdot4((int)(w4[u] & 0x0F0F0F0Fu), x.x, x.z);
          phv[u] = (float)sdot4((int)((w4[u] >> 4) & 0x0F0F0F0Fu), x.y, x.w);
        }
        *reinterpret_cast<float4*>(s_p + (R * 8 + jj) * XS_LD + 4 * gl) = pl;
        *reinterpret_cast<float4*>(s_p + (R * 8 + jj + 4) * XS_LD + 4 * gl) = ph;
        if (jj == 0) {
          const float4 xd = s_xd4[g];
          *reinterpret_cast<float4*>(s_d + R * XS_LD + 4 * gl) =
              make_float4(h2f((uint16_t)(dq[m].x & 0xFFFFu)) * xd.x, h2f((uint16_t)(dq[m].x >> 16)) * xd.y,
                          h2f((uint16_t)(dq[m].y & 0xFFFFu)) * xd.z, h2f((uint16_t)(dq[m].y >> 16)) * xd.w);
        }
      }
    }
    __syncthreads();
    if (wave == 0) {  // the chains over the chunk, block order
      const int nbc = min(XS_CB, nb - c0);
      const float4* p4 = reinterpret_cast<const float4*>(s_p + lane * XS_LD);
      const float4* d4 = reinterpret_cast<const float4*>(s_d + (lane >> 3) * XS_LD);
#pragma unroll 4
      for (int b4 = 0; b4 < nbc / 4; b4++) {
        const float4 p = p4[b4], d = d4[b4];
        acc = fmaf(d.x, p.x, acc);
        acc = fmaf(d.y, p.y, acc);
        acc = fmaf(d.z, p.z, acc);
        acc = fmaf(d.w, p.w, acc);
      }
    }
    __syncthreads();  // the chunk's LDS is refilled next
  };
  for (int c0 = 0; c0 < nb; c0 += 2 * XS_CB) {
    if (c0 + XS_CB < nb) issue(qb, db, c0 + XS_CB);
    chunk(qa, da, c0);
    if (c0 + XS_CB >= nb) break;
    if (c0 + 2 * XS_CB < nb) issue(qa, da, c0 + 2 * XS_CB);
    chunk(qb, db, c0 + XS_CB);
  }
  XL_MARK(2);
  if (wave == 0) {
    // hsum_float_8 (ops.cpp:324-330): ((a0 + a4) + (a2 + a6)) + ((a1 + a5) + (a3 + a7)), lanes R * 8 + k
    const float t4 = acc + dpp_f<DPP_ROW_SHL4>(acc);  // (lanes R * 8 + 0..3: a_k + a_k+4)
    const float u = t4 + dpp_f<DPP_QUAD_2301>(t4);
    const float r = u + dpp_f<DPP_QUAD_1032>(u);
    const int row = row0 + (lane >> 3);
    if ((lane & 7) == 0 && row < rows) a.out[row] = r;
  }
}

// repack: standard device Q4_0 ([rows][nb][16 B] + d [rows][nb]) -> XL
__global__ void xl_repack_kernel(const uint4* __restrict__ q0, const uint16_t* __restrict__ d0, int r0,
                                 const uint4* __restrict__ q1, const uint16_t* __restrict__ d1, int r1,
                                 const uint4* __restrict__ q2, const uint16_t* __restrict__ d2, bool gelu32, int rows,
                                 int nb, uint4* __restrict__ oq, uint2* __restrict__ od) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // (g, R, jj)
  const int ng = nb / 4;
  if (i >= (size_t)ng * rows * 4) return;
  const int jj = (int)(i & 3);
  const int R = (int)((i >> 2) % rows);
  const int g = (int)((i >> 2) / rows);
  const uint4* q;
  const uint16_t* d;
  int sr;
  if (gelu32) {  // gate 32 k.., up 32 k..
    const int u = R / 64, k = R % 64;
    q = k < 32 ? q0 : q1;
    d = k < 32 ? d0 : d1;
    sr = 32 * u + (k & 31);
  } else if (R < r0) {
    q = q0; d = d0; sr = R;
  } else if (R < r0 + r1) {
    q = q1; d = d1; sr = R - r0;
  } else {
    q = q2; d = d2; sr = R - r0 - r1;
  }
  const uint32_t* qb = reinterpret_cast<const uint32_t*>(q + (size_t)sr * nb + 4 * g);
  oq[i] = make_uint4(qb[jj], qb[4 + jj], qb[8 + jj], qb[12 + jj]);
  if (jj == 0) {
    const uint16_t* dr = d + (size_t)sr * nb + 4 * g;
    od[(size_t)g * rows + R] = make_uint2((uint32_t)dr[0] | ((uint32_t)dr[1] << 16), (uint32_t)dr[2] | ((uint32_t)dr[3] << 16));
  }
}


// ---------------------------------------------------------------------------
// exact attention (exact.h)
// ---------------------------------------------------------------------------
// the q or k row of one head held by a wave: element i = lane + 64 k (EPL per lane), its norm weights and the
// rope table entries loaded by the caller (every global operand of the kernel is issued at its start);
// run_norm's serial chain (ops.cpp:28-43) on the row staged in s_x, (scale * x) * w, then NEOX rope at pos
// (ops.cpp:67-95, the pinned build's contractions: v0 c - v1 s and v0 s + v1 c as one fma each) -- pairs
// (i, i + HD / 2) sit in one lane
#ifdef XA_STATS
__device__ unsigned g_xa_serial;  // scores taking the serial chain (all heads, one launch)
#endif
// f16 bits -> max(exponent field, 1) for a nonzero value (its ulp is 2^(code - 25)), 31 for +-0
__device__ __forceinline__ int xa_exp_code(uint16_t b) {
  return (b & 0x7FFF) == 0 ? 31 : max((b >> 10) & 0x1F, 1);
}
// wave reductions: the 16-lane rows on DPP, then two cross-row shuffles
__device__ __forceinline__ int xa_wave_min(int v) {
  v = min(v, dpp_i<DPP_QUAD_1032>(v));
  v = min(v, dpp_i<DPP_QUAD_2301>(v));
  v = min(v, dpp_i<DPP_ROW_MIRROR>(v));
  v = min(v, dpp_i<DPP_ROW_HALF_MIRROR>(v));
  v = min(v, __shfl_xor(v, 16));
  return min(v, __shfl_xor(v, 32));
}
__device__ __forceinline__ int xa_wave_max(int v) {
  v = max(v, dpp_i<DPP_QUAD_1032>(v));
  v = max(v, dpp_i<DPP_QUAD_2301>(v));
  v = max(v, dpp_i<DPP_ROW_MIRROR>(v));
  v = max(v, dpp_i<DPP_ROW_HALF_MIRROR>(v));
  v = max(v, __shfl_xor(v, 16));
  return max(v, __shfl_xor(v, 32));
}
__device__ __forceinline__ double xa_wave_sum_d(double v) {  // (exact where the summands allow: xa_exact_ok)
  v += dpp_d<DPP_QUAD_1032>(v);
  v += dpp_d<DPP_QUAD_2301>(v);
  v += dpp_d<DPP_ROW_MIRROR>(v);
  v += dpp_d<DPP_ROW_HALF_MIRROR>(v);
  v += __shfl_xor(v, 16);
  return v + __shfl_xor(v, 32);
}
// No add of the score chain rounds: every product q_i k_i (exact in f32) is a multiple of 2^m, m = (qcode - 25) +
// (kcode - 25), and every partial sum is at most |q|_1 max|k| < 2^(m + 52) in magnitude, so each is a multiple of
// 2^m below 2^(m + 53): representable, in any order.  kmeta 0 (unknown key) or a non-finite bound: false.
// The same with the product quanta bounded pair by pair: epair = min over i of the raw exponent fields of q_i
// and k_i summed (2^(e - 25) bounds the ulp of an f16 of exponent field e from below, zero and subnormals
// included), so every product is a multiple of 2^(epair - 50) -- a tiny q_i no longer needs a tiny k_i's
// bound at the same time (round 5: with the per-vector minima ~1 % of the 4B model's keys failed, each a
// 256-step serial chain in its work-group).
__device__ __forceinline__ bool xa_exact_ok_pair(int epair, double qn1, uint32_t kmeta) {
  if ((kmeta >> 16) == 0) return false;  // unknown key
  const double bound = qn1 * (double)h2f((uint16_t)(kmeta & 0x7FFFu));
  return bound < __longlong_as_double((long long)(epair - 50 + 52 + 1023) << 52);
}
typedef unsigned short xa_u16x2 __attribute__((ext_vector_type(2)));
// the packed exponent fields of a word of two f16 values
__device__ __forceinline__ xa_u16x2 xa_exp2(uint32_t w) {
  return __builtin_bit_cast(xa_u16x2, (w >> 10) & 0x001F001Fu);
}
__device__ __forceinline__ bool xa_exact_ok(int qcode, double qn1, uint32_t kmeta) {
  const int kcode = (int)(kmeta >> 16);
  if (kcode == 0) return false;
  const int m = (qcode - 25) + (kcode - 25);
  const double bound = qn1 * (double)h2f((uint16_t)(kmeta & 0x7FFFu));
  return bound < __longlong_as_double((long long)(m + 52 + 1023) << 52);
}

// element (kv head hkv, head dim d, key j) of the tiled V copy (exact.h XAttnArgs::vt)
template <int HD>
__device__ __forceinline__ size_t xa_vt_index(int hkv, int d, int j, int stride) {
  return (((size_t)hkv * (HD / 64) + d / 64) * (stride / 32) + j / 32) * 2048 + ((j & 31) >> 3) * 512 + (d & 63) * 8 +
         (j & 7);
}

template <int HD>
struct XaRow {
  static constexpr int EPL = HD / 64;
  float v[EPL], w[EPL];
};
template <int HD>
__device__ __forceinline__ void xa_load(XaRow<HD>& r, const float* __restrict__ src, const float* __restrict__ nw) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < XaRow<HD>::EPL; k++) {
    r.v[k] = src[lane + 64 * k];
    r.w[k] = nw[lane + 64 * k];
  }
}
template <int HD>
__device__ __forceinline__ void xa_row(const XaRow<HD>& in, const float (&c)[HD / 128 > 0 ? HD / 128 : 1],
                                       const float (&sn)[HD / 128 > 0 ? HD / 128 : 1], double eps, float* s_x,
                                       float (&r)[HD / 64]) {
  constexpr int EPL = HD / 64, HALF = HD / 2;
  static_assert(HD % 16 == 0, "xl_chain_spec2<1>: four segments of whole float4s");
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < EPL; k++) s_x[lane + 64 * k] = in.v[k];
  __syncthreads();
  const float sc = xl_rms_scale(xl_chain_spec2<1>(s_x, HD), HD, eps);  // the serial chain (one wave), speculative
  float nv[EPL];
#pragma unroll
  for (int k = 0; k < EPL; k++) nv[k] = (sc * in.v[k]) * in.w[k];
#pragma unroll
  for (int k = 0; k < EPL / 2; k++) {  // element lane + 64 k < HALF pairs with lane + 64 k + HALF
    const int kp = k + EPL / 2;
    r[k] = fmaf(nv[k], c[k], -(nv[kp] * sn[k]));
    r[kp] = fmaf(nv[k], sn[k], nv[kp] * c[k]);
  }
  __syncthreads();  // s_x reuse
  (void)HALF;
}

// The q row's and the new key's k row's norms at once (the new key's work-group, one wave): the half-wave h
// (0: q, 1: k) runs its row's serial chain speculatively over 2 segments of HD / 2, 16 lanes per segment with
// two candidates each (xl_chain2), so both rows' chains share the wave's issue slots instead of running one
// after the other (round 5: the new key's work-group was the scores launch's critical path).  Each row's scale
// is bit-identical to xl_chain's.
template <int HD>
__device__ __forceinline__ void xa_row2(const XaRow<HD>& inq, const XaRow<HD>& ink, const float (&c)[HD / 128 > 0 ? HD / 128 : 1],
                                        const float (&sn)[HD / 128 > 0 ? HD / 128 : 1], double eps, float* s_xq,
                                        float* s_xk, float (&rq)[HD / 64], float (&rk)[HD / 64]) {
  constexpr int EPL = HD / 64, L = HD / 2, L4 = L / 4, R = (L4 + 15) / 16;
  static_assert(HD % 32 == 0, "xa_row2: two segments of whole float4s");
  __shared__ double s_seg2[2][2];
  __shared__ float s_e2[2][64];
  __shared__ int s_base2[2][2];
  const int lane = threadIdx.x & 63, hh = lane >> 5, seg = (lane >> 4) & 1, c16 = lane & 15;
#pragma unroll
  for (int k = 0; k < EPL; k++) {
    s_xq[lane + 64 * k] = inq.v[k];
    s_xk[lane + 64 * k] = ink.v[k];
  }
  __syncthreads();
  const float* sx = hh ? s_xk : s_xq;
  {
    const float4* s4 = reinterpret_cast<const float4*>(sx + seg * L);
    float4 v[R];
#pragma unroll
    for (int r = 0; r < R; r++) v[r] = s4[min(c16 + 16 * r, L4 - 1)];
    double p = 0.0;
#pragma unroll
    for (int r = 0; r < R; r++)
      if (c16 + 16 * r < L4) {
        const double x = v[r].x, y = v[r].y, z = v[r].z, w = v[r].w;
        p = fma(x, x, fma(y, y, fma(z, z, fma(w, w, p))));
      }
    p += dpp_d<DPP_QUAD_1032>(p);
    p += dpp_d<DPP_QUAD_2301>(p);
    p += dpp_d<DPP_ROW_MIRROR>(p);
    p += dpp_d<DPP_ROW_HALF_MIRROR>(p);
    if (c16 == 0) s_seg2[hh][seg] = p;
  }
  __syncthreads();
  const int base = seg == 0 ? 0 : max(0, (int)__float_as_uint((float)s_seg2[hh][0]) - 16);
  float ea = seg == 0 ? 0.0f : __uint_as_float((uint32_t)(base + c16));
  float eb = seg == 0 ? 0.0f : __uint_as_float((uint32_t)(base + 16 + c16));
  xl_chain2(sx + seg * L, L, ea, eb);
  s_e2[hh][seg * 32 + c16] = ea;
  s_e2[hh][seg * 32 + 16 + c16] = eb;
  if (c16 == 0) s_base2[hh][seg] = base;
  __syncthreads();
  const float sq = xl_spec_walk<2>(s_xq, L, s_e2[0], s_base2[0], nullptr);
  const float sk = xl_spec_walk<2>(s_xk, L, s_e2[1], s_base2[1], nullptr);
  const float scq = xl_rms_scale(sq, HD, eps), sck = xl_rms_scale(sk, HD, eps);
  float nq[EPL], nk[EPL];
#pragma unroll
  for (int k = 0; k < EPL; k++) {
    nq[k] = (scq * inq.v[k]) * inq.w[k];
    nk[k] = (sck * ink.v[k]) * ink.w[k];
  }
#pragma unroll
  for (int k = 0; k < EPL / 2; k++) {  // NEOX rope, as xa_row
    const int kp = k + EPL / 2;
    rq[k] = fmaf(nq[k], c[k], -(nq[kp] * sn[k]));
    rq[kp] = fmaf(nq[k], sn[k], nq[kp] * c[k]);
    rk[k] = fmaf(nk[k], c[k], -(nk[kp] * sn[k]));
    rk[kp] = fmaf(nk[k], sn[k], nk[kp] * c[k]);
  }
  __syncthreads();  // s_xq / s_xk / s_e2 reuse
}

// BATCH (the batched prefill, launch_exact_attn_batch): token z = blockIdx.z at pos = *d_pos + z; its f16 query
// row comes from a.qh (the q/k launch normalised, roped and scaled it, and appended every token's K / V), and the
// split work-groups take all its keys 0 .. pos (no new-key work-group)
template <int HD, bool BATCH = false>
__global__ __launch_bounds__(64) void xattn_scores_kernel(XAttnArgs a) {
  constexpr int EPL = HD / 64, CPL = EPL / 2, QW = HD / 32;  // QW: 16-B words of a quarter row
  constexpr int KPC = 16;                                    // keys per chunk: 4 lanes (row quarters) per key
  __shared__ __attribute__((aligned(16))) float s_x[HD];
  __shared__ __attribute__((aligned(16))) float s_x2[HD];
  __shared__ __attribute__((aligned(16))) double s_q[HD];
  __shared__ __attribute__((aligned(16))) uint16_t s_k[HD];
  __shared__ __attribute__((aligned(16))) uint16_t s_qe[HD];  // the f16 query's exponent fields
  const int h = blockIdx.x, split = blockIdx.y, lane = threadIdx.x;
  const int z = BATCH ? (int)blockIdx.z : 0;
  const int pos = *a.d_pos + z;
  // work-groups split < XA_NSPLIT: the keys before pos (BATCH: up to pos) in chunks of 16, chunk split, split +
  // XA_NSPLIT, ..; the last one (split == XA_NSPLIT, decode only): the new key -- k norm + rope, the K / V append
  // and its score
  const int nk = BATCH ? pos + 1 : pos;
  const bool pos_wg = !BATCH && split == XA_NSPLIT;
  if (!pos_wg && split * KPC >= nk) return;  // no key chunk for this work-group (whole wave)
  const int hkv = h / (a.n_head / a.n_head_kv);
  const int kl = lane >> 2, qt = lane & 3;  // key of the chunk, quarter of its row
  XL_MARK(0);
  // every global operand first: q row + weights, the rope entries, the new key's k / v rows or the first K rows
  float c[CPL], sn[CPL];
  XaRow<HD> qr, kr_;
  uint16_t qb16[EPL];
  if constexpr (BATCH) {
    const uint16_t* qh = a.qh + ((size_t)z * a.n_head + h) * HD;
#pragma unroll
    for (int k = 0; k < EPL; k++) qb16[k] = qh[lane + 64 * k];
  } else {
    const float* cs = a.rope_cs + (size_t)pos * HD;
#pragma unroll
    for (int k = 0; k < CPL; k++) {
      const float2 t = reinterpret_cast<const float2*>(cs)[lane + 64 * k];
      c[k] = t.x;
      sn[k] = t.y;
    }
    xa_load<HD>(qr, a.qkv + (size_t)h * HD, a.q_norm_w);
  }
  float vrow[EPL];
  const uint16_t* kb = a.k_cache + (size_t)hkv * a.max_ctx * HD;
  const uint32_t* km = a.kmeta ? a.kmeta + (size_t)hkv * a.max_ctx : nullptr;
  uint4 wa[QW];
  uint32_t meta = 0u;
  auto ld_quarter = [&](uint4 (&w)[QW], int j) {
    const uint4* src = reinterpret_cast<const uint4*>(kb + (size_t)j * HD) + qt * QW;
#pragma unroll
    for (int u = 0; u < QW; u++) w[u] = src[u];
  };
  if (pos_wg) {
    xa_load<HD>(kr_, a.qkv + a.k_off + (size_t)hkv * HD, a.k_norm_w);
#pragma unroll
    for (int k = 0; k < EPL; k++) vrow[k] = a.qkv[a.v_off + (size_t)hkv * HD + lane + 64 * k];
  } else {
    const int j1 = min(split * KPC + kl, nk - 1);
    ld_quarter(wa, j1);
    meta = km ? km[j1] : 0u;
  }
  float r[EPL], rk2[EPL];
  if constexpr (!BATCH) {
    if (pos_wg) xa_row2<HD>(qr, kr_, c, sn, a.eps, s_x, s_x2, r, rk2);  // (uniform per work-group)
    else xa_row<HD>(qr, c, sn, a.eps, s_x, r);
  }
  XL_MARK(1);
  // the query's exactness words (xa_exact_ok): min over its nonzero elements of max(exponent field, 1), |q|_1
  int qcode = 31;
  double qn1 = 0.0;
#pragma unroll
  for (int k = 0; k < EPL; k++) {  // model.cpp:767 scale, then the score's f16 query (model.cpp:507)
    const uint16_t qb = BATCH ? qb16[k] : f2h_ggml(r[k] * a.attn_scale);
    s_q[lane + 64 * k] = (double)h2f(qb);
    s_qe[lane + 64 * k] = (qb >> 10) & 0x1F;
    qcode = min(qcode, xa_exp_code(qb));
    qn1 += fabs((double)h2f(qb));
  }
  qcode = xa_wave_min(qcode);
  qn1 = xa_wave_sum_d(qn1);
  int kcode_new = 31;
  uint32_t kmag_new = 0;
  if (pos_wg) {  // the new key: k norm + rope (xa_row2 above), K and V rows appended (model.cpp:440-474)
#pragma unroll
    for (int k = 0; k < EPL; k++) r[k] = rk2[k];
    uint16_t* kc = a.k_cache + ((size_t)hkv * a.max_ctx + pos) * HD;
    uint16_t* vc = a.v_cache + ((size_t)hkv * a.max_ctx + pos) * HD;
#pragma unroll
    for (int k = 0; k < EPL; k++) {
      const uint16_t kbits = f2h_ggml(r[k]), vbits = f2h_ggml(vrow[k]);
      s_k[lane + 64 * k] = kbits;
      kc[lane + 64 * k] = kbits;
      vc[lane + 64 * k] = vbits;
      a.vt[xa_vt_index<HD>(hkv, lane + 64 * k, pos, a.vt_stride)] = vbits;  // the tiled copy's column
      kcode_new = min(kcode_new, xa_exp_code(kbits));
      kmag_new = max(kmag_new, (uint32_t)(kbits & 0x7FFFu));
    }
    kcode_new = xa_wave_min(kcode_new);
    kmag_new = (uint32_t)xa_wave_max((int)kmag_new);
    if (lane == 0 && km) a.kmeta[(size_t)hkv * a.max_ctx + pos] = ((uint32_t)kcode_new << 16) | kmag_new;
    XL_MARK(2);
  }
  __syncthreads();
  XL_MARK(3);
  double* sc_out = a.scores + ((size_t)z * a.n_head + h) * a.max_ctx;
  // score = sum_i (double)(f16(k_i) * f16(q_i)), i in order, from 0.0 (model.cpp:504-509): the f32 product of two
  // f16 values is exact, so one f64 fma per element is the reference's rounding.  Where xa_exact_ok holds no add
  // of that chain rounds, so the row's four quarters are summed by four lanes and combined (the same bits); the
  // f64 element step costs ~25 cycles of one wave's issue (round 5, scripts/dev/xl_bench), so a key per lane was a
  // 6.4K-cycle loop.  Otherwise the serial chain, by one lane.
  auto serial = [&](const uint16_t* row) __attribute__((always_inline)) {
    const uint4* r4 = reinterpret_cast<const uint4*>(row);
    double acc = 0.0;
#pragma unroll 1
    for (int i0 = 0; i0 < HD / 8; i0 += 8) {
      uint4 w[8];
#pragma unroll
      for (int u = 0; u < 8; u++) w[u] = r4[i0 + u];
#pragma unroll
      for (int u = 0; u < 8; u++) {
        const uint32_t ww[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const int i = (i0 + u) * 8 + 2 * e;
          acc = fma((double)h2f((uint16_t)(ww[e] & 0xFFFF)), s_q[i], acc);
          acc = fma((double)h2f((uint16_t)(ww[e] >> 16)), s_q[i + 1], acc);
        }
      }
    }
    return acc;
  };
  if (pos_wg) {
    int ep = 64;
#pragma unroll
    for (int k = 0; k < EPL; k++) ep = min(ep, (int)((s_k[lane + 64 * k] >> 10) & 0x1F) + (int)s_qe[lane + 64 * k]);
    ep = xa_wave_min(ep);
    if (xa_exact_ok_pair(ep, qn1, ((uint32_t)kcode_new << 16) | kmag_new)) {  // (uniform) elements lane + 64 k
      double p = 0.0;
#pragma unroll
      for (int k = 0; k < EPL; k++) p = fma((double)h2f(s_k[lane + 64 * k]), s_q[lane + 64 * k], p);
      p = xa_wave_sum_d(p);
      if (lane == 0) sc_out[pos] = p;
    } else if (lane == 0) {
      sc_out[pos] = serial(s_k);
    }
  } else {
    const double2* q2 = reinterpret_cast<const double2*>(s_q + qt * (HD / 4));
    const xa_u16x2* qe2 = reinterpret_cast<const xa_u16x2*>(s_qe + qt * (HD / 4));
    for (int cc = split; cc * KPC < nk; cc += XA_NSPLIT) {
      const int j = cc * KPC + kl;
      const bool valid = j < nk;
      uint4 wn[QW];
      uint32_t mn = 0u;
      const bool more = (cc + XA_NSPLIT) * KPC < nk;  // (uniform) the next chunk's rows in flight
      if (more) {
        const int jn = min((cc + XA_NSPLIT) * KPC + kl, nk - 1);
        ld_quarter(wn, jn);
        mn = km ? km[jn] : 0u;
      }
      double p = 0.0;
      xa_u16x2 pm = {64, 64};  // min over this quarter's pairs of the two exponent fields' sum
#pragma unroll
      for (int u = 0; u < QW; u++) {
        const uint32_t ww[4] = {wa[u].x, wa[u].y, wa[u].z, wa[u].w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const double2 q = q2[u * 4 + e];
          p = fma((double)h2f((uint16_t)(ww[e] & 0xFFFF)), q.x, p);
          p = fma((double)h2f((uint16_t)(ww[e] >> 16)), q.y, p);
          pm = __builtin_elementwise_min(pm, xa_exp2(ww[e]) + qe2[u * 4 + e]);
        }
      }
      p += dpp_d<DPP_QUAD_1032>(p);  // the key's four quarters (exact where ok)
      p += dpp_d<DPP_QUAD_2301>(p);
      int ep = min((int)pm.x, (int)pm.y);
      ep = min(ep, dpp_i<DPP_QUAD_1032>(ep));
      ep = min(ep, dpp_i<DPP_QUAD_2301>(ep));
      const bool ok = xa_exact_ok_pair(ep, qn1, meta);
      if (valid && qt == 0) sc_out[j] = ok ? p : serial(kb + (size_t)j * HD);
#ifdef XA_STATS
      {
        const unsigned long long bal = __ballot(valid && qt == 0 && !ok);
        if (lane == 0 && bal) atomicAdd(&g_xa_serial, (unsigned)__popcll(bal));
      }
#endif
      if (more) {
#pragma unroll
        for (int u = 0; u < QW; u++) wa[u] = wn[u];
        meta = mn;
      }
    }
  }
  XL_MARK(4);
}

// f64 DPP move with a fill value for lanes without a source (row_mask ROWS: the rows written)
template <int CTRL, int ROWS>
__device__ __forceinline__ double xa_dpp_d_old(double v, double old) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(old), __double2loint(v), CTRL, ROWS, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(old), __double2hiint(v), CTRL, ROWS, 0xF, false);
  return __hiloint2double(hi, lo);
}
// inclusive prefix max across the wave: row_shr 1, 2, 4, 8 within the 16-lane rows, then row_bcast 15 / 31
__device__ __forceinline__ double xa_wave_incl_max(double v) {
  const double ninf = -INFINITY;
  v = fmax(v, xa_dpp_d_old<0x111, 0xF>(v, ninf));
  v = fmax(v, xa_dpp_d_old<0x112, 0xF>(v, ninf));
  v = fmax(v, xa_dpp_d_old<0x114, 0xF>(v, ninf));
  v = fmax(v, xa_dpp_d_old<0x118, 0xF>(v, ninf));
  v = fmax(v, xa_dpp_d_old<0x142, 0xA>(v, ninf));
  v = fmax(v, xa_dpp_d_old<0x143, 0xC>(v, ninf));
  return v;
}

constexpr int XA_CH = 1024;  // accum: keys per chunk in LDS

// eight steps of vec_mad_f16 for one head dim: acc (f16 in the low half) = f16(fma(f16 V[u], e[u], acc)), each
// step v_fma_mix_f32 (f16 operands widened exactly, one f32 rounding) then v_cvt_f16_f32 (round to nearest even):
// the reference's f32 fma and f32_to_f16, two dependent instructions per key with no padding between them
__device__ __forceinline__ void xa_mad8(uint32_t& acc, const uint32_t* v, const float* e) {
  asm volatile(
      "v_fma_mix_f32 %0, %1, %9, %0 op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %2, %10, %0 op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %3, %11, %0 op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %4, %12, %0 op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %5, %13, %0 op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %6, %14, %0 op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %7, %15, %0 op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %8, %16, %0 op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0"
      : "+v"(acc)
      : "v"(v[0]), "v"(v[1]), "v"(v[2]), "v"(v[3]), "v"(v[4]), "v"(v[5]), "v"(v[6]), "v"(v[7]), "v"(e[0]), "v"(e[1]),
        "v"(e[2]), "v"(e[3]), "v"(e[4]), "v"(e[5]), "v"(e[6]), "v"(e[7]));
}

// the same eight steps with the V values packed two to a register (key 2i in the low half, 2i + 1 in the high)
__device__ __forceinline__ void xa_mad8p(uint32_t& acc, const uint4 v, const float* e) {
  asm volatile(
      "v_fma_mix_f32 %0, %1, %5, %0 op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %1, %6, %0 op_sel:[1,0,0] op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %2, %7, %0 op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %2, %8, %0 op_sel:[1,0,0] op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %3, %9, %0 op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %3, %10, %0 op_sel:[1,0,0] op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %4, %11, %0 op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0\n\t"
      "v_fma_mix_f32 %0, %4, %12, %0 op_sel:[1,0,0] op_sel_hi:[1,0,1]\n\t"
      "v_cvt_f16_f32_e32 %0, %0"
      : "+v"(acc)
      : "v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w), "v"(e[0]), "v"(e[1]), "v"(e[2]), "v"(e[3]), "v"(e[4]), "v"(e[5]),
        "v"(e[6]), "v"(e[7]));
}

// xa_mad8p for eight keys holding a max move: before every key's step vec_scale_f16's acc = f16(f32(acc) * pe)
// (ops.cpp:1084-1090), as v_fma_mix_f32 with a -0.0 addend (x * pe + -0.0 is x * pe rounded once, the sign of a
// zero product kept) then v_cvt_f16_f32; pe is exactly 1.0 on the keys without a move, where the scale returns
// acc's own bits.  Branch-free: four dependent instructions per key instead of a uniform branch per key
#define XA_SCALE_STEP(V, E, P, SEL)                                          \
  "v_fma_mix_f32 %0, %0, " P ", %13 op_sel_hi:[1,0,0]\n\t"                  \
  "v_cvt_f16_f32_e32 %0, %0\n\t"                                             \
  "v_fma_mix_f32 %0, " V ", " E ", %0 " SEL "op_sel_hi:[1,0,1]\n\t"          \
  "v_cvt_f16_f32_e32 %0, %0\n\t"
__device__ __forceinline__ void xa_mad8s(uint32_t& acc, const uint4 v, const float* e, const float* pe) {
  asm volatile(XA_SCALE_STEP("%1", "%5", "%14", "") XA_SCALE_STEP("%1", "%6", "%15", "op_sel:[1,0,0] ")
               XA_SCALE_STEP("%2", "%7", "%16", "") XA_SCALE_STEP("%2", "%8", "%17", "op_sel:[1,0,0] ")
               XA_SCALE_STEP("%3", "%9", "%18", "") XA_SCALE_STEP("%3", "%10", "%19", "op_sel:[1,0,0] ")
               XA_SCALE_STEP("%4", "%11", "%20", "") XA_SCALE_STEP("%4", "%12", "%21", "op_sel:[1,0,0] ")
               : "+v"(acc)
               : "v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w), "v"(e[0]), "v"(e[1]), "v"(e[2]), "v"(e[3]), "v"(e[4]),
                 "v"(e[5]), "v"(e[6]), "v"(e[7]), "v"(0x80000000u), "v"(pe[0]), "v"(pe[1]), "v"(pe[2]), "v"(pe[3]),
                 "v"(pe[4]), "v"(pe[5]), "v"(pe[6]), "v"(pe[7]));
}
#undef XA_SCALE_STEP

// one step of xa_mad8p: key in the low (hi = 0) or high half of v
__device__ __forceinline__ void xa_mad1(uint32_t& acc, uint32_t v, float e, int hi) {
  if (hi)
    asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,0,1]\n\tv_cvt_f16_f32_e32 %0, %0"
                 : "+v"(acc) : "v"(v), "v"(e));
  else
    asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]\n\tv_cvt_f16_f32_e32 %0, %0" : "+v"(acc) : "v"(v), "v"(e));
}

// f32 -> f16, round to nearest even (= the reference's f32_to_f16 for every non-NaN input: llmi_selftest 0), as
// one instruction the compiler cannot fuse with the fma that produced its input
__device__ __forceinline__ uint16_t cvt_f16_rne(float f) {
  uint32_t r;
  asm volatile("v_cvt_f16_f32_e32 %0, %1" : "=v"(r) : "v"(f));
  return (uint16_t)r;
}

// (Tried: the V rows through an LDS ring filled by LDS-DMA three 64-key stages ahead -- 28.3 vs 24.6 us at 600
// keys in scripts/dev/xl_bench: the per-key chain, not the V loads, bounds this kernel.)
// BATCH: token z = blockIdx.y at pos = *d_pos + z (scores / out / xq at the token's rows)
template <int HD, bool BATCH = false>
__global__ __launch_bounds__((HD / 64 + 1) * 64) void xattn_accum_kernel(XAttnArgs a) {
  constexpr int NWV = HD / 64, T = (NWV + 1) * 64;
  constexpr int NWS = T / 64, KPT = (XA_CH + T - 1) / T;  // the branch pass: every wave, KPT keys per thread
  __shared__ double s_sc[XA_CH];
  static_assert(XA_CH / 32 <= 32, "the chunk's max-move words: one per lane of a half-wave");
  __shared__ __attribute__((aligned(16))) float s_e[XA_CH];   // e per key
  __shared__ __attribute__((aligned(16))) float s_pe[XA_CH];  // pe per key
  __shared__ uint32_t s_up[XA_CH / 32];
  __shared__ double s_tmax[NWS];  // the scan waves' maxima
  __shared__ float s_sacc;
  __shared__ uint64_t s_etab[32];  // expf's table (a per-lane global load each call, on the branch pass's chain)
  const int h = blockIdx.x, t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int z = BATCH ? (int)blockIdx.y : 0;
  const int n_keys = *a.d_pos + z + 1;
  const int hkv = h / (a.n_head / a.n_head_kv);
  const double* sc_in = a.scores + ((size_t)z * a.n_head + h) * a.max_ctx;
  double run_max = -INFINITY;
  uint16_t v16 = 0;  // f32_to_f16(0.0f)
  float s_acc = 0.0f;
  // this lane's head dim of the tiled V (wave < NWV: dims 64 wave ..), a 32-key batch as 4 loads of 8 keys, each
  // load one contiguous KB across the wave; tiles past the context stay inside the kv head and are never summed
  constexpr int NB = 4;  // V batches in flight (6: 5 spilled VGPRs, 354 vs 360 tok/s)
  const uint4* vtp = reinterpret_cast<const uint4*>(a.vt + xa_vt_index<HD>(hkv, min(wave, NWV - 1) * 64 + lane, 0, a.vt_stride));
  const int kb_last = a.vt_stride / 32 - 1;
  uint4 vb4[NB][4];
  auto ld = [&](uint4 (&dst)[4], int jb) {  // jb % 32 == 0
    const uint4* tp = vtp + (size_t)min(jb / 32, kb_last) * 256;  // a tile: 4 KB = 256 uint4
#pragma unroll
    for (int i = 0; i < 4; i++) dst[i] = tp[i * 64];
  };
  if (t < 32) s_etab[t] = llmi_glibc::exp2f_tab(t);
  XL_MARK(0);
#ifdef XA_STATS
  int st_batches = 0, st_slow = 0, st_moves = 0;
  const unsigned long long st_t0 = __builtin_amdgcn_s_memtime();
#endif
  for (int c0 = 0; c0 < n_keys; c0 += XA_CH) {
    const int nk = min(XA_CH, n_keys - c0);
    for (int i = t; i < nk; i += T)
      s_sc[i] = a.softcap > 0.0f ? llmi_glibc::softcap_score(sc_in[c0 + i], a.softcap) : sc_in[c0 + i];
    for (int i = t; i < XA_CH / 32; i += T) s_up[i] = 0u;
    __syncthreads();
    XL_MARK(1);
    // the max of every key before each key (max is exact, so any grouping): segments of KPT keys per thread,
    // an inclusive prefix max across each wave's 64 segments on DPP, then across the waves' totals.  (Round 5:
    // all T threads scan -- the 256-thread scan left keys 768.. of a chunk unscanned at head_dim 128.)
    double tmax = -INFINITY;
#pragma unroll
    for (int k = 0; k < KPT; k++) {
      const int j = t * KPT + k;
      if (j < nk) tmax = fmax(tmax, s_sc[j]);
    }
    tmax = xa_wave_incl_max(tmax);
    if (lane == 63) s_tmax[wave] = tmax;
    if (wave < NWV) {  // the chunk's first V batches, in flight during the branch pass below
#pragma unroll
      for (int b = 0; b < NB - 1; b++) ld(vb4[b], c0 + b * 32);
    }
    __syncthreads();
    {
      const double left = xa_dpp_d_old<0x138, 0xF>(tmax, -INFINITY);  // wave_shr:1: the previous segments' max
      double pm = run_max;                                             // max of every key before this segment
      for (int w = 0; w < wave; w++) pm = fmax(pm, s_tmax[w]);
      pm = fmax(pm, left);
#pragma unroll
      for (int k = 0; k < KPT; k++) {
        const int j = t * KPT + k;
        if (j >= nk) break;
        const double score = s_sc[j];
        const float prev = (float)pm;  // the reference's max_score before key j
        if (score > (double)prev) {    // model.cpp:520-532
          s_e[j] = 1.0f;
          s_pe[j] = llmi_glibc::expf_tab(prev - (float)score, s_etab);
          atomicOr(&s_up[j >> 5], 1u << (j & 31));
        } else {
          s_e[j] = llmi_glibc::expf_tab((float)(score - (double)prev), s_etab);
          s_pe[j] = 1.0f;
        }
        pm = fmax(pm, score);
      }
    }
#pragma unroll
    for (int w = 0; w < NWS; w++) run_max = fmax(run_max, s_tmax[w]);
    __syncthreads();
    XL_MARK(2);
    if (wave < NWV) {  // this lane's head dim from the transposed V: 8 keys per 16-B load, NB - 1 batches
      // of 32 keys in flight, and the next batch's e values read while this one is summed.  vec_scale_f16 when
      // the max moved, then vec_mad_f16 (ops.cpp:1084-1099)
      float eb[2][32];
      auto lde = [&](float (&dst)[32], int j0) {
        const float4* q4 = reinterpret_cast<const float4*>(s_e + min(j0, XA_CH - 32));
#pragma unroll
        for (int u4 = 0; u4 < 8; u4++) {
          const float4 q = q4[u4];
          dst[4 * u4] = q.x; dst[4 * u4 + 1] = q.y; dst[4 * u4 + 2] = q.z; dst[4 * u4 + 3] = q.w;
        }
      };
      lde(eb[0], 0);
      const uint32_t upv = s_up[lane & 31];  // batch i's max-move bits in lane i (read per batch by readlane)
      for (int j00 = 0; j00 < nk; j00 += 32 * NB) {
#pragma unroll
        for (int b = 0; b < NB; b++) {
          const int j0 = j00 + b * 32;
          ld(vb4[(b + NB - 1) % NB], c0 + j0 + (NB - 1) * 32);  // into the slot summed in the previous batch
          if (j0 >= nk) continue;
          lde(eb[(b + 1) & 1], j0 + 32);
          const uint32_t up = __builtin_amdgcn_readlane(upv, j0 >> 5);
          const int m = __builtin_amdgcn_readfirstlane(min(32, nk - j0));
          const float* e = eb[b & 1];
#ifdef XA_STATS
          if (wave == 0) { st_batches++; st_slow += up != 0; st_moves += __builtin_popcount(up); }
#endif
          if (up == 0 && m == 32) {
            uint32_t acc = v16;
#pragma unroll
            for (int i = 0; i < 4; i++) xa_mad8p(acc, vb4[b][i], e + 8 * i);
            v16 = (uint16_t)acc;
          } else {  // a max move in the batch, or its last keys: the pe values in registers too
            float pe[32];
#pragma unroll
            for (int u4 = 0; u4 < 8; u4++) {
              const float4 q = reinterpret_cast<const float4*>(s_pe + j0)[u4];
              pe[4 * u4] = q.x; pe[4 * u4 + 1] = q.y; pe[4 * u4 + 2] = q.z; pe[4 * u4 + 3] = q.w;
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // no LDS wait inside the key steps
            uint32_t acc = v16;
#pragma unroll
            for (int i = 0; i < 4; i++) {  // eight keys at a time: straight steps where the eight have no move,
              // scale + step for all eight where they hold one; key by key only in the context's last keys
              if (m >= 8 * (i + 1)) {
                if (((up >> (8 * i)) & 0xFFu) == 0) xa_mad8p(acc, vb4[b][i], e + 8 * i);
                else xa_mad8s(acc, vb4[b][i], e + 8 * i, pe + 8 * i);
                continue;
              }
#pragma unroll
              for (int u = 8 * i; u < 8 * i + 8; u++) {
                if (__builtin_expect(u < m, 1)) {  // wave-uniform; a move is the rare key (the branch falls through)
                  if (__builtin_expect((up & (1u << u)) != 0, 0))
                    acc = cvt_f16_rne((float)__builtin_bit_cast(_Float16, (uint16_t)acc) * pe[u]);
                  const uint4 w4 = vb4[b][u >> 3];
                  const uint32_t wv = ((u >> 1) & 3) == 0 ? w4.x : ((u >> 1) & 3) == 1 ? w4.y : ((u >> 1) & 3) == 2 ? w4.z : w4.w;
                  xa_mad1(acc, wv, e[u], u & 1);
                }
              }
            }
            v16 = (uint16_t)acc;
          }
        }
      }
    } else if (wave == NWV) {  // s_acc = s_acc * pe + e, keys in order (model.cpp:540), 32 keys' e per read, the
      // next batch's read in flight; pe is exactly 1 where the max did not move, so those steps are the add alone
      // (s_acc * 1.0f == s_acc: round 5, the mul + add chain outlasted the V chains once their loads were tiled)
      const uint32_t upv = s_up[lane & 31];
      float eb[2][32];
      auto lde = [&](float (&dst)[32], int j0) {
        const float4* q4 = reinterpret_cast<const float4*>(s_e + min(j0, XA_CH - 32));
#pragma unroll
        for (int u4 = 0; u4 < 8; u4++) {
          const float4 q = q4[u4];
          dst[4 * u4] = q.x; dst[4 * u4 + 1] = q.y; dst[4 * u4 + 2] = q.z; dst[4 * u4 + 3] = q.w;
        }
      };
      lde(eb[0], 0);
      for (int j00 = 0; j00 < nk; j00 += 64) {
#pragma unroll
        for (int b = 0; b < 2; b++) {
          const int j0 = j00 + 32 * b;
          if (j0 >= nk) break;
          lde(eb[b ^ 1], j0 + 32);
          const uint32_t up = __builtin_amdgcn_readlane(upv, j0 >> 5);
          const int m = __builtin_amdgcn_readfirstlane(min(32, nk - j0));
          const float* ev = eb[b];
          if (up == 0 && m == 32) {
#pragma unroll
            for (int u = 0; u < 32; u++) s_acc = s_acc + ev[u];
          } else {
            float pv[32];
#pragma unroll
            for (int u4 = 0; u4 < 8; u4++) {
              const float4 p = reinterpret_cast<const float4*>(s_pe + j0)[u4];
              pv[4 * u4] = p.x; pv[4 * u4 + 1] = p.y; pv[4 * u4 + 2] = p.z; pv[4 * u4 + 3] = p.w;
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {  // eight keys at a time: plain adds where the eight have no move, the
              // reference's s_acc * pe + e on all eight where they hold one (pe 1.0: the mul returns s_acc)
              if (m >= 8 * (i + 1)) {
                if (((up >> (8 * i)) & 0xFFu) == 0) {
#pragma unroll
                  for (int u = 8 * i; u < 8 * i + 8; u++) s_acc = s_acc + ev[u];
                } else {
#pragma unroll
                  for (int u = 8 * i; u < 8 * i + 8; u++) s_acc = s_acc * pv[u] + ev[u];
                }
                continue;
              }
#pragma unroll
              for (int u = 8 * i; u < 8 * i + 8; u++) {
                if (u < m) {
                  if (up & (1u << u)) s_acc = s_acc * pv[u];
                  s_acc = s_acc + ev[u];
                }
              }
            }
          }
        }
      }
    }
    XL_MARK(3);
    __syncthreads();  // the chunk's LDS is reused by the next one
  }
  XL_MARK(4);
#ifdef XA_STATS
  if (wave == 0 && lane == 0 && h == 0)
  {
    printf("xa_stats pos %d batches %d slow %d moves %d (cycles %lld) serial scores %u\n", n_keys - 1, st_batches, st_slow,
           st_moves, (long long)(__builtin_amdgcn_s_memtime() - st_t0), g_xa_serial);
    g_xa_serial = 0u;
  }
#endif
  if (wave == NWV && lane == 0) s_sacc = s_acc == 0.0f ? 0.0f : 1.0f / s_acc;
  __syncthreads();
  if (wave < NWV) {
    const int d = wave * 64 + lane;
    const float o = h2f(v16) * s_sacc;  // model.cpp:543-547
    const size_t zo = (size_t)z * a.n_head * HD;
    a.out[zo + (size_t)h * HD + d] = o;
    q8_block_store(o, true, a.xq + (zo + (size_t)h * HD + wave * 64) / 32 + (lane >> 5), lane & 31);
  }
}

// every f32 bit pattern: the hardware f32 -> f16 conversion (round to nearest even) against the reference's
// f32_to_f16 (gguf.cpp:68-95, f2h_ggml) -- the exact attention's accumulator chain uses the hardware one
__global__ void f16_selftest_kernel(unsigned long long* out) {
  const uint64_t n = 1ull << 32;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const float f = __uint_as_float((uint32_t)i);
    const uint16_t hw = f2h(f), sw = f2h_ggml(f);
    if (hw != sw) {
      const bool nan = f != f;
      atomicAdd(out + (nan ? 1 : 0), 1ull);
      if (!nan) atomicMin(out + 2, (unsigned long long)i);
    }
  }
}

// speculative chain vs the serial one: work-group g fills n = 2560 floats from a hash of (g, i) with a
// per-group scale and a sprinkling of large values (wide dynamic range: fallbacks happen), out[0] += mismatches,
// out[1] += fallback segments
__global__ __launch_bounds__(256) void chain_selftest_kernel(unsigned* out) {
  __shared__ __attribute__((aligned(16))) float s[2560];
  __shared__ float s_ref;
  const int g = blockIdx.x;
  const float scale = exp2f((float)((g * 37) % 41) - 20.0f);
  for (int i = threadIdx.x; i < 2560; i += 256) {
    uint32_t h = (uint32_t)(g * 2654435761u) ^ (uint32_t)(i * 2246822519u);
    h ^= h >> 15; h *= 0x2c1b3c6du; h ^= h >> 12; h *= 0x297a2d39u; h ^= h >> 15;
    float v = ((float)(h & 0xFFFFFF) / 16777216.0f - 0.5f) * scale;
    if ((h >> 24) == 0x7F && (g & 3) == 0) v *= 4096.0f;  // rare large terms: the chain jumps past the window
    s[i] = v;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const float r = xl_chain(s, 2560);
    if (threadIdx.x == 0) s_ref = r;
  }
  __syncthreads();
  const float v = (g & 1) ? xl_chain_spec2<4>(s, 2560, out + 1) : xl_chain_spec<4>(s, 2560, out + 1);
  if (threadIdx.x == 0 && __float_as_uint(v) != __float_as_uint(s_ref)) atomicAdd(out, 1u);
}

// ---------------------------------------------------------------------------
// Batched exact prefill (exact.h launch_exact_norm_batch / launch_exact_gemm / launch_exact_attn_batch): the
// prompt's tokens layer by layer, T at a time.  Every (row, token) keeps the reference's own chains: the same
// per-token norm chains as the decode prologues, the eight fma chains of ops.cpp:364-399 per (row, token), the
// per-token causal attention of model.cpp:478-550.  Only the order in which independent chains run changes.
// ---------------------------------------------------------------------------

// the q row (q heads) or the k row + V append (kv heads) of one token: blockIdx.x < n_head a q head, else kv head
// blockIdx.x - n_head; blockIdx.y the token (pos = *d_pos + y).  The same norm chain, rope and roundings as the
// decode scores kernel's xa_row / xa_row2 (bit-identical: every speculative chain equals the serial one)
template <int HD>
__global__ __launch_bounds__(64) void xattn_qk_batch_kernel(XAttnArgs a) {
  constexpr int EPL = HD / 64, CPL = EPL / 2;
  __shared__ __attribute__((aligned(16))) float s_x[HD];
  const int r = blockIdx.x, z = blockIdx.y, lane = threadIdx.x;
  const int pos = *a.d_pos + z;
  const float* qkv = a.qkv + (size_t)z * a.qkv_stride;
  const float* cs = a.rope_cs + (size_t)pos * HD;
  float c[CPL], sn[CPL];
#pragma unroll
  for (int k = 0; k < CPL; k++) {
    const float2 t = reinterpret_cast<const float2*>(cs)[lane + 64 * k];
    c[k] = t.x;
    sn[k] = t.y;
  }
  XaRow<HD> in;
  float rr[EPL];
  if (r < a.n_head) {  // the query: norm, rope, scale, the score's f16 rounding (model.cpp:762-794, 507)
    xa_load<HD>(in, qkv + (size_t)r * HD, a.q_norm_w);
    xa_row<HD>(in, c, sn, a.eps, s_x, rr);
    uint16_t* qh = a.qh + ((size_t)z * a.n_head + r) * HD;
#pragma unroll
    for (int k = 0; k < EPL; k++) qh[lane + 64 * k] = f2h_ggml(rr[k] * a.attn_scale);
    return;
  }
  const int hkv = r - a.n_head;  // the key: norm + rope, K and V appended at pos (model.cpp:440-474)
  float vrow[EPL];
  xa_load<HD>(in, qkv + a.k_off + (size_t)hkv * HD, a.k_norm_w);
#pragma unroll
  for (int k = 0; k < EPL; k++) vrow[k] = qkv[a.v_off + (size_t)hkv * HD + lane + 64 * k];
  xa_row<HD>(in, c, sn, a.eps, s_x, rr);
  uint16_t* kc = a.k_cache + ((size_t)hkv * a.max_ctx + pos) * HD;
  uint16_t* vc = a.v_cache + ((size_t)hkv * a.max_ctx + pos) * HD;
  int kcode = 31;
  uint32_t kmag = 0;
#pragma unroll
  for (int k = 0; k < EPL; k++) {
    const uint16_t kbits = f2h_ggml(rr[k]), vbits = f2h_ggml(vrow[k]);
    kc[lane + 64 * k] = kbits;
    vc[lane + 64 * k] = vbits;
    a.vt[xa_vt_index<HD>(hkv, lane + 64 * k, pos, a.vt_stride)] = vbits;
    kcode = min(kcode, xa_exp_code(kbits));
    kmag = max(kmag, (uint32_t)(kbits & 0x7FFFu));
  }
  kcode = xa_wave_min(kcode);
  kmag = (uint32_t)xa_wave_max((int)kmag);
  if (lane == 0 && a.kmeta) a.kmeta[(size_t)hkv * a.max_ctx + pos] = ((uint32_t)kcode << 16) | kmag;
}

// embedding rows as the decode's embed_norm_kernel reads them (model.cpp:240-344; F16 / F32 / Q8_0 tables)
__device__ __forceinline__ float xp_deq(uint32_t type, const uint8_t* row, int i) {
  switch (type) {
    case T_F16: return h2f(reinterpret_cast<const uint16_t*>(row)[i]);
    case T_F32: return reinterpret_cast<const float*>(row)[i];
    case T_Q8_0: {
      const uint8_t* b = row + (i / 32) * 34;
      return h2f((uint16_t)(b[0] | (b[1] << 8))) * (float)(int8_t)b[2 + (i & 31)];
    }
    default: return 0.0f;
  }
}

// One work-group per token: the residual step + norm + quantize_row_q8_0 of the decode's XL_PRE prologue
// (model.cpp:843-858 then 346-357, ops.cpp:116-139), or the embedding row * sqrt(n_embd) + attn_norm
// (model.cpp:709-736), each serial chain by xl_sumsq; the Q8_0 blocks to global memory.
template <int K4>
__global__ __launch_bounds__(256) void xp_norm_kernel(XpNormArgs a) {
  constexpr int NW = 4, T = 256;
  extern __shared__ float4 s_n4[];
  float* s_a = reinterpret_cast<float*>(s_n4);
  float* s_b = s_a + a.n;
  __shared__ float s_scale[2];
  const int t = threadIdx.x, z = blockIdx.x;
  const int n = a.n, n4 = n >> 2, nb = n / 32;
  float4* resid4 = reinterpret_cast<float4*>(a.resid + (size_t)z * n);
  const float4* wn4 = reinterpret_cast<const float4*>(a.w_next);
  float4 hv[K4], yv[K4], wv[K4], nv[K4];
  const bool embed = a.table != nullptr;
  const uint8_t* row = embed ? a.table + (size_t)a.tokens[z] * a.row_bytes : nullptr;
#pragma unroll
  for (int k = 0; k < K4; k++) {
    const int i = min(k * T + t, n4 - 1);
    if (embed) {
      hv[k] = make_float4(xp_deq(a.type, row, 4 * i) * a.emb_scale, xp_deq(a.type, row, 4 * i + 1) * a.emb_scale,
                          xp_deq(a.type, row, 4 * i + 2) * a.emb_scale, xp_deq(a.type, row, 4 * i + 3) * a.emb_scale);
    } else {
      hv[k] = resid4[i];
      yv[k] = reinterpret_cast<const float4*>(a.y + (size_t)z * n)[i];
      wv[k] = reinterpret_cast<const float4*>(a.w_post)[i];
    }
    nv[k] = wn4[i];
  }
  auto own = [&](int k) { return k * T + t < n4; };
  if (!embed) {
#pragma unroll
    for (int k = 0; k < K4; k++)
      if (own(k)) reinterpret_cast<float4*>(s_a)[k * T + t] = yv[k];
    __syncthreads();
    const float sc1 = xl_rms_scale(xl_sumsq<NW>(s_a, n, &s_scale[0]), n, a.eps);
#pragma unroll
    for (int k = 0; k < K4; k++) {  // the post norm, then the residual add
      hv[k].x = hv[k].x + (sc1 * yv[k].x) * wv[k].x;
      hv[k].y = hv[k].y + (sc1 * yv[k].y) * wv[k].y;
      hv[k].z = hv[k].z + (sc1 * yv[k].z) * wv[k].z;
      hv[k].w = hv[k].w + (sc1 * yv[k].w) * wv[k].w;
    }
  }
#pragma unroll
  for (int k = 0; k < K4; k++)
    if (own(k)) {
      reinterpret_cast<float4*>(s_b)[k * T + t] = hv[k];
      resid4[k * T + t] = hv[k];
    }
  __syncthreads();
  const float sc2 = xl_rms_scale(xl_sumsq<NW>(s_b, n, &s_scale[1]), n, a.eps);
  XBlock* xq = a.xq + (size_t)z * nb;
#pragma unroll
  for (int k = 0; k < K4; k++) {  // run_norm's (scale * x) * w, then the octet's Q8_0 block (8 lanes, a float4 each)
    const bool ok = own(k);       // (whole octets: n4 and T are multiples of 8)
    const float4 x = make_float4((sc2 * hv[k].x) * nv[k].x, (sc2 * hv[k].y) * nv[k].y, (sc2 * hv[k].z) * nv[k].z,
                                 (sc2 * hv[k].w) * nv[k].w);
    float amax = ok ? fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w))) : 0.0f;
    amax = fmaxf(amax, dpp_f<DPP_QUAD_1032>(amax));
    amax = fmaxf(amax, dpp_f<DPP_QUAD_2301>(amax));
    amax = fmaxf(amax, dpp_f<DPP_ROW_HALF_MIRROR>(amax));
    const float dd = amax / 127.0f;
    const float id = dd != 0.0f ? 1.0f / dd : 0.0f;
    const int q0 = nearest_int_fma(x.x, id), q1 = nearest_int_fma(x.y, id), q2 = nearest_int_fma(x.z, id),
              q3 = nearest_int_fma(x.w, id);
    const uint32_t w = (uint32_t)(q0 & 0xFF) | ((uint32_t)(q1 & 0xFF) << 8) | ((uint32_t)(q2 & 0xFF) << 16) |
                       ((uint32_t)(q3 & 0xFF) << 24);
    int sum = q0 + q1 + q2 + q3;
    sum += __shfl_xor(sum, 1);
    sum += __shfl_xor(sum, 2);
    sum += __shfl_xor(sum, 4);
    const int i4 = k * T + t, b = i4 >> 3, sl = i4 & 7;
    if (ok) {
      reinterpret_cast<uint32_t*>(xq + b)[sl] = w;  // words 0-3: q[0..15] (lo), 4-7: q[16..31] (hi)
      if (sl == 0) {
        xq[b].d = h2f(f2h_ggml(dd));
        xq[b].nsum8 = -8 * sum;
      }
    }
  }
}

// rows x tokens of an XL weight: a work-group owns 64 rows x 64 tokens, thread (rg, tg) = (t % 16, t / 16) the
// rows 4 rg .. and tokens 4 tg .., each (row, token) with the reference's eight accumulators over the blocks in
// order (ops.cpp:380-395: acc_j = fma(d, (float)isum_j, acc_j), d = f16(w.d) * f16(x.d)), then hsum_float_8.
// The integer dots take the nibbles as 16 (n - 8) (one shift-and-xor, signed bytes) and the scale as d / 16:
// 16 isum and d / 16 are exact rescalings, so every fma sees the reference's product d * isum.  Chunks of
// XG_CB blocks of the rows' weights and the tokens' quants are staged in LDS.
// The integer dot's conversion and the fma run packed (XG_PK, default): sdot4 accumulates onto the bits of 1.5 x 2^23,
// so the int32 result read as a float is 12582912 + 16 isum exactly (|16 isum| < 2^22), one v_pk_add_f32 removes the
// offset for two accumulators (exact: Sterbenz) and one v_pk_fma_f32 updates both (each lane's fma rounds once, as
// fmaf): 17 instead of 25 VALU issues per (row, token, block).  -DXG_NO_PK: the scalar form.
constexpr int XG_R = 64, XG_T = 64, XG_CB = 16;
typedef float xg_f2 __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256, 2) void xp_gemm_kernel(const uint4* __restrict__ wq, const uint2* __restrict__ wd,
                                                         int rows, int nb, const XBlock* __restrict__ x, int T,
                                                         float* __restrict__ out, int ldo, XBlock* __restrict__ hq) {
  __shared__ __attribute__((aligned(16))) uint4 s_w[XG_CB][XG_R];      // the row's 16 nibble bytes of the block
  __shared__ float s_wd[XG_CB][XG_R];                                   // f16(w.d) / 16
  __shared__ __attribute__((aligned(16))) uint4 s_x[XG_CB][XG_T][2];   // the token's 32 quants
  __shared__ float s_xd[XG_CB][XG_T];
  const int t = threadIdx.x, rg = t & 15, tg = t >> 4;
  const int row0 = blockIdx.x * XG_R, tok0 = blockIdx.y * XG_T, ng = nb >> 2;
  xg_f2 acc[4][4][4];  // accumulators s (x) and s + 4 (y) of (row 4 rg + i, token 4 tg + j)
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++)
#pragma unroll
      for (int s = 0; s < 4; s++) acc[i][j][s] = xg_f2{0.0f, 0.0f};
  for (int c0 = 0; c0 < nb; c0 += XG_CB) {
    // weights: XL qs[g][row][jj] = word jj of the group's 4 blocks -> s_w[block][row] words jj
#pragma unroll
    for (int m = 0; m < 4; m++) {
      const int i = t + 256 * m, jj = i & 3, R = (i >> 2) & 63, gl = i >> 8, g = (c0 >> 2) + gl;
      const bool in = g < ng && row0 + R < rows;
      const uint4 v = in ? wq[((size_t)g * rows + row0 + R) * 4 + jj] : make_uint4(0, 0, 0, 0);
      reinterpret_cast<uint32_t*>(&s_w[4 * gl + 0][R])[jj] = v.x;
      reinterpret_cast<uint32_t*>(&s_w[4 * gl + 1][R])[jj] = v.y;
      reinterpret_cast<uint32_t*>(&s_w[4 * gl + 2][R])[jj] = v.z;
      reinterpret_cast<uint32_t*>(&s_w[4 * gl + 3][R])[jj] = v.w;
    }
    {
      const int R = t & 63, gl = t >> 6, g = (c0 >> 2) + gl;
      const bool in = g < ng && row0 + R < rows;
      const uint2 dv = in ? wd[(size_t)g * rows + row0 + R] : make_uint2(0, 0);
      s_wd[4 * gl + 0][R] = h2f((uint16_t)(dv.x & 0xFFFFu)) * 0.0625f;
      s_wd[4 * gl + 1][R] = h2f((uint16_t)(dv.x >> 16)) * 0.0625f;
      s_wd[4 * gl + 2][R] = h2f((uint16_t)(dv.y & 0xFFFFu)) * 0.0625f;
      s_wd[4 * gl + 3][R] = h2f((uint16_t)(dv.y >> 16)) * 0.0625f;
    }
    // the tokens' quants and scales
#pragma unroll
    for (int m = 0; m < 8; m++) {
      const int i = t + 256 * m, half = i & 1, tk = (i >> 1) & 63, bl = i >> 7, b = c0 + bl, tok = tok0 + tk;
      const bool in = b < nb && tok < T;
      const XBlock* xb = x + (size_t)(in ? tok : 0) * nb + (in ? b : 0);
      s_x[bl][tk][half] = in ? (half ? *reinterpret_cast<const uint4*>(&xb->hi) : *reinterpret_cast<const uint4*>(&xb->lo))
                             : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int m = 0; m < 4; m++) {
      const int i = t + 256 * m, tk = i & 63, bl = i >> 6, b = c0 + bl, tok = tok0 + tk;
      const bool in = b < nb && tok < T;
      s_xd[bl][tk] = in ? x[(size_t)tok * nb + b].d : 0.0f;
    }
    __syncthreads();
    const int nbc = min(XG_CB, nb - c0);
    for (int bl = 0; bl < nbc; bl++) {
      uint32_t xl[4][4], xh[4][4];  // the four tokens' quants (lo: elements 0-15, hi: 16-31), one row at a time below
      float xd[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint4 a0 = s_x[bl][4 * tg + j][0], a1 = s_x[bl][4 * tg + j][1];
        xl[j][0] = a0.x; xl[j][1] = a0.y; xl[j][2] = a0.z; xl[j][3] = a0.w;
        xh[j][0] = a1.x; xh[j][1] = a1.y; xh[j][2] = a1.z; xh[j][3] = a1.w;
        xd[j] = s_xd[bl][4 * tg + j];
      }
#pragma unroll
      for (int i = 0; i < 4; i++) {
        const uint4 w = s_w[bl][4 * rg + i];
        const float dw = s_wd[bl][4 * rg + i];
        const uint32_t w4[4] = {w.x, w.y, w.z, w.w};
        uint32_t wl[4], wh[4];
#pragma unroll
        for (int s = 0; s < 4; s++) {
          wl[s] = ((w4[s] << 4) & 0xF0F0F0F0u) ^ 0x80808080u;  // 16 (low nibble - 8) per byte
          wh[s] = (w4[s] & 0xF0F0F0F0u) ^ 0x80808080u;         // 16 (high nibble - 8)
        }
#pragma unroll
        for (int j = 0; j < 4; j++) {
          const float d = dw * xd[j];
#pragma unroll
          for (int s = 0; s < 4; s++) {
#ifdef XG_NO_PK
            acc[i][j][s].x = fmaf(d, (float)sdot4((int)wl[s], (int)xl[j][s], 0), acc[i][j][s].x);
            acc[i][j][s].y = fmaf(d, (float)sdot4((int)wh[s], (int)xh[j][s], 0), acc[i][j][s].y);
#else
            constexpr int MAGIC = 0x4B400000;  // 1.5 x 2^23
            const xg_f2 p = xg_f2{__int_as_float(sdot4((int)wl[s], (int)xl[j][s], MAGIC)),
                                  __int_as_float(sdot4((int)wh[s], (int)xh[j][s], MAGIC))} -
                            xg_f2{12582912.0f, 12582912.0f};
            acc[i][j][s] = __builtin_elementwise_fma(xg_f2{d, d}, p, acc[i][j][s]);
#endif
          }
        }
      }
    }
    __syncthreads();  // the chunk's LDS is refilled next
  }
  // hsum_float_8 (ops.cpp:324-330): ((a0 + a4) + (a2 + a6)) + ((a1 + a5) + (a3 + a7))
  float r[4][4];
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const xg_f2* v = acc[i][j];  // v[s].x = a_s, v[s].y = a_(s + 4)
      r[i][j] = ((v[0].x + v[0].y) + (v[2].x + v[2].y)) + ((v[1].x + v[1].y) + (v[3].x + v[3].y));
    }
  if (!hq) {
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int row = row0 + 4 * rg + i, tok = tok0 + 4 * tg + j;
        if (row < rows && tok < T) out[(size_t)tok * ldo + row] = r[i][j];
      }
    return;
  }
  // GELU epilogue (gelu32 rows: 32 gate rows, then their 32 up rows): GELU(gate) * up of the work-group's 32
  // hidden units for each token (model.cpp:892-899), quantized as one Q8_0 block per token (ops.cpp:116-139)
  float* s_r = reinterpret_cast<float*>(&s_x[0][0][0]);  // [64 rows][65]
#pragma unroll
  for (int i = 0; i < 4; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) s_r[(4 * rg + i) * 65 + 4 * tg + j] = r[i][j];
  __syncthreads();
  const int u = t & 31, nh = rows / 64;
  for (int tk = t >> 5; tk < XG_T; tk += 8) {
    const int tok = tok0 + tk;
    const float v = gelu_mul1<true>(s_r[u * 65 + tk], s_r[(32 + u) * 65 + tk]);
    q8_block_store(v, tok < T, hq + (size_t)min(tok, T - 1) * nh + blockIdx.x, u);
  }
}

}  // namespace

void exact_selftest_chain(unsigned* host_out2) {
  unsigned* d = nullptr;
  LLMI_HIP(hipMalloc(&d, 8));
  LLMI_HIP(hipMemset(d, 0, 8));
  hipLaunchKernelGGL(chain_selftest_kernel, dim3(8192), dim3(256), 0, 0, d);
  LLMI_HIP(hipGetLastError());
  LLMI_HIP(hipMemcpy(host_out2, d, 8, hipMemcpyDeviceToHost));
  LLMI_HIP(hipFree(d));
}

void exact_selftest_f16(unsigned long long* host_out3) {
  unsigned long long* d = nullptr;
  LLMI_HIP(hipMalloc(&d, 24));
  const unsigned long long init[3] = {0, 0, ~0ull};
  LLMI_HIP(hipMemcpy(d, init, 24, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(f16_selftest_kernel, dim3(4096), dim3(256), 0, 0, d);
  LLMI_HIP(hipGetLastError());
  LLMI_HIP(hipMemcpy(host_out3, d, 24, hipMemcpyDeviceToHost));
  LLMI_HIP(hipFree(d));
}

bool xl_supported(const DevWeight& w) {
  return w.type == T_Q4_0 && !w.slab && w.cols % 128 == 0 && w.rows > 0;
}

XlWeight make_xl_weight(const XlSrc& src, hipStream_t s) {
  if (src.n < 1 || src.n > 3 || (src.gelu32 && src.n != 2)) throw std::runtime_error("xl: bad sources");
  const int cols = src.w[0]->cols;
  int rows = 0;
  size_t bytes = 0;
  for (int k = 0; k < src.n; k++) {
    if (!xl_supported(*src.w[k]) || src.w[k]->cols != cols) throw std::runtime_error("xl: unsupported weight");
    rows += src.w[k]->rows;
    bytes += src.w[k]->bytes;
  }
  if (src.gelu32 && (src.w[0]->rows != src.w[1]->rows || src.w[0]->rows % 32)) throw std::runtime_error("xl: gelu32 rows");
  if (rows % 16) throw std::runtime_error("xl: rows % 16 != 0");
  XlWeight x;
  x.rows = rows;
  x.nb = cols / 32;
  x.bytes = bytes;
  const size_t ng = (size_t)x.nb / 4;
  x.qs = static_cast<uint4*>(dev_alloc(ng * rows * 64 + 256));
  x.d = static_cast<uint2*>(dev_alloc(ng * rows * 8 + 256));
  auto Q = [&](int k) { return k < src.n ? reinterpret_cast<const uint4*>(src.w[k]->qs) : nullptr; };
  auto D = [&](int k) { return k < src.n ? src.w[k]->d : nullptr; };
  auto R = [&](int k) { return k < src.n ? src.w[k]->rows : 0; };
  const size_t n = ng * rows * 4;
  hipLaunchKernelGGL(xl_repack_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, Q(0), D(0), R(0), Q(1), D(1),
                     R(1), Q(2), D(2), src.gelu32, rows, x.nb, x.qs, x.d);
  LLMI_HIP(hipGetLastError());
  return x;
}

void free_xl_weight(XlWeight& w) {
  dev_free(w.qs);
  dev_free(w.d);
  w = XlWeight{};
}

bool exact_attn_supported(int head_dim, int n_head, int n_head_kv) {
  return (head_dim == 256 || head_dim == 128) && n_head_kv > 0 && n_head % n_head_kv == 0;
}

void launch_exact_attn(const XAttnArgs& a, hipStream_t s) {
  if (!exact_attn_supported(a.head_dim, a.n_head, a.n_head_kv) || !a.scores || !a.xq)
    throw std::runtime_error("exact attention: unsupported shape");
  if (a.head_dim == 256) {
    hipLaunchKernelGGL(xattn_scores_kernel<256>, dim3(a.n_head, XA_NSPLIT + 1), dim3(64), 0, s, a);
    hipLaunchKernelGGL(xattn_accum_kernel<256>, dim3(a.n_head), dim3(320), 0, s, a);
  } else {
    hipLaunchKernelGGL(xattn_scores_kernel<128>, dim3(a.n_head, XA_NSPLIT + 1), dim3(64), 0, s, a);
    hipLaunchKernelGGL(xattn_accum_kernel<128>, dim3(a.n_head), dim3(192), 0, s, a);
  }
  LLMI_HIP(hipGetLastError());
}

void launch_exact_gemv(const XlWeight& w, const XlArgs& a_in, int role, hipStream_t s) {
  XlArgs a = a_in;
  if (!w.qs || w.nb % 4 || w.rows % 16) throw std::runtime_error("exact gemv: bad weight");
  if (role != XL_PLAIN && a.n != w.nb * 32) throw std::runtime_error("exact gemv: input length != cols");
  if (role == XL_GELU && w.rows % 64) throw std::runtime_error("exact gemv: GELU rows % 64 != 0");
  if ((role == XL_PRE || role == XL_GELU) && a.n > 24 * 256) throw std::runtime_error("exact gemv: n > 6144");
  const size_t xe = (size_t)w.nb * 64 + (size_t)w.nb * 4;
  const size_t lds = xe + (role == XL_PLAIN ? 0 : (size_t)2 * a.n * 4);
  if (lds > 64 * 1024) throw std::runtime_error("exact gemv: activation exceeds LDS");
  auto go = [&](auto kern, int nw, int lpr = 4) {
    const int rpg = 64 / lpr * nw;  // rows per work-group
    const unsigned grid = (unsigned)((w.rows + rpg - 1) / rpg);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * nw), lds, s, w.qs, w.d, w.rows, w.nb, a);
  };
  // PRE / GELU: each thread holds 4 XL_K4 elements of the residual-step operands in registers
  const bool k3_2 = a.n <= 12 * 128, k3_4 = a.n <= 12 * 256;
  switch (role) {
    // PLAIN / QUANT: one wave per work-group, few of them (a row group per wave), so the registers go to weight
    // chunks in flight: 4 x 8 groups (32 KB per wave)
    case XL_PLAIN:  // the dots in parallel, the chains by one wave (exact_plain_split_kernel)
      hipLaunchKernelGGL(exact_plain_split_kernel, dim3((unsigned)(w.rows / XS_ROWS)), dim3(256), xe, s, w.qs, w.d, w.rows,
                         w.nb, a);
      break;
    case XL_QUANT: go(exact_gemv_kernel<1, XL_QUANT, 1, 4>, 1); break;
    case XL_PRE:
      if (k3_2) go(exact_gemv_kernel<2, XL_PRE, 3, 2>, 2);
      else if (k3_4 && w.rows % 16 == 0 && getenv("LLMI_XL_PRE_ROWS") == nullptr)  // (dev A/B: the 64-row form)
        hipLaunchKernelGGL((exact_gemv_kernel<4, XL_PRE, 3, 2, 4, 16>), dim3((unsigned)(w.rows / 16)), dim3(256), lds, s, w.qs,
                           w.d, w.rows, w.nb, a);
      else if (k3_4) go(exact_gemv_kernel<4, XL_PRE, 3, 2>, 4);
      else go(exact_gemv_kernel<4, XL_PRE, 6, 2>, 4);
      break;
    case XL_GELU:
      if (k3_4) go(exact_gemv_kernel<4, XL_GELU, 3, 1>, 4);  // (one chunk in flight: its operands return sooner)
      else go(exact_gemv_kernel<4, XL_GELU, 6, 2>, 4);
      break;
    default: throw std::runtime_error("exact gemv: bad role");
  }
  LLMI_HIP(hipGetLastError());
}


void launch_exact_attn_batch(const XAttnArgs& a, int T, hipStream_t s) {
  if (!exact_attn_supported(a.head_dim, a.n_head, a.n_head_kv) || !a.scores || !a.xq || !a.qh || !a.vt || T <= 0)
    throw std::runtime_error("exact attention batch: unsupported shape");
  const int nr = a.n_head + a.n_head_kv;
  if (a.head_dim == 256) {
    hipLaunchKernelGGL(xattn_qk_batch_kernel<256>, dim3(nr, T), dim3(64), 0, s, a);
    hipLaunchKernelGGL((xattn_scores_kernel<256, true>), dim3(a.n_head, XA_NSPLIT, T), dim3(64), 0, s, a);
    hipLaunchKernelGGL((xattn_accum_kernel<256, true>), dim3(a.n_head, T), dim3(320), 0, s, a);
  } else {
    hipLaunchKernelGGL(xattn_qk_batch_kernel<128>, dim3(nr, T), dim3(64), 0, s, a);
    hipLaunchKernelGGL((xattn_scores_kernel<128, true>), dim3(a.n_head, XA_NSPLIT, T), dim3(64), 0, s, a);
    hipLaunchKernelGGL((xattn_accum_kernel<128, true>), dim3(a.n_head, T), dim3(192), 0, s, a);
  }
  LLMI_HIP(hipGetLastError());
}

void launch_exact_norm_batch(const XpNormArgs& a, int T, hipStream_t s) {
  if (a.n % 128 || a.n > 6 * 4 * 256 || T <= 0 || !a.resid || !a.w_next || !a.xq || (!a.table && (!a.y || !a.w_post)))
    throw std::runtime_error("exact norm batch: bad arguments");
  if (a.table && a.type != T_F16 && a.type != T_F32 && a.type != T_Q8_0)
    throw std::runtime_error("exact norm batch: embedding table type");
  const size_t lds = (size_t)2 * a.n * 4;
  if (a.n <= 3 * 4 * 256) hipLaunchKernelGGL(xp_norm_kernel<3>, dim3(T), dim3(256), lds, s, a);
  else hipLaunchKernelGGL(xp_norm_kernel<6>, dim3(T), dim3(256), lds, s, a);
  LLMI_HIP(hipGetLastError());
}

void launch_exact_gemm(const XlWeight& w, const XBlock* x, int T, float* out, int ldo, XBlock* hq, hipStream_t s) {
  if (!w.qs || w.nb % 4 || w.rows % 16 || T <= 0 || !x || (!out && !hq)) throw std::runtime_error("exact gemm: bad arguments");
  if (hq && w.rows % 64) throw std::runtime_error("exact gemm: GELU rows % 64 != 0");
  const dim3 grid((unsigned)((w.rows + XG_R - 1) / XG_R), (unsigned)((T + XG_T - 1) / XG_T));
  hipLaunchKernelGGL(xp_gemm_kernel, grid, dim3(256), 0, s, w.qs, w.d, w.rows, w.nb, x, T, out, ldo, hq);
  LLMI_HIP(hipGetLastError());
}

}  // namespace llmi
