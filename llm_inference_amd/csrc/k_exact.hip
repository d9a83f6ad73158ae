// k_exact.hip -- the exact-order engine's Q4_0 GEMVs (exact.h): the
// reference's operation order (ops.cpp:364-399 mat_vec_mul_q4_0, ops.cpp:28-43
// rms_norm, ops.cpp:116-139 quantize_row_q8_0, model.cpp:843-924 residual /
// norm / GELU) with the weights streamed like the fast path's layer GEMVs.
#include <stdexcept>

#include "exact.h"

namespace llmi {

namespace {

constexpr int XL_P = 8;  // groups (4 blocks each) per chunk of loads

__device__ __forceinline__ float xl_rms_scale(float sum, int n, double eps) {  // ops.cpp:37-38
  return 1.0f / sqrtf((float)((double)(sum / (float)n) + eps));
}

// The reference's serial sum of squares (ops.cpp:33-36, contracted to fma by its build) over s[0..n) in LDS.
// Every lane of the calling wave runs the same chain (broadcast reads); the reads of the next 32 values are
// issued before the current 32 are consumed, so the chain is the fma latency alone (~4 cycles a step).
__device__ __forceinline__ float xl_chain(const float* s, int n) {
  const float4* s4 = reinterpret_cast<const float4*>(s);
  const int n4 = n >> 2, nfull = n4 & ~7;
  float sum = 0.0f;
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

template <int NW, int ROLE>
__global__ __launch_bounds__(NW * 64) void exact_gemv_kernel(const uint4* __restrict__ wq, const uint2* __restrict__ wd,
                                                             int rows, int nb, XlArgs a) {
  extern __shared__ int4 s_dyn[];
  int4* s_xe = s_dyn;                                                // [nb][4]
  float* s_xd = reinterpret_cast<float*>(s_dyn + (size_t)nb * 4);    // [nb]
  float* s_a = s_xd + nb;                                            // PRE: [n] y, then the XBlocks
  float* s_b = s_a + a.n;                                            // PRE: [n] h
  __shared__ float s_scale[2];
  __shared__ float s_rows[NW * 16];
  constexpr int T = NW * 64;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int rl = lane >> 2, jj = lane & 3;
  const int row = (blockIdx.x * NW + wave) * 16 + rl;
  const int ng = nb >> 2;
  // weight stream: issued first, the activation prologue runs while it is in flight
  const __amdgpu_buffer_rsrc_t rq = buf_rsrc(wq, (uint32_t)((size_t)ng * rows * 64));
  const __amdgpu_buffer_rsrc_t rd = buf_rsrc(wd, (uint32_t)((size_t)ng * rows * 8));
  const bool row_ok = row < rows;
  const int voq = row_ok ? (row * 4 + jj) * 16 : (1 << 30), vod = row_ok ? row * 8 : (1 << 30);
  const int sq = rows * 64, sd = rows * 8;
  XlChunk ca, cb;
  xl_load(ca, rq, rd, voq, vod, sq, sd, 0, ng);
  xl_load(cb, rq, rd, voq, vod, sq, sd, XL_P, ng);

  // ---- the activation: XE entries + scales in LDS ----
  if constexpr (ROLE == XL_PLAIN) {
    for (int i = t; i < nb * 4; i += T) {
      const XBlock& xb = a.xb[i >> 2];
      s_xe[i] = xe_entry(xb, i & 3);
      if ((i & 3) == 0) s_xd[i >> 2] = xb.d;
    }
  } else {
    const int n = a.n;
    XBlock* s_xb = reinterpret_cast<XBlock*>(s_a);
    if constexpr (ROLE == XL_QUANT) {
      for (int i = t; i < n; i += T) s_b[i] = a.y[i];
    } else {
      if (a.y) {
        for (int i = t; i < n; i += T) s_a[i] = a.y[i];
        __syncthreads();
        if (wave == 0) {
          const float sc = xl_rms_scale(xl_chain(s_a, n), n, a.eps);
          if (lane == 0) s_scale[0] = sc;
        }
        __syncthreads();
        const float sc1 = s_scale[0];
        for (int i = t; i < n; i += T) {  // model.cpp:843-858: the post norm, then the residual add
          const float h = a.resid_in[i] + (sc1 * s_a[i]) * a.w_post[i];
          s_b[i] = h;
          if (blockIdx.x == 0) a.resid_out[i] = h;
        }
      } else {
        for (int i = t; i < n; i += T) {
          const float h = a.resid_in[i];
          s_b[i] = h;
          if (blockIdx.x == 0 && a.resid_out != a.resid_in) a.resid_out[i] = h;
        }
      }
      __syncthreads();
      if (wave == 0) {
        const float sc = xl_rms_scale(xl_chain(s_b, n), n, a.eps);
        if (lane == 0) s_scale[1] = sc;
      }
      __syncthreads();
      const float sc2 = s_scale[1];
      for (int i = t; i < n; i += T) {  // run_norm: (scale * x) * w (model.cpp:352-357)
        const float x = (sc2 * s_b[i]) * a.w_next[i];
        s_b[i] = x;
        if (blockIdx.x == 0 && a.xn_out) a.xn_out[i] = x;
      }
    }
    __syncthreads();
    // quantize_row_q8_0 (ops.cpp:116-139): a DPP quad per block
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
  }
  __syncthreads();

  // ---- the rows: every block in order, chunks double-buffered ----
  float lo = 0.0f, hi = 0.0f;
  const float4* s_xd4 = reinterpret_cast<const float4*>(s_xd);
  for (int g0 = 0; g0 < ng; g0 += 2 * XL_P) {
    xl_eat(ca, g0, ng, jj, s_xe, s_xd4, lo, hi);
    if (g0 + 2 * XL_P < ng) xl_load(ca, rq, rd, voq, vod, sq, sd, g0 + 2 * XL_P, ng);
    if (g0 + XL_P >= ng) break;
    xl_eat(cb, g0 + XL_P, ng, jj, s_xe, s_xd4, lo, hi);
    if (g0 + 3 * XL_P < ng) xl_load(cb, rq, rd, voq, vod, sq, sd, g0 + 3 * XL_P, ng);
  }
  // hsum_float_8 (ops.cpp:324-330): ((a0 + a4) + (a2 + a6)) + ((a1 + a5) + (a3 + a7)); lane jj holds a_jj, a_jj+4
  const float t4 = lo + hi;
  const float u = t4 + dpp_f<DPP_QUAD_2301>(t4);  // jj 0: t0 + t2, jj 1: t1 + t3
  const float r = u + dpp_f<DPP_QUAD_1032>(u);    // jj 0: (t0 + t2) + (t1 + t3)
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
    if (jj == 0 && row_ok) a.out[row] = r;
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

}  // namespace

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
  LLMI_HIP(hipMalloc(&x.qs, ng * rows * 64 + 256));
  LLMI_HIP(hipMalloc(&x.d, ng * rows * 8 + 256));
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
  if (w.qs) (void)hipFree(w.qs);
  if (w.d) (void)hipFree(w.d);
  w = XlWeight{};
}

void launch_exact_gemv(const XlWeight& w, const XlArgs& a, int role, hipStream_t s) {
  if (!w.qs || w.nb % 4 || w.rows % 16) throw std::runtime_error("exact gemv: bad weight");
  if (role != XL_PLAIN && a.n != w.nb * 32) throw std::runtime_error("exact gemv: input length != cols");
  if (role == XL_GELU && w.rows % 64) throw std::runtime_error("exact gemv: GELU rows % 64 != 0");
  const size_t xe = (size_t)w.nb * 64 + (size_t)w.nb * 4;
  const size_t lds = xe + (role == XL_PLAIN ? 0 : (size_t)2 * a.n * 4);
  if (lds > 64 * 1024) throw std::runtime_error("exact gemv: activation exceeds LDS");
  auto go = [&](auto kern, int nw) {
    const unsigned grid = (unsigned)((w.rows + 16 * nw - 1) / (16 * nw));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * nw), lds, s, w.qs, w.d, w.rows, w.nb, a);
  };
  switch (role) {
    case XL_PLAIN: go(exact_gemv_kernel<1, XL_PLAIN>, 1); break;
    case XL_QUANT: go(exact_gemv_kernel<1, XL_QUANT>, 1); break;
    case XL_PRE: go(exact_gemv_kernel<2, XL_PRE>, 2); break;
    case XL_GELU: go(exact_gemv_kernel<4, XL_GELU>, 4); break;
    default: throw std::runtime_error("exact gemv: bad role");
  }
  LLMI_HIP(hipGetLastError());
}

}  // namespace llmi
