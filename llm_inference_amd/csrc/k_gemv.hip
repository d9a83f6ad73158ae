// k_gemv.hip -- quantized / f16 GEMV kernels for gfx950 (MI355X).
//
// Two families per weight type:
//   *_exact : the reference's AVX2 operation order, bit-for-bit
//             (Q4_0 ops.cpp:364-399, F16 ops.cpp:541-586, Q8_0 ops.cpp:806-824,
//             Q4_K 643-691, Q6_K 727-770, Q5_0 856-879, BF16 908-917).
//   *_fast  : HBM-streaming kernels.  A wavefront owns R whole rows and walks
//             them as a flat list of (row, block) items, one block per lane
//             per pass, so every weight wave-instruction is one coalesced
//             1 KiB (Q4_0: 64 x 16-B quants) non-temporal load.  All P passes
//             of a chunk are issued before any is consumed (loads in flight,
//             no data-dependent control flow between them); the (row, block)
//             of an item comes from one mul-hi, not a division loop.  Q4_0 and
//             Q8_0 block dots are exact integer v_dot4; only the fp32
//             accumulation across blocks and the wave reduction reassociate.
#include "kernels.h"

namespace llmi {


// ===========================================================================
// Q4_0 x Q8_0
// ===========================================================================
// exact: 8 lanes per row; lane j keeps the reference's AVX2 accumulator j
// (integer dot of elements 4j..4j+3 of every block, fma over blocks in order),
// then the hsum_float_8 tree ((a0+a4)+(a2+a6))+((a1+a5)+(a3+a7)).
__global__ __launch_bounds__(256) void gemv_q4_0_exact(const uint32_t* __restrict__ qs,
                                                       const uint16_t* __restrict__ wd, int rows, int nb,
                                                       const XBlock* __restrict__ xb, float* __restrict__ out) {
  const int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const int row = gl >> 3, j = gl & 7;
  float acc = 0.0f;
  if (row < rows) {
    const uint32_t* q = qs + (size_t)row * nb * 4 + (j & 3);
    const uint16_t* d = wd + (size_t)row * nb;
    for (int b = 0; b < nb; b++) {
      const uint32_t w = q[(size_t)b * 4];
      const int nib = j < 4 ? nib_lo(w) : nib_hi(w);
      const int xv = reinterpret_cast<const int*>(xb + b)[j];
      const int isum = sdot4(nib, xv, sdot4((int)0xF8F8F8F8u, xv, 0));  // sum (nib-8)*x
      const float sc = h2f(d[b]) * xb[b].d;
      acc = fmaf(sc, (float)isum, acc);
    }
  }
  float t = acc + __shfl_xor(acc, 4);
  t = t + __shfl_xor(t, 2);
  t = t + __shfl_xor(t, 1);
  if (row < rows && j == 0) out[row] = t;
}

template <int R>
__device__ __forceinline__ void acc_add(float (&acc)[R], int r, float v) {
#pragma unroll
  for (int k = 0; k < R; k++) acc[k] += (k == r) ? v : 0.0f;
}

template <int R>
__device__ __forceinline__ void rows_out(float (&acc)[R], int lane, int row0, int nrows, float* out) {
#pragma unroll
  for (int k = 0; k < R; k++) {
    const float s = wave_sum(acc[k]);
    if (lane == 0 && k < nrows) out[row0 + k] = s;
  }
}

// fast: R rows per wave, P passes (64 items each) issued per chunk.
template <int R, int P>
__global__ __launch_bounds__(256) void gemv_q4_0_fast(const uint4* __restrict__ qs, const uint16_t* __restrict__ wd,
                                                      int rows, int nb, uint32_t magic, const XBlock* __restrict__ xb,
                                                      float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (row0 >= rows) return;
  const int nrows = min(R, rows - row0);
  const int total = nrows * nb;
  const uint4* qw = qs + (size_t)row0 * nb;
  const uint16_t* dw = wd + (size_t)row0 * nb;
  float acc[R];
#pragma unroll
  for (int k = 0; k < R; k++) acc[k] = 0.0f;
  for (int c0 = 0; c0 < total; c0 += 64 * P) {
    uint4 q[P];
    float sw[P];
    int rr[P], bb[P];
#pragma unroll
    for (int p = 0; p < P; p++) {
      const int f = c0 + p * 64 + lane;
      const int fc = f < total ? f : 0;
      const int r = div_by_magic(fc, magic);
      rr[p] = f < total ? r : R;
      bb[p] = fc - r * nb;
      q[p] = ld_nt(qw + fc);
      sw[p] = h2f(ld_nt16(dw + fc));
    }
#pragma unroll
    for (int p = 0; p < P; p++) {
      const int4* xp = reinterpret_cast<const int4*>(xb + bb[p]);
      const int4 x0 = xp[0], x1 = xp[1], x2 = xp[2];
      int is = x2.y;  // nsum8
      is = sdot4(nib_lo(q[p].x), x0.x, is);
      is = sdot4(nib_lo(q[p].y), x0.y, is);
      is = sdot4(nib_lo(q[p].z), x0.z, is);
      is = sdot4(nib_lo(q[p].w), x0.w, is);
      is = sdot4(nib_hi(q[p].x), x1.x, is);
      is = sdot4(nib_hi(q[p].y), x1.y, is);
      is = sdot4(nib_hi(q[p].z), x1.z, is);
      is = sdot4(nib_hi(q[p].w), x1.w, is);
      acc_add<R>(acc, rr[p], (sw[p] * __int_as_float(x2.x)) * (float)is);
    }
  }
  rows_out<R>(acc, lane, row0, nrows, out);
}

// ===========================================================================
// Q8_0 x Q8_0
// ===========================================================================
// exact: one thread per row, single fp32 chain (ops.cpp:812-821):
//   row = fmaf((float)dot * d_w, d_x, row)
__global__ __launch_bounds__(256) void gemv_q8_0_exact(const int4* __restrict__ qs, const uint16_t* __restrict__ wd,
                                                       int rows, int nb, const XBlock* __restrict__ xb,
                                                       float* __restrict__ out) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= rows) return;
  float sum = 0.0f;
  for (int b = 0; b < nb; b++) {
    const int4 w0 = qs[((size_t)row * nb + b) * 2], w1 = qs[((size_t)row * nb + b) * 2 + 1];
    const int4 x0 = xb[b].lo, x1 = xb[b].hi;
    int dot = sdot4(w0.x, x0.x, 0);
    dot = sdot4(w0.y, x0.y, dot); dot = sdot4(w0.z, x0.z, dot); dot = sdot4(w0.w, x0.w, dot);
    dot = sdot4(w1.x, x1.x, dot); dot = sdot4(w1.y, x1.y, dot); dot = sdot4(w1.z, x1.z, dot);
    dot = sdot4(w1.w, x1.w, dot);
    sum = fmaf((float)dot * h2f(wd[(size_t)row * nb + b]), xb[b].d, sum);
  }
  out[row] = sum;
}

template <int R, int P>
__global__ __launch_bounds__(256) void gemv_q8_0_fast(const int4* __restrict__ qs, const uint16_t* __restrict__ wd,
                                                      int rows, int nb, uint32_t magic, const XBlock* __restrict__ xb,
                                                      float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (row0 >= rows) return;
  const int nrows = min(R, rows - row0);
  const int total = nrows * nb;
  const int4* qw = qs + (size_t)row0 * nb * 2;
  const uint16_t* dw = wd + (size_t)row0 * nb;
  float acc[R];
#pragma unroll
  for (int k = 0; k < R; k++) acc[k] = 0.0f;
  for (int c0 = 0; c0 < total; c0 += 64 * P) {
    int4 w0[P], w1[P];
    float sw[P];
    int rr[P], bb[P];
#pragma unroll
    for (int p = 0; p < P; p++) {
      const int f = c0 + p * 64 + lane;
      const int fc = f < total ? f : 0;
      const int r = div_by_magic(fc, magic);
      rr[p] = f < total ? r : R;
      bb[p] = fc - r * nb;
      w0[p] = ld_nt(qw + 2 * fc);
      w1[p] = ld_nt(qw + 2 * fc + 1);
      sw[p] = h2f(ld_nt16(dw + fc));
    }
#pragma unroll
    for (int p = 0; p < P; p++) {
      const int4* xp = reinterpret_cast<const int4*>(xb + bb[p]);
      const int4 x0 = xp[0], x1 = xp[1], x2 = xp[2];
      int dot = sdot4(w0[p].x, x0.x, 0);
      dot = sdot4(w0[p].y, x0.y, dot); dot = sdot4(w0[p].z, x0.z, dot); dot = sdot4(w0[p].w, x0.w, dot);
      dot = sdot4(w1[p].x, x1.x, dot); dot = sdot4(w1[p].y, x1.y, dot); dot = sdot4(w1[p].z, x1.z, dot);
      dot = sdot4(w1[p].w, x1.w, dot);
      acc_add<R>(acc, rr[p], (sw[p] * __int_as_float(x2.x)) * (float)dot);
    }
  }
  rows_out<R>(acc, lane, row0, nrows, out);
}

// ===========================================================================
// F16 (logits)
// ===========================================================================
typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ half2_t as_h2(uint32_t v) { return __builtin_bit_cast(half2_t, v); }

// exact: 4 lanes per row (lane l = AVX2 accumulator register sum[l], 8 fp32
// lanes m each), chunk loop in order, then (S0+S1)+(S2+S3), t_m = V_m+V_m+4,
// (t0+t1)+(t2+t3), then the serial scalar tail (ops.cpp:557-583).
__global__ __launch_bounds__(256) void gemv_f16_exact(const uint4* __restrict__ w, int rows, int cols,
                                                      const uint16_t* __restrict__ x16, float* __restrict__ out) {
  const int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const int row = gl >> 2, l = gl & 3;
  float s[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const int np = cols & ~31;
  if (row < rows) {
    const uint16_t* wr = reinterpret_cast<const uint16_t*>(w) + (size_t)row * cols;
    for (int k = 0; k < np; k += 32) {
      uint16_t wv[8], xv[8];
      if ((cols & 7) == 0) {
        *reinterpret_cast<uint4*>(wv) = *reinterpret_cast<const uint4*>(wr + k + 8 * l);
        *reinterpret_cast<uint4*>(xv) = *reinterpret_cast<const uint4*>(x16 + k + 8 * l);
      } else {
#pragma unroll
        for (int m = 0; m < 8; m++) { wv[m] = wr[k + 8 * l + m]; xv[m] = x16[k + 8 * l + m]; }
      }
#pragma unroll
      for (int m = 0; m < 8; m++) s[m] = fmaf(h2f(wv[m]), h2f(xv[m]), s[m]);
    }
  }
  float v[8];
#pragma unroll
  for (int m = 0; m < 8; m++) {
    const float a = s[m] + __shfl_xor(s[m], 1);  // l0: S0+S1, l2: S2+S3
    v[m] = a + __shfl_xor(a, 2);                 // l0: (S0+S1)+(S2+S3)
  }
  if (row < rows && l == 0) {
    const float t0 = v[0] + v[4], t1 = v[1] + v[5], t2 = v[2] + v[6], t3 = v[3] + v[7];
    float r = (t0 + t1) + (t2 + t3);
    const uint16_t* wr = reinterpret_cast<const uint16_t*>(w) + (size_t)row * cols;
    for (int k = np; k < cols; k++) r = fmaf(h2f(wr[k]), h2f(x16[k]), r);
    out[row] = r;
  }
}

__device__ __forceinline__ float dot8_f16(uint4 w, uint4 x, float acc) {
  acc = __builtin_amdgcn_fdot2(as_h2(w.x), as_h2(x.x), acc, false);
  acc = __builtin_amdgcn_fdot2(as_h2(w.y), as_h2(x.y), acc, false);
  acc = __builtin_amdgcn_fdot2(as_h2(w.z), as_h2(x.z), acc, false);
  acc = __builtin_amdgcn_fdot2(as_h2(w.w), as_h2(x.w), acc, false);
  return acc;
}

// fast, cols % 512 == 0 (P = cols/512 passes per row): x chunks held in
// registers for the whole kernel, grid-stride over rows, argmax folded in.
template <int P>
__global__ __launch_bounds__(256) void gemv_f16_fast_rows(const uint4* __restrict__ w, int rows,
                                                          const uint4* __restrict__ x16, float* __restrict__ out,
                                                          unsigned long long* __restrict__ amax_key) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * 4;
  uint4 xr[P];
#pragma unroll
  for (int p = 0; p < P; p++) xr[p] = x16[p * 64 + lane];
  float best = -INFINITY;
  int best_i = 0x7fffffff;
  for (int row = wave; row < rows; row += nwaves) {
    const uint4* wr = w + (size_t)row * (P * 64);
    uint4 wv[P];
#pragma unroll
    for (int p = 0; p < P; p++) wv[p] = ld_nt(wr + p * 64 + lane);
    float acc = 0.0f;
#pragma unroll
    for (int p = 0; p < P; p++) acc = dot8_f16(wv[p], xr[p], acc);
    acc = wave_sum(acc);
    if (lane == 0) {
      out[row] = acc;
      if (acc > best) { best = acc; best_i = row; }
    }
  }
  if (amax_key != nullptr && lane == 0 && best_i != 0x7fffffff) atomicMax(amax_key, argmax_key(best, best_i));
}

// fast, cols % 128 == 0 and cols <= 6144 (the logits tables: 1152/2560/3840/
// 5376 wide): P full passes of 64 lanes x 8 halves + a partial pass of T
// lanes (T = 16/32/48).  x in registers for the whole kernel; grid-stride
// over rows with the next row's loads in flight while the current row is
// reduced (the row loop is otherwise one memory latency per row); argmax
// folded in.
template <int P, int T>
__global__ __launch_bounds__(256) void gemv_f16_rows_pipe(const uint4* __restrict__ w, int rows,
                                                          const uint4* __restrict__ x16, float* __restrict__ out,
                                                          unsigned long long* __restrict__ amax_key) {
  constexpr int NP = P + (T ? 1 : 0);
  constexpr int RU4 = P * 64 + T;  // uint4 per row
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * 4;
  const int tl = T ? lane % (T ? T : 64) : lane;  // partial pass: lanes >= T re-read lane % T and drop it
  uint4 xr[NP];
#pragma unroll
  for (int p = 0; p < NP; p++) xr[p] = x16[p * 64 + (p < P ? lane : tl)];
  auto load_row = [&](uint4 (&v)[NP], int row) {
    const uint4* wr = w + (size_t)row * RU4;
#pragma unroll
    for (int p = 0; p < NP; p++) v[p] = ld_nt(wr + p * 64 + (p < P ? lane : tl));
  };
  float best = -INFINITY;
  int best_i = 0x7fffffff;
  int row = wave;
  uint4 cur[NP];
  load_row(cur, min(row, rows - 1));
  for (; row < rows; row += nwaves) {
    uint4 nxt[NP];
    load_row(nxt, min(row + nwaves, rows - 1));  // clamped: the last one re-reads a row just read
    float acc = 0.0f;
#pragma unroll
    for (int p = 0; p < P; p++) acc = dot8_f16(cur[p], xr[p], acc);
    if constexpr (T != 0) {
      const float t = dot8_f16(cur[P], xr[P], 0.0f);
      acc += lane < T ? t : 0.0f;
    }
    acc = wave_sum(acc);
    if (lane == 0) {
      out[row] = acc;
      if (acc > best) { best = acc; best_i = row; }
    }
#pragma unroll
    for (int p = 0; p < NP; p++) cur[p] = nxt[p];
  }
  if (amax_key != nullptr && lane == 0 && best_i != 0x7fffffff) atomicMax(amax_key, argmax_key(best, best_i));
}

// fast, general cols (cols % 8 == 0): flat (row, chunk) items like Q4_0.
template <int R, int P>
__global__ __launch_bounds__(256) void gemv_f16_fast(const uint4* __restrict__ w, int rows, int nc, uint32_t magic,
                                                     const uint4* __restrict__ x16, float* __restrict__ out,
                                                     unsigned long long* __restrict__ amax_key) {
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (row0 >= rows) return;
  const int nrows = min(R, rows - row0);
  const int total = nrows * nc;
  const uint4* wr = w + (size_t)row0 * nc;
  float acc[R];
#pragma unroll
  for (int k = 0; k < R; k++) acc[k] = 0.0f;
  for (int c0 = 0; c0 < total; c0 += 64 * P) {
    uint4 wv[P];
    int rr[P], cc[P];
#pragma unroll
    for (int p = 0; p < P; p++) {
      const int f = c0 + p * 64 + lane;
      const int fc = f < total ? f : 0;
      const int r = div_by_magic(fc, magic);
      rr[p] = f < total ? r : R;
      cc[p] = fc - r * nc;
      wv[p] = ld_nt(wr + fc);
    }
#pragma unroll
    for (int p = 0; p < P; p++) acc_add<R>(acc, rr[p], dot8_f16(wv[p], x16[cc[p]], 0.0f));
  }
  float best = -INFINITY;
  int best_i = 0x7fffffff;
#pragma unroll
  for (int k = 0; k < R; k++) {
    const float sum = wave_sum(acc[k]);
    if (lane == 0 && k < nrows) {
      out[row0 + k] = sum;
      if (sum > best) { best = sum; best_i = row0 + k; }
    }
  }
  if (amax_key != nullptr && lane == 0 && best_i != 0x7fffffff) atomicMax(amax_key, argmax_key(best, best_i));
}

// ===========================================================================
// K-quants, Q5_0, BF16: exact single-chain kernels (one thread per row)
// ===========================================================================
__device__ __forceinline__ uint16_t ld16(const uint8_t* p) { return (uint16_t)p[0] | ((uint16_t)p[1] << 8); }
__device__ __forceinline__ void scale_min_k4(int j, const uint8_t* q, int& d, int& m) {  // ops.cpp:633-641
  if (j < 4) { d = q[j] & 63; m = q[j + 4] & 63; }
  else { d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4); m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4); }
}

__global__ __launch_bounds__(256) void gemv_q4_k_exact(const uint8_t* __restrict__ wq, int rows, int nb,
                                                       const uint8_t* __restrict__ xk, float* __restrict__ out) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= rows) return;
  float sum = 0.0f;
  for (int b = 0; b < nb; b++) {
    const uint8_t* blk = wq + ((size_t)row * nb + b) * 144;
    const uint8_t* xbk = xk + (size_t)b * 292;
    const float xdv = *reinterpret_cast<const float*>(xbk);
    const float d = h2f(ld16(blk)) * xdv;
    const float mn = h2f(ld16(blk + 2)) * xdv;
    const uint8_t* q4 = blk + 16;
    const int8_t* q8 = reinterpret_cast<const int8_t*>(xbk + 4);
    const int16_t* bs = reinterpret_cast<const int16_t*>(xbk + 260);
    int is = 0;
    for (int j = 0; j < 256; j += 64) {
      int s, m;
      scale_min_k4(is, blk + 4, s, m);
      float d1 = d * (float)s, m1 = mn * (float)m;
      int a = 0;
      for (int l = 0; l < 32; ++l) a += (q4[l] & 0xF) * q8[l];
      sum = sum + fmaf((float)a, d1, -(m1 * (float)(bs[is * 2] + bs[is * 2 + 1])));
      scale_min_k4(is + 1, blk + 4, s, m);
      d1 = d * (float)s; m1 = mn * (float)m;
      a = 0;
      for (int l = 0; l < 32; ++l) a += (q4[l] >> 4) * q8[l + 32];
      sum = sum + fmaf((float)a, d1, -(m1 * (float)(bs[(is + 1) * 2] + bs[(is + 1) * 2 + 1])));
      q4 += 32; q8 += 64; is += 2;
    }
  }
  out[row] = sum;
}

__global__ __launch_bounds__(256) void gemv_q6_k_exact(const uint8_t* __restrict__ wq, int rows, int nb,
                                                       const uint8_t* __restrict__ xk, float* __restrict__ out) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= rows) return;
  float sum = 0.0f;
  for (int b = 0; b < nb; b++) {
    const uint8_t* blk = wq + ((size_t)row * nb + b) * 210;
    const uint8_t* xbk = xk + (size_t)b * 292;
    const float d = h2f(ld16(blk + 208)) * *reinterpret_cast<const float*>(xbk);
    const uint8_t* ql = blk;
    const uint8_t* qh = blk + 128;
    const int8_t* sc = reinterpret_cast<const int8_t*>(blk + 192);
    const int8_t* xq = reinterpret_cast<const int8_t*>(xbk + 4);
    for (int n = 0; n < 256; n += 128) {
      int part = 0;
      for (int l = 0; l < 32; ++l) {
        const int is = l / 16;
        const int q1 = (int8_t)((ql[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
        const int q2 = (int8_t)((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
        const int q3 = (int8_t)((ql[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
        const int q4 = (int8_t)((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
        part += sc[is + 0] * q1 * xq[l + 0];
        part += sc[is + 2] * q2 * xq[l + 32];
        part += sc[is + 4] * q3 * xq[l + 64];
        part += sc[is + 6] * q4 * xq[l + 96];
      }
      sum = fmaf((float)part, d, sum);
      ql += 64; qh += 32; sc += 8; xq += 128;
    }
  }
  out[row] = sum;
}

// ---- fast K-quant GEMVs: row-bound lanes (R rows per wave, L = 64/R lanes
// per row), one 32-element sub-block per lane per pass, integer 4-way dots
// against the Q8_K activation (ops.cpp:142-178), fp32 per-lane sums reduced
// across the row's lanes (the reference's order is kept only by the exact
// kernels above).
__device__ __forceinline__ int ld_i32u(const uint8_t* p) {  // 4-byte aligned
  return *reinterpret_cast<const int*>(p);
}

template <int R>
__device__ __forceinline__ float kq_row_sum(float v) {  // sum over the row's L lanes, result in every lane of it
  constexpr int L = 64 / R;
  if constexpr (L >= 2) v += dpp_f<DPP_QUAD_1032>(v);
  if constexpr (L >= 4) v += dpp_f<DPP_QUAD_2301>(v);
  if constexpr (L >= 8) v += dpp_f<DPP_ROW_HALF_MIRROR>(v);
  if constexpr (L >= 16) v += dpp_f<DPP_ROW_MIRROR>(v);
  if constexpr (L >= 32) v += __shfl_xor(v, 16);
  if constexpr (L >= 64) v += __shfl_xor(v, 32);
  return v;
}

// Q4_K (ops.cpp:614-697): 144-B super-blocks of 256: d, dmin (f16), 12 bytes of
// 6-bit scales/mins, 128 bytes of nibbles (sub-block 2c: low nibbles of
// qs[32c..32c+31], 2c+1: their high nibbles)
template <int R>
__global__ __launch_bounds__(256) void gemv_q4_k_fast(const uint8_t* __restrict__ wq, int rows, int nsb,
                                                      const uint8_t* __restrict__ xk, float* __restrict__ out) {
  constexpr int L = 64 / R;
  const int lane = threadIdx.x & 63, wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int row = wave * R + lane / L, j = lane % L;
  const uint8_t* wr = wq + (size_t)min(row, rows - 1) * nsb * 144;
  float acc = 0.0f;
  for (int u = j; u < nsb * 8; u += L) {
    const int b = u >> 3, sb = u & 7;
    const uint8_t* blk = wr + (size_t)b * 144;
    const uint4 hdr = *reinterpret_cast<const uint4*>(blk);
    const uint4 q0 = *reinterpret_cast<const uint4*>(blk + 16 + 32 * (sb >> 1));
    const uint4 q1 = *reinterpret_cast<const uint4*>(blk + 32 + 32 * (sb >> 1));
    const uint8_t* xb = xk + (size_t)b * 292;
    const float xd = *reinterpret_cast<const float*>(xb);
    const uint8_t* xq = xb + 4 + 32 * sb;
    const int16_t* bs = reinterpret_cast<const int16_t*>(xb + 260);
    const int sh = (sb & 1) * 4;
    int a = 0;
    a = sdot4((int)((q0.x >> sh) & 0x0F0F0F0Fu), ld_i32u(xq + 0), a);
    a = sdot4((int)((q0.y >> sh) & 0x0F0F0F0Fu), ld_i32u(xq + 4), a);
    a = sdot4((int)((q0.z >> sh) & 0x0F0F0F0Fu), ld_i32u(xq + 8), a);
    a = sdot4((int)((q0.w >> sh) & 0x0F0F0F0Fu), ld_i32u(xq + 12), a);
    a = sdot4((int)((q1.x >> sh) & 0x0F0F0F0Fu), ld_i32u(xq + 16), a);
    a = sdot4((int)((q1.y >> sh) & 0x0F0F0F0Fu), ld_i32u(xq + 20), a);
    a = sdot4((int)((q1.z >> sh) & 0x0F0F0F0Fu), ld_i32u(xq + 24), a);
    a = sdot4((int)((q1.w >> sh) & 0x0F0F0F0Fu), ld_i32u(xq + 28), a);
    uint8_t scb[12];
    __builtin_memcpy(scb, reinterpret_cast<const uint8_t*>(&hdr) + 4, 12);
    int sc, mn;
    scale_min_k4(sb, scb, sc, mn);
    const float d = h2f((uint16_t)(hdr.x & 0xFFFF)) * xd, dmin = h2f((uint16_t)(hdr.x >> 16)) * xd;
    acc += fmaf((float)a, d * (float)sc, -((dmin * (float)mn) * (float)(bs[2 * sb] + bs[2 * sb + 1])));
  }
  acc = kq_row_sum<R>(acc);
  if (j == 0 && row < rows) out[row] = acc;
}

// Q6_K (ops.cpp:699-785): 210-B super-blocks: ql[128], qh[64], int8 scales[16]
// (one per 16 elements), d (f16).  Lane sub-block m (elements 32m..32m+31):
// half n = m / 4, quarter jq = m % 4 -> ql[64n + 32(jq & 1) + l] nibble jq >= 2,
// qh[32n + l] bits 2jq..2jq+1, scales[8n + 2jq + (l >= 16)].
template <int R>
__global__ __launch_bounds__(256) void gemv_q6_k_fast(const uint8_t* __restrict__ wq, int rows, int nsb,
                                                      const uint8_t* __restrict__ xk, float* __restrict__ out) {
  constexpr int L = 64 / R;
  const int lane = threadIdx.x & 63, wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int row = wave * R + lane / L, j = lane % L;
  const uint8_t* wr = wq + (size_t)min(row, rows - 1) * nsb * 210;
  float acc = 0.0f;
  for (int u = j; u < nsb * 8; u += L) {
    const int b = u >> 3, m = u & 7, n = m >> 2, jq = m & 3;
    const uint8_t* blk = wr + (size_t)b * 210;  // 210-B blocks: 2-byte alignment only
    const uint8_t* ql = blk + 64 * n + 32 * (jq & 1);
    const uint8_t* qh = blk + 128 + 32 * n;
    const int8_t* sc = reinterpret_cast<const int8_t*>(blk + 192 + 8 * n + 2 * jq);
    const uint8_t* xb = xk + (size_t)b * 292;
    const float xd = *reinterpret_cast<const float*>(xb);
    const uint8_t* xq = xb + 4 + 32 * m;
    const int lsh = (jq >> 1) * 4, hsh = 2 * jq;
    // 210-B blocks are only 2-byte aligned: the 32 bytes of ql / qh come from 9
    // aligned dwords each, realigned with v_alignbyte (72 byte loads -> 18
    // dword loads; the 9th dword stays inside the block)
    const uint32_t* lw4 = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(ql) & ~(uintptr_t)3);
    const uint32_t* hw4 = reinterpret_cast<const uint32_t*>(reinterpret_cast<uintptr_t>(qh) & ~(uintptr_t)3);
    const uint32_t lal = (uint32_t)(reinterpret_cast<uintptr_t>(ql) & 3), hal = (uint32_t)(reinterpret_cast<uintptr_t>(qh) & 3);
    uint32_t lraw[9], hraw[9];
#pragma unroll
    for (int k = 0; k < 9; k++) {
      lraw[k] = lw4[k];
      hraw[k] = hw4[k];
    }
    int dot[2] = {0, 0};
#pragma unroll
    for (int w4 = 0; w4 < 8; w4++) {
      const uint32_t lw = __builtin_amdgcn_alignbyte(lraw[w4 + 1], lraw[w4], lal);
      const uint32_t hw = __builtin_amdgcn_alignbyte(hraw[w4 + 1], hraw[w4], hal);
      const uint32_t v = ((lw >> lsh) & 0x0F0F0F0Fu) | (((hw >> hsh) & 0x03030303u) << 4);  // 0..63 per byte
      const int q = (int)((v + 0x60606060u) ^ 0x80808080u);                                   // - 32 per byte
      dot[w4 >> 2] = sdot4(q, ld_i32u(xq + 4 * w4), dot[w4 >> 2]);
    }
    acc = fmaf((float)(sc[0] * dot[0] + sc[1] * dot[1]), h2f((uint16_t)(blk[208] | (blk[209] << 8))) * xd, acc);
  }
  acc = kq_row_sum<R>(acc);
  if (j == 0 && row < rows) out[row] = acc;
}

__global__ __launch_bounds__(256) void gemv_q5_0_exact(const uint8_t* __restrict__ wq, int rows, int nb,
                                                       const float* __restrict__ x, float* __restrict__ out) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= rows) return;
  float sum = 0.0f;
  for (int b = 0; b < nb; b++) {
    const uint8_t* blk = wq + ((size_t)row * nb + b) * 22;
    const float d = h2f(ld16(blk));
    const uint32_t qh = (uint32_t)blk[2] | ((uint32_t)blk[3] << 8) | ((uint32_t)blk[4] << 16) | ((uint32_t)blk[5] << 24);
    for (int i = 0; i < 16; ++i) {
      const uint8_t ql = blk[6 + i];
      const int q0 = (ql & 0x0F) | (((qh >> (i + 0)) & 1) << 4);
      const int q1 = (ql >> 4) | (((qh >> (i + 16)) & 1) << 4);
      sum = fmaf(d * (float)(q0 - 16), x[b * 32 + i], sum);
      sum = fmaf(d * (float)(q1 - 16), x[b * 32 + i + 16], sum);
    }
  }
  out[row] = sum;
}

// fast Q5_0 (ops.cpp:840-893 arithmetic, f32 x: d * (q - 16) * x per element): R rows per wave as a
// flat (row, block) item list like the Q8_0 kernel, one 22-B GGUF block per lane per pass (eleven 2-B
// loads: the blocks are 2-B aligned), the block's 32 products summed in the lane in element order, then
// the fp32 sums across blocks and lanes reassociated (fast mode)
template <int R, int P>
__global__ __launch_bounds__(256) void gemv_q5_0_fast(const uint16_t* __restrict__ wq, int rows, int nb, uint32_t magic,
                                                      const float* __restrict__ x, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int row0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (row0 >= rows) return;
  const int nrows = min(R, rows - row0);
  const int total = nrows * nb;
  const uint16_t* qw = wq + (size_t)row0 * nb * 11;
  float acc[R];
#pragma unroll
  for (int k = 0; k < R; k++) acc[k] = 0.0f;
  for (int c0 = 0; c0 < total; c0 += 64 * P) {
    uint16_t blk[P][11];
    int rr[P], bb[P];
#pragma unroll
    for (int p = 0; p < P; p++) {
      const int f = c0 + p * 64 + lane;
      const int fc = f < total ? f : 0;
      const int r = div_by_magic(fc, magic);
      rr[p] = f < total ? r : R;
      bb[p] = fc - r * nb;
#pragma unroll
      for (int k = 0; k < 11; k++) blk[p][k] = __builtin_nontemporal_load(qw + (size_t)fc * 11 + k);
    }
#pragma unroll
    for (int p = 0; p < P; p++) {
      const float d = h2f(blk[p][0]);
      const uint32_t qh = (uint32_t)blk[p][1] | ((uint32_t)blk[p][2] << 16);
      const float4* xv = reinterpret_cast<const float4*>(x + bb[p] * 32);
      float s = 0.0f;
#pragma unroll
      for (int i4 = 0; i4 < 4; i4++) {  // elements 4 i4 .. 4 i4 + 3 and 16 + the same
        const float4 xl = xv[i4], xh = xv[4 + i4];
        const float xa[4] = {xl.x, xl.y, xl.z, xl.w}, xb[4] = {xh.x, xh.y, xh.z, xh.w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
          const int i = 4 * i4 + e;
          const uint32_t qb = (blk[p][3 + (i >> 1)] >> (8 * (i & 1))) & 0xFF;  // byte i of the nibbles
          const int q0 = (int)(qb & 0x0F) | (int)(((qh >> i) & 1) << 4);
          const int q1 = (int)(qb >> 4) | (int)(((qh >> (i + 16)) & 1) << 4);
          s = fmaf(d * (float)(q0 - 16), xa[e], s);
          s = fmaf(d * (float)(q1 - 16), xb[e], s);
        }
      }
      acc_add<R>(acc, rr[p], s);
    }
  }
  rows_out<R>(acc, lane, row0, nrows, out);
}

__global__ __launch_bounds__(256) void gemv_bf16_exact(const uint16_t* __restrict__ w, int rows, int cols,
                                                       const float* __restrict__ x, float* __restrict__ out) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= rows) return;
  float sum = 0.0f;
  const uint16_t* wr = w + (size_t)row * cols;
  for (int c = 0; c < cols; c++) sum = fmaf(__uint_as_float((uint32_t)wr[c] << 16), x[c], sum);
  out[row] = sum;
}

// BF16 fast (ops.cpp:895-931 restated with reassociated sums): R rows per wave, L = 64 / R lanes per row, each
// lane streams 16-B runs of 8 weights (bf16 -> f32 is a 16-bit shift) against float4 pairs of x, then a
// row-group butterfly.  Rows whose length is not a multiple of 8 take the exact kernel.
template <int R>
__global__ __launch_bounds__(256) void gemv_bf16_fast(const uint4* __restrict__ w, int rows, int nc,
                                                      const float4* __restrict__ x, float* __restrict__ out) {
  constexpr int L = 64 / R;
  const int lane = threadIdx.x & 63, j = lane % L;
  const int row = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R + lane / L;
  const bool ok = row < rows;
  const uint4* wr = w + (size_t)(ok ? row : 0) * nc;
  float a0 = 0.0f, a1 = 0.0f;
  for (int c = j; c < nc; c += L) {
    const uint4 q = ok ? wr[c] : make_uint4(0, 0, 0, 0);
    const float4 x0 = x[2 * c], x1 = x[2 * c + 1];
    a0 = fmaf(__uint_as_float(q.x << 16), x0.x, a0);
    a1 = fmaf(__uint_as_float(q.x & 0xFFFF0000u), x0.y, a1);
    a0 = fmaf(__uint_as_float(q.y << 16), x0.z, a0);
    a1 = fmaf(__uint_as_float(q.y & 0xFFFF0000u), x0.w, a1);
    a0 = fmaf(__uint_as_float(q.z << 16), x1.x, a0);
    a1 = fmaf(__uint_as_float(q.z & 0xFFFF0000u), x1.y, a1);
    a0 = fmaf(__uint_as_float(q.w << 16), x1.z, a0);
    a1 = fmaf(__uint_as_float(q.w & 0xFFFF0000u), x1.w, a1);
  }
  float v = a0 + a1;
#pragma unroll
  for (int o = L / 2; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  if (j == 0 && ok) out[row] = v;
}

// ===========================================================================
// launcher
// ===========================================================================
// smallest R in {1,2,4,8} with R*items a multiple of 64 (full passes), capped
// at 8 (then the last pass is partially masked), and lowered again until the
// grid has a 4-wave work-group per CU (wide rows over few rows, e.g. the 1B
// down projection 1152 x 216 blocks, ran on 36 work-groups at R = 8)
static int rows_per_wave(int items_per_row, int rows) {
  int R = 1;
  while (R < 8 && (R * items_per_row) % 64 != 0) R *= 2;
  while (R > 1 && rows / (4 * R) < 256) R /= 2;
  return R;
}
// passes issued per chunk: all of them up to 8
static int passes_per_chunk(int R, int items_per_row) {
  const int passes = (R * items_per_row + 63) / 64;
  return passes >= 8 ? 8 : (passes >= 6 ? 6 : (passes >= 4 ? passes : (passes == 3 ? 4 : passes)));
}

template <template <int, int> class K>
struct dummy {};

#define LLMI_RP_CASE(KER, R, P, GRID, ...) \
  case R * 16 + P: hipLaunchKernelGGL((KER<R, P>), GRID, dim3(256), 0, s, __VA_ARGS__); break;
#define LLMI_RP_SWITCH(KER, R, P, GRID, ...)                                                                   \
  switch ((R) * 16 + (P)) {                                                                                     \
    LLMI_RP_CASE(KER, 1, 1, GRID, __VA_ARGS__) LLMI_RP_CASE(KER, 1, 2, GRID, __VA_ARGS__)                       \
    LLMI_RP_CASE(KER, 1, 4, GRID, __VA_ARGS__) LLMI_RP_CASE(KER, 1, 5, GRID, __VA_ARGS__)                       \
    LLMI_RP_CASE(KER, 1, 6, GRID, __VA_ARGS__) LLMI_RP_CASE(KER, 1, 7, GRID, __VA_ARGS__)                       \
    LLMI_RP_CASE(KER, 1, 8, GRID, __VA_ARGS__)                                                                  \
    LLMI_RP_CASE(KER, 2, 1, GRID, __VA_ARGS__) LLMI_RP_CASE(KER, 2, 2, GRID, __VA_ARGS__)                       \
    LLMI_RP_CASE(KER, 2, 4, GRID, __VA_ARGS__) LLMI_RP_CASE(KER, 2, 5, GRID, __VA_ARGS__)                       \
    LLMI_RP_CASE(KER, 2, 6, GRID, __VA_ARGS__) LLMI_RP_CASE(KER, 2, 7, GRID, __VA_ARGS__)                       \
    LLMI_RP_CASE(KER, 2, 8, GRID, __VA_ARGS__)                                                                  \
    LLMI_RP_CASE(KER, 4, 1, GRID, __VA_ARGS__) LLMI_RP_CASE(KER, 4, 2, GRID, __VA_ARGS__)                       \
    LLMI_RP_CASE(KER, 4, 4, GRID, __VA_ARGS__) LLMI_RP_CASE(KER, 4, 5, GRID, __VA_ARGS__)                       \
    LLMI_RP_CASE(KER, 4, 6, GRID, __VA_ARGS__) LLMI_RP_CASE(KER, 4, 7, GRID, __VA_ARGS__)                       \
    LLMI_RP_CASE(KER, 4, 8, GRID, __VA_ARGS__)                                                                  \
    LLMI_RP_CASE(KER, 8, 1, GRID, __VA_ARGS__) LLMI_RP_CASE(KER, 8, 2, GRID, __VA_ARGS__)                       \
    LLMI_RP_CASE(KER, 8, 4, GRID, __VA_ARGS__) LLMI_RP_CASE(KER, 8, 5, GRID, __VA_ARGS__)                       \
    LLMI_RP_CASE(KER, 8, 6, GRID, __VA_ARGS__) LLMI_RP_CASE(KER, 8, 7, GRID, __VA_ARGS__)                       \
    LLMI_RP_CASE(KER, 8, 8, GRID, __VA_ARGS__)                                                                  \
    default: throw std::runtime_error("gemv: no kernel for R/P");                                               \
  }

void launch_gemv(const DevWeight& w, const ActBuf& x, float* o, GemvMode mode, hipStream_t s,
                 unsigned long long* amax_key) {
  const int rows = w.rows;
  if (rows == 0) return;
  if (w.slab) throw std::runtime_error("gemv: slab-major weights are read by the layer kernels only");
  switch (w.type) {
    case T_Q4_0:
    case T_Q8_0: {
      const int nb = w.cols / 32;
      if (mode == GEMV_EXACT) {
        if (w.type == T_Q4_0)
          hipLaunchKernelGGL(gemv_q4_0_exact, dim3((rows * 8 + 255) / 256), dim3(256), 0, s,
                             (const uint32_t*)w.qs, w.d, rows, nb, x.q8.xb, o);
        else
          hipLaunchKernelGGL(gemv_q8_0_exact, dim3((rows + 255) / 256), dim3(256), 0, s, (const int4*)w.qs, w.d, rows,
                             nb, x.q8.xb, o);
      } else {
        const int R = rows_per_wave(nb, rows), P = passes_per_chunk(R, nb);
        const dim3 grid((rows + 4 * R - 1) / (4 * R));
        const uint32_t mg = div_magic(nb);
        if (w.type == T_Q4_0) {
          LLMI_RP_SWITCH(gemv_q4_0_fast, R, P, grid, (const uint4*)w.qs, w.d, rows, nb, mg, x.q8.xb, o)
        } else {
          LLMI_RP_SWITCH(gemv_q8_0_fast, R, P, grid, (const int4*)w.qs, w.d, rows, nb, mg, x.q8.xb, o)
        }
      }
      break;
    }
    case T_F16: {
      if (mode == GEMV_EXACT || (w.cols % 8) != 0) {
        hipLaunchKernelGGL(gemv_f16_exact, dim3((rows * 4 + 255) / 256), dim3(256), 0, s, (const uint4*)w.qs, rows,
                           w.cols, x.x16, o);
        // argmax for the exact path is taken by the caller from the logits
      } else if (w.cols % 128 == 0 && w.cols <= 6144) {
        const int u4 = w.cols / 8, P = u4 / 64, T = u4 % 64;  // T in {0, 16, 32, 48}
        // 8 waves per CU for 2560+ wide rows, 16 below (scripts/f16_sweep: the
        // pipelined row loop wants few long-lived waves; 4B/27B tables and
        // their 1/8 vocabulary shards 2-30% faster than 32 waves per CU)
        const int waves = std::min(rows, w.cols >= 2560 ? 256 * 8 : 256 * 16);
        const dim3 grid((waves + 3) / 4);
        switch (P * 4 + T / 16) {
#define LLMI_F16P(PP, TT)                                                                                  \
  case PP * 4 + TT / 16:                                                                                   \
    hipLaunchKernelGGL((gemv_f16_rows_pipe<PP, TT>), grid, dim3(256), 0, s, (const uint4*)w.qs, rows,     \
                       (const uint4*)x.x16, o, amax_key);                                                  \
    break;
#define LLMI_F16P4(PP) LLMI_F16P(PP, 0) LLMI_F16P(PP, 16) LLMI_F16P(PP, 32) LLMI_F16P(PP, 48)
          LLMI_F16P(0, 16) LLMI_F16P(0, 32) LLMI_F16P(0, 48) LLMI_F16P4(1) LLMI_F16P4(2) LLMI_F16P4(3)
          LLMI_F16P4(4) LLMI_F16P4(5) LLMI_F16P4(6) LLMI_F16P4(7) LLMI_F16P4(8) LLMI_F16P4(9) LLMI_F16P4(10)
          LLMI_F16P4(11) LLMI_F16P(12, 0)
#undef LLMI_F16P4
#undef LLMI_F16P
        }
      } else {
        const int nc = w.cols / 8;
        const int R = rows_per_wave(nc, rows), P = passes_per_chunk(R, nc);
        const dim3 grid((rows + 4 * R - 1) / (4 * R));
        LLMI_RP_SWITCH(gemv_f16_fast, R, P, grid, (const uint4*)w.qs, rows, nc, div_magic(nc), (const uint4*)x.x16,
                       o, amax_key)
      }
      break;
    }
    case T_Q4_K:
    case T_Q6_K: {
      const int nsb = w.cols / 256;
      if (mode == GEMV_EXACT) {
        if (w.type == T_Q4_K)
          hipLaunchKernelGGL(gemv_q4_k_exact, dim3((rows + 255) / 256), dim3(256), 0, s, (const uint8_t*)w.qs, rows,
                             nsb, x.q8k, o);
        else
          hipLaunchKernelGGL(gemv_q6_k_exact, dim3((rows + 255) / 256), dim3(256), 0, s, (const uint8_t*)w.qs, rows,
                             nsb, x.q8k, o);
        break;
      }
      // lanes per row: enough for one pass over the row's 8 nsb sub-blocks
      const int units = nsb * 8;
      const int R = units >= 64 ? 1 : units >= 32 ? 2 : units >= 16 ? 4 : 8;
      const dim3 grid((rows + 4 * R - 1) / (4 * R));
#define LLMI_KQ(RR)                                                                                             \
  case RR:                                                                                                      \
    if (w.type == T_Q4_K)                                                                                       \
      hipLaunchKernelGGL(gemv_q4_k_fast<RR>, grid, dim3(256), 0, s, (const uint8_t*)w.qs, rows, nsb, x.q8k, o); \
    else                                                                                                        \
      hipLaunchKernelGGL(gemv_q6_k_fast<RR>, grid, dim3(256), 0, s, (const uint8_t*)w.qs, rows, nsb, x.q8k, o); \
    break;
      switch (R) { LLMI_KQ(1) LLMI_KQ(2) LLMI_KQ(4) LLMI_KQ(8) }
#undef LLMI_KQ
      break;
    }
    case T_Q5_0: {
      const int nb = w.cols / 32;
      if (mode == GEMV_EXACT) {
        hipLaunchKernelGGL(gemv_q5_0_exact, dim3((rows + 255) / 256), dim3(256), 0, s, (const uint8_t*)w.qs, rows, nb,
                           x.xf, o);
      } else {
        const int R = rows_per_wave(nb, rows), P = std::min(4, passes_per_chunk(R, nb));  // 11 VGPRs per pass
        const dim3 grid((rows + 4 * R - 1) / (4 * R));
        switch (R * 16 + P) {
#define LLMI_Q5(RR, PP) \
  case RR * 16 + PP: hipLaunchKernelGGL((gemv_q5_0_fast<RR, PP>), grid, dim3(256), 0, s, (const uint16_t*)w.qs, rows, nb, div_magic(nb), x.xf, o); break;
#define LLMI_Q5R(RR) LLMI_Q5(RR, 1) LLMI_Q5(RR, 2) LLMI_Q5(RR, 4)
          LLMI_Q5R(1) LLMI_Q5R(2) LLMI_Q5R(4) LLMI_Q5R(8)
#undef LLMI_Q5R
#undef LLMI_Q5
          default: throw std::runtime_error("gemv: no Q5_0 kernel for R/P");
        }
      }
      break;
    }
    case T_BF16:
      if (mode == GEMV_EXACT || w.cols % 8 != 0) {
        hipLaunchKernelGGL(gemv_bf16_exact, dim3((rows + 255) / 256), dim3(256), 0, s, (const uint16_t*)w.qs, rows,
                           w.cols, x.xf, o);
      } else {  // lanes per row: the row's 16-B runs in about one pass, at least 8 lanes
        const int nc = w.cols / 8;
        const int R = nc >= 64 ? 1 : nc >= 32 ? 2 : nc >= 16 ? 4 : 8;
        const dim3 grid((rows + 4 * R - 1) / (4 * R));
        switch (R) {
#define LLMI_BF(RR)                                                                                               \
  case RR:                                                                                                        \
    hipLaunchKernelGGL(gemv_bf16_fast<RR>, grid, dim3(256), 0, s, (const uint4*)w.qs, rows, nc, (const float4*)x.xf, o); \
    break;
          LLMI_BF(1) LLMI_BF(2) LLMI_BF(4) LLMI_BF(8)
#undef LLMI_BF
        }
      }
      break;
    default:
      throw std::runtime_error("mat_vec_mul: unsupported tensor type " + std::to_string(w.type));
  }
  LLMI_HIP(hipGetLastError());
}

}  // namespace llmi
