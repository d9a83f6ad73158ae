// k_logits.hip -- greedy token selection by bounded screening + exact rescoring.
//
// The reference picks the next token as the first maximal logit of the F16
// token_embd GEMV (model.cpp:1019-1028 -> mat_vec_mul_fp16 ops.cpp:455-612,
// then std::max_element, main.cpp:193-194).  The fast path's F16 GEMV
// (k_gemv.hip gemv_f16_rows_pipe) reads the whole 1.34 GB table (4B) per
// token.  For the token id alone (the decode loop, llmi_session_enqueue) this
// file gets the SAME id from about half the bytes:
//
//   1. screen_prep: x16 (the f16-rounded final-norm output the F16 GEMV
//      multiplies with) -> Q8 blocks qx = rint(x / dx), dx = amax / 127, and
//      per block the bound weight c_b (below);
//   2. screen_gemv: an int8 copy of the table (per 32-block f16 scale d, made
//      once at load by quantize_table_q8) -> per row approx_r = sum_b d dx
//      isum_b and B_r = sum_b d_rb c_b; hi_r = approx_r + B_r + A is stored,
//      M = max_r (approx_r - B_r - A) is reduced by atomicMax;
//   3. screen_rescore: every row with hi_r >= M is recomputed EXACTLY as
//      gemv_f16_rows_pipe computes it (same lanes, same fdot2 chain, same
//      wave_sum) and reduced to the first-index argmax key (argmax_key).
//
// Why it is the same token: |fast_r - approx_r| <= B_r + A for every row,
// where fast_r is the F16 GEMV's value.  c_b = 0.5 |x_b|_1 (the table's
// rounding to d q, |w - d q| <= d/2 since d is rounded UP from amax/127) +
// 127.5 E_b (E_b = sum |x - dx qx|, |w| <= 127 d) + 127.5 k u (|x_b|_1 + E_b)
// (f32 rounding of both computations, k = n + 32, u = 2^-24), widened by
// 2^-10 and rounded up; A = 2^-14 |x|_1 covers f16/f32 denormal flushing.  If
// r* is the fast path's first maximal row and m attains M, then
// fast_r* >= fast_m >= approx_m - B_m - A = M and approx_r* + B_r* + A >=
// fast_r* >= M: r* (and every row tying with it) is a candidate, and the
// candidates are rescored with the fast path's exact arithmetic.  Worst case
// (e.g. x = 0: every row ties) every row is rescored: slower, never wrong.
// tests/test_logits_screen.py checks ids against the full GEMV, ties included.
#include "session_kernels.h"

namespace llmi {

namespace {

__device__ __forceinline__ float dot8_h(uint4 w, uint4 x, float acc) {  // = k_gemv.hip dot8_f16
  typedef _Float16 h2t __attribute__((ext_vector_type(2)));
  acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, w.x), __builtin_bit_cast(h2t, x.x), acc, false);
  acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, w.y), __builtin_bit_cast(h2t, x.y), acc, false);
  acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, w.z), __builtin_bit_cast(h2t, x.z), acc, false);
  acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, w.w), __builtin_bit_cast(h2t, x.w), acc, false);
  return acc;
}

__device__ __forceinline__ unsigned fkey(float f) {  // order-preserving float -> uint (0 below every float)
  const unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fkey_inv(unsigned k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// ---- load time: the table's int8 copy --------------------------------------
// one thread per (row, 32-block): d = f16 rounded UP from amax / 127 (so
// |q| <= 127 and |w - d q| <= d / 2 even for subnormal scales), q = rint(w / d)
__global__ void quantize_table_q8_kernel(const uint16_t* __restrict__ w, size_t n_blocks, int nb,
                                         uint4* __restrict__ qs, uint16_t* __restrict__ d) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n_blocks) return;
  const uint4* src = reinterpret_cast<const uint4*>(w + i * 32);
  float v[32];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const uint4 u = src[k];
    const uint32_t ws[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      v[k * 8 + 2 * j] = h2f((uint16_t)(ws[j] & 0xFFFF));
      v[k * 8 + 2 * j + 1] = h2f((uint16_t)(ws[j] >> 16));
    }
  }
  float amax = 0.0f;
#pragma unroll
  for (int k = 0; k < 32; k++) amax = fmaxf(amax, fabsf(v[k]));
  const float want = amax / 127.0f;
  uint16_t dh = f2h_ggml(want);
  if (h2f(dh) < want) dh = (uint16_t)(dh + 1);  // positive f16: next representable value up
  const float df = h2f(dh);
  uint32_t packed[8];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    uint32_t p = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      const int q = df > 0.0f ? (int)fminf(127.0f, fmaxf(-127.0f, rintf(v[4 * k + j] / df))) : 0;
      p |= (uint32_t)(q & 0xFF) << (8 * j);
    }
    packed[k] = p;
  }
  qs[2 * i] = make_uint4(packed[0], packed[1], packed[2], packed[3]);
  qs[2 * i + 1] = make_uint4(packed[4], packed[5], packed[6], packed[7]);
  d[i] = dh;
  (void)nb;
}

// ---- per token --------------------------------------------------------------
// one work-group of 1024 threads: DPP quad b < nb quantizes block b of x16 and
// computes c_b in f64 (screen_prep_quad, session_kernels.h); wave 0 sums A and
// resets M.  xs[b] = {qx[32], dx, c_b / 2, 0, 0}, xs[nb].a = A.  The decode
// loop's final norm runs the same two functions on its own x (NormOut::scr),
// so this launch serves only the other callers (time_kernel, unfolded norms).
__global__ __launch_bounds__(1024) void screen_prep_kernel(const uint16_t* __restrict__ x16, int n, ScreenX* __restrict__ xs,
                                                           unsigned* __restrict__ m_key) {
  __shared__ double s_l1[256];
  const int t = threadIdx.x, b = t >> 2, sub = t & 3, nb = n / 32;
  if (b < nb) {  // whole quads in or out together
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; i++) v[i] = h2f(x16[b * 32 + sub * 8 + i]);
    const double l1 = screen_prep_quad(v, sub, n, xs + b);
    if (sub == 0) s_l1[b] = l1;
  }
  __syncthreads();
  if (t < 64) screen_prep_total(s_l1, nb, xs, m_key);
}

// Screening GEMV: half a wave per row (lane j of a half owns 16-B chunks j,
// j + 32, ... of the row's int8 quants = half-blocks), grid-stride over row
// pairs with the next pair's loads in flight (as gemv_f16_rows_pipe).
// CPL: 16-B chunks per lane, ceil(2 nb / 32) (5 for 2560 columns; chunks
// past the row's 2 nb contribute nothing).
template <int CPL, int AHEAD, int LPR = 32>
__global__ __launch_bounds__(256) void screen_gemv_kernel(const uint4* __restrict__ qs, const uint16_t* __restrict__ d,
                                                          int rows, int nb, const ScreenX* __restrict__ xs,
                                                          float* __restrict__ hi, unsigned* __restrict__ m_key) {
  // LPR lanes per row (32: half a wave; 16: a quarter, for short rows -- 1B's 72 chunks fill 5 of 16 lanes'
  // passes instead of 3 of 32 lanes' at 75 %), RPW rows per wave
  static_assert(LPR == 32 || LPR == 16, "lanes per row");
  constexpr int RPW = 64 / LPR;
  const int NC = 2 * nb;  // 16-B chunks per row
  const int lane = threadIdx.x & 63, j = lane % LPR, sub = lane / LPR;
  int grp = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int ngrp = gridDim.x * 4;
  int4 xq[CPL];
  float xd[CPL], xc[CPL];
#pragma unroll
  for (int p = 0; p < CPL; p++) {
    const int c = p * LPR + j, b = min(c, NC - 1) >> 1;
    const bool ok = c < NC;
    const int4* xb = reinterpret_cast<const int4*>(xs + b);
    xq[p] = ok ? ((c & 1) ? xb[1] : xb[0]) : make_int4(0, 0, 0, 0);
    xd[p] = ok ? xs[b].dx : 0.0f;
    xc[p] = ok ? xs[b].c_half : 0.0f;
  }
  const float A = xs[nb].a;
  float mloc = -INFINITY;
  auto load = [&](uint4 (&q)[CPL], uint16_t (&s)[CPL], int r) {
    const uint4* qr = qs + (size_t)r * NC;
    const uint16_t* dr = d + (size_t)r * nb;
#pragma unroll
    for (int p = 0; p < CPL; p++) {
      const int c = min(p * LPR + j, NC - 1);  // clamped (masked by x = 0)
      q[p] = ld_nt(qr + c);
      s[p] = dr[c >> 1];
    }
  };
  auto row_sum = [](float v) { return LPR == 32 ? half_sum(v) : row16_sum(v); };
  int row = RPW * grp + sub;
  uint4 cq[CPL];
  uint16_t cs[CPL];
  load(cq, cs, min(row, rows - 1));
  // AHEAD = 2: a second row group in flight (bytes in flight per CU: MI355X_MICROARCH HBM latency x rate)
  uint4 mq[AHEAD > 1 ? CPL : 1];
  uint16_t ms[AHEAD > 1 ? CPL : 1];
  if constexpr (AHEAD > 1) load(mq, ms, min(row + RPW * ngrp, rows - 1));
  for (; RPW * grp < rows; grp += ngrp, row += RPW * ngrp) {
    uint4 nq[CPL];
    uint16_t ns[CPL];
    load(nq, ns, min(row + RPW * AHEAD * ngrp, rows - 1));
    float ap = 0.0f, bp = 0.0f;
#pragma unroll
    for (int p = 0; p < CPL; p++) {
      int is = 0;
      is = sdot4((int)cq[p].x, xq[p].x, is);
      is = sdot4((int)cq[p].y, xq[p].y, is);
      is = sdot4((int)cq[p].z, xq[p].z, is);
      is = sdot4((int)cq[p].w, xq[p].w, is);
      const float dw = h2f(cs[p]);
      ap += dw * (xd[p] * (float)is);
      bp += dw * xc[p];
    }
    ap = row_sum(ap);
    bp = row_sum(bp) * (1.0f + 0x1p-10f);
    if (j == 0 && row < rows) {
      hi[row] = (ap + bp) + A;
      mloc = fmaxf(mloc, (ap - bp) - A);
    }
#pragma unroll
    for (int p = 0; p < CPL; p++) {
      if constexpr (AHEAD > 1) {
        cq[p] = mq[p];
        cs[p] = ms[p];
        mq[p] = nq[p];
        ms[p] = ns[p];
      } else {
        cq[p] = nq[p];
        cs[p] = ns[p];
      }
    }
  }
  mloc = wave_max(mloc);
  if (lane == 0 && mloc > -INFINITY) atomicMax(m_key, fkey(mloc));
}

// Rescoring: each work-group scans its slice of hi[] for candidates (hi >= M)
// into LDS, then its waves recompute those rows exactly as
// gemv_f16_rows_pipe<P, T> does and fold the first-index argmax key.
template <int P, int T>
__global__ __launch_bounds__(256) void screen_rescore_kernel(const uint4* __restrict__ w, int rows,
                                                             const uint4* __restrict__ x16, const float* __restrict__ hi,
                                                             const unsigned* __restrict__ m_key, int slice,
                                                             unsigned long long* __restrict__ amax_key) {
  constexpr int NP = P + (T ? 1 : 0);
  constexpr int RU4 = P * 64 + T;
  extern __shared__ int s_cand[];  // [slice]
  __shared__ int s_n;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  if (t == 0) s_n = 0;
  __syncthreads();
  const float M = fkey_inv(*m_key);
  const int r0 = blockIdx.x * slice, r1 = min(rows, r0 + slice);
  for (int r = r0 + t; r < r1; r += 256)
    if (hi[r] >= M) s_cand[atomicAdd(&s_n, 1)] = r;
  __syncthreads();
  const int n = s_n;
  if (n == 0) return;
  const int tl = T ? lane % (T ? T : 64) : lane;
  uint4 xr[NP];
#pragma unroll
  for (int p = 0; p < NP; p++) xr[p] = x16[p * 64 + (p < P ? lane : tl)];
  unsigned long long best = 0;
  for (int k = wave; k < n; k += 4) {
    const int row = s_cand[k];
    const uint4* wr = w + (size_t)row * RU4;
    uint4 cur[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) cur[p] = ld_nt(wr + p * 64 + (p < P ? lane : tl));
    float acc = 0.0f;
#pragma unroll
    for (int p = 0; p < P; p++) acc = dot8_h(cur[p], xr[p], acc);
    if constexpr (T != 0) {
      const float tt = dot8_h(cur[P], xr[P], 0.0f);
      acc += lane < T ? tt : 0.0f;
    }
    acc = wave_sum(acc);
    const unsigned long long key = argmax_key(acc, (uint32_t)row);
    best = key > best ? key : best;
  }
  if (lane == 0 && best) atomicMax(amax_key, best);
}

// Exact-order rescoring (exact mode): every candidate row recomputed as the reference's AVX2
// mat_vec_mul_fp16 (ops.cpp:552-585) computes it -- 4 lanes per row, lane l = accumulator register sum[l]
// (8 fp32 lanes m), the 32-element chunks in order, then (S0 + S1) + (S2 + S3), t_m = V_m + V_m+4,
// (t0 + t1) + (t2 + t3) and the serial tail -- so the argmax is the reference's own (the screening bound holds
// for any summation order).  A work-group's 64 candidate slots at a time, chunks loaded 16 ahead.
__global__ __launch_bounds__(256) void screen_rescore_exact_kernel(const uint16_t* __restrict__ w, int rows, int cols,
                                                                   const uint16_t* __restrict__ x16,
                                                                   const float* __restrict__ hi,
                                                                   const unsigned* __restrict__ m_key, int slice,
                                                                   unsigned long long* __restrict__ amax_key) {
  extern __shared__ int s_cand[];  // [slice]
  __shared__ int s_n;
  const int t = threadIdx.x;
  if (t == 0) s_n = 0;
  __syncthreads();
  const float M = fkey_inv(*m_key);
  const int r0 = blockIdx.x * slice, r1 = min(rows, r0 + slice);
  for (int r = r0 + t; r < r1; r += 256)
    if (hi[r] >= M) s_cand[atomicAdd(&s_n, 1)] = r;
  __syncthreads();
  const int n = s_n;
  const int np = cols & ~31, l = t & 3;
  unsigned long long best = 0;
  for (int c0 = 0; c0 < n; c0 += 64) {
    const int ci = c0 + (t >> 2);
    const bool ok = ci < n;
    const int row = ok ? s_cand[ci] : s_cand[0];
    const uint16_t* wr = w + (size_t)row * cols;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int k0 = 0; k0 < np; k0 += 32 * 16) {
      uint4 wv[16], xv[16];
#pragma unroll
      for (int u = 0; u < 16; u++) {
        const int k = min(k0 + 32 * u, np - 32);
        wv[u] = *reinterpret_cast<const uint4*>(wr + k + 8 * l);
        xv[u] = *reinterpret_cast<const uint4*>(x16 + k + 8 * l);
      }
#pragma unroll
      for (int u = 0; u < 16; u++) {
        if (k0 + 32 * u >= np) break;
        const uint32_t ww[4] = {wv[u].x, wv[u].y, wv[u].z, wv[u].w}, xx[4] = {xv[u].x, xv[u].y, xv[u].z, xv[u].w};
#pragma unroll
        for (int e = 0; e < 4; e++) {
          acc[2 * e] = fmaf(h2f((uint16_t)(ww[e] & 0xFFFF)), h2f((uint16_t)(xx[e] & 0xFFFF)), acc[2 * e]);
          acc[2 * e + 1] = fmaf(h2f((uint16_t)(ww[e] >> 16)), h2f((uint16_t)(xx[e] >> 16)), acc[2 * e + 1]);
        }
      }
    }
    float v[8];
#pragma unroll
    for (int m = 0; m < 8; m++) {
      const float a = acc[m] + __shfl_xor(acc[m], 1);  // l0: S0 + S1, l2: S2 + S3
      v[m] = a + __shfl_xor(a, 2);                     // l0: (S0 + S1) + (S2 + S3)
    }
    if (ok && l == 0) {
      const float t0 = v[0] + v[4], t1 = v[1] + v[5], t2 = v[2] + v[6], t3 = v[3] + v[7];
      float r = (t0 + t1) + (t2 + t3);
      for (int k = np; k < cols; k++) r = fmaf(h2f(wr[k]), h2f(x16[k]), r);
      const unsigned long long key = argmax_key(r, (uint32_t)row);
      best = key > best ? key : best;
    }
  }
  if (best) atomicMax(amax_key, best);  // a few candidate lanes per launch
}

constexpr int RESCORE_SLICE = 1024;

}  // namespace

// the shapes whose fast F16 GEMV is gemv_f16_rows_pipe (k_gemv.hip
// launch_gemv): the rescoring reproduces exactly that kernel's rows
bool screen_supported(const DevWeight& table) {
  return table.type == T_F16 && table.cols % 128 == 0 && table.cols >= 128 && table.cols <= 6144 && table.rows > 0;
}

void alloc_screen_table(const DevWeight& table, ScreenTable& st, hipStream_t s) {
  const int nb = table.cols / 32;
  const size_t n_blocks = (size_t)table.rows * nb;
  st.qs = static_cast<decltype(st.qs)>(dev_alloc(n_blocks * 32));
  st.d = static_cast<decltype(st.d)>(dev_alloc(n_blocks * 2 + 64));
  st.xs = static_cast<decltype(st.xs)>(dev_alloc((size_t)(nb + 1) * sizeof(ScreenX)));
  st.hi = static_cast<decltype(st.hi)>(dev_alloc((size_t)table.rows * 4));
  st.m_key = static_cast<decltype(st.m_key)>(dev_alloc(64));
  LLMI_HIP(hipMemsetAsync(st.xs, 0, (size_t)(nb + 1) * sizeof(ScreenX), s));
  LLMI_HIP(hipMemsetAsync(st.m_key, 0, 64, s));
  st.rows = table.rows;
  st.cols = table.cols;
  st.bytes = n_blocks * 34;
  hipLaunchKernelGGL(quantize_table_q8_kernel, dim3((unsigned)((n_blocks + 255) / 256)), dim3(256), 0, s,
                     reinterpret_cast<const uint16_t*>(table.qs), n_blocks, nb, reinterpret_cast<uint4*>(st.qs), st.d);
  LLMI_HIP(hipGetLastError());
}

void free_screen_table(ScreenTable& st) {
  for (void* p : {(void*)st.qs, (void*)st.d, (void*)st.xs, (void*)st.hi, (void*)st.m_key})
    dev_free(p);
  st = ScreenTable{};
}

void launch_screen_argmax(const DevWeight& table, const ScreenTable& st, const uint16_t* x16,
                          unsigned long long* amax_key, hipStream_t s, bool prepped, bool exact) {
  if (table.rows != st.rows || table.cols != st.cols) throw std::runtime_error("screen: table mismatch");
  if (!screen_supported(table)) throw std::runtime_error("screen: unsupported logits table");
  const int n = table.cols, nb = n / 32;
  if (nb > 256) throw std::runtime_error("screen: n_embd > 8192");
  if (!prepped) hipLaunchKernelGGL(screen_prep_kernel, dim3(1), dim3(1024), 0, s, x16, n, st.xs, st.m_key);
  const int rows = table.rows;
  constexpr int wpc = 8;  // waves per CU (4B bench: 4, 12 and 16 slower, profiles/r03_screen_sweep.txt)
  // row groups in flight per lane group (4B bench: 1 -> 2 = 132.8 -> 127.7 us)
  constexpr int ahead = 2;
  // lanes per row: a quarter wave for short rows (<= 80 chunks: the 1B table's 72; 91 -> 74 us), else half a wave
  const int lpr = 2 * nb <= 80 ? 16 : 32;
  const int cpl = (2 * nb + lpr - 1) / lpr, rpw = 64 / lpr;
  const dim3 grid((std::min((rows + rpw - 1) / rpw, 256 * wpc) + 3) / 4);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, s, reinterpret_cast<const uint4*>(st.qs), st.d, rows, nb, st.xs, st.hi,
                       st.m_key);
  };
  switch (cpl) {
#define LLMI_SCR(C)                                                       \
  case C:                                                                 \
    if (lpr == 16) go(ahead > 1 ? screen_gemv_kernel<C, 2, 16> : screen_gemv_kernel<C, 1, 16>); \
    else go(ahead > 1 ? screen_gemv_kernel<C, 2, 32> : screen_gemv_kernel<C, 1, 32>);           \
    break;
    LLMI_SCR(1) LLMI_SCR(2) LLMI_SCR(3) LLMI_SCR(4) LLMI_SCR(5) LLMI_SCR(6) LLMI_SCR(7) LLMI_SCR(8) LLMI_SCR(9)
    LLMI_SCR(10) LLMI_SCR(11) LLMI_SCR(12)
#undef LLMI_SCR
    default: throw std::runtime_error("screen: unsupported n_embd");
  }
  LLMI_HIP(hipGetLastError());
  const int u4 = n / 8, P = u4 / 64, T = u4 % 64;
  const dim3 rg((rows + RESCORE_SLICE - 1) / RESCORE_SLICE);
  const size_t lds = RESCORE_SLICE * sizeof(int);
  if (exact) {
    hipLaunchKernelGGL(screen_rescore_exact_kernel, rg, dim3(256), lds, s, reinterpret_cast<const uint16_t*>(table.qs),
                       rows, n, x16, st.hi, st.m_key, RESCORE_SLICE, amax_key);
    LLMI_HIP(hipGetLastError());
    return;
  }
  switch (P * 4 + T / 16) {
#define LLMI_RSC(PP, TT)                                                                                          \
  case PP * 4 + TT / 16:                                                                                          \
    hipLaunchKernelGGL((screen_rescore_kernel<PP, TT>), rg, dim3(256), lds, s,                                   \
                       reinterpret_cast<const uint4*>(table.qs), rows, reinterpret_cast<const uint4*>(x16), st.hi, \
                       st.m_key, RESCORE_SLICE, amax_key);                                                        \
    break;
#define LLMI_RSC4(PP) LLMI_RSC(PP, 0) LLMI_RSC(PP, 16) LLMI_RSC(PP, 32) LLMI_RSC(PP, 48)
    LLMI_RSC(0, 16) LLMI_RSC(0, 32) LLMI_RSC(0, 48) LLMI_RSC4(1) LLMI_RSC4(2) LLMI_RSC4(3) LLMI_RSC4(4) LLMI_RSC4(5)
    LLMI_RSC4(6) LLMI_RSC4(7) LLMI_RSC4(8) LLMI_RSC4(9) LLMI_RSC4(10) LLMI_RSC4(11) LLMI_RSC(12, 0)
#undef LLMI_RSC4
#undef LLMI_RSC
    default: throw std::runtime_error("screen: unsupported logits width for the rescoring kernel");
  }
  LLMI_HIP(hipGetLastError());
}

}  // namespace llmi
