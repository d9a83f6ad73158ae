// k_elem.hip -- activation quantizers, norms, rope, elementwise ops (gfx950).
// All of these are bit-exact restatements of the reference ops (cited per
// kernel); the only reassociated op is rms_norm's sum in fast mode.
#include "kernels.h"

namespace llmi {

// ---------------------------------------------------------------------------
// quantize_row_q8_0 (ops.cpp:116-139): one 32-lane half-wave per block.
// amax is order-independent (exact); d = amax/127 (IEEE div), id = 1/d from
// the UNROUNDED d, stored d = f16(d), q = nearest_int(fma(x, id, magic)).
// Also emits nsum8 = -8 * sum(q) for the Q4_0 zero-point (exact integer).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void quantize_q8_0_kernel(const float* __restrict__ x, int n,
                                                            XBlock* __restrict__ xb) {
  const int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const int blk = gl >> 5;
  const bool ok = blk < n / 32;
  q8_block_store(ok ? x[gl] : 0.0f, ok, xb + (ok ? blk : 0), gl & 31);
}

void launch_quantize_q8_0(const float* x, int n, Q8Act out, hipStream_t s) {
  hipLaunchKernelGGL(quantize_q8_0_kernel, dim3((n + 255) / 256), dim3(256), 0, s, x, n, out.xb);
  LLMI_HIP(hipGetLastError());
}

// quantize_row_q8_k (ops.cpp:142-178): one 256-thread block per 256-element
// super-block.  `max` is the signed value of the FIRST element with the largest
// |x| (strict > scan) -> reduce (|x|, -index) lexicographically.
__global__ __launch_bounds__(256) void quantize_q8_k_kernel(const float* __restrict__ x, uint8_t* __restrict__ out) {
  __shared__ float s_ax[4];
  __shared__ int s_ix[4];
  __shared__ int s_bs[16];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const float v = x[blockIdx.x * 256 + t];
  float ax = fabsf(v);
  int ix = t;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float oa = __shfl_xor(ax, o);
    const int oi = __shfl_xor(ix, o);
    if (oa > ax || (oa == ax && oi < ix)) { ax = oa; ix = oi; }
  }
  if (lane == 0) { s_ax[w] = ax; s_ix[w] = ix; }
  __syncthreads();
  float amax = s_ax[0];
  int imax = s_ix[0];
  for (int k = 1; k < 4; k++)
    if (s_ax[k] > amax || (s_ax[k] == amax && s_ix[k] < imax)) { amax = s_ax[k]; imax = s_ix[k]; }
  uint8_t* blk = out + (size_t)blockIdx.x * 292;
  if (amax == 0.0f) {  // ops.cpp:158-163
    blk[4 + t] = 0;
    if (t < 16) { blk[260 + 2 * t] = 0; blk[261 + 2 * t] = 0; }
    if (t == 0) *reinterpret_cast<float*>(blk) = 0.0f;
    return;
  }
  const float mx = x[blockIdx.x * 256 + imax];
  const float iscale = -127.f / mx;
  int q = nearest_int_fma(iscale, v);
  q = q < -128 ? -128 : (q > 127 ? 127 : q);
  blk[4 + t] = (uint8_t)(int8_t)q;
  int sum = q;  // 16-lane group sums -> bsums
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
  if ((t & 15) == 0) {
    const int16_t s16 = (int16_t)sum;
    blk[260 + 2 * (t >> 4)] = (uint8_t)(s16 & 0xFF);
    blk[261 + 2 * (t >> 4)] = (uint8_t)((uint16_t)s16 >> 8);
  }
  if (t == 0) *reinterpret_cast<float*>(blk) = 1.0f / iscale;
  (void)s_bs;
}

void launch_quantize_q8_k(const float* x, int n, uint8_t* out, hipStream_t s) {
  hipLaunchKernelGGL(quantize_q8_k_kernel, dim3(n / 256), dim3(256), 0, s, x, out);
  LLMI_HIP(hipGetLastError());
}

// x -> f16 with round-to-nearest-even (ops.cpp:542-551: _mm256_cvtps_ph RNE)
__global__ void round_f16_kernel(const float* __restrict__ x, int n, uint16_t* __restrict__ o) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = f2h_ggml(x[i]);
}
void launch_round_f16(const float* x, int n, uint16_t* out, hipStream_t s) {
  hipLaunchKernelGGL(round_f16_kernel, dim3((n + 255) / 256), dim3(256), 0, s, x, n, out);
  LLMI_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// rms_norm (ops.cpp:28-43) [+ weight multiply, model.cpp:355-357]
//   sum = fma(v, v, sum) over i in order (exact mode: serial on lane 0),
//   mean = sum / (float)n,  s = 1 / sqrtf((float)((double)mean + eps)),
//   o = s * x, then o * w as a separate rounding.
// One 256-thread block per row.
// ---------------------------------------------------------------------------
template <bool EXACT>
__global__ __launch_bounds__(256) void rms_norm_kernel(const float* __restrict__ x, const float* __restrict__ w,
                                                       float* __restrict__ o, int n, double eps) {
  __shared__ float s_part[4];
  __shared__ float s_scale;
  const float* xr = x + (size_t)blockIdx.x * n;
  float* orow = o + (size_t)blockIdx.x * n;
  const int t = threadIdx.x;
  if (EXACT) {
    if (t == 0) {
      float sum = 0.0f;
      for (int i = 0; i < n; i++) sum = fmaf(xr[i], xr[i], sum);
      const float mean = sum / (float)n;
      s_scale = 1.0f / sqrtf((float)((double)mean + eps));
    }
  } else {
    float sum = 0.0f;
    for (int i = t; i < n; i += 256) sum = fmaf(xr[i], xr[i], sum);
    sum = wave_sum(sum);
    if ((t & 63) == 0) s_part[t >> 6] = sum;
    __syncthreads();
    if (t == 0) {
      const float tot = (s_part[0] + s_part[1]) + (s_part[2] + s_part[3]);
      const float mean = tot / (float)n;
      s_scale = 1.0f / sqrtf((float)((double)mean + eps));
    }
  }
  __syncthreads();
  const float sc = s_scale;
  for (int i = t; i < n; i += 256) {
    const float v = sc * xr[i];
    orow[i] = w ? v * w[i] : v;
  }
}

void launch_rms_norm(const float* x, const float* w, float* o, int n, int n_rows, double eps, bool exact,
                     hipStream_t s) {
  if (exact)
    hipLaunchKernelGGL(rms_norm_kernel<true>, dim3(n_rows), dim3(256), 0, s, x, w, o, n, eps);
  else
    hipLaunchKernelGGL(rms_norm_kernel<false>, dim3(n_rows), dim3(256), 0, s, x, w, o, n, eps);
  LLMI_HIP(hipGetLastError());
}

// softmax (ops.cpp:45-62): serial on one thread (it is not on the decode path;
// kept bit-exact for the ops.h surface).
__global__ void softmax_kernel(float* x, int n) {
  if (threadIdx.x != 0) return;
  float mx = x[0];
  for (int i = 0; i < n; i++) if (x[i] > mx) mx = x[i];
  float sum = 0.0f;
  for (int i = 0; i < n; i++) { x[i] = llmi_glibc::expf(x[i] - mx); sum += x[i]; }
  for (int i = 0; i < n; i++) x[i] /= sum;
}
void launch_softmax(float* x, int n, hipStream_t s) {
  hipLaunchKernelGGL(softmax_kernel, dim3(1), dim3(64), 0, s, x, n);
  LLMI_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// NEOX rope (ops.cpp:67-95).  (cos, sin) come from a host table built with
// glibc powf/sincosf (bit-identical angles); the rotation keeps the
// reference's contraction: v0' = fma(v0, c, -(v1*s)), v1' = fma(v0, s, v1*c).
// ---------------------------------------------------------------------------
__global__ void rope_kernel(float* __restrict__ t, int n_rows, int head_dim, int n_rot, const float* __restrict__ cs,
                            int rows_per_pos) {
  const int row = blockIdx.x;
  const int half = n_rot / 2;
  const float* c = cs + (size_t)(row / rows_per_pos) * half * 2;
  float* v = t + (size_t)row * head_dim;
  for (int i = threadIdx.x; i < half; i += blockDim.x) {
    const float co = c[2 * i], si = c[2 * i + 1];
    const float v0 = v[i], v1 = v[i + half];
    v[i] = fmaf(v0, co, -(v1 * si));
    v[i + half] = fmaf(v0, si, v1 * co);
  }
}
void launch_rope(float* t, int n_rows, int head_dim, int n_rot, const float* cs, int rows_per_pos, hipStream_t s) {
  hipLaunchKernelGGL(rope_kernel, dim3(n_rows), dim3(128), 0, s, t, n_rows, head_dim, n_rot, cs, rows_per_pos);
  LLMI_HIP(hipGetLastError());
}

__global__ void scale_kernel(float* t, int n, float sc) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) t[i] *= sc;
}
void launch_scale(float* t, int n, float sc, hipStream_t s) {
  hipLaunchKernelGGL(scale_kernel, dim3((n + 255) / 256), dim3(256), 0, s, t, n, sc);
  LLMI_HIP(hipGetLastError());
}

// vec_scale_f16 / vec_mad_f16 (ops.cpp:1084-1099)
__global__ void vec_scale_f16_kernel(uint16_t* y, int n, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = f2h_ggml(h2f(y[i]) * v);
}
__global__ void vec_mad_f16_kernel(uint16_t* y, const uint16_t* x, int n, float v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = f2h_ggml(fmaf(h2f(x[i]), v, h2f(y[i])));
}
void launch_vec_scale_f16(uint16_t* y, int n, float v, hipStream_t s) {
  hipLaunchKernelGGL(vec_scale_f16_kernel, dim3((n + 255) / 256), dim3(256), 0, s, y, n, v);
  LLMI_HIP(hipGetLastError());
}
void launch_vec_mad_f16(uint16_t* y, const uint16_t* x, int n, float v, hipStream_t s) {
  hipLaunchKernelGGL(vec_mad_f16_kernel, dim3((n + 255) / 256), dim3(256), 0, s, y, x, n, v);
  LLMI_HIP(hipGetLastError());
}

__global__ void gelu_mul_kernel(const float* g, const float* u, float* o, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) o[i] = gelu_mul1<true>(g[i], u[i]);
}
void launch_gelu_mul(const float* g, const float* u, float* o, int n, hipStream_t s) {
  hipLaunchKernelGGL(gelu_mul_kernel, dim3((n + 255) / 256), dim3(256), 0, s, g, u, o, n);
  LLMI_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// embedding rows -> f32 * scale (model.cpp:240-344, ops.cpp:958-1082)
// ---------------------------------------------------------------------------
__device__ float deq_elem(uint32_t type, const uint8_t* row, int i) {
  switch (type) {
    case T_F32: return reinterpret_cast<const float*>(row)[i];
    case T_F16: return h2f(reinterpret_cast<const uint16_t*>(row)[i]);
    case T_Q8_0: {
      const uint8_t* b = row + (i / 32) * 34;
      return h2f((uint16_t)(b[0] | (b[1] << 8))) * (float)(int8_t)b[2 + (i & 31)];
    }
    case T_Q5_0: {
      const uint8_t* b = row + (i / 32) * 22;
      const float d = h2f((uint16_t)(b[0] | (b[1] << 8)));
      const uint32_t qh = (uint32_t)b[2] | ((uint32_t)b[3] << 8) | ((uint32_t)b[4] << 16) | ((uint32_t)b[5] << 24);
      const int e = i & 31, k = e & 15;
      const int q = e < 16 ? ((b[6 + k] & 0x0F) | (((qh >> k) & 1) << 4)) : ((b[6 + k] >> 4) | (((qh >> (k + 16)) & 1) << 4));
      return d * (float)(q - 16);
    }
    case T_Q4_K: {
      const uint8_t* b = row + (i / 256) * 144;
      const int e = i & 255, is = e / 32, l = e & 31;
      const float d = h2f((uint16_t)(b[0] | (b[1] << 8))), mn = h2f((uint16_t)(b[2] | (b[3] << 8)));
      const uint8_t* q = b + 4;
      int sc, m;
      if (is < 4) { sc = q[is] & 63; m = q[is + 4] & 63; }
      else { sc = (q[is + 4] & 0xF) | ((q[is - 4] >> 6) << 4); m = (q[is + 4] >> 4) | ((q[is] >> 6) << 4); }
      const uint8_t qq = b[16 + (is / 2) * 32 + l];
      const int nib = (is & 1) ? (qq >> 4) : (qq & 0xF);
      return fmaf(d * (float)sc, (float)nib, -(mn * (float)m));
    }
    case T_Q6_K: {
      const uint8_t* b = row + (i / 256) * 210;
      const int e = i & 255, n = e / 128, r = e & 127, quad = r / 32, l = r & 31;
      const uint8_t* ql = b + n * 64;
      const uint8_t* qh = b + 128 + n * 32;
      const int8_t* sc = reinterpret_cast<const int8_t*>(b + 192 + n * 8);
      const float d = h2f((uint16_t)(b[208] | (b[209] << 8)));
      int q;
      if (quad == 0) q = (ql[l] & 0xF) | (((qh[l] >> 0) & 3) << 4);
      else if (quad == 1) q = (ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4);
      else if (quad == 2) q = (ql[l] >> 4) | (((qh[l] >> 4) & 3) << 4);
      else q = (ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4);
      return d * (float)sc[l / 16 + 2 * quad] * (float)(int8_t)(q - 32);
    }
    default: return 0.0f;
  }
}

__global__ void dequantize_rows_kernel(uint32_t type, const uint8_t* __restrict__ blocks, size_t row_bytes,
                                       const int32_t* __restrict__ ids, int n_cols, float scale, float* __restrict__ o) {
  const uint8_t* row = blocks + (size_t)ids[blockIdx.y] * row_bytes;
  float* orow = o + (size_t)blockIdx.y * n_cols;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n_cols; i += gridDim.x * blockDim.x) {
    const float v = deq_elem(type, row, i);
    orow[i] = scale == 1.0f ? v : v * scale;
  }
}

void launch_dequantize_rows(uint32_t type, const uint8_t* blocks, size_t row_bytes, const int32_t* row_ids, int n_ids,
                            int n_cols, float scale, float* o, hipStream_t s) {
  hipLaunchKernelGGL(dequantize_rows_kernel, dim3((n_cols + 255) / 256, n_ids), dim3(256), 0, s, type, blocks,
                     row_bytes, row_ids, n_cols, scale, o);
  LLMI_HIP(hipGetLastError());
}

}  // namespace llmi
