// k_prefill.hip -- batched prefill: T prompt tokens per launch instead of T
// decode steps (the reference runs T sequential
// GEMVs and scalar attention per token, model.cpp:752-756, 872-881, 907-912).
//
//   prefill_norm   per token: embedding / residual + RMSNorm -> Q8_0 blocks
//   prefill_gemm   Q4_0 weights x Q8_0 activations of T tokens on the int8
//                  matrix cores (v_mfma_i32_32x32x32_i8): one MFMA per
//                  32 rows x 32 tokens x one Q4_0 block, its exact int32 dot
//                  scaled by d_w * d_x into an fp32 accumulator
//   prefill_qk     per token and head: q/k RMSNorm + NEOX rope (+ q scale),
//                  K/V appended to the f16 cache
//   prefill_attn   causal attention of T queries over the cache (online
//                  softmax over 64-key tiles, fp32), output as Q8_0 blocks
//   prefill_gelu   GELU(gate) * up of the interleaved gate/up GEMM -> Q8_0
// Numerics are those of the fast decode path (Q8_0 activations, exact
// integer block dots, fp32 reassociated sums); the session checks prefill
// against the token loop and the reference (tests/test_prefill.py).
#include "attn.h"
#include "session_kernels.h"

namespace llmi {

namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float rms_scale_pf(float sum, int n, double eps) {  // ops.cpp:37-38
  return 1.0f / sqrtf((float)((double)(sum / (float)n) + eps));
}

template <int NWAVE>
__device__ __forceinline__ float block_sum(float v, float* red) {  // fixed order
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < NWAVE; i++) s += red[i];
  __syncthreads();
  return s;
}

// ---------------------------------------------------------------------------
// per-token residual / norm -> Q8_0
// ---------------------------------------------------------------------------
constexpr int PN_EPT = 32;  // n <= 256 * 32

__global__ __launch_bounds__(256) void prefill_norm_kernel(PrefillNorm a) {
  extern __shared__ float s_x[];  // [n]
  __shared__ float s_red[4];
  const int t = threadIdx.x, tok = blockIdx.x, n = a.n;
  float* resid = a.resid + (size_t)tok * n;
  float v[PN_EPT];
  if (a.table) {  // embedding row * sqrt(n_embd) (model.cpp:240-344)
    const uint8_t* row = a.table + (size_t)a.tokens[tok] * a.row_bytes;
#pragma unroll
    for (int k = 0; k < PN_EPT; k++) {
      const int i = t + k * 256;
      float e = 0.0f;
      if (i < n) {
        if (a.emb_type == T_F16) {
          e = h2f(reinterpret_cast<const uint16_t*>(row)[i]);
        } else {  // Q8_0: 34-B blocks, f16 scale then 32 int8
          const uint8_t* b = row + (i / 32) * 34;
          e = h2f((uint16_t)(b[0] | (b[1] << 8))) * (float)(int8_t)b[2 + i % 32];
        }
        e *= a.emb_scale;
        resid[i] = e;
      }
      v[k] = e;
    }
  } else {  // h = resid + rms(y) * w_post (y itself without post norm)
    const float* y = a.y + (size_t)tok * n;
    float yv[PN_EPT];
    float ss = 0.0f;
#pragma unroll
    for (int k = 0; k < PN_EPT; k++) {
      const int i = t + k * 256;
      yv[k] = i < n ? y[i] : 0.0f;
      v[k] = i < n ? resid[i] : 0.0f;
      ss = fmaf(yv[k], yv[k], ss);
    }
    const float sc1 = a.w_post ? rms_scale_pf(block_sum<4>(ss, s_red), n, a.eps) : 0.0f;
#pragma unroll
    for (int k = 0; k < PN_EPT; k++) {
      const int i = t + k * 256;
      if (i < n) {
        v[k] += a.w_post ? (sc1 * yv[k]) * a.w_post[i] : yv[k];
        resid[i] = v[k];
      }
    }
  }
  float ss2 = 0.0f;
#pragma unroll
  for (int k = 0; k < PN_EPT; k++) ss2 = fmaf(v[k], v[k], ss2);
  const float sc2 = rms_scale_pf(block_sum<4>(ss2, s_red), n, a.eps);
#pragma unroll
  for (int k = 0; k < PN_EPT; k++) {
    const int i = t + k * 256;
    if (i < n) s_x[i] = (sc2 * v[k]) * a.w_next[i];
  }
  __syncthreads();
  XBlock* xq = a.xq + (size_t)tok * a.xstride;
  for (int i = t; i < n / 8; i += 256) {  // a DPP quad of lanes per Q8_0 block
    const float4 f0 = reinterpret_cast<const float4*>(s_x)[2 * i], f1 = reinterpret_cast<const float4*>(s_x)[2 * i + 1];
    const float vv[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
    q8_block_quad(vv, i & 3, xq + (i >> 2));
  }
}

// ---------------------------------------------------------------------------
// GEMM: out[t][n] = sum_b d_w[n][b] d_x[t][b] * sum_k (q_w[n][b][k] - 8) q_x[t][b][k]
// Work-group: 32 weight rows x 128 tokens, wave w: tokens [32 w, 32 w + 32).
// MFMA lane maps (scripts/dev/mfma_i8_check): lane (r = l & 31, h = l >> 5)
// holds A[row r][k 16h..16h+15] (the low (h 0) or high (h 1) nibbles of the
// row's 16 quant bytes, in k order) and B[k 16h..][token r] (the token's
// Q8_0 q[16h..16h+15]); D[row (reg & 3) + 8 (reg >> 2) + 4 h][token r].
// ---------------------------------------------------------------------------
constexpr int PG_TOK = 128;

__device__ __forceinline__ size_t q4_block_index(int slab, int rows, int nb, int n, int b) {
  return slab ? ((size_t)(b >> 3) * rows + n) * 8 + (b & 7) : (size_t)n * nb + b;
}

__device__ __forceinline__ int q4_signed(uint32_t w) {  // 4 nibbles (bytes 0..15) -> int8 (n - 8)
  return (int)((w + 0x78787878u) ^ 0x80808080u);
}

__global__ __launch_bounds__(256) void prefill_gemm_kernel(PrefillGemm a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  uint16_t* s_dw = reinterpret_cast<uint16_t*>(s_dyn);                                   // [nb][32]
  float* s_o = reinterpret_cast<float*>(s_dyn + (((size_t)a.nb * 64 + 15) & ~(size_t)15));  // [4][32][33]
  const int t = threadIdx.x, lane = t & 63, w = t >> 6, r = lane & 31, h = lane >> 5;
  const int nb = a.nb, n0 = blockIdx.x * 32;
  const int tok0 = blockIdx.y * PG_TOK + w * 32;
  for (int i = t; i < 32 * nb; i += 256) {  // the tile's block scales, transposed
    const int row = i / nb, b = i % nb;
    s_dw[b * 32 + row] = a.wd[q4_block_index(a.slab, a.rows, nb, n0 + row, b)];
  }
  __syncthreads();
  const XBlock* xr = a.x + (size_t)min(tok0 + r, a.T - 1) * a.xstride;
  float acc[16];
#pragma unroll
  for (int i = 0; i < 16; i++) acc[i] = 0.0f;
  const v16i zero = {};
  uint4 wq = a.qs[q4_block_index(a.slab, a.rows, nb, n0 + r, 0)];
  int4 xq = h ? xr[0].hi : xr[0].lo;
  float dx = xr[0].d;
  for (int b = 0; b < nb; b++) {
    // next block in flight while this one is multiplied
    const int bn = min(b + 1, nb - 1);
    const uint4 wq_n = a.qs[q4_block_index(a.slab, a.rows, nb, n0 + r, bn)];
    const int4 xq_n = h ? xr[bn].hi : xr[bn].lo;
    const float dx_n = xr[bn].d;
    v4i A, B;
    A.x = q4_signed(h ? (wq.x >> 4) & 0x0F0F0F0Fu : wq.x & 0x0F0F0F0Fu);
    A.y = q4_signed(h ? (wq.y >> 4) & 0x0F0F0F0Fu : wq.y & 0x0F0F0F0Fu);
    A.z = q4_signed(h ? (wq.z >> 4) & 0x0F0F0F0Fu : wq.z & 0x0F0F0F0Fu);
    A.w = q4_signed(h ? (wq.w >> 4) & 0x0F0F0F0Fu : wq.w & 0x0F0F0F0Fu);
    B.x = xq.x;
    B.y = xq.y;
    B.z = xq.z;
    B.w = xq.w;
    const v16i D = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, B, zero, 0, 0, 0);
#pragma unroll
    for (int g = 0; g < 4; g++) {  // rows 8g + 4h .. +3: one 8-B read of 4 scales
      const uint2 d4 = *reinterpret_cast<const uint2*>(&s_dw[b * 32 + 8 * g + 4 * h]);
      const float s0 = h2f((uint16_t)(d4.x & 0xFFFF)) * dx, s1 = h2f((uint16_t)(d4.x >> 16)) * dx;
      const float s2 = h2f((uint16_t)(d4.y & 0xFFFF)) * dx, s3 = h2f((uint16_t)(d4.y >> 16)) * dx;
      acc[4 * g + 0] = fmaf(s0, (float)D[4 * g + 0], acc[4 * g + 0]);
      acc[4 * g + 1] = fmaf(s1, (float)D[4 * g + 1], acc[4 * g + 1]);
      acc[4 * g + 2] = fmaf(s2, (float)D[4 * g + 2], acc[4 * g + 2]);
      acc[4 * g + 3] = fmaf(s3, (float)D[4 * g + 3], acc[4 * g + 3]);
    }
    wq = wq_n;
    xq = xq_n;
    dx = dx_n;
  }
  // transpose through LDS so each token's 32 outputs are one 128-B store
  float* so = s_o + (size_t)w * 32 * 33;
#pragma unroll
  for (int reg = 0; reg < 16; reg++) so[r * 33 + (reg & 3) + 8 * (reg >> 2) + 4 * h] = acc[reg];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS writes done (wave-local hand-off)
#pragma unroll
  for (int i = 0; i < 16; i++) {
    const int idx = i * 64 + lane, tk = idx >> 5, row = idx & 31;
    if (tok0 + tk < a.T) a.out[(size_t)(tok0 + tk) * a.ostride + n0 + row] = so[tk * 33 + row];
  }
}

// ---------------------------------------------------------------------------
// q/k norm + rope (+ q scale) and the K/V cache append, one wave per row
// ---------------------------------------------------------------------------
template <int HD>
__global__ __launch_bounds__(64) void prefill_qk_kernel(PrefillQK a) {
  constexpr int DPL = HD >= 64 ? HD / 64 : 1;
  constexpr int PX = HD >= 64 ? 32 : HD / 2;
  const int lane = threadIdx.x, tok = blockIdx.x, row = blockIdx.y;
  const int pos = a.pos0 + tok;
  const float* qkv = a.qkv + (size_t)tok * a.qkv_stride;
  const bool ok = lane * DPL < HD;
  const int nq = a.n_head, nkv = a.n_head_kv;
  if (row >= nq + nkv) {  // v rows: f16 into the cache
    const int kvh = row - nq - nkv;
#pragma unroll
    for (int d = 0; d < DPL; d++) {
      const int i = lane * DPL + d;
      if (ok) a.v_cache[((size_t)kvh * a.max_ctx + pos) * HD + i] = f2h_ggml(qkv[a.v_off + kvh * HD + i]);
    }
    return;
  }
  const bool is_q = row < nq;
  const float* src = is_q ? qkv + row * HD : qkv + a.k_off + (row - nq) * HD;
  const float* nw = is_q ? a.q_norm_w : a.k_norm_w;
  const float* cs = a.rope_cs + (size_t)pos * HD;
  float v[DPL];
  float ss = 0.0f;
#pragma unroll
  for (int d = 0; d < DPL; d++) {
    const int i = min(lane * DPL + d, HD - 1);
    v[d] = src[i];
    ss = ok ? fmaf(v[d], v[d], ss) : ss;
  }
  ss = wave_sum(ss);
  const float sc = 1.0f / sqrtf((float)((double)(ss / (float)HD) + a.eps));
#pragma unroll
  for (int d = 0; d < DPL; d++) {
    const int i = lane * DPL + d;
    const int j = i < HD / 2 ? i : i - HD / 2;
    const float nv = ok ? (sc * v[d]) * nw[min(i, HD - 1)] : 0.0f;
    const float pn = __shfl_xor(nv, PX);
    const float c = cs[2 * min(j, HD / 2 - 1)], s = cs[2 * min(j, HD / 2 - 1) + 1];
    const float o = i < HD / 2 ? fmaf(nv, c, -(pn * s)) : fmaf(pn, s, nv * c);
    if (!ok) continue;
    if (is_q)
      a.q_out[((size_t)tok * nq + row) * HD + i] = f2h_ggml(o * a.attn_scale);
    else
      a.k_cache[((size_t)(row - nq) * a.max_ctx + pos) * HD + i] = f2h_ggml(o);
  }
}

// ---------------------------------------------------------------------------
// causal attention, one work-group per (kv head, query token), fp32 online
// softmax over 64-key tiles; output heads as Q8_0 blocks
// ---------------------------------------------------------------------------
template <int HD, int G>
__global__ __launch_bounds__(256) void prefill_attn_kernel(PrefillAttn a) {
  constexpr int CH = HD / 8;
  constexpr int TP0 = 4 / G;
  constexpr int TP = TP0 < CH ? TP0 : CH;
  constexpr int KS = HD + 8 * TP;
  constexpr int NLD = (64 * CH + 255) / 256;
  constexpr int NTD = HD / 4;
  constexpr int KP = 256 / NTD;
  __shared__ __attribute__((aligned(16))) uint16_t s_k[64 * KS];
  __shared__ __attribute__((aligned(16))) uint16_t s_v[64 * HD];
  __shared__ __attribute__((aligned(16))) uint16_t s_q[G][HD];
  __shared__ float s_p[G][64];
  __shared__ float s_alpha[G], s_l[G];
  __shared__ __attribute__((aligned(16))) float s_red[KP > 1 ? KP * G * HD : 4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int hkv = blockIdx.x, tok = blockIdx.y;
  const int n_keys = a.pos0 + tok + 1;
  const uint4* kb = reinterpret_cast<const uint4*>(a.k_cache + (size_t)hkv * a.max_ctx * HD);
  const uint4* vb = reinterpret_cast<const uint4*>(a.v_cache + (size_t)hkv * a.max_ctx * HD);
  uint4 kr[NLD], vr[NLD];
  auto load_tile = [&](int tl) {
#pragma unroll
    for (int i = 0; i < NLD; i++) {
      const int k = min(i * 256 + t, 64 * CH - 1);
      const int key = min(tl * 64 + k / CH, a.max_ctx - 1);
      kr[i] = kb[(size_t)key * CH + k % CH];
      vr[i] = vb[(size_t)key * CH + k % CH];
    }
  };
  for (int i = t; i < G * HD; i += 256)
    s_q[i / HD][i % HD] = a.q[((size_t)tok * a.n_head + hkv * G) * HD + i];
  load_tile(0);
  float m_run = -INFINITY, l_run = 0.0f;
  float acc[G][4];
#pragma unroll
  for (int g = 0; g < G; g++)
#pragma unroll
    for (int e = 0; e < 4; e++) acc[g][e] = 0.0f;
  const int d_own = 4 * (t % NTD), kp = t / NTD;
  typedef _Float16 h2t __attribute__((ext_vector_type(2)));
  for (int tile = 0; tile * 64 < n_keys; tile++) {
#pragma unroll
    for (int i = 0; i < NLD; i++) {  // keys past the query are zeroed (stale cache bits)
      const bool ok = tile * 64 + (i * 256 + t) / CH < n_keys;
      if (!ok) kr[i] = make_uint4(0, 0, 0, 0);
      if (!ok) vr[i] = make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NLD; i++) {
      const int k = i * 256 + t;
      if (k < 64 * CH) {
        *reinterpret_cast<uint4*>(&s_k[(k / CH) * KS + (k % CH) * 8]) = kr[i];
        *reinterpret_cast<uint4*>(&s_v[(k / CH) * HD + (k % CH) * 8]) = vr[i];
      }
    }
    __syncthreads();
    if ((tile + 1) * 64 < n_keys) load_tile(tile + 1);  // next tile in flight
    if (t < G * 64 * TP) {
      const int pr = t / TP, part = t % TP;
      const int g = pr / 64, j = pr % 64;
      const uint4* krow = reinterpret_cast<const uint4*>(&s_k[j * KS]);
      const uint4* qrow = reinterpret_cast<const uint4*>(s_q[g]);
      float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
      for (int i = 0; i < CH / TP; i++) {
        const uint4 kk = krow[i * TP + part], qq = qrow[i * TP + part];
        s0 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, kk.x), __builtin_bit_cast(h2t, qq.x), s0, false);
        s1 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, kk.y), __builtin_bit_cast(h2t, qq.y), s1, false);
        s0 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, kk.z), __builtin_bit_cast(h2t, qq.z), s0, false);
        s1 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, kk.w), __builtin_bit_cast(h2t, qq.w), s1, false);
      }
      float sc = s0 + s1;
#pragma unroll
      for (int o = 1; o < TP; o <<= 1) sc += __shfl_xor(sc, o);
      if (part == 0) s_p[g][j] = tile * 64 + j < n_keys ? sc : -INFINITY;
    }
    __syncthreads();
    if (w < G) {
      const float sc = s_p[w][lane];
      const float m_new = fmaxf(m_run, wave_max(sc));
      const float p = expf(sc - m_new);
      const float alpha = expf(m_run - m_new);
      l_run = l_run * alpha + wave_sum(p);
      m_run = m_new;
      s_p[w][lane] = p;
      if (lane == 0) s_alpha[w] = alpha;
    }
    __syncthreads();
#pragma unroll
    for (int g = 0; g < G; g++) {
      const float al = s_alpha[g];
#pragma unroll
      for (int e = 0; e < 4; e++) acc[g][e] *= al;
    }
#pragma unroll 4
    for (int j = kp; j < 64; j += KP) {
      const uint2 vv = *reinterpret_cast<const uint2*>(&s_v[j * HD + d_own]);
      const float v0 = h2f((uint16_t)(vv.x & 0xFFFF)), v1 = h2f((uint16_t)(vv.x >> 16));
      const float v2 = h2f((uint16_t)(vv.y & 0xFFFF)), v3 = h2f((uint16_t)(vv.y >> 16));
#pragma unroll
      for (int g = 0; g < G; g++) {
        const float p = s_p[g][j];
        acc[g][0] = fmaf(p, v0, acc[g][0]);
        acc[g][1] = fmaf(p, v1, acc[g][1]);
        acc[g][2] = fmaf(p, v2, acc[g][2]);
        acc[g][3] = fmaf(p, v3, acc[g][3]);
      }
    }
  }
  if (w < G && lane == 0) s_l[w] = l_run;
  if constexpr (KP > 1) {
#pragma unroll
    for (int g = 0; g < G; g++)
      *reinterpret_cast<float4*>(&s_red[(kp * G + g) * HD + d_own]) = make_float4(acc[g][0], acc[g][1], acc[g][2], acc[g][3]);
    __syncthreads();
    if (kp == 0) {
#pragma unroll
      for (int g = 0; g < G; g++)
        for (int rr = 1; rr < KP; rr++) {
          const float4 o = *reinterpret_cast<const float4*>(&s_red[(rr * G + g) * HD + d_own]);
          acc[g][0] += o.x;
          acc[g][1] += o.y;
          acc[g][2] += o.z;
          acc[g][3] += o.w;
        }
    }
  }
  __syncthreads();
  // heads' outputs (o / l) staged in s_k, then Q8_0 blocks (a quad per block)
  float* s_out = reinterpret_cast<float*>(s_k);
  if (kp == 0) {
#pragma unroll
    for (int g = 0; g < G; g++)
#pragma unroll
      for (int e = 0; e < 4; e++) s_out[g * HD + d_own + e] = acc[g][e] / s_l[g];
  }
  __syncthreads();
  XBlock* xo = a.xq + (size_t)tok * a.xstride + (size_t)hkv * G * HD / 32;
  for (int i = t; i < G * HD / 8; i += 256) {
    const float4 f0 = reinterpret_cast<const float4*>(s_out)[2 * i], f1 = reinterpret_cast<const float4*>(s_out)[2 * i + 1];
    const float vv[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
    q8_block_quad(vv, i & 3, xo + (i >> 2));
  }
}

// ---------------------------------------------------------------------------
// GELU(gate) * up from the interleaved gate/up GEMM rows -> Q8_0 (32 lanes a block)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void prefill_gelu_kernel(const float* __restrict__ gu, int F, int H,
                                                           XBlock* __restrict__ xq, int xstride) {
  const int tok = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
  const bool ok = i < F;
  const int ic = ok ? i : F - 1;
  const float* g = gu + (size_t)tok * 2 * F;
  const int base = 2 * H * (ic / H) + ic % H;
  const float v = gelu_mul1(g[base], g[base + H]);
  q8_block_store(v, ok, xq + (size_t)tok * xstride + ic / 32, threadIdx.x & 31);
}

}  // namespace

void launch_prefill_norm(const PrefillNorm& a, int T, hipStream_t s) {
  if (a.n > 256 * PN_EPT || a.n % 32) throw std::runtime_error("prefill_norm: n_embd");
  hipLaunchKernelGGL(prefill_norm_kernel, dim3(T), dim3(256), (size_t)a.n * 4, s, a);
  LLMI_HIP(hipGetLastError());
}

bool prefill_gemm_supported(const DevWeight& w) {
  return w.type == T_Q4_0 && w.rows % 32 == 0 && w.cols % 32 == 0 && (!w.slab || (w.cols / 32) % 8 == 0);
}

void launch_prefill_gemm(const DevWeight& w, const XBlock* x, int xstride, int T, float* out, int ostride,
                         hipStream_t s) {
  if (!prefill_gemm_supported(w)) throw std::runtime_error("prefill_gemm: unsupported weight");
  PrefillGemm a;
  a.qs = reinterpret_cast<const uint4*>(w.qs);
  a.wd = w.d;
  a.rows = w.rows;
  a.nb = w.cols / 32;
  a.slab = w.slab;
  a.x = x;
  a.xstride = xstride;
  a.T = T;
  a.out = out;
  a.ostride = ostride;
  const size_t lds = (((size_t)a.nb * 64 + 15) & ~(size_t)15) + 4 * 32 * 33 * 4;
  hipLaunchKernelGGL(prefill_gemm_kernel, dim3(w.rows / 32, (T + PG_TOK - 1) / PG_TOK), dim3(256), lds, s, a);
  LLMI_HIP(hipGetLastError());
}

void launch_prefill_qk(const PrefillQK& a, int T, hipStream_t s) {
  const dim3 grid(T, a.n_head + 2 * a.n_head_kv);
  switch (a.head_dim) {
    case 64: hipLaunchKernelGGL(prefill_qk_kernel<64>, grid, dim3(64), 0, s, a); break;
    case 128: hipLaunchKernelGGL(prefill_qk_kernel<128>, grid, dim3(64), 0, s, a); break;
    case 256: hipLaunchKernelGGL(prefill_qk_kernel<256>, grid, dim3(64), 0, s, a); break;
    default: throw std::runtime_error("prefill_qk: head_dim");
  }
  LLMI_HIP(hipGetLastError());
}

template <int HD>
static void attn_g(const PrefillAttn& a, int T, hipStream_t s) {
  const dim3 grid(a.n_head_kv, T);
  switch (a.n_head / a.n_head_kv) {
    case 1: hipLaunchKernelGGL((prefill_attn_kernel<HD, 1>), grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL((prefill_attn_kernel<HD, 2>), grid, dim3(256), 0, s, a); break;
    case 4: hipLaunchKernelGGL((prefill_attn_kernel<HD, 4>), grid, dim3(256), 0, s, a); break;
    default: throw std::runtime_error("prefill_attn: GQA group must be 1, 2 or 4");
  }
}

void launch_prefill_attn(const PrefillAttn& a, int T, hipStream_t s) {
  switch (a.head_dim) {
    case 64: attn_g<64>(a, T, s); break;
    case 128: attn_g<128>(a, T, s); break;
    case 256: attn_g<256>(a, T, s); break;
    default: throw std::runtime_error("prefill_attn: head_dim");
  }
  LLMI_HIP(hipGetLastError());
}

void launch_prefill_gelu(const float* gu, int F, int H, XBlock* xq, int xstride, int T, hipStream_t s) {
  if (F % 32 || H <= 0 || F % H) throw std::runtime_error("prefill_gelu: shape");
  hipLaunchKernelGGL(prefill_gelu_kernel, dim3((F + 255) / 256, T), dim3(256), 0, s, gu, F, H, xq, xstride);
  LLMI_HIP(hipGetLastError());
}

}  // namespace llmi
