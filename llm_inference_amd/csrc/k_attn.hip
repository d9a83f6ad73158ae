// k_attn.hip -- per-head q/k norm + rope + KV append, and decode attention.
//
// KV cache layout (per layer): [n_head_kv][max_ctx][head_dim] f16, so one
// head's history is one contiguous stream.  The current position lives in
// device memory (d_pos) so a whole decode step can be replayed as one
// hipGraph without re-capturing.
#include "attn.h"

namespace llmi {

// ---------------------------------------------------------------------------
// q/k per-head rms_norm * weight (model.cpp:762,792), NEOX rope at pos
// (model.cpp:764,794), q *= 1/sqrt(head_dim) (model.cpp:767), K and V rows
// rounded to f16 into the cache (model.cpp:442-474).
// grid = n_head + n_head_kv blocks of 256 threads; head_dim <= 256.
// ---------------------------------------------------------------------------
template <bool EXACT>
__global__ __launch_bounds__(256) void qk_norm_rope_kv_kernel(QKVArgs a) {
  __shared__ float s_x[256];
  __shared__ float s_part[4];
  __shared__ float s_scale;
  const int t = threadIdx.x;
  const int hd = a.head_dim;
  const int pos = *a.d_pos;
  const bool is_q = blockIdx.x < (unsigned)a.n_head;
  const int h = is_q ? blockIdx.x : blockIdx.x - a.n_head;
  const float* src = a.qkv + (is_q ? (size_t)h * hd : (size_t)a.k_off + (size_t)h * hd);
  const float* nw = is_q ? a.q_norm_w : a.k_norm_w;
  const float v = t < hd ? src[t] : 0.0f;
  if (t < hd) s_x[t] = v;
  __syncthreads();
  if (EXACT) {
    if (t == 0) {
      float sum = 0.0f;
      for (int i = 0; i < hd; i++) sum = fmaf(s_x[i], s_x[i], sum);
      s_scale = 1.0f / sqrtf((float)((double)(sum / (float)hd) + a.eps));
    }
  } else {
    float sum = wave_sum(v * v);
    if ((t & 63) == 0) s_part[t >> 6] = sum;
    __syncthreads();
    if (t == 0) {
      const float tot = (s_part[0] + s_part[1]) + (s_part[2] + s_part[3]);
      s_scale = 1.0f / sqrtf((float)((double)(tot / (float)hd) + a.eps));
    }
  }
  __syncthreads();
  const float nv = t < hd ? (s_scale * v) * nw[t] : 0.0f;
  __syncthreads();
  if (t < hd) s_x[t] = nv;
  __syncthreads();
  const int half = hd / 2;
  const float* cs = a.rope_cs + (size_t)pos * half * 2;
  float r = nv;
  if (t < half) {
    const float c = cs[2 * t], sn = cs[2 * t + 1];
    r = fmaf(s_x[t], c, -(s_x[t + half] * sn));
  } else if (t < hd) {
    const float c = cs[2 * (t - half)], sn = cs[2 * (t - half) + 1];
    r = fmaf(s_x[t - half], sn, s_x[t] * c);
  }
  if (t < hd) {
    if (is_q) {
      a.q_out[(size_t)h * hd + t] = r * a.attn_scale;
    } else {
      const size_t ci = ((size_t)h * a.max_ctx + pos) * hd + t;
      a.k_cache[ci] = f2h_ggml(r);
      a.v_cache[ci] = f2h_ggml(a.qkv[(size_t)a.v_off + (size_t)h * hd + t]);
    }
  }
}

void launch_qk_norm_rope_kv(const QKVArgs& a, bool exact, hipStream_t s) {
  const dim3 grid(a.n_head + a.n_head_kv);
  if (exact)
    hipLaunchKernelGGL(qk_norm_rope_kv_kernel<true>, grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(qk_norm_rope_kv_kernel<false>, grid, dim3(256), 0, s, a);
  LLMI_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// exact attention (model.cpp:481-547): one block per query head, keys in
// order; score = sequential double sum of exact f32 products f16(k)*f16(q);
// online max with double/float compares as in the reference; f16 V
// accumulator rounded every step (vec_scale_f16 / vec_mad_f16).
// expf is the device libm's (documented ulp-level difference from glibc).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void attn_exact_kernel(AttnArgs a) {
  __shared__ float s_prod[256];
  __shared__ float s_e, s_pe;
  __shared__ int s_resc;
  const int t = threadIdx.x, hd = a.head_dim;
  const int h = blockIdx.x;
  const int hkv = h / (a.n_head / a.n_head_kv);
  const int n_keys = *a.d_pos + 1;
  const float q16 = t < hd ? h2f(f2h_ggml(a.q[(size_t)h * hd + t])) : 0.0f;
  uint16_t vacc = f2h_ggml(0.0f);
  float s_acc = 0.0f, max_score = -INFINITY;
  const uint16_t* kb = a.k_cache + (size_t)hkv * a.max_ctx * hd;
  const uint16_t* vb = a.v_cache + (size_t)hkv * a.max_ctx * hd;
  for (int tk = 0; tk < n_keys; tk++) {
    if (t < hd) s_prod[t] = h2f(kb[(size_t)tk * hd + t]) * q16;
    __syncthreads();
    if (t == 0) {
      double score = 0.0;
      for (int i = 0; i < hd; i++) score += (double)s_prod[i];
      const float prev = max_score;
      float e, pe;
      int resc;
      if (score > (double)prev) {
        max_score = (float)score;
        e = 1.0f;
        pe = expf(prev - max_score);
        resc = 1;
      } else {
        e = expf((float)(score - (double)max_score));
        pe = 1.0f;
        resc = 0;
      }
      s_acc = s_acc * pe + e;
      s_e = e; s_pe = pe; s_resc = resc;
    }
    __syncthreads();
    if (t < hd) {
      if (s_resc) vacc = f2h_ggml(h2f(vacc) * s_pe);
      vacc = f2h_ggml(fmaf(h2f(vb[(size_t)tk * hd + t]), s_e, h2f(vacc)));
    }
    __syncthreads();
  }
  __shared__ float s_inv;
  if (t == 0) s_inv = s_acc == 0.0f ? 0.0f : 1.0f / s_acc;
  __syncthreads();
  if (t < hd) a.out[(size_t)h * hd + t] = h2f(vacc) * s_inv;
}

// ---------------------------------------------------------------------------
// fast split-K attention ("flash-decoding"): grid (n_head, n_split), one wave
// per block.  Block c walks key tiles c, c+n_split, ... of 64 keys (lane per
// key for QK^T, lane per head-dim slice for PV), keeping an online-softmax
// partial (m, l, acc[hd]) in fp32.  attn_combine merges the n_split partials.
// ---------------------------------------------------------------------------
// q/k head row norm (model.cpp:762/792, fast sum) + NEOX rope at the table row
// `cs` (ops.cpp:88-91 contraction) for a row held DPL elements per lane.
template <int HD>
__device__ __forceinline__ void norm_rope_row(const float* __restrict__ src, const float* __restrict__ nw,
                                              const float* __restrict__ cs, double eps, float (&out)[HD >= 64 ? HD / 64 : 1]) {
  constexpr int DPL = HD >= 64 ? HD / 64 : 1;
  constexpr int PX = HD >= 64 ? 32 : HD / 2;  // lane holding element i +- HD/2
  const int lane = threadIdx.x & 63;
  const bool ok = lane * DPL < HD;
  float v[DPL];
  float ss = 0.0f;
#pragma unroll
  for (int d = 0; d < DPL; d++) {
    v[d] = ok ? src[lane * DPL + d] : 0.0f;
    ss = fmaf(v[d], v[d], ss);
  }
  ss = wave_sum(ss);
  const float sc = 1.0f / sqrtf((float)((double)(ss / (float)HD) + eps));
#pragma unroll
  for (int d = 0; d < DPL; d++) {
    const int i = lane * DPL + d;
    const float n = ok ? (sc * v[d]) * nw[i] : 0.0f;
    const float pn = __shfl_xor(n, PX);
    const int j = i < HD / 2 ? i : i - HD / 2;
    const float c = ok ? cs[2 * j] : 0.0f, s = ok ? cs[2 * j + 1] : 0.0f;
    out[d] = i < HD / 2 ? fmaf(n, c, -(pn * s)) : fmaf(pn, s, n * c);
  }
}

// FUSED (session fast path): the block also performs the q/k per-head norm,
// rope and q scale of qk_norm_rope_kv_kernel, and the KV append of the current
// position: the block whose tile holds `pos` computes k/v of this token in
// registers, scores/accumulates that key from registers (no global write ->
// read hand-off inside the launch) and writes it to the cache for later steps.
template <int HD, bool FUSED>
__global__ __launch_bounds__(64) void attn_partial_kernel(AttnArgs a, QKVArgs qa) {
  constexpr int DPL = HD >= 64 ? HD / 64 : 1;  // head dims per lane in the PV phase
  __shared__ __attribute__((aligned(16))) uint16_t s_q[HD];
  __shared__ float s_p[64];
  const int lane = threadIdx.x;
  const bool pv_lane = (lane * DPL) < HD;
  const int h = blockIdx.x, c = blockIdx.y, nsplit = gridDim.y;
  const int group = a.n_head / a.n_head_kv;
  const int hkv = h / group;
  const int pos = *a.d_pos;
  const int n_keys = pos + 1;
  const bool own_new = FUSED && (pos / 64) % nsplit == c;
  float knew[DPL], vnew[DPL];
  float s_new = 0.0f;
  if (FUSED) {
    const float* cs = qa.rope_cs + (size_t)pos * (HD / 2) * 2;
    float qr[DPL];
    norm_rope_row<HD>(qa.qkv + (size_t)h * HD, qa.q_norm_w, cs, qa.eps, qr);
#pragma unroll
    for (int d = 0; d < DPL; d++)
      if (pv_lane) s_q[lane * DPL + d] = f2h_ggml(qr[d] * qa.attn_scale);
    if (own_new) {
      norm_rope_row<HD>(qa.qkv + qa.k_off + (size_t)hkv * HD, qa.k_norm_w, cs, qa.eps, knew);
      float part = 0.0f;
#pragma unroll
      for (int d = 0; d < DPL; d++) {
        const uint16_t k16 = f2h_ggml(knew[d]);
        const uint16_t v16 = f2h_ggml(pv_lane ? qa.qkv[qa.v_off + (size_t)hkv * HD + lane * DPL + d] : 0.0f);
        knew[d] = h2f(k16);
        vnew[d] = h2f(v16);
        if (pv_lane && h % group == 0) {  // one writer per kv head
          const size_t ci = ((size_t)hkv * a.max_ctx + pos) * HD + lane * DPL + d;
          qa.k_cache[ci] = k16;
          qa.v_cache[ci] = v16;
        }
      }
      __syncthreads();  // s_q complete
#pragma unroll
      for (int d = 0; d < DPL; d++)
        if (pv_lane) part = fmaf(knew[d], h2f(s_q[lane * DPL + d]), part);
      s_new = wave_sum(part);
    }
  } else {
    for (int i = lane; i < HD; i += 64) s_q[i] = f2h_ggml(a.q[(size_t)h * HD + i]);
  }
  __syncthreads();
  const uint4* kb = reinterpret_cast<const uint4*>(a.k_cache + (size_t)hkv * a.max_ctx * HD);
  const uint16_t* vb = a.v_cache + (size_t)hkv * a.max_ctx * HD;
  float m_run = -INFINITY, l_run = 0.0f;
  float acc[DPL];
#pragma unroll
  for (int d = 0; d < DPL; d++) acc[d] = 0.0f;
  typedef _Float16 h2t __attribute__((ext_vector_type(2)));
  for (int tile = c; tile * 64 < n_keys; tile += nsplit) {
    const int key = tile * 64 + lane;
    float sc = -INFINITY;
    if (FUSED && key == pos) {
      sc = s_new;
    } else if (key < n_keys) {
      const uint4* kr = kb + (size_t)key * (HD / 8);
      const uint4* qv = reinterpret_cast<const uint4*>(s_q);
      float s0 = 0.0f, s1 = 0.0f;
#pragma unroll 8
      for (int i = 0; i < HD / 8; i++) {
        const uint4 kk = kr[i], qq = qv[i];
        s0 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, kk.x), __builtin_bit_cast(h2t, qq.x), s0, false);
        s1 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, kk.y), __builtin_bit_cast(h2t, qq.y), s1, false);
        s0 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, kk.z), __builtin_bit_cast(h2t, qq.z), s0, false);
        s1 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, kk.w), __builtin_bit_cast(h2t, qq.w), s1, false);
      }
      sc = s0 + s1;
    }
    const float m_tile = wave_max(sc);
    const float m_new = fmaxf(m_run, m_tile);
    const float p = key < n_keys ? expf(sc - m_new) : 0.0f;
    const float alpha = expf(m_run - m_new);  // m_run = -inf on the first tile -> 0
    l_run = l_run * alpha + wave_sum(p);
    m_run = m_new;
    s_p[lane] = p;
    __syncthreads();
    const int nk = min(64, n_keys - tile * 64);
#pragma unroll
    for (int d = 0; d < DPL; d++) acc[d] *= alpha;
#pragma unroll 8
    for (int j = 0; j < nk && pv_lane; j++) {
      const float pj = s_p[j];
      const uint16_t* vr = vb + (size_t)(tile * 64 + j) * HD + lane * DPL;
      if (FUSED && tile * 64 + j == pos) {
#pragma unroll
        for (int d = 0; d < DPL; d++) acc[d] = fmaf(pj, vnew[d], acc[d]);
      } else if constexpr (DPL == 4) {
        const uint2 vv = *reinterpret_cast<const uint2*>(vr);
        acc[0] = fmaf(pj, h2f((uint16_t)(vv.x & 0xFFFF)), acc[0]);
        acc[1] = fmaf(pj, h2f((uint16_t)(vv.x >> 16)), acc[1]);
        acc[2] = fmaf(pj, h2f((uint16_t)(vv.y & 0xFFFF)), acc[2]);
        acc[3] = fmaf(pj, h2f((uint16_t)(vv.y >> 16)), acc[3]);
      } else {
#pragma unroll
        for (int d = 0; d < DPL; d++) acc[d] = fmaf(pj, h2f(vr[d]), acc[d]);
      }
    }
    __syncthreads();
  }
  float* part = a.partial + ((size_t)h * nsplit + c) * (HD + 2);
  if (pv_lane) {
#pragma unroll
    for (int d = 0; d < DPL; d++) part[lane * DPL + d] = acc[d];
  }
  if (lane == 0) { part[HD] = m_run; part[HD + 1] = l_run; }
}

// merge split partials per head; optionally quantize the head's output to
// Q8_0 blocks for the O projection (head_dim % 32 == 0).
// NSPLIT is a compile-time constant so every partial's (m, l, acc[t]) load is
// issued in one batch (one memory round trip instead of NSPLIT).
template <int NSPLIT>
__global__ __launch_bounds__(256) void attn_combine_kernel(AttnArgs a, Q8Act q8) {
  const int h = blockIdx.x, t = threadIdx.x, hd = a.head_dim;
  const float* part = a.partial + (size_t)h * NSPLIT * (hd + 2);
  float m[NSPLIT], l[NSPLIT], v[NSPLIT];
#pragma unroll
  for (int c = 0; c < NSPLIT; c++) {
    const float* pc = part + (size_t)c * (hd + 2);
    m[c] = pc[hd];
    l[c] = pc[hd + 1];
    v[c] = t < hd ? pc[t] : 0.0f;
  }
  float M = -INFINITY;
#pragma unroll
  for (int c = 0; c < NSPLIT; c++) M = fmaxf(M, m[c]);
  float L = 0.0f, o = 0.0f;
#pragma unroll
  for (int c = 0; c < NSPLIT; c++) {
    const float wc = l[c] == 0.0f ? 0.0f : expf(m[c] - M);
    L = fmaf(l[c], wc, L);
    o = fmaf(v[c], wc, o);
  }
  const float val = t < hd ? o / L : 0.0f;
  if (t < hd) a.out[(size_t)h * hd + t] = val;
  if (q8.xb != nullptr && t < hd) q8_block_store(val, true, q8.xb + ((h * hd + t) >> 5), t & 31);  // ops.cpp:116-139
}

template <int HD>
static void launch_partial(const AttnArgs& a, const QKVArgs* fused, int nsplit, hipStream_t s) {
  const dim3 grid(a.n_head, nsplit);
  if (fused)
    hipLaunchKernelGGL((attn_partial_kernel<HD, true>), grid, dim3(64), 0, s, a, *fused);
  else
    hipLaunchKernelGGL((attn_partial_kernel<HD, false>), grid, dim3(64), 0, s, a, QKVArgs{});
}

void launch_attention(const AttnArgs& a, bool exact, int nsplit, const Q8Act* q8, hipStream_t s,
                      const QKVArgs* fused) {
  if (exact) {
    hipLaunchKernelGGL(attn_exact_kernel, dim3(a.n_head), dim3(256), 0, s, a);
    LLMI_HIP(hipGetLastError());
    return;
  }
  if (nsplit != 16 && nsplit != 32) throw std::runtime_error("attention: nsplit must be 16 or 32");
  switch (a.head_dim) {
    case 16: launch_partial<16>(a, fused, nsplit, s); break;
    case 32: launch_partial<32>(a, fused, nsplit, s); break;
    case 64: launch_partial<64>(a, fused, nsplit, s); break;
    case 128: launch_partial<128>(a, fused, nsplit, s); break;
    case 256: launch_partial<256>(a, fused, nsplit, s); break;
    default: throw std::runtime_error("attention: unsupported head_dim " + std::to_string(a.head_dim));
  }
  LLMI_HIP(hipGetLastError());
  const Q8Act qq = q8 ? *q8 : Q8Act{};
  if (nsplit == 16)
    hipLaunchKernelGGL(attn_combine_kernel<16>, dim3(a.n_head), dim3(256), 0, s, a, qq);
  else
    hipLaunchKernelGGL(attn_combine_kernel<32>, dim3(a.n_head), dim3(256), 0, s, a, qq);
  LLMI_HIP(hipGetLastError());
}

}  // namespace llmi
