// k_attn.hip -- per-head q/k norm + rope + KV append, and decode attention.
//
// KV cache layout (per layer): [n_head_kv][max_ctx][head_dim] f16, so one
// head's history is one contiguous stream.  The current position lives in
// device memory (d_pos) so a whole decode step can be replayed as one
// hipGraph without re-capturing.
#include "attn.h"
#include <hip/hip_ext.h>
#include "layer_body.h"

namespace llmi {

// ---------------------------------------------------------------------------
// q/k per-head rms_norm * weight (model.cpp:762,792), NEOX rope at pos
// (model.cpp:764,794), q *= 1/sqrt(head_dim) (model.cpp:767), K and V rows
// rounded to f16 into the cache (model.cpp:442-474).
// grid = n_head + n_head_kv blocks of 256 threads; head_dim <= 256.
// ---------------------------------------------------------------------------
// rms_norm scale of one head row held as v (thread t < hd) and s_x (ops.cpp:28-43)
template <bool EXACT>
__device__ __forceinline__ float head_rms_scale(float v, const float* s_x, int hd, double eps, float* s_part,
                                                float* s_scale) {
  const int t = threadIdx.x;
  if (EXACT) {
    if (t == 0) {
      float sum = 0.0f;
      for (int i = 0; i < hd; i++) sum = fmaf(s_x[i], s_x[i], sum);
      *s_scale = 1.0f / sqrtf((float)((double)(sum / (float)hd) + eps));
    }
  } else {
    float sum = wave_sum(v * v);
    if ((t & 63) == 0) s_part[t >> 6] = sum;
    __syncthreads();
    if (t == 0) {
      const float tot = (s_part[0] + s_part[1]) + (s_part[2] + s_part[3]);
      *s_scale = 1.0f / sqrtf((float)((double)(tot / (float)hd) + eps));
    }
  }
  __syncthreads();
  return *s_scale;
}

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
  const float sc = head_rms_scale<EXACT>(v, s_x, hd, a.eps, s_part, &s_scale);
  const float nv = t < hd ? (sc * v) * nw[t] : 0.0f;
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
    }
  }
  if (!is_q) {  // the V row: as projected, or RMS-normalised without weight (Gemma-4)
    const float vv = t < hd ? a.qkv[(size_t)a.v_off + (size_t)h * hd + t] : 0.0f;
    float vo = vv;
    if (a.v_norm) {
      __syncthreads();  // s_x reuse
      if (t < hd) s_x[t] = vv;
      __syncthreads();
      vo = head_rms_scale<EXACT>(vv, s_x, hd, a.eps, s_part, &s_scale) * vv;
    }
    if (t < hd) a.v_cache[((size_t)h * a.max_ctx + pos) * hd + t] = f2h_ggml(vo);
  }
}

void launch_qk_norm_rope_kv(const QKVArgs& a, bool exact, hipStream_t s) {
  const dim3 grid(a.n_head + (a.has_kv ? a.n_head_kv : 0));
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
// expf is glibc's own algorithm (glibc_math.h), so the step is bit-exact.
// ---------------------------------------------------------------------------
// The serial loop is split into three exact parallel steps per chunk of keys:
//  (1) scores: thread per key, the reference's sequential double sum;
//  (2) the online max's decisions: the reference's running max after key j
//      is always fl(R_j), fl = rounding to float, R_j = max(s_0..s_j) in
//      double (induction over "s > (double)M ? M = (float)s" with monotone
//      rounding), so an exclusive prefix max in double gives every key's
//      branch and its e / pe (glibc expf) independently;
//  (3) per head dim, the f16 accumulator over the chunk's keys in order, and
//      s_acc = s_acc * pe + e in order (one thread).
constexpr int ATTN_EX_CH = 1024;  // keys per chunk (LDS: scores f64 + e, pe, branch)
__global__ __launch_bounds__(256) void attn_exact_kernel(AttnArgs a) {
  __shared__ float s_q[256];
  __shared__ double s_sc[ATTN_EX_CH];
  __shared__ float s_e[ATTN_EX_CH], s_pe[ATTN_EX_CH];
  __shared__ unsigned char s_up[ATTN_EX_CH];
  __shared__ double s_tmax[256];
  __shared__ float s_sacc;
  const int t = threadIdx.x, hd = a.head_dim;
  const int h = blockIdx.x;
  const int hkv = h / (a.n_head / a.n_head_kv);
  const int n_keys = *a.d_pos + 1;
  if (t < hd) s_q[t] = h2f(f2h_ggml(a.q[(size_t)h * hd + t]));
  uint16_t vacc = f2h_ggml(0.0f);
  float s_acc = 0.0f;
  double run_max = -INFINITY;  // R over the previous chunks
  const uint16_t* kb = a.k_cache + (size_t)hkv * a.max_ctx * hd;
  const uint16_t* vb = a.v_cache + (size_t)hkv * a.max_ctx * hd;
  __syncthreads();
  for (int c0 = 0; c0 < n_keys; c0 += ATTN_EX_CH) {
    const int nk = min(ATTN_EX_CH, n_keys - c0);
    // (1) scores, 4 consecutive keys per thread
    constexpr int KPT = ATTN_EX_CH / 256;
    double tmax = -INFINITY;
    for (int k = 0; k < KPT; k++) {
      const int j = t * KPT + k;
      if (j >= nk) break;
      const uint16_t* kr = kb + (size_t)(c0 + j) * hd;
      double score = 0.0;
      if (hd % 8 == 0) {  // 16-B loads of the row (rows are 16-B aligned), same summation order
        for (int i = 0; i < hd; i += 8) {
          const uint4 w = *reinterpret_cast<const uint4*>(kr + i);
          const uint32_t ww[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
          for (int e = 0; e < 4; e++) {
            score += (double)(h2f((uint16_t)(ww[e] & 0xFFFF)) * s_q[i + 2 * e]);
            score += (double)(h2f((uint16_t)(ww[e] >> 16)) * s_q[i + 2 * e + 1]);
          }
        }
      } else {
        for (int i = 0; i < hd; i++) score += (double)(h2f(kr[i]) * s_q[i]);
      }
      if (a.softcap > 0.0f) score = llmi_glibc::softcap_score(score, a.softcap);
      s_sc[j] = score;
      tmax = fmax(tmax, score);
    }
    s_tmax[t] = tmax;
    __syncthreads();
    // (2) exclusive prefix max over the threads' maxima (Hillis-Steele, max is exact), then per key
    for (int o = 1; o < 256; o <<= 1) {
      const double v = t >= o ? s_tmax[t - o] : -INFINITY;
      __syncthreads();
      s_tmax[t] = fmax(s_tmax[t], v);
      __syncthreads();
    }
    double pm = fmax(run_max, t > 0 ? s_tmax[t - 1] : -INFINITY);  // max of every key before this thread's first
    for (int k = 0; k < KPT; k++) {
      const int j = t * KPT + k;
      if (j >= nk) break;
      const double score = s_sc[j];
      const float prev = (float)pm;  // the reference's max_score before key j
      if (score > (double)prev) {
        s_e[j] = 1.0f;
        s_pe[j] = llmi_glibc::expf(prev - (float)score);
        s_up[j] = 1;
      } else {
        s_e[j] = llmi_glibc::expf((float)(score - (double)prev));
        s_pe[j] = 1.0f;
        s_up[j] = 0;
      }
      pm = fmax(pm, score);
    }
    run_max = fmax(run_max, s_tmax[255]);
    __syncthreads();
    // (3) the accumulators, keys in order
    if (t < hd) {
      for (int j = 0; j < nk; j++) {
        if (s_up[j]) vacc = f2h_ggml(h2f(vacc) * s_pe[j]);
        vacc = f2h_ggml(fmaf(h2f(vb[(size_t)(c0 + j) * hd + t]), s_e[j], h2f(vacc)));
      }
    }
    if (t == 0)
      for (int j = 0; j < nk; j++) s_acc = s_acc * s_pe[j] + s_e[j];
    __syncthreads();  // the chunk's LDS is reused by the next one
  }
  if (t == 0) s_sacc = s_acc == 0.0f ? 0.0f : 1.0f / s_acc;
  __syncthreads();
  if (t < hd) a.out[(size_t)h * hd + t] = h2f(vacc) * s_sacc;
}

// ---------------------------------------------------------------------------
// fast split-K attention ("flash-decoding"), ONE launch: grid (n_head_kv,
// ATTN_NSPLIT).  Work-group c walks key tiles c, c+NSPLIT, ... of 64 keys
// keeping an online-softmax partial (m, l, acc[hd]) per query head in fp32;
// the last work-group of each kv head to finish (agent-scope ticket) merges
// the NSPLIT partials, writes the heads' outputs and their Q8_0 blocks.
// ---------------------------------------------------------------------------
// q/k head row norm (model.cpp:762/792, fast sum) + NEOX rope at the table row
// `cs` (ops.cpp:88-91 contraction) for a row held DPL elements per lane, in two
// steps so the row's loads can be issued ahead of the K/V tile loads and the
// arithmetic run while the tile is in flight.
template <int HD>
struct RowLd {
  static constexpr int DPL = HD >= 64 ? HD / 64 : 1;
  float v[DPL], nw[DPL], c[DPL], s[DPL];
};

template <int N>
__device__ __forceinline__ void ld_vec(float (&dst)[N], const float* __restrict__ p) {  // N consecutive floats
  if constexpr (N == 4) {
    const float4 v = *reinterpret_cast<const float4*>(p);
    dst[0] = v.x; dst[1] = v.y; dst[2] = v.z; dst[3] = v.w;
  } else if constexpr (N == 2) {
    const float2 v = *reinterpret_cast<const float2*>(p);
    dst[0] = v.x; dst[1] = v.y;
  } else {
#pragma unroll
    for (int d = 0; d < N; d++) dst[d] = p[d];
  }
}

template <int HD>
__device__ __forceinline__ void row_load(RowLd<HD>& r, const float* __restrict__ src, const float* __restrict__ nw,
                                         const float* __restrict__ cs) {
  constexpr int DPL = RowLd<HD>::DPL;
  const int lane = threadIdx.x & 63;
  // elements i0 .. i0 + DPL - 1, one vector load per operand (lanes past the
  // row re-read its last elements: unconditional loads, masked later)
  const int i0 = min(lane, HD / DPL - 1) * DPL;
  const int j0 = i0 < HD / 2 ? i0 : i0 - HD / 2;  // DPL divides HD / 2
  if (src) ld_vec<DPL>(r.v, src + i0);
  ld_vec<DPL>(r.nw, nw + i0);
  // (cos, sin) pairs of elements j0 .. j0 + DPL - 1: 2 DPL consecutive floats
  float cs2[2 * DPL];
  if constexpr (DPL == 4) {
    float lo[4], hi[4];
    ld_vec<4>(lo, cs + 2 * j0);
    ld_vec<4>(hi, cs + 2 * j0 + 4);
#pragma unroll
    for (int d = 0; d < 4; d++) {
      cs2[d] = lo[d];
      cs2[4 + d] = hi[d];
    }
  } else {
    ld_vec<2 * DPL>(cs2, cs + 2 * j0);
  }
#pragma unroll
  for (int d = 0; d < DPL; d++) {
    r.c[d] = cs2[2 * d];
    r.s[d] = cs2[2 * d + 1];
  }
}

// row_load with the row itself read from granules (the attention block)
template <int HD>
__device__ __forceinline__ void row_load_gr(RowLd<HD>& r, const uint2* g, const float* __restrict__ nw,
                                            const float* __restrict__ cs, uint32_t tag, int* err) {
  constexpr int DPL = RowLd<HD>::DPL;
  row_load<HD>(r, nullptr, nw, cs);  // (nw, cs); the row comes from g
  const int lane = threadIdx.x & 63;
  uint32_t u[DPL];
  ld_granules<DPL>(u, g, min(lane, HD / DPL - 1) * DPL, tag, err);
#pragma unroll
  for (int d = 0; d < DPL; d++) r.v[d] = __uint_as_float(u[d]);
}

template <int HD>
__device__ __forceinline__ void row_finish(const RowLd<HD>& r, double eps, float (&out)[RowLd<HD>::DPL]) {
  constexpr int DPL = RowLd<HD>::DPL;
  constexpr int PX = HD >= 64 ? 32 : HD / 2;  // lane holding element i +- HD/2
  const int lane = threadIdx.x & 63;
  const bool ok = lane * DPL < HD;
  float ss = 0.0f;
#pragma unroll
  for (int d = 0; d < DPL; d++) ss = ok ? fmaf(r.v[d], r.v[d], ss) : ss;
  ss = wave_sum(ss);
  const float sc = 1.0f / sqrtf((float)((double)(ss / (float)HD) + eps));
#pragma unroll
  for (int d = 0; d < DPL; d++) {
    const int i = lane * DPL + d;
    const float n = ok ? (sc * r.v[d]) * r.nw[d] : 0.0f;
    const float pn = __shfl_xor(n, PX);
    out[d] = i < HD / 2 ? fmaf(n, r.c[d], -(pn * r.s[d])) : fmaf(pn, r.s[d], n * r.c[d]);
  }
}


// One work-group of 256 threads per (kv head, split) covering all G = n_head /
// n_head_kv query heads of that kv head, so each K/V tile is read from HBM
// once per split.  Per 64-key tile: every thread issues its 16-byte K and V
// chunk loads together (the tile is one contiguous 2*64*HD*2-byte stream;
// the first tile before the q/k prologue, each next tile right after the
// current one is in LDS), then
//   QK^T: TP threads per (query head, key) pair, interleaved 16-byte chunks,
//         v_dot2 f16 products in fp32, K rows padded by TP*16 bytes so the
//         ds_read_b128 of 16 lanes hit 16 distinct bank groups;
//   softmax: wave g keeps head g's running (m, l);
//   PV: thread owns 4 head dims (for all G heads) over a key residue class.
// FUSED (session fast path): the work-group also performs the q/k per-head
// norm, rope and q scale of qk_norm_rope_kv_kernel and the KV append of this
// token; the split owning `pos` substitutes the new k/v rows from LDS for the
// cache rows it is writing in the same launch.
// Hand-off of the partials to the merging work-group (MI355X_MICROARCH
// hand-off table, first row): sc1 stores, every storing wave's vmcnt(0),
// a workgroup barrier, one agent-scope add per work-group; the work-group
// whose add returns NSPLIT-1 reads every partial with sc1 loads.
#ifdef LLMI_ATTN_TRACE  // development: per-work-group phase timestamps (scripts/ab)
__device__ unsigned long long* g_attn_trace = nullptr;
void attn_set_trace(unsigned long long* p) { LLMI_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_attn_trace), &p, sizeof(p))); }
#define ATTN_MARK(ph)                                                                                  \
  do {                                                                                                 \
    if (g_attn_trace && threadIdx.x == 0)                                                             \
      g_attn_trace[((size_t)blockIdx.x * gridDim.y + blockIdx.y) * 8 + (ph)] = wall_clock64();        \
  } while (0)
#else
#define ATTN_MARK(ph) \
  do {                \
  } while (0)
#endif

template <int G>
constexpr int attn_tp() {  // threads per (query head, key) pair in QK^T
  return 4 / G;
}
template <int HD, int G>
constexpr int attn_ks() {  // padded K row stride (halves)
  return HD + 8 * (attn_tp<G>() < HD / 8 ? attn_tp<G>() : HD / 8);
}
template <int HD, int G>
constexpr int attn_kp() {  // PV key residue classes
  return 256 / (HD / 4);
}

// BLK (the attention-block kernel below): (hkv, c) come from the block's
// role split; the first K/V tile is issued, then the work-group reads this
// token's q/k/v rows from their granules (re-loading until the qkv
// work-groups' tags arrive); the merging work-group publishes the heads'
// Q8_0 blocks as granules for the o projection.
// KVD: virtual kv heads per cache head (GQA groups of 8 run as two work-group
// sets of 4 q heads over the same cache head: hkv indexes the q-head group,
// hkv / KVD the cache)
// NS: key-range splits per kv head (ATTN_NSPLIT; 16 in the 27B attention block, whose grid must stay co-resident)
template <int HD, int G, bool FUSED, int TK, bool BLK = false, int KVD = 1, int NS = ATTN_NSPLIT>
__device__ __forceinline__ void attn_split_body(const AttnArgs& a, const QKVArgs& qa, uint16_t* __restrict__ s_k,
                                                uint16_t* __restrict__ s_v, float* __restrict__ s_red,
                                                const int hkv, const int c, const BlockSync& bs) {
  static_assert(!BLK || FUSED, "BLK implies FUSED");
  const uint32_t btag = BLK ? *bs.epoch + 1u : 0u;  // granule tag, loaded up front
  BLK_MARK(bs, 0);
  static_assert(NS == 32 || NS == 16, "merge reductions are half-wave or row wide");
  static_assert(TK == 32 || TK == 64, "key tile: 32 or 64 keys");
  constexpr int CH = HD / 8;                         // 16-byte chunks per row
  constexpr int TP0 = 4 / G;                         // threads per (head, key) pair
  constexpr int TP = TP0 < CH ? TP0 : CH;
  constexpr int KS = HD + 8 * TP;                    // padded K row stride (halves)
  constexpr int NLD = (TK * CH + 255) / 256;         // chunk loads per thread per tile
  constexpr int NTD = HD / 4;                        // PV: 4 head dims per thread, NTD threads per key class
  constexpr int KP = 256 / NTD;                      // key residue classes in PV
  constexpr int DPL = RowLd<HD>::DPL;
  static_assert(KS == attn_ks<HD, G>() && KP == attn_kp<HD, G>(), "LDS carve-up");
  __shared__ __attribute__((aligned(16))) uint16_t s_q[G][HD];
  __shared__ __attribute__((aligned(16))) uint16_t s_new[FUSED ? 2 : 1][FUSED ? HD : 8];
  __shared__ float s_p[G][TK];
  __shared__ float s_alpha[G];
  __shared__ int s_last;
  __shared__ __attribute__((aligned(16))) float s_outbuf[TK * KS * 2 >= G * HD * 4 ? 1 : G * HD];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  ATTN_MARK(0);
  const int pos = *a.d_pos;
  const int n_keys = pos + 1;
  const bool own_new = FUSED && (pos / TK) % NS == c;
  const int hkc = hkv / KVD;  // cache head
  // KVD > 1 with FUSED: the even virtual head appends the cache head's new K/V row (below); every virtual head's
  // own_new work-group takes the new row from LDS (s_new), never from the cache
  const uint4* kb = reinterpret_cast<const uint4*>(a.k_cache + (size_t)hkc * a.max_ctx * HD);
  const uint4* vb = reinterpret_cast<const uint4*>(a.v_cache + (size_t)hkc * a.max_ctx * HD);
  uint4 kr[NLD], vr[NLD];
  // unconditional loads of tile `tl` (rows clamped into the cache); keys past
  // n_keys are zeroed (the cache beyond pos may hold stale or NaN bits)
  auto load_tile = [&](int tl) {
#pragma unroll
    for (int i = 0; i < NLD; i++) {
      const int k = min(i * 256 + t, TK * CH - 1);
      const int key = min(tl * TK + k / CH, a.max_ctx - 1);
      const size_t gi = (size_t)key * CH + k % CH;
      kr[i] = kb[gi];
      vr[i] = vb[gi];
    }
  };
  auto mask_tile = [&](int tl) {
#pragma unroll
    for (int i = 0; i < NLD; i++) {
      const bool ok = tl * TK + (i * 256 + t) / CH < n_keys;
      if (!ok) kr[i] = make_uint4(0, 0, 0, 0);
      if (!ok) vr[i] = make_uint4(0, 0, 0, 0);
    }
  };

  // ---- prologue loads, then the first tile, then the prologue arithmetic ----
  const float* cs = FUSED ? qa.rope_cs + (size_t)pos * (HD / 2) * 2 : nullptr;
  RowLd<HD> rq, rk;
  float vrow[DPL];
  if (FUSED && !BLK) {
    if (w < G) row_load<HD>(rq, qa.qkv + (size_t)(hkv * G + w) * HD, qa.q_norm_w, cs);
    if (w == (G & 3)) row_load<HD>(rk, qa.qkv + qa.k_off + (size_t)hkc * HD, qa.k_norm_w, cs);
    if (w == ((G + 1) & 3)) {
      ld_vec<DPL>(vrow, qa.qkv + qa.v_off + (size_t)hkc * HD + min(lane, HD / DPL - 1) * DPL);
    }
  }
  int tile = c;
  load_tile(tile);
  if constexpr (BLK) {  // the history tile is in flight; now this token's rows, from their granules
    const uint32_t tag = btag;
    if (w < G) row_load_gr<HD>(rq, bs.g_qkv + (size_t)(hkv * G + w) * HD, qa.q_norm_w, cs, tag, bs.err);
    if (w == (G & 3)) row_load_gr<HD>(rk, bs.g_qkv + qa.k_off + (size_t)hkc * HD, qa.k_norm_w, cs, tag, bs.err);
    if (w == ((G + 1) & 3)) {
      uint32_t u[DPL];
      ld_granules<DPL>(u, bs.g_qkv + qa.v_off + (size_t)hkc * HD, min(lane, HD / DPL - 1) * DPL, tag, bs.err);
#pragma unroll
      for (int d = 0; d < DPL; d++) vrow[d] = __uint_as_float(u[d]);
    }
    BLK_MARK(bs, 1);
  }
  if (FUSED) {
    const bool ok = lane * DPL < HD;
    if (w < G) {
      float qr[DPL];
      row_finish<HD>(rq, qa.eps, qr);
#pragma unroll
      for (int d = 0; d < DPL; d++)
        if (ok) s_q[w][lane * DPL + d] = f2h_ggml(qr[d] * qa.attn_scale);
    }
    if (w == (G & 3)) {
      float kn[DPL];
      row_finish<HD>(rk, qa.eps, kn);
#pragma unroll
      for (int d = 0; d < DPL; d++) {
        const uint16_t k16 = f2h_ggml(kn[d]);
        if (ok) s_new[0][lane * DPL + d] = k16;
        if (ok && own_new && hkv % KVD == 0) qa.k_cache[((size_t)hkc * a.max_ctx + pos) * HD + lane * DPL + d] = k16;
      }
    }
    if (w == ((G + 1) & 3)) {
#pragma unroll
      for (int d = 0; d < DPL; d++) {
        const uint16_t v16 = f2h_ggml(vrow[d]);
        if (ok) s_new[FUSED ? 1 : 0][lane * DPL + d] = v16;
        if (ok && own_new && hkv % KVD == 0) qa.v_cache[((size_t)hkc * a.max_ctx + pos) * HD + lane * DPL + d] = v16;
      }
    }
  } else {
    for (int i = t; i < G * HD; i += 256) s_q[i / HD][i % HD] = f2h_ggml(a.q[(size_t)hkv * G * HD + i]);
  }

  float m_run = -INFINITY, l_run = 0.0f;  // head w's running max / sum (waves w < G)
  float acc[G][4];
#pragma unroll
  for (int g = 0; g < G; g++)
#pragma unroll
    for (int e = 0; e < 4; e++) acc[g][e] = 0.0f;
  const int d_own = 4 * (t % NTD), kp = t / NTD;
  typedef _Float16 h2t __attribute__((ext_vector_type(2)));
  ATTN_MARK(1);
  BLK_MARK(bs, 2);
  for (; tile * TK < n_keys; tile += NS) {
    mask_tile(tile);
    __syncthreads();  // previous tile's LDS reads done (first time: s_q / s_new written)
#pragma unroll
    for (int i = 0; i < NLD; i++) {
      const int k = i * 256 + t;
      const int j = k / CH, pc = k % CH;
      if (k < TK * CH && !(FUSED && tile * TK + j == pos)) {
        *reinterpret_cast<uint4*>(&s_k[j * KS + pc * 8]) = kr[i];
        *reinterpret_cast<uint4*>(&s_v[j * HD + pc * 8]) = vr[i];
      }
    }
    if (FUSED && tile == pos / TK && t < CH) {  // the new row, written in this launch
      const int j = pos % TK;
      *reinterpret_cast<uint4*>(&s_k[j * KS + t * 8]) = reinterpret_cast<const uint4*>(s_new[0])[t];
      *reinterpret_cast<uint4*>(&s_v[j * HD + t * 8]) = reinterpret_cast<const uint4*>(s_new[FUSED ? 1 : 0])[t];
    }
    __syncthreads();
    ATTN_MARK(2);
    if ((tile + NS) * TK < n_keys) load_tile(tile + NS);  // next tile in flight during this one's math
    if (t < G * TK * TP) {
      const int pr = t / TP, part = t % TP;
      const int g = pr / TK, j = pr % TK;
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
      if (a.softcap > 0.0f) sc = a.softcap * tanhf(sc / a.softcap);  // model.cpp:511-513
      if (part == 0) s_p[g][j] = tile * TK + j < n_keys ? sc : -INFINITY;
    }
    __syncthreads();
    if (w < G) {
      const float sc = lane < TK ? s_p[w][lane] : -INFINITY;
      const float m_new = fmaxf(m_run, wave_max(sc));
      const float p = expf(sc - m_new);  // masked keys: exp(-inf) = 0
      const float alpha = expf(m_run - m_new);  // first tile: exp(-inf) = 0
      l_run = l_run * alpha + wave_sum(p);
      m_run = m_new;
      if (lane < TK) s_p[w][lane] = p;
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
    for (int j = kp; j < TK; j += KP) {
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
  if constexpr (KP > 1) {
#pragma unroll
    for (int g = 0; g < G; g++)
      *reinterpret_cast<float4*>(&s_red[(kp * G + g) * HD + d_own]) =
          make_float4(acc[g][0], acc[g][1], acc[g][2], acc[g][3]);
    __syncthreads();
    if (kp == 0) {
#pragma unroll
      for (int g = 0; g < G; g++)
        for (int r = 1; r < KP; r++) {
          const float4 o = *reinterpret_cast<const float4*>(&s_red[(r * G + g) * HD + d_own]);
          acc[g][0] += o.x;
          acc[g][1] += o.y;
          acc[g][2] += o.z;
          acc[g][3] += o.w;
        }
    }
  }

  ATTN_MARK(3);
  // ---- publish the partial, take a ticket --------------------------------
  float* part0 = a.partial + (size_t)hkv * G * NS * (HD + 2);  // [G][NS][HD + 2]
  // reset: this work-group puts the ticket back to 0 for the next launch (the one that reads it last)
  auto merge_heads = [&](auto gmc, int g0, bool reset) {
    constexpr int GM = decltype(gmc)::value;
  // ---- merge the NS partials of GM heads from head g0 (the last work-group: all G; DUAL: one each) ----
  // One batch of loads: the (m, l) pairs first (the weights are reduced while
  // the rest lands), then every thread's partial accumulators for its (g, d)
  // outputs.  w_c = l_c ? exp(m_c - M) : 0, L = sum_c l_c w_c (half-wave
  // tree), o = sum_c fma(v_c, w_c) in split order, out = o / L.
  // per (head g, split cc) weight w = l ? exp(m - M_g) : 0 and L_g = sum l w,
  // by half-wave (NS = 32) or 16-lane row (NS = 16) reductions: lane t holds split t % NS of head t / NS
  float* pg0 = part0 + (size_t)g0 * NS * (HD + 2);  // head g0's partials
  float mv = -INFINITY, lv = 0.0f;
  if (t < GM * NS) {
    const float* pm = pg0 + ((size_t)(t / NS) * NS + t % NS) * (HD + 2) + HD;
    mv = ld_sc1(pm);
    lv = ld_sc1(pm + 1);
  }
  constexpr int PAIRS = (GM * HD + 255) / 256;
  float v[PAIRS][NS];
  // splits that own no key (c TK >= n_keys: m = -inf, l = 0, zero
  // accumulator, weight 0) are read out of bounds -- 0 without memory
  // traffic, and the loads stay unconditional (8-15 of 32 at pos 512-768)
  const int n_act = min(NS, (n_keys + TK - 1) / TK);
  const __amdgpu_buffer_rsrc_t rpart = buf_rsrc(pg0, (uint32_t)(GM * NS * (HD + 2) * 4));
#pragma unroll
  for (int p = 0; p < PAIRS; p++) {
    const int idx = min(t + p * 256, GM * HD - 1);
    const int eg = (idx / HD) * NS * (HD + 2) + idx % HD;
#pragma unroll
    for (int cc = 0; cc < NS; cc++)
      v[p][cc] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(
          rpart, cc < n_act ? (eg + cc * (HD + 2)) * 4 : (1 << 30), 0, BUF_SC1));
  }
  __shared__ float s_wt[G][NS];  // [GM] used
  __shared__ float s_L[G];
  ATTN_MARK(6);
  if (w < (GM * NS + 63) / 64) {  // whole waves
    const float M = NS == 32 ? half_max(mv) : row16_max(mv);
    const float wt = lv == 0.0f ? 0.0f : expf(mv - M);
    const float L = NS == 32 ? half_sum(lv * wt) : row16_sum(lv * wt);
    if (t < GM * NS) {
      s_wt[t / NS][t % NS] = wt;
      if (t % NS == 0) s_L[t / NS] = L;
    }
  }
  __syncthreads();
  float* s_out = TK * KS * 2 >= G * HD * 4 ? reinterpret_cast<float*>(s_k) : s_outbuf;  // [GM][HD]
#pragma unroll
  for (int p = 0; p < PAIRS; p++) {
    const int idx = t + p * 256;
    if (idx < GM * HD) {
      const int g = idx / HD;
      float o = 0.0f;
#pragma unroll
      for (int cc = 0; cc < NS; cc++) o = fmaf(v[p][cc], s_wt[g][cc], o);
      const float val = o / s_L[g];
      a.out[((size_t)hkv * G + g0) * HD + idx] = val;
      s_out[idx] = val;
    }
  }
  ATTN_MARK(7);
  if (a.q8 != nullptr && HD % 32 == 0) {  // Q8_0 blocks of the heads' outputs (ops.cpp:116-139), 4 lanes per block
    __syncthreads();
    constexpr int NBK = HD % 32 == 0 ? G * HD / 32 : 1, NBM = HD % 32 == 0 ? GM * HD / 32 : 1;
    __shared__ __attribute__((aligned(16))) XBlock s_q8[BLK ? NBK : 1];
    for (int i = t; i < GM * HD / 8; i += 256) {
      const float4 f0 = reinterpret_cast<const float4*>(s_out)[2 * i], f1 = reinterpret_cast<const float4*>(s_out)[2 * i + 1];
      const float vv[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
      XBlock* xb = BLK ? s_q8 + (i >> 2) : a.q8 + ((size_t)hkv * G + g0) * HD / 32 + (i >> 2);
      if (a.q8k) q8k_block_quad(vv, i & 3, xb);
      else q8_block_quad(vv, i & 3, xb);
    }
    if constexpr (BLK) {  // the blocks' words as granules for the o projection
      __syncthreads();
      const uint32_t tag = btag;
      uint2* dst = bs.g_xo + ((size_t)hkv * NBK + (size_t)g0 * HD / 32) * 12;
      const uint32_t* src = reinterpret_cast<const uint32_t*>(s_q8);
      for (int i = t; i < NBM * 12; i += 256) st_granule(dst + i, src[i], tag);
      BLK_MARK(bs, 4);
    }
  }
  ATTN_MARK(5);
  if (reset && t == 0) __hip_atomic_store(a.ticket + hkv, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
  };


  if (kp == 0) {
#pragma unroll
    for (int g = 0; g < G; g++)
#pragma unroll
      for (int e = 0; e < 4; e++) st_sc1(part0 + ((size_t)g * NS + c) * (HD + 2) + d_own + e, acc[g][e]);
  }
  if (w < G && lane == 0) {
    st_sc1(part0 + ((size_t)w * NS + c) * (HD + 2) + HD, m_run);
    st_sc1(part0 + ((size_t)w * NS + c) * (HD + 2) + HD + 1, l_run);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // DUAL (the block with G = 2): the last split merges head 1 and the second-to-last, once the last ticket is
  // in, merges head 0 -- the two merges run in parallel instead of one work-group reading both heads' partials
  constexpr bool DUAL = BLK && G == 2;
  if (t == 0) {
    const unsigned old = __hip_atomic_fetch_add(a.ticket + hkv, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = old == NS - 1 ? 1 : (DUAL && old == NS - 2) ? 2 : 0;
  }
  __syncthreads();
  ATTN_MARK(4);
  BLK_MARK(bs, 3);
  const int role = s_last;
  if (role == 0) return;
  if constexpr (DUAL) {
    if (role == 2) {  // every partial is published once the ticket reaches NS (bounded wait)
      __shared__ int s_ok;
      if (t == 0) {
        int n = 0;
        s_ok = 1;
        const uint64_t t0 = wall_clock64();
        while (__hip_atomic_load(a.ticket + hkv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)NS) {
          if (++n >= BLOCK_SPIN_LIMIT) {
            __hip_atomic_store(bs.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_ok = 0;
            break;
          }
        }
        if (wall_clock64() - t0 > BLOCK_SLOW_TICKS)
          __hip_atomic_fetch_add(bs.err + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      // timed out: no merge from incomplete partials and no ticket reset (the
      // slow split still adds to it); the host zeroes every ticket when it
      // reports the error (Session::check_device_error)
      if (s_ok == 0) return;
    }
    merge_heads(std::integral_constant<int, 1>{}, role == 1 ? 1 : 0, role == 2);
  } else {
    merge_heads(std::integral_constant<int, G>{}, 0, true);
  }
  // the launch's tag advance (BlockSync::done): the kv head's last split counts once, its merged blocks published
  // (every split of the head incremented the ticket after its granule waits, so each had used the tag)
  if (BLK && role == 1 && t == 0) block_count_done(block_count(bs.done), bs.done_n, bs.done, bs.epoch);
}

// Key tiles of 32 keys while every split owns at most one tile (short
// context: half the bytes per work-group before its first score), 64 keys
// beyond (fewer tile rounds per split).  scripts/ab A/B, 4B shapes: pos 100
// 7.8 vs 9.0 us, pos 700 8.3 vs 9.2 us with 32-key tiles; 64-key tiles win
// from pos ~1000 (2000: 9.9 vs 10.2 us).
template <int HD, int G, bool FUSED, int KVD = 1>
__global__ __launch_bounds__(256) void attn_split_kernel(AttnArgs a, QKVArgs qa) {
  // K/V tiles and the PV reduction buffer sized once for 64-key tiles (the
  // two bodies share them: LDS size sets how fast work-groups are dispatched)
  constexpr int KS = attn_ks<HD, G>(), KP = attn_kp<HD, G>();
  __shared__ __attribute__((aligned(16))) uint16_t s_k[64 * KS];
  __shared__ __attribute__((aligned(16))) uint16_t s_v[64 * HD];
  __shared__ __attribute__((aligned(16))) float s_red[KP > 1 ? KP * G * HD : 4];
  if (*a.d_pos + 1 <= 32 * ATTN_NSPLIT)
    attn_split_body<HD, G, FUSED, 32, false, KVD>(a, qa, s_k, s_v, s_red, blockIdx.x, blockIdx.y, BlockSync{});
  else
    attn_split_body<HD, G, FUSED, 64, false, KVD>(a, qa, s_k, s_v, s_red, blockIdx.x, blockIdx.y, BlockSync{});
}

template <int HD, int G>
static void launch_split_g(const AttnArgs& a, const QKVArgs* fused, hipStream_t s) {
  // (GQA pairs as two virtual kv heads of one q head measured slower on 27B: 213 vs 216 tok/s)
  const dim3 grid(a.n_head_kv, ATTN_NSPLIT);
  if (fused)
    hipLaunchKernelGGL((attn_split_kernel<HD, G, true>), grid, dim3(256), 0, s, a, *fused);
  else
    hipLaunchKernelGGL((attn_split_kernel<HD, G, false>), grid, dim3(256), 0, s, a, QKVArgs{});
}

// GQA group 8 (Gemma-4 E2B: 8 q heads on one kv head): two sets of
// work-groups of 4 q heads each read the same cache head (the history is
// read twice; the 4-head body's registers and LDS are unchanged)
template <int HD>
static void launch_split_g8(const AttnArgs& a, const QKVArgs* fused, hipStream_t s) {
  if (fused) throw std::runtime_error("attention: GQA group 8 runs the unfused q/k launch");
  const dim3 grid(a.n_head_kv * 2, ATTN_NSPLIT);
  hipLaunchKernelGGL((attn_split_kernel<HD, 4, false, 2>), grid, dim3(256), 0, s, a, QKVArgs{});
}

template <int HD>
static void launch_split(const AttnArgs& a, const QKVArgs* fused, hipStream_t s) {
  switch (a.n_head / a.n_head_kv) {
    case 1: launch_split_g<HD, 1>(a, fused, s); break;
    case 2: launch_split_g<HD, 2>(a, fused, s); break;
    case 4: launch_split_g<HD, 4>(a, fused, s); break;
    case 8: launch_split_g8<HD>(a, fused, s); break;
    default: throw std::runtime_error("attention: GQA group must be 1, 2, 4 or 8");
  }
}

void launch_attention(const AttnArgs& a, bool exact, hipStream_t s, const QKVArgs* fused) {
  if (exact) {
    hipLaunchKernelGGL(attn_exact_kernel, dim3(a.n_head), dim3(256), 0, s, a);
    LLMI_HIP(hipGetLastError());
    return;
  }
  if (a.n_head_kv <= 0 || a.n_head % a.n_head_kv != 0) throw std::runtime_error("attention: n_head % n_head_kv != 0");
  if (!a.partial || !a.ticket || !a.out) throw std::runtime_error("attention: missing partial / ticket / out buffer");
  if (a.q8k && (a.n_head / a.n_head_kv) * a.head_dim % 256 != 0 && (a.n_head / a.n_head_kv) != 8)
    throw std::runtime_error("attention: Q8_K output needs whole super-blocks per kv head");
  switch (a.head_dim) {
    case 16: launch_split<16>(a, fused, s); break;
    case 32: launch_split<32>(a, fused, s); break;
    case 64: launch_split<64>(a, fused, s); break;
    case 128: launch_split<128>(a, fused, s); break;
    case 256: launch_split<256>(a, fused, s); break;
    default: throw std::runtime_error("attention: unsupported head_dim " + std::to_string(a.head_dim));
  }
  LLMI_HIP(hipGetLastError());
}


// ---------------------------------------------------------------------------
// Attention block: the qkv projection, attention and the o projection of one
// decode layer in ONE launch (fast single-device path).  Work-group roles by
// index: [0, nq) the qkv GEMV (layer_body, PLAIN for layer 0 else PRO:
// residual + norms + Q8_0 in the prologue), [nq, nq + n_kv NSPLIT) the split
// attention (attn_split_body, 32-key tiles), then the o GEMV (layer_body
// PLAIN).  Every hand-off goes one way, from lower to higher work-group
// indices, as data-tagged granules (common.h): the qkv work-groups store their
// rows as {value, tag}; a kv head's attention work-groups issue their first
// K/V tile, then re-load the head's q/k/v row granules until the tags are this
// launch's; the split partials meet in the last-arriving work-group per head
// (agent ticket, as in the standalone kernel), which stores the heads' Q8_0
// blocks as granules; the o work-groups issue their weight slices, then
// re-load the block granules.  So the o weights and the K/V history stream
// while the qkv GEMV runs, and no hand-off waits on a drain or a counter.
// The tag is the layer's launch count + 1 (BlockSync::epoch), advanced by the
// launch itself once every wave of it has used it (BlockSync::done, common.h
// block_count); waits are bounded (a timeout sets bs.err, the host reports
// it).  Numerics are those of the three separate kernels (same
// bodies, same per-row order) except the o rows' lane order (R4).
// ---------------------------------------------------------------------------
namespace {

template <int HD, int G>
constexpr size_t block_attn_lds() {  // s_k + s_v (32-key tiles) + s_red
  return (size_t)32 * attn_ks<HD, G>() * 2 + (size_t)32 * HD * 2 +
         (attn_kp<HD, G>() > 1 ? (size_t)attn_kp<HD, G>() * G * HD * 4 : 16);
}

// WTQ / WTO: weight formats of qkv and o (layer_body WT: 0 Q4_0, or kq Q4_K /
// Q6_K); WTQB != 0: the qkv rows from nqa work-groups on are a second weight
// of that format (Q4_K_M: q|k Q4_K, v Q6_K), granules and outputs continuing
// after the first weight's rows
constexpr int WT_W8 = 3;  // Q8_0 weights in the block (layer_body W8), beside the kq formats WT_Q4_K / WT_Q6_K

// PXF: the qkv prologue / o epilogue honour the fused exchange (tensor-parallel ranks; layer_body PXF)
template <int HD, int G, int QR, int QP, int QE, int QROLE, int OR, int OP, int OE, int WTQ = 0, int WTQB = 0,
          int WTO = 0, int KVD = 1, int NS = ATTN_NSPLIT, bool PXF = false>
__global__ __launch_bounds__(256) void attn_block_kernel(LayerGemv qg, LayerGemv og, AttnArgs aa, QKVArgs qa,
                                                        BlockSync bs, int nq, LayerGemv qgb, int nqa) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  int b = blockIdx.x;
  const int na = aa.n_head_kv * NS;
  if (b < nq) {
    bool second = false;
    if constexpr (WTQB != 0) {
      if (b >= nqa) {
        second = true;
        BlockSync bsb = bs;
        bsb.g_qkv += qg.rows;
        layer_body<QR, 4, QP, QE, QROLE, false, true, SYNC_SIG, 0, false, WTQB == WT_W8 ? 0 : WTQB>(qgb, b - nqa, s_dyn, bsb);
      }
    }
    if (!second)
      layer_body<QR, 4, QP, QE, QROLE, false, true, SYNC_SIG, 0, WTQ == WT_W8, WTQ == WT_W8 ? 0 : WTQ, 0, PXF>(qg, b, s_dyn,
                                                                                                           bs);
  } else if (b - nq < na) {
    b -= nq;
    constexpr int KS = attn_ks<HD, G>();
    uint16_t* s_k = reinterpret_cast<uint16_t*>(s_dyn);
    uint16_t* s_v = s_k + 32 * KS;
    float* s_red = reinterpret_cast<float*>(s_v + 32 * HD);
    // KVD > 1: aa.n_head_kv counts virtual kv heads (G q heads each, KVD per cache head)
    attn_split_body<HD, G, true, 32, true, KVD, NS>(aa, qa, s_k, s_v, s_red, b % aa.n_head_kv, b / aa.n_head_kv, bs);
  } else {
    b -= nq + na;
    layer_body<OR, 4, OP, OE, ROLE_PLAIN, false, true, SYNC_WAIT, 0, WTO == WT_W8, WTO == WT_W8 ? 0 : WTO, 0, PXF>(og, b, s_dyn,
                                                                                                            bs);
  }
}

using BlockFn = void (*)(dim3, size_t, const LayerGemv&, const LayerGemv&, const AttnArgs&, const QKVArgs&,
                         const BlockSync&, int, const LayerGemv&, int, hipStream_t);

template <int HD, int G, int QR, int QP, int QE, int QROLE, int OR, int OP, int OE, int WTQ, int WTQB, int WTO,
          int KVD = 1, int NS = ATTN_NSPLIT>
void block_launch(dim3 grid, size_t lds, const LayerGemv& qg, const LayerGemv& og, const AttnArgs& aa,
                  const QKVArgs& qa, const BlockSync& bs, int nq, const LayerGemv& qgb, int nqa, hipStream_t s) {
  if (qg.px || og.px) {  // the fused-exchange variant (tensor-parallel ranks): co-resident too, or refused
    auto kern = attn_block_kernel<HD, G, QR, QP, QE, QROLE, OR, OP, OE, WTQ, WTQB, WTO, KVD, NS, true>;
    int per_cu = 0, n_cu = 0, dev = 0;
    LLMI_HIP(hipGetDevice(&dev));
    LLMI_HIP(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev));
    LLMI_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(kern), 256, lds));
    if ((long)grid.x > (long)std::max(0, per_cu - 1) * n_cu)
      throw std::runtime_error("attention block: the fused-exchange variant's grid is not co-resident");
    hipLaunchKernelGGL(kern, grid, dim3(256), lds, s, qg, og, aa, qa, bs, nq, qgb, nqa);
    return;
  }
  KernelTiming& kt = kernel_timing();
  if (kt.start) {  // bench: events signalled by this dispatch itself (its duration as rocprofv3 reports it)
    hipExtLaunchKernelGGL((attn_block_kernel<HD, G, QR, QP, QE, QROLE, OR, OP, OE, WTQ, WTQB, WTO, KVD, NS>), grid, dim3(256),
                          (uint32_t)lds, s, kt.start, kt.stop, 0u, qg, og, aa, qa, bs, nq, qgb, nqa);
    kt = KernelTiming{};
    return;
  }
  hipLaunchKernelGGL((attn_block_kernel<HD, G, QR, QP, QE, QROLE, OR, OP, OE, WTQ, WTQB, WTO, KVD, NS>), grid, dim3(256), lds, s,
                     qg, og, aa, qa, bs, nq, qgb, nqa);
}

struct BlockCfg {
  int nb_qkv, nb_o, hd, g, qrole;
  int QR, QP, QE, OR, OP, OE;
  size_t attn_lds;
  BlockFn fn;
  const void* kern;  // the kernel (occupancy query)
  int wtq, wtqb, wto;  // weight formats (layer_body WT): qkv, second qkv weight (0: none), o
  int kvd;             // virtual kv heads per cache head (attention work-groups of g / kvd q heads)
  int ns = ATTN_NSPLIT;  // key-range splits per kv head
};
#define LLMI_BCFGW(NBQ, NBO, HD, G, QROLE, QR, QP, QE, OR, OP, OE, WTQ, WTQB, WTO)                          \
  {NBQ, NBO, HD, G, QROLE, QR, QP, QE, OR, OP, OE, block_attn_lds<HD, G>(),                                  \
   block_launch<HD, G, QR, QP, QE, QROLE, OR, OP, OE, WTQ, WTQB, WTO>,                                        \
   reinterpret_cast<const void*>(&attn_block_kernel<HD, G, QR, QP, QE, QROLE, OR, OP, OE, WTQ, WTQB, WTO>), WTQ, \
   WTQB, WTO, 1}
// GQA group GM split over KVD virtual kv heads (G = GM / KVD q heads per attention work-group); WT: the
// weight format of qkv and o (0 Q4_0, WT_W8 Q8_0: P counts 16-B half-block passes)
#define LLMI_BCFGVW(NBQ, NBO, HD, GM, KVD, QROLE, QR, QP, QE, OR, OP, OE, WT)                                       \
  {NBQ, NBO, HD, GM, QROLE, QR, QP, QE, OR, OP, OE, block_attn_lds<HD, GM / KVD>(),                                 \
   block_launch<HD, GM / KVD, QR, QP, QE, QROLE, OR, OP, OE, WT, 0, WT, KVD>,                                       \
   reinterpret_cast<const void*>(&attn_block_kernel<HD, GM / KVD, QR, QP, QE, QROLE, OR, OP, OE, WT, 0, WT, KVD>), WT, \
   0, WT, KVD}
#define LLMI_BCFGV(NBQ, NBO, HD, GM, KVD, QROLE, QR, QP, QE, OR, OP, OE) \
  LLMI_BCFGVW(NBQ, NBO, HD, GM, KVD, QROLE, QR, QP, QE, OR, OP, OE, 0)
#define LLMI_BCFG(NBQ, NBO, HD, G, QROLE, QR, QP, QE, OR, OP, OE) \
  LLMI_BCFGW(NBQ, NBO, HD, G, QROLE, QR, QP, QE, OR, OP, OE, 0, 0, 0)
// NS key-range splits per kv head instead of ATTN_NSPLIT (Q4_0)
#define LLMI_BCFGS(NBQ, NBO, HD, G, QROLE, QR, QP, QE, OR, OP, OE, NS)                                            \
  {NBQ, NBO, HD, G, QROLE, QR, QP, QE, OR, OP, OE, block_attn_lds<HD, G>(),                                        \
   block_launch<HD, G, QR, QP, QE, QROLE, OR, OP, OE, 0, 0, 0, 1, NS>,                                             \
   reinterpret_cast<const void*>(&attn_block_kernel<HD, G, QR, QP, QE, QROLE, OR, OP, OE, 0, 0, 0, 1, NS>), 0, 0, 0, 1, NS}
// qkv: 4 waves x QR rows per work-group (rows per work-group must divide
// head_dim); o: 4 waves x OR rows.  E as in k_layer.hip's table.
const BlockCfg kBlockCfgs[] = {
    // 4B: qkv 4096 rows -> 256 WGs, o 2560 -> 80 WGs (8 rows per wave: fewer
    // work-groups polling the merged blocks; A/B 913-915 vs 910 tok/s with 4
    // rows per wave (160 WGs), 902 with 2 (320 WGs))
    LLMI_BCFG(80, 64, 256, 2, ROLE_PRO, 4, 5, 10, 8, 8, 1),
    LLMI_BCFG(80, 64, 256, 2, ROLE_PLAIN, 4, 5, 1, 8, 8, 1),   // 4B layer 0
    // 1B: GQA group 4 as two virtual kv heads of 2 (64 attention WGs, two merges of 2 heads)
    LLMI_BCFGV(36, 32, 256, 4, 2, ROLE_PRO, 4, 3, 5, 4, 2, 1),
    LLMI_BCFGV(36, 32, 256, 4, 2, ROLE_PLAIN, 4, 3, 1, 4, 2, 1),
    LLMI_BCFG(36, 32, 256, 4, ROLE_PRO, 4, 3, 5, 4, 2, 1),     // 1B:  qkv 1536 rows -> 96 WGs, o 1152 -> 72
    LLMI_BCFG(36, 32, 256, 4, ROLE_PLAIN, 4, 3, 1, 4, 2, 1),   // 1B layer 0
    // 1B Q8_0 (BASELINE configs[3]): the same, Q8_0 weights (72 / 64 half-block units per qkv / o row)
    LLMI_BCFGVW(36, 32, 256, 4, 2, ROLE_PRO, 4, 5, 5, 4, 4, 1, WT_W8),
    LLMI_BCFGVW(36, 32, 256, 4, 2, ROLE_PLAIN, 4, 5, 1, 4, 4, 1, WT_W8),
    // 4B Q4_K_M (kq weights): q|k Q4_K + v Q6_K, or all Q4_K; o Q4_K; the Q4_0 geometry
    LLMI_BCFGW(80, 64, 256, 2, ROLE_PRO, 4, 5, 10, 8, 8, 1, WT_Q4_K, WT_Q6_K, WT_Q4_K),
    LLMI_BCFGW(80, 64, 256, 2, ROLE_PLAIN, 4, 5, 1, 8, 8, 1, WT_Q4_K, WT_Q6_K, WT_Q4_K),
    LLMI_BCFGW(80, 64, 256, 2, ROLE_PRO, 4, 5, 10, 8, 8, 1, WT_Q4_K, 0, WT_Q4_K),
    LLMI_BCFGW(80, 64, 256, 2, ROLE_PLAIN, 4, 5, 1, 8, 8, 1, WT_Q4_K, 0, WT_Q4_K),
    // 27B (PLAIN only: the residual + norms run as their own launch, whose 5376-wide prologue would not fit the
    // registers): qkv 8192 rows -> 256 WGs, 16 kv heads x 16 splits -> 256 attention WGs, o 5376 -> 168 WGs
    // (680 in all; with 32 splits and 4 rows per wave, 1192, the grid is not co-resident)
    LLMI_BCFGS(168, 128, 128, 2, ROLE_PLAIN, 8, 21, 2, 8, 16, 2, 16),
};
#undef LLMI_BCFG
#undef LLMI_BCFGW

int wt_of_w(const DevWeight* w) {
  if (!w) return 0;
  return w->type == T_Q4_K ? WT_Q4_K : w->type == T_Q6_K ? WT_Q6_K : w->type == T_Q8_0 ? WT_W8 : 0;
}

const BlockCfg* find_block_cfg(int nb_qkv, int nb_o, int hd, int g, int qrole, int wtq = 0, int wtqb = 0,
                               int wto = 0) {
  for (const auto& c : kBlockCfgs)
    if (c.nb_qkv == nb_qkv && c.nb_o == nb_o && c.hd == hd && c.g == g && c.qrole == qrole && c.wtq == wtq &&
        c.wtqb == wtqb && c.wto == wto)
      return &c;
  return nullptr;
}

void fill_gemv(const DevWeight& w, LayerGemv& a) {
  a.qs = reinterpret_cast<const uint4*>(w.qs);
  a.wd = w.d;
  a.kdd = w.kdd;
  a.kqh = w.kqh;
  a.slab = w.slab;
  a.rows = w.rows;
  a.nb = w.cols / 32;
  a.magic = div_magic(a.nb);
  a.n = w.cols;
}

}  // namespace

// grid and dynamic LDS of one attention-block launch (qkv WGs, attention WGs, o WGs)
struct BlockGeom {
  int nq, na, no;
  size_t lds;
};
static BlockGeom block_geom(const BlockCfg& c, const DevWeight& wqkv, const DevWeight* wqkv_b, const DevWeight& wo,
                            int n_head_kv, int qrole) {
  BlockGeom g;
  g.nq = (wqkv.rows + (wqkv_b ? wqkv_b->rows : 0) + 4 * c.QR - 1) / (4 * c.QR);
  g.na = n_head_kv * c.kvd * c.ns;
  g.no = (wo.rows + 4 * c.OR - 1) / (4 * c.OR);
  const size_t lds_q = (size_t)(wqkv.cols / 32) * sizeof(XBlock) + 16 + (qrole == ROLE_PRO ? (size_t)wqkv.cols * 4 : 0);
  const size_t lds_o = (size_t)(wo.cols / 32) * sizeof(XBlock) + 16;
  g.lds = std::max({lds_q, lds_o, c.attn_lds});
  return g;
}

// Deadlock freedom.  The block's waits go one way only: attention
// work-groups wait for qkv work-groups' granules, o work-groups for the
// merged blocks; no producer ever waits for a consumer.  HIP promises no
// dispatch order (MI355X_MICROARCH, correctness boundaries), so the launch is
// admitted only if EVERY work-group of the grid can be resident at once:
// then each producer holds (or will get) a slot regardless of which
// work-groups were dispatched first, and all spins end.  The occupancy API can
// report one block per CU too many at these SGPR counts (98-100, same table),
// so one block per CU is kept in reserve.  A wait that still overruns its
// bound sets bs.err (reported, never silently used).
static bool block_co_resident(const BlockCfg& c, const BlockGeom& g) {
  static int n_cu = 0;
  if (n_cu == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return false;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, c.kern, 256, g.lds) != hipSuccess) return false;
  const long capacity = (long)std::max(0, per_cu - 1) * n_cu;
  return g.nq + g.na + g.no <= capacity;
}

bool attn_block_supported(const DevWeight& wqkv, const DevWeight* wqkv_b, const DevWeight& wo, int head_dim,
                          int n_head, int n_head_kv, int qrole) {
  const bool q40 = (wqkv.type == T_Q4_0 || wqkv.type == T_Q8_0) && wo.type == wqkv.type && !wqkv_b && !wqkv.slab &&
                   !wo.slab;
  const bool kq = wqkv.kq && wo.kq && (!wqkv_b || (wqkv_b->kq && wqkv_b->cols == wqkv.cols));
  if (!q40 && !kq) return false;
  if (wqkv.cols % 32 || wo.cols % 32 || n_head_kv <= 0 || n_head % n_head_kv) return false;
  const int g = n_head / n_head_kv;
  for (int role : {qrole}) {
    const BlockCfg* c = find_block_cfg(wqkv.cols / 32, wo.cols / 32, head_dim, g, role, wt_of_w(&wqkv),
                                       wt_of_w(wqkv_b), wt_of_w(&wo));
    if (!c || head_dim % (4 * c->QR) != 0) return false;
    if (wqkv_b && wqkv.rows % (4 * c->QR) != 0) return false;
    if (!block_co_resident(*c, block_geom(*c, wqkv, wqkv_b, wo, n_head_kv, role))) return false;
  }
  return wqkv.rows + (wqkv_b ? wqkv_b->rows : 0) == (n_head + 2 * n_head_kv) * head_dim &&
         wo.cols == n_head * head_dim;
}

int launch_attn_block(const DevWeight& wqkv, const DevWeight* wqkv_b, LayerGemv qg, int qrole, const DevWeight& wo,
                      LayerGemv og, const AttnArgs& aa, const QKVArgs& qa, BlockSync bs, hipStream_t s) {
  if (!attn_block_supported(wqkv, wqkv_b, wo, aa.head_dim, aa.n_head, aa.n_head_kv, qrole))
    throw std::runtime_error("attention block: unsupported shapes");
  const int g = aa.n_head / aa.n_head_kv, hd = aa.head_dim;
  const BlockCfg& c = *find_block_cfg(wqkv.cols / 32, wo.cols / 32, hd, g, qrole, wt_of_w(&wqkv), wt_of_w(wqkv_b),
                                      wt_of_w(&wo));
  if ((c.wto == WT_Q4_K || c.wto == WT_Q6_K) != (aa.q8k != 0))
    throw std::runtime_error("attention block: a kq o projection reads Q8_K blocks (and only it)");
  if (!bs.epoch || !bs.done || !bs.g_qkv || !bs.g_xo || !bs.err || !aa.q8 || !aa.partial || !aa.ticket || !qa.qkv ||
      qa.qkv != qg.out)
    throw std::runtime_error("attention block: missing buffers");
  if (qrole == ROLE_PRO ? (!qg.y || !qg.resid_in || !qg.resid_out || !qg.w_next || qg.resid_in == qg.resid_out)
                        : !qg.xg)
    throw std::runtime_error("attention block: missing qkv operands");
  if (og.xg != aa.q8 || !og.out) throw std::runtime_error("attention block: o projection must read the merged blocks");
  fill_gemv(wqkv, qg);
  fill_gemv(wo, og);
  LayerGemv qgb = qg;
  if (wqkv_b) {
    fill_gemv(*wqkv_b, qgb);
    qgb.out = qg.out + wqkv.rows;
    qgb.resid_out = nullptr;
    qgb.xn_out = nullptr;
  }
  const int nbq = qg.nb, nbo = og.nb;
  // one pass group per lane (no MULTI) and enough prologue / x-copy slots
  auto passes = [](int nb, int R) { return (nb + 64 / R - 1) / (64 / R); };
  const int uq = c.wtq == WT_W8 ? 2 * nbq : nbq, uo = c.wto == WT_W8 ? 2 * nbo : nbo;  // 16-B units per row
  if (passes(uq, c.QR) > c.QP || passes(uo, c.OR) > c.OP) throw std::runtime_error("attention block: P too small");
  if (qrole == ROLE_PRO ? wqkv.cols > c.QE * 256 : 3 * nbq > c.QE * 256) throw std::runtime_error("attention block: qkv E");
  if (3 * nbo > c.OE * 256) throw std::runtime_error("attention block: o E");
  const BlockGeom bg = block_geom(c, wqkv, wqkv_b, wo, aa.n_head_kv, qrole);
  const int nqa = wqkv_b ? wqkv.rows / (4 * c.QR) : bg.nq;
  AttnArgs av = aa;  // virtual kv heads: the attention role's head count
  av.n_head_kv *= c.kvd;
  if (og.px && og.px_out >= 0 && bg.no > PX_MAX_CS) throw std::runtime_error("attention block: more fused-exchange producers than checksum slots");
  if (qg.px && qg.px_in >= 0 && (qg.px_in_nwg <= 0 || qg.px_in_nwg > PX_MAX_CS)) throw std::runtime_error("attention block: fused exchange read without its producer count");
  bs.done_n = (unsigned)(bg.no + av.n_head_kv);  // the o work-groups and the kv heads' final merges (k_attn: role 1)
  c.fn(dim3(bg.nq + bg.na + bg.no), bg.lds, qg, og, av, qa, bs, bg.nq, qgb, nqa, s);
  LLMI_HIP(hipGetLastError());
  return bg.no;
}

}  // namespace llmi
