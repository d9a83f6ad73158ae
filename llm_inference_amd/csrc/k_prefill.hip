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
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void store_f16x8(uint16_t* dst, const float (&v)[8]) {  // 16-B aligned
  uint4 o;
  o.x = __builtin_bit_cast(uint32_t, f16x2v{(_Float16)v[0], (_Float16)v[1]});
  o.y = __builtin_bit_cast(uint32_t, f16x2v{(_Float16)v[2], (_Float16)v[3]});
  o.z = __builtin_bit_cast(uint32_t, f16x2v{(_Float16)v[4], (_Float16)v[5]});
  o.w = __builtin_bit_cast(uint32_t, f16x2v{(_Float16)v[6], (_Float16)v[7]});
  *reinterpret_cast<uint4*>(dst) = o;
}

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
template <int NWAVE>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float m = 0.0f;
#pragma unroll
  for (int i = 0; i < NWAVE; i++) m = fmaxf(m, red[i]);
  __syncthreads();
  return m;
}

// f16 activations of the f16 prefill (GEMM v7): a token's row is its Q8_0 blocks (quantize_row_q8_0,
// ops.cpp:116-139 -- the values the reference's mat_vec_mul reads) dequantized and scaled by 2^-s, s chosen per
// token from the row's max |x| so that the largest value lands in [2^14, 2^15): f16(f16(d) q 2^-s) is the
// reference's d q to one f16 rounding with no overflow, and the power of two is exact (the GEMM multiplies its
// outputs by 2^s).  token_xs returns 2^-s (1 for an all-zero or non-finite row) and stores 2^s.
__device__ __forceinline__ float token_xs(float amax, float* tscale) {
  int f = 127;
  if (amax > 0.0f && amax <= 3.4e38f) {
    const int e = (int)((__float_as_uint(amax) >> 23) & 0xFFu) - 127;
    f = min(max(127 + 14 - e, 2), 252);
  }
  if (tscale) *tscale = __uint_as_float((uint32_t)(254 - f) << 23);
  return __uint_as_float((uint32_t)f << 23);
}
// one Q8_0 block held by a DPP quad of lanes (8 elements each, as q8_block_quad: the same max, d and quants),
// written as the 8 f16 values f16(f16(d) q xs); every lane of the quad must execute it
__device__ __forceinline__ void q8_f16_quad(const float (&v)[8], float xs, uint16_t* dst) {
  float amax = 0.0f;
#pragma unroll
  for (int k = 0; k < 8; k++) amax = fmaxf(amax, fabsf(v[k]));
  amax = fmaxf(amax, dpp_f<DPP_QUAD_1032>(amax));
  amax = fmaxf(amax, dpp_f<DPP_QUAD_2301>(amax));
  const float dd = amax / 127.0f;
  const float id = dd != 0.0f ? 1.0f / dd : 0.0f;
  const float ds = h2f(f2h_ggml(dd)) * xs;  // exact (a power of two)
  float o[8];
#pragma unroll
  for (int k = 0; k < 8; k++) o[k] = (float)nearest_int_fma(v[k], id) * ds;  // exact in f32: 11 x 7 bits
  store_f16x8(dst, o);
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
  if (a.x16) {  // f16 rows of the token's dequantized Q8_0 blocks, scaled per token (token_xs)
    float amax = 0.0f;
    for (int i = t; i < n; i += 256) amax = fmaxf(amax, fabsf(s_x[i]));
    const float xs = token_xs(block_max<4>(amax, s_red), t == 0 && a.tscale ? a.tscale + tok : nullptr);
    for (int i = t; i < n / 8; i += 256) {  // a DPP quad per block (n % 32 == 0: whole quads)
      const float4 f0 = reinterpret_cast<const float4*>(s_x)[2 * i], f1 = reinterpret_cast<const float4*>(s_x)[2 * i + 1];
      const float vv[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
      q8_f16_quad(vv, xs, a.x16 + (size_t)tok * a.x16stride + 8 * i);
    }
    return;
  }
  XBlock* xq = a.xq + (size_t)tok * a.xstride;
  for (int i = t; i < n / 8; i += 256) {  // a DPP quad of lanes per Q8_0 block (Q8_K: a half-wave per super-block)
    const float4 f0 = reinterpret_cast<const float4*>(s_x)[2 * i], f1 = reinterpret_cast<const float4*>(s_x)[2 * i + 1];
    const float vv[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
    if (a.q8k) q8k_block_quad(vv, i & 3, xq + (i >> 2));
    else q8_block_quad(vv, i & 3, xq + (i >> 2));
  }
}


// residual mode, vectorized: a DPP quad of lanes per Q8_0 block (lane t & 3 owns elements 8 (t & 3) ..
// + 7 of block t / 4 + 64 k), float4 loads, x quantized from registers (the decode layer prologue's scheme,
// layer_body.h); EB = ceil(nb / 64) rounds.  Per token the same arithmetic whatever the chunk.
template <int EB>
__global__ __launch_bounds__(256) void prefill_norm_res_kernel(PrefillNorm a) {
  __shared__ float s_red[4];
  const int t = threadIdx.x, tok = blockIdx.x, n = a.n, nb = n / 32, sub = t & 3;
  float* resid = a.resid + (size_t)tok * n;
  const float* y = a.y + (size_t)tok * n;
  float4 y4[EB][2], r4[EB][2];
  auto in_row = [&](int k) { return t / 4 + 64 * k < nb; };
#pragma unroll
  for (int k = 0; k < EB; k++) {
    const int e = (min(t / 4 + 64 * k, nb - 1) * 32 + sub * 8) / 4;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      y4[k][h] = reinterpret_cast<const float4*>(y)[e + h];
      r4[k][h] = reinterpret_cast<const float4*>(resid)[e + h];
    }
  }
  float sc1 = 0.0f;
  if (a.w_post) {
    float ss = 0.0f;
#pragma unroll
    for (int k = 0; k < EB; k++)
      if (in_row(k))
#pragma unroll
        for (int h = 0; h < 2; h++) {
          ss = fmaf(y4[k][h].x, y4[k][h].x, ss);
          ss = fmaf(y4[k][h].y, y4[k][h].y, ss);
          ss = fmaf(y4[k][h].z, y4[k][h].z, ss);
          ss = fmaf(y4[k][h].w, y4[k][h].w, ss);
        }
    sc1 = rms_scale_pf(block_sum<4>(ss, s_red), n, a.eps);
  }
  float ss2 = 0.0f;
#pragma unroll
  for (int k = 0; k < EB; k++) {
    const int e = (min(t / 4 + 64 * k, nb - 1) * 32 + sub * 8) / 4;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      float4& r = r4[k][h];
      const float4 yv = y4[k][h];
      if (a.w_post) {
        const float4 wp = reinterpret_cast<const float4*>(a.w_post)[e + h];
        r.x += (sc1 * yv.x) * wp.x;
        r.y += (sc1 * yv.y) * wp.y;
        r.z += (sc1 * yv.z) * wp.z;
        r.w += (sc1 * yv.w) * wp.w;
      } else {
        r.x += yv.x;
        r.y += yv.y;
        r.z += yv.z;
        r.w += yv.w;
      }
      if (in_row(k)) {
        ss2 = fmaf(r.x, r.x, ss2);
        ss2 = fmaf(r.y, r.y, ss2);
        ss2 = fmaf(r.z, r.z, ss2);
        ss2 = fmaf(r.w, r.w, ss2);
        reinterpret_cast<float4*>(resid)[e + h] = r;
      }
    }
  }
  const float sc2 = rms_scale_pf(block_sum<4>(ss2, s_red), n, a.eps);
  XBlock* xq = a.xq + (size_t)tok * a.xstride;
  float v[EB][8];
  float amax = 0.0f;
#pragma unroll
  for (int k = 0; k < EB; k++) {
    const int b = min(t / 4 + 64 * k, nb - 1), e = (b * 32 + sub * 8) / 4;
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const float4 r = r4[k][h], wn = reinterpret_cast<const float4*>(a.w_next)[e + h];
      v[k][4 * h + 0] = (sc2 * r.x) * wn.x;
      v[k][4 * h + 1] = (sc2 * r.y) * wn.y;
      v[k][4 * h + 2] = (sc2 * r.z) * wn.z;
      v[k][4 * h + 3] = (sc2 * r.w) * wn.w;
    }
    if (in_row(k))
#pragma unroll
      for (int i = 0; i < 8; i++) amax = fmaxf(amax, fabsf(v[k][i]));
  }
  // f16 rows: the token's scale 2^-s from its max |x| first (token_xs)
  const float xs = a.x16 ? token_xs(block_max<4>(amax, s_red), t == 0 && a.tscale ? a.tscale + tok : nullptr) : 1.0f;
#pragma unroll
  for (int k = 0; k < EB; k++) {
    const int b = min(t / 4 + 64 * k, nb - 1);
    if (!in_row(k)) continue;  // whole quads in or out
    if (a.x16) q8_f16_quad(v[k], xs, a.x16 + (size_t)tok * a.x16stride + b * 32 + sub * 8);
    else if (a.q8k) q8k_block_quad(v[k], sub, xq + b);  // half-waves = super-blocks (blocks t / 4 + 64 k)
    else q8_block_quad(v[k], sub, xq + b);
  }
}

// ---------------------------------------------------------------------------
// GEMM: out[t][n] = sum_b d_w[n][b] d_x[t][b] * sum_k (q_w[n][b][k] - 8) q_x[t][b][k]
// MFMA lane maps (scripts/dev/mfma_i8_check): lane (r = l & 31, h = l >> 5)
// holds A[row r][k 16h..16h+15] (the low (h 0) or high (h 1) nibbles of the
// row's 16 quant bytes, in k order) and B[k 16h..][token r] (the token's
// Q8_0 q[16h..16h+15]); D[row (reg & 3) + 8 (reg >> 2) + 4 h][token r].
// (GEMMs v1-v4 were retired in round 3: v5 with one K group per output computes
// v1's fmaf chain bit for bit; tests/golden/prefill_v1_ref.npz pins it.)
// ---------------------------------------------------------------------------

__device__ __forceinline__ size_t q4_block_index(int slab, int rows, int nb, int n, int b) {
  return slab ? ((size_t)(b >> 3) * rows + n) * 8 + (b & 7) : (size_t)n * nb + b;
}


// LDS-DMA issue as inline asm: hipcc's own glds builtin makes it wait vmcnt(0)
// before every later LDS read (it cannot tell which stage a ds_read touches),
// which would drain the ring; an asm load is outside its s_waitcnt
// bookkeeping, so the kernel's counted waits are the only ones
// (cdna_hip_programming.md, the LDS-DMA recipe: M0 is written in the same
// statement that uses it).
__device__ __forceinline__ void glds16(const void* g, unsigned char* lds_wave_base) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds_wave_base);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(dst)
               : "memory");
}
__device__ __forceinline__ void glds4(const void* g, unsigned char* lds_wave_base) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)lds_wave_base);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(dst)
               : "memory");
}

// ---------------------------------------------------------------------------
// GEMM v5 (default): eight waves per work-group in a WR x WT x WK grid -- WR
// row groups of 32 weight rows, WT token groups of 32 NT tokens, WK groups that
// split the blocks of K (block b goes to group b % WK) -- so the narrow and
// long-K projections still put two work-groups on every CU (64 x 64 tiles
// with K split 2, 32 x 64 with K split 4).
//  * Each DMA piece of the LDS ring reads whole runs of memory: a row's 4
//    consecutive Q4_0 blocks, a token's 4 consecutive XBlocks (v1-v4 and the
//    first v5 took 16 B from a different 128-B line in every lane, so L2 moved
//    8x the bytes); XOR-swizzled slots keep the fragment reads conflict-free.
//  * Per block and 32 x 32 tile: one v_mfma_i32_32x32x32_i8 for the exact
//    integer dots, and one v_mfma_f32_32x32x16_f16 for the 32 x 32 scale
//    products d_w[row] * d_x[tok] (an outer product with k = 0 only, exact in
//    f32), so the VALU does only (float)isum and the FMA per output; the VALU
//    epilogue of block b - 1 runs while block b's MFMAs execute (ping-pong
//    result registers, no copies).
//  * Block id -> tile: the token tiles of one weight row tile get equal
//    blockIdx % 8 (one XCD under round-robin placement: the row tile is
//    fetched into one L2; speed only, never correctness).
//  * Per output: acc_g = fmaf(d_w * d_x, (float)isum, acc_g) over the blocks of
//    group g in order; out = ((acc_0 + acc_1) + acc_2) + ... in group order.
//    WK = 1 is bit-identical to v1 / v3 / v4 (retired); every WK is independent of the
//    chunking (a token's outputs do not depend on the other tokens).
// Measured (4B, 512 tokens): qkv 39 -> 32, o 31 -> 25, gate_up 162 -> 133,
// down 124 -> 96 us.  The compute alone (LLMI_PG5_NODMA build) is ~2/3 of it:
// the VALU issue of ~55 instructions per block and tile (unpack, 16
// conversions, 16 FMAs) at ~4 cycles each bounds this int8 design.
// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Stage image (KB = 4 blocks), every DMA piece reading whole runs of memory (v3/v4/first-cut v5 pieces took
// 16 B from a different 128-B line in every lane -- row stride of the weights, token stride of the
// activations -- so L2 moved 8x the bytes):
//   wq [MR rows][4]    16-B quant blocks; lane i of a piece reads row i / 4's run of 4 blocks (64 B),
//                      stored at slot b ^ sw(row), sw = (row >> 2) & 3 (conflict-free A reads)
//   wd [2 pairs][MR]   u32 = f16 scales of blocks (2p, 2p + 1)
//   xq [TN tok][4][3]  the token's 4 XBlocks (4 x 48 B contiguous) as 16-B parts, block slot
//                      b ^ sw(tok): B fragment = part h, d_x = first dword of part 2
//   (W8: Q8_0 weights -- wq [MR rows][2 KB] 16-B halves of the 32-B blocks, lane i of a piece reading row
//   i / 8's 128-B run, half slot s ^ (row & 7): the A fragment is half h of the block as it lies, no unpack)
//   (KQ: Q4_K (1) / Q6_K (2) weights in the kq layout -- wq / wd hold the 16-B nibble sub-blocks and their u16
//   scale words as Q4_0's blocks and scales; dd [64] the rows' u32 super-block word (d | dmin) of the stage;
//   Q6_K qh [MR][4] the sub-blocks' 8 B of high bits; the activation blocks hold Q8_K quants)
template <int WR, int WT, int WK, int NT, int NS, bool W8 = false, int KQ = 0>
struct PG5 {
  static constexpr int KB = 4, WB = W8 ? 32 : 16;  // weight bytes per block
  static constexpr int NW = WR * WT * WK, MR = 32 * WR, TN = 32 * NT * WT;
  static constexpr int P_WQ = KB * MR * (WB / 16) / 64, P_WD = (KB / 2) * MR / 64, P_XQ = TN * KB * 3 / 64;
  static constexpr int P_DD = KQ ? (MR + 63) / 64 : 0, P_QH = KQ == 2 ? MR / 32 : 0;
  static constexpr int P = P_WQ + P_WD + P_DD + P_QH + P_XQ, PW = (P + NW - 1) / NW;
  static constexpr int O_WD = KB * MR * WB, O_DD = O_WD + (KB / 2) * MR * 4, O_QH = O_DD + P_DD * 256;
  static constexpr int O_XQ = O_QH + P_QH * 1024;
  static constexpr int STAGE = O_XQ + TN * KB * 48;
  static constexpr int EPI = NW * 32 * 33 * 4;  // one 32-token group of every wave, padded rows
  static constexpr int LDS = STAGE * NS > EPI ? STAGE * NS : EPI;
  static_assert(KB % WK == 0, "K groups");
  static_assert(KB * MR % 64 == 0 && (KB / 2) * MR % 64 == 0 && TN * KB * 3 % 64 == 0, "pieces of 64 lanes");
  static_assert(PW * (NS - 2) <= 63, "vmcnt range");
};

__device__ __forceinline__ int pg5_sw(int i) { return (i >> 2) & 3; }
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}
typedef _Float16 h2x8 __attribute__((ext_vector_type(8)));
typedef float v16f __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int pg_q6_bytes(uint32_t nib4, uint32_t hb, int k) {  // 4 six-bit values - 32 (int8)
  const uint32_t v = nib4 | (((hb >> (2 * k)) & 0x03030303u) << 4);
  return (int)((v + 0x60606060u) ^ 0x80808080u);
}

template <int WR, int WT, int WK, int NT, int NS, bool W8, int KQ = 0>
__global__ __launch_bounds__(64 * WR * WT * WK, KQ == 2 ? 1 : (WK == 1 || NT > 1) ? 2 : 4) void prefill_gemm5_kernel(PrefillGemm a) {
  using C = PG5<WR, WT, WK, NT, NS, W8, KQ>;
  constexpr int KB = C::KB;
  __shared__ __attribute__((aligned(16))) unsigned char s_ring[C::LDS];
  const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6), r = lane & 31, h = lane >> 5;
  const int wr = w % WR, wt = (w / WR) % WT, kg = w / (WR * WT);
  const uint32_t nsh = 4u * h;  // the lane half's nibble (low: k 0-15, high: k 16-31): one variable shift
  const int nb = a.nb, nst = nb / KB;
  // tile of this work-group
  const int n_rt = a.rows / C::MR, n_tt = (a.T + C::TN - 1) / C::TN;
  const int bid = blockIdx.x;
  int rt, tt;
  if (n_rt % 8 == 0) {
    const int j = bid >> 3;
    rt = (j / n_tt) * 8 + (bid & 7);
    tt = j % n_tt;
  } else {
    rt = bid / n_tt;
    tt = bid % n_tt;
  }
  const int n0 = rt * C::MR, tk0 = tt * C::TN;
  // this wave's DMA pieces (64 lanes each; wave w issues pieces w, w + NW, ... of every stage): per piece
  // kind, lane pointer at chunk 0 and LDS offset within a stage, computed once; per chunk only a scalar
  // offset is added (weights: kb blocks, or for the slab layout kb / 8 slabs + kb % 8)
  const unsigned char* pb[C::PW];
  int pk[C::PW], po[C::PW];
#ifdef LLMI_PG5_DUP  // development A/B: every wave issues PW pieces (the surplus ones duplicate others)
  const bool full_last = true;
#else
  const bool full_last = w + (C::PW - 1) * C::NW < C::P;  // wave-uniform: P not a multiple of NW
#endif
#pragma unroll
  for (int i = 0; i < C::PW; i++) {
    const int p = (w + i * C::NW) % C::P;
    if (p < C::P_WQ && W8) {  // unit u: row u / 2KB, half slot u % 2KB (row-major Q8_0 blocks)
      const int u = p * 64 + lane, row = u / (2 * KB), hs = (u % (2 * KB)) ^ (row & 7);
      pk[i] = 0;
      pb[i] = reinterpret_cast<const unsigned char*>(a.qs) + ((size_t)(n0 + row) * nb + (hs >> 1)) * 32 + (hs & 1) * 16;
      po[i] = p * 1024;
    } else if (p < C::P_WQ) {
      const int u = p * 64 + lane, row = u / KB, b = (u % KB) ^ pg5_sw(row);
      pk[i] = 0;
      pb[i] = reinterpret_cast<const unsigned char*>(a.qs + q4_block_index(a.slab, a.rows, nb, n0 + row, b));
      po[i] = p * 1024;
    } else if (p < C::P_WQ + C::P_WD) {  // unit u: block pair u / MR, row u % MR
      const int q = p - C::P_WQ, u = q * 64 + lane;
      pk[i] = 1;
      pb[i] = reinterpret_cast<const unsigned char*>(a.wd + q4_block_index(a.slab, a.rows, nb, n0 + u % C::MR, 2 * (u / C::MR)));
      po[i] = C::O_WD + q * 256;
    } else if (p < C::P_WQ + C::P_WD + C::P_DD) {  // unit u: row u % MR, the stage's super-block word
      const int q = p - C::P_WQ - C::P_WD, u = (q * 64 + lane) % C::MR;
      pk[i] = 3;
      pb[i] = reinterpret_cast<const unsigned char*>(a.kdd + (size_t)(n0 + u) * (a.slab ? 1 : nb / 8));
      po[i] = C::O_DD + q * 256;
    } else if (p < C::P_WQ + C::P_WD + C::P_DD + C::P_QH) {  // unit u: row u / 2, sub-blocks 2 (u % 2) .. + 1
      const int q = p - C::P_WQ - C::P_WD - C::P_DD, u = q * 64 + lane;
      pk[i] = 4;
      pb[i] = reinterpret_cast<const unsigned char*>(a.kqh + q4_block_index(a.slab, a.rows, nb, n0 + u / 2, 2 * (u % 2)));
      po[i] = C::O_QH + q * 1024;
    } else {  // unit u: (token, block slot, part)
      const int q = p - C::P_WQ - C::P_WD - C::P_DD - C::P_QH, u = q * 64 + lane;
      const int tok = u / (3 * KB), rem = u % (3 * KB), b = (rem / 3) ^ pg5_sw(tok);
      pk[i] = 2;
      pb[i] = reinterpret_cast<const unsigned char*>(a.x + (size_t)min(tk0 + tok, a.T - 1) * a.xstride + b) + 16 * (rem % 3);
      po[i] = C::O_XQ + q * 1024;
    }
  }
  auto issue = [&](int c) {
#ifdef LLMI_PG5_NODMA  // development: compute floor (LDS never filled)
    return;
#endif
    const int kb = c * KB;
    const long wofs = a.slab ? (long)(kb >> 3) * a.rows * 8 + (kb & 7) : kb;  // weight block-index offset
    unsigned char* st = s_ring + (c % NS) * C::STAGE;
#pragma unroll
    for (int i = 0; i < C::PW; i++) {
      if (i == C::PW - 1 && !full_last) break;  // P not a multiple of NW: this wave has PW - 1 pieces
      const int k = pk[i];
      const long off = k == 0   ? wofs * C::WB
                       : k == 1 ? wofs * 2
                       : k == 3 ? (long)(kb >> 3) * (a.slab ? a.rows : 1) * 4
                       : k == 4 ? wofs * 8
                                : (long)kb * (long)sizeof(XBlock);
      if (k == 1 || k == 3) glds4(pb[i] + off, st + po[i]);
      else glds16(pb[i] + off, st + po[i]);
    }
  };
  auto wait_ahead = [&](int ahead) {  // stages issued after the current one that may stay in flight
    static_assert(NS >= 2 && NS <= 8, "NS");
    static_for<NS - 1>([&](auto kc) {  // the first k with ahead >= NS - 2 - k waits for PW * (NS - 2 - k)
      constexpr int k = decltype(kc)::value, n = NS - 2 - k;
      if (ahead == n) {
        if (full_last) vm_wait<C::PW * n>();
        else vm_wait<(C::PW - 1) * n>();
      }
    });
  };
  for (int c = 0; c < NS - 1 && c < nst; c++) issue(c);
  float acc[NT][16];
#pragma unroll
  for (int j = 0; j < NT; j++)
#pragma unroll
    for (int i = 0; i < 16; i++) acc[j][i] = 0.0f;
  const v16i zero = {};
  const v16f zerof = {};
  // per-lane LDS addresses (within a stage) of the A row and the B tokens, block slot 0; slots XOR-swizzled
  const int arow = 32 * wr + r, a_sw = pg5_sw(arow);
  int b_base[NT], b_sw[NT];
#pragma unroll
  for (int j = 0; j < NT; j++) {
    const int tok = 32 * (wt * NT + j) + r;
    b_base[j] = C::O_XQ + tok * KB * 48;
    b_sw[j] = pg5_sw(tok);
  }
  // Software pipeline, one block deep, across stage boundaries: the MFMAs of block b are issued, then the
  // VALU epilogue of block b - 1 runs on the matrix pipe's previous results while they execute; the LDS
  // operands of block b + 1 are read before either.  (The carried results live in registers, so a stage's
  // slot may be refilled once its MFMAs have read it.)  The scale products s[row][tok] = d_w[row] * d_x[tok]
  // come from one f16 MFMA (k = 0 only: an outer product, exact in f32 -- 11-bit x 11-bit significands),
  // so the VALU keeps only (float)isum and the FMA per output.
  // KQ: the scale products s[row][tok] = (d sc)[row] d_x[tok] (d_x: the Q8_K super-block's f32 d) from an f32
  // MFMA (k = 0 only, one rounding); Q4_K's min term sum_b (dmin m)[row][b] (d_x bsum)[tok][b] accumulates on
  // the matrix pipe (Macc, subtracted at the end: t = fma(d sc, isum, -(dmin m) d_x bsum), ops.cpp:614-706);
  // Q6_K's two 16-element scales split the i8 product by lane half (A zeroed on the other half: i0, i1) and
  // take two scale products (ops.cpp:708-785)
  struct Ops {
    v4i A, A1;
    h2x8 As;
    float aS, aS1, aM;
    v4i B[NT];
    float dx[NT];
    int ns[NT];
  };
  auto load_ops = [&](const unsigned char* st, int bb) {
    Ops o;
    const int b = bb * WK + kg;
    if constexpr (KQ != 0) {
      const uint4 q = *reinterpret_cast<const uint4*>(st + (arow * KB + (b ^ a_sw)) * 16);
      const uint32_t wp = reinterpret_cast<const uint32_t*>(st + C::O_WD)[(b >> 1) * C::MR + arow];
      const uint32_t sw = (wp >> (16 * (b & 1))) & 0xFFFFu;
      const uint32_t dd = reinterpret_cast<const uint32_t*>(st + C::O_DD)[arow];
      const float d = h2f((uint16_t)(dd & 0xFFFFu));
      const uint32_t n0_ = (q.x >> nsh) & 0x0F0F0F0Fu, n1_ = (q.y >> nsh) & 0x0F0F0F0Fu;
      const uint32_t n2_ = (q.z >> nsh) & 0x0F0F0F0Fu, n3_ = (q.w >> nsh) & 0x0F0F0F0Fu;
      if constexpr (KQ == 1) {
        o.A.x = (int)n0_;
        o.A.y = (int)n1_;
        o.A.z = (int)n2_;
        o.A.w = (int)n3_;
        o.aS = h ? 0.0f : d * (float)(sw & 0xFFu);
        o.aM = h ? 0.0f : h2f((uint16_t)(dd >> 16)) * (float)(sw >> 8);
      } else {
        const uint2 hb = *reinterpret_cast<const uint2*>(st + C::O_QH + arow * 32 + b * 8);
        const uint32_t hw = h ? hb.y : hb.x;
        v4i A6;
        A6.x = pg_q6_bytes(n0_, hw, 0);
        A6.y = pg_q6_bytes(n1_, hw, 1);
        A6.z = pg_q6_bytes(n2_, hw, 2);
        A6.w = pg_q6_bytes(n3_, hw, 3);
        const v4i z4 = {};
        o.A = h ? z4 : A6;
        o.A1 = h ? A6 : z4;
        o.aS = h ? 0.0f : d * (float)(int8_t)(sw & 0xFFu);
        o.aS1 = h ? 0.0f : d * (float)(int8_t)(sw >> 8);
      }
    } else if constexpr (W8) {
      const uint4 q = *reinterpret_cast<const uint4*>(st + (arow * 2 * KB + ((2 * b + h) ^ (arow & 7))) * 16);
      o.A.x = (int)q.x;
      o.A.y = (int)q.y;
      o.A.z = (int)q.z;
      o.A.w = (int)q.w;
    } else {
      const uint4 q = *reinterpret_cast<const uint4*>(st + (arow * KB + (b ^ a_sw)) * 16);
      // 16 (n - 8) as int8: the nibble moved to the byte's top ((n ^ 8) << 4 = (n << 4) ^ 0x80), two ops a word;
      // the dots come out 16x (exact: |16 isum| < 2^20) and so does every fmaf chain (power-of-two scaling
      // commutes with rounding), undone once per output at the end -- bit-identical to unscaled int8 (n - 8)
      const uint32_t lsh = 4u - nsh;
      o.A.x = (int)(((q.x << lsh) & 0xF0F0F0F0u) ^ 0x80808080u);
      o.A.y = (int)(((q.y << lsh) & 0xF0F0F0F0u) ^ 0x80808080u);
      o.A.z = (int)(((q.z << lsh) & 0xF0F0F0F0u) ^ 0x80808080u);
      o.A.w = (int)(((q.w << lsh) & 0xF0F0F0F0u) ^ 0x80808080u);
    }
    if constexpr (KQ == 0) {
      const int par = WK == 1 ? (bb & 1) : (kg & 1);  // the block's f16 in the scale pair
      const uint32_t wp = reinterpret_cast<const uint32_t*>(st + C::O_WD)[(b >> 1) * C::MR + arow];
      o.As = h2x8{};
      o.As[0] = __builtin_bit_cast(_Float16, (uint16_t)(h ? 0u : (wp >> (16 * par)) & 0xFFFFu));
    }
#pragma unroll
    for (int j = 0; j < NT; j++) {
      const unsigned char* xb = st + b_base[j] + (b ^ b_sw[j]) * 48;
      const uint4 xv = *reinterpret_cast<const uint4*>(xb + 16 * h);
      o.dx[j] = *reinterpret_cast<const float*>(xb + 32);
      if constexpr (KQ == 1) o.ns[j] = *reinterpret_cast<const int*>(xb + 36);
      o.B[j].x = (int)xv.x;
      o.B[j].y = (int)xv.y;
      o.B[j].z = (int)xv.z;
      o.B[j].w = (int)xv.w;
    }
    return o;
  };
  // results of two blocks in flight, ping-pong by the block count's parity (compile-time indices: no copies)
  v16i Dr[2][NT];
  v16f Sr[2][NT];
  v16i Dr2[KQ == 2 ? 2 : 1][NT];
  v16f Sr2[KQ == 2 ? 2 : 1][NT];
  v16f Macc[KQ == 1 ? NT : 1];
#pragma unroll
  for (int j = 0; j < NT; j++) {
    Dr[1][j] = zero;
    Sr[1][j] = zerof;  // fmaf(+0, +0, acc) leaves acc unchanged
    if constexpr (KQ == 2) {
      Dr2[1][j] = zero;
      Sr2[1][j] = zerof;
    }
    if constexpr (KQ == 1) Macc[j] = zerof;
  }
  auto epi = [&](auto sl) {
    constexpr int S = decltype(sl)::value;
#pragma unroll
    for (int j = 0; j < NT; j++)
#pragma unroll
      for (int reg = 0; reg < 16; reg++) {
        acc[j][reg] = fmaf(Sr[S][j][reg], (float)Dr[S][j][reg], acc[j][reg]);
        if constexpr (KQ == 2) acc[j][reg] = fmaf(Sr2[S][j][reg], (float)Dr2[S][j][reg], acc[j][reg]);
      }
  };
  constexpr int NB = KB / WK;  // blocks per stage and wave
  auto stage = [&](int c, auto first) {  // first: slot of the stage's first block
    wait_ahead(min(NS - 2, nst - 1 - c));
    __builtin_amdgcn_s_barrier();  // every wave's pieces of stage c landed; stage c - 1 is no longer read
    if (c + NS - 1 < nst) issue(c + NS - 1);
#ifdef LLMI_PG5_NOCOMP  // development: DMA + barrier floor
    if (c >= 0) return;
#endif
    const unsigned char* st = s_ring + (c % NS) * C::STAGE;
    Ops o[2];
    o[0] = load_ops(st, 0);
    static_for<NB>([&](auto bbc) {
      constexpr int bb = decltype(bbc)::value;
      constexpr int sl = (decltype(first)::value + bb) & 1;
      if constexpr (bb + 1 < NB) o[(bb + 1) & 1] = load_ops(st, bb + 1);
#pragma unroll
      for (int j = 0; j < NT; j++) {
        const Ops& op = o[bb & 1];
        Dr[sl][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(op.A, op.B[j], zero, 0, 0, 0);
        if constexpr (KQ != 0) {
          const float bS = h ? 0.0f : op.dx[j];
          Sr[sl][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(op.aS, bS, zerof, 0, 0, 0);
          if constexpr (KQ == 1)
            Macc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(op.aM, h ? 0.0f : op.dx[j] * (float)op.ns[j], Macc[j], 0, 0, 0);
          if constexpr (KQ == 2) {
            Dr2[sl][j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(op.A1, op.B[j], zero, 0, 0, 0);
            Sr2[sl][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(op.aS1, bS, zerof, 0, 0, 0);
          }
        } else {
          h2x8 Bs = {};
          Bs[0] = h ? (_Float16)0.0f : (_Float16)op.dx[j];  // d_x is an f16 value (q8 block scale): exact
          Sr[sl][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(op.As, Bs, zerof, 0, 0, 0);
        }
      }
      epi(std::integral_constant<int, sl ^ 1>{});  // the previous block's results
    });
  };
  if constexpr (NB % 2 == 0) {
    for (int c = 0; c < nst; c++) stage(c, std::integral_constant<int, 0>{});
    epi(std::integral_constant<int, 1>{});
  } else {
    int c = 0;
    for (; c + 1 < nst; c += 2) {
      stage(c, std::integral_constant<int, 0>{});
      stage(c + 1, std::integral_constant<int, 1>{});
    }
    if (c < nst) {
      stage(c, std::integral_constant<int, 0>{});
      epi(std::integral_constant<int, 0>{});
    } else {
      epi(std::integral_constant<int, 1>{});
    }
  }
  if constexpr (KQ == 1) {  // the Q4_K min terms
#pragma unroll
    for (int j = 0; j < NT; j++)
#pragma unroll
      for (int reg = 0; reg < 16; reg++) acc[j][reg] -= Macc[j][reg];
  }
  // epilogue, one 32-token group at a time: every wave's tile (rows x 32 tokens) to LDS, then the K groups
  // summed in group order and stored row-contiguous per token
  float* ep = reinterpret_cast<float*>(s_ring);
#pragma unroll
  for (int j = 0; j < NT; j++) {
    __builtin_amdgcn_s_barrier();  // the ring / the previous group's tiles are no longer read
    float* mine = ep + (size_t)w * 32 * 33;
#pragma unroll
    for (int reg = 0; reg < 16; reg++) mine[r * 33 + (reg & 3) + 8 * (reg >> 2) + 4 * h] = acc[j][reg];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int i = t; i < WT * C::MR * 32; i += 64 * C::NW) {
      const int row = i % C::MR, tk = (i / C::MR) % 32, gt = i / (C::MR * 32);
      const int tok = tk0 + 32 * (gt * NT + j) + tk;
      float v = 0.0f;
#pragma unroll
      for (int g = 0; g < WK; g++) {
        const int ww = (g * WT + gt) * WR + row / 32;  // wave (wr = row / 32, wt = gt, kg = g)
        const float p = ep[(size_t)ww * 32 * 33 + tk * 33 + row % 32];
        v = g ? v + p : p;
      }
      if (tok < a.T) a.out[(size_t)tok * a.ostride + n0 + row] = KQ == 0 && !W8 ? v * 0.0625f : v;  // Q4_0: 16x
    }
  }
}

// ---------------------------------------------------------------------------
// GEMM v6 (f16 prefill, BASELINE configs[2]'s "F16 MFMA prefill GEMM"):
// f16 activations [T][K] (written so by the norm / attention / GELU
// producers instead of Q8_0 blocks) times the Q4_0 weights dequantized to f16
// in registers, w = f16(d_w * (q - 8)) (one rounding), on
// v_mfma_f32_32x32x16_f16 with the fp32 accumulator carried over all of K:
// no per-block epilogue -- the v5 VALU bound (conversions and FMAs per 32-k
// block) is gone; a wave dequantizes its 32 rows' block once for NT token
// groups.  The v5 frame: LDS-DMA ring of KB-block stages filled by whole runs
// of memory (a row's KB blocks, a token's KB x 64 B), XOR-swizzled 16-B slots,
// waves in a WR x WT x WK grid (WK groups split K: block b -> group b % WK,
// partial sums added in group order), token tiles of a row tile on one XCD.
// Deterministic and independent of the chunking; within the fast budget of
// the Q8_0 path (an f16 product per weight instead of Q8_0 activations).
// ---------------------------------------------------------------------------
// Weight types (WQ): 0 Q4_0 (d_w per block), 1 Q4_K and 2 Q6_K in the kq layout (kernels.h: per 32-element
// sub-block 16 B of nibbles in the Q4_0 order and a u16 scale word, per 256-element super-block a u32 of
// d (| dmin), Q6_K also 8 B of high bits) -- w = f16(d sc q - dmin m) (Q4_K) or f16(d sc (q6 - 32)) (Q6_K),
// the K-quant prefill (the reference runs it as a token loop of mat_vec_mul_q4_k / _q6_k, ops.cpp:614-785).
template <int WR, int WT, int WK, int NT, int KB, int NS, int WQ>
struct PG6 {
  static constexpr int NW = WR * WT * WK, MR = 32 * WR, TN = 32 * NT * WT;
  static constexpr int XU = KB * 4;  // 16-B activation units per token per stage
  static constexpr int P_WQ = KB * MR / 64, P_WD = (KB / 2) * MR / 64, P_DD = WQ ? MR / 64 : 0,
                       P_QH = WQ == 2 ? (KB / 2) * MR / 64 : 0, P_X = TN * XU / 64;
  static constexpr int P = P_WQ + P_WD + P_DD + P_QH + P_X, PW = (P + NW - 1) / NW;
  static constexpr int O_WD = KB * MR * 16, O_DD = O_WD + (KB / 2) * MR * 4, O_QH = O_DD + (WQ ? MR * 4 : 0),
                       O_X = O_QH + (WQ == 2 ? MR * KB * 8 : 0);
  static constexpr int STAGE = O_X + TN * XU * 16;
  static constexpr int EPI = NW * 32 * 33 * 4;
  static constexpr int LDS = STAGE * NS > EPI ? STAGE * NS : EPI;
  static_assert(KB % WK == 0 && (KB == 2 || KB == 4), "KB");
  static_assert(KB * MR % 64 == 0 && (KB / 2) * MR % 64 == 0 && TN * XU % 64 == 0 && MR % 64 == 0, "pieces of 64 lanes");
  static_assert(PW * (NS - 2) <= 63, "vmcnt range");
};

template <int KB>
__device__ __forceinline__ int pg6_wsw(int row) { return KB == 4 ? (row >> 2) & 3 : (row >> 3) & 1; }

template <int WR, int WT, int WK, int NT, int KB, int NS, int WQ>
__global__ __launch_bounds__(512, 2) void prefill_gemm6_kernel(PrefillGemm16 a) {
  using C = PG6<WR, WT, WK, NT, KB, NS, WQ>;
  typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
  __shared__ __attribute__((aligned(16))) unsigned char s_ring[C::LDS];
  const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6), r = lane & 31, h = lane >> 5;
  const int wr = w % WR, wt = (w / WR) % WT, kg = w / (WR * WT);
  const int nb = a.nb, nst = nb / KB, nsb = nb / 8;
  const int n_rt = a.rows / C::MR, n_tt = (a.T + C::TN - 1) / C::TN;
  const int bid = blockIdx.x;
  int rt, tt;
  if (n_rt % 8 == 0) {
    const int j = bid >> 3;
    rt = (j / n_tt) * 8 + (bid & 7);
    tt = j % n_tt;
  } else {
    rt = bid / n_tt;
    tt = bid % n_tt;
  }
  const int n0 = rt * C::MR, tk0 = tt * C::TN;
  const unsigned char* pb[C::PW];
  int pk[C::PW], po[C::PW];
#ifdef LLMI_PG5_DUP  // development A/B: every wave issues PW pieces (the surplus ones duplicate others)
  const bool full_last = true;
#else
  const bool full_last = w + (C::PW - 1) * C::NW < C::P;  // wave-uniform: P not a multiple of NW
#endif
#pragma unroll
  for (int i = 0; i < C::PW; i++) {
    int p = (w + i * C::NW) % C::P;
    if (p < C::P_WQ) {  // unit u: row u / KB, block slot u % KB
      const int u = p * 64 + lane, row = u / KB, b = (u % KB) ^ pg6_wsw<KB>(row);
      pk[i] = 0;
      pb[i] = reinterpret_cast<const unsigned char*>(a.qs + q4_block_index(a.slab, a.rows, nb, n0 + row, b));
      po[i] = p * 1024;
      continue;
    }
    p -= C::P_WQ;
    if (p < C::P_WD) {  // unit u: block pair u / MR, row u % MR (f16 scales / kq scale words)
      const int u = p * 64 + lane;
      pk[i] = 1;
      pb[i] = reinterpret_cast<const unsigned char*>(a.wd + q4_block_index(a.slab, a.rows, nb, n0 + u % C::MR, 2 * (u / C::MR)));
      po[i] = C::O_WD + p * 256;
      continue;
    }
    p -= C::P_WD;
    if (p < C::P_DD) {  // unit u: row u, the super-block word of the stage
      const int u = p * 64 + lane;
      pk[i] = 3;
      pb[i] = reinterpret_cast<const unsigned char*>(a.kdd + (size_t)(n0 + u) * (a.slab ? 1 : nsb));
      po[i] = C::O_DD + p * 256;
      continue;
    }
    p -= C::P_DD;
    if (p < C::P_QH) {  // unit u: row u / (KB / 2), sub-block pair u % (KB / 2): 16 B of high bits
      const int u = p * 64 + lane, row = u / (KB / 2), pr = u % (KB / 2);
      pk[i] = 4;
      pb[i] = reinterpret_cast<const unsigned char*>(a.kqh + q4_block_index(a.slab, a.rows, nb, n0 + row, 2 * pr));
      po[i] = C::O_QH + p * 1024;
      continue;
    }
    p -= C::P_QH;
    {  // unit u: (token, slot), the token's row of KB x 32 f16 as XU units, slot = unit ^ (tok & (XU - 1))
      const int u = p * 64 + lane;
      const int tok = u / C::XU, un = (u % C::XU) ^ (tok & (C::XU - 1));
      pk[i] = 2;
      pb[i] = reinterpret_cast<const unsigned char*>(a.x + (size_t)min(tk0 + tok, a.T - 1) * a.xstride + un * 8);
      po[i] = C::O_X + p * 1024;
    }
  }
  auto issue = [&](int c) {
    const int kb = c * KB;
    const long wofs = a.slab ? (long)(kb >> 3) * a.rows * 8 + (kb & 7) : kb;
    unsigned char* st = s_ring + (c % NS) * C::STAGE;
#pragma unroll
    for (int i = 0; i < C::PW; i++) {
      if (i == C::PW - 1 && !full_last) break;  // P not a multiple of NW: this wave has PW - 1 pieces
      const int k = pk[i];
      const long off = k == 0   ? wofs * 16
                       : k == 1 ? wofs * 2
                       : k == 2 ? (long)kb * 64
                       : k == 3 ? (long)(kb >> 3) * (a.slab ? a.rows : 1) * 4
                                : wofs * 8;
      if (k == 1 || k == 3) glds4(pb[i] + off, st + po[i]);
      else glds16(pb[i] + off, st + po[i]);
    }
  };
  auto wait_ahead = [&](int ahead) {
    static_for<NS - 1>([&](auto kc) {
      constexpr int k = decltype(kc)::value, n = NS - 2 - k;
      if (ahead == n) vm_wait<C::PW * n>();
    });
  };
  for (int c = 0; c < NS - 1 && c < nst; c++) issue(c);
  v16f acc[NT];
#pragma unroll
  for (int j = 0; j < NT; j++) acc[j] = v16f{};
  const int arow = 32 * wr + r, a_sw = pg6_wsw<KB>(arow);
  int b_base[NT], b_sw[NT];
#pragma unroll
  for (int j = 0; j < NT; j++) {
    const int tok = 32 * (wt * NT + j) + r;
    b_base[j] = C::O_X + tok * C::XU * 16;
    b_sw[j] = tok & (C::XU - 1);
  }
  const f16x2v m1024 = {(_Float16)-1024.0f, (_Float16)-1024.0f};
  const f16x2v m1032 = {(_Float16)-1032.0f, (_Float16)-1032.0f};
  const f16x2v m1056 = {(_Float16)-1056.0f, (_Float16)-1056.0f};
  for (int c = 0; c < nst; c++) {
    wait_ahead(min(NS - 2, nst - 1 - c));
    __builtin_amdgcn_s_barrier();
    if (c + NS - 1 < nst) issue(c + NS - 1);
    const unsigned char* st = s_ring + (c % NS) * C::STAGE;
    const uint32_t* wd = reinterpret_cast<const uint32_t*>(st + C::O_WD);
#pragma unroll
    for (int bb = 0; bb < KB / WK; bb++) {
      const int b = bb * WK + kg;
      // A: bytes 8h .. 8h + 7 of the row's block: low nibbles = k 8h.. (MFMA 0), high = k 16 + 8h.. (MFMA 1)
      const uint2 qb = *reinterpret_cast<const uint2*>(st + (arow * KB + (b ^ a_sw)) * 16 + 8 * h);
      const uint32_t wp = wd[(b >> 1) * C::MR + arow];
      const uint32_t sw16 = (WK == 1 ? (bb & 1) : (kg & 1)) ? (wp >> 16) : (wp & 0xFFFFu);
      f16x2v s0, s1, o0 = {}, o1 = {};  // MFMA 0 / 1: w = q * s + o, q the stored integer
      if constexpr (WQ == 0) {
        s0 = s1 = __builtin_bit_cast(f16x2v, sw16 | (sw16 << 16));
      } else {
        const uint32_t ddw = reinterpret_cast<const uint32_t*>(st + C::O_DD)[arow];
        const float d = h2f((uint16_t)(ddw & 0xFFFF));
        if constexpr (WQ == 1) {  // d sc q - dmin m
          const float sc = d * (float)(sw16 & 0xFF), mn = h2f((uint16_t)(ddw >> 16)) * (float)(sw16 >> 8);
          const _Float16 sh = (_Float16)sc, mh = (_Float16)(-mn);
          s0 = s1 = f16x2v{sh, sh};
          o0 = o1 = f16x2v{mh, mh};
        } else {  // d sc_g (q6 - 32), sc_g: int8 per 16 elements
          const _Float16 a0 = (_Float16)(d * (float)(int)(int8_t)(sw16 & 0xFF));
          const _Float16 a1 = (_Float16)(d * (float)(int)(int8_t)(sw16 >> 8));
          s0 = f16x2v{a0, a0};
          s1 = f16x2v{a1, a1};
        }
      }
      uint2 qh2 = {};
      if constexpr (WQ == 2) qh2 = *reinterpret_cast<const uint2*>(st + C::O_QH + (arow * KB + b) * 8);
      f16x8 A0, A1;
      const uint32_t dw[2] = {qb.x, qb.y};
#pragma unroll
      for (int e = 0; e < 2; e++) {
        const uint32_t v = dw[e], vh = v >> 4;
#pragma unroll
        for (int pr = 0; pr < 2; pr++) {  // bytes 2 pr, 2 pr + 1 of the dword = elements 8h + 4e + 2pr, +1
          const uint32_t sel = pr ? 0x0C030C02u : 0x0C010C00u;
          uint32_t lo = __builtin_amdgcn_perm(0u, v, sel) & 0x000F000Fu;
          uint32_t hi = __builtin_amdgcn_perm(0u, vh, sel) & 0x000F000Fu;
          if constexpr (WQ == 2) {  // high bits: element 4k + i at bits 2k.. of byte i (k = 2h + e, i = 2pr, 2pr + 1)
            const int k = 2 * h + e;
            const uint32_t hl = __builtin_amdgcn_perm(0u, (qh2.x >> (2 * k)) & 0x03030303u, sel);
            const uint32_t hh = __builtin_amdgcn_perm(0u, (qh2.y >> (2 * k)) & 0x03030303u, sel);
            lo |= hl << 4;
            hi |= hh << 4;
          }
          const f16x2v bl = __builtin_bit_cast(f16x2v, lo | 0x64006400u);  // 1024 + q
          const f16x2v bh = __builtin_bit_cast(f16x2v, hi | 0x64006400u);
          f16x2v fl, fh;
          if constexpr (WQ == 0) {
            fl = (bl + m1032) * s0;
            fh = (bh + m1032) * s1;
          } else if constexpr (WQ == 1) {
            fl = __builtin_elementwise_fma(bl + m1024, s0, o0);
            fh = __builtin_elementwise_fma(bh + m1024, s1, o1);
          } else {
            fl = (bl + m1056) * s0;
            fh = (bh + m1056) * s1;
          }
          A0[4 * e + 2 * pr] = fl[0];
          A0[4 * e + 2 * pr + 1] = fl[1];
          A1[4 * e + 2 * pr] = fh[0];
          A1[4 * e + 2 * pr + 1] = fh[1];
        }
      }
#pragma unroll
      for (int j = 0; j < NT; j++) {
        const unsigned char* xr = st + b_base[j];
        const f16x8 B0 = *reinterpret_cast<const f16x8*>(xr + (((4 * b + h) ^ b_sw[j]) * 16));
        const f16x8 B1 = *reinterpret_cast<const f16x8*>(xr + (((4 * b + 2 + h) ^ b_sw[j]) * 16));
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A0, B0, acc[j], 0, 0, 0);
        acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A1, B1, acc[j], 0, 0, 0);
      }
    }
  }
  float* ep = reinterpret_cast<float*>(s_ring);
#pragma unroll
  for (int j = 0; j < NT; j++) {
    __builtin_amdgcn_s_barrier();
    float* mine = ep + (size_t)w * 32 * 33;
#pragma unroll
    for (int reg = 0; reg < 16; reg++) mine[r * 33 + (reg & 3) + 8 * (reg >> 2) + 4 * h] = acc[j][reg];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    for (int i = t; i < WT * C::MR * 32; i += 64 * C::NW) {
      const int row = i % C::MR, tk = (i / C::MR) % 32, gt = i / (C::MR * 32);
      const int tok = tk0 + 32 * (gt * NT + j) + tk;
      float v = 0.0f;
#pragma unroll
      for (int g = 0; g < WK; g++) {
        const int ww = (g * WT + gt) * WR + row / 32;
        const float p = ep[(size_t)ww * 32 * 33 + tk * 33 + row % 32];
        v = g ? v + p : p;
      }
      if (tok < a.T) a.out[(size_t)tok * a.ostride + n0 + row] = a.tscale ? v * a.tscale[tok] : v;
    }
  }
}

// ---------------------------------------------------------------------------
// GEMM v7 (the default prefill GEMM for Q4_0 weights; BASELINE configs[2]'s "F16 MFMA prefill GEMM"):
//   out[t][n] = 2^s_t sum_k f16(d_w (q - 8))[n][k] x16[t][k]
// on v_mfma_f32_32x32x16_f16 with the fp32 accumulator carried over all of K in k order, where x16 holds the
// producers' Q8_0 blocks dequantized and scaled by 2^-s_t per token (token_xs): every product is the reference's
// Q8_0 x Q4_0 term (ops.cpp:364-399) to two f16 roundings, with no per-block epilogue (v5's bound: a conversion
// and an FMA per output and block on the VALU) and no per-wave dequantization (v6's: every wave unpacked its rows
// for its own token tile).
//  * Work-group tile MR x TN = (32 NR WR) x (32 NT WT): WR x WT waves, each NR x NT MFMA tiles of 32 x 32.
//  * Stage = 64 k (two Q4_0 blocks).  Every thread loads its weight row's blocks (ATPR threads per row) and its
//    token's 64 f16 (BTPT threads per token) into registers two stages ahead, then writes them to an f16 LDS
//    tile pair (double-buffered): the weights dequantized ONCE per work-group (f16(1024 + n) - 1032 exactly,
//    then x d: one rounding), the activations as loaded.  LDS rows are 128 B (64 f16), 16-B units XOR-swizzled
//    (pg7_slot) so the fragment reads and the writes are conflict-free.
//  * Software-pipelined, one barrier per stage: the MFMAs of stage c (buffer c & 1) run with stage c + 1's
//    dequantization and LDS writes (buffer (c + 1) & 1) placed between their k steps; the barrier before
//    stage c + 1 sees every wave's writes of it and every read of stage c.
//  * Deterministic and independent of the chunking (a token's outputs read only its own x16 row).
// ---------------------------------------------------------------------------
template <int WR, int WT, int NR, int NT>
struct PG7 {
  static constexpr int NW = WR * WT, NTH = 64 * NW, MR = 32 * NR * WR, TN = 32 * NT * WT;
  static constexpr int ATPR = NTH / MR;  // threads per weight row: 1 (the stage's two blocks) or 2 (one each)
  static constexpr int BTPT = NTH / TN;  // threads per token row (TN * BTPT == NTH)
  static constexpr int BU = 8 / BTPT;    // 16-B units of the stage's token rows per thread: unit g = u NTH + t is
                                         // unit g % 8 of token g / 8 (8 lanes read a token's 128-B run)
  static constexpr int BUF = (MR + TN) * 128, LDS = 2 * BUF;
  static_assert((ATPR == 1 || ATPR == 2) && MR * ATPR == NTH, "weight rows per thread");
  static_assert((BTPT == 1 || BTPT == 2 || BTPT == 4 || BTPT == 8) && TN * BTPT == NTH, "token rows per thread");
};

// 16-B unit u of LDS row `row` (128-B rows): XOR swizzle by the Gray code of the row's low bits, conflict-free for
// the fragment reads (ds_read_b128's 16-lane groups: rows {0-3, 12-15, 20-27} and {4-11, 16-19, 28-31} of a tile,
// one unit each) and the writes (ds_write_b128's 8-lane groups: 8 rows, or 4 rows x 2 blocks, or a token's 8 units)
__device__ __forceinline__ int pg7_slot(int row, int u) { return row * 8 + (u ^ ((row ^ (row >> 1)) & 7)); }

// 8 quants' low (or high) nibbles -> 8 f16 weights f16(d (n - 8)), as a 16-B unit
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ u32x4 pg7_deq(uint32_t w0, uint32_t w1, f16x2v s) {
  const f16x2v m1032 = {(_Float16)-1032.0f, (_Float16)-1032.0f};
  const uint32_t n0 = w0 & 0x0F0F0F0Fu, n1 = w1 & 0x0F0F0F0Fu;
  u32x4 o;  // bytes {b, 0x64} = f16 1024 + b: v_perm with the constant 0x64 bytes as its second source
  o.x = __builtin_bit_cast(uint32_t, (__builtin_bit_cast(f16x2v, __builtin_amdgcn_perm(0x64646464u, n0, 0x04010400u)) + m1032) * s);
  o.y = __builtin_bit_cast(uint32_t, (__builtin_bit_cast(f16x2v, __builtin_amdgcn_perm(0x64646464u, n0, 0x04030402u)) + m1032) * s);
  o.z = __builtin_bit_cast(uint32_t, (__builtin_bit_cast(f16x2v, __builtin_amdgcn_perm(0x64646464u, n1, 0x04010400u)) + m1032) * s);
  o.w = __builtin_bit_cast(uint32_t, (__builtin_bit_cast(f16x2v, __builtin_amdgcn_perm(0x64646464u, n1, 0x04030402u)) + m1032) * s);
  return o;
}

template <int WR, int WT, int NR, int NT, int OCC = 1, int NS = 2>
__global__ __launch_bounds__(64 * WR * WT, OCC) void prefill_gemm7_kernel(PrefillGemm16 a) {
  using C = PG7<WR, WT, NR, NT>;
  typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
  __shared__ __attribute__((aligned(16))) unsigned char s_t[C::LDS];
  const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6), r = lane & 31, h = lane >> 5;
  const int wr = w % WR, wt = w / WR;
  const int nb = a.nb, nst = nb / 2;
  const int n_rt = a.rows / C::MR, n_tt = (a.T + C::TN - 1) / C::TN;
  const int bid = blockIdx.x;
  int rt, tt;
  if (n_rt % 8 == 0) {  // the token tiles of a row tile on one XCD (round-robin placement: speed only)
    const int j = bid >> 3;
    rt = (j / n_tt) * 8 + (bid & 7);
    tt = j % n_tt;
  } else {
    rt = bid / n_tt;
    tt = bid % n_tt;
  }
  const int n0 = rt * C::MR, tk0 = tt * C::TN;
  // this thread's loads: weight row arow (block ablk of a stage when two threads share the row), token btok
  const int arow = t / C::ATPR, ablk = t % C::ATPR;
  int xoff[C::BU];  // element offset of this thread's units u (stage 0)
  static_for<C::BU>([&](auto uc) {
    constexpr int u = decltype(uc)::value;
    const int g = u * C::NTH + t;
    xoff[u] = min(tk0 + (g >> 3), a.T - 1) * a.xstride + (g & 7) * 8;
  });
  // the register stages (two, ping-pong): the row's quants (blocks 2c, 2c + 1, or block 2c + ablk), their f16
  // scales, the token's f16 values
  constexpr int NQ = 3 - C::ATPR;
  u32x4 qr[NS][NQ], xr[NS][C::BU];  // NS register sets (native vectors: HIP's uint4 copies are memcpys SROA
  uint32_t dr[NS];                   // leaves in scratch)
  auto load = [&](u32x4 (&q)[NQ], uint32_t& d, u32x4 (&x)[C::BU], int c) {
    const size_t qi = q4_block_index(a.slab, a.rows, nb, n0 + arow, 2 * c + ablk);  // 2c, 2c + 1 adjacent (even)
    const u32x4* qs = reinterpret_cast<const u32x4*>(a.qs);
    q[0] = qs[qi];
    if constexpr (C::ATPR == 1) {
      q[1] = qs[qi + 1];
      d = *reinterpret_cast<const uint32_t*>(a.wd + qi);
    } else {
      d = a.wd[qi];
    }
    static_for<C::BU>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      x[u] = *reinterpret_cast<const u32x4*>(a.x + xoff[u] + 64 * c);
    });
  };
  // (compile-time indices throughout: a private array indexed in a loop before unrolling is promoted to LDS /
  // scratch by the backend)
  // the next stage's LDS writes in four parts, each placed after one k step's MFMAs (part p: weight units of
  // block-unit group p -- dequantized -- and a quarter of the token's units)
  auto put_part = [&](const u32x4 (&q)[NQ], uint32_t d, const u32x4 (&x)[C::BU], int buf, auto pc) {
    constexpr int p = decltype(pc)::value;
    unsigned char* As = s_t + buf * C::BUF;
    unsigned char* Bs = As + C::MR * 128;
    // weights: NQ blocks x 4 units; part p takes units 4 NQ p / 4 .. (block j = unit / 4)
    static_for<NQ>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      static_for<4>([&](auto uc) {
        constexpr int u = decltype(uc)::value;
        if constexpr ((4 * j + u) * 4 / (4 * NQ) == p) {
          const int blk = C::ATPR == 1 ? j : ablk;
          const uint32_t dh = j ? d >> 16 : d & 0xFFFFu;
          const f16x2v sc = __builtin_bit_cast(f16x2v, dh | (dh << 16));
          // block element e < 16: low nibble of byte e (units 0, 1); e >= 16: high nibble of byte e - 16 (2, 3)
          const uint32_t w0 = u & 1 ? q[j].z : q[j].x, w1 = u & 1 ? q[j].w : q[j].y;
          *reinterpret_cast<u32x4*>(As + pg7_slot(arow, 4 * blk + u) * 16) =
              u >= 2 ? pg7_deq(w0 >> 4, w1 >> 4, sc) : pg7_deq(w0, w1, sc);
        }
      });
    });
    static_for<C::BU>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      if constexpr (u * 4 / C::BU == p) {
        const int g = u * C::NTH + t;
        *reinterpret_cast<u32x4*>(Bs + pg7_slot(g >> 3, g & 7) * 16) = x[u];
      }
    });
  };
  auto put = [&](const u32x4 (&q)[NQ], uint32_t d, const u32x4 (&x)[C::BU], int buf) {
    static_for<4>([&](auto pc) { put_part(q, d, x, buf, pc); });
  };
  v16f acc[NR][NT];
  static_for<NR>([&](auto ic) { static_for<NT>([&](auto jc) { acc[decltype(ic)::value][decltype(jc)::value] = v16f{}; }); });
  // stage in buffer buf through the MFMAs, the next stage's writes (into the other buffer) between the k steps
  auto compute = [&](int buf, const u32x4 (&q)[NQ], uint32_t d, const u32x4 (&x)[C::BU]) {
    const unsigned char* As = s_t + buf * C::BUF;
    const unsigned char* Bs = As + C::MR * 128;
    static_for<4>([&](auto kc) {  // 16 k per MFMA: lane half h holds k 16 ks + 8 h .. + 7 (unit 2 ks + h)
      constexpr int ks = decltype(kc)::value;
      f16x8 A[NR], B[NT];
      static_for<NR>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        A[i] = *reinterpret_cast<const f16x8*>(As + pg7_slot(32 * (NR * wr + i) + r, 2 * ks + h) * 16);
      });
      static_for<NT>([&](auto jc) {
        constexpr int j = decltype(jc)::value;
        B[j] = *reinterpret_cast<const f16x8*>(Bs + pg7_slot(32 * (NT * wt + j) + r, 2 * ks + h) * 16);
      });
      static_for<NR>([&](auto ic) {
        static_for<NT>([&](auto jc) {
          constexpr int i = decltype(ic)::value, j = decltype(jc)::value;
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A[i], B[j], acc[i][j], 0, 0, 0);
        });
      });
      put_part(q, d, x, buf ^ 1, kc);
    });
  };
  // Pipeline: register set s holds stage c (even c: set 0) two stages after its loads were issued; iteration c
  // waits at the barrier for every wave's writes of stage c (and so for every read of the other buffer by
  // stage c - 1), computes stage c while writing stage c + 1 from the other set, then reloads that set with
  // stage c + 3
  // Register set s % NS holds stage s from NS stages before its LDS writes (the load latency hidden behind NS
  // stages of MFMAs).  nst % NS == 0: the unrolled loop body is branch-free; past the last stage the loads repeat
  // it and the writes land in the buffer nothing reads any more.
  static_for<NS>([&](auto sc) {
    constexpr int k = decltype(sc)::value;
    load(qr[k], dr[k], xr[k], k);
  });
  put(qr[0], dr[0], xr[0], 0);
  load(qr[0], dr[0], xr[0], min(NS, nst - 1));
  int c0 = 0;
  do {  // (a do-while with a straight body: the accumulators stay in place, no per-iteration copies)
    static_for<NS>([&](auto jc) {
      constexpr int j = decltype(jc)::value, nx = (j + 1) % NS;
      __syncthreads();
      compute(j & 1, qr[nx], dr[nx], xr[nx]);  // stage c0 + j; writes stage c0 + j + 1 from set nx
      load(qr[nx], dr[nx], xr[nx], min(c0 + j + 1 + NS, nst - 1));
    });
    c0 += NS;
  } while (c0 < nst);
  // D[row 8 (i >> 2) + 4 h + (i & 3)][token r] of every tile, times the token's 2^s: float4 row runs
  static_for<NT>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    const int tok = tk0 + 32 * (NT * wt + j) + r;
    if (tok < a.T) {
      const float sc = a.tscale ? a.tscale[tok] : 1.0f;
      float* orow = a.out + (size_t)tok * a.ostride + n0 + 4 * h;
      static_for<NR>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        static_for<4>([&](auto gc) {
          constexpr int g = decltype(gc)::value;
          *reinterpret_cast<float4*>(orow + 32 * (NR * wr + i) + 8 * g) = make_float4(
              acc[i][j][4 * g] * sc, acc[i][j][4 * g + 1] * sc, acc[i][j][4 * g + 2] * sc, acc[i][j][4 * g + 3] * sc);
        });
      });
    }
  });
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
      if (a.softcap > 0.0f) sc = a.softcap * tanhf(sc / a.softcap);  // model.cpp:511-513
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
// causal attention on the matrix cores (default): one work-group per (kv head,
// block of 32 query tokens), one wave per query head of the GQA group; 32-key
// tiles of K and V stream into a double-buffered LDS image by LDS-DMA (rows of
// the cache as they lie, 16-B units XOR-swizzled by key: conflict-free reads).
//   S^T = K Q^T   (v_mfma_f32_32x32x16_f16 over head_dim; Q^T fragments held
//                  in registers): a lane holds 16 keys' scores of its query
//   online softmax per query in fp32 (the other 16 keys in lane ^ 32)
//   O^T += V^T P^T  P^T from the score registers as is (f16), the MFMA's k
//                  order permuted to the registers' key order; V^T by
//                  ds_read_b64_tr_b16 (transposing LDS read) from the
//                  row-major V image
// Output heads as Q8_0 blocks (quantize_row_q8_0 arithmetic, the 32 values of
// a block in lanes q and q + 32).  A query's result depends only on the cache
// and its own q: exact under re-chunking.
// ---------------------------------------------------------------------------
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef __fp16 fp16x4 __attribute__((__vector_size__(4 * sizeof(__fp16))));

// The attention's outputs for one query (lanes r and r + 32 of a wave hold 16 of every 32 head dims): O^T / l as
// f16 rows, Q8_K (head_dim 256: the head is one super-block, NI = 8) or Q8_0 blocks i0 .. i0 + NI - 1
template <int HD, int NI>
__device__ __forceinline__ void attn_emit(const PrefillAttn& a, const v16f (&o)[NI], float l_run, int i0, int tok,
                                          int hq, int h) {
  if (a.x16) {  // f16 rows of the dequantized Q8_0 blocks (as below), unscaled: |O| <= max |V| of the f16 cache
    uint16_t* xo16 = a.x16 + (size_t)tok * a.x16stride + (size_t)hq * HD + 32 * i0;
#pragma unroll
    for (int i = 0; i < NI; i++) {
      float v[16];
      float amax = 0.0f;
#pragma unroll
      for (int reg = 0; reg < 16; reg++) {
        v[reg] = o[i][reg] / l_run;
        amax = fmaxf(amax, fabsf(v[reg]));
      }
      amax = fmaxf(amax, __shfl_xor(amax, 32));
      const float dd = amax / 127.0f;
      const float id = dd != 0.0f ? 1.0f / dd : 0.0f;
      const float ds = h2f(f2h_ggml(dd));
#pragma unroll
      for (int gq = 0; gq < 4; gq++) {  // dims 32 i + 8 gq + 4 h .. + 3
        float q[4];
#pragma unroll
        for (int e = 0; e < 4; e++) q[e] = (float)nearest_int_fma(v[4 * gq + e], id) * ds;
        uint2 o2;
        o2.x = __builtin_bit_cast(uint32_t, f16x2v{(_Float16)q[0], (_Float16)q[1]});
        o2.y = __builtin_bit_cast(uint32_t, f16x2v{(_Float16)q[2], (_Float16)q[3]});
        *reinterpret_cast<uint2*>(xo16 + 32 * i + 8 * gq + 4 * h) = o2;
      }
    }
    return;
  }
  XBlock* xo = a.xq + (size_t)tok * a.xstride + (size_t)hq * HD / 32 + i0;
  if constexpr (HD == 256 && NI == HD / 32) {
    if (a.q8k) {  // Q8_K (ops.cpp:142-178): the head's 256 dims are one super-block, lanes r and r + 32
      float ax = 0.0f;
#pragma unroll
      for (int i = 0; i < HD / 32; i++)
#pragma unroll
        for (int reg = 0; reg < 16; reg++) ax = fmaxf(ax, fabsf(o[i][reg] / l_run));
      ax = fmaxf(ax, __shfl_xor(ax, 32));
      int key = 0x7FFFFFFF;  // the first dim attaining max |x|, with its sign
#pragma unroll
      for (int i = 0; i < HD / 32; i++)
#pragma unroll
        for (int reg = 0; reg < 16; reg++) {
          const float v = o[i][reg] / l_run;
          const int dim = 32 * i + 8 * (reg >> 2) + 4 * h + (reg & 3);
          if (fabsf(v) == ax) key = min(key, (dim << 1) | (v < 0.0f ? 1 : 0));
        }
      key = min(key, __shfl_xor(key, 32));
      const float iscale = ax != 0.0f ? -127.f / ((key & 1) ? -ax : ax) : 0.0f;
#pragma unroll
      for (int i = 0; i < HD / 32; i++) {
        int sum = 0;
        uint32_t wq[4];
#pragma unroll
        for (int gq = 0; gq < 4; gq++) {
          wq[gq] = 0;
#pragma unroll
          for (int e = 0; e < 4; e++) {
            int qv = ax != 0.0f ? nearest_int_fma(iscale, o[i][4 * gq + e] / l_run) : 0;
            qv = qv < -128 ? -128 : (qv > 127 ? 127 : qv);
            sum += qv;
            wq[gq] |= (uint32_t)(qv & 0xFF) << (8 * e);
          }
        }
        sum += __shfl_xor(sum, 32);
        uint32_t* qb = reinterpret_cast<uint32_t*>(xo + i);
#pragma unroll
        for (int gq = 0; gq < 4; gq++) qb[2 * gq + h] = wq[gq];
        if (h == 0) {
          xo[i].d = ax != 0.0f ? 1.0f / iscale : 0.0f;
          xo[i].nsum8 = sum;
        }
      }
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < NI; i++) {
    float v[16];
    float amax = 0.0f;
#pragma unroll
    for (int reg = 0; reg < 16; reg++) {
      v[reg] = o[i][reg] / l_run;
      amax = fmaxf(amax, fabsf(v[reg]));
    }
    amax = fmaxf(amax, __shfl_xor(amax, 32));
    const float dd = amax / 127.0f;
    const float id = dd != 0.0f ? 1.0f / dd : 0.0f;
    int sum = 0;
    uint32_t wq[4];
#pragma unroll
    for (int gq = 0; gq < 4; gq++) {
      wq[gq] = 0;
#pragma unroll
      for (int e = 0; e < 4; e++) {
        const int qv = nearest_int_fma(v[4 * gq + e], id);
        sum += qv;
        wq[gq] |= (uint32_t)(qv & 0xFF) << (8 * e);
      }
    }
    sum += __shfl_xor(sum, 32);
    uint32_t* qb = reinterpret_cast<uint32_t*>(xo + i);
#pragma unroll
    for (int gq = 0; gq < 4; gq++) qb[2 * gq + h] = wq[gq];  // bytes 8 gq + 4 h .. + 3
    if (h == 0) {
      xo[i].d = h2f(f2h_ggml(dd));
      xo[i].nsum8 = -8 * sum;
    }
  }
}

template <int HD, int G, int S>
__global__ __launch_bounds__(64 * G * S) void prefill_attn_mfma_kernel(PrefillAttn a, int T) {
  constexpr int U = HD / 8;                // 16-B units per cache row
  constexpr int SWM = U < 16 ? U - 1 : 15;  // swizzle mask (units)
  constexpr int ROWB = HD * 2;              // bytes per cache row
  constexpr int TILE = 32 * ROWB;           // bytes per K (or V) tile
  constexpr int NW = G * S;                 // waves: head g = w % G, key split s = w / G
  constexpr int P = S * 2 * TILE / 1024;    // DMA pieces per round (S tiles, K then V)
  static_assert(P % NW == 0 && P / NW <= 63, "pieces");
  constexpr int RPP = 1024 / ROWB;          // cache rows per piece
  constexpr int RING = 2 * S * 2 * TILE;    // two rounds of S tiles
  constexpr int MERGE = (S - 1) * G * 64 * (HD / 2 + 2) * 4;
  __shared__ __attribute__((aligned(16))) unsigned char s_kv[RING > MERGE ? RING : MERGE];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), r = lane & 31, h = lane >> 5;
  const int g = w % G, sp = w / G;
  // heaviest (last) query blocks first: dispatch order is a speed matter only
  const int hk = blockIdx.x, qb = gridDim.y - 1 - blockIdx.y, tok0 = qb * 32, hq = hk * G + g;
  const int qtok = min(tok0 + r, T - 1);
  const int qpos = a.pos0 + tok0 + r;                       // this lane's query position
  const int last_pos = a.pos0 + min(tok0 + 32, T) - 1;     // the block's last query
  const int first_pos = a.pos0 + tok0;
  const int n_tiles = last_pos / 32 + 1, n_rounds = (n_tiles + S - 1) / S;
  // key splits across work-groups: round q (tiles S q .. S q + S - 1) is work-group q % KS's (blockIdx.z) -- a
  // function of the key position only, so chunk-exact and the same on tensor-parallel ranks; a query block with
  // fewer rounds than KS uses its first n_rounds work-groups
  const int KS = a.ks, ks = blockIdx.z, nks = min(KS, n_rounds);
  if (ks >= nks) return;  // whole work-group, before any barrier
  const int my_rounds = (n_rounds - ks + KS - 1) / KS;
  const size_t cache0 = (size_t)hk * a.max_ctx;
  // local round lr (global round ks + lr KS): its tiles into ring half lr & 1; tile S q + j at slot j of the half
  auto tile_ptr = [&](int lr, int j) { return s_kv + ((lr & 1) * S + j) * 2 * TILE; };
  auto issue = [&](int lr) {
    const int round = ks + lr * KS;
#pragma unroll
    for (int i = 0; i < P / NW; i++) {
      const int p = w + i * NW, j = p / (2 * TILE / 1024), q = p % (2 * TILE / 1024);
      const int kind = q / (TILE / 1024), pp = q % (TILE / 1024);
      const int row = pp * RPP + lane / U, slot = lane % U, u = slot ^ (row & SWM);
      const int key = min(32 * (S * round + j) + row, a.max_ctx - 1);
      const uint16_t* src = (kind ? a.v_cache : a.k_cache) + (cache0 + key) * HD + u * 8;
      glds16(src, tile_ptr(lr, j) + kind * TILE + pp * 1024);
    }
  };
  issue(0);
  typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
  // Q^T fragments: lane (query r, h) holds q[d = 16 c + 8 h .. + 7]
  f16x8 qf[HD / 16];
  const uint4* qrow = reinterpret_cast<const uint4*>(a.q + ((size_t)qtok * a.n_head + hq) * HD);
#pragma unroll
  for (int c = 0; c < HD / 16; c++) qf[c] = __builtin_bit_cast(f16x8, qrow[2 * c + h]);
  v16f o[HD / 32];
#pragma unroll
  for (int i = 0; i < HD / 32; i++) o[i] = v16f{};
  float m_run = -INFINITY, l_run = 0.0f;
  const int lg = lane >> 4, li = lane & 15, tq = li >> 2, tp = li & 3;  // tr_b16 group / position
  for (int lr = 0; lr < my_rounds; lr++) {
    vm_wait<0>();
    __builtin_amdgcn_s_barrier();  // round landed in every wave; the previous round's half is free
    if (lr + 1 < my_rounds) issue(lr + 1);
    const int t = S * (ks + lr * KS) + sp;  // this split's tile
    if (t >= n_tiles) continue;             // wave-uniform; no cross-lane read is skipped by part of a wave
    const unsigned char* kt = tile_ptr(lr, sp);
    const unsigned char* vt = kt + TILE;
    // S^T: rows = keys (A from the K image), cols = queries
    v16f sc = {};
#pragma unroll
    for (int c = 0; c < HD / 16; c++) {
      const f16x8 kf = *reinterpret_cast<const f16x8*>(kt + r * ROWB + (((2 * c + h) ^ (r & SWM)) * 16));
      sc = __builtin_amdgcn_mfma_f32_32x32x16_f16(kf, qf[c], sc, 0, 0, 0);
    }
    if (a.softcap > 0.0f) {  // model.cpp:511-513 (before the mask: a masked score is replaced, never read)
#pragma unroll
      for (int reg = 0; reg < 16; reg++) sc[reg] = a.softcap * tanhf(sc[reg] / a.softcap);
    }
    // causal mask (select, never arithmetic on a masked score) + online softmax
    const bool diag = 32 * t + 31 > first_pos;
    float mt = -INFINITY;
#pragma unroll
    for (int reg = 0; reg < 16; reg++) {
      const int key = 32 * t + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      if (diag && key > qpos) sc[reg] = -INFINITY;
      mt = fmaxf(mt, sc[reg]);
    }
    mt = fmaxf(mt, __shfl_xor(mt, 32));
    const float m_new = fmaxf(m_run, mt);
    // a split's first tile may be fully masked for some queries (m_new = -inf): keep its terms 0
    const float alpha = m_new == -INFINITY ? 1.0f : expf(m_run - m_new);
    float ps = 0.0f;
    f16x8 pb[2];
#pragma unroll
    for (int reg = 0; reg < 16; reg++) {
      const float pv = m_new == -INFINITY ? 0.0f : expf(sc[reg] - m_new);
      ps += pv;
      pb[reg >> 3][reg & 7] = (_Float16)pv;
    }
    ps += __shfl_xor(ps, 32);
    l_run = l_run * alpha + ps;
    m_run = m_new;
#pragma unroll
    for (int i = 0; i < HD / 32; i++) o[i] *= alpha;
    // O^T += V^T P^T: MFMA kk (keys 16 kk ..) takes element j = key (j & 3) + 8 (j >> 2) + 4 h + 16 kk;
    // V^T fragment by two transposing reads (rows = keys 16 kk + 4 h + {0, 8} + 0..3)
#pragma unroll
    for (int kk = 0; kk < 2; kk++) {
#pragma unroll
      for (int i = 0; i < HD / 32; i++) {
        const int gh = lg >> 1;  // the h of this 16-lane group
        const int col = 32 * i + 16 * (lg & 1) + 4 * tp;  // first of the 4 columns this lane addresses
        // (the v4f16 form, joined by a shuffle: element-wise extraction from the v4i16 form was
        // miscompiled into a splat of element 0 -- scripts/dev/pv_check.hip)
        f16x4 vv[2];
#pragma unroll
        for (int e = 0; e < 2; e++) {
          const int key = 16 * kk + 4 * gh + 8 * e + tq;
          const int off = key * ROWB + (((col >> 3) ^ (key & SWM)) * 16) + (col & 7) * 2;
          vv[e] = __builtin_bit_cast(f16x4, __builtin_amdgcn_ds_read_tr16_b64_v4f16(
                                                 (__attribute__((address_space(3))) fp16x4*)(vt + off)));
        }
        const f16x8 vf = __builtin_shufflevector(vv[0], vv[1], 0, 1, 2, 3, 4, 5, 6, 7);
        o[i] = __builtin_amdgcn_mfma_f32_32x32x16_f16(vf, pb[kk], o[i], 0, 0, 0);
      }
    }
  }
  // merge the key splits of each head through LDS (split 0 combines, in split order)
  if constexpr (S > 1) {
    vm_wait<0>();
    __builtin_amdgcn_s_barrier();  // every wave is done with the ring
    float* mg = reinterpret_cast<float*>(s_kv);
    if (sp > 0) {
      float* my = mg + (size_t)((sp - 1) * G + g) * 64 * (HD / 2 + 2);
      my[lane] = m_run;
      my[64 + lane] = l_run;
#pragma unroll
      for (int i = 0; i < HD / 32; i++)
#pragma unroll
        for (int reg = 0; reg < 16; reg++) my[128 + (i * 16 + reg) * 64 + lane] = o[i][reg];
    }
    __syncthreads();
    if (sp > 0) return;
#pragma unroll
    for (int s2 = 1; s2 < S; s2++) {
      const float* ot = mg + (size_t)((s2 - 1) * G + g) * 64 * (HD / 2 + 2);
      const float m2 = ot[lane], l2 = ot[64 + lane];
      const float mm = fmaxf(m_run, m2);
      const float a1 = m_run == -INFINITY ? 0.0f : expf(m_run - mm), a2 = m2 == -INFINITY ? 0.0f : expf(m2 - mm);
      l_run = l_run * a1 + l2 * a2;
      m_run = mm;
#pragma unroll
      for (int i = 0; i < HD / 32; i++)
#pragma unroll
        for (int reg = 0; reg < 16; reg++) o[i][reg] = o[i][reg] * a1 + ot[128 + (i * 16 + reg) * 64 + lane] * a2;
    }
  }
  if (nks > 1) {  // this work-group's partial (m, l, O^T); prefill_attn_merge_kernel combines them
    float* pp = a.part + (((size_t)hq * gridDim.y + qb) * KS + ks) * (64 * (HD / 2 + 2));
    pp[lane] = m_run;
    pp[64 + lane] = l_run;
#pragma unroll
    for (int i = 0; i < HD / 32; i++)
#pragma unroll
      for (int q4 = 0; q4 < 4; q4++)
        reinterpret_cast<float4*>(pp + 128)[(i * 4 + q4) * 64 + lane] =
            make_float4(o[i][4 * q4], o[i][4 * q4 + 1], o[i][4 * q4 + 2], o[i][4 * q4 + 3]);
    return;
  }
  // O = O^T / l -> Q8_0 blocks (32 head dims = one tile column; lanes q and q + 32 hold 16 each), or f16
  if (tok0 + r >= T) return;  // after the last LDS read: the partner lane of a live query is also out
  attn_emit<HD, HD / 32>(a, o, l_run, 0, tok0 + r, hq, h);
}

// Key-split partials of the query blocks that have more than one (prefill_attn_mfma_kernel, a.ks > 1): one wave
// per (head, query block, 32 head dims) -- or per (head, query block) for Q8_K output (one super-block per
// head) -- rescales every partial against their maximum and sums them in split order, then writes the outputs
// as the attention kernel does.  Spread over the chip: the partials of one query block are read by HD / 32
// work-groups at once rather than by the one work-group that counted in last (round 3, first cut: 26.8 us).
template <int HD, int NI>
__global__ __launch_bounds__(64) void prefill_attn_merge_kernel(PrefillAttn a, int T, int S) {
  const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
  const int hq = blockIdx.x, nqb = gridDim.y, qb = nqb - 1 - blockIdx.y, tok0 = qb * 32, i0 = blockIdx.z * NI;
  const int last_pos = a.pos0 + min(tok0 + 32, T) - 1;
  const int n_rounds = (last_pos / 32 + 1 + S - 1) / S, KS = a.ks, nks = min(KS, n_rounds);
  if (nks <= 1) return;  // written by the attention kernel
  constexpr int SLAB = 64 * (HD / 2 + 2);
  const float* pp = a.part + ((size_t)hq * nqb + qb) * KS * SLAB;
  float wk[PREFILL_ATTN_KS_MAX];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < PREFILL_ATTN_KS_MAX; k++) {
    wk[k] = k < nks ? pp[k * SLAB + lane] : -INFINITY;
    m = fmaxf(m, wk[k]);
  }
  float l = 0.0f;
#pragma unroll
  for (int k = 0; k < PREFILL_ATTN_KS_MAX; k++)
    if (k < nks) {  // m finite: partial 0 holds key 0
      wk[k] = wk[k] == -INFINITY ? 0.0f : expf(wk[k] - m);
      l = k ? l + wk[k] * pp[k * SLAB + 64 + lane] : wk[k] * pp[k * SLAB + 64 + lane];
    }
  v16f o[NI];
  if constexpr (NI > 1) {  // the whole head (Q8_K): partial by partial, every quad's loads in flight
    for (int k = 0; k < nks; k++) {
      const float4* src = reinterpret_cast<const float4*>(pp + k * SLAB + 128);
#pragma unroll
      for (int i = 0; i < NI; i++)
#pragma unroll
        for (int q4 = 0; q4 < 4; q4++) {
          const float4 v = src[((i0 + i) * 4 + q4) * 64 + lane];
          const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int e = 0; e < 4; e++) o[i][4 * q4 + e] = k ? o[i][4 * q4 + e] + wk[k] * vv[e] : wk[k] * vv[e];
        }
    }
  } else
#pragma unroll
  for (int i = 0; i < NI; i++)
#pragma unroll
    for (int q4 = 0; q4 < 4; q4++) {
      float4 v[PREFILL_ATTN_KS_MAX];
#pragma unroll
      for (int k = 0; k < PREFILL_ATTN_KS_MAX; k++)
        if (k < nks) v[k] = reinterpret_cast<const float4*>(pp + k * SLAB + 128)[((i0 + i) * 4 + q4) * 64 + lane];
#pragma unroll
      for (int k = 0; k < PREFILL_ATTN_KS_MAX; k++)
        if (k < nks) {
          const float vv[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
          for (int e = 0; e < 4; e++) o[i][4 * q4 + e] = k ? o[i][4 * q4 + e] + wk[k] * vv[e] : wk[k] * vv[e];
        }
    }
  if (tok0 + r >= T) return;
  attn_emit<HD, NI>(a, o, l, i0, tok0 + r, hq, h);
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

// GELU(gate) * up -> Q8_0, vectorized: a thread per 8 consecutive hidden units (one DPP quad per Q8_0 block),
// float4 loads from the interleaved gate/up rows (H % 8 == 0: the 8 units sit in one H-group)
__global__ __launch_bounds__(256) void prefill_gelu8_kernel(const float* __restrict__ gu, int F, int H,
                                                            XBlock* __restrict__ xq, int xstride, int q8k) {
  const int tok = blockIdx.y, i = blockIdx.x * 256 + threadIdx.x;
  if (i * 8 >= F) return;  // whole quads (F % 32 == 0); Q8_K: whole half-waves (F % 256 == 0)
  const int u = 8 * i;
  const float* g = gu + (size_t)tok * 2 * F + 2 * H * (u / H) + u % H;
  const float4 g0 = reinterpret_cast<const float4*>(g)[0], g1 = reinterpret_cast<const float4*>(g)[1];
  const float4 u0 = reinterpret_cast<const float4*>(g + H)[0], u1 = reinterpret_cast<const float4*>(g + H)[1];
  const float v[8] = {gelu_mul1(g0.x, u0.x), gelu_mul1(g0.y, u0.y), gelu_mul1(g0.z, u0.z), gelu_mul1(g0.w, u0.w),
                      gelu_mul1(g1.x, u1.x), gelu_mul1(g1.y, u1.y), gelu_mul1(g1.z, u1.z), gelu_mul1(g1.w, u1.w)};
  if (q8k) q8k_block_quad(v, i & 3, xq + (size_t)tok * xstride + i / 4);
  else q8_block_quad(v, i & 3, xq + (size_t)tok * xstride + i / 4);
}

// GELU(gate) * up -> f16 rows (the f16 prefill): one 1024-thread work-group per token, NJ groups of 8 hidden units
// per thread held in registers until the token's max |x| is known (token_xs), then written as the dequantized
// Q8_0 blocks
template <int NJ>
__global__ __launch_bounds__(1024) void prefill_gelu16_kernel(const float* __restrict__ gu, int F, int H,
                                                              uint16_t* __restrict__ x16, int x16stride,
                                                              float* __restrict__ tscale) {
  __shared__ float s_red[16];
  const int tok = blockIdx.x, t = threadIdx.x, n8 = F / 8;
  float v[NJ][8];
  float amax = 0.0f;
#pragma unroll
  for (int j = 0; j < NJ; j++) {
    const int i = t + 1024 * j;
    if (i >= n8) break;
    const int u = 8 * i;
    const float* g = gu + (size_t)tok * 2 * F + 2 * H * (u / H) + u % H;
    const float4 g0 = reinterpret_cast<const float4*>(g)[0], g1 = reinterpret_cast<const float4*>(g)[1];
    const float4 u0 = reinterpret_cast<const float4*>(g + H)[0], u1 = reinterpret_cast<const float4*>(g + H)[1];
    v[j][0] = gelu_mul1(g0.x, u0.x);
    v[j][1] = gelu_mul1(g0.y, u0.y);
    v[j][2] = gelu_mul1(g0.z, u0.z);
    v[j][3] = gelu_mul1(g0.w, u0.w);
    v[j][4] = gelu_mul1(g1.x, u1.x);
    v[j][5] = gelu_mul1(g1.y, u1.y);
    v[j][6] = gelu_mul1(g1.z, u1.z);
    v[j][7] = gelu_mul1(g1.w, u1.w);
#pragma unroll
    for (int e = 0; e < 8; e++) amax = fmaxf(amax, fabsf(v[j][e]));
  }
  const float xs = token_xs(block_max<16>(amax, s_red), t == 0 ? tscale + tok : nullptr);
#pragma unroll
  for (int j = 0; j < NJ; j++) {
    const int i = t + 1024 * j;
    if (i >= n8) break;  // whole quads (F % 32 == 0)
    q8_f16_quad(v[j], xs, x16 + (size_t)tok * x16stride + 8 * i);
  }
}

}  // namespace

void launch_prefill_norm(const PrefillNorm& a, int T, hipStream_t s) {
  if (a.n > 256 * PN_EPT || a.n % 32) throw std::runtime_error("prefill_norm: n_embd");
  if (a.q8k && (a.n % 256 || a.x16)) throw std::runtime_error("prefill_norm: Q8_K blocks need n % 256 == 0");
  const int eb = (a.n / 32 + 63) / 64;
  if (!a.table && eb <= 3) {
    switch (eb) {
      case 1: hipLaunchKernelGGL(prefill_norm_res_kernel<1>, dim3(T), dim3(256), 0, s, a); break;
      case 2: hipLaunchKernelGGL(prefill_norm_res_kernel<2>, dim3(T), dim3(256), 0, s, a); break;
      default: hipLaunchKernelGGL(prefill_norm_res_kernel<3>, dim3(T), dim3(256), 0, s, a); break;
    }
    LLMI_HIP(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL(prefill_norm_kernel, dim3(T), dim3(256), (size_t)a.n * 4, s, a);
  LLMI_HIP(hipGetLastError());
}

bool prefill_gemm_supported(const DevWeight& w) {  // GEMM v5: 32-row tiles, 4-block K steps
  if (w.type == T_Q8_0) return w.rows % 32 == 0 && w.cols % 128 == 0 && !w.slab;
  if (w.type == T_Q4_K || w.type == T_Q6_K) return w.kq && w.rows % 32 == 0 && w.cols % 256 == 0;  // Q8_K x
  return w.type == T_Q4_0 && w.rows % 32 == 0 && w.cols % 128 == 0 && (!w.slab || (w.cols / 32) % 8 == 0);
}

template <int WR, int WT, int WK, int NT, int NS>
static bool try_gemm5(const PrefillGemm& a, hipStream_t s) {
  using C = PG5<WR, WT, WK, NT, NS>;
  if (a.rows % C::MR || a.nb % C::KB) return false;
  const int n = (a.rows / C::MR) * ((a.T + C::TN - 1) / C::TN);
  if (a.kq == 1)
    hipLaunchKernelGGL((prefill_gemm5_kernel<WR, WT, WK, NT, NS, false, 1>), dim3(n), dim3(64 * C::NW), 0, s, a);
  else if (a.kq == 2)
    hipLaunchKernelGGL((prefill_gemm5_kernel<WR, WT, WK, NT, NS, false, 2>), dim3(n), dim3(64 * C::NW), 0, s, a);
  else if (a.w8)
    hipLaunchKernelGGL((prefill_gemm5_kernel<WR, WT, WK, NT, NS, true>), dim3(n), dim3(64 * C::NW), 0, s, a);
  else
    hipLaunchKernelGGL((prefill_gemm5_kernel<WR, WT, WK, NT, NS, false>), dim3(n), dim3(64 * C::NW), 0, s, a);
  return true;
}

// v5 geometry (LLMI_PG5=<name> forces one for A/B; 4B 512-token prefill, us per GEMM qkv / o /
// gate_up / down: mid 32.2 / 26.1 / 133.0 / 100.1, small 37.1 / 25.0 / 168.2 / 95.5, wide (128 x 64, no K
// split) 32.2 / 25.3 / 145.8 / 103.7; a 6-stage ring, 64 tokens per wave or a 128 x 128 tile were slower):
// 64 x 64 tiles with K split 2 (mid), or 32 x 64 with K split 4 (small) for the long-K GEMMs.  The K split
// is chosen from K alone, so a tensor-parallel shard (fewer rows) sums every output in the same order as the
// whole weight (tests/test_tp.py: bit-identical).  Round 3: sixteen-wave work-groups (x16: 128 x 64 tiles, and
// 64 x 64 with K split 4 for down; y16: 64 x 128 / 128 x 32) cut the L2 -> LDS bytes by a third yet ran
// 130 / 118 and 134 / 113 us (gate_up / down) against 128 / 99: not the bound.  Two token tiles per wave (NT 2,
// 3 stages: 128 x 64 / 64 x 64 K split 4, or 64 x 128 / 32 x 128): 130 / 115 and 141 / 130 against 124 / 97 --
// the unpack and weight-scale work they share is not worth the registers (occupancy 2).
static bool launch_gemm5(const PrefillGemm& a, hipStream_t s) {
  const char* f = getenv("LLMI_PG5");
  const std::string c = f ? f : a.nb >= 160 ? "small" : "mid";
  if (c == "big" && try_gemm5<4, 2, 1, 2, 3>(a, s)) return true;
  if (c == "wide" && try_gemm5<4, 2, 1, 1, 3>(a, s)) return true;
  if (c == "x16") return a.nb >= 160 ? try_gemm5<2, 2, 4, 1, 4>(a, s) : try_gemm5<4, 2, 2, 1, 4>(a, s);
  if (c == "y16") return a.nb >= 160 ? try_gemm5<4, 1, 4, 1, 4>(a, s) : try_gemm5<2, 4, 2, 1, 4>(a, s);
  if (c == "small") return try_gemm5<1, 2, 4, 1, 4>(a, s);
  return try_gemm5<2, 2, 2, 1, 4>(a, s) || try_gemm5<1, 4, 2, 1, 4>(a, s);  // K split 2, 64 or 32 rows
}

template <int WR, int WT, int WK, int NT, int KB, int NS, int WQ>
static bool try_gemm6(const PrefillGemm16& a, hipStream_t s) {
  using C = PG6<WR, WT, WK, NT, KB, NS, WQ>;
  if (a.rows % C::MR || a.nb % KB) return false;
  const int n = (a.rows / C::MR) * ((a.T + C::TN - 1) / C::TN);
  hipLaunchKernelGGL((prefill_gemm6_kernel<WR, WT, WK, NT, KB, NS, WQ>), dim3(n), dim3(64 * C::NW), 0, s, a);
  return true;
}

template <int WQ>
static bool gemm6_geometry(const PrefillGemm16& a, hipStream_t s) {
  if (const char* f = getenv("LLMI_PG6_GEO")) {  // development A/B (scripts/dev/pg7_bench)
    const std::string c = f;
    if (c == "a") return try_gemm6<2, 1, 4, 2, 4, 3, WQ>(a, s);  // 64 x 64, K split 4
    if (c == "b") return try_gemm6<2, 2, 2, 2, 2, 3, WQ>(a, s);  // 64 x 128, K split 2
    if (c == "c") return try_gemm6<4, 1, 2, 2, 4, 3, WQ>(a, s);  // 128 x 64, K split 2
    if (c == "d") return try_gemm6<2, 1, 4, 1, 4, 3, WQ>(a, s);  // 64 x 32, K split 4
    if (c == "e") return try_gemm6<2, 1, 4, 2, 4, 4, WQ>(a, s);  // 64 x 64, K split 4, 4 stages
    if (c == "f") return try_gemm6<2, 2, 2, 2, 4, 3, WQ>(a, s);  // 64 x 128, K split 2, KB 4
    if (c == "g") return try_gemm6<4, 2, 1, 2, 2, 3, WQ>(a, s);  // 128 x 128, no K split
  }
  // K >= 5120: 64 x 64 tiles, K split 4; shorter K: 128 x 64 tiles with K split 2 where the rows allow (4B qkv /
  // o 27.7 / 21.1 us against 31.0 / 24.6 for 64 x 128, scripts/dev/pg7_bench) -- block b to K group b % WK in
  // every form, so the sums do not depend on the tile
  if (a.nb >= 160 && try_gemm6<2, 1, 4, 2, 4, 3, WQ>(a, s)) return true;
  return try_gemm6<4, 1, 2, 2, 4, 3, WQ>(a, s) || try_gemm6<2, 2, 2, 2, 2, 3, WQ>(a, s);
}

bool prefill_gemm16_supported(const DevWeight& w) {
  if (w.type == T_Q4_0) return prefill_gemm_supported(w) && w.rows % 64 == 0 && (w.cols / 32) % 4 == 0;
  return (w.type == T_Q4_K || w.type == T_Q6_K) && w.kq && w.rows % 64 == 0 && w.cols % 256 == 0;
}

bool prefill_gemm7_supported(const DevWeight& w) {
  return w.type == T_Q4_0 && w.rows % 128 == 0 && w.cols % 128 == 0 && (!w.slab || (w.cols / 32) % 8 == 0);
}

template <int WR, int WT, int NR, int NT, int OCC = 1>
static bool try_gemm7(const PrefillGemm16& a, hipStream_t s) {
  using C = PG7<WR, WT, NR, NT>;
  if (a.rows % C::MR || a.nb % 4) return false;  // an even number of 64-k stages
  const int n = (a.rows / C::MR) * ((a.T + C::TN - 1) / C::TN);
  // register stages in flight: 2 (LLMI_PG7_NS=4 for four: slower on the 4B shapes, scripts/dev/pg7_bench)
  static const int ns = getenv("LLMI_PG7_NS") ? atoi(getenv("LLMI_PG7_NS")) : 2;
  if (ns == 4 && a.nb % 8 == 0)  // four register stages in flight (a multiple of 4 stages)
    hipLaunchKernelGGL((prefill_gemm7_kernel<WR, WT, NR, NT, OCC, 4>), dim3(n), dim3(C::NTH), 0, s, a);
  else
    hipLaunchKernelGGL((prefill_gemm7_kernel<WR, WT, NR, NT, OCC, 2>), dim3(n), dim3(C::NTH), 0, s, a);
  return true;
}

// v7 geometry (LLMI_PG7=<name> forces one for A/B): 128 x 128 tiles for the wide projections, 64 x 128 for the
// narrow ones (more work-groups), narrower token tiles for short chunks
static bool launch_gemm7(const PrefillGemm16& a, bool wide, hipStream_t s) {
  const char* f = getenv("LLMI_PG7");
  const std::string c = f ? f : "";
  if (c == "256x256") return try_gemm7<2, 2, 4, 4>(a, s);
  if (c == "256x128") return try_gemm7<2, 2, 4, 2>(a, s);
  if (c == "128x256") return try_gemm7<2, 2, 2, 4>(a, s);
  if (c == "128x128") return try_gemm7<2, 2, 2, 2>(a, s);
  if (c == "256x64") return try_gemm7<4, 1, 2, 2>(a, s);
  if (c == "128x64") return try_gemm7<2, 1, 2, 2>(a, s);
  if (c == "128x128o2") return try_gemm7<2, 2, 2, 2, 2>(a, s);
  if (c == "64x128") return try_gemm7<1, 2, 2, 2>(a, s);
  if (a.T <= 32) return try_gemm7<4, 1, 2, 1>(a, s) || try_gemm7<2, 1, 2, 1>(a, s);
  if (a.T <= 64) return try_gemm7<4, 1, 2, 2>(a, s) || try_gemm7<2, 1, 2, 2>(a, s);
  return wide ? try_gemm7<2, 2, 2, 2>(a, s) : try_gemm7<1, 2, 2, 2>(a, s);
}

// v6 geometry: the K split depends on K alone (tensor-parallel shards
// sum in the same order as the whole weight)
void launch_prefill_gemm16(const DevWeight& w, const uint16_t* x, int xstride, int T, float* out, int ostride,
                           const float* tscale, hipStream_t s) {
  // Q4_0: v7 with 128 x 128 tiles where they fill the chip twice over (gate_up: 640 work-groups at T = 512), v6
  // elsewhere (its K split over wave groups keeps 256-320 work-groups of 8 waves busy where v7 has 80-128).
  // In-model, 4B 512-token prefill (scripts/dev/pfprof_geo.sh): 9.76 ms this way, 9.97 with v7 64 x 128 tiles
  // for qkv / o (which scripts/dev/pg7_bench -- 20 launches of one GEMM, weights warm in the Infinity Cache --
  // has ahead), 10.2 with v6 everywhere, 10.9-11.2 with the int8 v5
  const bool wide = (w.rows / 128) * ((T + 127) / 128) >= 512;
  const bool v6 = getenv("LLMI_PG6") || (!getenv("LLMI_PG7") && !wide && prefill_gemm16_supported(w));
  if (prefill_gemm7_supported(w) && !v6) {
    PrefillGemm16 a;
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
    a.tscale = tscale;
    if (!launch_gemm7(a, wide, s)) throw std::runtime_error("prefill_gemm16: shape outside the v7 geometries");
    LLMI_HIP(hipGetLastError());
    return;
  }
  if (!prefill_gemm16_supported(w)) throw std::runtime_error("prefill_gemm16: unsupported weight");
  PrefillGemm16 a;
  a.tscale = tscale;
  a.qs = reinterpret_cast<const uint4*>(w.qs);
  a.wd = w.d;
  a.kdd = w.kdd;
  a.kqh = w.kqh;
  a.rows = w.rows;
  a.nb = w.cols / 32;
  a.slab = w.slab;
  a.x = x;
  a.xstride = xstride;
  a.T = T;
  a.out = out;
  a.ostride = ostride;
  const bool ok = w.type == T_Q4_0 ? gemm6_geometry<0>(a, s) : w.type == T_Q4_K ? gemm6_geometry<1>(a, s)
                                                                                : gemm6_geometry<2>(a, s);
  if (!ok) throw std::runtime_error("prefill_gemm16: shape");
  LLMI_HIP(hipGetLastError());
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
  a.w8 = w.type == T_Q8_0;
  a.kq = w.type == T_Q4_K ? 1 : w.type == T_Q6_K ? 2 : 0;
  a.kdd = w.kdd;
  a.kqh = w.kqh;
  a.x = x;
  a.xstride = xstride;
  a.T = T;
  a.out = out;
  a.ostride = ostride;
  if (!launch_gemm5(a, s)) throw std::runtime_error("prefill_gemm: shape outside the v5 geometries");
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
  const int G = a.n_head / a.n_head_kv;
  if ((a.x16 || a.q8k) && (getenv("LLMI_PREFILL_ATTN_V1") || (G != 1 && G != 2 && G != 4)))
    throw std::runtime_error("prefill_attn: f16 / Q8_K output needs the MFMA kernel (GQA group 1, 2 or 4)");
  if (a.q8k && (HD != 256 || a.x16)) throw std::runtime_error("prefill_attn: Q8_K output needs head_dim 256");
  if (!getenv("LLMI_PREFILL_ATTN_V1") && HD >= 64) {
    if (a.ks > 1 && (!a.part || a.ks > PREFILL_ATTN_KS_MAX))
      throw std::runtime_error("prefill_attn: key splits need the partial scratch");
    const dim3 grid(a.n_head_kv, (T + 31) / 32, std::max(1, a.ks));
    // key splits per work-group (LDS: two rounds of S tiles, and the merge); S depends on head_dim only, so a
    // tensor-parallel rank (fewer heads per kv head: smaller G) merges the same splits as the whole model
    // (bit-identical).  head_dim 256 at G 1 / 4 spills some of the 128 O^T + 64 Q^T registers (correct, slower).
    constexpr int S4 = HD >= 256 ? 2 : 4;
    int S = 0;
    switch (G) {
      case 1: hipLaunchKernelGGL((prefill_attn_mfma_kernel<HD, 1, S4>), grid, dim3(64 * S4), 0, s, a, T); S = S4; break;
      case 2: hipLaunchKernelGGL((prefill_attn_mfma_kernel<HD, 2, S4>), grid, dim3(128 * S4), 0, s, a, T); S = S4; break;
      case 4:
        hipLaunchKernelGGL((prefill_attn_mfma_kernel<HD, 4, HD == 128 ? 2 : S4>), grid, dim3(256 * (HD == 128 ? 2 : S4)),
                           0, s, a, T);
        S = HD == 128 ? 2 : S4;
        break;
      default: break;
    }
    if (S) {
      const int nqb = (T + 31) / 32;
      if (a.ks > 1 && (a.pos0 + T - 1) / 32 + 1 > S) {  // some query block has more than one partial
        if constexpr (HD == 256) {
          if (a.q8k) {
            hipLaunchKernelGGL((prefill_attn_merge_kernel<HD, HD / 32>), dim3(a.n_head, nqb, 1), dim3(64), 0, s, a, T, S);
            return;
          }
        }
        hipLaunchKernelGGL((prefill_attn_merge_kernel<HD, 1>), dim3(a.n_head, nqb, HD / 32), dim3(64), 0, s, a, T, S);
      }
      return;
    }
  }
  const dim3 grid(a.n_head_kv, T);
  switch (G) {
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

void launch_prefill_gelu(const float* gu, int F, int H, XBlock* xq, int xstride, int T, hipStream_t s, uint16_t* x16,
                         int x16stride, int q8k, float* tscale) {
  if (q8k && (H % 8 || F % 256)) throw std::runtime_error("prefill_gelu: Q8_K output needs H % 8 == 0, F % 256 == 0");
  if (F % 32 || H <= 0 || F % H) throw std::runtime_error("prefill_gelu: shape");
  if (x16) {
    if (H % 8 || !tscale) throw std::runtime_error("prefill_gelu: f16 output needs H % 8 == 0 and the token scales");
    const int nj = (F / 8 + 1023) / 1024;
#define LLMI_GELU16(N) \
  case N: hipLaunchKernelGGL(prefill_gelu16_kernel<N>, dim3(T), dim3(1024), 0, s, gu, F, H, x16, x16stride, tscale); break;
    switch (nj) {
      LLMI_GELU16(1) LLMI_GELU16(2) LLMI_GELU16(3) LLMI_GELU16(4)
      default: throw std::runtime_error("prefill_gelu: f16 output needs n_ff <= 32768");
    }
#undef LLMI_GELU16
    LLMI_HIP(hipGetLastError());
    return;
  }
  if (H % 8 == 0) {
    hipLaunchKernelGGL(prefill_gelu8_kernel, dim3((F / 8 + 255) / 256, T), dim3(256), 0, s, gu, F, H, xq, xstride, q8k);
    LLMI_HIP(hipGetLastError());
    return;
  }
  hipLaunchKernelGGL(prefill_gelu_kernel, dim3((F + 255) / 256, T), dim3(256), 0, s, gu, F, H, xq, xstride);
  LLMI_HIP(hipGetLastError());
}

}  // namespace llmi
