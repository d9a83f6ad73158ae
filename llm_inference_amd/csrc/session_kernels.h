// session_kernels.h -- weight upload and the fused decode-step glue kernels.
#pragma once

#include "attn.h"
#include "kernels.h"
#include "px.h"

namespace llmi {

size_t gguf_bytes(uint32_t type, size_t rows, size_t cols);
bool gemv_type_supported(uint32_t type);
DevWeight alloc_weight(uint32_t type, int rows, int cols, size_t slack = 64);  // slack: bytes allocated past qs / d
void upload_rows(DevWeight& w, int dst_row0, const void* host, int rows, hipStream_t s);
void free_weight(DevWeight& w);
// device memory of the sessions (k_session.hip): released for reuse at once unless a session is being constructed
// while another is alive (then when the last construction ends); session_live(+1 / -1) brackets a session's
// lifetime, session_constructed() the end of its constructor
void* dev_alloc(size_t bytes);  // session / weight memory (cached when released, k_session.hip)
void dev_free(void* p);
void session_live(int delta);
void session_constructed(bool ok);
void dev_mem_stats(size_t* live, size_t* cached, size_t* grave);  // (llmi_selftest 2)
// Q4_0 row-major blocks -> slab-major (k_layer.hip's a.slab layout): slabs of
// 8 blocks x all rows, block b of row r at (b / 8) rows 8 + r 8 + b % 8.
void to_slab_layout(DevWeight& w, hipStream_t s);
// Q4_K / Q6_K GGUF rows -> the kq sub-block layout of the fused layer kernels (kernels.h)
void to_kq_layout(DevWeight& w, hipStream_t s, int slab = 0);

// outputs of a norm that feeds a GEMV: xn (always), plus optionally the Q8_0
// blocks and/or the f16-rounded copy the next GEMV consumes
struct ScreenX;
struct NormOut {
  float* xn = nullptr;
  XBlock* q8 = nullptr;
  uint16_t* x16 = nullptr;
  uint8_t* q8k = nullptr;  // Q8_K super-blocks (292 B, quantize_row_q8_k) for Q4_K / Q6_K consumers
  // the screened token selection's per-token x16 blocks (k_logits.hip step 1), written by the final norm so
  // the decode loop needs no screen_prep launch; scr_mkey: M, reset here
  ScreenX* scr = nullptr;
  unsigned* scr_mkey = nullptr;
};
// resid = (resid + rms(y) * w_post) * post_scale (y itself when w_post is null;
// post_scale: Gemma-4 layer output scale, 1 = none); outputs rms(resid) * w_next
void launch_residual_norm(const float* y, const float* w_post, float* resid, const float* w_next, const NormOut& out,
                          int n, double eps, bool exact, hipStream_t s, float post_scale = 1.0f);
// Gemma-4 per-layer inputs (model.cpp:676-701): inp[l][i] = (rms(proj[l])[i] * nw[i] + inp[l][i]) / sqrt(2),
// proj already scaled by 1/sqrt(n_embd); one work-group per layer
void launch_ple_combine(const float* proj, const float* nw, float* inp, int n_layer, int n_epl, double eps, bool exact,
                        hipStream_t s);
// final logit soft-capping (model.cpp:1036-1041): x = cap * tanhf(x / cap), glibc tanhf
void launch_softcap(float* x, int n, float cap, hipStream_t s);
void launch_embed_norm(uint32_t type, const uint8_t* table, size_t row_bytes, const int32_t* d_token,
                       float emb_scale, float* resid, const float* w, const NormOut& out, int n, double eps,
                       bool exact, hipStream_t s);
// the decode loop's token feedback (launch_finalize_token) + the next step's embed_norm, one launch
void launch_finalize_embed_norm(unsigned long long* keys, int n_keys, int shard, int32_t* d_token, int32_t* d_pos,
                                int32_t* ring, int32_t* ring_idx, int ring_cap, uint32_t type, const uint8_t* table,
                                size_t row_bytes, float emb_scale, float* resid, const float* w, const NormOut& out,
                                int n, double eps, bool exact, hipStream_t s);
// q8k (n % 256 == 0): the GELU output's Q8_K super-blocks for a Q4_K / Q6_K down projection
void launch_gelu_quant(const float* gu, int n, float* hid, const Q8Act* q8, hipStream_t s, uint8_t* q8k = nullptr);
// Q4_0 GEMV with the decode step's neighbours fused in (k_layer.hip)
// LAYER_GELU_X: the GELU epilogue on x blocks given (a residual/norm launch wrote them: 27B, where the GELU
// prologue's per-work-group residual/norm costs more than a launch of its own)
enum LayerRole { LAYER_PLAIN = 0, LAYER_PRO = 1, LAYER_GELU = 2, LAYER_QUANT = 3, LAYER_GELU_X = 6 };
struct LayerGemv {
  const uint4* qs = nullptr;  // set by launch_layer_gemv from the weight
  const uint16_t* wd = nullptr;
  int rows = 0, nb = 0;
  uint32_t magic = 0;
  int slab = 0;                // weight layout: 0 row-major blocks, 1 slab-major (DevWeight::slab)
  const XBlock* xg = nullptr;  // PLAIN: the activation's Q8_0 blocks
  // PRO / GELU: resid_out = resid_in + rms(y) * w_post (y itself when w_post
  // is null); x = rms(resid_out) * w_next.  QUANT: x = y.
  const float* y = nullptr;
  const float* w_post = nullptr;
  const float* resid_in = nullptr;
  float* resid_out = nullptr;
  const float* w_next = nullptr;
  float* xn_out = nullptr;  // optional copy of x (work-group 0)
  int n = 0;
  double eps = 0;
  float* out = nullptr;     // PLAIN / PRO / QUANT: [rows]
  float* hid = nullptr;     // GELU: [rows / 2] = GELU(gate) * up
  XBlock* hq = nullptr;     // GELU with 32 units per work-group: also their Q8_0 block (the down launch's x)
  const uint32_t* kdd = nullptr;  // kq weights (Q4_K / Q6_K): super-block d words, Q6_K high bits
  const uint2* kqh = nullptr;
  // tensor-parallel ranks, fused exchanges (px.h; px: the session's device-resident link): px_in -- the
  // activation (y for PRO / GELU / QUANT, the x blocks for PLAIN) is read from this rank's mailbox instead of
  // y / xg; px_out -- every output word (out rows; GELU: hid, or the hq blocks when hq is set) is also pushed
  // to every rank's mailbox
  const PxLink* px = nullptr;
  int px_in = -1, px_in_ws = 0;  // >= 0: the exchange (step number, words per rank) read instead of y / xg
  int px_in_nwg = 0;             // the work-groups that pushed it (checksum granules per rank)
  int px_out = -1;               // >= 0: the exchange the outputs are pushed into
};
// Cross-work-group hand-offs of the attention-block kernel (k_attn.hip):
// qkv rows -> the kv head's attention work-groups -> the o projection, as
// data-tagged granules (common.h st_granule / ld_granules) in per-layer buffers.
struct BlockSync {
  // this layer's launch count: granule tag = *epoch + 1, read by every wave at its start.  The launch advances it
  // itself, once every wave of it has read it: *done counts the o work-groups (each once its waves have used
  // their tag) and the kv heads' final merges (each once every split of its head -- and so every qkv work-group
  // those splits waited on -- has used it); the add that completes the count (done_n) resets *done and advances
  // *epoch.  So no launch sequence (timed launches alone, a skipped or repeated neighbour launch) can leave a tag
  // that the next launch would take for its own, and no add sits on the launch's critical path
  unsigned* epoch = nullptr;
  unsigned* done = nullptr;
  unsigned done_n = 0;
  uint2* g_qkv = nullptr;           // [qkv rows] granules of the qkv GEMV output
  uint2* g_xo = nullptr;            // [n_head * head_dim / 32][12] granules of the attention output's Q8_0 blocks
  int* err = nullptr;               // set when a bounded wait gives up (the step's results are invalid)
  unsigned long long* trace = nullptr;  // development: [work-group][8] wall clocks (LLMI_BLOCK_TRACE)
};
bool layer_gemv_supported(const DevWeight& w, int role);
// ---- batched prefill (k_prefill.hip) ----
struct PrefillNorm {  // per token: embedding (table != null) or residual + norm, then x -> Q8_0
  const uint8_t* table = nullptr;
  uint32_t emb_type = 0;
  size_t row_bytes = 0;
  const int32_t* tokens = nullptr;
  float emb_scale = 1.0f;
  const float* y = nullptr;       // [T][n] projection output (residual mode)
  const float* w_post = nullptr;  // null: plain residual add
  float* resid = nullptr;         // [T][n] in/out
  const float* w_next = nullptr;
  XBlock* xq = nullptr;           // [T][xstride] out
  int xstride = 0, n = 0;
  double eps = 0;
  uint16_t* x16 = nullptr;        // non-null: f16 rows [T][x16stride] of the dequantized Q8_0 blocks, scaled per
  int x16stride = 0;              // token by 2^-s (GEMMs v6 / v7)
  float* tscale = nullptr;        // [T] 2^s per token (x16 rows)
  int q8k = 0;                    // 1: Q8_K quants in the blocks (super-block d, block sums; n % 256 == 0)
};
struct PrefillGemm {
  const uint4* qs = nullptr;
  const uint16_t* wd = nullptr;
  int rows = 0, nb = 0, slab = 0, w8 = 0;  // w8: Q8_0 weights (qs [rows][nb][32 B])
  int kq = 0;                              // 1 / 2: Q4_K / Q6_K weights in the kq layout (x: Q8_K blocks)
  const uint32_t* kdd = nullptr;
  const uint2* kqh = nullptr;
  const XBlock* x = nullptr;
  int xstride = 0, T = 0;
  float* out = nullptr;
  int ostride = 0;
};
struct PrefillGemm16 {  // f16 activations [T][xstride elements] (k_prefill.hip GEMM v6)
  const uint4* qs = nullptr;
  const uint16_t* wd = nullptr;   // Q4_0: f16 d per block; kq: the u16 scale word per sub-block
  const uint32_t* kdd = nullptr;  // kq: per super-block d (| dmin)
  const uint2* kqh = nullptr;     // Q6_K kq: high bits per sub-block
  int rows = 0, nb = 0, slab = 0;
  const uint16_t* x = nullptr;
  int xstride = 0, T = 0;
  float* out = nullptr;
  int ostride = 0;
  const float* tscale = nullptr;  // [T] 2^s of the x16 rows (null: 1)
};
struct PrefillQK {
  const float* qkv = nullptr;  // [T][qkv_stride]
  int qkv_stride = 0, k_off = 0, v_off = 0, n_head = 0, n_head_kv = 0, head_dim = 0;
  const float *q_norm_w = nullptr, *k_norm_w = nullptr, *rope_cs = nullptr;
  float attn_scale = 1.0f;
  double eps = 0;
  uint16_t* q_out = nullptr;  // [T][n_head][head_dim] f16, scaled
  uint16_t *k_cache = nullptr, *v_cache = nullptr;
  int max_ctx = 0, pos0 = 0;
};
struct PrefillAttn {
  const uint16_t* q = nullptr;
  const uint16_t *k_cache = nullptr, *v_cache = nullptr;
  int n_head = 0, n_head_kv = 0, head_dim = 0, max_ctx = 0, pos0 = 0;
  XBlock* xq = nullptr;  // [T][xstride]: the heads' outputs as Q8_0 blocks
  int xstride = 0;
  uint16_t* x16 = nullptr;  // non-null: the heads' outputs as f16 rows [T][x16stride] (GEMM v6)
  int x16stride = 0;
  int q8k = 0;              // 1: Q8_K quants (one super-block per head: head_dim 256)
  // key splits across work-groups (MFMA kernel): round q of a query block's key tiles goes to work-group q % ks;
  // partials [head][query block][ks] (64 (head_dim / 2 + 2) floats each), combined by a merge launch
  int ks = 1;
  float* part = nullptr;
  float softcap = 0.0f;     // attention.logit_softcapping (model.cpp:511-513); 0: none
};
constexpr int PREFILL_ATTN_KS_MAX = 8;
void launch_prefill_norm(const PrefillNorm& a, int T, hipStream_t s);
bool prefill_gemm_supported(const DevWeight& w);
void launch_prefill_gemm(const DevWeight& w, const XBlock* x, int xstride, int T, float* out, int ostride,
                         hipStream_t s);
// f16 activations (x16 rows scaled per token, tscale = 2^s per token or null for 1): GEMM v7 for Q4_0 weights
// (the default prefill GEMM where prefill_gemm7_supported), v6 for the K-quants
bool prefill_gemm16_supported(const DevWeight& w);
bool prefill_gemm7_supported(const DevWeight& w);
void launch_prefill_gemm16(const DevWeight& w, const uint16_t* x, int xstride, int T, float* out, int ostride,
                           const float* tscale, hipStream_t s);
void launch_prefill_qk(const PrefillQK& a, int T, hipStream_t s);
void launch_prefill_attn(const PrefillAttn& a, int T, hipStream_t s);
void launch_prefill_gelu(const float* gu, int F, int H, XBlock* xq, int xstride, int T, hipStream_t s,
                         uint16_t* x16 = nullptr, int x16stride = 0, int q8k = 0, float* tscale = nullptr);

// the weight layout the launch-table entry for (w's shape, role) reads
int layer_gemv_slab(const DevWeight& w, int role);
// GELU role: hidden units per work-group (the gate/up interleave group), 0 if unsupported
int layer_gemv_gelu_group(int cols, uint32_t type = T_Q4_0);
// returns the launch's work-group count (a fused exchange's producing work-groups: px.h checksums)
int launch_layer_gemv(const DevWeight& w, LayerGemv a, int role, hipStream_t s);
// K-quant q|k (Q4_K) + v (Q6_K), both in the kq layout, in one launch (qkv roles)
bool layer_gemv2_supported(const DevWeight& wa, const DevWeight& wb, int role);
void launch_layer_gemv2(const DevWeight& wa, const DevWeight& wb, LayerGemv a, int role, hipStream_t s);
// Q8_K quants of x in XBlocks (the activation of a PLAIN kq layer launch), n % 256 == 0
void launch_quantize_q8k_xblocks(const float* x, int n, XBlock* xb, hipStream_t s);
void launch_argmax(const float* x, int n, unsigned long long* key, hipStream_t s);
// Greedy token by bounded screening + exact rescoring (k_logits.hip): the
// same first-index argmax as the fast F16 logits GEMV, from an int8 copy of
// the table plus the candidate rows re-read in f16.
struct ScreenX {  // one 32-block of x16 quantized: qx[32], dx, c_b / 2; .a of entry nb = A
  int4 lo, hi;
  float dx, c_half, a, pad;
};
static_assert(sizeof(ScreenX) == 48, "ScreenX layout");
struct ScreenTable {
  uint8_t* qs = nullptr;     // [rows][nb][32] int8
  uint16_t* d = nullptr;     // [rows][nb] f16 scales (rounded up)
  ScreenX* xs = nullptr;     // [nb + 1] per token
  float* hi = nullptr;       // [rows] upper bounds
  unsigned* m_key = nullptr; // max lower bound (order-preserving key)
  int rows = 0, cols = 0;
  size_t bytes = 0;          // qs + d bytes streamed per token
};
bool screen_supported(const DevWeight& table);
void alloc_screen_table(const DevWeight& table, ScreenTable& st, hipStream_t s);
void free_screen_table(ScreenTable& st);
// prepped: st.xs / st.m_key already hold this token's x16 blocks (a norm with NormOut::scr wrote them)
// exact: the candidates are rescored in the reference's AVX2 order (gemv_f16_exact) instead of the fast GEMV's
void launch_screen_argmax(const DevWeight& table, const ScreenTable& st, const uint16_t* x16,
                          unsigned long long* amax_key, hipStream_t s, bool prepped = false, bool exact = false);

// ---- the screening's x16 blocks (k_logits.hip step 1), shared by screen_prep_kernel and norm_outputs ----
constexpr float SCREEN_DENORM = 6.103515625e-05f;  // 2^-14: smallest normal f16
// one DPP quad per 32-block b (sub = lane & 3 holds v = elements 8 sub .. 8 sub + 7 of the f16-rounded x):
// qx = rint(x / dx), dx = amax / 127, c_b (k_logits.hip header) into *o, entry .a = 0; returns |x_b|_1 (f64,
// quad total).  Quad sums are in a different order than a serial chain: c_b and A are bounds widened by 2^-10
// and rounded up, so any order is valid (the f64 rounding is ~2^-47 relative).
__device__ __forceinline__ double screen_prep_quad(const float (&v)[8], int sub, int n, ScreenX* __restrict__ o) {
  float amax = 0.0f;
#pragma unroll
  for (int i = 0; i < 8; i++) amax = fmaxf(amax, fabsf(v[i]));
  amax = fmaxf(amax, __shfl_xor(amax, 1));
  amax = fmaxf(amax, __shfl_xor(amax, 2));
  const float dx = amax / 127.0f;
  double l1 = 0.0, e = 0.0, den = 0.0;
  uint32_t packed[2] = {0, 0};
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const int q = dx > 0.0f ? (int)fminf(127.0f, fmaxf(-127.0f, rintf(v[i] / dx))) : 0;
    packed[i / 4] |= (uint32_t)(q & 0xFF) << (8 * (i % 4));
    l1 += fabs((double)v[i]);
    e += fabs((double)v[i] - (double)dx * (double)q);
    if (fabsf(v[i]) < SCREEN_DENORM) den += fabs((double)v[i]);
  }
#pragma unroll
  for (int m = 1; m <= 2; m <<= 1) {
    l1 += __shfl_xor(l1, m);
    e += __shfl_xor(e, m);
    den += __shfl_xor(den, m);
  }
  int* words = reinterpret_cast<int*>(o);  // lo = qx words 0..3, hi = 4..7: this lane's 8 quants are words 2 sub, 2 sub + 1
  words[2 * sub] = (int)packed[0];
  words[2 * sub + 1] = (int)packed[1];
  if (sub == 0) {
    const double k_u = (double)(n + 32) * 0x1p-24;
    double c = 0.5 * l1 + 127.5 * e + 127.5 * k_u * (l1 + e) + 127.5 * den;
    c *= 1.0 + 0x1p-10;
    reinterpret_cast<float4*>(o)[2] = make_float4(dx, __double2float_ru(0.5 * c), 0.0f, 0.0f);
  }
  return l1;
}
// all nb blocks' l1 in s_l1 (visible to the caller's first wave): A into xs[nb].a, M reset -- wave 0 only
__device__ __forceinline__ void screen_prep_total(const double* s_l1, int nb, ScreenX* __restrict__ xs,
                                                  unsigned* __restrict__ m_key) {
  const int lane = threadIdx.x & 63;
  double tot = 0.0;
  for (int b = lane; b < nb; b += 64) tot += s_l1[b];
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) tot += __shfl_xor(tot, m);
  if (lane == 0) {
    // A: denormal flushing of the table's f16 values (2^-14 per |x|), doubled
    xs[nb].a = __double2float_ru(2.0 * (double)SCREEN_DENORM * tot * (1.0 + 0x1p-10));
    *m_key = 0u;
  }
}
void launch_finalize_token(unsigned long long* keys, int n_keys, int shard, int32_t* d_token, int32_t* d_pos,
                           int32_t* ring, int32_t* ring_idx, int ring_cap, hipStream_t s);
// d_token = token, d_pos = pos (and ring_idx = 0 when reset): the token loop's inputs, in stream order
void launch_set_token_pos(int32_t* d_token, int32_t* d_pos, int32_t* ring_idx, int token, int pos, bool reset,
                          hipStream_t s);

}  // namespace llmi
