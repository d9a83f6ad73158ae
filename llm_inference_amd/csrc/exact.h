// exact.h -- the exact-order decode engine (k_exact.hip): the reference's AVX2
// arithmetic, bit for bit, at streaming speed.
//
// The reference's Q4_0 row (ops.cpp:364-399) keeps eight fp32 accumulators,
// one per 4-element slot of a 32-element block, each a serial fma chain over
// the row's blocks in order, then hsum_float_8.  A lane here is one row's pair
// of slots (jj, jj + 4): it walks every block of its row in order, so the chains
// are the reference's, while 16 rows x 4 lanes per wave read whole lines from
// the XL weight layout below.
//
// XL layout of a Q4_0 weight [rows][nb] (nb % 4 == 0), group g = blocks 4g..4g+3:
//   qs [g][row][jj] 16 B = bytes 4jj..4jj+3 of the four blocks' 16-B quants
//   d  [g][row]     8 B  = the four blocks' f16 scales
// so one wave-instruction of a group reads 16 rows x 64 B = 1 KB contiguous.
#pragma once

#include "session_kernels.h"

namespace llmi {

struct XlWeight {
  uint4* qs = nullptr;
  uint2* d = nullptr;
  int rows = 0, nb = 0;
  size_t bytes = 0;  // algorithmic (GGUF) bytes
};

// sources of an XL weight: rows [0, n) of each device Q4_0 weight (row-major blocks), concatenated, or (gelu32)
// two weights gate / up interleaved in groups of 32 rows (gate 32 k.., up 32 k..) for the GELU epilogue
struct XlSrc {
  const DevWeight* w[3] = {nullptr, nullptr, nullptr};
  int n = 0;
  bool gelu32 = false;
};
bool xl_supported(const DevWeight& w);
XlWeight make_xl_weight(const XlSrc& src, hipStream_t s);
void free_xl_weight(XlWeight& w);

enum XlRole {
  XL_PLAIN = 0,  // x = the Q8_0 blocks at xb
  XL_QUANT = 1,  // x = quantize_row_q8_0(y)
  XL_PRE = 2,    // h = resid_in (+ rms(y) * w_post when y); resid_out = h; x = Q8_0(rms(h) * w_next)
  XL_GELU = 3,   // XL_PRE, then GELU(gate) * up of the work-group's 32 units -> hid, hq (one Q8_0 block)
};
struct XlArgs {
  const XBlock* xb = nullptr;
  const float* y = nullptr;
  const float* w_post = nullptr;
  const float* resid_in = nullptr;
  float* resid_out = nullptr;
  const float* w_next = nullptr;
  float* xn_out = nullptr;  // optional: x before quantization (work-group 0)
  int n = 0;                // input length (= nb * 32)
  double eps = 0;
  float* out = nullptr;     // PLAIN / QUANT / PRE: [rows]
  float* hid = nullptr;     // GELU: [rows / 2]
  XBlock* hq = nullptr;     // GELU: [rows / 64]
};
void launch_exact_gemv(const XlWeight& w, const XlArgs& a, int role, hipStream_t s);

// Exact decode attention of one layer (model.cpp:430-550 with the q / k norms, rope and scale of
// model.cpp:762-794 and the KV append of model.cpp:440-474), as two wide launches:
//   scores: grid (n_head, XA_NSPLIT), one wave each: the head's q row (its serial norm chain, rope, scale,
//           f16 rounding), the new key's K / V rows where the wave owns the current position (the same bits
//           written by every q head of the kv head), then one key per lane -- the reference's sequential
//           double sum over the head dims -- into scores[head][key];
//   accum:  one work-group per head: per 1024-key chunk the exclusive prefix max of the scores in double
//           (the reference's running max is always the float rounding of it), every key's branch and its
//           e / pe (glibc expf), then per head dim the f16 V accumulator in key order (vec_scale_f16 /
//           vec_mad_f16) and, on an extra wave, s_acc in key order; out = f16(v) * (1 / s_acc), and its
//           Q8_0 blocks for the o projection.
constexpr int XA_NSPLIT = 32;  // scores: work-groups per head, each taking key chunks of 64 split apart
struct XAttnArgs {
  const float* qkv = nullptr;
  int k_off = 0, v_off = 0;
  int n_head = 0, n_head_kv = 0, head_dim = 0;
  const float* q_norm_w = nullptr;
  const float* k_norm_w = nullptr;
  const float* rope_cs = nullptr;  // [max_ctx][head_dim / 2][2]
  float attn_scale = 1.0f;
  double eps = 0;
  uint16_t* k_cache = nullptr;
  uint16_t* v_cache = nullptr;
  int max_ctx = 0;
  const int* d_pos = nullptr;
  double* scores = nullptr;  // [n_head][max_ctx]
  float* out = nullptr;      // [n_head][head_dim]
  XBlock* xq = nullptr;      // [n_head * head_dim / 32]
  float softcap = 0.0f;      // attention.logit_softcapping (model.cpp:511-513); 0: none
  // the V cache in the accumulate kernel's read order (vt_stride % 32 == 0 keys per kv head): tiles of 64 head
  // dims x 32 keys, [n_head_kv][head_dim / 64][vt_stride / 32][4 key octets][64 dims][8 keys] f16 (xa_vt_index):
  // the scores kernel appends the new key's column, the accumulate kernel's 64 lanes (dims) read one key octet of
  // a tile as one contiguous 1-KB load (16 B = 8 keys per lane)
  uint16_t* vt = nullptr;
  int vt_stride = 0;
  // per key [n_head_kv][max_ctx]: (min over its nonzero elements of max(f16 exponent field, 1)) << 16 | max |k| as
  // f16 bits, written with the K row; 0 = unknown (the score then takes the serial chain)
  uint32_t* kmeta = nullptr;
  // batched prefill (launch_exact_attn_batch): T tokens at positions *d_pos + z, z < T; their q|k|v rows at
  // qkv + z qkv_stride; the f16 query rows [T][n_head][head_dim] (written by the batch's q/k launch); scores at
  // [T][n_head][max_ctx], out at [T][n_head * head_dim], xq at [T][n_head * head_dim / 32]
  uint16_t* qh = nullptr;
  int qkv_stride = 0;
};
bool exact_attn_supported(int head_dim, int n_head, int n_head_kv);
void launch_exact_attn(const XAttnArgs& a, hipStream_t s);
// The exact attention of T prompt tokens at once (model.cpp:430-550 per token, causal over keys 0 .. pos + z):
// every token's q / k row norms, rope, the K / V appends, then every (token, head)'s scores and its accumulator
// chain -- each token's arithmetic exactly that of its own decode step.
void launch_exact_attn_batch(const XAttnArgs& a, int T, hipStream_t s);

// Batched exact prefill (k_exact.hip): the prompt's tokens before the last run layer by layer, T at a time, each
// (row, token) with the reference's own accumulator chains.
// norm: per token, h = (embed ? table row * emb_scale : resid + rms(y) * w_post), resid = h, x = Q8_0(rms(h) * w_next)
struct XpNormArgs {
  const uint8_t* table = nullptr;  // embed: the GGUF rows (F16 / F32 / Q8_0), row_bytes apart
  size_t row_bytes = 0;
  uint32_t type = 0;
  const int32_t* tokens = nullptr;
  float emb_scale = 1.0f;
  const float* y = nullptr;        // [T][n] (pre)
  const float* w_post = nullptr;
  float* resid = nullptr;          // [T][n], in place
  const float* w_next = nullptr;
  XBlock* xq = nullptr;            // [T][n / 32]
  int n = 0;
  double eps = 0;
};
void launch_exact_norm_batch(const XpNormArgs& a, int T, hipStream_t s);
// rows x T tokens of an XL weight on the tokens' Q8_0 blocks x [T][nb]: out [T][ldo] (plain), or (gelu32 weights)
// GELU(gate) * up of each 32-unit group -> hq [T][rows / 64] Q8_0 blocks
void launch_exact_gemm(const XlWeight& w, const XBlock* x, int T, float* out, int ldo, XBlock* hq, hipStream_t s);
// self-test (synchronous): over every f32 bit pattern, out[0] = non-NaN inputs whose hardware f16 conversion
// differs from the reference's f32_to_f16, out[1] = NaN inputs that differ, out[2] = the first non-NaN one
void exact_selftest_f16(unsigned long long* out3);
// self-test (synchronous): 8192 vectors of 2560 floats through the speculative norm chain and the serial one:
// out[0] = results that differ, out[1] = segments that fell back to the serial chain
void exact_selftest_chain(unsigned* out2);

}  // namespace llmi
