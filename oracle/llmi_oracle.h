/*
 * llmi_oracle.h -- CPU restatement of the reference's decode-path arithmetic.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this library, and only as the checker
 * (or the timed CPU baseline) -- never as a product path.  The product
 * (llm_inference_amd/libllmi.so) never links or calls it.
 *
 * Every function restates one reference function (corywalker/llm_inference,
 * snapshot 2026-05-01) in plain C with the SAME floating-point operation order
 * the reference gets from its pinned build (Bazel `-c opt` = -O2 -DNDEBUG;
 * ops.cpp additionally -mavx2 -mfma -mf16c, BUILD:41-53; gguf.cpp/model.cpp
 * without -mfma).  Every FMA the reference's compiler contracts is written as
 * an explicit fmaf(); the file is compiled with -ffp-contract=off so nothing
 * else is fused.  Parity of this restatement is pinned bit-for-bit against the
 * reference itself (oracle/_ref, built from /root/reference sources by
 * oracle/Makefile) through the fixtures in tests/golden/.
 *
 * Weight buffers use the GGUF on-disk block layouts (ops.h:11-31, 89-102).
 */
#ifndef LLMI_ORACLE_H
#define LLMI_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ggml tensor type ids (gguf.h:30-46) */
enum {
  ORC_F32 = 0, ORC_F16 = 1, ORC_Q4_0 = 2, ORC_Q5_0 = 6, ORC_Q8_0 = 8,
  ORC_Q4_K = 12, ORC_Q6_K = 14, ORC_BF16 = 30
};

/* fp16/bf16 conversions: gguf.cpp:40-113, 395-402 */
float orc_f16_to_f32(uint16_t h);
uint16_t orc_f32_to_f16(float f);
float orc_bf16_to_f32(uint16_t h);

/* bytes per row of `n_cols` elements of ggml type `type` (0 if unsupported) */
size_t orc_row_bytes(uint32_t type, size_t n_cols);

/* activation quantizers: ops.cpp:116-139 (34-byte BlockQ8_0) and
 * ops.cpp:142-178 (292-byte block_q8_K) */
void orc_quantize_row_q8_0(const float* x, size_t n, uint8_t* y);
void orc_quantize_row_q8_k(const float* x, size_t n, uint8_t* y);

/* o[n_rows] = W[n_rows x n_cols] * x : ops.cpp:933-956 dispatch (Q4_0, Q4_K,
 * Q6_K, Q8_0, Q5_0, BF16) plus F16 (ops.cpp:455-612).  Returns 0, or -1 for
 * an unsupported type.  n_threads splits rows in contiguous chunks exactly as
 * ops.cpp:439-450 (results do not depend on it). */
int orc_mat_vec_mul(uint32_t type, const void* w, size_t n_rows, size_t n_cols,
                    const float* x, float* o, int n_threads);

/* one row of a quantized embedding table -> f32: ops.cpp:958-1082 (Q4_K,
 * Q6_K, Q8_0, Q5_0); F16/F32 handled too (model.cpp:247-257) */
/* Q4_0 / Q8_0 rows against an already-quantized activation (34-B BlockQ8_0) */
int orc_mat_vec_mul_q8(uint32_t type, const void* w, size_t n_rows, size_t n_cols, const void* xq, float* o,
                       int n_threads);
int orc_dequantize_row(uint32_t type, const void* blocks, size_t n_cols,
                       float* o);

/* ops.cpp:28-43 (returns -1 when eps <= 0 where the reference exit(1)s) */
int orc_rms_norm(float* o, const float* x, size_t n, double eps);
/* ops.cpp:45-62 */
void orc_softmax(float* x, size_t n);
/* ops.cpp:67-95; t is [n_tokens][n_heads][head_dim] contiguous */
void orc_rope(float* t, size_t n_tokens, size_t n_heads, size_t head_dim,
              int n_rot, float base, float freq_scale, int pos);
/* ops.cpp:97-105 */
void orc_scale(float* t, size_t n, float s);
/* ops.cpp:1084-1099 */
void orc_vec_scale_f16(uint16_t* y, size_t n, float v);
void orc_vec_mad_f16(uint16_t* y, const uint16_t* x, size_t n, float v);

/* GELU(tanh) * up, model.cpp:892-899 (compiled without FMA) */
void orc_gelu_mul(float* o, const float* gate, const float* up, size_t n);

/* One head of decode/prefill attention against an f16 KV history:
 * model.cpp:481-547.  k,v: [n_keys][head_dim] f16 for that kv head; q: f32
 * [head_dim] (already normed/roped/scaled).  out: f32 [head_dim]. */
void orc_attn_head(const float* q, const uint16_t* k, const uint16_t* v,
                   size_t n_keys, size_t head_dim, float* out);
/* the same with the attention logit soft-cap of model.cpp:511-513 (cap <= 0: none) */
void orc_attn_head_cap(const float* q, const uint16_t* k, const uint16_t* v,
                       size_t n_keys, size_t head_dim, float cap, float* out);

/* ---- whole-model forward (Gemma-3 GGUF), model.cpp:706-1049 ---- */
typedef struct orc_model orc_model;
/* gguf bytes must outlive the model (borrowed, like the reference's mmap) */
orc_model* orc_model_create(const uint8_t* gguf, size_t size, int n_threads,
                            int max_ctx);
void orc_model_destroy(orc_model* m);
/* logits of the LAST token (vocab floats); returns 0 / negative error */
int orc_model_forward(orc_model* m, const int* tokens, int n_tokens, int pos,
                      float* logits);
int orc_model_vocab(const orc_model* m);
/* test-only variant: float64 attention math instead of the reference's f16
 * accumulator (orc_attn_head_f64) -- pins the GPU fast path, NOT the reference */
void orc_model_set_attn_f64(orc_model* m, int on);
void orc_attn_head_f64(const float* q, const uint16_t* k, const uint16_t* v, size_t n_keys, size_t head_dim,
                       float* out);
void orc_attn_head_f64_cap(const float* q, const uint16_t* k, const uint16_t* v, size_t n_keys, size_t head_dim,
                           float cap, float* out);
const char* orc_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
