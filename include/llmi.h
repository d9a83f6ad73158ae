/*
 * llmi.h -- C ABI of the MI355X-native decode path for corywalker/llm_inference.
 *
 * Library: llm_inference_amd/libllmi.so (HIP, gfx950).  Plain C types only:
 * pointers, sizes, status codes.  No exceptions cross this boundary; every
 * entry point returns llmi_status (0 = OK) and llmi_last_error() holds the
 * reference's own message text for the failure (thread-local).
 *
 * Two layers:
 *  (1) ops.h drop-in (host buffers, synchronous: results are complete on
 *      return, like the reference's fork/join GEMVs, ops.cpp:450).  One entry
 *      point per reference function; the reference line each one replaces is
 *      cited.  The C++ functions with the reference's exact ops.h signatures
 *      are integration/ops_mi355x.cpp, built in place of ops.cpp
 *      (INTEGRATION.md shows the Bazel wiring).
 *  (2) device session: the whole Gemma-3 forward of Model::forward
 *      (model.cpp:706-1049) resident on one MI355X, weights uploaded once from
 *      the caller's GGUF bytes (the GGUF loader/format is unchanged), each
 *      decode token replayed as one hipGraph.
 *
 * Numerics: LLMI_EXACT selects kernels that reproduce the reference's AVX2
 * operation order bit-for-bit (GEMVs, quantizers, norms, rope, f16 vector ops);
 * the default (fast) kernels reassociate reductions across a wavefront and
 * are checked to the tolerances stated in DESIGN.md.
 */
#ifndef LLMI_H
#define LLMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  LLMI_OK = 0,
  LLMI_E_SIZE = 1,   /* input size mismatch: ops.cpp:196-198 ("input vector size mismatch") */
  LLMI_E_TYPE = 2,   /* unsupported tensor type: ops.cpp:953-954 */
  LLMI_E_ARG = 3,    /* invalid argument (e.g. eps <= 0: ops.cpp:29-32, which exit(1)s) */
  LLMI_E_HIP = 4,    /* HIP runtime failure */
  LLMI_E_GGUF = 5,   /* malformed GGUF / missing metadata: gguf.cpp:276-277, model.cpp:64-66 */
  LLMI_E_NODEV = 6,  /* no usable gfx950 device */
  LLMI_E_RANGE = 7   /* context overflow / token id out of range */
} llmi_status;

/* flags */
#define LLMI_EXACT 1u      /* bit-exact AVX2-order kernels */
#define LLMI_NO_GRAPH 2u   /* session: launch kernels eagerly instead of one hipGraph per token */
#define LLMI_TP_PEER 4u    /* session: tensor-parallel rank of tp_size processes (one per GPU) exchanging by
                              one-shot peer push (llmi_session_peer_connect) instead of RCCL */

const char* llmi_last_error(void);
int llmi_version(void);

/* ---------------------------------------------------------------------------
 * (1) ops.h drop-in -- host pointers, synchronous
 * ------------------------------------------------------------------------- */
/* init_ops(int n_threads), ops.cpp:21-24: selects the HIP device instead of a
 * thread count; must precede the other calls (implicitly device 0 otherwise). */
int llmi_init_ops(int device);

/* mat_vec_mul, ops.cpp:933-956 (+ mat_vec_mul_fp16, ops.cpp:455-612, for
 * type 1 = F16): o[n_rows] = W[n_rows x n_cols] * x.  W is in GGUF block
 * layout (row-major blocks, ops.h:11-31/89-102), types Q4_0 2, Q5_0 6, Q8_0 8,
 * Q4_K 12, Q6_K 14, BF16 30, F16 1.  x_len must equal n_cols. */
int llmi_mat_vec_mul(uint32_t type, const void* w, size_t n_rows, size_t n_cols, const float* x, size_t x_len,
                     float* o, uint32_t flags);

/* Weight handles: upload (and repack) a GGUF weight once, then multiply many
 * times -- what the compat layer does per TensorInfo (keyed by its mmap
 * pointer) so a model.cpp-driven decode moves only x and o per call. */
typedef struct llmi_weight llmi_weight;
int llmi_weight_create(uint32_t type, const void* w, size_t n_rows, size_t n_cols, llmi_weight** out);
int llmi_weight_mat_vec_mul(const llmi_weight* w, const float* x, size_t x_len, float* o, uint32_t flags);
/* device-pointer form on a caller stream (hipStream_t passed as void*) */
int llmi_weight_mat_vec_mul_dev(const llmi_weight* w, const float* x_dev, float* o_dev, uint32_t flags,
                                void* stream);
void llmi_weight_destroy(llmi_weight* w);

int llmi_quantize_row_q8_0(const float* x, size_t n, void* y);  /* ops.cpp:116-139, 34-B BlockQ8_0 out */
int llmi_quantize_row_q8_k(const float* x, size_t n, void* y);  /* ops.cpp:142-178, 292-B block_q8_K out */
/* dequantize_{q4_k,q6_k,q8_0,q5_0}_row, ops.cpp:958-1082 (+F16/F32) */
int llmi_dequantize_row(uint32_t type, const void* blocks, size_t n_cols, float* o);
int llmi_rms_norm(float* o, const float* x, size_t n, double eps, uint32_t flags); /* ops.cpp:28-43 */
int llmi_softmax(float* x, size_t n);                                              /* ops.cpp:45-62 */
/* rope, ops.cpp:67-95; t is [n_tokens][n_heads][head_dim] contiguous, in place */
int llmi_rope(float* t, size_t n_tokens, size_t n_heads, size_t head_dim, int n_rot, float freq_base,
              float freq_scale, int pos);
int llmi_scale(float* t, size_t n, float s);                                      /* ops.cpp:97-105 */
int llmi_vec_scale_f16(uint16_t* y, size_t n, float v);                           /* ops.cpp:1084-1089 */
int llmi_vec_mad_f16(uint16_t* y, const uint16_t* x, size_t n, float v);          /* ops.cpp:1091-1099 */

/* Decode attention of Model::run_attn (model.cpp:478-550) for one query
 * token against an f16 KV history: q [n_head][head_dim] f32 (already
 * normed/roped/scaled), k/v [n_head_kv][n_keys][head_dim] f16 bits, out
 * [n_head][head_dim] f32.  LLMI_EXACT = the reference's sequential algorithm
 * (double scores, f16 V accumulator); default = split-K fp32. */
int llmi_attention(const float* q, const uint16_t* k, const uint16_t* v, int n_head, int n_head_kv, int n_keys,
                   int head_dim, float* out, uint32_t flags);
/* GELU(tanh)(gate) * up, model.cpp:892-899 */
int llmi_gelu_mul(const float* gate, const float* up, size_t n, float* out);

/* ---------------------------------------------------------------------------
 * (2) device session (Gemma-3 GGUF)
 * ------------------------------------------------------------------------- */
typedef struct llmi_session llmi_session;
typedef struct llmi_tp_group llmi_tp_group;

typedef struct {
  int device;          /* HIP device ordinal */
  uint32_t flags;      /* LLMI_EXACT | LLMI_NO_GRAPH */
  int max_ctx;         /* KV-cache capacity in positions (default 4096) */
  int attn_split;      /* fast attention key-range splits: 0 = default (32, the only value) */
  /* Row-sharded tensor parallelism (north star: "weights shard row-wise across
   * the 8 GPUs of one node with an RCCL all-gather"; the reference itself is
   * single-device).  Active when tp_id or tp_group is non-NULL: this session
   * is rank tp_rank of tp_size and holds 1/tp_size of every projection's
   * output rows (q/k/v heads, o/down rows, gate/up hidden units, vocabulary
   * rows); after each projection the slices are all-gathered.  Fast kernels
   * only (not with LLMI_EXACT).  Every rank must make the same session calls. */
  int tp_rank, tp_size;
  const void* tp_id;        /* LLMI_TP_ID_BYTES from llmi_tp_unique_id on one rank: RCCL over xGMI */
  llmi_tp_group* tp_group;  /* or: ranks on one device in one process (tests; one host thread per rank) */
  /* or (both NULL, flags LLMI_TP_PEER): the one-shot push exchange between processes, below */
} llmi_session_opts;

#define LLMI_TP_ID_BYTES 128
/* new RCCL communicator id (ncclGetUniqueId); distribute it to every rank */
int llmi_tp_unique_id(void* out);
/* single-device group of `size` ranks: the push exchange split around a host barrier (LLMI_TP_EXCHANGE=copy:
 * device-to-device slice copies) */
int llmi_tp_group_create(int size, llmi_tp_group** out);
void llmi_tp_group_destroy(llmi_tp_group* g);

/* One-shot push exchange (replaces ncclAllGather, the exchange of ops.cpp:439-450's row split
 * across devices): every rank writes its slice of each all-gather as data-tagged 8-byte granules {word, tag}
 * straight into every peer's mailbox through xGMI peer mappings, then polls its own mailbox -- one kernel per
 * exchange, captured in the token's hipGraph.  A LLMI_TP_PEER session: after creation, every rank publishes
 * its mailbox handle, and before its first forward connects to all of them (rank order, tp_size x
 * LLMI_PEER_HANDLE_BYTES); the handles travel by any host channel (bench.py: torch.distributed). */
#define LLMI_PEER_HANDLE_BYTES 64
int llmi_session_peer_handle(const llmi_session* s, void* out);
int llmi_session_peer_connect(llmi_session* s, const void* handles);

/* Parses the GGUF (format of gguf.cpp:274-304, hparams of model.cpp:58-167)
 * and uploads every weight.  The bytes are only read during the call. */
int llmi_session_create(const void* gguf, size_t size, const llmi_session_opts* opts, llmi_session** out);
void llmi_session_destroy(llmi_session* s);

/* Model::forward(tokens, pos) (model.cpp:706): runs n_tokens tokens at
 * positions pos..pos+n_tokens-1 and returns the LAST token's logits
 * (vocab floats, may be NULL) and its greedy argmax (may be NULL).
 * Fast sessions on one device run n_tokens > 1 as a batched prefill (int8
 * MFMA GEMMs over the tokens, causal attention over the cache) instead of
 * the reference's token loop (model.cpp:752-756); LLMI_NO_PREFILL=1 in the
 * environment forces the token loop. */
int llmi_session_forward(llmi_session* s, const int32_t* tokens, int n_tokens, int pos, float* logits,
                         int32_t* argmax);

/* Layer-by-layer triage: llmi_session_forward's token
 * loop, one token at a time with eager launches, appending the
 * intermediates the reference prints under --verbose (model.cpp VERBOSE
 * print_tensor calls: inp_scaled, attn_norm-L, Qcur-L, Kcur-L, Vcur-L,
 * kqv_out-L, "attention results (node_30 for MUL_MAT)-L", sa_out-L,
 * ffn_norm-L, ffn_geglu-L, ffn_out-L, l_out-L, result_norm, result_output)
 * to the text file `path` in tensor.h's print_tensor format, so the two
 * dumps pair by name and occurrence (scripts/compare_dumps.py, the
 * compare_tensors.py counterpart).  Slow; the results equal forward's. */
int llmi_session_dump(llmi_session* s, const int32_t* tokens, int n_tokens, int pos, const char* path);

/* Op-level parity taps (test hook; the per-op counterpart of
 * llmi_session_dump).  Runs the SAME kernels the decode graph (or, for
 * n_tokens > 1 on a batched-prefill session, the prefill) launches, eagerly,
 * and after each launch copies the buffers it produced to the host and calls
 * fn(user, name, layer, data, bytes) -- e.g. "qkv_g" (the attention block's
 * q|k|v rows as {value, tag} granules), "attn", "xo_g", "o", "kc"/"vc" (the
 * layer's KV cache), "ffn_resid", "ffn_norm", "hid", "down", "result_norm",
 * "logits"/"token"; the prefill taps its GEMM inputs ("pf_x_<proj>", Q8_0
 * blocks) and outputs ("pf_<proj>").  flags bit 0: the decode-loop step
 * (screened token selection) instead of forward's full logits.  Slow; the
 * session's state advances exactly as llmi_session_forward's. */
typedef void (*llmi_trace_fn)(void* user, const char* name, int layer, const void* data, size_t bytes);
int llmi_session_trace(llmi_session* s, const int32_t* tokens, int n_tokens, int pos, uint32_t flags,
                       llmi_trace_fn fn, void* user);

/* Greedy decode loop of main.cpp:172-224 kept on the device: token `first`
 * at position `pos`, then n_steps forwards, each feeding its argmax to the
 * next without a host round trip.  out_tokens[i] = argmax after step i. */
int llmi_session_generate(llmi_session* s, int32_t first, int pos, int n_steps, int32_t* out_tokens);

/* Enqueue n_steps decode steps without waiting (bench); llmi_session_sync
 * waits and copies the produced tokens (may be NULL). */
int llmi_session_enqueue(llmi_session* s, int32_t first, int pos, int n_steps);
int llmi_session_sync(llmi_session* s, int32_t* out_tokens, int n);

typedef struct {
  int n_layer, n_embd, n_ff, n_head, n_head_kv, head_dim, vocab, max_ctx;
  size_t weight_bytes;        /* device bytes of all uploaded weights */
  size_t bytes_per_token;     /* algorithmic HBM bytes of one decode token, KV excluded */
  size_t kv_bytes_per_pos;    /* + this many bytes per attended position */
  int kernels_per_token;      /* launches captured in the decode graph */
  int tp_rank, tp_size;       /* weight_bytes / bytes_per_token / kv_bytes_per_pos are this rank's */
  int batched_prefill;        /* 1: llmi_session_forward runs n_tokens > 1 as a batched (MFMA) prefill */
  int screened_logits;        /* 1: llmi_session_enqueue/generate pick each greedy token by int8 screening +
                                 exact f16 rescoring (same ids as the full F16 logits GEMV; forward keeps it) */
  size_t screen_bytes;        /* bytes of the int8 screening table streamed per decode-loop token */
  int prefill_f16_redo;       /* f16 prefills whose final norm row came out non-finite and were recomputed on the
                                 int8 path (never a non-finite result; the per-token scales make it unreachable short
                                 of an attention output past 65504) */
  int layer_engine;           /* always 0: the round-3 layer engine (one launch per decode layer) measured slower
                                 than three launches and was removed in round 6 */
  int ffn_engine;             /* always 0: the FFN engine (gate_up + GELU + down as one launch), likewise */
  int tp_exchange;            /* tensor-parallel exchange: 0 none, 1 RCCL, 2 device copies, 3 one-shot push, 4 one-shot
                                 push fused into the decode launches (the default push mode) */
  long long block_slow_waits; /* attention-block hand-off waits (per wave) that took over 20 us, since creation */
  int exact_engine;           /* 1: LLMI_EXACT runs on the exact-order engine (k_exact.hip: the reference's
                                 arithmetic with streamed GEMVs and fused norms), 0: the per-op exact kernels */
  int exact_batched_prefill;  /* 1: an exact session runs a prompt's tokens before the last layer by layer, T at a
                                 time (the reference's chains per (row, token)), then the last as a decode step */
  int prefill_gemm;           /* the batched prefill's GEMM: 7 f16 MFMA on f16 rows of the dequantized Q8_0 activation
                                 blocks (Q4_0 layers, one device: the default), 5 int8 MFMA on Q8_0 / Q8_K blocks
                                 (LLMI_PREFILL_F16=0, Q8_0 weights, tensor-parallel ranks), 6 f16 for K-quant layers
                                 (LLMI_PREFILL_F16=1); 0 no batched prefill */
} llmi_session_info;
int llmi_session_get_info(const llmi_session* s, llmi_session_info* info);

/* Benchmark hook: time `reps` passes over one decode kernel family, every
 * launch with the real arguments of the decode step and bracketed by HIP
 * events its own dispatch signals, on the session stream:
 *   0 = attention block (qkv + attention + o, one launch per layer; KV
 *       history read at the session's current position),
 *   1 = F16 logits GEMV, 2 = the decode loop's screened token selection,
 *   3 = gate_up (+ norm prologue + GELU), 4 = down (+ Q8_0 prologue),
 *   5 = qkv / o / gate_up / down as standalone layer GEMVs (round-1 family),
 *   6, 7 = the removed layer / FFN engines (always 0 / 0).
 * Returns the mean microseconds and the mean algorithmic bytes per launch
 * (0 / 0 when the family does not exist on this session). */
int llmi_session_time_kernel(llmi_session* s, int which, int reps, double* us_per_launch, double* bytes_per_launch);

/* Device self-tests of arithmetic the exact kernels rely on (synchronous, current device):
 *   0 = every f32 bit pattern through the hardware f32 -> f16 conversion vs the reference's f32_to_f16
 *       (gguf.cpp:68-95): out[0] non-NaN mismatches, out[1] NaN mismatches, out[2] first non-NaN mismatch;
 *   1 = the exact engine's speculative rms_norm sum-of-squares chain vs the serial chain (ops.cpp:33-36) on 8192
 *       vectors of 2560: out[0] differing results (must be 0), out[1] segments recomputed serially;
 *   2 = (no GPU work) the sessions' device memory: out[0] bytes allocated, out[1] bytes released and kept for
 *       reuse, out[2] bytes held back while sessions were constructed concurrently. */
int llmi_selftest(int which, unsigned long long* out);

#ifdef __cplusplus
}
#endif
#endif
