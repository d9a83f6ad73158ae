// session.h -- device-resident Gemma-3 decode session (behind llmi_session_*).
#pragma once

#include <cstdio>
#include <memory>
#include <string>
#include <utility>
#include <vector>

#include "../../include/llmi.h"
#include "collective.h"
#include "exact.h"
#include "gguf_reader.h"
#include "session_kernels.h"

namespace llmi {

struct status_error : std::runtime_error {
  int code;
  status_error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

struct HParams {  // model.h:22-43 (Gemma-3 subset)
  std::string arch;
  int n_layer = 0, n_embd = 0, n_ff = 0, n_head = 0, n_head_kv = 0;
  int hd_k = 0, hd_k_swa = 0, hd_v = 0, hd_v_swa = 0;
  double eps = 0;
  float rope_base = 0, rope_scale = 1.0f, attn_scale = 1.0f;
  std::vector<bool> swa_layers;
  // Gemma-4 (model.cpp:117-166)
  bool gemma4 = false;
  int n_epl = 0;             // embedding_length_per_layer(_input)
  int kv_from = -1;          // n_layer_kv_from_start: layers >= kv_from read an earlier layer's cache
  float final_softcap = 0;   // attention.final_logit_softcapping
  float attn_softcap = 0;    // attention.logit_softcapping (model.cpp:130-133, 511-513)
};

struct GemvPart {  // one weight GEMV writing rows [out_off, out_off + rows)
  DevWeight w;
  int out_off = 0;
};

struct LayerDev {
  std::vector<GemvPart> qkv;  // 1 part when q|k|v share a type (fused), else 3
  int k_off = 0, v_off = 0, qkv_rows = 0;
  GemvPart o;
  std::vector<GemvPart> gate_up;  // 1 part (fused rows [gate; up]) or 2
  GemvPart down;
  float *attn_norm = nullptr, *q_norm = nullptr, *k_norm = nullptr;
  float *post_attn_norm = nullptr, *ffn_norm = nullptr, *post_ffw_norm = nullptr;
  bool is_swa = false;
  bool gu_interleaved = false;  // gate_up rows in groups of 32 (k_layer.hip GELU epilogue)
  bool fused = false;           // every projection runs as gemv_q4_0_layer
  int hd = 0;
  uint16_t *kc = nullptr, *vc = nullptr;
  uint16_t* vt = nullptr;      // exact-order engine: the V cache in 64-dim x 32-key tiles (exact.h)
  uint32_t* kmeta = nullptr;   // exact-order engine: per-key exponent / magnitude words (exact.h XAttnArgs::kmeta)
  // Gemma-4
  bool has_kv = true;            // false: shared-KV layer, kc/vc alias layer kv_src's cache
  int kv_src = -1;
  GemvPart ple_gate, ple_proj;   // per-layer embedding step (model.cpp:926-966), BF16 usually
  float* ple_post_norm = nullptr;
  float out_scale = 1.0f;        // layer output scale (model.cpp:968-977)
  // the exact-order engine (exact.h): q|k|v, o, gate/up (32-unit interleave), down in the XL layout
  XlWeight xqkv, xo, xgu, xdn;
};

class Session {
 public:
  Session(const uint8_t* gguf, size_t size, const llmi_session_opts& opts);
  ~Session();
  Session(const Session&) = delete;
  Session& operator=(const Session&) = delete;

  void forward(const int32_t* tokens, int n_tokens, int pos, float* logits, int32_t* argmax);
  void forward_dump(const int32_t* tokens, int n_tokens, int pos, const char* path);
  void forward_trace(const int32_t* tokens, int n_tokens, int pos, bool gen, llmi_trace_fn fn, void* user);
  void enqueue(int32_t first, int pos, int n_steps);
  void sync(int32_t* out_tokens, int n);
  void info(llmi_session_info* out) const;
  void time_kernel(int which, int reps, double* us, double* bytes);
  void peer_handle(void* out) const;
  void peer_connect(const void* handles);

 private:
  void release();
  void load_hparams(const GGUFView& g);
  void setup_tp();
  void upload(const GGUFView& g);
  void alloc_buffers();
  void build_rope_tables();
  // gen: the decode loop's step (token id only: screened logits when screen_)
  // fold_embed: the step ends with the NEXT step's embed_norm inside the token feedback launch and starts at
  // layer 0 (the decode-loop graph; enqueue launches the first embed_norm itself)
  // logits false: the layers and the final norm only (a prompt token whose logits nobody reads: model.cpp:983-1001
  // computes the logits of the last prompt position only)
  void record_step(hipStream_t s, bool gen = false, bool fold_embed = false, bool logits = true);
  bool embed_fold_ok() const;
  NormOut embed_out() const;
  bool down_plain(const LayerDev& Ld) const;
  void record_logits(hipStream_t s, bool gen = false);  // xn_ / act_.x16 -> logits, argmax key, token feedback
  void prefill(const int32_t* tokens, int n, int pos);  // batched (k_prefill.hip)
  bool prefill_f16_ok() const;  // the batched prefill's activations as f16 rows (GEMM v7 / v6)
  bool prefill_run(const int32_t* tokens, int n, int pos, bool allow_f16);  // true: ran the f16 path
  void gather_cols(void* buf, size_t pitch_b, size_t slice_b, int T, hipStream_t s);
  void ensure_prefill_buffers(int cap);
  void record_layers(hipStream_t s, bool x_q8);
  void record_layers_fused(hipStream_t s, bool x_q8);
  // exact mode on the exact-order engine (k_exact.hip): Q4_0 Gemma-3 layers, reference arithmetic, streamed
  bool xl_ = false;
  double* xa_scores_ = nullptr;  // exact attention scores [n_head][max_ctx]
  XBlock* xa_xq_ = nullptr;      // exact attention output's Q8_0 blocks (the o projection's x)
  void setup_xl();
  void record_layers_xl(hipStream_t s);
  // exact mode's prompt: tokens [0, n) at positions pos.. through every layer, T at a time (k_exact.hip batched
  // kernels), leaving their K / V in the caches -- the reference computes nothing else of them that is kept
  // (model.cpp:983-1001: the logits of the last prompt position only, which runs as a decode step)
  bool xp_ok() const;
  void exact_prefill(const int32_t* tokens, int n, int pos);
  int xp_cap_ = 0;
  int32_t* xp_tok_ = nullptr;
  float *xp_resid_ = nullptr, *xp_o_ = nullptr, *xp_d_ = nullptr, *xp_qkv_ = nullptr, *xp_att_ = nullptr;
  XBlock *xp_xq_ = nullptr, *xp_hq_ = nullptr, *xp_axq_ = nullptr;
  uint16_t* xp_qh_ = nullptr;
  double* xp_sc_ = nullptr;
  void prepare_act(uint32_t wtype, const float* x, int n, ActBuf& act, hipStream_t s);
  void gemv_parts(const std::vector<GemvPart>& parts, const float* x, int n_in, float* out, hipStream_t s,
                  bool x_ready);
  // LLMI_DUP ablation (diagnostics): kernel families launched twice per step,
  // so the step-time delta is that family's in-graph cost
  int dup(const char* k) const { return dup_.find(k) != std::string::npos ? 2 : 1; }
  void set_token_pos(int32_t token, int pos, bool reset_ring);
  // the step graphs: STEP_LOGITS (forward: full logits + argmax), STEP_GEN (the decode loop: token id only, the
  // next embedding folded in), STEP_HIDDEN (a prompt token before the last: no logits)
  enum { STEP_LOGITS = 0, STEP_GEN = 1, STEP_HIDDEN = 2, N_STEP_KINDS = 3 };
  void ensure_graph(int kind);
  // llmi_session_dump: eager steps with print_tensor-format dumps (dump_ set)
  std::FILE* dump_ = nullptr;
  void dump(const std::string& name, const float* dev, int n, hipStream_t s);
  // llmi_session_trace: host copies of what each launch produced (eager steps)
  llmi_trace_fn trace_fn_ = nullptr;
  void* trace_user_ = nullptr;
  void tap(const char* name, int layer, const void* dev, size_t bytes, hipStream_t s);
  void run_step(int kind = STEP_LOGITS);
  float* dev_f32_copy(const GGUFView& g, const GTensor* t, int n);
  // every allocation is zeroed ON THE SESSION'S STREAM, so the zeroing is ordered before every kernel of this
  // session that uses the buffer (null-stream hipMemset / hipMemcpy are not ordered with a non-blocking stream;
  // DESIGN.md section 7, the round-5 tensor-parallel finding)
  template <typename T>
  T* dalloc(size_t count) {
    void* p = dev_alloc(count * sizeof(T) + 64);
    allocs_.push_back(p);
    LLMI_HIP(hipMemsetAsync(p, 0, count * sizeof(T) + 64, stream_));
    return static_cast<T*>(p);
  }
  // host bytes -> device, on the session's stream, complete on return (the host buffer may go away)
  void h2d(void* dst, const void* src, size_t bytes) {
    LLMI_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, stream_));
    LLMI_HIP(hipStreamSynchronize(stream_));
  }
  bool live_ = false;          // counted in session_live (k_session.hip)
  bool constructing_ = false;  // between session_live(+1) and session_constructed()

  llmi_session_opts opts_;
  bool exact_ = false, use_graph_ = true;
  bool fuse_layers_ = false;  // fast path: norms / GELU folded into the Q4_0 GEMVs
  bool block_ = false;        // fast path: qkv + attention + o as one launch per layer (k_attn.hip)
  bool block_pro_ = false;
  long long slow_waits_ = 0;  // block hand-off waits over 20 us (blk_err_[1], accumulated at every sync)
  // the attention block's granule tags: [n_layer] launch counts, each advanced by its own launch
  // (BlockSync::done: [n_layer] the launch's counted work-groups, back to 0 when it advances)
  unsigned* blk_epoch_ = nullptr;
  unsigned* blk_done_ = nullptr;
  uint2* blk_gqkv_ = nullptr;      // [n_layer][qkv rows] granules
  // Gemma-4 per-layer inputs (model.cpp:568-704)
  DevWeight ple_table_{};          // raw GGUF rows [vocab][n_layer * n_epl] (F16 / Q6_K / Q4_K), lookups only
  size_t ple_row_bytes_ = 0;
  std::vector<GemvPart> ple_model_proj_;  // n_embd -> n_layer * n_epl (optional)
  float* ple_proj_norm_ = nullptr;
  float *inp_pl_ = nullptr, *ple_proj_out_ = nullptr, *ple_g_ = nullptr, *ple_u_ = nullptr, *ple_tmp_ = nullptr;
  uint2* blk_gxo_ = nullptr;       // [n_layer][n_head * hd / 32 * 12] granules
  size_t blk_gqkv_stride_ = 0, blk_gxo_stride_ = 0;
  int* blk_err_ = nullptr;       // set by a bounded wait that gave up
  unsigned long long* blk_trace_ = nullptr;  // LLMI_BLOCK_TRACE (development)
  int blk_trace_layer_ = -1;
  XBlock* hq_ = nullptr;         // the GELU launch's Q8_0 blocks of hid (down as a PLAIN launch, 32-unit groups)
  XBlock* blk_xo_ = nullptr;     // attention output Q8_0 blocks (layer 0's qkv still reads act_.q8 in the launch)
  void check_device_error();
  // a tensor-parallel session whose exchange failed (or that threw between two exchanges) may be out of step with
  // its peers: every later call is refused until the group is re-created
  void ensure_usable() const;
  template <class F> void tp_guarded(F&& f);
  bool broken_ = false;
  bool ex_gemv_ = false, ex_norm_ = false, ex_attn_ = false, ex_logits_ = false;  // per kernel family
  HParams hp_;
  int vocab_ = 0, max_ctx_ = 4096;
  hipStream_t stream_ = nullptr;
  std::vector<void*> allocs_;
  std::vector<LayerDev> L_;
  DevWeight embd_;            // token_embd (logits GEMV + embedding rows)
  size_t embd_row_bytes_ = 0;
  const uint8_t* embd_raw_ = nullptr;  // GGUF-layout rows for embedding lookups
  float* out_norm_ = nullptr;
  float *rope_swa_ = nullptr, *rope_glb_ = nullptr;
  // activations
  float *resid2_ = nullptr, *resid_scratch_ = nullptr;
  unsigned* ticket_ = nullptr;
  float *resid_ = nullptr, *xn_ = nullptr, *qkv_ = nullptr, *q_ = nullptr, *attn_ = nullptr, *part_ = nullptr;
  float *o_out_ = nullptr, *gu_ = nullptr, *hid_ = nullptr, *d_out_ = nullptr, *logits_ = nullptr;
  ActBuf act_{};
  int32_t *d_token_ = nullptr, *d_pos_ = nullptr, *ring_ = nullptr, *ring_idx_ = nullptr;
  unsigned long long* amax_key_ = nullptr;
  int32_t* h_stage_ = nullptr;  // pinned: token, pos, ring_idx
  hipGraph_t graphs_[N_STEP_KINDS] = {};          // per step kind (ensure_graph)
  hipGraphExec_t graph_execs_[N_STEP_KINDS] = {};
  bool screen_ = false;                     // k_logits.hip: token ids by screening + exact rescoring
  ScreenTable scr_;
  bool rec_gen_ = false;       // record_step: this step ends with the screened token selection
  bool scr_prepped_ = false;   // the final norm wrote scr_.xs (no screen_prep launch)
  bool rec_fold_ = false;      // record_step(fold_embed): record_logits ends with finalize + embed_norm
  void screen_norm(NormOut& o);  // the final norm also writes the screening's x16 blocks where they will be used
  int kernels_per_token_ = 0;
  std::string dup_;
  size_t weight_bytes_ = 0;
  // row-sharded tensor parallelism; tp_ = false and G = 1
  // for a whole-model session.  This rank owns q heads [rank*nh_, +nh_),
  // kv heads [kv0_, +nkv_), o/down rows [rank*e_sh_, +e_sh_), hidden units
  // [rank*f_sh_, +f_sh_) and vocabulary rows [rank*v_sh_, +v_rows_)
  bool tp_ = false;
  int tp_rank_ = 0, tp_size_ = 1;
  std::unique_ptr<Collective> coll_;
  int nh_ = 0, nkv_ = 0, kv0_ = 0, e_sh_ = 0, f_sh_ = 0, v_sh_ = 0, v_rows_ = 0;
  bool tp_rep_attn_ = false;  // tensor parallel: qkv + attention replicated on every rank (setup_tp)
  // fused exchanges (px.h): the producing launches push, the consuming ones read their mailbox -- push-exchange
  // collectives, the fused layer path, no dumps / traces (LLMI_TP_FUSED=0: standalone exchange launches)
  int xa_vt_stride_ = 0;  // exact-order engine: keys per kv head of the tiled V caches (max_ctx rounded up to 32)
  bool px_fused_ = false;
  PxLink* d_px_ = nullptr;  // the device-resident link (px_prepare, before the first recorded step)
  int px_k_ = 0;            // fused exchanges recorded since the last standalone one
  void px_prepare();
  bool px_on() const { return px_fused_ && d_px_ && !dump_ && !trace_fn_; }
  int px_take() {  // the skip of a standalone exchange recorded now (its tag follows the fused ones)
    const int k = px_k_;
    px_k_ = 0;
    return k;
  }
  DevWeight logits_w_;  // the logits GEMV's rows: embd_ itself, or this rank's slice
  bool own_logits_w_ = false;
  // batched prefill (fast fused path, one device): chunk buffers
  bool prefill_ok_ = false;
  int pf_cap_ = 0, pf_xs_ = 0, pf_ostride_ = 0;
  int32_t* pf_tokens_ = nullptr;
  float *pf_resid_ = nullptr, *pf_out_ = nullptr;
  XBlock* pf_xq_ = nullptr;
  uint16_t* pf_x16_ = nullptr;  // f16 prefill activations [cap][pf_xs_ * 32]: dequantized Q8_0 blocks x 2^-s (v7 / v6)
  float* pf_tscale_ = nullptr;  // [cap] 2^s per token of pf_x16_ (the GEMMs' output scale)
  int T_cur_ = 0;              // tokens of the prefill chunk being enqueued
  int pf_f16_redo_ = 0;        // f16 prefills whose activations overflowed f16 and were recomputed on the int8 path
  bool pf_kq_ = false;         // K-quant layers: the batched prefill runs the f16 path
  uint16_t* pf_q_ = nullptr;
  float* pf_apart_ = nullptr;  // prefill attention: key-split partials
  int pf_attn_ks_ = 4;
  uint8_t* pf_gather_ = nullptr;  // tensor parallel: all-gather staging of the prefill slices
};

}  // namespace llmi
