// session.cpp -- the Gemma-3 forward of Model::forward (model.cpp:706-1049)
// resident on one MI355X.  Weights are parsed from the caller's GGUF bytes
// (loader semantics of gguf.cpp / model.cpp:58-238) and uploaded once; each
// token is one replay of a captured hipGraph whose kernels read the token id
// and position from device memory, so a greedy decode never returns to the
// host between tokens.
#include "session.h"

#include <cmath>
#include <functional>
#include <cstdio>
#include <cstring>

namespace llmi {

static int meta_u32(const GGUFView& g, const std::string& k, bool required, int dflt = 0) {
  const GValue* v = g.find(k);
  if (!v) {
    if (required) throw status_error(LLMI_E_GGUF, "Failed to find metadata key: " + k);  // model.cpp:64-66
    return dflt;
  }
  return (int)v->u32;
}

void Session::load_hparams(const GGUFView& g) {  // model.cpp:58-167
  const GValue* a = g.find("general.architecture");
  if (!a) throw status_error(LLMI_E_GGUF, "Failed to find metadata key: general.architecture");
  hp_.arch = a->str;
  const std::string p = hp_.arch + ".";
  hp_.n_layer = meta_u32(g, p + "block_count", true);
  hp_.n_embd = meta_u32(g, p + "embedding_length", true);
  hp_.n_ff = meta_u32(g, p + "feed_forward_length", true);
  hp_.n_head = meta_u32(g, p + "attention.head_count", true);
  hp_.n_head_kv = meta_u32(g, p + "attention.head_count_kv", true);
  const GValue* eps = g.find(p + "attention.layer_norm_rms_epsilon");
  const GValue* rb = g.find(p + "rope.freq_base");
  if (!eps) throw status_error(LLMI_E_GGUF, "Failed to find metadata key: " + p + "attention.layer_norm_rms_epsilon");
  if (!rb) throw status_error(LLMI_E_GGUF, "Failed to find metadata key: " + p + "rope.freq_base");
  hp_.eps = (double)eps->f32();  // f32 metadata widened to double (model.cpp:84-85)
  hp_.rope_base = rb->f32();
  hp_.rope_scale = 1.0f;         // model.cpp:87-92
  hp_.hd_k = meta_u32(g, p + "attention.key_length", false, hp_.n_embd / hp_.n_head);
  hp_.hd_k_swa = meta_u32(g, p + "attention.key_length_swa", false, hp_.hd_k);
  hp_.hd_v = meta_u32(g, p + "attention.value_length", false, hp_.hd_k);
  hp_.hd_v_swa = meta_u32(g, p + "attention.value_length_swa", false, hp_.hd_v);
  hp_.attn_scale = 1.0f / std::sqrt(float(hp_.hd_k));  // model.cpp:120
  if (const GValue* sw = g.find(p + "attention.sliding_window_pattern"))
    for (const auto& v : sw->arr) hp_.swa_layers.push_back((v.u32 & 0xFF) != 0);
  if (const GValue* v = g.find(p + "attention.logit_softcapping")) hp_.attn_softcap = v->f32();
  // ALiBi (model.cpp:125-128, 492-518): no Gemma file sets it, and the reference's bias term
  // slope * (t_k - (pos + t)) is evaluated in uint32_t (a wrapped, huge positive bias); refused, never ignored
  if (const GValue* v = g.find(p + "attention.max_alibi_bias"))
    if (v->f32() > 0.0f) throw status_error(LLMI_E_GGUF, "unsupported: " + p + "attention.max_alibi_bias");
  if (const GValue* v = g.find(p + "attention.final_logit_softcapping")) hp_.final_softcap = v->f32();
  // Gemma-4 (model.cpp:119-122, 148-166): attention scale 1, per-layer
  // embedding width, the first layer that reads an earlier layer's cache
  hp_.gemma4 = hp_.arch == "gemma4";
  if (hp_.gemma4) hp_.attn_scale = 1.0f;
  const GValue* epl = g.find(p + "embedding_length_per_layer");
  if (!epl) epl = g.find(p + "embedding_length_per_layer_input");
  hp_.n_epl = epl ? (int)epl->u32 : 0;
  if (const GValue* sk = g.find(p + "attention.shared_kv_layers")) hp_.kv_from = hp_.n_layer - (int)sk->u32;
  if (hp_.gemma4 || hp_.kv_from >= 0 || hp_.n_epl > 0) fuse_layers_ = false;  // Gemma-3 launch tables only
  if (hp_.hd_k != hp_.hd_v || hp_.hd_k_swa != hp_.hd_v_swa)
    throw status_error(LLMI_E_GGUF, "key_length != value_length is not supported");
  if (hp_.n_head % hp_.n_head_kv) throw status_error(LLMI_E_GGUF, "head_count % head_count_kv != 0");
}

float* Session::dev_f32_copy(const GGUFView& g, const GTensor* t, int n) {
  if (!t) return nullptr;
  if (t->type != T_F32) throw status_error(LLMI_E_TYPE, "norm weight " + t->name + " is not F32");
  if ((int)t->shape[0] < n) throw status_error(LLMI_E_SIZE, "norm weight " + t->name + " too short");
  float* d = dalloc<float>(t->shape[0] + 256);  // + 1 KB of slack past the vector
  h2d(d, g.tensor_data(*t), t->shape[0] * 4);
  return d;
}

// rows [r0, r0 + n) of one GGUF weight
struct RowSlice {
  const GTensor* t;
  int r0, n;
};
// LLMI_PREFILL_F16: unset -1 (the f16 prefill for Q4_0 layers on one device, GEMM v7), "0" off (the int8 GEMM v5
// everywhere), "1" on (K-quant layers too, GEMM v6)
static int prefill_f16_env() {
  const char* e = getenv("LLMI_PREFILL_F16");
  return e ? (e[0] == '1' ? 1 : 0) : -1;
}

static RowSlice all_rows(const GTensor* t) { return RowSlice{t, 0, (int)t->shape[1]}; }
static const void* slice_data(const GGUFView& g, const RowSlice& r) {
  return (const uint8_t*)g.tensor_data(*r.t) + gguf_bytes(r.t->type, r.r0, (int)r.t->shape[0]);
}

// one GEMV part per slice, or a fused part when every slice shares type/cols
static std::vector<GemvPart> make_parts(const GGUFView& g, const std::vector<RowSlice>& ts, hipStream_t s,
                                        size_t& wbytes) {
  std::vector<GemvPart> parts;
  bool same = true;
  for (auto& r : ts) same &= r.t->type == ts[0].t->type && r.t->shape[0] == ts[0].t->shape[0];
  auto check = [](const GTensor* t) {
    if (!gemv_type_supported(t->type))
      throw status_error(LLMI_E_TYPE, "mat_vec_mul: unsupported tensor type " + std::to_string(t->type));
  };
  if (same) {
    int rows = 0;
    for (auto& r : ts) { check(r.t); rows += r.n; }
    GemvPart p;
    p.w = alloc_weight(ts[0].t->type, rows, (int)ts[0].t->shape[0]);
    int r0 = 0;
    for (auto& r : ts) {
      upload_rows(p.w, r0, slice_data(g, r), r.n, s);
      r0 += r.n;
    }
    wbytes += p.w.bytes;
    parts.push_back(p);
  } else {
    // runs of consecutive slices sharing type and width become one part
    // (Q4_K_M: q|k Q4_K in one launch, v Q6_K in another)
    int off = 0;
    for (size_t i = 0; i < ts.size();) {
      size_t j = i + 1;
      while (j < ts.size() && ts[j].t->type == ts[i].t->type && ts[j].t->shape[0] == ts[i].t->shape[0]) j++;
      int rows = 0;
      for (size_t k = i; k < j; k++) { check(ts[k].t); rows += ts[k].n; }
      GemvPart p;
      p.w = alloc_weight(ts[i].t->type, rows, (int)ts[i].t->shape[0]);
      int r0 = 0;
      for (size_t k = i; k < j; k++) {
        upload_rows(p.w, r0, slice_data(g, ts[k]), ts[k].n, s);
        r0 += ts[k].n;
      }
      p.out_off = off;
      off += rows;
      wbytes += p.w.bytes;
      parts.push_back(p);
      i = j;
    }
  }
  return parts;
}

// Row shards of a tensor-parallel rank.  q heads split
// evenly; kv heads split evenly when they divide, else each rank keeps the one
// kv head its q heads read (replicated K/V rows, as the reference's GQA
// mapping head / (n_head / n_head_kv), model.cpp:478-550, requires).
void Session::setup_tp() {
  const int G = tp_size_, r = tp_rank_;
  if (hp_.n_embd % G || hp_.n_ff % G)
    throw status_error(LLMI_E_ARG, "tensor parallel: embedding_length / feed_forward_length % tp_size != 0");
  e_sh_ = hp_.n_embd / G;
  f_sh_ = hp_.n_ff / G;
  // Two modes, chosen per model (LLMI_TP_HEAD_SHARD=0 / 1 forces one):
  //  replicated: the q|k|v projection and the attention on every rank (all heads, the whole KV cache),
  //    o / gate_up / down row-sharded -- three all-gathers per layer instead of four, and the attention
  //    block (qkv + attention + the rank's o rows in one launch) on the ranks;
  //  head-sharded: the heads split as well (an all-gather of the heads' outputs before o).
  // Replicating costs every rank the whole q|k|v weight per layer.  Measured per-rank kernel time without the
  // exchange (profiles/r02_tp_solo.jsonl): 4B (n_embd 2560) replicated 0.97 / 0.93 / 0.91 ms vs head-sharded
  // 1.01 / 0.97 / 0.92 at tp 2 / 4 / 8; 27B (n_embd 5376, 24.8 MB of q|k|v per layer) 3.66 / 2.90 / 2.79 vs
  // 3.37 / 2.45 / 2.32.  So the heads are sharded by default for the wide models whose kv heads divide
  // evenly over the ranks (n_embd >= 4096: 12B, 27B), replicated otherwise.
  const char* hs = getenv("LLMI_TP_HEAD_SHARD");
  const bool wide = hp_.n_embd >= 4096 && hp_.n_head % G == 0 && hp_.n_head_kv % G == 0;
  tp_rep_attn_ = hs ? atoi(hs) == 0 : !wide;
  // exact mode: the exact-order engine's attention runs every head on every rank (its two launches read the whole
  // q|k|v row set); o, gate/up and down are row-sharded -- each row's accumulator chains are the whole model's
  if (exact_) {
    if (tp_ && hs && atoi(hs) != 0) throw status_error(LLMI_E_ARG, "tensor parallel exact mode: heads are not sharded");
    tp_rep_attn_ = true;
  }
  if (tp_rep_attn_) {
    nh_ = hp_.n_head;
    nkv_ = hp_.n_head_kv;
    kv0_ = 0;
    return;
  }
  if (hp_.n_head % G) throw status_error(LLMI_E_ARG, "tensor parallel: head_count % tp_size != 0");
  nh_ = hp_.n_head / G;
  const int grp = hp_.n_head / hp_.n_head_kv;
  if (hp_.n_head_kv % G == 0) {
    nkv_ = hp_.n_head_kv / G;
    kv0_ = r * nkv_;
  } else if (grp % nh_ == 0) {
    nkv_ = 1;
    kv0_ = r * nh_ / grp;
  } else {
    throw status_error(LLMI_E_ARG, "tensor parallel: q heads of a rank span several kv heads");
  }
}

void Session::upload(const GGUFView& g) {  // model.cpp:169-238 tensor map
  const GTensor* te = g.tensor("token_embd.weight");
  const GTensor* on = g.tensor("output_norm.weight");
  if (!te || !on) throw status_error(LLMI_E_GGUF, "missing token_embd.weight / output_norm.weight");
  vocab_ = (int)te->shape[1];
  if ((int)te->shape[0] != hp_.n_embd) throw status_error(LLMI_E_SIZE, "token_embd width != embedding_length");
  // embed_tokens supports F16/Q6_K/Q8_0/Q5_0 (model.cpp:247-331), the logits
  // path F16/Q6_K/Q4_K/Q8_0/Q5_0 (model.cpp:999-1034): the intersection
  if (te->type != T_F16 && te->type != T_Q6_K && te->type != T_Q8_0 && te->type != T_Q5_0)
    throw status_error(LLMI_E_TYPE, "Error: embed_tokens: Unsupported token embedding tensor type: " +
                                        std::to_string(te->type));
  embd_ = alloc_weight(te->type, vocab_, hp_.n_embd);
  upload_rows(embd_, 0, g.tensor_data(*te), vocab_, stream_);
  embd_row_bytes_ = gguf_bytes(te->type, 1, hp_.n_embd);
  embd_raw_ = (const uint8_t*)embd_.qs;
  if (te->type == T_Q8_0) {  // the GEMV copy is repacked; keep GGUF rows for lookups
    uint8_t* raw = dalloc<uint8_t>(embd_.bytes);
    h2d(raw, g.tensor_data(*te), embd_.bytes);
    embd_raw_ = raw;
  }
  weight_bytes_ += embd_.bytes;
  v_sh_ = (vocab_ + tp_size_ - 1) / tp_size_;
  v_rows_ = std::min(v_sh_, vocab_ - tp_rank_ * v_sh_);
  if (v_rows_ <= 0) throw status_error(LLMI_E_ARG, "tensor parallel: tp_size > vocabulary rows");
  if (tp_) {  // this rank's vocabulary rows for the logits GEMV (embd_ stays whole for lookups)
    logits_w_ = alloc_weight(te->type, v_rows_, hp_.n_embd);
    upload_rows(logits_w_, 0, slice_data(g, RowSlice{te, tp_rank_ * v_sh_, v_rows_}), v_rows_, stream_);
    own_logits_w_ = true;
    weight_bytes_ += logits_w_.bytes;
  } else {
    logits_w_ = embd_;
  }
  out_norm_ = dev_f32_copy(g, on, hp_.n_embd);
  // Gemma-4 per-layer token embeddings (model.cpp:178-188, 568-704)
  const GTensor* pt = g.tensor("token_embd_per_layer.weight");
  if (!pt) pt = g.tensor("per_layer_token_embd.weight");
  if (pt) {
    if (tp_) throw status_error(LLMI_E_ARG, "tensor parallel: per-layer embeddings are not supported");
    const int row_el = hp_.n_epl * hp_.n_layer;
    if (pt->type != T_F16 && pt->type != T_Q6_K && pt->type != T_Q4_K)
      throw status_error(LLMI_E_TYPE, "Error: get_per_layer_inputs: Unsupported tensor type: " +
                                          std::to_string(pt->type));
    if (hp_.n_epl <= 0 || (int)pt->shape[0] != row_el || (int)pt->shape[1] < vocab_)
      throw status_error(LLMI_E_SIZE, "per-layer token embedding shape != [n_epl * n_layer, vocab]");
    ple_table_.type = pt->type;
    ple_table_.rows = (int)pt->shape[1];
    ple_table_.cols = row_el;
    ple_row_bytes_ = gguf_bytes(pt->type, 1, row_el);
    ple_table_.bytes = ple_row_bytes_ * pt->shape[1];
    uint8_t* raw = dalloc<uint8_t>(ple_table_.bytes);
    h2d(raw, g.tensor_data(*pt), ple_table_.bytes);
    ple_table_.qs = raw;
    if (const GTensor* mp = g.tensor("per_layer_model_proj.weight")) {
      if ((int)mp->shape[0] != hp_.n_embd || (int)mp->shape[1] != row_el)
        throw status_error(LLMI_E_SIZE, "per_layer_model_proj shape != [n_embd, n_epl * n_layer]");
      ple_model_proj_ = make_parts(g, {all_rows(mp)}, stream_, weight_bytes_);
      const GTensor* pn = g.tensor("per_layer_proj_norm.weight");
      if (!pn) throw status_error(LLMI_E_GGUF, "missing per_layer_proj_norm.weight");
      ple_proj_norm_ = dev_f32_copy(g, pn, hp_.n_epl);
    }
  }
  L_.resize(hp_.n_layer);
  for (int l = 0; l < hp_.n_layer; l++) {
    auto T = [&](const char* n, bool req = true) -> const GTensor* {
      const std::string name = "blk." + std::to_string(l) + "." + n;
      const GTensor* t = g.tensor(name);
      if (!t && req) throw status_error(LLMI_E_GGUF, "missing tensor " + name);
      return t;
    };
    auto T2 = [&](const char* a, const char* b) { const GTensor* t = T(a, false); return t ? t : T(b, false); };
    LayerDev& Ld = L_[l];
    Ld.is_swa = l < (int)hp_.swa_layers.size() ? hp_.swa_layers[l] : (l % 6 < 5);  // model.cpp:723-729
    Ld.hd = Ld.is_swa ? hp_.hd_k_swa : hp_.hd_k;
    // shared KV (model.cpp:775-777, 832-835): no K/V projections; the cache of
    // layer kv_from - 2 (SWA) or kv_from - 1 (global) is read instead
    Ld.has_kv = hp_.kv_from < 0 || l < hp_.kv_from;
    if (!Ld.has_kv) {
      if (tp_) throw status_error(LLMI_E_ARG, "tensor parallel: shared-KV layers are not supported");
      Ld.kv_src = hp_.kv_from - (Ld.is_swa ? 2 : 1);
      if (Ld.kv_src < 0 || Ld.kv_src >= l || !L_[Ld.kv_src].has_kv || L_[Ld.kv_src].is_swa != Ld.is_swa)
        throw status_error(LLMI_E_GGUF, "shared-KV layer " + std::to_string(l) + " reads layer " +
                                            std::to_string(Ld.kv_src) + " (no cache of the same attention kind)");
    }
    const GTensor* q = T("attn_q.weight");
    const GTensor* k = Ld.has_kv ? T("attn_k.weight") : nullptr;
    const GTensor* v = Ld.has_kv ? T("attn_v.weight") : nullptr;
    if ((int)q->shape[1] < hp_.n_head * Ld.hd ||
        (Ld.has_kv && ((int)k->shape[1] < hp_.n_head_kv * Ld.hd || (int)v->shape[1] < hp_.n_head_kv * Ld.hd)))
      throw status_error(LLMI_E_SIZE, "attention projection rows < heads * head_dim");
    const int hd = Ld.hd, r = tp_rank_;
    const std::vector<RowSlice> qkv_rows =
        !Ld.has_kv ? std::vector<RowSlice>{all_rows(q)}
        : tp_ && !tp_rep_attn_ ? std::vector<RowSlice>{{q, r * nh_ * hd, nh_ * hd}, {k, kv0_ * hd, nkv_ * hd}, {v, kv0_ * hd, nkv_ * hd}}
              : std::vector<RowSlice>{all_rows(q), all_rows(k), all_rows(v)};
    Ld.qkv = make_parts(g, qkv_rows, stream_, weight_bytes_);
    Ld.k_off = qkv_rows[0].n;
    Ld.v_off = Ld.has_kv ? qkv_rows[0].n + qkv_rows[1].n : qkv_rows[0].n;
    Ld.qkv_rows = 0;
    for (const auto& rs : qkv_rows) Ld.qkv_rows += rs.n;
    const GTensor* o = T("attn_output.weight");
    if ((int)o->shape[0] != hp_.n_head * Ld.hd || (int)o->shape[1] != hp_.n_embd)
      throw status_error(LLMI_E_SIZE, "mat_vec_mul_q4_0: input vector size mismatch (attn_output)");
    const RowSlice o_rows = tp_ ? RowSlice{o, r * e_sh_, e_sh_} : all_rows(o);
    Ld.o = make_parts(g, {o_rows}, stream_, weight_bytes_)[0];
    const GTensor *gt = T("ffn_gate.weight"), *up = T("ffn_up.weight"), *dn = T("ffn_down.weight");
    if ((int)gt->shape[1] != hp_.n_ff || (int)up->shape[1] != hp_.n_ff || (int)dn->shape[0] != hp_.n_ff)
      throw status_error(LLMI_E_SIZE, "ffn shapes do not match feed_forward_length");
    // the fused layer path (k_layer.hip) needs every projection in its launch
    // table; decided from the GGUF shapes before upload because it changes
    // the gate/up row order
    auto slab_of = [](const GTensor* t, int role) {
      DevWeight w;
      w.type = t->type;
      w.cols = (int)t->shape[0];
      return layer_gemv_slab(w, role);
    };
    auto shape_ok = [](const GTensor* t, int rows, int role) {
      DevWeight w;
      w.type = t->type;
      w.rows = rows;
      w.cols = (int)t->shape[0];
      return layer_gemv_supported(w, role);
    };
    const bool qkv_same = Ld.has_kv && q->type == k->type && q->type == v->type && q->shape[0] == k->shape[0] &&
                          q->shape[0] == v->shape[0];
    bool want_fused =
        fuse_layers_ && qkv_same && (gt->type == T_Q4_0 || gt->type == T_Q8_0) && up->type == gt->type &&
        gt->shape[0] == up->shape[0] &&
        (int)q->shape[0] == hp_.n_embd && (int)gt->shape[0] == hp_.n_embd &&
        shape_ok(q, Ld.qkv_rows, LAYER_PRO) && shape_ok(q, Ld.qkv_rows, LAYER_PLAIN) &&
        slab_of(q, LAYER_PRO) == slab_of(q, LAYER_PLAIN) &&  // one qkv layout serves both roles
        shape_ok(o, o_rows.n, LAYER_PLAIN) && shape_ok(gt, 2 * (tp_ ? f_sh_ : hp_.n_ff), LAYER_GELU) &&
        shape_ok(dn, tp_ ? e_sh_ : (int)dn->shape[1], LAYER_QUANT);
    // K-quant layers (Q4_K_M: q, k, o, gate, up Q4_K; v, down Q6_K or Q4_K) in the kq launch table,
    // one device: q|k and v in one launch when v is Q6_K
    auto kq_t = [](const GTensor* t) { return t && (t->type == T_Q4_K || t->type == T_Q6_K); };
    bool kq_path = fuse_layers_ && !tp_ && Ld.has_kv && q->type == T_Q4_K && k->type == T_Q4_K && kq_t(v) &&
                   kq_t(o) && kq_t(gt) && up->type == gt->type && kq_t(dn) && q->shape[0] == k->shape[0] &&
                   q->shape[0] == v->shape[0] && (int)q->shape[0] == hp_.n_embd && (int)gt->shape[0] == hp_.n_embd &&
                   shape_ok(o, o_rows.n, LAYER_PLAIN) && shape_ok(gt, 2 * hp_.n_ff, LAYER_GELU) &&
                   shape_ok(dn, (int)dn->shape[1], LAYER_QUANT) && (hp_.n_head * Ld.hd) % 256 == 0;
    if (kq_path) {
      if (v->type == T_Q4_K) {
        kq_path = shape_ok(q, Ld.qkv_rows, LAYER_PRO) && shape_ok(q, Ld.qkv_rows, LAYER_PLAIN);
      } else {
        DevWeight wa, wb;
        wa.type = T_Q4_K;
        wa.rows = qkv_rows[0].n + qkv_rows[1].n;
        wa.cols = (int)q->shape[0];
        wb.type = T_Q6_K;
        wb.rows = qkv_rows[2].n;
        wb.cols = wa.cols;
        kq_path = layer_gemv2_supported(wa, wb, LAYER_PRO) && layer_gemv2_supported(wa, wb, LAYER_PLAIN);
      }
    }
    want_fused = want_fused || kq_path;
    if (tp_ && !want_fused && !exact_)
      throw status_error(LLMI_E_ARG, "tensor parallel: layer " + std::to_string(l) +
                                         " shards are not in the fused Q4_0 launch table");
    if (want_fused) {
      // rows interleaved in groups of H (gate H k.., up H k..) for the fused
      // GELU epilogue of gemv_q4_0_layer (k_layer.hip): a work-group of 2H
      // rows owns matching gate and up rows.  A tensor-parallel rank keeps
      // hidden units [rank * F, (rank + 1) * F).
      const int cols = (int)gt->shape[0], F = tp_ ? f_sh_ : hp_.n_ff;
      const int H = layer_gemv_gelu_group(cols, gt->type);
      const size_t rb = gguf_bytes(gt->type, 1, cols);
      std::vector<uint8_t> il((size_t)2 * F * rb);
      const size_t h0 = (size_t)r * F * rb;
      const uint8_t *sg = (const uint8_t*)g.tensor_data(*gt) + h0, *su = (const uint8_t*)g.tensor_data(*up) + h0;
      for (int k = 0; k < F / H; k++) {
        std::memcpy(&il[(size_t)(2 * H * k) * rb], sg + (size_t)(H * k) * rb, H * rb);
        std::memcpy(&il[(size_t)(2 * H * k + H) * rb], su + (size_t)(H * k) * rb, H * rb);
      }
      GemvPart p;
      p.w = alloc_weight(gt->type, 2 * F, cols);
      upload_rows(p.w, 0, il.data(), 2 * F, stream_);
      weight_bytes_ += p.w.bytes;
      Ld.gate_up = {p};
      Ld.gu_interleaved = true;
    } else if (tp_) {  // (exact mode) this rank's hidden units of gate and of up
      Ld.gate_up = make_parts(g, {RowSlice{gt, r * f_sh_, f_sh_}, RowSlice{up, r * f_sh_, f_sh_}}, stream_, weight_bytes_);
    } else {
      Ld.gate_up = make_parts(g, {all_rows(gt), all_rows(up)}, stream_, weight_bytes_);
    }
    Ld.down = make_parts(g, {tp_ ? RowSlice{dn, r * e_sh_, e_sh_} : all_rows(dn)}, stream_, weight_bytes_)[0];
    const bool qkv_ok =
        Ld.qkv.size() == 1 ? layer_gemv_supported(Ld.qkv[0].w, LAYER_PRO) && layer_gemv_supported(Ld.qkv[0].w, LAYER_PLAIN)
        : Ld.qkv.size() == 2 && layer_gemv2_supported(Ld.qkv[0].w, Ld.qkv[1].w, LAYER_PRO) &&
              layer_gemv2_supported(Ld.qkv[0].w, Ld.qkv[1].w, LAYER_PLAIN);
    Ld.fused = Ld.gu_interleaved && qkv_ok && layer_gemv_supported(Ld.o.w, LAYER_PLAIN) &&
               layer_gemv_supported(Ld.gate_up[0].w, LAYER_GELU) && layer_gemv_supported(Ld.down.w, LAYER_QUANT);
    Ld.attn_norm = dev_f32_copy(g, T("attn_norm.weight"), hp_.n_embd);
    Ld.q_norm = dev_f32_copy(g, T("attn_q_norm.weight"), Ld.hd);
    Ld.k_norm = Ld.has_kv ? dev_f32_copy(g, T("attn_k_norm.weight"), Ld.hd) : nullptr;
    Ld.ffn_norm = dev_f32_copy(g, T("ffn_norm.weight"), hp_.n_embd);
    Ld.post_attn_norm = dev_f32_copy(g, T2("post_attention_norm.weight", "attn_post_norm.weight"), hp_.n_embd);
    Ld.post_ffw_norm = dev_f32_copy(g, T2("post_ffw_norm.weight", "ffn_post_norm.weight"), hp_.n_embd);
    if (Ld.has_kv) {
      const size_t kv = (size_t)nkv_ * max_ctx_ * Ld.hd;
      Ld.kc = dalloc<uint16_t>(kv);
      Ld.vc = dalloc<uint16_t>(kv);
    } else {
      Ld.kc = L_[Ld.kv_src].kc;
      Ld.vc = L_[Ld.kv_src].vc;
    }
    // Gemma-4 per-layer embedding step and output scale (model.cpp:215-233, 926-977)
    if (ple_table_.qs) {
      const GTensor* pg = T2("per_layer_inp_gate.weight", "inp_gate.weight");
      const GTensor* pp = T2("per_layer_proj.weight", "proj.weight");
      const GTensor* pn = T2("per_layer_post_norm.weight", "post_norm.weight");
      if (!pg || !pp || !pn) throw status_error(LLMI_E_GGUF, "missing per-layer embedding tensors in layer " + std::to_string(l));
      if ((int)pg->shape[0] != hp_.n_embd || (int)pg->shape[1] != hp_.n_epl || (int)pp->shape[0] != hp_.n_epl ||
          (int)pp->shape[1] != hp_.n_embd)
        throw status_error(LLMI_E_SIZE, "per-layer embedding projection shapes in layer " + std::to_string(l));
      Ld.ple_gate = make_parts(g, {all_rows(pg)}, stream_, weight_bytes_)[0];
      Ld.ple_proj = make_parts(g, {all_rows(pp)}, stream_, weight_bytes_)[0];
      Ld.ple_post_norm = dev_f32_copy(g, pn, hp_.n_embd);
    }
    if (const GTensor* os = T2("out_scale.weight", "layer_output_scale.weight")) {
      if (os->type != T_F32) throw status_error(LLMI_E_TYPE, "layer output scale is not F32");
      std::memcpy(&Ld.out_scale, g.tensor_data(*os), 4);
    }
  }
  // The fused path runs only when EVERY layer fits it; otherwise the layers
  // that were prepared for it go back to the plain gate/up order.
  bool all_fused = fuse_layers_;
  for (const auto& Ld : L_) all_fused &= Ld.fused;
  for (int l = 0; l < hp_.n_layer && !all_fused; l++) {
    LayerDev& Ld = L_[l];
    Ld.fused = false;
    if (!Ld.gu_interleaved) continue;
    const std::string b = "blk." + std::to_string(l) + ".";
    for (auto& p : Ld.gate_up) {
      weight_bytes_ -= p.w.bytes;
      free_weight(p.w);
    }
    Ld.gate_up = make_parts(g, {all_rows(g.tensor(b + "ffn_gate.weight")), all_rows(g.tensor(b + "ffn_up.weight"))},
                            stream_, weight_bytes_);
    Ld.gu_interleaved = false;
  }
  if (all_fused) {  // the weight layouts the fused launch-table entries read
    auto relayout = [&](DevWeight& w, int role) {
      if (w.type == T_Q4_K || w.type == T_Q6_K) to_kq_layout(w, stream_, layer_gemv_slab(w, role));
      else if (layer_gemv_slab(w, role)) to_slab_layout(w, stream_);
    };
    for (auto& Ld : L_) {
      for (auto& p : Ld.qkv) relayout(p.w, LAYER_PRO);
      relayout(Ld.o.w, LAYER_PLAIN);
      relayout(Ld.gate_up[0].w, LAYER_GELU);
      relayout(Ld.down.w, LAYER_QUANT);
    }
  }
}

void Session::alloc_buffers() {
  const int E = hp_.n_embd, F = hp_.n_ff;
  int maxq = 0, maxqkv = 0, maxhd = 0;
  for (auto& l : L_) {
    maxq = std::max(maxq, hp_.n_head * l.hd);
    maxqkv = std::max(maxqkv, l.qkv_rows);
    maxhd = std::max(maxhd, l.hd);
  }
  const int maxcols = std::max({E, F, maxq, vocab_ > 0 ? E : 0});
  resid_ = dalloc<float>(E);
  resid2_ = dalloc<float>(E);
  resid_scratch_ = dalloc<float>(E);
  xn_ = dalloc<float>(E);
  qkv_ = dalloc<float>(maxqkv);
  q_ = dalloc<float>(maxq);
  attn_ = dalloc<float>(maxq);
  part_ = dalloc<float>((size_t)hp_.n_head * ATTN_NSPLIT * (maxhd + 2));
  ticket_ = dalloc<unsigned>(hp_.n_head);  // per (virtual) kv head, zeroed; the attention kernel resets it after use
  o_out_ = dalloc<float>(E);
  gu_ = dalloc<float>(2 * (size_t)F);
  hid_ = dalloc<float>(F);
  hq_ = dalloc<XBlock>(F / 32 + 1);
  d_out_ = dalloc<float>(E);
  logits_ = dalloc<float>((size_t)tp_size_ * v_sh_);
  act_.q8.xb = dalloc<XBlock>(maxcols / 32 + 1);
  act_.q8.nb = maxcols / 32;
  act_.q8k = dalloc<uint8_t>((size_t)(maxcols / 256 + 1) * 292);
  act_.x16 = dalloc<uint16_t>(maxcols);
  d_token_ = dalloc<int32_t>(1);
  d_pos_ = dalloc<int32_t>(1);
  ring_ = dalloc<int32_t>(max_ctx_);
  ring_idx_ = dalloc<int32_t>(1);
  amax_key_ = dalloc<unsigned long long>(tp_size_);  // one argmax key per rank's vocabulary slice
  if (ple_table_.qs) {
    const size_t row_el = (size_t)hp_.n_epl * hp_.n_layer;
    inp_pl_ = dalloc<float>(row_el);
    ple_proj_out_ = dalloc<float>(row_el);
    ple_g_ = dalloc<float>(hp_.n_epl);
    ple_u_ = dalloc<float>(hp_.n_epl);
    ple_tmp_ = dalloc<float>(E);
  }
  LLMI_HIP(hipHostMalloc((void**)&h_stage_, 64, hipHostMallocDefault));
}

void Session::build_rope_tables() {
  // (cos, sin) of ((float)pos * freq_i) / freq_scale with freq_i =
  // 1/powf(base, (float)(2i)/n_rot), glibc on the host exactly like
  // ops.cpp:79-83; one table per rope base used by the layers.
  auto make = [&](float base, int hd) {
    const int half = hd / 2;
    std::vector<float> h((size_t)max_ctx_ * half * 2);
    for (int i = 0; i < half; i++) {
      const float freq = 1.0f / powf(base, (float)(2 * i) / (float)hd);
      for (int p = 0; p < max_ctx_; p++) {
        const float val = ((float)(uint32_t)p * freq) / hp_.rope_scale;
        h[((size_t)p * half + i) * 2] = cosf(val);
        h[((size_t)p * half + i) * 2 + 1] = sinf(val);
      }
    }
    float* d = dalloc<float>(h.size());
    h2d(d, h.data(), h.size() * 4);
    return d;
  };
  rope_swa_ = make(10000.0f, hp_.hd_k_swa);  // model.cpp:732
  rope_glb_ = make(hp_.rope_base, hp_.hd_k);
}

Session::Session(const uint8_t* gguf, size_t size, const llmi_session_opts& opts) : opts_(opts) {
  exact_ = (opts.flags & LLMI_EXACT) != 0;
  ex_gemv_ = ex_norm_ = ex_attn_ = ex_logits_ = exact_;
  if (const char* e = getenv("LLMI_EXACT_PARTS")) {  // diagnostics: mix exact/fast kernel families
    const std::string s(e);
    ex_gemv_ = s.find("gemv") != std::string::npos;
    ex_norm_ = s.find("norm") != std::string::npos;
    ex_attn_ = s.find("attn") != std::string::npos;
    ex_logits_ = s.find("logits") != std::string::npos;
  }
  fuse_layers_ = !ex_gemv_ && !ex_norm_ && getenv("LLMI_NO_FUSE") == nullptr;
  if (const char* d = getenv("LLMI_DUP")) dup_ = d;  // diagnostics: launch these kernels twice
  use_graph_ = (opts.flags & LLMI_NO_GRAPH) == 0;
  max_ctx_ = opts.max_ctx > 0 ? opts.max_ctx : 4096;
  if (opts.attn_split != 0 && opts.attn_split != ATTN_NSPLIT)
    throw status_error(LLMI_E_ARG, "attn_split must be 0 or " + std::to_string(ATTN_NSPLIT));
  // LLMI_TP_SOLO (diagnostics): rank tp_rank of tp_size alone, no exchange
  const bool tp_solo = getenv("LLMI_TP_SOLO") != nullptr && opts.tp_size > 1 && !opts.tp_id && !opts.tp_group;
  const bool tp_peer = (opts.flags & LLMI_TP_PEER) != 0 && !opts.tp_id && !opts.tp_group && !tp_solo;
  tp_ = opts.tp_id != nullptr || opts.tp_group != nullptr || tp_solo || tp_peer;
  if (tp_) {
    tp_rank_ = opts.tp_rank;
    tp_size_ = opts.tp_size;
    if (tp_size_ < 1 || tp_rank_ < 0 || tp_rank_ >= tp_size_)
      throw status_error(LLMI_E_ARG, "tensor parallel: tp_rank / tp_size out of range");
    // the fused fast path, or exact mode on the exact-order engine (rows sharded, the chains of each row kept)
    const bool exact_all = exact_ && ex_gemv_ && ex_norm_ && ex_attn_ && ex_logits_;
    if ((!fuse_layers_ && !exact_all) || !dup_.empty())
      throw status_error(LLMI_E_ARG, "tensor parallel needs the fused fast path or exact mode (no LLMI_NO_FUSE / "
                                     "LLMI_EXACT_PARTS / LLMI_DUP)");
  }
  LLMI_HIP(hipSetDevice(opts.device));
  session_live(+1);  // (release() ends it: every path out of here, normal or not, runs release())
  live_ = true;
  constructing_ = true;
  try {
    LLMI_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    if (tp_) {
      coll_ = tp_solo         ? make_null(tp_rank_, tp_size_)
              : opts.tp_group ? make_local(reinterpret_cast<LocalGroup*>(opts.tp_group), tp_rank_, tp_size_, stream_)
              : tp_peer       ? make_peer(tp_rank_, tp_size_, stream_)
                              : make_rccl(tp_rank_, tp_size_, opts.tp_id);
      if (!coll_->graph_safe()) use_graph_ = false;
      const char* fx = getenv("LLMI_TP_FUSED");
      px_fused_ = coll_->fused_capable() && !(fx && atoi(fx) == 0);
    }
    GGUFView g(gguf, size);
    load_hparams(g);
    setup_tp();
    upload(g);
    alloc_buffers();
    build_rope_tables();
    setup_xl();
    if (tp_ && exact_ && !xl_)
      throw status_error(LLMI_E_ARG, "tensor parallel exact mode needs the exact-order engine (Q4_0 Gemma-3 layers, "
                                     "hidden units per rank % 32 == 0, embedding rows per rank % 16 == 0)");
    // batched prefill: the fast fused layout on one device, shapes the
    // prefill kernels cover (otherwise forward() runs the token loop)
    // (a tensor-parallel rank: its shards' GEMMs, the slices all-gathered per
    // projection; Q8_0 block slices need 32-aligned head and hidden shards)
    bool pf = fuse_layers_ && (embd_.type == T_F16 || embd_.type == T_Q8_0) && hp_.n_embd <= 8192 &&
              hp_.n_embd % 32 == 0 && hp_.n_ff % 32 == 0 && (!tp_ || (f_sh_ % 32 == 0 && coll_));
    // Q4_0 layers: the f16 GEMM (v7, default on one device) or the int8 one (v5); Q8_0 layers: v5; K-quant (kq)
    // layers: v5 on Q8_K blocks, or the f16 GEMM v6 (LLMI_PREFILL_F16=1)
    auto q40 = [](const DevWeight& w) { return w.type == T_Q4_0 || w.type == T_Q8_0; };
    auto gemm_ok = [&](const DevWeight& w) {
      return prefill_gemm_supported(w) || (!q40(w) && prefill_f16_env() == 1 && prefill_gemm16_supported(w));
    };
    for (const auto& l : L_) {
      bool ok = l.fused && (l.hd == 64 || l.hd == 128 || l.hd == 256) && gemm_ok(l.o.w) && gemm_ok(l.gate_up[0].w) &&
                gemm_ok(l.down.w) && !l.qkv.empty();
      for (const auto& part : l.qkv) ok = ok && gemm_ok(part.w);
      bool kq = !q40(l.o.w) || !q40(l.gate_up[0].w) || !q40(l.down.w);
      for (const auto& part : l.qkv) kq = kq || !q40(part.w);
      if (ok && kq)  // 8-unit GELU writes; Q8_K blocks: whole super-blocks (a head of 256, 256-aligned rank slices)
        ok = layer_gemv_gelu_group(l.gate_up[0].w.cols, l.gate_up[0].w.type) % 8 == 0 &&
             (prefill_f16_env() == 1 ||
              (l.hd == 256 && hp_.n_embd % 256 == 0 && hp_.n_ff % 256 == 0 && (!tp_ || f_sh_ % 256 == 0)));
      pf = pf && ok;
      pf_kq_ = pf_kq_ || kq;
    }
    // K-quant layers: the int8 GEMM on Q8_K activation blocks (the decode's quantization); the f16 path
    // (LLMI_PREFILL_F16=1) is opt-in -- its f16 activations are further from the reference's Q8_K arithmetic
    // than the fast-mode budget
    const int grp = nkv_ > 0 ? nh_ / nkv_ : 0;
    prefill_ok_ = pf && (grp == 1 || grp == 2 || grp == 4);
    // attention block (qkv + attention + o in one launch): the fused fast
    // path on one device, shapes in k_attn.hip's table; LLMI_NO_BLOCK=1 keeps
    // the three launches (A/B)
    bool blk = fuse_layers_ && (!tp_ || tp_rep_attn_) && dup_.empty() && getenv("LLMI_NO_BLOCK") == nullptr &&
               (grp == 1 || grp == 2 || grp == 4);
    bool pro = true;
    for (const auto& l : L_) {
      const DevWeight* wb = l.qkv.size() > 1 ? &l.qkv[1].w : nullptr;
      blk = blk && l.fused && l.hd % 32 == 0 && attn_block_supported(l.qkv[0].w, wb, l.o.w, l.hd, nh_, nkv_, LAYER_PLAIN);
      pro = pro && attn_block_supported(l.qkv[0].w, wb, l.o.w, l.hd, nh_, nkv_, LAYER_PRO);
    }
    block_ = blk;
    // 27B: the 5376-wide residual/norm prologue does not fit the block's registers at a co-resident grid, so
    // launch_residual_norm runs first and the block's qkv role reads the Q8_0 blocks it wrote
    block_pro_ = blk && pro;
    // greedy token ids by screening (k_logits.hip): the fast F16 logits path
    // (a tensor-parallel rank screens its vocabulary shard; the keys meet in
    // finalize as before); LLMI_FULL_LOGITS=1 keeps the full GEMV in the loop
    // exact mode: the same screening, the candidates rescored in the reference's order
    screen_ = embd_.type == T_F16 && logits_w_.type == T_F16 && screen_supported(logits_w_) &&
              hp_.final_softcap <= 0.0f &&
              getenv("LLMI_FULL_LOGITS") == nullptr;
    if (screen_) alloc_screen_table(logits_w_, scr_, stream_);
    if (block_) {
      int maxrows = 0, maxhd0 = 0;
      for (const auto& l : L_) {
        maxrows = std::max(maxrows, l.qkv_rows);
        maxhd0 = std::max(maxhd0, l.hd);
      }
      blk_epoch_ = dalloc<unsigned>(hp_.n_layer);
      blk_done_ = dalloc<unsigned>((size_t)hp_.n_layer * 32);  // (a 128-B line per layer)
      blk_gqkv_stride_ = (size_t)maxrows;
      blk_gxo_stride_ = (size_t)nh_ * maxhd0 / 32 * 12;
      blk_gqkv_ = dalloc<uint2>((size_t)hp_.n_layer * blk_gqkv_stride_);
      blk_gxo_ = dalloc<uint2>((size_t)hp_.n_layer * blk_gxo_stride_);
      blk_err_ = dalloc<int>(2);
      if (const char* tr = getenv("LLMI_BLOCK_TRACE")) {  // development: per-work-group phase clocks of one layer
        blk_trace_layer_ = atoi(tr);
        blk_trace_ = dalloc<unsigned long long>(4096 * 8);
      }
      int maxhd = 0;
      for (const auto& l : L_) maxhd = std::max(maxhd, l.hd);
      blk_xo_ = dalloc<XBlock>((size_t)nh_ * maxhd / 32 + 1);
    }
    // the batched prefill's chunk buffers for a default-sized prompt now, not inside the first forward (the
    // allocations and their zeroing were ~3 ms of the first 512-token prefill: 14.3 vs 11.0 ms)
    if (prefill_ok_) ensure_prefill_buffers(std::min(512, max_ctx_));
    LLMI_HIP(hipStreamSynchronize(stream_));  // every zeroing and copy above complete before the first call
    // one two-token batched prefill at position 0 (one device): the first forward of a session paid ~3 ms more
    // than later ones (14.3 vs 11.2 ms for 512 tokens: the prefill kernels' first launches), now paid here; the
    // K / V rows it writes are rewritten by the first prompt (LLMI_NO_WARMUP=1: skip)
    if (prefill_ok_ && !tp_ && max_ctx_ >= 2 && getenv("LLMI_NO_WARMUP") == nullptr) {
      const int32_t warm[2] = {0, 0};
      set_token_pos(warm[1], 1, true);
      prefill(warm, 2, 0);
      // the f16 path's wide-tile GEMM (v7: gate_up at full chunks only) is not launched by two tokens: once more
      // over the whole chunk buffer into scratch (4B: ~80 us here instead of the first prompt's)
      if (prefill_f16_ok() && pf_cap_ > 256)
        for (const auto& part : L_[0].gate_up)
          launch_prefill_gemm16(part.w, pf_x16_, pf_xs_ * 32, pf_cap_, pf_out_, pf_ostride_, pf_tscale_, stream_);
      LLMI_HIP(hipStreamSynchronize(stream_));
    }
    constructing_ = false;
    session_constructed(true);
  } catch (const gguf_error& e) {
    release();
    throw status_error(LLMI_E_GGUF, e.what());
  } catch (...) {
    release();
    throw;
  }
}

Session::~Session() { release(); }

void Session::release() {
  // nothing of this session may still run when its graphs and memory go (a broken session's kernels may still be
  // spinning up to LLMI_PX_TIMEOUT_MS; enqueue() without sync() leaves work in flight): drain, errors ignored
  if (stream_) (void)hipStreamSynchronize(stream_);
  for (int k = 0; k < N_STEP_KINDS; k++) {
    if (graph_execs_[k]) (void)hipGraphExecDestroy(graph_execs_[k]);
    if (graphs_[k]) (void)hipGraphDestroy(graphs_[k]);
    graph_execs_[k] = nullptr;
    graphs_[k] = nullptr;
  }
  free_screen_table(scr_);
  for (auto& l : L_) {
    for (XlWeight* x : {&l.xqkv, &l.xo, &l.xgu, &l.xdn}) free_xl_weight(*x);
    for (auto& p : l.qkv) free_weight(p.w);
    for (auto& p : l.gate_up) free_weight(p.w);
    free_weight(l.o.w);
    free_weight(l.down.w);
    free_weight(l.ple_gate.w);
    free_weight(l.ple_proj.w);
  }
  L_.clear();
  for (auto& p : ple_model_proj_) free_weight(p.w);
  ple_model_proj_.clear();
  ple_table_ = DevWeight{};  // its bytes are an allocs_ entry
  if (own_logits_w_) free_weight(logits_w_);
  own_logits_w_ = false;
  free_weight(embd_);
  for (void* p : allocs_) dev_free(p);
  allocs_.clear();
  if (h_stage_) (void)hipHostFree(h_stage_);
  h_stage_ = nullptr;
  coll_.reset();
  if (stream_) (void)hipStreamDestroy(stream_);
  stream_ = nullptr;
  if (constructing_) session_constructed(false);
  constructing_ = false;
  if (live_) session_live(-1);
  live_ = false;
}

// Activation format each weight type consumes (ops.cpp:209-210, 630-631, 724-725, 542-551)
void Session::prepare_act(uint32_t wtype, const float* x, int n, ActBuf& act, hipStream_t s) {
  act.xf = x;
  switch (wtype) {
    case T_Q4_0: case T_Q8_0: launch_quantize_q8_0(x, n, act.q8, s); kernels_per_token_++; break;
    case T_Q4_K: case T_Q6_K: launch_quantize_q8_k(x, n, act.q8k, s); kernels_per_token_++; break;
    case T_F16: launch_round_f16(x, n, act.x16, s); kernels_per_token_++; break;
    default: break;  // Q5_0 / BF16 read f32 x directly
  }
}

void Session::gemv_parts(const std::vector<GemvPart>& parts, const float* x, int n_in, float* out, hipStream_t s,
                         bool x_ready) {
  uint32_t prepared = 0xFFFFFFFFu;
  for (const auto& p : parts) {
    const uint32_t kind = (p.w.type == T_Q8_0) ? T_Q4_0 : (p.w.type == T_Q6_K ? T_Q4_K : p.w.type);
    // x_ready: act_ already holds x in the format this kind reads (Q8_0 or Q8_K, the producer chose it)
    if (!(x_ready && (kind == T_Q4_0 || kind == T_Q4_K)) && kind != prepared) prepare_act(p.w.type, x, n_in, act_, s);
    act_.xf = x;
    prepared = kind;
    launch_gemv(p.w, act_, out + p.out_off, ex_gemv_ ? GEMV_EXACT : GEMV_FAST, s);
    kernels_per_token_++;
  }
}

// One decode token.  Reads *d_token_/*d_pos_, ends with the token feedback.
// the down projection as a PLAIN launch on the GELU launch's Q8_0 blocks: one device (a rank's hid slice is
// all-gathered as f32), 32 hidden units per GELU work-group, a PLAIN table entry for the shape
// (27B down 19.3 -> 14.5 us against the QUANT launch, profiles/r02_down_plain_ab.txt)
bool Session::down_plain(const LayerDev& Ld) const {
  const DevWeight& g = Ld.gate_up[0].w;
  // a tensor-parallel rank: its GELU blocks are all-gathered instead of its f32 hid (whole blocks per rank)
  return (!tp_ || f_sh_ % 32 == 0) && (Ld.down.w.type == T_Q4_0 || Ld.down.w.type == T_Q8_0) &&
         layer_gemv_gelu_group(g.cols, g.type) == 32 && layer_gemv_supported(Ld.down.w, LAYER_PLAIN);
}

// the screened token selection's step 1 (k_logits.hip screen_prep) in the final norm's launch: its x16 blocks,
// A and the M reset from the same f16 roundings
void Session::screen_norm(NormOut& o) {
  if (!rec_gen_ || !screen_ || o.x16 != act_.x16 || hp_.n_embd > 8192) return;
  o.scr = scr_.xs;
  o.scr_mkey = scr_.m_key;
  scr_prepped_ = true;
}

// a norm feeding GEMV parts also writes their Q8_0 activation when every
// part consumes Q8_0 (one fewer launch); Q8_K blocks for K-quant parts
static NormOut norm_out_for(const std::vector<GemvPart>& consumer, float* xn, const ActBuf& act, bool ex_norm) {
  auto is_q8 = [](uint32_t t) { return t == T_Q4_0 || t == T_Q8_0; };
  NormOut o;
  o.xn = xn;
  bool q8 = !consumer.empty(), q8k = !consumer.empty();
  for (const auto& p : consumer) {
    q8 &= is_q8(p.w.type);
    q8k &= (p.w.type == T_Q4_K || p.w.type == T_Q6_K) && p.w.cols % 256 == 0;
  }
  if (q8) o.q8 = act.q8.xb;
  if (q8k && !ex_norm) o.q8k = act.q8k;  // exact mode keeps the reference's separate quantize launch
  return o;
}

NormOut Session::embed_out() const { return norm_out_for(L_[0].qkv, xn_, act_, ex_norm_); }

// the decode-loop graph may end with the next token's embed_norm (launch_finalize_embed_norm): one launch fewer
// per token
bool Session::embed_fold_ok() const {
  return use_graph_ && screen_ && (embd_.type == T_F16 || embd_.type == T_Q8_0) && !ple_table_.qs;
}

void Session::record_step(hipStream_t s, bool gen, bool fold_embed, bool logits) {
  kernels_per_token_ = 0;
  px_k_ = 0;
  rec_gen_ = gen;
  scr_prepped_ = false;
  rec_fold_ = fold_embed && gen && embed_fold_ok() && !dump_ && !trace_fn_;
  const int E = hp_.n_embd;
  const float emb_scale = std::sqrt(static_cast<float>(E));  // model.cpp:337-338
  auto nout = [&](const std::vector<GemvPart>& consumer) { return norm_out_for(consumer, xn_, act_, ex_norm_); };
  bool x_q8 = false;  // xn_'s Q8_0 blocks are already in act_
  const void* x_blocks = nullptr;  // where they are (Q8_0: act_.q8.xb, Q8_K: act_.q8k)
  if (embd_.type == T_F16 || embd_.type == T_Q8_0) {
    const NormOut o = nout(L_[0].qkv);
    if (!rec_fold_) {  // folded: the previous step's token feedback launch (or enqueue) ran it
      launch_embed_norm(embd_.type, embd_raw_, embd_row_bytes_, d_token_, emb_scale, resid_, L_[0].attn_norm, o, E,
                        hp_.eps, ex_norm_, s);
      kernels_per_token_++;
    }
    x_q8 = o.q8 != nullptr || o.q8k != nullptr;
    x_blocks = o.q8k ? (const void*)o.q8k : (const void*)o.q8;
  } else {
    launch_dequantize_rows(embd_.type, embd_raw_, embd_row_bytes_, d_token_, 1, E, emb_scale, resid_, s);
    launch_rms_norm(resid_, L_[0].attn_norm, xn_, E, 1, hp_.eps, ex_norm_, s);
    kernels_per_token_ += 2;
  }
  dump("inp_scaled", resid_, E, s);  // model.cpp:711-713
  if (ple_table_.qs) {  // Gemma-4 per-layer inputs (model.cpp:715-719, 568-704)
    const int NL = hp_.n_layer, EP = hp_.n_epl;
    launch_dequantize_rows(ple_table_.type, (const uint8_t*)ple_table_.qs, ple_row_bytes_, d_token_, 1, NL * EP,
                           std::sqrt((float)EP), inp_pl_, s);
    kernels_per_token_++;
    if (!ple_model_proj_.empty()) {
      gemv_parts(ple_model_proj_, resid_, E, ple_proj_out_, s, false);
      launch_scale(ple_proj_out_, NL * EP, 1.0f / std::sqrt((float)E), s);
      launch_ple_combine(ple_proj_out_, ple_proj_norm_, inp_pl_, NL, EP, hp_.eps, ex_norm_, s);
      kernels_per_token_ += 2;
      if (ple_model_proj_[0].w.type != T_BF16 && ple_model_proj_[0].w.type != T_F32) x_q8 = false;  // act_ reused
    }
  }
  dump("attn_norm-0", xn_, E, s);
  tap("inp_scaled", -1, resid_, (size_t)E * 4, s);
  tap("attn_norm", 0, xn_, (size_t)E * 4, s);
  // Q8_0: XBlocks; Q8_K: the reference's 292-B block_q8_K (norm_outputs, k_session.hip)
  if (x_q8) tap("xq", 0, x_blocks, x_blocks == (const void*)act_.q8k ? (size_t)(E / 256) * 292 : (size_t)(E / 32) * sizeof(XBlock), s);
  bool fused = fuse_layers_;
  for (const auto& l : L_) fused &= l.fused;
  if (tp_ && !fused && !xl_) throw status_error(LLMI_E_ARG, "tensor parallel needs the fused layer path");
  const bool xl_step =
      xl_ && !dump_ && !(trace_fn_ && getenv("LLMI_TRACE_PER_OP")) && x_q8 && x_blocks == (const void*)act_.q8.xb;
  // an exact tensor-parallel rank has only the exact-order engine's shards (record_layers runs whole matrices
  // and has no exchanges): refuse rather than produce a wrong step
  if (tp_ && exact_ && !xl_step)
    throw status_error(LLMI_E_ARG, "tensor parallel exact mode: this step cannot run on the exact-order engine "
                                   "(dumps and per-op traces are single-device only)");
  if (xl_step) {
    record_layers_xl(s);
  } else if (fused) {
    record_layers_fused(s, x_q8);
  } else {
    record_layers(s, x_q8);
  }
  if (logits) record_logits(s, gen);
  rec_gen_ = scr_prepped_ = rec_fold_ = false;
}

void Session::record_logits(hipStream_t s, bool gen) {
  const int E = hp_.n_embd;
  // logits (model.cpp:993-1034): F16 table -> mat_vec_mul_fp16, else mat_vec_mul
  // (a tensor-parallel rank: its vocabulary rows, its own argmax key, then
  // the keys all-gathered and reduced in finalize)
  if (embd_.type != T_F16) prepare_act(embd_.type, xn_, E, act_, s);
  const bool fold = !ex_logits_ && embd_.type == T_F16 && E % 8 == 0 && hp_.final_softcap <= 0.0f;
  float* lg = logits_ + (size_t)tp_rank_ * v_sh_;
  unsigned long long* key = amax_key_ + tp_rank_;
  if (gen && screen_) {  // token id only: int8 screening + exact rescoring of the candidates
    launch_screen_argmax(logits_w_, scr_, act_.x16, key, s, scr_prepped_, ex_logits_);
    kernels_per_token_ += scr_prepped_ ? 2 : 3;
    tap("x16", -1, act_.x16, (size_t)E * 2, s);
  } else {
    for (int r = 0; r < dup("logits"); r++)
      launch_gemv(logits_w_, act_, lg, ex_logits_ ? GEMV_EXACT : GEMV_FAST, s, fold ? key : nullptr);
    kernels_per_token_++;
    if (hp_.final_softcap > 0.0f) {  // model.cpp:1036-1041
      launch_softcap(lg, v_rows_, hp_.final_softcap, s);
      kernels_per_token_++;
    }
    dump("result_output", lg, v_rows_, s);  // model.cpp:1046
    tap("logits", -1, lg, (size_t)v_rows_ * 4, s);
  }
  if (!fold && !(gen && screen_)) {  // (the screened selection folds its own key; logits_ is stale then)
    launch_argmax(lg, v_rows_, key, s);
    kernels_per_token_++;
  }
  if (tp_) coll_->all_gather(amax_key_, sizeof(unsigned long long), s, px_take());
  if (rec_fold_)
    launch_finalize_embed_norm(amax_key_, tp_size_, v_sh_, d_token_, d_pos_, ring_, ring_idx_, max_ctx_, embd_.type,
                               embd_raw_, embd_row_bytes_, std::sqrt(static_cast<float>(E)), resid_, L_[0].attn_norm,
                               embed_out(), E, hp_.eps, ex_norm_, s);
  else
    launch_finalize_token(amax_key_, tp_size_, v_sh_, d_token_, d_pos_, ring_, ring_idx_, max_ctx_, s);
  kernels_per_token_++;
  tap("token", -1, d_token_, 4, s);
}

void Session::ensure_prefill_buffers(int cap) {
  if (cap <= pf_cap_) return;
  const int E = hp_.n_embd, F = hp_.n_ff;
  int maxq = 0, maxqkv = 0;
  for (const auto& l : L_) {
    maxq = std::max(maxq, hp_.n_head * l.hd);
    maxqkv = std::max(maxqkv, l.qkv_rows);
  }
  pf_xs_ = std::max({E, F, maxq}) / 32;
  pf_ostride_ = std::max({maxqkv, E, 2 * F});
  // grow-only; the previous chunk buffers stay allocated until the session ends
  pf_tokens_ = dalloc<int32_t>(cap);
  pf_resid_ = dalloc<float>((size_t)cap * E);
  pf_out_ = dalloc<float>((size_t)cap * pf_ostride_);
  pf_xq_ = dalloc<XBlock>((size_t)cap * pf_xs_);
  pf_x16_ = dalloc<uint16_t>((size_t)cap * pf_xs_ * 32);
  pf_tscale_ = dalloc<float>((size_t)cap);
  pf_q_ = dalloc<uint16_t>((size_t)cap * maxq);
  int maxhd = 0;
  for (const auto& l : L_) maxhd = std::max(maxhd, l.hd);
  const size_t nqb = (size_t)(cap + 31) / 32;
  pf_apart_ = dalloc<float>((size_t)nh_ * nqb * PREFILL_ATTN_KS_MAX * 64 * (maxhd / 2 + 2));
  if (tp_)  // all-gather staging: the largest exchanged [T][row] activation (f32 rows or Q8_0 block rows)
    pf_gather_ = dalloc<uint8_t>((size_t)cap * std::max({(size_t)E * 4, (size_t)pf_xs_ * sizeof(XBlock), (size_t)pf_xs_ * 64}));
  pf_cap_ = cap;
}

// Batched prefill of n prompt tokens at positions pos.. (chunks of up to
// LLMI_PREFILL_CHUNK, default 256): per layer one MFMA GEMM per projection
// over the chunk, per-token norms / rope / KV append, causal attention over
// the cache; the last token's logits then go through the decode tail.
// Tensor-parallel prefill exchange: every rank has written its column slice
// [T][slice_b bytes] at column rank * slice_b of buf (row pitch pitch_b);
// packs it into pf_gather_, all-gathers the per-rank [T][slice_b] blocks and
// scatters every rank's block back to its columns of buf.
void Session::gather_cols(void* buf, size_t pitch_b, size_t slice_b, int T, hipStream_t s) {
  // push exchange: the exchange kernel reads this rank's column slice and writes the peers' in place (no staging
  // copies: every byte moves in a kernel, ordered and cache-coherent with the GEMMs around it)
  if (coll_->all_gather_cols(buf, pitch_b, slice_b, T, s, px_take())) return;
  const size_t blk = slice_b * T;
  uint8_t* g = reinterpret_cast<uint8_t*>(pf_gather_);
  uint8_t* b = reinterpret_cast<uint8_t*>(buf);
  LLMI_HIP(hipMemcpy2DAsync(g + tp_rank_ * blk, slice_b, b + tp_rank_ * slice_b, pitch_b, slice_b, T,
                            hipMemcpyDeviceToDevice, s));
  coll_->all_gather(g, blk, s);
  for (int r = 0; r < tp_size_; r++)
    if (r != tp_rank_)
      LLMI_HIP(hipMemcpy2DAsync(b + r * slice_b, pitch_b, g + r * blk, slice_b, slice_b, T, hipMemcpyDeviceToDevice, s));
}

// The f16 path writes its activations as f16 rows scaled per token so that none overflows (token_xs); only an
// attention output past 65504 (the f16 cache's limit) could still become inf, and the GEMMs then produce
// non-finite rows.  Such a row reaches the last token's final norm through the residual stream
// or, via the KV cache, through attention (a non-last token's row can escape only in the last layer's FFN, whose
// output feeds nothing but that token's own residual).  So a finite final norm row proves no f16 activation that
// matters overflowed; otherwise the prefill is recomputed on the int8 path (the reference's Q8 numerics), which
// overwrites the same KV rows -- never a non-finite result.
void Session::prefill(const int32_t* tokens, int n, int pos) {
  if (!prefill_run(tokens, n, pos, true)) return;
  std::vector<float> h((size_t)hp_.n_embd);
  LLMI_HIP(hipMemcpyAsync(h.data(), xn_, h.size() * 4, hipMemcpyDeviceToHost, stream_));
  LLMI_HIP(hipStreamSynchronize(stream_));
  for (float v : h)
    if (!std::isfinite(v)) {
      pf_f16_redo_++;
      prefill_run(tokens, n, pos, false);
      return;
    }
}

bool Session::prefill_f16_ok() const {
  const int G = nh_ / std::max(nkv_, 1);
  const int fmode = prefill_f16_env();
  bool v7 = true;  // every projection of every layer a GEMM v7 weight
  for (const auto& l : L_) {
    v7 = v7 && prefill_gemm7_supported(l.o.w) && prefill_gemm7_supported(l.gate_up[0].w) && prefill_gemm7_supported(l.down.w);
    for (const auto& part : l.qkv) v7 = v7 && prefill_gemm7_supported(part.w);
  }
  return !tp_ && ((fmode == -1 && v7) || (fmode == 1 && (pf_kq_ || L_[0].o.w.type == T_Q4_0))) &&
         !getenv("LLMI_PREFILL_ATTN_V1") && (G == 1 || G == 2 || G == 4) &&
         layer_gemv_gelu_group(L_[0].gate_up[0].w.cols, L_[0].gate_up[0].w.type) % 8 == 0;
}

bool Session::prefill_run(const int32_t* tokens, int n, int pos, bool allow_f16) {
  hipStream_t s = stream_;
  const int E = hp_.n_embd, F = hp_.n_ff;
  // 512 tokens per chunk: the prefill GEMMs' weight tiles are re-read once per
  // 64-token tile, their activation tiles once per 64-row tile, and a longer
  // chunk fills the chip with more work-groups (4B, 512-token prompt: 21.4 ms
  // at 256-token chunks, 17.4 ms at 512)
  int chunk = 512;
  if (const char* c = getenv("LLMI_PREFILL_CHUNK")) chunk = std::max(1, atoi(c));
  // attention key splits across work-groups: a constant (never a function of the heads per rank), so tensor-
  // parallel ranks merge the same partials in the same order as one device
  pf_attn_ks_ = 4;
  if (const char* c = getenv("LLMI_PREFILL_ATTN_KS")) pf_attn_ks_ = std::min(std::max(1, atoi(c)), PREFILL_ATTN_KS_MAX);
  ensure_prefill_buffers(std::min(chunk, n));
  const int XS = pf_xs_, X16 = pf_xs_ * 32;
  const int r = tp_rank_;  // tensor parallel: this rank's column slices (0 on one device)
  const float emb_scale = std::sqrt(static_cast<float>(E));  // model.cpp:337-338
  // Activations: f16 rows of the dequantized Q8_0 blocks, scaled per token by 2^-s (the producers' token_xs), and
  // the f16 MFMA GEMM v7 (Q4_0 layers, one device: the default) -- every product the reference's Q8_0 x Q4_0 term
  // to two f16 roundings; or Q8_0 blocks and the int8 GEMM v5 (LLMI_PREFILL_F16=0, Q8_0 weights, tensor-parallel
  // ranks: a token's scale would differ between the ranks' GELU slices); K-quant layers: Q8_K blocks and v5's
  // K-quant form, or (LLMI_PREFILL_F16=1) f16 rows and GEMM v6.  DESIGN.md section 4.2
  const bool f16_all = allow_f16 && prefill_f16_ok();
  // the last layer past its K / V appends (one token: the trim below) takes the int8 path: the f16 GEMMs' tiles
  // are slow for T = 1 (4B: gate_up 38 vs 24 us, down 52 vs 43)
  bool f16 = f16_all;
  int q8k = pf_kq_ && !f16 ? 1 : 0;
  // t0: the first token row the rest of a layer runs on (the last layer: only the prompt's final token needs its
  // o / FFN -- every other token's last-layer state is its K / V rows, already in the cache: model.cpp:983-1001)
  int t0 = 0;
  // scaled: the x16 rows carry the token scales in pf_tscale_ (the attention's output rows do not: |O| <= max |V|)
  auto gemm = [&](const DevWeight& w, float* out, int ostride, bool scaled) {
    if (f16)
      launch_prefill_gemm16(w, pf_x16_ + (size_t)t0 * X16, X16, T_cur_, out + (size_t)t0 * ostride, ostride,
                            scaled ? pf_tscale_ + t0 : nullptr, s);
    else launch_prefill_gemm(w, pf_xq_ + (size_t)t0 * XS, XS, T_cur_, out + (size_t)t0 * ostride, ostride, s);
  };
  auto xtap = [&](const char* name, const char* sname, int l) {  // sname: the token scales' tap (scaled rows)
    if (f16) {
      tap(name, l, pf_x16_ + (size_t)t0 * X16, (size_t)T_cur_ * X16 * 2, s);
      if (sname) tap(sname, l, pf_tscale_ + t0, (size_t)T_cur_ * 4, s);
    } else {
      tap(name, l, pf_xq_ + (size_t)t0 * XS, (size_t)T_cur_ * XS * sizeof(XBlock), s);
    }
  };
  auto xgather = [&](int cols) {  // this rank's activation columns [r * cols, (r + 1) * cols) to every rank
    if (!tp_) return;
    if (f16) gather_cols(pf_x16_ + (size_t)t0 * X16, (size_t)X16 * 2, (size_t)cols * 2, T_cur_, s);
    else gather_cols(pf_xq_ + (size_t)t0 * XS, (size_t)XS * sizeof(XBlock), (size_t)(cols / 32) * sizeof(XBlock), T_cur_, s);
  };
  const bool trim = getenv("LLMI_PREFILL_FULL_LAST") == nullptr;  // (A/B: the last layer over every token)
  for (int c0 = 0; c0 < n; c0 += pf_cap_) {
    const int T = std::min(pf_cap_, n - c0), p0 = pos + c0;
    T_cur_ = T;
    const bool last_chunk = c0 + T == n;
    LLMI_HIP(hipMemcpyAsync(pf_tokens_, tokens + c0, (size_t)T * 4, hipMemcpyHostToDevice, s));
    PrefillNorm en;
    en.table = embd_raw_;
    en.emb_type = embd_.type;
    en.row_bytes = embd_row_bytes_;
    en.tokens = pf_tokens_;
    en.emb_scale = emb_scale;
    en.resid = pf_resid_;
    en.w_next = L_[0].attn_norm;
    en.xq = pf_xq_;
    en.xstride = XS;
    en.n = E;
    en.eps = hp_.eps;
    en.x16 = f16 ? pf_x16_ : nullptr;
    en.x16stride = X16;
    en.tscale = f16 ? pf_tscale_ : nullptr;
    en.q8k = q8k;
    launch_prefill_norm(en, T, s);
    for (int l = 0; l < hp_.n_layer; l++) {
      const LayerDev& Ld = L_[l];
      const int hd = Ld.hd;
      t0 = 0;
      T_cur_ = T;
      f16 = f16_all;
      q8k = pf_kq_ && !f16 ? 1 : 0;
      xtap("pf_x_qkv", "pf_xs_qkv", l);
      for (size_t pi = 0, r0 = 0; pi < Ld.qkv.size(); r0 += Ld.qkv[pi].w.rows, pi++)  // q|k|v, or q|k and v (kq)
        gemm(Ld.qkv[pi].w, pf_out_ + r0, Ld.qkv_rows, true);
      tap("pf_qkv", l, pf_out_, (size_t)T * Ld.qkv_rows * 4, s);
      PrefillQK qk;
      qk.qkv = pf_out_;
      qk.qkv_stride = Ld.qkv_rows;
      qk.k_off = Ld.k_off;
      qk.v_off = Ld.v_off;
      qk.n_head = nh_;
      qk.n_head_kv = nkv_;
      qk.head_dim = hd;
      qk.q_norm_w = Ld.q_norm;
      qk.k_norm_w = Ld.k_norm;
      qk.rope_cs = Ld.is_swa ? rope_swa_ : rope_glb_;
      qk.attn_scale = hp_.attn_scale;
      qk.eps = hp_.eps;
      qk.q_out = pf_q_;
      qk.k_cache = Ld.kc;
      qk.v_cache = Ld.vc;
      qk.max_ctx = max_ctx_;
      qk.pos0 = p0;
      launch_prefill_qk(qk, T, s);
      if (trim && l + 1 == hp_.n_layer) {  // the last layer past its K / V appends: the final token only
        if (!last_chunk) break;
        t0 = T - 1;
        T_cur_ = 1;
      }
      // the last layer's attention output and FFN on the int8 path (Q4_0 layers: v5 takes every shape the f16
      // path does), trimmed or not (LLMI_PREFILL_FULL_LAST: the same arithmetic for the final token)
      if (l + 1 == hp_.n_layer && !pf_kq_) f16 = false;
      const int Tq = T_cur_;
      PrefillAttn at;
      at.softcap = hp_.attn_softcap;
      at.q = pf_q_ + (size_t)t0 * nh_ * hd;
      at.k_cache = Ld.kc;
      at.v_cache = Ld.vc;
      at.n_head = nh_;
      at.n_head_kv = nkv_;
      at.head_dim = hd;
      at.max_ctx = max_ctx_;
      at.pos0 = p0 + t0;
      const int hb = nh_ * hd / 32;  // this rank's heads' Q8_0 blocks per token
      const int hr = tp_rep_attn_ ? 0 : r;  // replicated attention: every rank has all heads
      at.xq = pf_xq_ + (size_t)t0 * XS + (size_t)hr * hb;
      at.xstride = XS;
      at.x16 = f16 ? pf_x16_ + (size_t)t0 * X16 + (size_t)hr * nh_ * hd : nullptr;
      at.x16stride = X16;
      at.q8k = q8k;
      at.ks = pf_attn_ks_;
      at.part = pf_apart_;
      launch_prefill_attn(at, Tq, s);
      if (!tp_rep_attn_) xgather(nh_ * hd);
      tap("pf_q", l, pf_q_, (size_t)T * nh_ * hd * 2, s);
      tap("kc", l, Ld.kc, (size_t)nkv_ * max_ctx_ * hd * 2, s);
      tap("vc", l, Ld.vc, (size_t)nkv_ * max_ctx_ * hd * 2, s);
      xtap("pf_x_o", nullptr, l);
      gemm(Ld.o.w, pf_out_ + (size_t)r * e_sh_, E, false);
      if (tp_) gather_cols(pf_out_ + (size_t)t0 * E, (size_t)E * 4, (size_t)e_sh_ * 4, Tq, s);
      tap("pf_o", l, pf_out_ + (size_t)t0 * E, (size_t)Tq * E * 4, s);
      PrefillNorm rn;  // post-attention norm + residual, then ffn_norm
      rn.y = pf_out_ + (size_t)t0 * E;
      rn.w_post = Ld.post_attn_norm;
      rn.resid = pf_resid_ + (size_t)t0 * E;
      rn.w_next = Ld.ffn_norm;
      rn.xq = pf_xq_ + (size_t)t0 * XS;
      rn.xstride = XS;
      rn.n = E;
      rn.eps = hp_.eps;
      rn.x16 = f16 ? pf_x16_ + (size_t)t0 * X16 : nullptr;
      rn.x16stride = X16;
      rn.tscale = f16 ? pf_tscale_ + t0 : nullptr;
      rn.q8k = q8k;
      launch_prefill_norm(rn, Tq, s);
      tap("pf_resid_attn", l, rn.resid, (size_t)Tq * E * 4, s);
      xtap("pf_x_gate_up", "pf_xs_gate_up", l);
      const int FL = tp_ ? f_sh_ : F;  // this rank's hidden units
      gemm(Ld.gate_up[0].w, pf_out_, 2 * FL, true);
      tap("pf_gate_up", l, pf_out_ + (size_t)t0 * 2 * FL, (size_t)Tq * 2 * F * 4, s);
      launch_prefill_gelu(pf_out_ + (size_t)t0 * 2 * FL, FL, layer_gemv_gelu_group(Ld.gate_up[0].w.cols, Ld.gate_up[0].w.type),
                          pf_xq_ + (size_t)t0 * XS + (size_t)r * (FL / 32), XS, Tq, s,
                          f16 ? pf_x16_ + (size_t)t0 * X16 + (size_t)r * FL : nullptr, X16, q8k,
                          f16 ? pf_tscale_ + t0 : nullptr);
      xgather(FL);
      xtap("pf_x_down", "pf_xs_down", l);
      gemm(Ld.down.w, pf_out_ + (size_t)r * e_sh_, E, true);
      if (tp_) gather_cols(pf_out_ + (size_t)t0 * E, (size_t)E * 4, (size_t)e_sh_ * 4, Tq, s);
      tap("pf_down", l, pf_out_ + (size_t)t0 * E, (size_t)Tq * E * 4, s);
      if (l + 1 < hp_.n_layer) {  // post-ffw norm + residual, then the next attn_norm
        PrefillNorm fn = rn;
        fn.w_post = Ld.post_ffw_norm;
        fn.w_next = L_[l + 1].attn_norm;
        launch_prefill_norm(fn, T, s);
        tap("pf_resid_ffn", l, pf_resid_, (size_t)T * E * 4, s);
      }
    }
    if (last_chunk) {  // the last token: final residual + output_norm -> logits (decode tail)
      NormOut o2;
      o2.xn = xn_;
      if (embd_.type == T_F16) o2.x16 = act_.x16;
      launch_residual_norm(pf_out_ + (size_t)(T - 1) * E, L_.back().post_ffw_norm, pf_resid_ + (size_t)(T - 1) * E,
                           out_norm_, o2, E, hp_.eps, false, s);
      record_logits(s);
    }
  }
  return f16_all;
}

// Fast path with every projection a gemv_q4_0_layer launch: 5 launches per
// layer (qkv [+ residual/norm prologue], attention, o, gate_up [+ prologue +
// GELU epilogue], down [+ Q8_0 of the GELU output]).  The residual stream
// ping-pongs between resid_ and resid2_ (a prologue's work-group 0 writes the
// buffer its sibling work-groups are not reading).
void Session::record_layers_fused(hipStream_t s, bool x_q8) {
  const int E = hp_.n_embd;
  float* cur = resid_;
  float* other = resid2_;
  // tensor-parallel ranks: the o, GELU and down outputs go to the peers from the producing launches' epilogues
  // and the consumers read their mailbox (px.h) -- no exchange launches but the attention output's (head-sharded
  // mode), the last layer's down and the argmax keys
  bool pxf = tp_ && px_on();
  for (const auto& l : L_) pxf = pxf && l.qkv.size() == 1;  // (the two-weight q|k|v launch has no fused variant)
  int k_d = -1;  // the previous layer's down exchange, read by this layer's qkv prologue
  std::vector<int> px_nwg;  // exchange k -> the work-groups that push it (their checksum granules, px.h)
  auto fx_in = [&](LayerGemv& g, int k, int ws) {
    if (k < 0) return;
    g.px = d_px_;
    g.px_in = k;
    g.px_in_ws = ws;
    g.px_in_nwg = k < (int)px_nwg.size() ? px_nwg[k] : 0;
  };
  auto fx_out = [&](LayerGemv& g) {
    g.px = d_px_;
    g.px_out = px_k_++;
    return g.px_out;
  };
  auto fx_nwg = [&](const LayerGemv& g, int nwg) {  // after the producing launch
    if (g.px_out < 0) return;
    if ((int)px_nwg.size() <= g.px_out) px_nwg.resize(g.px_out + 1, 0);
    px_nwg[g.px_out] = nwg;
  };
  for (int l = 0; l < hp_.n_layer; l++) {
    LayerDev& Ld = L_[l];
    const int hd = Ld.hd;
    unsigned* epoch = block_ ? blk_epoch_ + l : nullptr;
    const std::string L = std::to_string(l);
    if (block_ && !dump_) {  // qkv + attention + o: one launch (k_attn.hip attention block)
      LayerGemv g;
      int qrole = LAYER_PLAIN;
      if (l == 0) {
        if (Ld.qkv[0].w.kq) {  // Q8_K quants in XBlocks for the kq qkv
          launch_quantize_q8k_xblocks(xn_, E, act_.q8.xb, s);
          kernels_per_token_++;
        } else if (!x_q8) {
          launch_quantize_q8_0(xn_, E, act_.q8, s);
          kernels_per_token_++;
        }
        g.xg = act_.q8.xb;
      } else if (block_pro_) {
        qrole = LAYER_PRO;
        g.y = d_out_;
        g.w_post = L_[l - 1].post_ffw_norm;
        g.resid_in = cur;
        g.resid_out = other;
        g.w_next = Ld.attn_norm;
        g.eps = hp_.eps;
        fx_in(g, k_d, e_sh_);
        std::swap(cur, other);
      } else {  // model.cpp:722-756: residual + post-FFN norm, attention norm, Q8_0 blocks; the block reads them
        NormOut on;
        on.xn = xn_;
        on.q8 = act_.q8.xb;
        launch_residual_norm(d_out_, L_[l - 1].post_ffw_norm, cur, Ld.attn_norm, on, E, hp_.eps, false, s);
        kernels_per_token_++;
        tap("attn_resid", l, cur, (size_t)E * 4, s);
        tap("attn_norm", l, xn_, (size_t)E * 4, s);
        g.xg = act_.q8.xb;
      }
      g.out = qkv_;
      QKVArgs qa{qkv_, Ld.k_off, Ld.v_off, nh_, nkv_, hd, Ld.q_norm, Ld.k_norm,
                 Ld.is_swa ? rope_swa_ : rope_glb_, hp_.attn_scale, hp_.eps, q_, Ld.kc, Ld.vc, max_ctx_, d_pos_};
      AttnArgs aa{q_, Ld.kc, Ld.vc, nh_, nkv_, hd, max_ctx_, d_pos_, part_, attn_, ticket_, blk_xo_};
      LayerGemv go;
      go.xg = blk_xo_;
      go.out = o_out_ + (size_t)tp_rank_ * e_sh_;  // this rank's o rows (all of them on one device)
      if (pxf) fx_out(go);
      BlockSync bs;
      bs.epoch = epoch;
      bs.done = blk_done_ + (size_t)l * 32;
      bs.g_qkv = blk_gqkv_ + (size_t)l * blk_gqkv_stride_;
      bs.g_xo = blk_gxo_ + (size_t)l * blk_gxo_stride_;
      bs.err = blk_err_;
      if (blk_trace_ && l == blk_trace_layer_) bs.trace = blk_trace_;
      if (trace_fn_ && qrole == LAYER_PRO) g.xn_out = xn_;
      aa.q8k = Ld.o.w.kq ? 1 : 0;
      aa.softcap = hp_.attn_softcap;
      fx_nwg(go, launch_attn_block(Ld.qkv[0].w, Ld.qkv.size() > 1 ? &Ld.qkv[1].w : nullptr, g, qrole, Ld.o.w, go, aa,
                                   qa, bs, s));
      kernels_per_token_++;
      if (trace_fn_) {  // the launch's products: residual / norm (prologue), q|k|v and xo granules, attention, o
        if (qrole == LAYER_PRO) {
          tap("attn_resid", l, cur, (size_t)E * 4, s);
          tap("attn_norm", l, xn_, (size_t)E * 4, s);
        }
        tap("qkv_g", l, bs.g_qkv, (size_t)Ld.qkv_rows * 8, s);
        tap("attn", l, attn_, (size_t)nh_ * hd * 4, s);
        tap("xo_g", l, bs.g_xo, (size_t)nh_ * hd / 32 * 12 * 8, s);
        tap("o", l, o_out_, (size_t)E * 4, s);
        tap("kc", l, Ld.kc, (size_t)nkv_ * max_ctx_ * hd * 2, s);
        tap("vc", l, Ld.vc, (size_t)nkv_ * max_ctx_ * hd * 2, s);
      }
    } else {
      LayerGemv g;
      const bool kq = Ld.qkv[0].w.kq != 0;  // K-quant layer: Q8_K activations in XBlocks
      auto qkv_launch = [&](const LayerGemv& gg, int role) {
        if (Ld.qkv.size() == 2) launch_layer_gemv2(Ld.qkv[0].w, Ld.qkv[1].w, gg, role, s);
        else launch_layer_gemv(Ld.qkv[0].w, gg, role, s);
      };
      if (l == 0) {
        if (kq) {
          launch_quantize_q8k_xblocks(xn_, E, act_.q8.xb, s);
          kernels_per_token_++;
        } else if (!x_q8) {
          launch_quantize_q8_0(xn_, E, act_.q8, s);
          kernels_per_token_++;
        }
        g.xg = act_.q8.xb;
        g.out = qkv_;
        for (int r = 0; r < dup("qkv"); r++) qkv_launch(g, LAYER_PLAIN);
      } else {
        g.y = d_out_;
        g.w_post = L_[l - 1].post_ffw_norm;
        g.resid_in = cur;
        g.resid_out = other;
        g.w_next = Ld.attn_norm;
        g.eps = hp_.eps;
        g.out = qkv_;
        if (dump_ || trace_fn_) g.xn_out = xn_;
        fx_in(g, k_d, e_sh_);
        for (int r = 0; r < dup("qkv"); r++) qkv_launch(g, LAYER_PRO);
        tap("attn_resid", l, other, (size_t)E * 4, s);
        tap("attn_norm", l, xn_, (size_t)E * 4, s);
        dump("l_out-" + std::to_string(l - 1), other, E, s);
        dump("attn_norm-" + L, xn_, E, s);
        std::swap(cur, other);
      }
      kernels_per_token_++;
      tap("qkv", l, qkv_, (size_t)Ld.qkv_rows * 4, s);
      dump("Qcur-" + L, qkv_, nh_ * hd, s);
      dump("Kcur-" + L, qkv_ + Ld.k_off, nkv_ * hd, s);
      dump("Vcur-" + L, qkv_ + Ld.v_off, nkv_ * hd, s);
      // this rank's heads (all of them without tensor parallelism)
      QKVArgs qa{qkv_, Ld.k_off, Ld.v_off, nh_, nkv_, hd, Ld.q_norm, Ld.k_norm,
                 Ld.is_swa ? rope_swa_ : rope_glb_, hp_.attn_scale, hp_.eps, q_, Ld.kc, Ld.vc, max_ctx_, d_pos_};
      const bool q8_in_combine = hd % 32 == 0;
      if (tp_ && !q8_in_combine) throw status_error(LLMI_E_ARG, "tensor parallel: head_dim % 32 != 0");
      const int hb = nh_ * hd / 32;  // Q8_0 blocks of this rank's heads
      const int hr = tp_rep_attn_ ? 0 : tp_rank_;  // the heads' place in the all-heads vector
      AttnArgs aa{q_, Ld.kc, Ld.vc, nh_, nkv_, hd, max_ctx_, d_pos_, part_, attn_,
                  ticket_, q8_in_combine ? act_.q8.xb + (size_t)hr * hb : nullptr};
      aa.q8k = Ld.o.w.kq ? 1 : 0;  // the kq o projection reads Q8_K quants
      aa.softcap = hp_.attn_softcap;
      for (int r = 0; r < dup("attn"); r++) launch_attention(aa, false, s, &qa);
      kernels_per_token_++;
      tap("attn", l, attn_, (size_t)nh_ * hd * 4, s);
      tap("kc", l, Ld.kc, (size_t)nkv_ * max_ctx_ * hd * 2, s);
      tap("vc", l, Ld.vc, (size_t)nkv_ * max_ctx_ * hd * 2, s);
      dump("kqv_out-" + L, attn_, nh_ * hd, s);
      if (!q8_in_combine) {
        launch_quantize_q8_0(attn_, hp_.n_head * hd, act_.q8, s);
        kernels_per_token_++;
      }
      if (tp_ && !tp_rep_attn_) coll_->all_gather(act_.q8.xb, (size_t)hb * sizeof(XBlock), s, px_take());
      LayerGemv go;
      go.xg = act_.q8.xb;
      go.out = o_out_ + (size_t)tp_rank_ * e_sh_;
      if (pxf) fx_out(go);
      tap("xo", l, act_.q8.xb, (size_t)hp_.n_head * hd / 32 * sizeof(XBlock), s);
      for (int r = 0; r < dup("o_proj"); r++) fx_nwg(go, launch_layer_gemv(Ld.o.w, go, LAYER_PLAIN, s));
      tap("o", l, o_out_, (size_t)E * 4, s);
      dump("attention results (node_30 for MUL_MAT)-" + L, o_out_, E, s);
    }
    const int k_o = pxf ? px_k_ - 1 : -1;  // the o launch's exchange (the block's or the standalone o's)
    if (pxf) coll_->fused_point(s);
    else if (tp_) coll_->all_gather(o_out_, (size_t)e_sh_ * sizeof(float), s, px_take());
    LayerGemv gg;
    gg.y = o_out_;
    gg.w_post = Ld.post_attn_norm;
    gg.resid_in = cur;
    gg.resid_out = other;
    gg.w_next = Ld.ffn_norm;
    gg.eps = hp_.eps;
    gg.hid = hid_ + (size_t)tp_rank_ * f_sh_;
    const bool dplain = down_plain(Ld);
    if (dplain) gg.hq = hq_ + (size_t)tp_rank_ * (f_sh_ / 32);
    if (dump_ || trace_fn_) gg.xn_out = xn_;
    const bool gfx = pxf;
    int k_h = -1;
    if (gfx) {
      fx_in(gg, k_o, e_sh_);
      k_h = fx_out(gg);
    }
    for (int r = 0; r < dup("gate_up"); r++)
      fx_nwg(gg, launch_layer_gemv(Ld.gate_up[0].w, gg, LAYER_GELU, s));
    tap("ffn_resid", l, other, (size_t)E * 4, s);
    tap("ffn_norm", l, xn_, (size_t)E * 4, s);
    tap("hid", l, hid_, (size_t)hp_.n_ff * 4, s);
    dump("sa_out-" + L, other, E, s);
    dump("ffn_norm-" + L, xn_, E, s);
    dump("ffn_geglu-" + L, hid_, hp_.n_ff, s);
    std::swap(cur, other);
    if (gfx) coll_->fused_point(s);
    else if (tp_ && dplain) coll_->all_gather(hq_, (size_t)(f_sh_ / 32) * sizeof(XBlock), s, px_take());
    else if (tp_) coll_->all_gather(hid_, (size_t)f_sh_ * sizeof(float), s, px_take());
    LayerGemv gd;
    gd.y = hid_;  // QUANT: GELU output quantized per block in the down launch
    gd.xg = hq_;  // PLAIN: the blocks the GELU launch wrote
    gd.out = d_out_ + (size_t)tp_rank_ * e_sh_;
    fx_in(gd, k_h, dplain ? f_sh_ / 32 * 12 : f_sh_);
    // the next layer's qkv prologue reads the down exchange from its mailbox (the 27B attention block's PLAIN
    // role reads the blocks of a residual_norm launch instead, and the last layer's feeds the final norm)
    const bool dfx = gfx && l + 1 < hp_.n_layer && (!block_ || block_pro_);
    k_d = dfx ? fx_out(gd) : -1;
    for (int r = 0; r < dup("down"); r++) fx_nwg(gd, launch_layer_gemv(Ld.down.w, gd, dplain ? LAYER_PLAIN : LAYER_QUANT, s));
    tap("down", l, d_out_, (size_t)E * 4, s);
    if (dfx) coll_->fused_point(s);
    else if (tp_) coll_->all_gather(d_out_, (size_t)e_sh_ * sizeof(float), s, px_take());
    dump("ffn_out-" + L, d_out_, E, s);
    kernels_per_token_ += block_ ? 2 : 3;  // (o, when not in the attention block,) gate_up, down
  }
  // final residual + output_norm (-> xn_, and f16 x for an F16 logits table)
  NormOut o2;
  o2.xn = xn_;
  if (embd_.type == T_F16) o2.x16 = act_.x16;
  screen_norm(o2);
  launch_residual_norm(d_out_, L_.back().post_ffw_norm, cur, out_norm_, o2, E, hp_.eps, false, s);
  kernels_per_token_++;
  tap("final_resid", -1, cur, (size_t)E * 4, s);
  tap("result_norm", -1, xn_, (size_t)E * 4, s);
  dump("l_out-" + std::to_string(hp_.n_layer - 1), cur, E, s);
  dump("result_norm", xn_, E, s);
}

// Exact mode on the exact-order engine (exact.h): every Gemma-3 layer with Q4_0 q, k, v, o, gate, up and down
// (the 4B / 1B / 27B Q4_0 files) gets XL copies of its weights; LLMI_EXACT_XL=0 keeps the per-op exact kernels.
void Session::setup_xl() {
  if (!exact_ || hp_.gemma4 || ple_table_.qs || getenv("LLMI_EXACT_PARTS")) return;
  if (const char* e = getenv("LLMI_EXACT_XL"))
    if (atoi(e) == 0 && !tp_) return;
  const int F = tp_ ? f_sh_ : hp_.n_ff;  // this rank's hidden units
  if (hp_.n_embd % 128 || hp_.n_ff % 128 || F % 32 || (tp_ && e_sh_ % 16) ||
      2 * (size_t)hp_.n_embd * 4 + hp_.n_embd / 32 * 68 > 60 * 1024)
    return;
  for (const auto& l : L_) {
    bool ok = l.has_kv && !l.qkv.empty() && !l.gate_up.empty() && (hp_.n_head * l.hd) % 128 == 0 &&
              exact_attn_supported(l.hd, hp_.n_head, hp_.n_head_kv);
    for (const auto& p : l.qkv) ok = ok && xl_supported(p.w);
    for (const auto& p : l.gate_up) ok = ok && xl_supported(p.w);
    int gu_rows = 0;
    for (const auto& p : l.gate_up) gu_rows += p.w.rows;
    ok = ok && xl_supported(l.o.w) && xl_supported(l.down.w) && gu_rows == 2 * F && !l.gu_interleaved &&
         (l.gate_up.size() == 1 || l.gate_up[0].w.rows == F) && l.down.w.cols == hp_.n_ff;
    if (!ok) return;
  }
  for (auto& l : L_) {
    // gate and up: one part of rows [gate; up] (same type) or two parts
    DevWeight gate = l.gate_up[0].w, up;
    if (l.gate_up.size() == 1) {
      const int nb = gate.cols / 32;
      gate.rows = F;
      up = gate;
      up.qs = static_cast<uint8_t*>(gate.qs) + (size_t)F * nb * 16;
      up.d = gate.d + (size_t)F * nb;
      gate.bytes = up.bytes = gguf_bytes(T_Q4_0, F, gate.cols);
    } else {
      up = l.gate_up[1].w;
    }
    XlSrc q;
    for (auto& p : l.qkv) q.w[q.n++] = &p.w;
    l.xqkv = make_xl_weight(q, stream_);
    XlSrc o;
    o.w[o.n++] = &l.o.w;
    l.xo = make_xl_weight(o, stream_);
    XlSrc gu;
    gu.w[gu.n++] = &gate;
    gu.w[gu.n++] = &up;
    gu.gelu32 = true;
    l.xgu = make_xl_weight(gu, stream_);
    XlSrc d;
    d.w[d.n++] = &l.down.w;
    l.xdn = make_xl_weight(d, stream_);
  }
  int maxhd = 0;
  for (const auto& l : L_) maxhd = std::max(maxhd, l.hd);
  xa_scores_ = dalloc<double>((size_t)hp_.n_head * max_ctx_);
  xa_xq_ = dalloc<XBlock>((size_t)hp_.n_head * maxhd / 32);
  xa_vt_stride_ = (max_ctx_ + 31) / 32 * 32;
  for (auto& l : L_) {  // the tiled V caches (zeroed: columns past the context are loaded, never summed)
    const size_t n = (size_t)hp_.n_head_kv * l.hd * xa_vt_stride_;
    l.vt = dalloc<uint16_t>(n);
    LLMI_HIP(hipMemsetAsync(l.vt, 0, n * 2, stream_));
    l.kmeta = dalloc<uint32_t>((size_t)hp_.n_head_kv * max_ctx_);  // (dalloc zeroes: every key unknown)
  }
  LLMI_HIP(hipStreamSynchronize(stream_));
  xl_ = true;
}

// One decode step's layers on the exact-order engine: per layer q|k|v (the previous layer's post-FFN norm and
// residual + this layer's attn_norm in its prologue), q/k norm + rope + KV append, attention, o (its input
// quantized in the prologue), gate|up (post-attention norm + residual + ffn_norm in the prologue, GELU * up and
// the hidden Q8_0 blocks in the epilogue), down.  The residual stream alternates between resid_ and resid2_ (a
// prologue's work-group 0 writes the new residual while the others still read the old one).
void Session::record_layers_xl(hipStream_t s) {
  const int E = hp_.n_embd;
  float* ra = resid_;
  float* rb = resid2_;
  for (int l = 0; l < hp_.n_layer; l++) {
    LayerDev& Ld = L_[l];
    const int hd = Ld.hd;
    XlArgs q;
    q.n = E;
    q.eps = hp_.eps;
    q.out = qkv_;
    if (l == 0) {  // the embedding launch wrote attn_norm(x)'s Q8_0 blocks
      q.xb = act_.q8.xb;
      launch_exact_gemv(Ld.xqkv, q, XL_PLAIN, s);
    } else {
      q.y = d_out_;
      q.w_post = L_[l - 1].post_ffw_norm;
      q.resid_in = ra;
      q.resid_out = rb;
      q.w_next = Ld.attn_norm;
      launch_exact_gemv(Ld.xqkv, q, XL_PRE, s);
      std::swap(ra, rb);
    }
    XAttnArgs xa;
    xa.qkv = qkv_;
    xa.k_off = Ld.k_off;
    xa.v_off = Ld.v_off;
    xa.n_head = hp_.n_head;
    xa.n_head_kv = hp_.n_head_kv;
    xa.head_dim = hd;
    xa.q_norm_w = Ld.q_norm;
    xa.k_norm_w = Ld.k_norm;
    xa.rope_cs = Ld.is_swa ? rope_swa_ : rope_glb_;
    xa.attn_scale = hp_.attn_scale;
    xa.eps = hp_.eps;
    xa.k_cache = Ld.kc;
    xa.v_cache = Ld.vc;
    xa.max_ctx = max_ctx_;
    xa.d_pos = d_pos_;
    xa.scores = xa_scores_;
    xa.out = attn_;
    xa.xq = xa_xq_;
    xa.softcap = hp_.attn_softcap;
    xa.vt = Ld.vt;
    xa.vt_stride = xa_vt_stride_;
    xa.kmeta = Ld.kmeta;
    launch_exact_attn(xa, s);
    // tensor-parallel ranks: this rank's rows of o, gate/up (its hidden units) and down, each slice all-gathered
    // before its consumer (whose residual / norm prologue runs on the whole vector on every rank)
    XlArgs o;
    o.xb = xa_xq_;
    o.out = o_out_ + (size_t)tp_rank_ * e_sh_;
    launch_exact_gemv(Ld.xo, o, XL_PLAIN, s);
    if (tp_) coll_->all_gather(o_out_, (size_t)e_sh_ * sizeof(float), s, px_take());
    XlArgs gu;
    gu.y = o_out_;
    gu.w_post = Ld.post_attn_norm;
    gu.resid_in = ra;
    gu.resid_out = rb;
    gu.w_next = Ld.ffn_norm;
    gu.n = E;
    gu.eps = hp_.eps;
    gu.hid = hid_ + (size_t)tp_rank_ * f_sh_;
    gu.hq = hq_ + (size_t)tp_rank_ * (f_sh_ / 32);
    launch_exact_gemv(Ld.xgu, gu, XL_GELU, s);
    if (tp_) coll_->all_gather(hq_, (size_t)(f_sh_ / 32) * sizeof(XBlock), s, px_take());
    std::swap(ra, rb);
    XlArgs dn;
    dn.xb = hq_;
    dn.out = d_out_ + (size_t)tp_rank_ * e_sh_;
    launch_exact_gemv(Ld.xdn, dn, XL_PLAIN, s);
    if (tp_) coll_->all_gather(d_out_, (size_t)e_sh_ * sizeof(float), s, px_take());
    kernels_per_token_ += 6;
  }
  // the last layer's post-FFN norm + residual, then output_norm (model.cpp:915-924, 986)
  NormOut o2;
  o2.xn = xn_;
  if (embd_.type == T_F16) o2.x16 = act_.x16;
  screen_norm(o2);
  launch_residual_norm(d_out_, L_.back().post_ffw_norm, ra, out_norm_, o2, E, hp_.eps, true, s);
  kernels_per_token_++;
}

bool Session::xp_ok() const {
  return xl_ && !tp_ && !dump_ && !trace_fn_ && (embd_.type == T_F16 || embd_.type == T_F32 || embd_.type == T_Q8_0) &&
         hp_.n_embd % 128 == 0 && hp_.n_embd <= 6144 && getenv("LLMI_XP_OFF") == nullptr;
}

void Session::exact_prefill(const int32_t* tokens, int n, int pos) {
  hipStream_t s = stream_;
  const int E = hp_.n_embd, F = hp_.n_ff;
  int chunk = 256;
  if (const char* c = getenv("LLMI_XP_CHUNK")) chunk = std::max(1, atoi(c));
  const int cap = std::min(chunk, n);
  if (cap > xp_cap_) {  // grow-only chunk buffers
    int maxq = 0, maxqkv = 0;
    for (const auto& l : L_) {
      maxq = std::max(maxq, hp_.n_head * l.hd);
      maxqkv = std::max(maxqkv, l.qkv_rows);
    }
    xp_tok_ = dalloc<int32_t>(cap);
    xp_resid_ = dalloc<float>((size_t)cap * E);
    xp_o_ = dalloc<float>((size_t)cap * E);
    xp_d_ = dalloc<float>((size_t)cap * E);
    xp_qkv_ = dalloc<float>((size_t)cap * maxqkv);
    xp_att_ = dalloc<float>((size_t)cap * maxq);
    xp_xq_ = dalloc<XBlock>((size_t)cap * (E / 32));
    xp_hq_ = dalloc<XBlock>((size_t)cap * (F / 32));
    xp_axq_ = dalloc<XBlock>((size_t)cap * (maxq / 32));
    xp_qh_ = dalloc<uint16_t>((size_t)cap * maxq);
    xp_sc_ = dalloc<double>((size_t)cap * hp_.n_head * max_ctx_);
    xp_cap_ = cap;
  }
  for (int c0 = 0; c0 < n; c0 += cap) {
    const int T = std::min(cap, n - c0);
    LLMI_HIP(hipMemcpyAsync(xp_tok_, tokens + c0, (size_t)T * 4, hipMemcpyHostToDevice, s));
    LLMI_HIP(hipStreamSynchronize(s));  // (the host array may go away)
    set_token_pos(tokens[c0], pos + c0, c0 == 0);  // d_pos: the chunk's first position
    for (int l = 0; l < hp_.n_layer; l++) {
      LayerDev& Ld = L_[l];
      XpNormArgs na;  // residual step + attn_norm, or the embedding (model.cpp:709-736, 843-858)
      na.resid = xp_resid_;
      na.w_next = Ld.attn_norm;
      na.xq = xp_xq_;
      na.n = E;
      na.eps = hp_.eps;
      if (l == 0) {
        na.table = embd_raw_;
        na.row_bytes = embd_row_bytes_;
        na.type = embd_.type;
        na.tokens = xp_tok_;
        na.emb_scale = std::sqrt(static_cast<float>(E));  // model.cpp:337-338
      } else {
        na.y = xp_d_;
        na.w_post = L_[l - 1].post_ffw_norm;
      }
      launch_exact_norm_batch(na, T, s);
      launch_exact_gemm(Ld.xqkv, xp_xq_, T, xp_qkv_, Ld.qkv_rows, nullptr, s);
      XAttnArgs xa;
      xa.qkv = xp_qkv_;
      xa.qkv_stride = Ld.qkv_rows;
      xa.k_off = Ld.k_off;
      xa.v_off = Ld.v_off;
      xa.n_head = hp_.n_head;
      xa.n_head_kv = hp_.n_head_kv;
      xa.head_dim = Ld.hd;
      xa.q_norm_w = Ld.q_norm;
      xa.k_norm_w = Ld.k_norm;
      xa.rope_cs = Ld.is_swa ? rope_swa_ : rope_glb_;
      xa.attn_scale = hp_.attn_scale;
      xa.eps = hp_.eps;
      xa.k_cache = Ld.kc;
      xa.v_cache = Ld.vc;
      xa.max_ctx = max_ctx_;
      xa.d_pos = d_pos_;
      xa.scores = xp_sc_;
      xa.out = xp_att_;
      xa.xq = xp_axq_;
      xa.softcap = hp_.attn_softcap;
      xa.vt = Ld.vt;
      xa.vt_stride = xa_vt_stride_;
      xa.kmeta = Ld.kmeta;
      xa.qh = xp_qh_;
      launch_exact_attn_batch(xa, T, s);
      if (l + 1 == hp_.n_layer) break;  // the last layer's K / V are in the cache: nothing after it is kept
      launch_exact_gemm(Ld.xo, xp_axq_, T, xp_o_, E, nullptr, s);
      XpNormArgs nf;  // post-attention norm + residual, ffn_norm (model.cpp:843-858, 872-881)
      nf.y = xp_o_;
      nf.w_post = Ld.post_attn_norm;
      nf.resid = xp_resid_;
      nf.w_next = Ld.ffn_norm;
      nf.xq = xp_xq_;
      nf.n = E;
      nf.eps = hp_.eps;
      launch_exact_norm_batch(nf, T, s);
      launch_exact_gemm(Ld.xgu, xp_xq_, T, nullptr, 0, xp_hq_, s);
      launch_exact_gemm(Ld.xdn, xp_hq_, T, xp_d_, E, nullptr, s);
    }
  }
}

void Session::record_layers(hipStream_t s, bool x_q8) {
  const int E = hp_.n_embd, F = hp_.n_ff;
  auto is_q8 = [](uint32_t t) { return t == T_Q4_0 || t == T_Q8_0; };
  auto nout = [&](const std::vector<GemvPart>& consumer) {
    NormOut o;
    o.xn = xn_;
    bool q8 = !consumer.empty(), q8k = !consumer.empty();
    for (const auto& p : consumer) {
      q8 &= is_q8(p.w.type);
      q8k &= (p.w.type == T_Q4_K || p.w.type == T_Q6_K) && p.w.cols % 256 == 0;
    }
    if (q8) o.q8 = act_.q8.xb;
    if (q8k && !ex_norm_) o.q8k = act_.q8k;  // exact mode keeps the reference's separate quantize launch
    return o;
  };
  for (int l = 0; l < hp_.n_layer; l++) {
    LayerDev& Ld = L_[l];
    const int hd = Ld.hd;
    for (int r = 0; r < dup("qkv"); r++) gemv_parts(Ld.qkv, xn_, E, qkv_, s, x_q8);
    const std::string L = std::to_string(l);
    dump("Qcur-" + L, qkv_, hp_.n_head * hd, s);
    if (Ld.has_kv) {
      dump("Kcur-" + L, qkv_ + Ld.k_off, hp_.n_head_kv * hd, s);
      dump("Vcur-" + L, qkv_ + Ld.v_off, hp_.n_head_kv * hd, s);
    }
    QKVArgs qa{qkv_, Ld.k_off, Ld.v_off, hp_.n_head, hp_.n_head_kv, hd, Ld.q_norm, Ld.k_norm,
               Ld.is_swa ? rope_swa_ : rope_glb_, hp_.attn_scale, hp_.eps, q_, Ld.kc, Ld.vc, max_ctx_, d_pos_};
    qa.has_kv = Ld.has_kv;
    qa.v_norm = hp_.gemma4 && Ld.has_kv;  // model.cpp:813-829
    // norm/rope/KV-append inside the attention launch (Gemma-3 rows only)
    const bool fuse_qk = !ex_attn_ && !ex_norm_ && Ld.has_kv && !qa.v_norm && hp_.n_head <= 4 * hp_.n_head_kv;
    if (!fuse_qk) {
      launch_qk_norm_rope_kv(qa, ex_norm_, s);
      kernels_per_token_++;
    }
    const bool o_q8 = is_q8(Ld.o.w.type);
    const bool fused_q8 = !ex_attn_ && o_q8 && hd % 32 == 0;
    AttnArgs aa{q_, Ld.kc, Ld.vc, hp_.n_head, hp_.n_head_kv, hd, max_ctx_, d_pos_, part_, attn_,
                ticket_, fused_q8 ? act_.q8.xb : nullptr};
    aa.softcap = hp_.attn_softcap;
    for (int r = 0; r < dup("attn"); r++) launch_attention(aa, ex_attn_, s, fuse_qk ? &qa : nullptr);
    kernels_per_token_++;
    dump("kqv_out-" + L, attn_, hp_.n_head * hd, s);
    for (int r = 0; r < dup("o_proj"); r++) gemv_parts({Ld.o}, attn_, hp_.n_head * hd, o_out_, s, fused_q8);
    dump("attention results (node_30 for MUL_MAT)-" + L, o_out_, E, s);
    NormOut o1 = nout(Ld.gate_up);
    launch_residual_norm(o_out_, Ld.post_attn_norm, resid_, Ld.ffn_norm, o1, E, hp_.eps, ex_norm_, s);
    dump("sa_out-" + L, resid_, E, s);
    dump("ffn_norm-" + L, xn_, E, s);
    if (dup("norm") > 1)  // ablation: the same launch on a scratch residual (values irrelevant)
      launch_residual_norm(o_out_, Ld.post_attn_norm, resid_scratch_, Ld.ffn_norm, o1, E, hp_.eps, ex_norm_, s);
    kernels_per_token_++;
    for (int r = 0; r < dup("gate_up"); r++)
      gemv_parts(Ld.gate_up, xn_, E, gu_, s, o1.q8 != nullptr || o1.q8k != nullptr);
    const bool d_q8 = Ld.down.w.type == T_Q4_0 || Ld.down.w.type == T_Q8_0;
    const bool d_q8k = !ex_norm_ && (Ld.down.w.type == T_Q4_K || Ld.down.w.type == T_Q6_K) && F % 256 == 0;
    for (int r = 0; r < dup("gelu"); r++)
      launch_gelu_quant(gu_, F, hid_, d_q8 ? &act_.q8 : nullptr, s, d_q8k ? act_.q8k : nullptr);
    kernels_per_token_++;
    dump("ffn_geglu-" + L, hid_, F, s);
    for (int r = 0; r < dup("down"); r++) gemv_parts({Ld.down}, hid_, F, d_out_, s, d_q8 || d_q8k);
    dump("ffn_out-" + L, d_out_, E, s);
    const bool last = l + 1 == hp_.n_layer;
    const float* w_next = last ? out_norm_ : L_[l + 1].attn_norm;
    NormOut o2 = last ? NormOut{} : nout(L_[l + 1].qkv);
    o2.xn = xn_;
    if (last && embd_.type == T_F16) o2.x16 = act_.x16;  // logits input, ops.cpp:542-551
    if (last) screen_norm(o2);
    if (ple_table_.qs) {  // Gemma-4 per-layer embedding step (model.cpp:926-966), then the output scale
      const int EP = hp_.n_epl;
      launch_residual_norm(d_out_, Ld.post_ffw_norm, resid_, w_next, NormOut{xn_}, E, hp_.eps, ex_norm_, s);
      gemv_parts({Ld.ple_gate}, resid_, E, ple_g_, s, false);
      launch_gelu_mul(ple_g_, inp_pl_ + (size_t)l * EP, ple_u_, EP, s);
      gemv_parts({Ld.ple_proj}, ple_u_, EP, ple_tmp_, s, false);
      launch_residual_norm(ple_tmp_, Ld.ple_post_norm, resid_, w_next, o2, E, hp_.eps, ex_norm_, s, Ld.out_scale);
      kernels_per_token_ += 3;
    } else {
      launch_residual_norm(d_out_, Ld.post_ffw_norm, resid_, w_next, o2, E, hp_.eps, ex_norm_, s, Ld.out_scale);
    }
    x_q8 = o2.q8 != nullptr || o2.q8k != nullptr;
    kernels_per_token_++;
    dump("l_out-" + L, resid_, E, s);
    dump(last ? std::string("result_norm") : "attn_norm-" + std::to_string(l + 1), xn_, E, s);
  }
}

void Session::ensure_graph(int kind) {
  hipGraph_t& g = graphs_[kind];
  hipGraphExec_t& ge = graph_execs_[kind];
  if (!use_graph_ || ge) return;
  const bool gen = kind == STEP_GEN;
  LLMI_HIP(hipStreamBeginCapture(stream_, hipStreamCaptureModeThreadLocal));
  try {
    record_step(stream_, gen, gen, kind != STEP_HIDDEN);
  } catch (...) {
    hipGraph_t gg;
    (void)hipStreamEndCapture(stream_, &gg);
    throw;
  }
  LLMI_HIP(hipStreamEndCapture(stream_, &g));
  LLMI_HIP(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
}

// gen: a decode-loop step (only the token id is kept); otherwise the full
// logits vector is produced (forward)
// the fused exchanges' device-resident link, once the collective is connected (before the first recorded step:
// no allocation or copy inside a graph capture)
void Session::px_prepare() {
  if (!px_fused_ || d_px_) return;
  PxLink l;
  coll_->fused_link(l);
  PxLink* d = dalloc<PxLink>(1);
  h2d(d, &l, sizeof(l));
  d_px_ = d;
}

void Session::run_step(int kind) {
  px_prepare();
  if (kind == STEP_GEN && !screen_) kind = STEP_LOGITS;
  // a tensor-parallel rank keeps the logits of every step: the standalone exchanges of the skipped launches are
  // counted by every rank alike, but the argmax keys' all-gather is part of the logits tail
  if (kind == STEP_HIDDEN && tp_) kind = STEP_LOGITS;
  if (use_graph_) {
    ensure_graph(kind);
    LLMI_HIP(hipGraphLaunch(graph_execs_[kind], stream_));
  } else {
    record_step(stream_, kind == STEP_GEN, false, kind != STEP_HIDDEN);
  }
}

// The token and position travel as kernel arguments of a one-thread launch in stream order.  (Round 2 staged
// them in a pinned buffer: a hipStreamSynchronize + two 4-byte H2D copies before every step-graph replay of the
// token loop; under rocprofv3 --kernel-trace that sequence aborted after ~33 replays with
// HSA_STATUS_ERROR_INVALID_PACKET_FORMAT, while the decode loop -- replays only -- profiled clean.)
void Session::set_token_pos(int32_t token, int pos, bool reset_ring) {
  launch_set_token_pos(d_token_, d_pos_, ring_idx_, token, pos, reset_ring, stream_);
}

void Session::ensure_usable() const {
  if (broken_)
    throw status_error(LLMI_E_HIP, "tensor-parallel session unusable after a failed exchange (its exchange count may "
                                   "differ from its peers'): destroy and re-create every rank's session");
}

template <class F> void Session::tp_guarded(F&& f) {
  ensure_usable();
  try {
    f();
  } catch (...) {
    if (tp_) broken_ = true;
    throw;
  }
}

void Session::forward(const int32_t* tokens, int n, int pos, float* logits, int32_t* argmax) {
  if (n <= 0) throw status_error(LLMI_E_ARG, "forward: no tokens");
  if (pos < 0 || pos + n > max_ctx_) throw status_error(LLMI_E_RANGE, "forward: context overflow");
  for (int i = 0; i < n; i++)
    if (tokens[i] < 0 || tokens[i] >= vocab_) throw status_error(LLMI_E_RANGE, "forward: token id out of range");
  tp_guarded([&] {
    if (n > 1 && prefill_ok_ && getenv("LLMI_NO_PREFILL") == nullptr) {
      set_token_pos(tokens[n - 1], pos + n - 1, true);  // what the token loop leaves behind
      prefill(tokens, n, pos);
    } else if (n > 1 && xp_ok()) {  // exact mode: the prompt but its last token batched, then the last one's step
      exact_prefill(tokens, n - 1, pos);
      set_token_pos(tokens[n - 1], pos + n - 1, false);
      run_step(STEP_LOGITS);
    } else {
      for (int i = 0; i < n; i++) {  // only the last token's logits are computed (model.cpp:983-1001)
        set_token_pos(tokens[i], pos + i, i == 0);
        run_step(i + 1 < n ? STEP_HIDDEN : STEP_LOGITS);
      }
    }
    // every rank of a tensor-parallel group gathers the full logits (collective)
    if (tp_) coll_->all_gather(logits_, (size_t)v_sh_ * sizeof(float), stream_, px_take());
    if (logits) LLMI_HIP(hipMemcpyAsync(logits, logits_, (size_t)vocab_ * 4, hipMemcpyDeviceToHost, stream_));
    if (argmax) LLMI_HIP(hipMemcpyAsync(argmax, d_token_, 4, hipMemcpyDeviceToHost, stream_));
    LLMI_HIP(hipStreamSynchronize(stream_));
    check_device_error();
  });
}

// tensor.h print_tensor_generic for a {n, 1, 1, 1} tensor: 3 leading and 3
// trailing values ("%12.4f") around "..., " when n > 6, then the float
// left-to-right sum (std::accumulate) as "sum = %.6f"
void Session::dump(const std::string& name, const float* dev, int n, hipStream_t s) {
  if (!dump_) return;
  LLMI_HIP(hipStreamSynchronize(s));
  std::vector<float> h((size_t)n);
  LLMI_HIP(hipMemcpy(h.data(), dev, (size_t)n * 4, hipMemcpyDeviceToHost));
  std::fprintf(dump_, "%s = {%d, 1, 1, 1}\n    [\n     [\n      [", name.c_str(), n);
  for (int i = 0; i < n; i++) {
    if (i == 3 && n > 6) {
      std::fprintf(dump_, "..., ");
      i = n - 3;
    }
    std::fprintf(dump_, "%12.4f", h[(size_t)i]);
    if (i < n - 1) std::fprintf(dump_, ", ");
  }
  float sum = 0.0f;
  for (float v : h) sum += v;
  std::fprintf(dump_, "],\n     ],\n    ]\n    sum = %.6f\n", sum);
}

void Session::tap(const char* name, int layer, const void* dev, size_t bytes, hipStream_t s) {
  if (!trace_fn_) return;
  LLMI_HIP(hipStreamSynchronize(s));
  std::vector<uint8_t> h(bytes);
  LLMI_HIP(hipMemcpy(h.data(), dev, bytes, hipMemcpyDeviceToHost));
  trace_fn_(trace_user_, name, layer, h.data(), bytes);
}

// llmi_session_trace: the launches of forward() (batched prefill for n > 1
// when the session runs it, else the token loop) or of one decode-loop step
// (gen), eager, each followed by host copies of what it produced
void Session::forward_trace(const int32_t* tokens, int n, int pos, bool gen, llmi_trace_fn fn, void* user) {
  if (n <= 0) throw status_error(LLMI_E_ARG, "trace: no tokens");
  if (pos < 0 || pos + n > max_ctx_) throw status_error(LLMI_E_RANGE, "trace: context overflow");
  for (int i = 0; i < n; i++)
    if (tokens[i] < 0 || tokens[i] >= vocab_) throw status_error(LLMI_E_RANGE, "trace: token id out of range");
  // (a tensor-parallel rank traces too -- every rank of the group must call it: the standalone exchanges run)
  const bool graph = use_graph_;
  use_graph_ = false;
  trace_fn_ = fn;
  trace_user_ = user;
  auto done = [&] {
    trace_fn_ = nullptr;
    trace_user_ = nullptr;
    use_graph_ = graph;
  };
  try {
    if (n > 1 && prefill_ok_ && getenv("LLMI_NO_PREFILL") == nullptr) {
      set_token_pos(tokens[n - 1], pos + n - 1, true);
      prefill(tokens, n, pos);
    } else {
      for (int i = 0; i < n; i++) {
        set_token_pos(tokens[i], pos + i, i == 0);
        record_step(stream_, gen && screen_);
      }
    }
    LLMI_HIP(hipStreamSynchronize(stream_));
  } catch (...) {
    done();
    throw;
  }
  done();
  check_device_error();
}

void Session::forward_dump(const int32_t* tokens, int n, int pos, const char* path) {
  if (n <= 0) throw status_error(LLMI_E_ARG, "dump: no tokens");
  if (pos < 0 || pos + n > max_ctx_) throw status_error(LLMI_E_RANGE, "dump: context overflow");
  for (int i = 0; i < n; i++)
    if (tokens[i] < 0 || tokens[i] >= vocab_) throw status_error(LLMI_E_RANGE, "dump: token id out of range");
  if (tp_) throw status_error(LLMI_E_ARG, "dump: one device only");
  std::FILE* f = std::fopen(path, "a");
  if (!f) throw status_error(LLMI_E_ARG, std::string("dump: cannot open ") + path);
  const bool graph = use_graph_;
  use_graph_ = false;  // eager: every launch can be followed by a copy
  dump_ = f;
  auto done = [&] {
    dump_ = nullptr;
    use_graph_ = graph;
    std::fclose(f);
  };
  try {
    for (int i = 0; i < n; i++) {
      set_token_pos(tokens[i], pos + i, i == 0);
      record_step(stream_, false);
    }
    LLMI_HIP(hipStreamSynchronize(stream_));
  } catch (...) {
    done();
    throw;
  }
  done();
  check_device_error();
}

void Session::enqueue(int32_t first, int pos, int n_steps) {
  if (first < 0 || first >= vocab_) throw status_error(LLMI_E_RANGE, "token id out of range");
  if (pos < 0 || pos + n_steps > max_ctx_) throw status_error(LLMI_E_RANGE, "generate: context overflow");
  tp_guarded([&] {
    set_token_pos(first, pos, true);
    if (n_steps > 0 && screen_ && embed_fold_ok()) {  // the folded step graph starts at layer 0: the first embedding here
      const int E = hp_.n_embd;
      launch_embed_norm(embd_.type, embd_raw_, embd_row_bytes_, d_token_, std::sqrt(static_cast<float>(E)), resid_,
                        L_[0].attn_norm, embed_out(), E, hp_.eps, ex_norm_, stream_);
    }
    for (int i = 0; i < n_steps; i++) run_step(STEP_GEN);
  });
}

void Session::sync(int32_t* out, int n) {
  tp_guarded([&] {
    if (out && n > 0)
      LLMI_HIP(hipMemcpyAsync(out, ring_, (size_t)std::min(n, max_ctx_) * 4, hipMemcpyDeviceToHost, stream_));
    LLMI_HIP(hipStreamSynchronize(stream_));
    check_device_error();
  });
}

// a bounded in-kernel wait that gave up (k_attn.hip attention block): the
// results since the last check are invalid -- report it, never return them
void Session::peer_handle(void* out) const {
  if (!coll_) throw status_error(LLMI_E_ARG, "peer handle: not a tensor-parallel session");
  coll_->peer_handle(out);
}

void Session::peer_connect(const void* handles) {
  if (!coll_) throw status_error(LLMI_E_ARG, "peer connect: not a tensor-parallel session");
  if (!handles) throw status_error(LLMI_E_ARG, "peer connect: no handles");
  coll_->peer_connect(handles);
}

void Session::check_device_error() {
  if (const int e = coll_ ? coll_->failed() : 0) {  // the push exchange: a wait past its bound, or a bad checksum
    broken_ = true;
    throw status_error(LLMI_E_HIP, (e == 2 ? std::string("tensor-parallel push exchange: a received slice failed its "
                                                         "checksum (device results invalid)")
                                           : std::string("tensor-parallel push exchange: a peer's slice did not arrive "
                                                         "within LLMI_PX_TIMEOUT_MS (device results invalid)")) +
                                       coll_->fail_detail());
  }
  if (blk_trace_) {  // development: append the last traced launch (work-group x 8 clocks) to LLMI_BLOCK_TRACE_OUT
    std::vector<unsigned long long> h(4096 * 8);
    LLMI_HIP(hipMemcpy(h.data(), blk_trace_, h.size() * 8, hipMemcpyDeviceToHost));
    if (const char* path = getenv("LLMI_BLOCK_TRACE_OUT"))
      if (FILE* f = fopen(path, "ab")) {
        fwrite(h.data(), 8, h.size(), f);
        fclose(f);
      }
  }
  if (!blk_err_) return;
  int ev[2] = {0, 0};
  LLMI_HIP(hipMemcpyAsync(ev, blk_err_, sizeof(ev), hipMemcpyDeviceToHost, stream_));
  LLMI_HIP(hipStreamSynchronize(stream_));
  const int e = ev[0];
  if (ev[1]) {
    slow_waits_ += ev[1];
    LLMI_HIP(hipMemsetAsync(blk_err_ + 1, 0, sizeof(int), stream_));
    LLMI_HIP(hipStreamSynchronize(stream_));
  }
  if (e) {  // reported once: the flag and every attention ticket are cleared so the session's next call starts clean
    LLMI_HIP(hipMemsetAsync(blk_err_, 0, sizeof(int), stream_));
    LLMI_HIP(hipMemsetAsync(ticket_, 0, sizeof(unsigned) * (size_t)hp_.n_head, stream_));
    LLMI_HIP(hipStreamSynchronize(stream_));
    throw status_error(LLMI_E_HIP, "attention block: a cross-work-group wait timed out (device results invalid)");
  }
}

void Session::info(llmi_session_info* o) const {
  o->n_layer = hp_.n_layer;
  o->n_embd = hp_.n_embd;
  o->n_ff = hp_.n_ff;
  o->n_head = hp_.n_head;
  o->n_head_kv = hp_.n_head_kv;
  o->head_dim = hp_.hd_k;
  o->vocab = vocab_;
  o->max_ctx = max_ctx_;
  o->weight_bytes = weight_bytes_;
  o->tp_rank = tp_rank_;
  o->tp_size = tp_size_;
  o->batched_prefill = prefill_ok_ ? 1 : 0;
  o->screened_logits = screen_ ? 1 : 0;
  o->screen_bytes = screen_ ? scr_.bytes : 0;
  o->prefill_f16_redo = pf_f16_redo_;
  o->layer_engine = 0;  // (the round-3 engines were removed in round 6: DESIGN.md section 4.3)
  o->ffn_engine = 0;
  o->tp_exchange = coll_ ? (px_fused_ && coll_->kind() == EX_PUSH ? EX_PUSH_FUSED : coll_->kind()) : 0;
  o->block_slow_waits = slow_waits_;
  o->exact_engine = xl_ ? 1 : 0;
  o->exact_batched_prefill = xp_ok() ? 1 : 0;
  o->prefill_gemm = !prefill_ok_ ? 0 : prefill_f16_ok() ? (pf_kq_ ? 6 : 7) : 5;
  size_t b = logits_w_.bytes;  // this rank's bytes
  for (const auto& l : L_) {
    for (const auto& p : l.qkv) b += p.w.bytes;
    for (const auto& p : l.gate_up) b += p.w.bytes;
    b += l.o.w.bytes + l.down.w.bytes;
  }
  o->bytes_per_token = b;
  size_t kv = 0;
  for (const auto& l : L_) kv += (size_t)2 * nkv_ * l.hd * 2;
  o->kv_bytes_per_pos = kv;
  o->kernels_per_token = kernels_per_token_;
}

void Session::time_kernel(int which, int reps, double* us, double* bytes) {
  if (which == 1) {  // F16 logits GEMV (forward's full logits)
    *us = *bytes = 0.0;
    if (reps <= 0) return;
    std::vector<hipEvent_t> ev(2 * (size_t)reps);
    for (auto& e : ev) LLMI_HIP(hipEventCreate(&e));
    LLMI_HIP(hipStreamSynchronize(stream_));
    for (int r = 0; r < reps; r++) {
      LLMI_HIP(hipEventRecord(ev[2 * r], stream_));
      launch_gemv(logits_w_, act_, logits_, exact_ ? GEMV_EXACT : GEMV_FAST, stream_, amax_key_);
      LLMI_HIP(hipEventRecord(ev[2 * r + 1], stream_));
    }
    LLMI_HIP(hipStreamSynchronize(stream_));
    double tot = 0;
    for (int r = 0; r < reps; r++) {
      float ms = 0;
      LLMI_HIP(hipEventElapsedTime(&ms, ev[2 * r], ev[2 * r + 1]));
      tot += ms;
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    *us = tot * 1000.0 / reps;
    *bytes = (double)logits_w_.bytes;
    LLMI_HIP(hipMemsetAsync(amax_key_, 0, 8 * (size_t)tp_size_, stream_));
    LLMI_HIP(hipStreamSynchronize(stream_));
    return;
  }
  if (which == 2) {  // the decode loop's token selection: prep + screening GEMV + rescoring
    *us = *bytes = 0.0;
    if (!screen_ || reps <= 0) return;
    std::vector<hipEvent_t> ev(2 * (size_t)reps);
    for (auto& e : ev) LLMI_HIP(hipEventCreate(&e));
    LLMI_HIP(hipStreamSynchronize(stream_));
    for (int r = 0; r < reps; r++) {
      LLMI_HIP(hipEventRecord(ev[2 * r], stream_));
      launch_screen_argmax(logits_w_, scr_, act_.x16, amax_key_, stream_, false, ex_logits_);
      LLMI_HIP(hipEventRecord(ev[2 * r + 1], stream_));
    }
    LLMI_HIP(hipStreamSynchronize(stream_));
    double tot = 0;
    for (int r = 0; r < reps; r++) {
      float ms = 0;
      LLMI_HIP(hipEventElapsedTime(&ms, ev[2 * r], ev[2 * r + 1]));
      tot += ms;
    }
    for (auto& e : ev) (void)hipEventDestroy(e);
    *us = tot * 1000.0 / reps;
    *bytes = (double)scr_.bytes;
    LLMI_HIP(hipMemsetAsync(amax_key_, 0, 8 * (size_t)tp_size_, stream_));
    LLMI_HIP(hipStreamSynchronize(stream_));
    return;
  }
  // launches of one decode kernel family, each bracketed by events that its
  // own dispatch signals (hipExtLaunchKernel: the kernel's duration as
  // rocprofv3 reports it, no launch gap), on the session stream
  // (torch.cuda.Event would only see torch's stream), layers in decode order
  // so every launch streams its own weights from HBM.  Real arguments; the
  // prologues' residual writes go to a scratch buffer.
  //   0: attention block (qkv + attention + o; KV history at the current pos)
  //   3: gate_up (prologue + GELU)   4: down (QUANT)
  //   5: the r01 family: qkv PRO, o PLAIN, gate_up, down as standalone launches
  bool fused = fuse_layers_;
  for (const auto& l : L_) fused &= l.fused;
  if (!fused || (which == 0 && !block_) || which == 6 || which == 7 || which < 0 ||
      which > 7 || reps <= 0) {
    *us = *bytes = 0.0;
    return;
  }
  LLMI_HIP(hipStreamSynchronize(stream_));
  int pos = 0;
  LLMI_HIP(hipMemcpy(&pos, d_pos_, 4, hipMemcpyDeviceToHost));
  struct Item {
    std::function<void()> launch;
    double bytes;
  };
  std::vector<Item> items;
  for (size_t i = 0; i < L_.size(); i++) {
    LayerDev& Ld = L_[i];
    const int hd = Ld.hd;
    LayerGemv q;
    q.y = d_out_;
    q.w_post = i ? L_[i - 1].post_ffw_norm : Ld.post_ffw_norm;
    q.resid_in = resid_;
    q.resid_out = resid_scratch_;
    q.w_next = Ld.attn_norm;
    q.eps = hp_.eps;
    q.out = qkv_;
    if (which == 0) {
      const double kv = 2.0 * nkv_ * hd * 2.0 * (pos + 1);
      items.push_back({[this, &Ld, q, hd, i]() {
                         QKVArgs qa{qkv_, Ld.k_off, Ld.v_off, nh_, nkv_, hd, Ld.q_norm, Ld.k_norm,
                                    Ld.is_swa ? rope_swa_ : rope_glb_, hp_.attn_scale, hp_.eps, q_, Ld.kc, Ld.vc,
                                    max_ctx_, d_pos_};
                         AttnArgs aa{q_, Ld.kc, Ld.vc, nh_, nkv_, hd, max_ctx_, d_pos_, part_, attn_, ticket_, blk_xo_};
                         LayerGemv go;
                         go.xg = blk_xo_;
                         go.out = o_out_;
                         BlockSync bs;
                         bs.epoch = blk_epoch_ + i;  // (the launch advances it itself: every timed launch waits)
                         bs.done = blk_done_ + i * 32;
                         bs.g_qkv = blk_gqkv_ + i * blk_gqkv_stride_;
                         bs.g_xo = blk_gxo_ + i * blk_gxo_stride_;
                         bs.err = blk_err_;
                         aa.q8k = Ld.o.w.kq ? 1 : 0;
                         aa.softcap = hp_.attn_softcap;
                         LayerGemv qq = q;  // PLAIN block (27B): the x blocks of the last norm launch
                         if (!block_pro_) qq.xg = act_.q8.xb;
                         launch_attn_block(Ld.qkv[0].w, Ld.qkv.size() > 1 ? &Ld.qkv[1].w : nullptr, qq,
                                           block_pro_ ? LAYER_PRO : LAYER_PLAIN, Ld.o.w, go, aa, qa, bs, stream_);
                       },
                       (double)Ld.qkv[0].w.bytes + (double)Ld.o.w.bytes + kv});
    }
    if (which == 5) {
      items.push_back({[this, &Ld, q]() { launch_layer_gemv(Ld.qkv[0].w, q, LAYER_PRO, stream_); },
                       (double)Ld.qkv[0].w.bytes});
      LayerGemv o;
      o.xg = act_.q8.xb;
      o.out = o_out_;
      items.push_back({[this, &Ld, o]() { launch_layer_gemv(Ld.o.w, o, LAYER_PLAIN, stream_); }, (double)Ld.o.w.bytes});
    }
    if (which == 3 || which == 5) {
      LayerGemv gu = q;
      gu.w_next = Ld.ffn_norm;
      gu.out = nullptr;
      gu.hid = hid_;
      if (down_plain(Ld)) gu.hq = hq_;
      items.push_back({[this, &Ld, gu]() { launch_layer_gemv(Ld.gate_up[0].w, gu, LAYER_GELU, stream_); },
                       (double)Ld.gate_up[0].w.bytes});
    }
    if (which == 4 || which == 5) {
      LayerGemv d;
      d.y = hid_;
      d.xg = hq_;
      d.out = d_out_;
      const int drole = down_plain(Ld) ? LAYER_PLAIN : LAYER_QUANT;
      items.push_back({[this, &Ld, d, drole]() { launch_layer_gemv(Ld.down.w, d, drole, stream_); },
                       (double)Ld.down.w.bytes});
    }
  }
  std::vector<hipEvent_t> ev(2 * items.size() * reps);
  for (auto& e : ev) LLMI_HIP(hipEventCreate(&e));
  size_t k = 0;
  double tot_bytes = 0;
  for (int r = 0; r < reps; r++)
    for (size_t j = 0; j < items.size(); j++) {
      kernel_timing() = KernelTiming{ev[k], ev[k + 1]};
      k += 2;
      items[j].launch();
      tot_bytes += items[j].bytes;
    }
  LLMI_HIP(hipStreamSynchronize(stream_));
  check_device_error();
  double tot_ms = 0;
  for (size_t e = 0; e < k; e += 2) {
    float ms = 0;
    LLMI_HIP(hipEventElapsedTime(&ms, ev[e], ev[e + 1]));
    tot_ms += ms;
  }
  for (auto& e : ev) (void)hipEventDestroy(e);
  const double n = (double)(k / 2);
  *us = tot_ms * 1000.0 / n;
  *bytes = tot_bytes / n;
  LLMI_HIP(hipMemsetAsync(amax_key_, 0, 8 * (size_t)tp_size_, stream_));
  LLMI_HIP(hipStreamSynchronize(stream_));
}

}  // namespace llmi
