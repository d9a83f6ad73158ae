// attn.h -- argument blocks for the attention-side kernels (k_attn.hip).
#pragma once

#include "kernels.h"

namespace llmi {
struct LayerGemv;
struct BlockSync;
}

namespace llmi {

struct QKVArgs {
  const float* qkv;       // fused QKV GEMV output: q at 0, k at k_off, v at v_off
  int k_off, v_off;
  int n_head, n_head_kv, head_dim;
  const float* q_norm_w;  // [head_dim] f32 (attn_q_norm.weight)
  const float* k_norm_w;  // [head_dim] f32 (attn_k_norm.weight)
  const float* rope_cs;   // [max_ctx][head_dim/2][2] (cos, sin) for this layer's base
  float attn_scale;       // 1/sqrt(head_dim) (model.cpp:120)
  double eps;
  float* q_out;           // [n_head][head_dim]
  uint16_t* k_cache;      // [n_head_kv][max_ctx][head_dim]
  uint16_t* v_cache;
  int max_ctx;
  const int* d_pos;       // device position of this token
  int has_kv = 1;         // 0: shared-KV layer (model.cpp:775-777): q only, the cache is another layer's
  int v_norm = 0;         // 1: RMSNorm (no weight) of each V row before the append (Gemma-4, model.cpp:813-829)
};

constexpr int ATTN_NSPLIT = 32;  // key-range splits of the fast attention (work-groups per kv head)

struct AttnArgs {
  const float* q;         // [n_head][head_dim], normed/roped/scaled
  const uint16_t* k_cache;
  const uint16_t* v_cache;
  int n_head, n_head_kv, head_dim, max_ctx;
  const int* d_pos;       // keys 0..*d_pos are attended (no window: model.cpp:501)
  float* partial;         // fast path scratch [n_head][ATTN_NSPLIT][head_dim + 2]
  float* out;             // [n_head][head_dim]
  unsigned* ticket;       // fast path: [n_head_kv] zeroed counters (reset by the kernel)
  XBlock* q8;             // optional: Q8_0 blocks of out (head_dim % 32 == 0)
  int q8k = 0;            // 1: q8 holds Q8_K quants instead (q8k_block_quad; G * head_dim % 256 == 0): kq o projection
  float softcap = 0.0f;   // attention.logit_softcapping (model.cpp:511-513); 0: none
};

void launch_qk_norm_rope_kv(const QKVArgs& a, bool exact, hipStream_t s);
// exact: attn_exact_kernel -> out.  fast: one split-K launch whose last
// work-group per kv head merges the partials (-> out, and Q8_0 blocks of out
// when a.q8 != nullptr and head_dim % 32 == 0).
// fused != nullptr (fast path only): the kernel also does the q/k norm +
// rope + q scale + KV append of qk_norm_rope_kv (one launch fewer).
void launch_attention(const AttnArgs& a, bool exact, hipStream_t s, const QKVArgs* fused = nullptr);
// qkv GEMV (qrole LAYER_PLAIN / LAYER_PRO) + fused attention + o GEMV in one
// launch (k_attn.hip, attention block); qg.out must be qa.qkv, og.xg must be
// aa.q8.  attn_block_supported: a launch-table entry exists for the shapes and
// the qkv role (LAYER_PLAIN: x blocks given; LAYER_PRO: residual + norms in the
// launch's prologue), and its grid is co-resident.
// wqkv_b: the second qkv weight of a q|k Q4_K + v Q6_K layer (kq layout), or null
bool attn_block_supported(const DevWeight& wqkv, const DevWeight* wqkv_b, const DevWeight& wo, int head_dim,
                          int n_head, int n_head_kv, int qrole);
// returns the o projection's work-group count (the producers of its fused exchange)
int launch_attn_block(const DevWeight& wqkv, const DevWeight* wqkv_b, LayerGemv qg, int qrole, const DevWeight& wo,
                       LayerGemv og,
                       const AttnArgs& aa, const QKVArgs& qa, BlockSync bs, hipStream_t s);

}  // namespace llmi
