// k_layer.hip -- the decode step's Q4_0 GEMVs with their neighbours fused in.
//
// One launch per projection instead of norm / quantize / GEMV / GELU launches.
// Roles (what a work-group does around the weight stream):
//   PLAIN : the activation's Q8_0 blocks are copied global -> LDS.
//   PRO   : the residual step that precedes the GEMV (model.cpp:843-858 and
//           915-924 + the next run_norm) is recomputed by every work-group
//           from the previous GEMV's output -- h = resid + rms(y)*w_post,
//           x = rms(h)*w_next, Q8_0 blocks of x (ops.cpp:116-139) -- into LDS.
//           Work-group 0 publishes h (resid_out, a ping-pong buffer: the other
//           work-groups of the same launch still read resid_in).
//   GELU  : PRO, and gate/up rows interleaved in groups of H at upload, so a
//           work-group of 2H rows owns gate[Hb..Hb+H) and up[Hb..Hb+H) and
//           finishes GELU(gate)*up (model.cpp:892-899) for those H units.
//   QUANT : the f32 activation (the GELU output) is quantized to Q8_0 blocks
//           into LDS, one block per thread (no cross-lane reductions).
// Geometry: one fat work-group per CU where the prologue is per-work-group
// work (PRO/GELU/QUANT), so that work is done 256 times, not once per 16 rows.
// The weight stream is the gemv_q4_0_fast scheme (k_gemv.hip): a wave owns R
// rows as a flat (row, block) item list, one 16-B non-temporal load per lane
// per pass, a chunk of P passes in flight.  The activation (with its
// prologue) is complete in LDS before the weights are issued (see the note at
// the weight issue).
#include "session_kernels.h"

#include <hip/hip_ext.h>

#include "layer_body.h"

namespace llmi {

namespace {

// PXF: the fused-exchange variant (tensor-parallel ranks: a.px set; layer_body PXF)
template <int R, int NW, int P, int E, int ROLE, bool MULTI, bool EARLY, int PE = 0, bool W8 = false, int WT = 0,
          int RW = 0, bool PXF = false>
__global__ __launch_bounds__(NW * 64 + (role_help(ROLE) ? E * 64 : 0)) void gemv_q4_0_layer(LayerGemv a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  layer_body<R, NW, P, E, ROLE, MULTI, EARLY, 0, PE, W8, WT, RW, PXF>(a, blockIdx.x, s_dyn, BlockSync{});
}

// K-quant q|k|v of two weight types in one launch (Q4_K_M: q, k Q4_K, v Q6_K):
// work-groups [0, nwg_a) stream the first weight, the rest the second; both
// run the same prologue (b has no resid_out / xn_out: work-group 0 of a
// publishes them)
template <int R, int NW, int P, int E, int ROLE, bool EARLY, int PE, int WTA, int WTB>
__global__ __launch_bounds__(NW * 64) void gemv_kq2_layer(LayerGemv a, LayerGemv b, int nwg_a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  if ((int)blockIdx.x < nwg_a)
    layer_body<R, NW, P, E, ROLE, false, EARLY, 0, PE, false, WTA>(a, blockIdx.x, s_dyn, BlockSync{});
  else
    layer_body<R, NW, P, E, ROLE, false, EARLY, 0, PE, false, WTB>(b, blockIdx.x - nwg_a, s_dyn, BlockSync{});
}

// ---- launch table ----------------------------------------------------------
// One instantiation per (activation length, role) of the Gemma-3 1B/4B/12B/27B
// projections; shapes outside the table take the unfused path (session.cpp).
// Geometry aims at ~256 work-groups (one per CU) so per-work-group prologue
// work is done once per CU and every CU streams the same bytes:
//   R: rows per wave, NW: waves per work-group, P: passes (64 items) per
//   chunk, MULTI: more than one chunk per wave, EARLY: see the kernel,
//   E: PLAIN -- 16-B x loads per thread (ceil(3 nb / 64 NW));
//      PRO/GELU -- prologue elements per thread (ceil(32 nb / 64 NW));
//      QUANT -- rounds of 8-float quad lanes (ceil(4 nb / 64 NW)).
using LaunchFn = void (*)(dim3, size_t, const LayerGemv&, hipStream_t);
using Launch2Fn = void (*)(dim3, size_t, const LayerGemv&, const LayerGemv&, int, hipStream_t);

template <int R, int NW, int P, int E, int ROLE, bool MULTI, bool EARLY, int PE = 0, bool W8 = false, int WT = 0,
          int RW = 0>
void launch_cfg(dim3 grid, size_t lds, const LayerGemv& a, hipStream_t s) {
  const dim3 block(NW * 64 + (role_help(ROLE) ? E * 64 : 0));
  if (a.px) {  // the fused-exchange variant (tensor-parallel ranks)
    hipLaunchKernelGGL((gemv_q4_0_layer<R, NW, P, E, ROLE, MULTI, EARLY, PE, W8, WT, RW, true>), grid, block, lds, s, a);
    return;
  }
  KernelTiming& kt = kernel_timing();
  if (kt.start) {
    hipExtLaunchKernelGGL((gemv_q4_0_layer<R, NW, P, E, ROLE, MULTI, EARLY, PE, W8, WT, RW>), grid, block, (uint32_t)lds,
                          s, kt.start, kt.stop, 0u, a);
    kt = KernelTiming{};
    return;
  }
  hipLaunchKernelGGL((gemv_q4_0_layer<R, NW, P, E, ROLE, MULTI, EARLY, PE, W8, WT, RW>), grid, block, lds, s, a);
}

template <int R, int NW, int P, int E, int ROLE, bool EARLY, int PE, int WTA, int WTB>
void launch_cfg2(dim3 grid, size_t lds, const LayerGemv& a, const LayerGemv& b, int nwg_a, hipStream_t s) {
  hipLaunchKernelGGL((gemv_kq2_layer<R, NW, P, E, ROLE, EARLY, PE, WTA, WTB>), grid, dim3(NW * 64), lds, s, a, b, nwg_a);
}
// the two-weight launch exists for the qkv roles of the Q4_K entries only
template <int R, int NW, int P, int E, int ROLE, bool EARLY, int PE, int WT>
constexpr Launch2Fn fn2_of() {
  if constexpr ((ROLE == ROLE_PRO || ROLE == ROLE_PLAIN) && WT == WT_Q4_K)
    return launch_cfg2<R, NW, P, E, ROLE, EARLY, PE, WT_Q4_K, WT_Q6_K>;
  else
    return nullptr;
}

struct LayerCfg {
  int nb, role, R, NW, P, E;
  bool multi;
  int slab;  // weight layout this entry reads (sweep: slab pays for R >= 4 on big matrices)
  bool help;  // PRO/GELU with E helper waves (role_help)
  LaunchFn fn;
  bool w8 = false;  // Q8_0 weights (P counts half-block passes)
  int wt = 0;       // kq weights: WT_Q4_K / WT_Q6_K
  Launch2Fn fn2 = nullptr;  // kq: q|k Q4_K + v Q6_K in one launch (PRO / PLAIN qkv entries)
  int rows_max = 0;  // > 0: a tensor-parallel shard entry, for weights of at most this many rows
  int rw = 0;        // > 0: waves carrying rows (layer_body RW), the others only share the prologue
};

#define LLMI_LCFG(NB, ROLE, R, NW, P, E, MULTI, EARLY, SLAB) \
  {NB, ROLE, R, NW, P, E, MULTI, SLAB, false, launch_cfg<R, NW, P, E, ROLE, MULTI, EARLY>}
// shard entries (tensor-parallel ranks' row slices, at most RMAX rows): the whole matrix's entry with fewer waves
// per work-group, so a slice still puts work-groups on most CUs.  Only roles whose per-row arithmetic does not
// depend on NW (PLAIN: x blocks copied; QUANT: per-block quantization) and with the whole entry's R and P (a
// row's lane split and pass order): a rank's rows stay bit-identical to the one-device session's
#define LLMI_LCFGR(NB, ROLE, R, NW, P, E, MULTI, EARLY, SLAB, RMAX) \
  {NB, ROLE, R, NW, P, E, MULTI, SLAB, false, launch_cfg<R, NW, P, E, ROLE, MULTI, EARLY>, false, 0, nullptr, RMAX}
// PRO / GELU shards: all NW waves run the prologue (its reductions unchanged), RW of them carry rows
#define LLMI_LCFGW(NB, ROLE, R, NW, P, E, MULTI, EARLY, RW, RMAX)                                                  \
  {NB, ROLE, R, NW, P, E, MULTI, 0, false, launch_cfg<R, NW, P, E, ROLE, MULTI, EARLY, 0, false, 0, RW>, false, 0, \
   nullptr, RMAX, RW}
#define LLMI_LCFGPR(NB, ROLE, R, NW, P, E, SLAB, PE, RMAX) \
  {NB, ROLE, R, NW, P, E, false, SLAB, false, launch_cfg<R, NW, P, E, ROLE, false, false, PE>, false, 0, nullptr, RMAX}
// late roles with the first PE passes issued right after the prologue's loads
#define LLMI_LCFGP(NB, ROLE, R, NW, P, E, SLAB, PE) \
  {NB, ROLE, R, NW, P, E, false, SLAB, false, launch_cfg<R, NW, P, E, ROLE, false, false, PE>}
// Q8_0 weights: row-major, single chunk (P passes of 16-B half blocks)
// kq entries, one per weight type (+ the q|k Q4_K, v Q6_K launch for qkv roles)
#define LLMI_LCFGK1(NB, ROLE, R, NW, P, E, EARLY, PE, WT, SLAB)                                        \
  {NB, ROLE, R, NW, P, E, false, SLAB, false, launch_cfg<R, NW, P, E, ROLE, false, EARLY, PE, false, WT>, false, WT, \
   fn2_of<R, NW, P, E, ROLE, EARLY, PE, WT>()}
#define LLMI_LCFGK(NB, ROLE, R, NW, P, E, EARLY, PE, SLAB)                                     \
  LLMI_LCFGK1(NB, ROLE, R, NW, P, E, EARLY, PE, WT_Q4_K, SLAB), \
      LLMI_LCFGK1(NB, ROLE, R, NW, P, E, EARLY, PE, WT_Q6_K, SLAB)
#define LLMI_LCFG8(NB, ROLE, R, NW, P, E, EARLY) \
  {NB, ROLE, R, NW, P, E, false, 0, false, launch_cfg<R, NW, P, E, ROLE, false, EARLY, 0, true>, true}
// late W8 roles with the first PE passes issued right after the prologue's loads
#define LLMI_LCFG8P(NB, ROLE, R, NW, P, E, PE) \
  {NB, ROLE, R, NW, P, E, false, 0, false, launch_cfg<R, NW, P, E, ROLE, false, false, PE, true>, true}
#ifndef LLMI_W8_GELU_PE
#define LLMI_W8_GELU_PE 7  // 1B Q8_0 gate_up: PE 0 / 3 / 5 / 7 / 8 = 6.71 / 6.39 / 6.23 / 5.68 / 6.24 us
#endif
// PRO / GELU entries with NH helper waves (template role ROLE_PRO_H / ROLE_GELU_H)
#define LLMI_LCFGH(NB, ROLE, R, NW, P, NH, MULTI, SLAB) \
  {NB, ROLE, R, NW, P, NH, MULTI, SLAB, true,          \
   launch_cfg<R, NW, P, NH, ROLE == ROLE_PRO ? ROLE_PRO_H : ROLE_GELU_H, MULTI, true>}
// (scripts/gemv_sweep: 4B gate_up GELU 9.1 -> 8.5 us with R8 NW10 slab, 7.8
// us issuing 7 of its 10 passes before the prologue (PE7; all 10: 8.8 us);
// 4B down 5.8 -> 5.4 us with PE3 (of 5) instead of EARLY; 27B
// gate_up 35.8 -> 26.3 us with R8 NW8 P4 slab, qkv 10.4 -> 10.0 us, down
// 24 -> 17-19.5 us issuing the weights after the quantized x is in LDS)
#ifndef KQ_GU_SLAB
#define KQ_GU_SLAB 1
#endif
const LayerCfg kLayerCfgs[] = {
    // PLAIN: x blocks copied to LDS
    LLMI_LCFG(32, ROLE_PLAIN, 2, 2, 1, 1, false, true, 0),     // 1B o        1152 rows -> 288 WGs
    LLMI_LCFG(36, ROLE_PLAIN, 8, 1, 5, 2, false, true, 0),     // 1B qkv l0   1536 rows -> 192 WGs
    LLMI_LCFG(64, ROLE_PLAIN, 1, 10, 1, 1, false, true, 0),    // 4B o        2560 rows -> 256 WGs
    LLMI_LCFG(80, ROLE_PLAIN, 4, 4, 5, 1, false, true, 0),     // 4B qkv l0   4096 rows -> 256 WGs
    LLMI_LCFG(120, ROLE_PLAIN, 8, 4, 8, 2, true, true, 0),     // 12B qkv l0  8192 rows -> 256 WGs
    // (an o shard entry, NW 2: 4.60 vs 3.98 us per 27B tp-8 rank launch -- the x copy of 336 work-groups; dropped)
    LLMI_LCFG(128, ROLE_PLAIN, 1, 8, 2, 1, false, true, 0),    // 12B/27B o   3840/5376 rows -> 480/672 WGs
    // (27B qkv row-major: the attention block reads it so; slab-major was 10.0 vs 10.4 us standalone)
    LLMI_LCFG(168, ROLE_PLAIN, 8, 4, 7, 2, true, true, 0),     // 27B qkv l0  8192 rows -> 256 WGs
    // PRO: residual + norm prologue
    LLMI_LCFG(36, ROLE_PRO, 8, 2, 5, 9, false, true, 0),       // 1B qkv      96 WGs
    LLMI_LCFG(80, ROLE_PRO, 4, 4, 5, 10, false, true, 0),      // 4B qkv      256 WGs
    LLMI_LCFG(120, ROLE_PRO, 8, 4, 8, 15, true, true, 0),      // 12B qkv     256 WGs
    LLMI_LCFGW(168, ROLE_PRO, 4, 8, 6, 11, true, true, 1, 1024),  // 27B qkv shard (tp 8): 1 row wave -> 256 WGs
    LLMI_LCFGW(168, ROLE_PRO, 4, 8, 6, 11, true, true, 2, 2048),  // 27B qkv shard (tp 4): 2 row waves -> 256 WGs
    LLMI_LCFG(168, ROLE_PRO, 4, 8, 6, 11, true, true, 0),      // 27B qkv     256 WGs
    // GELU: prologue + GELU epilogue, 2H = R NW interleaved gate/up rows per WG
    LLMI_LCFGP(36, ROLE_GELU, 8, 8, 5, 3, 0, 3),              // 1B  13824 rows, H 32 -> 216 WGs (PE3: 5.9 -> 5.1 us)
    LLMI_LCFGP(80, ROLE_GELU, 8, 10, 10, 4, 1, 7),            // 4B  20480 rows, H 40 -> 256 WGs (PE7: 8.4 -> 7.8 us)
    LLMI_LCFG(120, ROLE_GELU, 8, 8, 8, 8, true, false, 0),     // 12B 30720 rows, H 32 -> 480 WGs
    // (a 27B gate_up shard entry with longer weight chunks -- P 7 or 11 instead of 4, more bytes in flight per
    // work-group of the tp-8 rank's 84; P does not change a row's pass order: 2.12-2.13 vs 2.08 ms per rank token,
    // and the 2-row-wave qkv shard 2.13; not kept)
    LLMI_LCFG(168, ROLE_GELU, 8, 8, 4, 11, true, false, 1),    // 27B 43008 rows, H 32 -> 672 WGs
    // PLAIN down: the GELU launch (32 units per work-group) wrote the Q8_0 blocks (LayerGemv::hq), so the down
    // launch copies 24-42 KB of blocks instead of quantizing the whole f32 hid in every work-group
    // (scripts/gemv_sweep 27b.down: plain R1 NW8 P6 15.0 us vs quant 19.5 us)
    LLMI_LCFG(216, ROLE_PLAIN, 1, 4, 4, 3, false, true, 0),    // 1B down     1152 rows -> 288 WGs
    LLMI_LCFGR(672, ROLE_PLAIN, 1, 4, 6, 8, true, true, 0, 2688),  // 27B down shard (tp 2-8) -> 168-672 WGs
    LLMI_LCFG(672, ROLE_PLAIN, 1, 8, 6, 4, true, true, 0),     // 27B down    5376 rows -> 672 WGs
    // QUANT: f32 activation quantized into LDS (down projection)
    LLMI_LCFG(216, ROLE_QUANT, 1, 4, 4, 4, false, true, 0),    // 1B down     1152 rows -> 288 WGs (6.5 -> 5.0 us)
    // (a 4B QUANT shard entry, NW 2: 0.948 vs 0.907 ms per tp-8 rank -- 160 work-groups each quantizing the
    // whole 40 KB hid; not kept)
    LLMI_LCFGP(320, ROLE_QUANT, 1, 10, 5, 2, 0, 3),           // 4B down     2560 rows -> 256 WGs (PE3: 5.8 -> 5.4 us)
    LLMI_LCFG(480, ROLE_QUANT, 1, 8, 8, 4, false, true, 0),    // 12B down    3840 rows -> 480 WGs
    LLMI_LCFG(672, ROLE_QUANT, 1, 8, 6, 6, true, false, 0),    // 27B down    5376 rows -> 672 WGs
    // Q8_0 weights (Gemma-3 1B Q8_0, BASELINE configs[3]): 2 nb half-block units per row
    LLMI_LCFG8(36, ROLE_PLAIN, 4, 2, 5, 1, true),     // 1B qkv l0   1536 rows -> 192 WGs
    LLMI_LCFG8(36, ROLE_PRO, 4, 4, 5, 5, true),       // 1B qkv      96 WGs
    LLMI_LCFG8(32, ROLE_PLAIN, 1, 4, 1, 1, true),     // 1B o        1152 rows -> 288 WGs
    LLMI_LCFG8P(36, ROLE_GELU, 8, 8, 9, 3, LLMI_W8_GELU_PE),  // 1B gate_up  13824 rows, H 32 -> 216 WGs
    LLMI_LCFG8(216, ROLE_QUANT, 1, 4, 7, 4, true),    // 1B down     1152 rows -> 288 WGs
    LLMI_LCFG8(216, ROLE_PLAIN, 1, 4, 7, 3, true),    // 1B down from the GELU launch's blocks
    // K-quant weights in the kq layout (Gemma-3 4B Q4_K_M, BASELINE configs[3]): the Q4_0 4B
    // geometry (a 32-element sub-block per 16-B unit, as a Q4_0 block), row-major
    LLMI_LCFGK(80, ROLE_PLAIN, 4, 4, 5, 1, true, 0, 0),      // 4B qkv l0   4096 rows -> 256 WGs
    LLMI_LCFGK(80, ROLE_PRO, 4, 4, 5, 10, true, 0, 0),       // 4B qkv      256 WGs
    LLMI_LCFGK(64, ROLE_PLAIN, 1, 10, 1, 1, true, 0, 0),     // 4B o        2560 rows -> 256 WGs
    LLMI_LCFGK(80, ROLE_GELU, 8, 10, 10, 4, false, 7, KQ_GU_SLAB),  // 4B gate_up  20480 rows, H 40 -> 256 WGs
    LLMI_LCFGK(320, ROLE_QUANT, 1, 10, 5, 2, false, 3, 0),   // 4B down     2560 rows -> 256 WGs
};
#undef LLMI_LCFG

int wt_of(uint32_t type) { return type == T_Q4_K ? WT_Q4_K : type == T_Q6_K ? WT_Q6_K : 0; }

// rows: the weight's row count (0: unknown -- only whole-matrix entries); shard entries come first in the table
const LayerCfg* find_cfg(int nb, int role, uint32_t type = T_Q4_0, int rows = 0) {
  if (type != T_Q4_0 && type != T_Q8_0 && type != T_Q4_K && type != T_Q6_K) return nullptr;
  for (const auto& c : kLayerCfgs) {
    if (c.rows_max > 0 && (rows <= 0 || rows > c.rows_max)) continue;
    if (c.nb == nb && c.role == role && c.w8 == (type == T_Q8_0) && c.wt == wt_of(type)) return &c;
  }
  return nullptr;
}

}  // namespace

#ifdef LLMI_LAYER_TRACE
void layer_set_trace(unsigned long long* p) { LLMI_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_layer_trace), &p, sizeof(p))); }
#endif

KernelTiming& kernel_timing() {
  thread_local KernelTiming kt;
  return kt;
}

bool layer_gemv_supported(const DevWeight& w, int role) {
  const bool k = w.type == T_Q4_K || w.type == T_Q6_K;
  if ((w.type != T_Q4_0 && w.type != T_Q8_0 && !k) || w.cols % (k ? 256 : 32) != 0 || w.rows <= 0) return false;
  const LayerCfg* c = find_cfg(w.cols / 32, role, w.type, w.rows);
  if (!c) return false;
  if ((role == LAYER_GELU || role == LAYER_GELU_X) && w.rows % (c->R * (c->rw ? c->rw : c->NW)) != 0) return false;
  return true;
}

int layer_gemv_slab(const DevWeight& w, int role) {
  const LayerCfg* c = w.cols % 32 == 0 ? find_cfg(w.cols / 32, role, w.type) : nullptr;
  return c ? c->slab : 0;
}

int layer_gemv_gelu_group(int cols, uint32_t type) {
  const LayerCfg* c = cols % 32 == 0 ? find_cfg(cols / 32, LAYER_GELU, type) : nullptr;
  return c ? c->R * (c->rw ? c->rw : c->NW) / 2 : 0;
}

int launch_layer_gemv(const DevWeight& w, LayerGemv a, int role, hipStream_t s) {
  if (!layer_gemv_supported(w, role)) throw std::runtime_error("layer gemv: unsupported weight");
  const bool pro = role == LAYER_PRO || role == LAYER_GELU;
  if (pro && (!a.y || !a.resid_in || !a.resid_out || !a.w_next || a.resid_in == a.resid_out))
    throw std::runtime_error("layer gemv: missing prologue operand");
  const bool xin = role == LAYER_PLAIN || role == LAYER_GELU_X;  // x blocks copied to LDS
  if (xin && !a.xg) throw std::runtime_error("layer gemv: missing activation blocks");
  if (role == LAYER_QUANT && !a.y) throw std::runtime_error("layer gemv: missing activation");
  if (role == LAYER_GELU || role == LAYER_GELU_X ? !a.hid : !a.out) throw std::runtime_error("layer gemv: missing output");
  const LayerCfg& c = *find_cfg(w.cols / 32, role, w.type, w.rows);
  const int nb = w.cols / 32, nu = c.w8 ? 2 * nb : nb;  // 16-B units per row
  const bool rb = c.R == 1 || c.R == 2 || c.R == 4 || c.R == 8 || c.R == 16;
  if (!c.multi && (rb ? (nu + 64 / c.R - 1) / (64 / c.R) > c.P : c.R * nb > 64 * c.P))
    throw std::runtime_error("layer gemv: table entry needs MULTI");
  if (pro && !c.help && w.cols > c.E * c.NW * 64) throw std::runtime_error("layer gemv: prologue E too small");
  if (pro && c.help && (w.cols % (c.E * 32) != 0 || w.cols > c.E * 256 * HELP_K4))
    throw std::runtime_error("layer gemv: helper segments must be whole Q8_0 blocks within HELP_K4");
  if (xin && 3 * nb > c.E * c.NW * 64) throw std::runtime_error("layer gemv: x copy E too small");
  if (role == LAYER_QUANT && 4 * nb > c.E * c.NW * 64) throw std::runtime_error("layer gemv: quant E too small");
  if (w.slab != c.slab) throw std::runtime_error("layer gemv: weight layout does not match the launch table");
  if (c.wt && !w.kq) throw std::runtime_error("layer gemv: K-quant weight not in the kq layout");
  if (c.rw && (w.slab || c.help || c.w8 || c.wt)) throw std::runtime_error("layer gemv: RW entries are row-major Q4_0");
  a.qs = reinterpret_cast<const uint4*>(w.qs);
  a.wd = w.d;
  a.kdd = w.kdd;
  a.kqh = w.kqh;
  a.slab = w.slab;
  a.rows = w.rows;
  a.nb = nb;
  a.magic = div_magic(nb);
  a.n = w.cols;
  // x blocks + pad slot of the x copy (+ the f32 x staging of the prologue)
  const size_t lds = (size_t)nb * sizeof(XBlock) + 16 + (pro ? (size_t)w.cols * 4 : 0);
  const int rows_per_wg = (c.rw ? c.rw : c.NW) * c.R;
  const int nwg = (w.rows + rows_per_wg - 1) / rows_per_wg;
  if (a.px && a.px_out >= 0 && nwg > PX_MAX_CS) throw std::runtime_error("layer gemv: more fused-exchange producers than checksum slots");
  if (a.px && a.px_in >= 0 && (a.px_in_nwg <= 0 || a.px_in_nwg > PX_MAX_CS)) throw std::runtime_error("layer gemv: fused exchange read without its producer count");
  c.fn(dim3(nwg), lds, a, s);
  LLMI_HIP(hipGetLastError());
  return nwg;
}

// q|k (Q4_K) and v (Q6_K) rows of one q|k|v projection in one launch: the
// outputs are contiguous (b's rows follow a's)
bool layer_gemv2_supported(const DevWeight& wa, const DevWeight& wb, int role) {
  if (wa.type != T_Q4_K || wb.type != T_Q6_K || wa.cols != wb.cols || wa.cols % 256) return false;
  if (!layer_gemv_supported(wa, role) || !layer_gemv_supported(wb, role)) return false;
  const LayerCfg* c = find_cfg(wa.cols / 32, role, wa.type);
  return c && c->fn2 && wa.rows % (c->NW * c->R) == 0;
}

void launch_layer_gemv2(const DevWeight& wa, const DevWeight& wb, LayerGemv a, int role, hipStream_t s) {
  if (!layer_gemv2_supported(wa, wb, role) || !wa.kq || !wb.kq) throw std::runtime_error("layer gemv2: unsupported");
  if (role == LAYER_PRO && (!a.y || !a.resid_in || !a.resid_out || !a.w_next || a.resid_in == a.resid_out))
    throw std::runtime_error("layer gemv2: missing prologue operand");
  if (role == LAYER_PLAIN && !a.xg) throw std::runtime_error("layer gemv2: missing activation blocks");
  if (role != LAYER_PRO && role != LAYER_PLAIN) throw std::runtime_error("layer gemv2: qkv roles only");
  const LayerCfg& c = *find_cfg(wa.cols / 32, role, wa.type);
  const int nb = wa.cols / 32;
  if ((nb + 64 / c.R - 1) / (64 / c.R) > c.P) throw std::runtime_error("layer gemv2: P too small");
  if (role == LAYER_PRO && wa.cols > c.E * c.NW * 64) throw std::runtime_error("layer gemv2: prologue E too small");
  if (role == LAYER_PLAIN && 3 * nb > c.E * c.NW * 64) throw std::runtime_error("layer gemv2: x copy E too small");
  a.rows = wa.rows;
  a.nb = nb;
  a.magic = div_magic(nb);
  a.n = wa.cols;
  a.slab = 0;
  LayerGemv b = a;
  a.qs = reinterpret_cast<const uint4*>(wa.qs);
  a.wd = wa.d;
  a.kdd = wa.kdd;
  a.kqh = wa.kqh;
  b.qs = reinterpret_cast<const uint4*>(wb.qs);
  b.wd = wb.d;
  b.kdd = wb.kdd;
  b.kqh = wb.kqh;
  b.rows = wb.rows;
  b.out = a.out + wa.rows;
  b.resid_out = nullptr;
  b.xn_out = nullptr;
  const int rpw = c.NW * c.R, nwa = wa.rows / rpw, nwb = (wb.rows + rpw - 1) / rpw;
  const size_t lds = (size_t)nb * sizeof(XBlock) + 16 + (role == LAYER_PRO ? (size_t)wa.cols * 4 : 0);
  c.fn2(dim3(nwa + nwb), lds, a, b, nwa, s);
  LLMI_HIP(hipGetLastError());
}

// x -> Q8_K quants in XBlocks (q8k_block_quad: d = super-block d, nsum8 = block sum) for a
// PLAIN kq launch; 64 threads = 2 super-blocks per work-group, n % 256 == 0
__global__ __launch_bounds__(64) void quantize_q8k_xblocks_kernel(const float* __restrict__ x, int n,
                                                                   XBlock* __restrict__ xb) {
  const int t = threadIdx.x, sbk = blockIdx.x * 2 + (t >> 5);
  const bool ok = sbk * 256 < n;  // whole half-waves in or out
  const int b = sbk * 8 + ((t >> 2) & 7), sub = t & 3;
  float v[8];
#pragma unroll
  for (int k = 0; k < 8; k++) v[k] = ok ? x[b * 32 + sub * 8 + k] : 0.0f;
  if (ok) q8k_block_quad(v, sub, xb + b);
}
void launch_quantize_q8k_xblocks(const float* x, int n, XBlock* xb, hipStream_t s) {
  if (n % 256) throw std::runtime_error("quantize_q8k_xblocks: n % 256 != 0");
  hipLaunchKernelGGL(quantize_q8k_xblocks_kernel, dim3((n / 256 + 1) / 2), dim3(64), 0, s, x, n, xb);
  LLMI_HIP(hipGetLastError());
}


}  // namespace llmi
