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

template <int R, int NW, int P, int E, int ROLE, bool MULTI, bool EARLY, int PE = 0, bool W8 = false>
__global__ __launch_bounds__(NW * 64 + (role_help(ROLE) ? E * 64 : 0)) void gemv_q4_0_layer(LayerGemv a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  // the attention block's granule tag of this layer, for its next launch
  if (a.epoch && blockIdx.x == 0 && threadIdx.x == 0) *a.epoch += 1u;
  layer_body<R, NW, P, E, ROLE, MULTI, EARLY, 0, PE, W8>(a, blockIdx.x, s_dyn, BlockSync{});
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

template <int R, int NW, int P, int E, int ROLE, bool MULTI, bool EARLY, int PE = 0, bool W8 = false>
void launch_cfg(dim3 grid, size_t lds, const LayerGemv& a, hipStream_t s) {
  const dim3 block(NW * 64 + (role_help(ROLE) ? E * 64 : 0));
  KernelTiming& kt = kernel_timing();
  if (kt.start) {
    hipExtLaunchKernelGGL((gemv_q4_0_layer<R, NW, P, E, ROLE, MULTI, EARLY, PE, W8>), grid, block, (uint32_t)lds, s,
                          kt.start, kt.stop, 0u, a);
    kt = KernelTiming{};
    return;
  }
  hipLaunchKernelGGL((gemv_q4_0_layer<R, NW, P, E, ROLE, MULTI, EARLY, PE, W8>), grid, block, lds, s, a);
}

struct LayerCfg {
  int nb, role, R, NW, P, E;
  bool multi;
  int slab;  // weight layout this entry reads (sweep: slab pays for R >= 4 on big matrices)
  bool help;  // PRO/GELU with E helper waves (role_help)
  LaunchFn fn;
  bool w8 = false;  // Q8_0 weights (P counts half-block passes)
};

#define LLMI_LCFG(NB, ROLE, R, NW, P, E, MULTI, EARLY, SLAB) \
  {NB, ROLE, R, NW, P, E, MULTI, SLAB, false, launch_cfg<R, NW, P, E, ROLE, MULTI, EARLY>}
// late roles with the first PE passes issued right after the prologue's loads
#define LLMI_LCFGP(NB, ROLE, R, NW, P, E, SLAB, PE) \
  {NB, ROLE, R, NW, P, E, false, SLAB, false, launch_cfg<R, NW, P, E, ROLE, false, false, PE>}
// Q8_0 weights: row-major, single chunk (P passes of 16-B half blocks)
#define LLMI_LCFG8(NB, ROLE, R, NW, P, E, EARLY) \
  {NB, ROLE, R, NW, P, E, false, 0, false, launch_cfg<R, NW, P, E, ROLE, false, EARLY, 0, true>, true}
// PRO / GELU entries with NH helper waves (template role ROLE_PRO_H / ROLE_GELU_H)
#define LLMI_LCFGH(NB, ROLE, R, NW, P, NH, MULTI, SLAB) \
  {NB, ROLE, R, NW, P, NH, MULTI, SLAB, true,          \
   launch_cfg<R, NW, P, NH, ROLE == ROLE_PRO ? ROLE_PRO_H : ROLE_GELU_H, MULTI, true>}
// (scripts/gemv_sweep: 4B gate_up GELU 9.1 -> 8.5 us with R8 NW10 slab, 7.8
// us issuing 7 of its 10 passes before the prologue (PE7; all 10: 8.8 us);
// 4B down 5.8 -> 5.4 us with PE3 (of 5) instead of EARLY; 27B
// gate_up 35.8 -> 26.3 us with R8 NW8 P4 slab, qkv 10.4 -> 10.0 us, down
// 24 -> 17-19.5 us issuing the weights after the quantized x is in LDS)
const LayerCfg kLayerCfgs[] = {
    // PLAIN: x blocks copied to LDS
    LLMI_LCFG(32, ROLE_PLAIN, 2, 2, 1, 1, false, true, 0),     // 1B o        1152 rows -> 288 WGs
    LLMI_LCFG(36, ROLE_PLAIN, 8, 1, 5, 2, false, true, 0),     // 1B qkv l0   1536 rows -> 192 WGs
    LLMI_LCFG(64, ROLE_PLAIN, 1, 10, 1, 1, false, true, 0),    // 4B o        2560 rows -> 256 WGs
    LLMI_LCFG(80, ROLE_PLAIN, 4, 4, 5, 1, false, true, 0),     // 4B qkv l0   4096 rows -> 256 WGs
    LLMI_LCFG(120, ROLE_PLAIN, 8, 4, 8, 2, true, true, 0),     // 12B qkv l0  8192 rows -> 256 WGs
    LLMI_LCFG(128, ROLE_PLAIN, 1, 8, 2, 1, false, true, 0),    // 12B/27B o   3840/5376 rows -> 480/672 WGs
    LLMI_LCFG(168, ROLE_PLAIN, 8, 4, 7, 2, true, true, 1),     // 27B qkv l0  8192 rows -> 256 WGs
    // PRO: residual + norm prologue
    LLMI_LCFG(36, ROLE_PRO, 8, 2, 5, 9, false, true, 0),       // 1B qkv      96 WGs
    LLMI_LCFG(80, ROLE_PRO, 4, 4, 5, 10, false, true, 0),      // 4B qkv      256 WGs
    LLMI_LCFG(120, ROLE_PRO, 8, 4, 8, 15, true, true, 0),      // 12B qkv     256 WGs
    LLMI_LCFG(168, ROLE_PRO, 4, 8, 6, 11, true, true, 1),      // 27B qkv     256 WGs
    // GELU: prologue + GELU epilogue, 2H = R NW interleaved gate/up rows per WG
    LLMI_LCFGP(36, ROLE_GELU, 8, 8, 5, 3, 0, 3),              // 1B  13824 rows, H 32 -> 216 WGs (PE3: 5.9 -> 5.1 us)
    LLMI_LCFGP(80, ROLE_GELU, 8, 10, 10, 4, 1, 7),            // 4B  20480 rows, H 40 -> 256 WGs (PE7: 8.4 -> 7.8 us)
    LLMI_LCFG(120, ROLE_GELU, 8, 8, 8, 8, true, false, 0),     // 12B 30720 rows, H 32 -> 480 WGs
    LLMI_LCFG(168, ROLE_GELU, 8, 8, 4, 11, true, false, 1),    // 27B 43008 rows, H 32 -> 672 WGs
    // QUANT: f32 activation quantized into LDS (down projection)
    LLMI_LCFG(216, ROLE_QUANT, 1, 4, 4, 4, false, true, 0),    // 1B down     1152 rows -> 288 WGs (6.5 -> 5.0 us)
    LLMI_LCFGP(320, ROLE_QUANT, 1, 10, 5, 2, 0, 3),           // 4B down     2560 rows -> 256 WGs (PE3: 5.8 -> 5.4 us)
    LLMI_LCFG(480, ROLE_QUANT, 1, 8, 8, 4, false, true, 0),    // 12B down    3840 rows -> 480 WGs
    LLMI_LCFG(672, ROLE_QUANT, 1, 8, 6, 6, true, false, 0),    // 27B down    5376 rows -> 672 WGs
    // Q8_0 weights (Gemma-3 1B Q8_0, BASELINE configs[3]): 2 nb half-block units per row
    LLMI_LCFG8(36, ROLE_PLAIN, 4, 2, 5, 1, true),     // 1B qkv l0   1536 rows -> 192 WGs
    LLMI_LCFG8(36, ROLE_PRO, 4, 4, 5, 5, true),       // 1B qkv      96 WGs
    LLMI_LCFG8(32, ROLE_PLAIN, 1, 4, 1, 1, true),     // 1B o        1152 rows -> 288 WGs
    LLMI_LCFG8(36, ROLE_GELU, 8, 8, 9, 3, false),     // 1B gate_up  13824 rows, H 32 -> 216 WGs
    LLMI_LCFG8(216, ROLE_QUANT, 1, 4, 7, 4, true),    // 1B down     1152 rows -> 288 WGs
};
#undef LLMI_LCFG

const LayerCfg* find_cfg(int nb, int role, uint32_t type = T_Q4_0) {
  if (type != T_Q4_0 && type != T_Q8_0) return nullptr;
  for (const auto& c : kLayerCfgs)
    if (c.nb == nb && c.role == role && c.w8 == (type == T_Q8_0)) return &c;
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
  if ((w.type != T_Q4_0 && w.type != T_Q8_0) || w.cols % 32 != 0 || w.rows <= 0) return false;
  const LayerCfg* c = find_cfg(w.cols / 32, role, w.type);
  if (!c) return false;
  if (role == LAYER_GELU && w.rows % (c->R * c->NW) != 0) return false;
  return true;
}

int layer_gemv_slab(const DevWeight& w, int role) {
  const LayerCfg* c = w.cols % 32 == 0 ? find_cfg(w.cols / 32, role, w.type) : nullptr;
  return c ? c->slab : 0;
}

int layer_gemv_gelu_group(int cols, uint32_t type) {
  const LayerCfg* c = cols % 32 == 0 ? find_cfg(cols / 32, LAYER_GELU, type) : nullptr;
  return c ? c->R * c->NW / 2 : 0;
}

void launch_layer_gemv(const DevWeight& w, LayerGemv a, int role, hipStream_t s) {
  if (!layer_gemv_supported(w, role)) throw std::runtime_error("layer gemv: unsupported weight");
  const bool pro = role == LAYER_PRO || role == LAYER_GELU;
  if (pro && (!a.y || !a.resid_in || !a.resid_out || !a.w_next || a.resid_in == a.resid_out))
    throw std::runtime_error("layer gemv: missing prologue operand");
  if (role == LAYER_PLAIN && !a.xg) throw std::runtime_error("layer gemv: missing activation blocks");
  if (role == LAYER_QUANT && !a.y) throw std::runtime_error("layer gemv: missing activation");
  if (role == LAYER_GELU ? !a.hid : !a.out) throw std::runtime_error("layer gemv: missing output");
  const LayerCfg& c = *find_cfg(w.cols / 32, role, w.type);
  const int nb = w.cols / 32, nu = c.w8 ? 2 * nb : nb;  // 16-B units per row
  const bool rb = c.R == 1 || c.R == 2 || c.R == 4 || c.R == 8 || c.R == 16;
  if (!c.multi && (rb ? (nu + 64 / c.R - 1) / (64 / c.R) > c.P : c.R * nb > 64 * c.P))
    throw std::runtime_error("layer gemv: table entry needs MULTI");
  if (pro && !c.help && w.cols > c.E * c.NW * 64) throw std::runtime_error("layer gemv: prologue E too small");
  if (pro && c.help && (w.cols % (c.E * 32) != 0 || w.cols > c.E * 256 * HELP_K4))
    throw std::runtime_error("layer gemv: helper segments must be whole Q8_0 blocks within HELP_K4");
  if (role == LAYER_PLAIN && 3 * nb > c.E * c.NW * 64) throw std::runtime_error("layer gemv: x copy E too small");
  if (role == LAYER_QUANT && 4 * nb > c.E * c.NW * 64) throw std::runtime_error("layer gemv: quant E too small");
  if (w.slab != c.slab) throw std::runtime_error("layer gemv: weight layout does not match the launch table");
  a.qs = reinterpret_cast<const uint4*>(w.qs);
  a.wd = w.d;
  a.slab = w.slab;
  a.rows = w.rows;
  a.nb = nb;
  a.magic = div_magic(nb);
  a.n = w.cols;
  // x blocks + pad slot of the x copy (+ the f32 x staging of the prologue)
  const size_t lds = (size_t)nb * sizeof(XBlock) + 16 + (pro ? (size_t)w.cols * 4 : 0);
  const int rows_per_wg = c.NW * c.R;
  c.fn(dim3((w.rows + rows_per_wg - 1) / rows_per_wg), lds, a, s);
  LLMI_HIP(hipGetLastError());
}


}  // namespace llmi
