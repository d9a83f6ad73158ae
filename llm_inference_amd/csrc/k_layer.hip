// k_layer.hip -- the decode step's Q4_0 GEMVs with their neighbours fused in.
//
// One launch per projection instead of norm / quantize / GEMV / GELU launches:
//   PRO  : the residual step that precedes the GEMV (model.cpp:843-858 and
//          915-924 + the next run_norm) is recomputed by every work-group from
//          the previous GEMV's output -- h = resid + rms(y)*w_post,
//          x = rms(h)*w_next, Q8_0 blocks of x (ops.cpp:116-139) -- straight
//          into LDS.  Work-group 0 publishes h (resid_out, a ping-pong buffer:
//          the other work-groups of the same launch still read resid_in).
//   !PRO : the activation's Q8_0 blocks are copied global -> LDS once per WG.
//   GELU : gate/up rows are interleaved in groups of 32 at upload, so a WG of
//          64 rows owns gate[32k..32k+31] and up[32k..32k+31]; it finishes
//          GELU(gate)*up (model.cpp:892-899) for those 32 hidden units and
//          their Q8_0 block for the down projection.
// The weight stream is the gemv_q4_0_fast scheme (k_gemv.hip): a wave owns R
// rows as a flat (row, block) item list, one 16-B non-temporal load per lane
// per pass, a chunk of P passes in flight; the first chunk is issued before
// the prologue so its HBM latency hides the prologue's L2 round trip, and
// each later chunk is issued before the previous one is consumed.
#include "session_kernels.h"

#include <hip/hip_ext.h>

namespace llmi {

namespace {



template <int NW>
__device__ __forceinline__ float wg_sum(float v, float* red) {  // fixed order, identical in every WG
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float s = 0.0f;
#pragma unroll
  for (int i = 0; i < NW; i++) s += red[i];
  return s;
}

__device__ __forceinline__ float rms_scale_d(float sum, int n, double eps) {  // ops.cpp:37-38
  return 1.0f / sqrtf((float)((double)(sum / (float)n) + eps));
}

template <int P>
struct Chunk {  // raw loaded words only: (row, block) are recomputed when eaten, and
  uint4 q[P];   // converting scales at load time would wait for them
  uint16_t sw[P];
};

template <int P>
__device__ __forceinline__ void load_chunk(Chunk<P>& c, const uint4* qw, const uint16_t* dw, int c0, int total,
                                           int lane) {
#pragma unroll
  for (int p = 0; p < P; p++) {
    const int f = c0 + p * 64 + lane;
    const int fc = f < total ? f : 0;  // clamped: always a valid address
    c.q[p] = ld_nt(qw + fc);
    c.sw[p] = ld_nt16(dw + fc);
  }
}

template <int R, int P>
__device__ __forceinline__ void eat_chunk(const Chunk<P>& c, int c0, int total, int nb, uint32_t magic, int lane,
                                          const XBlock* s_x, float (&acc)[R]) {
#pragma unroll
  for (int p = 0; p < P; p++) {
    const int f = c0 + p * 64 + lane;
    const int fc = f < total ? f : 0;
    const int r = div_by_magic(fc, magic);
    const int rr = f < total ? r : R;  // items past the wave's rows add to no row
    const int bb = fc - r * nb;
    const int4* xp = reinterpret_cast<const int4*>(s_x + bb);
    const int4 x0 = xp[0], x1 = xp[1], x2 = xp[2];
    int is = x2.y;  // nsum8
    is = sdot4(nib_lo(c.q[p].x), x0.x, is);
    is = sdot4(nib_lo(c.q[p].y), x0.y, is);
    is = sdot4(nib_lo(c.q[p].z), x0.z, is);
    is = sdot4(nib_lo(c.q[p].w), x0.w, is);
    is = sdot4(nib_hi(c.q[p].x), x1.x, is);
    is = sdot4(nib_hi(c.q[p].y), x1.y, is);
    is = sdot4(nib_hi(c.q[p].z), x1.z, is);
    is = sdot4(nib_hi(c.q[p].w), x1.w, is);
    const float v = (h2f(c.sw[p]) * __int_as_float(x2.x)) * (float)is;
#pragma unroll
    for (int k = 0; k < R; k++) acc[k] += (k == rr) ? v : 0.0f;
    // keep the scheduler from hoisting every pass's LDS x reads up front
    // (it would hold 12 VGPRs per pass live; other waves hide the LDS latency)
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int R, int NW, int P, int E, bool PRO, bool GELU, bool MULTI>
__global__ __launch_bounds__(NW * 64) void gemv_q4_0_layer(LayerGemv a) {
  constexpr int EPT = E, X_LD = E;
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  XBlock* s_x = reinterpret_cast<XBlock*>(s_dyn);
  __shared__ float s_red[2][NW];
  __shared__ float s_rows[GELU ? 64 : 1];
  constexpr int T = NW * 64;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int nb = a.nb;
  const int row0 = (blockIdx.x * NW + w) * R;
  const int nrows = max(0, min(R, a.rows - row0));
  const int total = nrows * nb;
  const uint4* qw = a.qs + (size_t)min(row0, a.rows - 1) * nb;
  const uint16_t* dw = a.wd + (size_t)min(row0, a.rows - 1) * nb;

  Chunk<P> ca, cb;
  if constexpr (PRO) {
    // prologue operands first: loads return in issue order, so issuing them
    // ahead of the weight chunk lets the norm run while the weights stream
    const int n = a.n;
    float yv[EPT], rv[EPT], wp[EPT], wn[EPT];
#pragma unroll
    for (int k = 0; k < EPT; k++) {
      const int i = t + k * T;
      const bool ok = i < n;
      yv[k] = ok ? a.y[i] : 0.0f;
      rv[k] = ok ? a.resid_in[i] : 0.0f;
      wp[k] = (ok && a.w_post) ? a.w_post[i] : 0.0f;
      wn[k] = ok ? a.w_next[i] : 0.0f;
    }
    load_chunk<P>(ca, qw, dw, 0, total, lane);  // unconditional (valid clamped rows): a
    // branch here would merge wait counts to vmcnt(0) at the first prologue use
    if constexpr (MULTI) load_chunk<P>(cb, qw, dw, 64 * P, total, lane);  // both chunks in flight
    float ss = 0.0f;
#pragma unroll
    for (int k = 0; k < EPT; k++) ss = fmaf(yv[k], yv[k], ss);
    const float sc1 = rms_scale_d(wg_sum<NW>(ss, s_red[0]), n, a.eps);
    float ss2 = 0.0f;
#pragma unroll
    for (int k = 0; k < EPT; k++) {
      const float h = rv[k] + (a.w_post ? (sc1 * yv[k]) * wp[k] : yv[k]);  // no post-norm: plain add
      rv[k] = h;
      ss2 = fmaf(h, h, ss2);
      const int i = t + k * T;
      if (blockIdx.x == 0 && i < n) a.resid_out[i] = h;
    }
    const float sc2 = rms_scale_d(wg_sum<NW>(ss2, s_red[1]), n, a.eps);
    // x staged as f32 in LDS, then one thread per Q8_0 block (no cross-lane
    // reductions on this latency-critical path)
    float* s_xf = reinterpret_cast<float*>(s_dyn + (size_t)nb * sizeof(XBlock) + 16);
#pragma unroll
    for (int k = 0; k < EPT; k++) {
      const int i = t + k * T;
      const float xv = (sc2 * rv[k]) * wn[k];
      if (i < n) {
        s_xf[i] = xv;
        if (blockIdx.x == 0 && a.xn_out) a.xn_out[i] = xv;
      }
    }
    __syncthreads();
    for (int b = t; b < nb; b += T) q8_block_serial(s_xf + 32 * b, s_x + b);
  } else {
    // x blocks -> LDS: clamped unconditional loads (no branch between them
    // and the weight loads, so the stores wait only for their own data)
    const uint4* src = reinterpret_cast<const uint4*>(a.xg);
    uint4* dst = reinterpret_cast<uint4*>(s_x);
    const int n16 = nb * 3;
    uint4 xr[X_LD];
#pragma unroll
    for (int k = 0; k < X_LD; k++) xr[k] = src[min(t + k * T, n16 - 1)];
    load_chunk<P>(ca, qw, dw, 0, total, lane);
    if constexpr (MULTI) load_chunk<P>(cb, qw, dw, 64 * P, total, lane);
#pragma unroll
    for (int k = 0; k < X_LD; k++) dst[min(t + k * T, n16)] = xr[k];  // slot n16: LDS pad (discarded)
  }
  __syncthreads();

  float acc[R];
#pragma unroll
  for (int k = 0; k < R; k++) acc[k] = 0.0f;
  if constexpr (!MULTI) {
    eat_chunk<R, P>(ca, 0, total, nb, a.magic, lane, s_x, acc);
  } else {
    // chunks 0 and 1 were issued before the prologue; each later chunk is
    // issued as soon as its register buffer has been consumed
    constexpr int CH = 64 * P;
    for (int c0 = 0; c0 < total; c0 += 2 * CH) {
      eat_chunk<R, P>(ca, c0, total, nb, a.magic, lane, s_x, acc);
      if (c0 + 2 * CH < total) load_chunk<P>(ca, qw, dw, c0 + 2 * CH, total, lane);
      if (c0 + CH >= total) break;
      eat_chunk<R, P>(cb, c0 + CH, total, nb, a.magic, lane, s_x, acc);
      if (c0 + 3 * CH < total) load_chunk<P>(cb, qw, dw, c0 + 3 * CH, total, lane);
    }
  }

  if constexpr (GELU) {
#pragma unroll
    for (int k = 0; k < R; k++) {
      const float s = wave_sum(acc[k]);
      if (lane == 0) s_rows[w * R + k] = s;
    }
    __syncthreads();
    if (t < 32) {
      const int j = blockIdx.x * 32 + t;  // hidden unit
      const float v = gelu_mul1(s_rows[t], s_rows[32 + t]);
      a.hid[j] = v;
      q8_block_store(v, true, a.hq8 + blockIdx.x, t);
    }
  } else {
#pragma unroll
    for (int k = 0; k < R; k++) {
      const float s = wave_sum(acc[k]);
      if (lane == 0 && k < nrows) a.out[row0 + k] = s;
    }
  }
}

// ---- launch table ----------------------------------------------------------
// One instantiation per (activation length, role) of the Gemma-3 1B/4B/12B/27B
// projections; shapes outside the table take the unfused path (session.cpp).
//   R: rows per wave (R * nb a multiple of 64 where possible), P: passes per
//   chunk, E: see the kernel, NW: waves per WG (8 when the prologue's vector
//   exceeds 12 elements per thread of a 256-thread WG, and for GELU: 64 rows).
enum { ROLE_PLAIN = 0, ROLE_PRO = 1, ROLE_GELU = 2 };

using LaunchFn = void (*)(dim3, size_t, const LayerGemv&, hipStream_t);

template <int R, int NW, int P, int E, int ROLE, bool MULTI>
void launch_cfg(dim3 grid, size_t lds, const LayerGemv& a, hipStream_t s) {
  KernelTiming& kt = kernel_timing();
  if (kt.start) {
    hipExtLaunchKernelGGL((gemv_q4_0_layer<R, NW, P, E, ROLE != ROLE_PLAIN, ROLE == ROLE_GELU, MULTI>), grid,
                          dim3(NW * 64), (uint32_t)lds, s, kt.start, kt.stop, 0u, a);
    kt = KernelTiming{};
    return;
  }
  hipLaunchKernelGGL((gemv_q4_0_layer<R, NW, P, E, ROLE != ROLE_PLAIN, ROLE == ROLE_GELU, MULTI>), grid, dim3(NW * 64),
                     lds, s, a);
}

struct LayerCfg {
  int nb, role, R, NW, P;
  bool multi;
  LaunchFn fn;
};

#define LLMI_LCFG(NB, ROLE, R, NW, P, E, MULTI) {NB, ROLE, R, NW, P, MULTI, launch_cfg<R, NW, P, E, ROLE, MULTI>}
const LayerCfg kLayerCfgs[] = {
    // plain: x blocks copied to LDS (E = 16-B loads per thread = ceil(3 nb / 256))
    LLMI_LCFG(32, ROLE_PLAIN, 2, 4, 1, 1, false),    // 1B o (4 x 256)
    LLMI_LCFG(36, ROLE_PLAIN, 8, 4, 5, 1, false),    // 1B qkv, layer 0
    LLMI_LCFG(64, ROLE_PLAIN, 1, 4, 1, 1, false),    // 4B o (8 x 256)
    LLMI_LCFG(80, ROLE_PLAIN, 4, 4, 5, 1, false),    // 4B qkv, layer 0
    LLMI_LCFG(120, ROLE_PLAIN, 8, 4, 8, 2, true),    // 12B qkv, layer 0
    LLMI_LCFG(128, ROLE_PLAIN, 1, 4, 2, 2, false),   // 12B / 27B o (16 x 256, 32 x 128)
    LLMI_LCFG(168, ROLE_PLAIN, 8, 4, 7, 2, true),    // 27B qkv, layer 0
    LLMI_LCFG(216, ROLE_PLAIN, 8, 4, 7, 4, true),    // 1B down
    LLMI_LCFG(320, ROLE_PLAIN, 1, 4, 5, 4, false),   // 4B down
    LLMI_LCFG(480, ROLE_PLAIN, 2, 4, 8, 8, true),    // 12B down
    LLMI_LCFG(672, ROLE_PLAIN, 2, 4, 7, 8, true),    // 27B down
    // residual + norm prologue (E = prologue elements per thread)
    LLMI_LCFG(36, ROLE_PRO, 8, 4, 5, 12, false),
    LLMI_LCFG(80, ROLE_PRO, 4, 4, 5, 12, false),
    LLMI_LCFG(120, ROLE_PRO, 8, 8, 8, 12, true),
    LLMI_LCFG(168, ROLE_PRO, 8, 8, 7, 12, true),
    // prologue + GELU epilogue: NW x R = 64 interleaved gate/up rows per work-group
    LLMI_LCFG(36, ROLE_GELU, 8, 8, 5, 6, false),
    LLMI_LCFG(80, ROLE_GELU, 4, 16, 5, 3, false),    // 16 waves x 4 rows: one 5-pass chunk per wave
    LLMI_LCFG(120, ROLE_GELU, 4, 16, 8, 6, false),
    LLMI_LCFG(168, ROLE_GELU, 8, 8, 7, 12, true),
};
#undef LLMI_LCFG

const LayerCfg* find_cfg(int nb, int role) {
  for (const auto& c : kLayerCfgs)
    if (c.nb == nb && c.role == role) return &c;
  return nullptr;
}

}  // namespace

KernelTiming& kernel_timing() {
  thread_local KernelTiming kt;
  return kt;
}

bool layer_gemv_supported(const DevWeight& w, bool pro, bool gelu, int n_pro) {
  if (w.type != T_Q4_0 || w.cols % 32 != 0 || w.rows <= 0) return false;
  if (pro && n_pro != w.cols) return false;
  if (gelu && (!pro || w.rows % 64 != 0)) return false;
  return find_cfg(w.cols / 32, gelu ? ROLE_GELU : (pro ? ROLE_PRO : ROLE_PLAIN)) != nullptr;
}

void launch_layer_gemv(const DevWeight& w, LayerGemv a, bool pro, bool gelu, hipStream_t s) {
  if (!layer_gemv_supported(w, pro, gelu, pro ? w.cols : 0)) throw std::runtime_error("layer gemv: unsupported weight");
  if (pro ? (!a.y || !a.resid_in || !a.resid_out || !a.w_next || a.resid_in == a.resid_out) : !a.xg)
    throw std::runtime_error("layer gemv: missing prologue operand");
  if (gelu ? (!a.hid || !a.hq8) : !a.out) throw std::runtime_error("layer gemv: missing output");
  const LayerCfg& c = *find_cfg(w.cols / 32, gelu ? ROLE_GELU : (pro ? ROLE_PRO : ROLE_PLAIN));
  if (!c.multi && c.R * (w.cols / 32) > 64 * c.P) throw std::runtime_error("layer gemv: table entry needs MULTI");
  a.qs = reinterpret_cast<const uint4*>(w.qs);
  a.wd = w.d;
  a.rows = w.rows;
  a.nb = w.cols / 32;
  a.magic = div_magic(a.nb);
  if (pro) a.n = w.cols;
  // x blocks + pad slot of the x copy (+ the f32 x staging of the prologue)
  const size_t lds = (size_t)a.nb * sizeof(XBlock) + 16 + (pro ? (size_t)a.n * 4 : 0);
  const int rows_per_wg = c.NW * c.R;
  c.fn(dim3((w.rows + rows_per_wg - 1) / rows_per_wg), lds, a, s);
  LLMI_HIP(hipGetLastError());
}

}  // namespace llmi
