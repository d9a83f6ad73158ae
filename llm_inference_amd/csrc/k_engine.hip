// k_engine.hip -- the layer engine: one Gemma-3 decode layer (Q4_0 weights)
// as ONE persistent launch of one 1024-thread work-group per CU.
//
// Why: the decode layer is a chain of dependent
// all-to-all steps -- x -> qkv -> attention -> o -> gate_up -> down -- over
// 53 MB of weights (4B).  As three launches (attention block, gate_up, down)
// each projection's weight stream starts only when its launch does, so the
// layer costs the chain's latency PLUS most of the FFN stream.  Decode weights
// do not depend on activations: here every CU issues its whole slice of the
// layer's weights at launch start (qkv, o and gate_up rows into the worker
// waves' registers, the down rows into LDS by LDS-DMA), and the chain's
// hand-offs run while those bytes land.  By the time the FFN's inputs arrive
// the FFN weights are on chip; what is left is the chain.
//
// Work-group geometry (grid = one work-group per CU, all co-resident: the
// host admits the launch only if the occupancy query gives >= 1 per CU):
//   waves 0-3   "comm" waves: the hand-off polls that come before the weight
//               stream has landed (q/k/v rows, merged attention blocks), the
//               K/V tile LDS-DMA, the attention's softmax / PV and merge;
//   waves 4-15  "worker" waves (768 lanes): hold the weight slices; they
//               never poll global memory while their loads may be in flight
//               (a poll's vmcnt(0) would wait for the whole slice).
// Every phase is executed by all 16 waves (roles differ inside a phase), so
// the phases are separated by plain work-group barriers.
//
// Per CU c (rows of each matrix split in contiguous ranges, row-major Q4_0):
//   P1  residual + post_ffw norm + attn_norm of the previous layer's output
//       (every CU, redundantly: 3 x E floats) -> Q8_0 x in LDS
//   P2  qkv rows [c rq, ..) -> data-tagged granules g_qkv
//   P3  CUs c < n_kv kvd NSPLIT: one (kv head, key split) of the split-K
//       attention (as k_attn.hip's attention block), the last two arrivers
//       per head merge one head each -> the heads' Q8_0 blocks as granules
//   P4  o rows [c ro, ..) from the merged blocks -> granules g_o
//   P5  every CU: residual + post_attn norm + ffn_norm of o -> Q8_0 x2 in LDS
//       (work-group 0 publishes the residual)
//   P6  gate_up: ru hidden units (gate + up rows interleaved in groups of ru
//       at upload), GELU(gate) * up -> granules g_hid
//   P7  every CU: the whole GELU output from the granules, quantized to Q8_0
//   P8  down rows [c rd, ..) from the LDS copy of the weights -> y_out
// Numerics: the fast path's (reference ops.cpp:116-139 quantization of every
// activation, Q4_0 x Q8_0 block dots, model.cpp:430-566 attention in fp32
// split-K); only the summation order of the projections' block sums differs
// from the attention-block path (row sums of per-block products).
// Hand-offs: common.h granules (tag = *epoch + 1, work-group 0 advances the
// epoch at the end), every wait bounded (timeout -> *err, the grid drains).
#include "session_kernels.h"

#include <hip/hip_ext.h>

namespace llmi {

namespace {

constexpr int ENG_T = 1024, ENG_NW = 16, ENG_CW = 4, ENG_LW = (ENG_NW - ENG_CW) * 64, ENG_TK = 32;

// development: per-CU phase clocks (100 MHz) of one traced layer, [cu][16] (builds with -DLLMI_BLOCK_TRACE,
// scripts/engine_trace.py)
#ifdef LLMI_BLOCK_TRACE
#define ENG_MARK(ph)                                                                   \
  do {                                                                                 \
    if (a.trace && threadIdx.x == 0) a.trace[(size_t)blockIdx.x * 16 + (ph)] = wall_clock64(); \
  } while (0)
#else
#define ENG_MARK(ph) \
  do {               \
  } while (0)
#endif

// LDS-DMA of 16 B per lane (1 KB per wave) to the wave-uniform LDS byte address
// `lds`; asm so that hipcc's s_waitcnt bookkeeping does not drain it (the
// waits are explicit: cdna_hip_programming.md section 5.7, LDS-DMA recipe)
__device__ __forceinline__ void eng_glds16(const void* g, const void* lds) {
  const uint32_t dst = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)lds);
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(g), "s"(dst)
               : "memory");
}

// one Q4_0 block x one Q8_0 activation block (ops.cpp:334-381 arithmetic, the
// zero point folded into nsum8)
__device__ __forceinline__ float eng_dot(const uint4 q, uint16_t sw, const XBlock* xb) {
  const int4* xp = reinterpret_cast<const int4*>(xb);
  const int4 x0 = xp[0], x1 = xp[1], x2 = xp[2];
  int is = x2.y;
  is = sdot4(nib_lo(q.x), x0.x, is);
  is = sdot4(nib_lo(q.y), x0.y, is);
  is = sdot4(nib_lo(q.z), x0.z, is);
  is = sdot4(nib_lo(q.w), x0.w, is);
  is = sdot4(nib_hi(q.x), x1.x, is);
  is = sdot4(nib_hi(q.y), x1.y, is);
  is = sdot4(nib_hi(q.z), x1.z, is);
  is = sdot4(nib_hi(q.w), x1.w, is);
  return (h2f(sw) * __int_as_float(x2.x)) * (float)is;
}

// quantize_row_q8_0 (ops.cpp:116-139) of one 32-element block held by 8
// consecutive lanes, 4 elements each (lane & 7 = sub owns elements 4 sub ..
// 4 sub + 3): the 8-lane max / integer sum by a quad butterfly and a
// half-row mirror.  Bit-identical to q8_block_store (order-free max and
// integer sums).  All 8 lanes of every octet must execute it.
__device__ __forceinline__ void q8_block_oct(const float4 x, int sub, XBlock* __restrict__ blk) {
  float amax = fmaxf(fmaxf(fabsf(x.x), fabsf(x.y)), fmaxf(fabsf(x.z), fabsf(x.w)));
  amax = fmaxf(amax, dpp_f<DPP_QUAD_1032>(amax));
  amax = fmaxf(amax, dpp_f<DPP_QUAD_2301>(amax));
  amax = fmaxf(amax, dpp_f<DPP_ROW_HALF_MIRROR>(amax));
  const float dd = amax / 127.0f;
  const float id = dd != 0.0f ? 1.0f / dd : 0.0f;
  const int q0 = nearest_int_fma(x.x, id), q1 = nearest_int_fma(x.y, id);
  const int q2 = nearest_int_fma(x.z, id), q3 = nearest_int_fma(x.w, id);
  int s = (q0 + q1) + (q2 + q3);
  s += dpp_i<DPP_QUAD_1032>(s);
  s += dpp_i<DPP_QUAD_2301>(s);
  s += dpp_i<DPP_ROW_HALF_MIRROR>(s);
  reinterpret_cast<uint32_t*>(blk)[sub] =
      (uint32_t)(q0 & 0xFF) | ((uint32_t)(q1 & 0xFF) << 8) | ((uint32_t)(q2 & 0xFF) << 16) | ((uint32_t)q3 << 24);
  if (sub == 0) {
    blk->d = h2f(f2h_ggml(dd));
    blk->nsum8 = -8 * s;
  }
}

// sum of v over the work-group (fixed order: DPP wave sums, then the 16 wave
// totals in wave order); red: 16 floats of LDS not in use by another sum
__device__ __forceinline__ float eng_block_sum(float v, float* red) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < ENG_NW; k++) s += red[k];
  return s;
}

// row sums of sv[nrows][nb] (the per-block products of a projection): wave
// w takes rows w, w + 16, ...; out(r, sum) by lane 0 (wave-uniform loop)
template <class F>
__device__ __forceinline__ void eng_row_sums(const float* sv, int nrows, int nb, F&& out) {
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  for (int r = w; r < nrows; r += ENG_NW) {
    float s = 0.0f;
    for (int j = lane; j < nb; j += 64) s += sv[r * nb + j];
    s = wave_sum(s);
    if (lane == 0) out(r, s);
  }
}

__device__ __forceinline__ float4 u4f(const uint32_t (&u)[4]) {
  return make_float4(__uint_as_float(u[0]), __uint_as_float(u[1]), __uint_as_float(u[2]), __uint_as_float(u[3]));
}

// comm-wave sweep of K sets of 4 data-tagged granules (set k of this lane at granule offset off[k], if
// act[k]): every set's loads are issued before any tag is checked, then only the sets whose tags are
// not yet this launch's are re-loaded (bounded: a timeout sets *err and leaves the values invalid)
template <int K>
__device__ __forceinline__ void eng_sweep(uint32_t (&v)[K][4], const uint2* g, const int (&off)[K], const bool (&act)[K],
                                          uint32_t tag, int* err) {
  const __amdgpu_buffer_rsrc_t r = buf_rsrc(g, 1u << 30);
  bool done[K];
  uint4 lo[K], hi[K];
#pragma unroll
  for (int k = 0; k < K; k++) {
    const int o = act[k] ? off[k] * 8 : (1 << 30);
    lo[k] = buf_ld16_sc1(r, o);
    hi[k] = buf_ld16_sc1(r, o + 16);
  }
  bool all = true;
#pragma unroll
  for (int k = 0; k < K; k++) {
    done[k] = !act[k] || ((lo[k].y == tag) & (lo[k].w == tag) & (hi[k].y == tag) & (hi[k].w == tag));
    all &= done[k];
  }
  int n = 0;
  while (!all) {
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int k = 0; k < K; k++)
      if (!done[k]) {
        lo[k] = buf_ld16_sc1(r, off[k] * 8);
        hi[k] = buf_ld16_sc1(r, off[k] * 8 + 16);
      }
    all = true;
#pragma unroll
    for (int k = 0; k < K; k++) {
      done[k] = done[k] || ((lo[k].y == tag) & (lo[k].w == tag) & (hi[k].y == tag) & (hi[k].w == tag));
      all &= done[k];
    }
    if (++n >= BLOCK_SPIN_LIMIT) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      break;
    }
    asm volatile("" ::: "memory");
  }
#pragma unroll
  for (int k = 0; k < K; k++) {
    v[k][0] = lo[k].x;
    v[k][1] = lo[k].z;
    v[k][2] = hi[k].x;
    v[k][3] = hi[k].z;
  }
}

}  // namespace

// LDS carve-up, host and device (byte offsets; every region 1 KB aligned)
struct EngLds {
  int dq, dd, kv, vq, x, xo, resid, pn, fn, total;
};
__host__ __device__ inline int eng_align(int b) { return (b + 1023) & ~1023; }
__host__ __device__ inline EngLds eng_lds(const EngineLayer& a, int hd, int g) {
  const int nbE = a.E / 32, nbO = a.n_head * hd / 32, nbF = a.Fu / 32;
  const int ud = a.rd * nbF;
  EngLds L;
  int o = 0;
  L.dq = o;
  o += eng_align(ud * 16);
  L.dd = o;
  o += eng_align(ud * 2);
  // kv region: K / V tiles + PV class sums (attention); later the o / gate_up
  // block products, the GELU output's Q8_0 blocks and the down products
  const int kv_attn = ENG_TK * hd * 2 * 2 + 4 * g * hd * 4;
  const int kv_o = eng_align(a.E * 4) + a.E * 4, kv_g = 2 * a.ru * nbE * 4;  // P4/P5: o products, then o (f32)
  const int kv_d = eng_align(nbF * (int)sizeof(XBlock)) + ud * 4;
  int kvb = kv_attn;
  if (kv_o > kvb) kvb = kv_o;
  if (kv_g > kvb) kvb = kv_g;
  if (kv_d > kvb) kvb = kv_d;
  L.kv = o;
  o += eng_align(kvb);
  L.vq = o;
  o += eng_align(a.rq * nbE * 4);
  L.x = o;
  o += eng_align(nbE * (int)sizeof(XBlock));
  L.xo = o;
  o += eng_align(nbO * (int)sizeof(XBlock));
  L.resid = o;
  o += eng_align(a.E * 4);
  L.pn = o;  // post_attn_norm / ffn_norm weights (LDS-DMA at launch start, read in P5)
  o += eng_align(a.E * 4);
  L.fn = o;
  o += eng_align(a.E * 4);
  L.total = o;
  return L;
}

// the FFN engine's carve-up: down rows, the gate_up products / GELU blocks + down products, x2
__host__ __device__ inline EngLds eng_ffn_lds(const EngineLayer& a) {
  const int nbE = a.E / 32, nbF = a.Fu / 32, ud = a.rd * nbF;
  EngLds L{};
  int o = 0;
  L.dq = o;
  o += eng_align(ud * 16);
  L.dd = o;
  o += eng_align(ud * 2);
  const int kv_g = 2 * a.ru * nbE * 4, kv_d = eng_align(nbF * (int)sizeof(XBlock)) + ud * 4;
  L.kv = o;
  o += eng_align(kv_g > kv_d ? kv_g : kv_d);
  L.x = o;
  o += eng_align(nbE * (int)sizeof(XBlock));
  L.total = o;
  return L;
}

namespace {

// barrier of the four comm waves only (the worker waves are streaming weights meanwhile): an LDS arrival
// counter; n counts this thread's barriers x ENG_CW (uniform over the comm waves)
__device__ __forceinline__ void eng_cbar(unsigned* c, unsigned& n) {
  n += ENG_CW;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's LDS writes are done before it arrives
  if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(c, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
  while (__hip_atomic_load(c, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < n) __builtin_amdgcn_s_sleep(0);
  asm volatile("" ::: "memory");
}

// sum over the comm waves (fixed order); red: ENG_CW floats not in use by another sum
__device__ __forceinline__ float eng_csum(float v, float* red, unsigned* c, unsigned& n) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  eng_cbar(c, n);
  return (red[0] + red[1]) + (red[2] + red[3]);
}

// row sums by NWV waves (rows w, w + NWV, ...; out(r, sum) by lane 0)
template <int NWV, class F>
__device__ __forceinline__ void eng_row_sums_n(const float* sv, int nrows, int nb, F&& out) {
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), lane = threadIdx.x & 63;
  for (int r = w; r < nrows; r += NWV) {
    float s = 0.0f;
    for (int j = lane; j < nb; j += 64) s += sv[r * nb + j];
    s = wave_sum(s);
    if (lane == 0) out(r, s);
  }
}

template <int HD, int G, int PQ, int PO, int PG, bool FIRST>
__global__ __launch_bounds__(ENG_T) void layer_engine_kernel(EngineLayer a) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char s_dyn[];
  constexpr int NS = ATTN_NSPLIT, TK = ENG_TK, CH = HD / 8, DPL = HD / 64;
  static_assert(HD == 256 && G == 2, "engine attention: head_dim 256, 2 q heads per (virtual) kv head");
  constexpr int CT = ENG_CW * 64;  // comm threads
  static_assert(CT % (G * TK) == 0, "scores: whole lane groups per (head, key) pair");
  constexpr int LPP = CT / (G * TK);  // lanes per (head, key) pair
  __shared__ float s_red[2][ENG_NW];
  __shared__ float s_cred[2][ENG_CW];
  __shared__ unsigned s_cbar;
  __shared__ __attribute__((aligned(16))) float s_raw[(G + 2) * HD];
  __shared__ __attribute__((aligned(16))) uint16_t s_q[G][HD];
  __shared__ __attribute__((aligned(16))) uint16_t s_new[2][HD];
  __shared__ float s_p[G][TK];
  __shared__ float s_alpha[G];
  __shared__ float s_wt[NS];
  __shared__ float s_L;
  __shared__ int s_flag;
  __shared__ __attribute__((aligned(16))) float s_mo[HD];
  __shared__ __attribute__((aligned(16))) XBlock s_mq[HD / 32];
  __shared__ float s_gu[256];

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const bool cw = w < ENG_CW;
  const int wl = t - CT;  // worker lane (waves 4-15)
  const int cu = blockIdx.x;
  const int E = a.E, nbE = E / 32, nbO = a.n_head * HD / 32, nbF = a.Fu / 32;
  const EngLds L = eng_lds(a, HD, G);
  const uint4* s_dq = reinterpret_cast<const uint4*>(s_dyn + L.dq);
  const uint16_t* s_dd = reinterpret_cast<const uint16_t*>(s_dyn + L.dd);
  uint16_t* s_k = reinterpret_cast<uint16_t*>(s_dyn + L.kv);
  uint16_t* s_v = s_k + TK * HD;
  float* s_pv = reinterpret_cast<float*>(s_v + TK * HD);  // [4][G][HD] PV class sums
  float* s_kvf = reinterpret_cast<float*>(s_dyn + L.kv);  // the kv region as floats (after the attention)
  float* s_vq = reinterpret_cast<float*>(s_dyn + L.vq);
  XBlock* s_x = reinterpret_cast<XBlock*>(s_dyn + L.x);
  XBlock* s_xo = reinterpret_cast<XBlock*>(s_dyn + L.xo);
  float4* s_resid = reinterpret_cast<float4*>(s_dyn + L.resid);

  ENG_MARK(0);
  const uint32_t tag = *a.epoch + 1u;
  const int pos = *a.d_pos;
  const int n4 = E / 4;
  const bool pt = t < n4;  // prologue threads: elements 4t .. 4t + 3 (whole octets: E % 32 == 0)
  if (t == 0) s_cbar = 0;

  // ---- P0: the prologue's operands, then the qkv rows (raw barriers order the issue) ----
  // Memory queues are first-come-first-served across the chip, so a latency-critical load issued while a
  // bulk stream is in flight waits for its backlog (profiles/r03_engine_trace.txt).  Here only the qkv rows
  // are issued with the prologue; the gate_up and down rows are streamed by the worker waves at a bounded
  // depth while the comm waves run the attention and the o projection (P3-P5).
  const int ti = min(t, n4 - 1);
  const float4 r4i = reinterpret_cast<const float4*>(a.resid_in)[ti];
  float4 y4 = make_float4(0.f, 0.f, 0.f, 0.f), p4 = y4, nw4 = y4;
  if constexpr (!FIRST) {  // (the session requires w_post: Gemma-3's post_ffw_norm)
    y4 = reinterpret_cast<const float4*>(a.y_in)[ti];
    p4 = reinterpret_cast<const float4*>(a.w_post)[ti];
    nw4 = reinterpret_cast<const float4*>(a.attn_norm)[ti];
  }
  if constexpr (FIRST) {  // layer 0: x arrives as Q8_0 blocks
    for (int i = t; i < nbE * 3; i += ENG_T) reinterpret_cast<uint4*>(s_x)[i] = reinterpret_cast<const uint4*>(a.x0)[i];
  }
  __builtin_amdgcn_s_barrier();
  const int nvh = a.n_kv * a.kvd;
  const bool attn_cu = cu < nvh * NS;
  const int hkv = attn_cu ? cu % nvh : 0, split = attn_cu ? cu / nvh : 0, hkc = hkv / a.kvd;
  const int n_keys = pos + 1;
  auto dma_tile = [&](int tile) {  // comm waves: K / V tile -> s_k / s_v, 2 rows per wave instruction
    for (int i = w; i < TK; i += ENG_CW) {
      const bool isv = i >= TK / 2;
      const int ii = isv ? i - TK / 2 : i;
      const int j = 2 * ii + (lane >> 5), key = tile * TK + j;
      const uint16_t* base = isv ? a.v_cache : a.k_cache;
      const void* src = key < n_keys ? static_cast<const void*>(base + ((size_t)hkc * a.max_ctx + key) * HD + (lane & 31) * 8)
                                     : static_cast<const void*>(a.zero + (lane & 31));
      eng_glds16(src, (isv ? s_v : s_k) + ii * 2 * HD);
    }
  };
  // worker slices: unit u = p LW + j (j < LW = (768 / nb) nb) is block j % nb of row u / nb, so a lane's
  // activation block is fixed across passes; every wave issues the same loads (empty descriptors for the
  // comm waves), so hipcc's s_waitcnt counts agree on every path
  const int lwq = (ENG_LW / nbE) * nbE, lwo = (CT / nbO) * nbO;
  const int nrq = max(0, min(a.nq - cu * a.rq, a.rq)), nro = max(0, min(E - cu * a.ro, a.ro));
  const int nrd = max(0, min(E - cu * a.rd, a.rd));
  const int Uq = nrq * nbE, Uo = nro * nbO, Ug = 2 * a.ru * nbE, Ud = nrd * nbF;
  const uint32_t on = cw ? 0u : 1u;
  const int jq = cw ? lwq : wl;
  const bool okq = jq < lwq;
  uint4 wq[PQ], wg[PG];
  uint16_t sq[PQ], sg[PG];
  {
    const __amdgpu_buffer_rsrc_t rq = buf_rsrc(a.q_qs + (size_t)cu * a.rq * nbE, on * Uq * 16),
                                 rqd = buf_rsrc(a.q_d + (size_t)cu * a.rq * nbE, on * Uq * 2);
#pragma unroll
    for (int p = 0; p < PQ; p++) {
      const int u = okq ? p * lwq + jq : (1 << 24);
      wq[p] = buf_ld16(rq, u * 16, 0);
      sq[p] = buf_ld2(rqd, u * 2, 0);
    }
  }

  // ---- P1: residual + post_ffw norm + attn_norm -> Q8_0 x (all waves) ------
  float4 r4 = r4i;
  if constexpr (!FIRST) {
    if (!pt) y4 = make_float4(0.f, 0.f, 0.f, 0.f);
    float ss = 0.0f;
    ss = fmaf(y4.x, y4.x, ss);
    ss = fmaf(y4.y, y4.y, ss);
    ss = fmaf(y4.z, y4.z, ss);
    ss = fmaf(y4.w, y4.w, ss);
    const float sc1 = 1.0f / sqrtf((float)((double)(eng_block_sum(ss, s_red[0]) / (float)E) + a.eps));
    ENG_MARK(11);
    r4.x += (sc1 * y4.x) * p4.x;
    r4.y += (sc1 * y4.y) * p4.y;
    r4.z += (sc1 * y4.z) * p4.z;
    r4.w += (sc1 * y4.w) * p4.w;
    float ss2 = 0.0f;
    if (pt) {
      ss2 = fmaf(r4.x, r4.x, ss2);
      ss2 = fmaf(r4.y, r4.y, ss2);
      ss2 = fmaf(r4.z, r4.z, ss2);
      ss2 = fmaf(r4.w, r4.w, ss2);
    }
    const float sc2 = 1.0f / sqrtf((float)((double)(eng_block_sum(ss2, s_red[1]) / (float)E) + a.eps));
    if (pt) {
      const float4 x4 = make_float4((sc2 * r4.x) * nw4.x, (sc2 * r4.y) * nw4.y, (sc2 * r4.z) * nw4.z, (sc2 * r4.w) * nw4.w);
      q8_block_oct(x4, t & 7, s_x + (t >> 3));
    }
  }
  if (pt) s_resid[t] = r4;
  __syncthreads();
  ENG_MARK(1);

  // ---- P2: qkv rows -> granules (all waves) --------------------------------
  if (!cw && okq) {
    const XBlock* xb = s_x + jq % nbE;
#pragma unroll
    for (int p = 0; p < PQ; p++) {
      const int u = p * lwq + jq;
      if (u < Uq) s_vq[u] = eng_dot(wq[p], sq[p], xb);  // row-major products: [row][block]
    }
  }
  __syncthreads();
  ENG_MARK(12);
  eng_row_sums(s_vq, nrq, nbE, [&](int r, float v) { st_granule(a.g_qkv + cu * a.rq + r, __float_as_uint(v), tag); });
  ENG_MARK(2);

  if (!cw) {
    // ---- worker waves: the gate_up rows (registers), then the down rows (LDS-DMA), at most DEPTH passes
    // of 1 KB per wave in flight (12 waves x DEPTH KB per CU, a few MB chip-wide), so the comm waves' hand-offs
    // do not queue behind the layer's 44 MB ----
    constexpr int DEPTH = 3;
    const __amdgpu_buffer_rsrc_t rg = buf_rsrc(a.g_qs + (size_t)cu * 2 * a.ru * nbE, on * Ug * 16),
                                 rgd = buf_rsrc(a.g_d + (size_t)cu * 2 * a.ru * nbE, on * Ug * 2);
#pragma unroll
    for (int p = 0; p < PG; p++) {
      const int u = okq ? p * lwq + jq : (1 << 24);
      wg[p] = buf_ld16(rg, u * 16, 0);
      sg[p] = buf_ld2(rgd, u * 2, 0);
      if (p >= DEPTH) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * DEPTH) : "memory");
    }
    const unsigned char* dq = reinterpret_cast<const unsigned char*>(a.d_qs + (size_t)cu * a.rd * nbF);
    const unsigned char* dd = reinterpret_cast<const unsigned char*>(a.d_d + (size_t)cu * a.rd * nbF);
    const int nqi = (Ud * 16 + 1023) / 1024, ndi = (Ud * 2 + 1023) / 1024;
    for (int i = w - ENG_CW; i < nqi + ndi; i += ENG_NW - ENG_CW) {
      if (i < nqi) eng_glds16(dq + i * 1024 + lane * 16, s_dyn + L.dq + i * 1024);
      else eng_glds16(dd + (i - nqi) * 1024 + lane * 16, s_dyn + L.dd + (i - nqi) * 1024);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DEPTH) : "memory");
    }
  } else {
    // ---- comm waves: P3 attention, P4 o projection, P5 residual + norms (comm-wave barriers only) ----
    unsigned nb_c = 0;
    uint4 wo[PO];
    uint16_t so[PO];
    const int jo = t, oko = jo < lwo;
    {  // the o rows (comm registers), the K / V tile and the FFN norm weights
      if (attn_cu) dma_tile(split);
      const int nk = (E * 4 + 1023) / 1024;
      for (int i = w; i < 2 * nk; i += ENG_CW) {
        const bool f = i >= nk;
        const int ii = f ? i - nk : i;
        eng_glds16(reinterpret_cast<const unsigned char*>(f ? a.ffn_norm : a.post_attn_norm) + ii * 1024 + lane * 16,
                   s_dyn + (f ? L.fn : L.pn) + ii * 1024);
      }
      const __amdgpu_buffer_rsrc_t ro = buf_rsrc(a.o_qs + (size_t)cu * a.ro * nbO, (uint32_t)Uo * 16),
                                   rod = buf_rsrc(a.o_d + (size_t)cu * a.ro * nbO, (uint32_t)Uo * 2);
#pragma unroll
      for (int p = 0; p < PO; p++) {
        const int u = oko ? p * lwo + jo : (1 << 24);
        wo[p] = buf_ld16(ro, u * 16, 0);
        so[p] = buf_ld2(rod, u * 2, 0);
      }
    }
    // ---- P3: attention (one (virtual kv head, split) per CU c < n_kv kvd NSPLIT) ----
    if (attn_cu) {
      const int own_tile = pos / TK;
      const bool own_new = own_tile % NS == split;
      {  // this head group's q rows, the k row and the v row from their granules
        constexpr int K = ((G + 2) * HD / 4 + CT - 1) / CT;
        int off[K];
        bool act[K];
        uint32_t u[K][4];
#pragma unroll
        for (int k = 0; k < K; k++) {
          const int e = (k * CT + t) * 4;
          act[k] = e < (G + 2) * HD;
          off[k] = e < G * HD         ? hkv * G * HD + e
                   : e < (G + 1) * HD ? a.k_off + hkc * HD + (e - G * HD)
                                      : a.v_off + hkc * HD + (e - (G + 1) * HD);
        }
        eng_sweep<K>(u, a.g_qkv, off, act, tag, a.err);
#pragma unroll
        for (int k = 0; k < K; k++)
          if (act[k]) *reinterpret_cast<float4*>(s_raw + (k * CT + t) * 4) = u4f(u[k]);
      }
      eng_cbar(&s_cbar, nb_c);
      ENG_MARK(3);
      if (w < G + 2) {  // per-row norm + NEOX rope (model.cpp:762-767, 792-794): waves 0..G-1 q heads, G the k row, G+1 v
        const int i0 = lane * DPL;
        float v[DPL];
#pragma unroll
        for (int d = 0; d < DPL; d++) v[d] = s_raw[w * HD + i0 + d];
        if (w <= G) {
          const float* nwp = (w < G ? a.q_norm : a.k_norm) + i0;
          const int j0 = i0 < HD / 2 ? i0 : i0 - HD / 2;
          const float* cs = a.rope_cs + (size_t)pos * (HD / 2) * 2 + 2 * j0;
          float nw[DPL], c[DPL], sn[DPL];
#pragma unroll
          for (int d = 0; d < DPL; d++) {
            nw[d] = nwp[d];
            c[d] = cs[2 * d];
            sn[d] = cs[2 * d + 1];
          }
          float ss = 0.0f;
#pragma unroll
          for (int d = 0; d < DPL; d++) ss = fmaf(v[d], v[d], ss);
          ss = wave_sum(ss);
          const float sc = 1.0f / sqrtf((float)((double)(ss / (float)HD) + a.eps));
#pragma unroll
          for (int d = 0; d < DPL; d++) {
            const int i = i0 + d;
            const float n = (sc * v[d]) * nw[d];
            const float pn = __shfl_xor(n, 32);
            const float r = i < HD / 2 ? fmaf(n, c[d], -(pn * sn[d])) : fmaf(pn, sn[d], n * c[d]);
            if (w < G) {
              s_q[w][i] = f2h_ggml(r * a.attn_scale);
            } else {
              const uint16_t k16 = f2h_ggml(r);
              s_new[0][i] = k16;
              if (own_new && hkv % a.kvd == 0) a.k_cache[((size_t)hkc * a.max_ctx + pos) * HD + i] = k16;
            }
          }
        } else {
#pragma unroll
          for (int d = 0; d < DPL; d++) {
            const uint16_t v16 = f2h_ggml(v[d]);
            s_new[1][i0 + d] = v16;
            if (own_new && hkv % a.kvd == 0) a.v_cache[((size_t)hkc * a.max_ctx + pos) * HD + i0 + d] = v16;
          }
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the first tile's LDS-DMA (landed long ago: the polls waited)
      eng_cbar(&s_cbar, nb_c);
      float m_run = -INFINITY, l_run = 0.0f;  // head w's running max / sum (waves w < G)
      float acc[G][4];
#pragma unroll
      for (int g = 0; g < G; g++)
#pragma unroll
        for (int e = 0; e < 4; e++) acc[g][e] = 0.0f;
      const int d_own = 4 * lane, kp = w;  // PV: 4 head dims, key class w
      typedef _Float16 h2t __attribute__((ext_vector_type(2)));
      for (int tile = split; tile * TK < n_keys; tile += NS) {
        if (tile != split) {  // later tiles (contexts past NSPLIT * TK keys): loaded here
          dma_tile(tile);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          eng_cbar(&s_cbar, nb_c);
        }
        if (tile == own_tile) {  // this token's k / v row, written in this launch
          const int j = pos % TK;
          if (t < CH) reinterpret_cast<uint4*>(s_k + j * HD)[t] = reinterpret_cast<const uint4*>(s_new[0])[t];
          else if (t < 2 * CH) reinterpret_cast<uint4*>(s_v + j * HD)[t - CH] = reinterpret_cast<const uint4*>(s_new[1])[t - CH];
          eng_cbar(&s_cbar, nb_c);
        }
        {  // scores: LPP lanes per (head, key); each lane 32 / LPP chunks, the chunk order rotated by the key
           // (conflict-free LDS reads of unpadded rows)
          const int pr = t / LPP, part = t % LPP, g = pr / TK, j = pr % TK;
          const uint4* krow = reinterpret_cast<const uint4*>(s_k + j * HD);
          const uint4* qrow = reinterpret_cast<const uint4*>(s_q[g]);
          float s0 = 0.0f, s1 = 0.0f;
#pragma unroll
          for (int i = 0; i < CH / LPP; i++) {
            const int c = (part + LPP * i + LPP * j) & (CH - 1);
            const uint4 kk = krow[c], qq = qrow[c];
            s0 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, kk.x), __builtin_bit_cast(h2t, qq.x), s0, false);
            s1 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, kk.y), __builtin_bit_cast(h2t, qq.y), s1, false);
            s0 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, kk.z), __builtin_bit_cast(h2t, qq.z), s0, false);
            s1 = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2t, kk.w), __builtin_bit_cast(h2t, qq.w), s1, false);
          }
          float sc = s0 + s1;
#pragma unroll
          for (int o = 1; o < LPP; o <<= 1) sc += __shfl_xor(sc, o);
          if (part == 0) s_p[g][j] = tile * TK + j < n_keys ? sc : -INFINITY;
        }
        eng_cbar(&s_cbar, nb_c);
        if (w < G) {
          const float sc = lane < TK ? s_p[w][lane] : -INFINITY;
          const float m_new = fmaxf(m_run, wave_max(sc));
          const float p = expf(sc - m_new);          // masked keys: exp(-inf) = 0
          const float alpha = expf(m_run - m_new);   // first tile: exp(-inf) = 0
          l_run = l_run * alpha + wave_sum(p);
          m_run = m_new;
          if (lane < TK) s_p[w][lane] = p;
          if (lane == 0) s_alpha[w] = alpha;
        }
        eng_cbar(&s_cbar, nb_c);
#pragma unroll
        for (int g = 0; g < G; g++) {
          const float al = s_alpha[g];
#pragma unroll
          for (int e = 0; e < 4; e++) acc[g][e] *= al;
        }
#pragma unroll 4
        for (int j = kp; j < TK; j += ENG_CW) {
          const uint2 vv = *reinterpret_cast<const uint2*>(s_v + j * HD + d_own);
          const float v0 = h2f((uint16_t)(vv.x & 0xFFFF)), v1 = h2f((uint16_t)(vv.x >> 16));
          const float v2 = h2f((uint16_t)(vv.y & 0xFFFF)), v3 = h2f((uint16_t)(vv.y >> 16));
#pragma unroll
          for (int g = 0; g < G; g++) {
            const float p = s_p[g][j];
            acc[g][0] = fmaf(p, v0, acc[g][0]);
            acc[g][1] = fmaf(p, v1, acc[g][1]);
            acc[g][2] = fmaf(p, v2, acc[g][2]);
            acc[g][3] = fmaf(p, v3, acc[g][3]);
          }
        }
        eng_cbar(&s_cbar, nb_c);  // the tile's LDS is reused by the next one
      }
      // the 4 key classes -> the split's partial (sc1 stores), then the head's ticket
      if (kp > 0) {
#pragma unroll
        for (int g = 0; g < G; g++)
          *reinterpret_cast<float4*>(s_pv + ((kp * G + g) * HD + d_own)) = make_float4(acc[g][0], acc[g][1], acc[g][2], acc[g][3]);
      }
      eng_cbar(&s_cbar, nb_c);
      float* part0 = a.partial + (size_t)hkv * G * NS * (HD + 2);  // [G][NS][HD + 2]
      if (w == 0) {
#pragma unroll
        for (int g = 0; g < G; g++) {
          for (int r = 1; r < ENG_CW; r++) {
            const float4 o = *reinterpret_cast<const float4*>(s_pv + ((r * G + g) * HD + d_own));
            acc[g][0] += o.x;
            acc[g][1] += o.y;
            acc[g][2] += o.z;
            acc[g][3] += o.w;
          }
#pragma unroll
          for (int e = 0; e < 4; e++) st_sc1(part0 + ((size_t)g * NS + split) * (HD + 2) + d_own + e, acc[g][e]);
        }
      }
      if (w < G && lane == 0) {
        st_sc1(part0 + ((size_t)w * NS + split) * (HD + 2) + HD, m_run);
        st_sc1(part0 + ((size_t)w * NS + split) * (HD + 2) + HD + 1, l_run);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      eng_cbar(&s_cbar, nb_c);
      if (t == 0) {
        const unsigned old = __hip_atomic_fetch_add(a.ticket + hkv, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_flag = old == NS - 1 ? 1 : old == NS - 2 ? 2 : 0;
      }
      eng_cbar(&s_cbar, nb_c);
      int role = s_flag;
      if (role == 2) {  // second-to-last: merges head 0 once the last ticket is in (bounded wait)
        eng_cbar(&s_cbar, nb_c);  // every thread has read s_flag
        if (t == 0) {
          int n = 0;
          s_flag = 2;
          while (__hip_atomic_load(a.ticket + hkv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)NS) {
            if (++n >= BLOCK_SPIN_LIMIT) {
              __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              s_flag = 0;  // no merge from incomplete partials, no ticket reset (the host zeroes the tickets)
              break;
            }
          }
        }
        eng_cbar(&s_cbar, nb_c);
        role = s_flag;
      }
      if (role != 0) {
        const int g0 = role == 1 ? 1 : 0;
        const float* pg = part0 + (size_t)g0 * NS * (HD + 2);
        const int n_act = min(NS, (n_keys + TK - 1) / TK);
        float mv = -INFINITY, lv = 0.0f;
        float v[NS];
        if (t < NS) {
          mv = ld_sc1(pg + t * (HD + 2) + HD);
          lv = ld_sc1(pg + t * (HD + 2) + HD + 1);
        }
        const __amdgpu_buffer_rsrc_t rp = buf_rsrc(pg, (uint32_t)(NS * (HD + 2) * 4));
#pragma unroll
        for (int cc = 0; cc < NS; cc++)
          v[cc] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rp, cc < n_act ? (cc * (HD + 2) + t) * 4 : (1 << 30), 0, BUF_SC1));
        if (w == 0) {  // lanes 0-31: the splits' (m, l)
          const float M = half_max(mv);
          const float wt = lv == 0.0f ? 0.0f : expf(mv - M);
          const float Ls = half_sum(lv * wt);
          if (t < NS) s_wt[t] = wt;
          if (t == 0) s_L = Ls;
        }
        eng_cbar(&s_cbar, nb_c);
        float o = 0.0f;
#pragma unroll
        for (int cc = 0; cc < NS; cc++) o = fmaf(v[cc], s_wt[cc], o);
        s_mo[t] = o / s_L;
        eng_cbar(&s_cbar, nb_c);
        if (t < HD / 4) q8_block_oct(reinterpret_cast<const float4*>(s_mo)[t], t & 7, s_mq + (t >> 3));
        eng_cbar(&s_cbar, nb_c);
        if (t < HD / 32 * 12)
          st_granule(a.g_xo + ((size_t)(hkv * G + g0) * HD / 32) * 12 + t, reinterpret_cast<const uint32_t*>(s_mq)[t], tag);
        if (role == 2 && t == 0) __hip_atomic_store(a.ticket + hkv, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    ENG_MARK(4);
    // ---- P4: o rows from the merged blocks -> granules g_o (comm waves) ----
    for (int i = t; i < nbO * 3; i += CT) {  // 12 words per block, 4 granules per set
      int off[1] = {4 * i};
      bool act[1] = {true};
      uint32_t u[1][4];
      eng_sweep<1>(u, a.g_xo, off, act, tag, a.err);
      reinterpret_cast<uint4*>(s_xo)[i] = make_uint4(u[0][0], u[0][1], u[0][2], u[0][3]);
    }
    eng_cbar(&s_cbar, nb_c);
    ENG_MARK(5);
    if (oko) {
      const XBlock* xb = s_xo + jo % nbO;
#pragma unroll
      for (int p = 0; p < PO; p++) {
        const int u = p * lwo + jo;
        if (u < Uo) s_kvf[u] = eng_dot(wo[p], so[p], xb);
      }
    }
    eng_cbar(&s_cbar, nb_c);
    eng_row_sums_n<ENG_CW>(s_kvf, nro, nbO, [&](int r, float v) { st_granule(a.g_o + cu * a.ro + r, __float_as_uint(v), tag); });
    ENG_MARK(6);
    // ---- P5: residual + post_attn norm + ffn_norm -> Q8_0 x2 (comm waves) ----
    float* s_of = s_kvf + eng_align(E * 4) / 4;  // o, f32 [E] (past the o products still being read)
    {
      constexpr int K = 3;
      for (int i0 = 0; i0 < n4; i0 += K * CT) {
        int off[K];
        bool act[K];
        uint32_t u[K][4];
#pragma unroll
        for (int k = 0; k < K; k++) {
          off[k] = 4 * (i0 + k * CT + t);
          act[k] = i0 + k * CT + t < n4;
        }
        eng_sweep<K>(u, a.g_o, off, act, tag, a.err);
#pragma unroll
        for (int k = 0; k < K; k++)
          if (act[k]) reinterpret_cast<float4*>(s_of)[i0 + k * CT + t] = u4f(u[k]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the norm weights' LDS-DMA
    eng_cbar(&s_cbar, nb_c);
    ENG_MARK(13);
    {
      constexpr int KE = 4;  // float4 groups per comm thread: E / 4 <= 4 x 256
      const float4* pn = reinterpret_cast<const float4*>(s_dyn + L.pn);
      const float4* fn = reinterpret_cast<const float4*>(s_dyn + L.fn);
      float4 o4[KE], h[KE];
      float ss = 0.0f;
#pragma unroll
      for (int k = 0; k < KE; k++) {
        const int i = k * CT + t;
        o4[k] = i < n4 ? reinterpret_cast<const float4*>(s_of)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
        ss = fmaf(o4[k].x, o4[k].x, ss);
        ss = fmaf(o4[k].y, o4[k].y, ss);
        ss = fmaf(o4[k].z, o4[k].z, ss);
        ss = fmaf(o4[k].w, o4[k].w, ss);
      }
      const float sc1 = 1.0f / sqrtf((float)((double)(eng_csum(ss, s_cred[0], &s_cbar, nb_c) / (float)E) + a.eps));
      float ss2 = 0.0f;
#pragma unroll
      for (int k = 0; k < KE; k++) {
        const int i = k * CT + t;
        if (i < n4) {
          const float4 r = s_resid[i], p = pn[i];
          h[k] = make_float4(r.x + (sc1 * o4[k].x) * p.x, r.y + (sc1 * o4[k].y) * p.y, r.z + (sc1 * o4[k].z) * p.z,
                             r.w + (sc1 * o4[k].w) * p.w);
          ss2 = fmaf(h[k].x, h[k].x, ss2);
          ss2 = fmaf(h[k].y, h[k].y, ss2);
          ss2 = fmaf(h[k].z, h[k].z, ss2);
          ss2 = fmaf(h[k].w, h[k].w, ss2);
          if (cu == 0) reinterpret_cast<float4*>(a.resid_out)[i] = h[k];
        } else {
          h[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
      }
      const float sc2 = 1.0f / sqrtf((float)((double)(eng_csum(ss2, s_cred[1], &s_cbar, nb_c) / (float)E) + a.eps));
#pragma unroll
      for (int k = 0; k < KE; k++) {
        const int i = k * CT + t;
        if (k * CT < n4 && i < n4) {  // whole octets (n4 % 8 == 0)
          const float4 f = fn[i];
          q8_block_oct(make_float4((sc2 * h[k].x) * f.x, (sc2 * h[k].y) * f.y, (sc2 * h[k].z) * f.z, (sc2 * h[k].w) * f.w),
                       i & 7, s_x + (i >> 3));
        }
      }
    }
  }
  __syncthreads();  // P6: the comm waves' x2 and the workers' slices meet
  ENG_MARK(7);

  // ---- P6: gate_up + GELU -> granules g_hid --------------------------------
  if (!cw && okq) {
    const XBlock* xb = s_x + jq % nbE;
#pragma unroll
    for (int p = 0; p < PG; p++) {
      const int u = p * lwq + jq;
      if (u < Ug) s_kvf[u] = eng_dot(wg[p], sg[p], xb);
    }
  }
  __syncthreads();
  ENG_MARK(14);
  eng_row_sums(s_kvf, 2 * a.ru, nbE, [&](int r, float v) { s_gu[r] = v; });
  __syncthreads();
  ENG_MARK(15);
  if (t < a.ru) {  // model.cpp:892-899
    const float hv = gelu_mul1(s_gu[t], s_gu[a.ru + t]);
    st_granule(a.g_hid + cu * a.ru + t, __float_as_uint(hv), tag);
  }
  ENG_MARK(8);

  // ---- P7: the whole GELU output -> Q8_0 blocks in LDS (comm waves sweep) ----
  XBlock* s_hx = reinterpret_cast<XBlock*>(s_dyn + L.kv);
  float* s_vd = reinterpret_cast<float*>(s_dyn + L.kv + eng_align(nbF * (int)sizeof(XBlock)));
  if (cw) {
    constexpr int K = 5;
    const int nsets = a.Fu / 4;
    for (int i0 = 0; i0 < nsets; i0 += K * CT) {
      int off[K];
      bool act[K];
      uint32_t u[K][4];
#pragma unroll
      for (int k = 0; k < K; k++) {
        const int i = i0 + k * CT + t;
        off[k] = 4 * i;
        act[k] = i < nsets;
      }
      eng_sweep<K>(u, a.g_hid, off, act, tag, a.err);
#pragma unroll
      for (int k = 0; k < K; k++) {
        const int i = i0 + k * CT + t;
        if (i0 + k * CT < nsets)  // whole octets (nsets % 8 == 0)
          if (i < nsets) q8_block_oct(u4f(u[k]), i & 7, s_hx + (i >> 3));
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the down rows' LDS-DMA (worker waves)
  __syncthreads();
  ENG_MARK(9);

  // ---- P8: down rows -> y_out (weights in LDS; a thread's activation block is fixed) ----
  {
    const int lwd = (ENG_T / nbF) * nbF;
    if (t < lwd) {
      const XBlock* xb = s_hx + t % nbF;
      for (int u = t; u < Ud; u += lwd) s_vd[u] = eng_dot(s_dq[u], s_dd[u], xb);
    }
  }
  __syncthreads();
  eng_row_sums(s_vd, nrd, nbF, [&](int r, float v) { a.y_out[cu * a.rd + r] = v; });
  ENG_MARK(10);
  if (cu == 0 && t == 0) *a.epoch = tag;  // every CU read the epoch before any CU got past P7
}

// ---------------------------------------------------------------------------
// FFN engine: gate_up + GELU + down of one layer as ONE launch of one 1024-thread work-group per CU, after
// the attention block (k_attn.hip).  The down rows (LDS-DMA) and the gate_up rows (worker registers) are
// issued at launch start, behind the prologue operands; the GELU output crosses CUs once (granules, comm-wave
// sweep) instead of through a launch boundary plus a re-read of the FFN weights' stream start.
//   P5  every CU: residual + post_attn norm + ffn_norm of o (the block's output) -> Q8_0 x2
//   P6  gate_up: ru hidden units per CU, GELU(gate) * up -> granules g_hid
//   P7  every CU: the whole GELU output -> Q8_0 blocks in LDS
//   P8  down rows [c rd, ..) -> y_out; work-group 0 advances the attention block's epoch (blk_epoch)
// ---------------------------------------------------------------------------
template <int PG>
__global__ __launch_bounds__(ENG_T) void ffn_engine_kernel(EngineLayer a) {
  extern __shared__ __attribute__((aligned(1024))) unsigned char s_dyn[];
  __shared__ float s_red[2][ENG_NW];
  __shared__ float s_gu[256];
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const bool cw = w < ENG_CW;
  const int wl = t - ENG_CW * 64;
  const int cu = blockIdx.x;
  const int E = a.E, nbE = E / 32, nbF = a.Fu / 32;
  const EngLds L = eng_ffn_lds(a);
  const uint4* s_dq = reinterpret_cast<const uint4*>(s_dyn + L.dq);
  const uint16_t* s_dd = reinterpret_cast<const uint16_t*>(s_dyn + L.dd);
  float* s_kvf = reinterpret_cast<float*>(s_dyn + L.kv);
  XBlock* s_x = reinterpret_cast<XBlock*>(s_dyn + L.x);
  ENG_MARK(0);
  const uint32_t tag = *a.epoch + 1u;
  const int n4 = E / 4;
  const bool pt = t < n4;
  // P0: the prologue operands (unconditional loads, masked below), then the weight slices
  const int ti = min(t, n4 - 1);
  const float4 o4i = reinterpret_cast<const float4*>(a.y_in)[ti];
  const float4 r4 = reinterpret_cast<const float4*>(a.resid_in)[ti];
  const float4 pn = reinterpret_cast<const float4*>(a.post_attn_norm)[ti];
  const float4 fn = reinterpret_cast<const float4*>(a.ffn_norm)[ti];
  __builtin_amdgcn_s_barrier();
  const int lwq = (ENG_LW / nbE) * nbE;
  const int nrd = max(0, min(E - cu * a.rd, a.rd));
  const int Ug = 2 * a.ru * nbE, Ud = nrd * nbF;
  const uint32_t on = cw ? 0u : 1u;
  const int jq = cw ? lwq : wl;
  const bool okq = jq < lwq;
  uint4 wg[PG];
  uint16_t sg[PG];
  {
    const __amdgpu_buffer_rsrc_t rg = buf_rsrc(a.g_qs + (size_t)cu * 2 * a.ru * nbE, on * Ug * 16),
                                 rgd = buf_rsrc(a.g_d + (size_t)cu * 2 * a.ru * nbE, on * Ug * 2);
#pragma unroll
    for (int p = 0; p < PG; p++) {
      const int u = okq ? p * lwq + jq : (1 << 24);
      wg[p] = buf_ld16(rg, u * 16, 0);
      sg[p] = buf_ld2(rgd, u * 2, 0);
    }
  }
  __builtin_amdgcn_s_barrier();
  if (!cw) {  // the down rows by LDS-DMA (>= 8 KB of allocation slack: whole 1-KB pieces)
    const unsigned char* dq = reinterpret_cast<const unsigned char*>(a.d_qs + (size_t)cu * a.rd * nbF);
    const unsigned char* dd = reinterpret_cast<const unsigned char*>(a.d_d + (size_t)cu * a.rd * nbF);
    const int nqi = (Ud * 16 + 1023) / 1024, ndi = (Ud * 2 + 1023) / 1024;
    for (int i = w - ENG_CW; i < nqi + ndi; i += ENG_NW - ENG_CW) {
      if (i < nqi) eng_glds16(dq + i * 1024 + lane * 16, s_dyn + L.dq + i * 1024);
      else eng_glds16(dd + (i - nqi) * 1024 + lane * 16, s_dyn + L.dd + (i - nqi) * 1024);
    }
  }
  // P5: residual + post_attn norm + ffn_norm -> Q8_0 x2 (model.cpp:843-858, 915-924 + run_norm)
  {
    const float4 o4 = pt ? o4i : make_float4(0.f, 0.f, 0.f, 0.f);
    float ss = 0.0f;
    ss = fmaf(o4.x, o4.x, ss);
    ss = fmaf(o4.y, o4.y, ss);
    ss = fmaf(o4.z, o4.z, ss);
    ss = fmaf(o4.w, o4.w, ss);
    const float sc1 = 1.0f / sqrtf((float)((double)(eng_block_sum(ss, s_red[0]) / (float)E) + a.eps));
    const float4 h = make_float4(r4.x + (sc1 * o4.x) * pn.x, r4.y + (sc1 * o4.y) * pn.y, r4.z + (sc1 * o4.z) * pn.z,
                                 r4.w + (sc1 * o4.w) * pn.w);
    float ss2 = 0.0f;
    if (pt) {
      ss2 = fmaf(h.x, h.x, ss2);
      ss2 = fmaf(h.y, h.y, ss2);
      ss2 = fmaf(h.z, h.z, ss2);
      ss2 = fmaf(h.w, h.w, ss2);
      if (cu == 0) reinterpret_cast<float4*>(a.resid_out)[t] = h;
    }
    const float sc2 = 1.0f / sqrtf((float)((double)(eng_block_sum(ss2, s_red[1]) / (float)E) + a.eps));
    if (pt)
      q8_block_oct(make_float4((sc2 * h.x) * fn.x, (sc2 * h.y) * fn.y, (sc2 * h.z) * fn.z, (sc2 * h.w) * fn.w), t & 7,
                   s_x + (t >> 3));
  }
  __syncthreads();
  ENG_MARK(7);
  // P6: gate_up + GELU -> granules g_hid
  if (!cw && okq) {
    const XBlock* xb = s_x + jq % nbE;
#pragma unroll
    for (int p = 0; p < PG; p++) {
      const int u = p * lwq + jq;
      if (u < Ug) s_kvf[u] = eng_dot(wg[p], sg[p], xb);
    }
  }
  __syncthreads();
  ENG_MARK(14);
  eng_row_sums(s_kvf, 2 * a.ru, nbE, [&](int r, float v) { s_gu[r] = v; });
  __syncthreads();
  ENG_MARK(15);
  if (t < a.ru) {  // model.cpp:892-899
    const float hv = gelu_mul1(s_gu[t], s_gu[a.ru + t]);
    st_granule(a.g_hid + cu * a.ru + t, __float_as_uint(hv), tag);
  }
  ENG_MARK(8);
  // P7: the whole GELU output -> Q8_0 blocks in LDS (comm waves; 5 sets of 4 granules per lane in flight)
  XBlock* s_hx = reinterpret_cast<XBlock*>(s_dyn + L.kv);
  float* s_vd = reinterpret_cast<float*>(s_dyn + L.kv + eng_align(nbF * (int)sizeof(XBlock)));
  if (cw) {
    constexpr int K = 5;
    const int nsets = a.Fu / 4;
    for (int i0 = 0; i0 < nsets; i0 += K * ENG_CW * 64) {
      int off[K];
      bool act[K];
      uint32_t u[K][4];
#pragma unroll
      for (int k = 0; k < K; k++) {
        const int i = i0 + k * ENG_CW * 64 + t;
        off[k] = 4 * i;
        act[k] = i < nsets;
      }
      eng_sweep<K>(u, a.g_hid, off, act, tag, a.err);
#pragma unroll
      for (int k = 0; k < K; k++) {
        const int i = i0 + k * ENG_CW * 64 + t;
        if (i0 + k * ENG_CW * 64 < nsets)
          if (i < nsets) q8_block_oct(u4f(u[k]), i & 7, s_hx + (i >> 3));
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the down rows' LDS-DMA (worker waves)
  __syncthreads();
  ENG_MARK(9);
  // P8: down rows -> y_out
  {
    const int lwd = (ENG_T / nbF) * nbF;
    if (t < lwd) {
      const XBlock* xb = s_hx + t % nbF;
      for (int u = t; u < Ud; u += lwd) s_vd[u] = eng_dot(s_dq[u], s_dd[u], xb);
    }
  }
  __syncthreads();
  eng_row_sums(s_vd, nrd, nbF, [&](int r, float v) { a.y_out[cu * a.rd + r] = v; });
  ENG_MARK(10);
  if (cu == 0 && t == 0) {
    *a.epoch = tag;                     // every CU read the epoch before any CU got past P7
    if (a.blk_epoch) *a.blk_epoch += 1u;  // the attention block's granule tag of this layer (gate_up's job before)
  }
}

template <int PG>
void ffn_launch(int grid, size_t lds, const EngineLayer& a, hipStream_t s) {
  KernelTiming& kt = kernel_timing();
  if (kt.start) {
    hipExtLaunchKernelGGL((ffn_engine_kernel<PG>), dim3(grid), dim3(ENG_T), (uint32_t)lds, s, kt.start, kt.stop, 0u, a);
    kt = KernelTiming{};
    return;
  }
  hipLaunchKernelGGL((ffn_engine_kernel<PG>), dim3(grid), dim3(ENG_T), lds, s, a);
}

struct EngCfg {
  int hd, g, pq, po, pg;
  const void* kern[2];
  void (*fn[2])(int, size_t, const EngineLayer&, hipStream_t);
};

template <int HD, int G, int PQ, int PO, int PG, bool FIRST>
void eng_launch(int grid, size_t lds, const EngineLayer& a, hipStream_t s) {
  KernelTiming& kt = kernel_timing();
  if (kt.start) {
    hipExtLaunchKernelGGL((layer_engine_kernel<HD, G, PQ, PO, PG, FIRST>), dim3(grid), dim3(ENG_T), (uint32_t)lds, s,
                          kt.start, kt.stop, 0u, a);
    kt = KernelTiming{};
    return;
  }
  hipLaunchKernelGGL((layer_engine_kernel<HD, G, PQ, PO, PG, FIRST>), dim3(grid), dim3(ENG_T), lds, s, a);
}

#define LLMI_ECFG(HD, G, PQ, PO, PG)                                                                    \
  {HD, G, PQ, PO, PG,                                                                                  \
   {reinterpret_cast<const void*>(&layer_engine_kernel<HD, G, PQ, PO, PG, false>),                     \
    reinterpret_cast<const void*>(&layer_engine_kernel<HD, G, PQ, PO, PG, true>)},                     \
   {eng_launch<HD, G, PQ, PO, PG, false>, eng_launch<HD, G, PQ, PO, PG, true>}}
const EngCfg kEngCfgs[] = {
    LLMI_ECFG(256, 2, 2, 3, 9),  // 4B: qkv 16 rows x 80 blocks, o 10 x 64 (comm lanes), gate_up 80 x 80 (down 10 x 320 in LDS)
    LLMI_ECFG(256, 2, 1, 1, 3),  // 1B (virtual kv heads of 2): qkv 6 x 36, o 5 x 32, gate_up 54 x 36 (down 5 x 216)
};
#undef LLMI_ECFG

int eng_n_cu() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = -1;
  }
  return n;
}

const EngCfg* eng_find(const EngineLayer& a, int hd, int g) {
  // worker lanes per pass: a whole number of rows' blocks (each lane keeps one activation block)
  auto passes = [](int units, int nb, int lanes) { const int lw = (lanes / nb) * nb; return (units + lw - 1) / lw; };
  const int nbE = a.E / 32, nbO = a.n_head * hd / 32;
  if (nbE > ENG_LW || nbO > ENG_CW * 64 || a.Fu / 32 > ENG_T) return nullptr;
  for (const auto& c : kEngCfgs)  // qkv / gate_up on the worker lanes, o on the comm lanes
    if (c.hd == hd && c.g == g && c.pq == passes(a.rq * nbE, nbE, ENG_LW) &&
        c.po == passes(a.ro * nbO, nbO, ENG_CW * 64) && c.pg == passes(2 * a.ru * nbE, nbE, ENG_LW))
      return &c;
  return nullptr;
}

}  // namespace

// per-CU split of a layer's rows; false when the shapes are outside the engine
bool engine_plan(int E, int F, int n_head, int n_kv, int hd, int qkv_rows, EngineLayer& a) {
  const int ncu = eng_n_cu();
  if (ncu <= 0 || hd != 256 || n_kv <= 0 || n_head % n_kv || E % 32 || F % 32 || E / 4 > ENG_T) return false;
  const int grp = n_head / n_kv;
  const int kvd = grp / 2;  // virtual kv heads of 2 q heads
  if (grp % 2 || n_kv * kvd * ATTN_NSPLIT > ncu || F % ncu || (F / 4) % 8 || 2 * (F / ncu) > 256) return false;
  a.E = E;
  a.Fu = F;
  a.n_head = n_head;
  a.n_kv = n_kv;
  a.kvd = kvd;
  a.nq = qkv_rows;
  a.rq = (qkv_rows + ncu - 1) / ncu;
  a.ro = (E + ncu - 1) / ncu;
  a.rd = a.ro;
  a.ru = F / ncu;
  if (!eng_find(a, hd, 2)) return false;
  const EngLds L = eng_lds(a, hd, 2);
  if (L.total > 160 * 1024 - 8 * 1024) return false;  // + the kernel's static LDS
  const EngCfg* c = eng_find(a, hd, 2);
  for (int k = 0; k < 2; k++) {
    int per_cu = 0;
    if (hipFuncSetAttribute(c->kern[k], hipFuncAttributeMaxDynamicSharedMemorySize, L.total) != hipSuccess) return false;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, c->kern[k], ENG_T, L.total) != hipSuccess || per_cu < 1)
      return false;
  }
  return true;
}

int engine_units(const EngineLayer& a) { return a.ru; }

void launch_layer_engine(const EngineLayer& a, bool first, hipStream_t s) {
  const EngCfg* c = eng_find(a, 256, 2);
  if (!c) throw std::runtime_error("layer engine: no launch configuration for the shapes");
  if (!a.q_qs || !a.o_qs || !a.g_qs || !a.d_qs || !a.epoch || !a.g_qkv || !a.g_xo || !a.g_o || !a.g_hid || !a.err ||
      !a.zero || !a.y_out || !a.resid_in || !a.resid_out || a.resid_in == a.resid_out ||
      (first ? !a.x0 : (!a.y_in || !a.w_post)) || !a.attn_norm || !a.post_attn_norm || !a.ffn_norm)
    throw std::runtime_error("layer engine: missing buffers");
  const EngLds L = eng_lds(a, 256, 2);
  c->fn[first ? 1 : 0](eng_n_cu(), (size_t)L.total, a, s);
  LLMI_HIP(hipGetLastError());
}


// ---- FFN engine ----
namespace {
struct FfnCfg {
  int pg;
  const void* kern;
  void (*fn)(int, size_t, const EngineLayer&, hipStream_t);
};
#define LLMI_FCFG(PG) {PG, reinterpret_cast<const void*>(&ffn_engine_kernel<PG>), ffn_launch<PG>}
const FfnCfg kFfnCfgs[] = {LLMI_FCFG(9), LLMI_FCFG(3), LLMI_FCFG(11)};  // 4B (80 rows x 80 blocks), 1B, 12B-like
#undef LLMI_FCFG
const FfnCfg* ffn_find(const EngineLayer& a) {
  const int nbE = a.E / 32;
  if (nbE > ENG_LW || a.Fu / 32 > ENG_T) return nullptr;
  const int lw = (ENG_LW / nbE) * nbE, pg = (2 * a.ru * nbE + lw - 1) / lw;
  for (const auto& c : kFfnCfgs)
    if (c.pg == pg) return &c;
  return nullptr;
}
}  // namespace

bool ffn_engine_plan(int E, int F, EngineLayer& a) {
  const int ncu = eng_n_cu();
  if (ncu <= 0 || E % 32 || F % 32 || E / 4 > ENG_T || F % ncu || (F / 4) % 8 || 2 * (F / ncu) > 256) return false;
  a.E = E;
  a.Fu = F;
  a.ro = a.rd = (E + ncu - 1) / ncu;
  a.ru = F / ncu;
  const FfnCfg* c = ffn_find(a);
  if (!c) return false;
  const EngLds L = eng_ffn_lds(a);
  if (L.total > 150 * 1024) return false;
  int per_cu = 0;
  if (hipFuncSetAttribute(c->kern, hipFuncAttributeMaxDynamicSharedMemorySize, L.total) != hipSuccess) return false;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, c->kern, ENG_T, L.total) != hipSuccess || per_cu < 1)
    return false;
  return true;
}

void launch_ffn_engine(const EngineLayer& a, hipStream_t s) {
  const FfnCfg* c = ffn_find(a);
  if (!c) throw std::runtime_error("FFN engine: no launch configuration for the shapes");
  if (!a.g_qs || !a.d_qs || !a.epoch || !a.g_hid || !a.err || !a.y_in || !a.y_out || !a.resid_in || !a.resid_out ||
      a.resid_in == a.resid_out || !a.post_attn_norm || !a.ffn_norm)
    throw std::runtime_error("FFN engine: missing buffers");
  c->fn(eng_n_cu(), (size_t)eng_ffn_lds(a).total, a, s);
  LLMI_HIP(hipGetLastError());
}

}  // namespace llmi
