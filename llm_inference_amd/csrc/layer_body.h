// layer_body.h -- device code of the decode step's Q4_0 layer GEMVs
// (k_layer.hip), shared with the attention-block kernel (k_attn.hip).
#pragma once

#include "session_kernels.h"

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

// Row-bound lanes (RB): R = 64 / L rows per wave, lane = k L + j works on row
// k only, blocks j, j + L, j + 2L, ...  A pass (64 lanes) covers L consecutive
// blocks of each of the wave's R rows (R full 128-B lines of quants), so a
// lane needs no (row, block) division and keeps ONE accumulator: about a
// third of the flat mapping's VALU work per block (PMC: the flat mapping's
// per-item row select and division kept the VALU ~50% busy at 4.5 TB/s).
// Lane offsets are affine in the pass index for both weight layouts:
// q at voq + pass * sq, scale at vod + pass * sd (see the kernel).
template <int R, int P>
__device__ __forceinline__ void load_chunk_rb(Chunk<P>& c, __amdgpu_buffer_rsrc_t rq, __amdgpu_buffer_rsrc_t rd,
                                              int voq, int vod, int sq, int sd, int pass0, int npass) {
#pragma unroll
  for (int p = 0; p < P; p++) {
    // blocks past the row's end read the next row / slab (masked when eaten)
    // or, past the matrix, 0 from the descriptor's bound; passes past the last
    // one are sent out of bounds (0, no memory traffic) so the loads stay
    // unconditional (all of the offset in voffset: the range check does not
    // cover soffset)
    const int pi = pass0 + p;
    const bool in = pi < npass;
    c.q[p] = buf_ld16(rq, in ? voq + pi * sq : (1 << 30), 0);
    c.sw[p] = buf_ld2(rd, in ? vod + pi * sd : (1 << 30), 0);
  }
}

// passes [P0, P1) of a chunk only (the rest issued by another call)
template <int R, int P, int P0, int P1>
__device__ __forceinline__ void load_chunk_rb_part(Chunk<P>& c, __amdgpu_buffer_rsrc_t rq, __amdgpu_buffer_rsrc_t rd,
                                                   int voq, int vod, int sq, int sd, int npass) {
#pragma unroll
  for (int p = P0; p < P1; p++) {
    const bool in = p < npass;
    c.q[p] = buf_ld16(rq, in ? voq + p * sq : (1 << 30), 0);
    c.sw[p] = buf_ld2(rd, in ? vod + p * sd : (1 << 30), 0);
  }
}

// Q8_0 weights (W8): a lane's 16-B unit is HALF a block (unit u = block
// u / 2, elements 16 (u % 2) ..; L is even, so the half is lane-fixed: j % 2),
// dotted with the matching half of the activation block; no zero point
template <int R, int P>
__device__ __forceinline__ void eat_chunk_rb_w8(const Chunk<P>& c, int pass0, int nb, int j, bool row_ok,
                                                const XBlock* s_x, float& acc) {
  constexpr int L = 64 / R;
  static_assert(L % 2 == 0, "W8: even lanes per row");
  const int nu = 2 * nb;
#pragma unroll
  for (int p = 0; p < P; p++) {
    const int u = (pass0 + p) * L + j;
    const bool ok = row_ok && u < nu;
    const XBlock* xb = s_x + (u < nu ? u >> 1 : nb - 1);
    const int4 xq = *reinterpret_cast<const int4*>(reinterpret_cast<const char*>(xb) + (j & 1) * 16);
    const float dx = xb->d;
    int is = sdot4((int)c.q[p].x, xq.x, 0);
    is = sdot4((int)c.q[p].y, xq.y, is);
    is = sdot4((int)c.q[p].z, xq.z, is);
    is = sdot4((int)c.q[p].w, xq.w, is);
    const float v = (h2f(c.sw[p]) * dx) * (float)is;
    acc += ok ? v : 0.0f;
    asm volatile("" ::: "memory");
  }
}

template <int R, int P>
__device__ __forceinline__ void eat_chunk_rb(const Chunk<P>& c, int pass0, int nb, int j, bool row_ok,
                                             const XBlock* s_x, float& acc) {
  constexpr int L = 64 / R;
#pragma unroll
  for (int p = 0; p < P; p++) {
    const int b = (pass0 + p) * L + j;
    const bool ok = row_ok && b < nb;
    const int4* xp = reinterpret_cast<const int4*>(s_x + (b < nb ? b : nb - 1));
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
    acc += ok ? v : 0.0f;
    // compiler fence: keeps each pass's LDS x reads next to their use (hoisted,
    // they hold ~10 VGPRs per pass live across the chunk)
    asm volatile("" ::: "memory");
  }
}

// ---- K-quant weights in the kq layout (kernels.h): WT 1 = Q4_K, 2 = Q6_K ----
// A lane's 16-B unit is one 32-element sub-block u (like a Q4_0 block), plus
// its scale word (the Chunk's sw), the super-block's d / dmin word and, for
// Q6_K, the 8 bytes of high bits.  The activation blocks in LDS hold Q8_K
// quants (q8k_block_quad: d = the super-block's d, nsum8 = the block's sum).
enum { WT_Q4_0 = 0, WT_Q4_K = 1, WT_Q6_K = 2 };
template <int P, int WT>
struct ChunkX : Chunk<P> {
  uint32_t dd[WT ? P : 1];
  uint2 qh[WT == WT_Q6_K ? P : 1];
};
struct KqOff {  // lane offsets (bytes) and per-pass strides of the four kq arrays
  __amdgpu_buffer_rsrc_t rdd, rqh;
  int vdd, vqh, sdd, sqh;
};
template <int P, int WT, int P0, int P1>
__device__ __forceinline__ void load_chunk_kq(ChunkX<P, WT>& c, __amdgpu_buffer_rsrc_t rq, __amdgpu_buffer_rsrc_t rd,
                                              const KqOff& k, int voq, int vod, int sq, int sd, int pass0, int npass) {
#pragma unroll
  for (int p = P0; p < P1; p++) {
    const int pi = pass0 + p;
    const bool in = pi < npass;
    c.q[p] = buf_ld16(rq, in ? voq + pi * sq : (1 << 30), 0);
    c.sw[p] = buf_ld2(rd, in ? vod + pi * sd : (1 << 30), 0);
    c.dd[p] = __builtin_amdgcn_raw_buffer_load_b32(k.rdd, in ? k.vdd + pi * k.sdd : (1 << 30), 0, BUF_NT);
    if constexpr (WT == WT_Q6_K) {
      typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
      const u32x2_t h = __builtin_amdgcn_raw_buffer_load_b64(k.rqh, in ? k.vqh + pi * k.sqh : (1 << 30), 0, BUF_NT);
      c.qh[p] = make_uint2(h.x, h.y);
    }
  }
}
__device__ __forceinline__ int q6_bytes(uint32_t nib4, uint32_t h, int k) {  // 4 six-bit values - 32, as signed bytes
  const uint32_t v = nib4 | (((h >> (2 * k)) & 0x03030303u) << 4);  // 0..63 per byte
  return (int)((v + 0x60606060u) ^ 0x80808080u);
}
template <int R, int P, int WT>
__device__ __forceinline__ void eat_chunk_kq(const ChunkX<P, WT>& c, int pass0, int nb, int j, bool row_ok,
                                             const XBlock* s_x, float& acc) {
  constexpr int L = 64 / R;
#pragma unroll
  for (int p = 0; p < P; p++) {
    const int u = (pass0 + p) * L + j;
    const bool ok = row_ok && u < nb;
    const int4* xp = reinterpret_cast<const int4*>(s_x + (u < nb ? u : nb - 1));
    const int4 x0 = xp[0], x1 = xp[1], x2 = xp[2];
    const float xd = __int_as_float(x2.x);
    const uint4 q = c.q[p];
    float v;
    if constexpr (WT == WT_Q4_K) {  // ops.cpp:614-697: fmaf(d sc, isum, -(dmin m bsum)) per sub-block
      int is = sdot4(nib_lo(q.x), x0.x, 0);
      is = sdot4(nib_lo(q.y), x0.y, is);
      is = sdot4(nib_lo(q.z), x0.z, is);
      is = sdot4(nib_lo(q.w), x0.w, is);
      is = sdot4(nib_hi(q.x), x1.x, is);
      is = sdot4(nib_hi(q.y), x1.y, is);
      is = sdot4(nib_hi(q.z), x1.z, is);
      is = sdot4(nib_hi(q.w), x1.w, is);
      const float d = h2f((uint16_t)(c.dd[p] & 0xFFFF)) * xd, mn = h2f((uint16_t)(c.dd[p] >> 16)) * xd;
      v = fmaf(d * (float)(c.sw[p] & 0xFF), (float)is, -((mn * (float)(c.sw[p] >> 8)) * (float)x2.y));
    } else {  // Q6_K (ops.cpp:699-785): d * (sc0 isum0 + sc1 isum1), elements 0-15 / 16-31
      const uint2 h = c.qh[p];
      int i0 = sdot4(q6_bytes((uint32_t)nib_lo(q.x), h.x, 0), x0.x, 0);
      i0 = sdot4(q6_bytes((uint32_t)nib_lo(q.y), h.x, 1), x0.y, i0);
      i0 = sdot4(q6_bytes((uint32_t)nib_lo(q.z), h.x, 2), x0.z, i0);
      i0 = sdot4(q6_bytes((uint32_t)nib_lo(q.w), h.x, 3), x0.w, i0);
      int i1 = sdot4(q6_bytes((uint32_t)nib_hi(q.x), h.y, 0), x1.x, 0);
      i1 = sdot4(q6_bytes((uint32_t)nib_hi(q.y), h.y, 1), x1.y, i1);
      i1 = sdot4(q6_bytes((uint32_t)nib_hi(q.z), h.y, 2), x1.z, i1);
      i1 = sdot4(q6_bytes((uint32_t)nib_hi(q.w), h.y, 3), x1.w, i1);
      const int part = (int)(int8_t)(c.sw[p] & 0xFF) * i0 + (int)(int8_t)(c.sw[p] >> 8) * i1;
      v = (h2f((uint16_t)(c.dd[p] & 0xFFFF)) * xd) * (float)part;
    }
    acc += ok ? v : 0.0f;
    asm volatile("" ::: "memory");
  }
}

// sum over each row's L lanes; row k's total ends up in lane k L (R >= 4) or
// is returned for every k through `tot` (R <= 2)
template <int R>
__device__ __forceinline__ float rb_row_sums(float v, float (&tot)[R <= 2 ? R : 1]) {
  constexpr int L = 64 / R;
  if constexpr (L >= 2) v += dpp_f<DPP_QUAD_1032>(v);
  if constexpr (L >= 4) v += dpp_f<DPP_QUAD_2301>(v);
  if constexpr (L >= 8) v += dpp_f<DPP_ROW_HALF_MIRROR>(v);
  if constexpr (L >= 16) v += dpp_f<DPP_ROW_MIRROR>(v);
  if constexpr (R == 1) tot[0] = (lane_f(v, 0) + lane_f(v, 16)) + (lane_f(v, 32) + lane_f(v, 48));
  if constexpr (R == 2) {
    tot[0] = lane_f(v, 0) + lane_f(v, 16);
    tot[1] = lane_f(v, 32) + lane_f(v, 48);
  }
  return v;
}

#ifdef LLMI_LAYER_TRACE  // development: per-work-group phase timestamps (scripts/gemv_sweep)
__device__ unsigned long long* g_layer_trace = nullptr;
#define LAYER_MARK(ph)                                                                                     \
  do {                                                                                                     \
    if (g_layer_trace && threadIdx.x == 0) g_layer_trace[(size_t)blockIdx.x * 8 + (ph)] = wall_clock64(); \
  } while (0)
#else
#define LAYER_MARK(ph) \
  do {                 \
  } while (0)
#endif

// GELU(gate) * up of a work-group's H hidden units -> hid; with H = 32 (one Q8_0 block per work-group) and
// a.hq also the block (quantize_row_q8_0, ops.cpp:116-139, of the same f32 values, 32 lanes), so the down
// launch reads blocks (PLAIN) instead of quantizing the whole hid in every work-group (QUANT)
// fused exchange (a.px_out): the hq block's 12 words (8 of quants, d, nsum8, two zero pads) or the hid values
// are pushed to every rank's mailbox as well
// (returns this thread's checksum terms of the pushed words, px.h)
template <int H>
__device__ __forceinline__ uint32_t gelu_out(const LayerGemv& a, int bid, const float* s_rows, int t, bool fout,
                                             uint32_t tout) {
  if (t >= H) return 0u;
  const float g = gelu_mul1(s_rows[t], s_rows[H + t]);
  a.hid[bid * H + t] = g;
  if constexpr (H == 32) {
    if (a.hq) {
      const Q8Lane b = q8_block_lane(g);
      reinterpret_cast<int8_t*>(a.hq + bid)[t] = (int8_t)b.q;
      if (t == 0) {
        a.hq[bid].d = b.d;
        a.hq[bid].nsum8 = b.nsum8;
      }
      if (fout) {
        const int j = t & 7;
        uint32_t w = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) w |= (uint32_t)(__shfl(b.q, 4 * j + k) & 0xFF) << (8 * k);
        if (t < 12) {
          const uint32_t v = t < 8 ? w : t == 8 ? __float_as_uint(b.d) : t == 9 ? (uint32_t)b.nsum8 : 0u;
          px_push_word(*a.px, tout, bid * 12 + t, v);
          return px_term(v, a.px->rank, bid * 12 + t);
        }
      }
      return 0u;
    }
  }
  if (fout) {
    px_push_word(*a.px, tout, bid * H + t, __float_as_uint(g));
    return px_term(__float_as_uint(g), a.px->rank, bid * H + t);
  }
  return 0u;
}

enum { SYNC_SIG = 1, SYNC_WAIT = 2 };
enum { ROLE_PLAIN = LAYER_PLAIN, ROLE_PRO = LAYER_PRO, ROLE_GELU = LAYER_GELU, ROLE_QUANT = LAYER_QUANT,
       // PRO / GELU with E extra HELPER waves that do the prologue while the
       // NW streaming waves' weight loads are already in flight
       ROLE_PRO_H = 4, ROLE_GELU_H = 5, ROLE_GELU_X = LAYER_GELU_X };
constexpr bool role_help(int r) { return r == ROLE_PRO_H || r == ROLE_GELU_H; }
constexpr int HELP_K4 = 6;  // float4 per helper lane and operand: n <= E * 256 * HELP_K4

// EARLY: issue the weight stream right after the activation loads (small
// weight slices per CU: the issue stall is short and the latency overlaps);
// otherwise after the activation is complete in LDS (see the weight issue).
//
// HELPER roles (ROLE_PRO_H / ROLE_GELU_H, E = NH helper waves after the NW
// streaming waves): the helpers issue the prologue operand loads, one raw
// s_barrier puts them ahead of the weight stream in the CU's queue, then the
// streaming waves issue their weights while the helpers run the residual/norm
// (partial sums exchanged through LDS with a counter, no workgroup barrier)
// and quantize x into LDS; a second raw s_barrier hands x over.  The norm's
// latency hides under the weights' instead of preceding them.
// SYNC (the attention-block kernel in k_attn.hip; 0 everywhere else):
//   SYNC_SIG  -- the qkv rows are published as data-tagged granules (bs.g_qkv);
//   SYNC_WAIT -- (PLAIN) the weight stream is issued first, then the o
//                projection's x blocks are read from their granules
//                (bs.g_xo), each lane re-loading until the tags are this
//                launch's.
// PE (late roles, !EARLY): the first PE passes of the weight chunk are issued
// right after the prologue's operand loads, the rest once x is in LDS -- a
// CU's first weight bytes stream during the prologue without stalling its
// waves at the issue (PE small against the CU's in-flight capacity).
// W8: Q8_0 weights (qs [rows][nb][32 B], row-major) instead of Q4_0.
// WT: K-quant weights in the kq layout (WT_Q4_K / WT_Q6_K; row-major, single
// chunk, R <= 8): the activation blocks hold Q8_K quants (q8k_block_quad).
// RW (0: NW): only waves [0, RW) carry rows; all NW waves run the prologue, so
// its reductions -- and every row's arithmetic -- are those of the RW = NW
// launch while a work-group owns fewer rows (tensor-parallel shard entries:
// more work-groups for a rank's slice, rows bit-identical to one device's;
// row-major weights only).
// PXF: the fused-exchange code (a.px_in / a.px_out honoured); false compiles it out (the one-device launches)
template <int R, int NW, int P, int E, int ROLE, bool MULTI, bool EARLY, int SYNC = 0, int PE = 0, bool W8 = false,
          int WT = 0, int RW0 = 0, bool PXF = false>
__device__ __forceinline__ void layer_body(const LayerGemv& a, const int bid, unsigned char* s_dyn,
                                           const BlockSync& bs) {
  constexpr bool HELP = role_help(ROLE);
  constexpr bool PRO = ROLE == ROLE_PRO || ROLE == ROLE_GELU || HELP;
  constexpr bool GELU = ROLE == ROLE_GELU || ROLE == ROLE_GELU_H || ROLE == ROLE_GELU_X;
  constexpr bool RB = R == 1 || R == 2 || R == 4 || R == 8 || R == 16;  // row-bound lanes, else flat items
  static_assert(!HELP || RB, "helper roles use the row-bound stream");
  constexpr int L = RB ? 64 / R : 64;
  static_assert(PE == 0 || (RB && !MULTI && !EARLY && PE < P), "PE: single-chunk row-bound late roles");
  static_assert(!W8 || (RB && R <= 16), "W8: row-bound lanes");
  static_assert(WT == 0 || (RB && R <= 8 && !MULTI && !HELP && !W8), "kq: single-chunk row-bound lanes");
  static_assert(!(PXF && HELP), "fused exchange: not in the helper roles (their LDS words are ordered differently)");
  LAYER_MARK(0);
  BLK_MARK(bs, 0);
  constexpr int EPT = E, X_LD = E;
  XBlock* s_x = reinterpret_cast<XBlock*>(s_dyn);
  __shared__ float s_red[2][NW];
  __shared__ float s_rows[GELU ? NW * R : 1];
  constexpr int T = NW * 64;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int nb = a.nb;
  constexpr int RW = RW0 > 0 ? RW0 : NW;
  static_assert(RW <= NW && (RW == NW || R == 1 || R == 2 || R == 4 || R == 8 || R == 16), "RW: row-bound lanes");
  const int row0 = (bid * RW + w) * R;
  static_assert(SYNC != SYNC_SIG || ROLE == ROLE_PLAIN || ROLE == ROLE_PRO, "SIG: qkv roles (-> g_qkv)");
  static_assert(SYNC != SYNC_WAIT || ROLE == ROLE_PLAIN, "WAIT: the o projection (<- g_xo)");
  // this launch's granule tag, loaded up front (its latency hides under the prologue)
  const uint32_t btag = SYNC != 0 ? *bs.epoch + 1u : 0u;
  unsigned bcount = 0u;  // SYNC_WAIT (the o work-groups): the tag advance's count, its add's return
  // fused exchanges (tensor-parallel ranks): the tags of the exchange read and of the one written
  const bool fin = PXF && a.px_in >= 0, fout = PXF && a.px_out >= 0;
  const uint32_t tin = fin ? px_link_tag(*a.px, a.px_in) : 0u;
  const uint32_t tout = fout ? px_link_tag(*a.px, a.px_out) : 0u;
  // checksum terms (px.h): of the words this thread pushed / read; the LDS words of their work-group sums
  uint32_t pxs = 0u, pxc = 0u;
  __shared__ uint32_t s_pxs[PXF ? 5 + 2 * PX_MAX_RANKS : 1];
  if (PXF && t < 5 + 2 * PX_MAX_RANKS) s_pxs[t] = 0u;  // (ordered before their use by the barrier after the prologue)
  // the checksum granule of the pushed words, and (the first PX_CHECK_WG work-groups) the check of the words read:
  // every thread of the work-group, at each exit
  auto px_finish = [&]() {
    if constexpr (PXF) {
      if (fout) px_push_checksum(*a.px, tout, bid, pxs, &s_pxs[0]);
      if (fin && bid < PX_CHECK_WG) px_verify(*a.px, tin, a.px_in_nwg, pxc, &s_pxs[1], ROLE * 1000 + a.px_in, bid, a.px_in_ws,
                                                   ROLE == ROLE_PLAIN ? a.nb * 12 : a.nb * 32);
    }
  };
  // SIG: rows are published write-through; the work-group's rows lie in one
  // kv head's group (host-checked: rows per work-group divide head_dim)
  auto put_out = [&](float* p, float v) {
    if constexpr (SYNC == SYNC_SIG) {
      st_granule(bs.g_qkv + (p - a.out), __float_as_uint(v), btag);
    } else {
      *p = v;
      if (fout) {
        px_push_word(*a.px, tout, (int)(p - a.out), __float_as_uint(v));
        pxs += px_term(__float_as_uint(v), a.px->rank, (int)(p - a.out));
      }
    }
  };
  // (RW0 == 0: the expressions of the all-waves launch exactly -- a select the compiler cannot fold away
  // reshuffled the attention block's registers and cost it 1 %)
  const int nrows = RW0 == 0 ? max(0, min(R, a.rows - row0)) : w < RW ? max(0, min(R, a.rows - row0)) : 0;
  const int total = nrows * nb;
  const uint4* qw = a.qs + (size_t)min(row0, a.rows - 1) * nb;
  const uint16_t* dw = a.wd + (size_t)min(row0, a.rows - 1) * nb;
  // RB: this lane's row.  Row-major blocks: descriptors over the wave's rows
  // (wave-uniform base), block b of row k at (k nb + b) x 16 B.  Slab-major
  // (a.slab, nb % 8 == 0, L % 8 == 0): slabs of 8 blocks x all rows, block b
  // of row r at ((b / 8) rows + r) x 128 + (b % 8) x 16 B, so a pass of every
  // wave reads inside the same slab and the chip sweeps memory in order.
  const int rk = lane / L, rj = lane % L;
  const bool row_ok = rk < nrows;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  const int wrow0 = (bid * RW + wu) * R;
  // no rows: every weight load out of bounds (no traffic)
  const int wrows = RW0 == 0 ? max(0, a.rows - wrow0) : wu < RW ? max(0, a.rows - wrow0) : 0;
  __amdgpu_buffer_rsrc_t rq, rd;
  int voq, vod, sq, sd;
  KqOff kq{};
  if (WT != 0 && a.slab) {  // kq slab-major: super-block s of row r at (s rows + r), its 8 sub-blocks contiguous
    const int r = wrow0 + rk, sl = rj >> 3, j8 = rj & 7, ps = (L / 8) * a.rows;
    rq = buf_rsrc(a.qs, (uint32_t)a.rows * nb * 16);
    rd = buf_rsrc(a.wd, (uint32_t)a.rows * nb * 2);
    voq = (sl * a.rows + r) * 128 + j8 * 16;
    vod = (sl * a.rows + r) * 16 + j8 * 2;
    sq = ps * 128;
    sd = ps * 16;
    kq.rdd = buf_rsrc(a.kdd, (uint32_t)a.rows * (nb / 8) * 4);
    kq.vdd = (sl * a.rows + r) * 4;
    kq.sdd = ps * 4;
    if constexpr (WT == WT_Q6_K) {
      kq.rqh = buf_rsrc(a.kqh, (uint32_t)a.rows * nb * 8);
      kq.vqh = (sl * a.rows + r) * 64 + j8 * 8;
      kq.sqh = ps * 64;
    }
  } else if constexpr (WT != 0) {  // kq layout: row-major sub-blocks, super-block words, Q6_K high bits
    const int nsb = nb / 8;
    rq = buf_rsrc(a.qs + (size_t)min(wrow0, a.rows) * nb, (uint32_t)wrows * nb * 16);
    rd = buf_rsrc(a.wd + (size_t)min(wrow0, a.rows) * nb, (uint32_t)wrows * nb * 2);
    voq = (rk * nb + rj) * 16;
    vod = (rk * nb + rj) * 2;
    sq = L * 16;
    sd = L * 2;
    kq.rdd = buf_rsrc(a.kdd + (size_t)min(wrow0, a.rows) * nsb, (uint32_t)wrows * nsb * 4);
    kq.vdd = (rk * nsb + (rj >> 3)) * 4;
    kq.sdd = (L / 8) * 4;
    if constexpr (WT == WT_Q6_K) {
      kq.rqh = buf_rsrc(a.kqh + (size_t)min(wrow0, a.rows) * nb, (uint32_t)wrows * nb * 8);
      kq.vqh = (rk * nb + rj) * 8;
      kq.sqh = L * 8;
    }
  } else if (a.slab) {
    rq = buf_rsrc(a.qs, (uint32_t)a.rows * nb * 16);
    rd = buf_rsrc(a.wd, (uint32_t)a.rows * nb * 2);
    const int r = wrow0 + rk;
    voq = ((rj >> 3) * a.rows + r) * 128 + (rj & 7) * 16;
    vod = ((rj >> 3) * a.rows + r) * 16 + (rj & 7) * 2;
    sq = (L / 8) * a.rows * 128;
    sd = (L / 8) * a.rows * 16;
  } else if constexpr (W8) {  // 16-B units = half blocks; the scale of unit u is block u / 2's
    const int nu = 2 * nb;
    rq = buf_rsrc(a.qs + (size_t)min(wrow0, a.rows) * nu, (uint32_t)wrows * nu * 16);
    rd = buf_rsrc(a.wd + (size_t)min(wrow0, a.rows) * nb, (uint32_t)wrows * nb * 2);
    voq = (rk * nu + rj) * 16;
    vod = (rk * nb + (rj >> 1)) * 2;
    sq = L * 16;
    sd = L;  // (L / 2) scales of 2 B per pass
  } else {
    rq = buf_rsrc(a.qs + (size_t)min(wrow0, a.rows) * nb, (uint32_t)wrows * nb * 16);
    rd = buf_rsrc(a.wd + (size_t)min(wrow0, a.rows) * nb, (uint32_t)wrows * nb * 2);
    voq = (rk * nb + rj) * 16;
    vod = (rk * nb + rj) * 2;
    sq = L * 16;
    sd = L * 2;
  }
  const int npass = ((W8 ? 2 * nb : nb) + L - 1) / L;

  ChunkX<P, WT> ca, cb;
  auto issue_weights = [&]() {
    if constexpr (WT != 0) {
      load_chunk_kq<P, WT, 0, P>(ca, rq, rd, kq, voq, vod, sq, sd, 0, npass);
    } else if constexpr (RB) {
      load_chunk_rb<R, P>(ca, rq, rd, voq, vod, sq, sd, 0, npass);
      if constexpr (MULTI) load_chunk_rb<R, P>(cb, rq, rd, voq, vod, sq, sd, P, npass);
    } else {
      load_chunk<P>(ca, qw, dw, 0, total, lane);  // unconditional (valid clamped rows)
      if constexpr (MULTI) load_chunk<P>(cb, qw, dw, 64 * P, total, lane);
    }
  };
  auto issue_head = [&]() {  // passes [0, PE)
    if constexpr (PE > 0 && WT != 0) load_chunk_kq<P, WT, 0, PE>(ca, rq, rd, kq, voq, vod, sq, sd, 0, npass);
    else if constexpr (PE > 0) load_chunk_rb_part<R, P, 0, PE>(ca, rq, rd, voq, vod, sq, sd, npass);
  };
  auto issue_tail = [&]() {  // passes [PE, P), or everything
    if constexpr (PE > 0 && WT != 0) load_chunk_kq<P, WT, PE, P>(ca, rq, rd, kq, voq, vod, sq, sd, 0, npass);
    else if constexpr (PE > 0) load_chunk_rb_part<R, P, PE, P>(ca, rq, rd, voq, vod, sq, sd, npass);
    else issue_weights();
  };
  const bool helper = HELP && w >= NW;
  if constexpr (HELP) {
    constexpr int NH = E;
    __shared__ float s_hred[2][NH];
    __shared__ int s_hcnt[2];
    float* s_xf = reinterpret_cast<float*>(s_dyn + (size_t)nb * sizeof(XBlock) + 16);
    const int n = a.n, hi = w - NW, seg = n / NH, e0 = hi * seg;
    float4 hy[HELP_K4], hr[HELP_K4], hp[HELP_K4], hn[HELP_K4];
    if (helper) {
      if (hi == 0 && lane < 2) s_hcnt[lane] = 0;
#pragma unroll
      for (int k = 0; k < HELP_K4; k++) {
        const int i = e0 + min((k * 64 + lane) * 4, seg - 4);  // clamped, masked below
        hy[k] = *reinterpret_cast<const float4*>(a.y + i);
        hr[k] = *reinterpret_cast<const float4*>(a.resid_in + i);
        hp[k] = a.w_post ? *reinterpret_cast<const float4*>(a.w_post + i) : make_float4(0.f, 0.f, 0.f, 0.f);
        hn[k] = *reinterpret_cast<const float4*>(a.w_next + i);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the counter reset, before the barrier
    }
    __builtin_amdgcn_s_barrier();  // helpers' operand loads are queued ahead of the weights
    if (!helper) {
      issue_weights();
    } else {
      // helper partial sums -> LDS; every helper adds them in the same order
      auto hsum = [&](int ph, float part) -> float {
        if constexpr (NH == 1) return part;
        if (lane == 0) {
          s_hred[ph][hi] = part;
          __hip_atomic_fetch_add(&s_hcnt[ph], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        while (__hip_atomic_load(&s_hcnt[ph], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) < NH)
          __builtin_amdgcn_s_sleep(1);
        float tot = 0.0f;
#pragma unroll
        for (int j = 0; j < NH; j++) tot += s_hred[ph][j];
        return tot;
      };
      float ss = 0.0f;
#pragma unroll
      for (int k = 0; k < HELP_K4; k++) {
        if ((k * 64 + lane) * 4 < seg) {
          ss = fmaf(hy[k].x, hy[k].x, ss);
          ss = fmaf(hy[k].y, hy[k].y, ss);
          ss = fmaf(hy[k].z, hy[k].z, ss);
          ss = fmaf(hy[k].w, hy[k].w, ss);
        }
      }
      const float sc1 = rms_scale_d(hsum(0, wave_sum(ss)), n, a.eps);
      float ss2 = 0.0f;
#pragma unroll
      for (int k = 0; k < HELP_K4; k++) {
        float4& h = hr[k];
        if (a.w_post) {
          h.x += (sc1 * hy[k].x) * hp[k].x;
          h.y += (sc1 * hy[k].y) * hp[k].y;
          h.z += (sc1 * hy[k].z) * hp[k].z;
          h.w += (sc1 * hy[k].w) * hp[k].w;
        } else {  // no post-norm: plain add
          h.x += hy[k].x;
          h.y += hy[k].y;
          h.z += hy[k].z;
          h.w += hy[k].w;
        }
        const int i = e0 + (k * 64 + lane) * 4;
        if ((k * 64 + lane) * 4 < seg) {
          ss2 = fmaf(h.x, h.x, ss2);
          ss2 = fmaf(h.y, h.y, ss2);
          ss2 = fmaf(h.z, h.z, ss2);
          ss2 = fmaf(h.w, h.w, ss2);
          if (bid == 0) *reinterpret_cast<float4*>(a.resid_out + i) = h;
        }
      }
      const float sc2 = rms_scale_d(hsum(1, wave_sum(ss2)), n, a.eps);
#pragma unroll
      for (int k = 0; k < HELP_K4; k++) {
        const int i = e0 + (k * 64 + lane) * 4;
        if ((k * 64 + lane) * 4 < seg) {
          const float4 x = make_float4((sc2 * hr[k].x) * hn[k].x, (sc2 * hr[k].y) * hn[k].y,
                                       (sc2 * hr[k].z) * hn[k].z, (sc2 * hr[k].w) * hn[k].w);
          *reinterpret_cast<float4*>(s_xf + i) = x;
          if (bid == 0 && a.xn_out) *reinterpret_cast<float4*>(a.xn_out + i) = x;
        }
      }
      // this helper's Q8_0 blocks (seg % 32 == 0), a DPP quad per block; the
      // wave's own LDS writes above are ordered before these reads
      for (int i = lane; i < seg / 8; i += 64) {
        const float4 f0 = reinterpret_cast<const float4*>(s_xf + e0)[2 * i];
        const float4 f1 = reinterpret_cast<const float4*>(s_xf + e0)[2 * i + 1];
        const float v[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
        q8_block_quad(v, i & 3, s_x + e0 / 32 + (i >> 2));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();  // x blocks complete in LDS (no vmcnt wait: the weights stay in flight)
  } else if constexpr (PRO) {
    // prologue operands first: loads return in issue order, so issuing them
    // ahead of the weight chunk lets the norm run while the weights stream.
    // A DPP quad of lanes per Q8_0 block (lane t & 3 owns elements 8 (t & 3)
    // .. + 7 of block t / 4 + k T / 4): vector loads, and x is quantized from
    // registers (no f32 staging of x in LDS).
    constexpr int QB = T / 4;         // blocks per round
    constexpr int EB = (E + 7) / 8;   // rounds: E = ceil(32 nb / T)
    const int n = a.n, sub = t & 3;
    float4 y4[EB][2], r4[EB][2], p4[EB][2], n4[EB][2];
    // buffer loads: slots past the last block are sent out of bounds (0, no
    // memory traffic; 37.5 % of the 4B qkv slots, 50 % of gate_up's) while
    // every load stays unconditional
    const uint32_t vbytes = (uint32_t)nb * 128;
    const __amdgpu_buffer_rsrc_t ry = buf_rsrc(a.y, vbytes), rr = buf_rsrc(a.resid_in, vbytes),
                                 rp = buf_rsrc(a.w_post, a.w_post ? vbytes : 0u), rn = buf_rsrc(a.w_next, vbytes);
    const bool yfx = fin;  // y from this rank's mailbox (fused exchange), after the local operands
#pragma unroll
    for (int k = 0; k < EB; k++) {
      const int b = t / 4 + k * QB;
      const int off = b < nb ? (b * 32 + sub * 8) * 4 : (1 << 30);
#pragma unroll
      for (int h = 0; h < 2; h++) {
        if (!yfx) y4[k][h] = buf_ldf4(ry, off + 16 * h);
        r4[k][h] = buf_ldf4(rr, off + 16 * h);
        p4[k][h] = buf_ldf4(rp, off + 16 * h);
        n4[k][h] = buf_ldf4(rn, off + 16 * h);
      }
    }
    if constexpr (EARLY) issue_weights();
    else issue_head();
    if (yfx) {  // (the weights' first passes are in flight while the peers' words arrive)
#pragma unroll
      for (int k = 0; k < EB; k++) {
        const int b = t / 4 + k * QB;
#pragma unroll
        for (int h = 0; h < 2; h++)
          y4[k][h] = b < nb ? px_read_f4(*a.px, tin, a.px_in_ws, b * 32 + sub * 8 + 4 * h, pxc, true)
                            : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    auto in_row = [&](int k) { return t / 4 + k * QB < nb; };
    float ss = 0.0f;
#pragma unroll
    for (int k = 0; k < EB; k++) {
      if (in_row(k)) {
#pragma unroll
        for (int h = 0; h < 2; h++) {
          ss = fmaf(y4[k][h].x, y4[k][h].x, ss);
          ss = fmaf(y4[k][h].y, y4[k][h].y, ss);
          ss = fmaf(y4[k][h].z, y4[k][h].z, ss);
          ss = fmaf(y4[k][h].w, y4[k][h].w, ss);
        }
      }
    }
    LAYER_MARK(1);
    BLK_MARK(bs, 5);
    const float sc1 = rms_scale_d(wg_sum<NW>(ss, s_red[0]), n, a.eps);
    LAYER_MARK(2);
    BLK_MARK(bs, 6);
    float ss2 = 0.0f;
#pragma unroll
    for (int k = 0; k < EB; k++) {
#pragma unroll
      for (int h = 0; h < 2; h++) {
        float4& r = r4[k][h];
        const float4 y = y4[k][h], wp = p4[k][h];
        if (a.w_post) {
          r.x += (sc1 * y.x) * wp.x;
          r.y += (sc1 * y.y) * wp.y;
          r.z += (sc1 * y.z) * wp.z;
          r.w += (sc1 * y.w) * wp.w;
        } else {  // no post-norm: plain add
          r.x += y.x;
          r.y += y.y;
          r.z += y.z;
          r.w += y.w;
        }
        if (in_row(k)) {
          ss2 = fmaf(r.x, r.x, ss2);
          ss2 = fmaf(r.y, r.y, ss2);
          ss2 = fmaf(r.z, r.z, ss2);
          ss2 = fmaf(r.w, r.w, ss2);
          if (bid == 0 && a.resid_out) *reinterpret_cast<float4*>(a.resid_out + (t / 4 + k * QB) * 32 + sub * 8 + 4 * h) = r;
        }
      }
    }
    const float sc2 = rms_scale_d(wg_sum<NW>(ss2, s_red[1]), n, a.eps);
    LAYER_MARK(3);
    BLK_MARK(bs, 7);
#pragma unroll
    for (int k = 0; k < EB; k++) {
      float v[8];
#pragma unroll
      for (int h = 0; h < 2; h++) {
        const float4 r = r4[k][h], wn = n4[k][h];
        v[4 * h + 0] = (sc2 * r.x) * wn.x;
        v[4 * h + 1] = (sc2 * r.y) * wn.y;
        v[4 * h + 2] = (sc2 * r.z) * wn.z;
        v[4 * h + 3] = (sc2 * r.w) * wn.w;
      }
      if (in_row(k)) {  // whole quads (one block per quad); kq: whole half-waves (one super-block each)
        const int b = t / 4 + k * QB;
        if constexpr (WT != 0) q8k_block_quad(v, sub, s_x + b);
        else q8_block_quad(v, sub, s_x + b);
        if (bid == 0 && a.xn_out) {
          *reinterpret_cast<float4*>(a.xn_out + b * 32 + sub * 8) = make_float4(v[0], v[1], v[2], v[3]);
          *reinterpret_cast<float4*>(a.xn_out + b * 32 + sub * 8 + 4) = make_float4(v[4], v[5], v[6], v[7]);
        }
      }
    }
  } else if constexpr (ROLE == ROLE_QUANT) {
    // a DPP quad of lanes per Q8_0 block (8 floats each): the first E rounds'
    // floats are loaded before the weights and quantized while they stream
    const float4* yb = reinterpret_cast<const float4*>(a.y);
    float4 xr[E][2];
    if (!fin) {
#pragma unroll
      for (int r = 0; r < E; r++) {
        const int i = min(t + r * T, 4 * nb - 1);
        xr[r][0] = yb[2 * i];
        xr[r][1] = yb[2 * i + 1];
      }
    }
    if constexpr (EARLY) issue_weights();
    else issue_head();
    if (fin) {  // fused exchange: from this rank's mailbox, the weights' first passes in flight
#pragma unroll
      for (int r = 0; r < E; r++) {
        const int i = min(t + r * T, 4 * nb - 1);
        const bool own = t + r * T < 4 * nb;  // (clamped duplicates are not counted)
        xr[r][0] = px_read_f4(*a.px, tin, a.px_in_ws, 8 * i, pxc, own);
        xr[r][1] = px_read_f4(*a.px, tin, a.px_in_ws, 8 * i + 4, pxc, own);
      }
    }
#pragma unroll
    for (int r = 0; r < E; r++) {
      const int i = t + r * T;
      if (r * T < 4 * nb) {  // uniform: whole quads are in or out together (4 nb, T multiples of 4)
        const float v[8] = {xr[r][0].x, xr[r][0].y, xr[r][0].z, xr[r][0].w,
                            xr[r][1].x, xr[r][1].y, xr[r][1].z, xr[r][1].w};
        if (i < 4 * nb) {
          if constexpr (WT != 0) q8k_block_quad(v, i & 3, s_x + (i >> 2));
          else q8_block_quad(v, i & 3, s_x + (i >> 2));
        }
      }
    }
  } else {
    // x blocks -> LDS: clamped unconditional loads (no branch between them
    // and the weight loads, so the stores wait only for their own data)
    const uint4* src = reinterpret_cast<const uint4*>(a.xg);
    uint4* dst = reinterpret_cast<uint4*>(s_x);
    const int n16 = nb * 3;
    uint4 xr[X_LD];
    if constexpr (SYNC == SYNC_WAIT) {
      // the weights are independent of the hand-off: in flight before the wait
      issue_weights();
      const uint32_t tag = btag;
      // counted for the launch's tag advance (BlockSync::done) as soon as every wave holds its tag: the asm
      // operand waits for the tag's load only (issued first; loads complete in order), then one add whose
      // return is checked at the end (an add after the hand-off queued behind the other o work-groups' adds and
      // held the launch's tail: 894 vs 918 tok/s)
      asm volatile("" ::"v"(tag));
      __syncthreads();
      if (t == 0) bcount = block_count(bs.done);
#pragma unroll
      for (int k = 0; k < X_LD; k++) {
        uint32_t v[4];
        ld_granules<4>(v, bs.g_xo, min(t + k * T, n16 - 1) * 4, tag, bs.err);
        xr[k] = make_uint4(v[0], v[1], v[2], v[3]);
      }
      BLK_MARK(bs, 4);
    } else if (fin) {  // fused exchange: the blocks from this rank's mailbox (the weights in flight first)
      issue_weights();  // (all of them: the late tail issue below is skipped)
#pragma unroll
      for (int k = 0; k < X_LD; k++) {
        uint32_t v[4];
        px_read_words<4>(*a.px, tin, a.px_in_ws, 4 * min(t + k * T, n16 - 1), v, pxc, t + k * T < n16);
        xr[k] = make_uint4(v[0], v[1], v[2], v[3]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < X_LD; k++) xr[k] = src[min(t + k * T, n16 - 1)];
      if constexpr (EARLY) issue_weights();
    }
#pragma unroll
    for (int k = 0; k < X_LD; k++) dst[min(t + k * T, n16)] = xr[k];  // slot n16: LDS pad (discarded)
  }
  // The activation is complete in LDS BEFORE the weight stream is issued.
  // Issuing weights first does not overlap anything: a CU accepts its waves'
  // weight loads only as fast as its miss queue drains, so any barrier after
  // the weight issue (the prologue's reductions, the x hand-off) waits for
  // most of the CU's weight bytes (phase trace: +2.5-4 us per launch).
  // (HELPER roles: handled above.)
  if constexpr (!HELP) {
    __syncthreads();
    if constexpr (!EARLY && SYNC != SYNC_WAIT)
      if (!(ROLE == ROLE_PLAIN && fin)) issue_tail();
  }

  LAYER_MARK(4);
  BLK_MARK(bs, 1);
  if constexpr (RB) {
    float acc1 = 0.0f;
    if (helper) {
      // helpers have no rows
    } else if constexpr (!MULTI) {
      if constexpr (WT != 0) eat_chunk_kq<R, P, WT>(ca, 0, nb, rj, row_ok, s_x, acc1);
      else if constexpr (W8) eat_chunk_rb_w8<R, P>(ca, 0, nb, rj, row_ok, s_x, acc1);
      else eat_chunk_rb<R, P>(ca, 0, nb, rj, row_ok, s_x, acc1);
    } else {
      // unconditional loads (out-of-range passes return 0 without traffic):
      // no loop-carried phis, so the chunk registers are not copied
      for (int p0 = 0; p0 < npass; p0 += 2 * P) {
        if constexpr (W8) eat_chunk_rb_w8<R, P>(ca, p0, nb, rj, row_ok, s_x, acc1);
        else eat_chunk_rb<R, P>(ca, p0, nb, rj, row_ok, s_x, acc1);
        load_chunk_rb<R, P>(ca, rq, rd, voq, vod, sq, sd, p0 + 2 * P, npass);
        if constexpr (W8) eat_chunk_rb_w8<R, P>(cb, p0 + P, nb, rj, row_ok, s_x, acc1);
        else eat_chunk_rb<R, P>(cb, p0 + P, nb, rj, row_ok, s_x, acc1);
        load_chunk_rb<R, P>(cb, rq, rd, voq, vod, sq, sd, p0 + 3 * P, npass);
      }
    }
    LAYER_MARK(5);
    BLK_MARK(bs, 2);
    float tot[R <= 2 ? R : 1];
    const float v = rb_row_sums<R>(acc1, tot);
    if constexpr (GELU) {
      if (!helper) {
        if constexpr (R <= 2) {
          if (lane == 0)
            for (int k = 0; k < R; k++) s_rows[w * R + k] = tot[k];
        } else {
          if (rj == 0) s_rows[w * R + rk] = v;
        }
      }
      __syncthreads();
      constexpr int H = RW * R / 2;  // hidden units of this work-group
      pxs += gelu_out<H>(a, bid, s_rows, t, fout, tout);
    } else if (!helper) {
      if constexpr (R <= 2) {
        if (lane == 0)
          for (int k = 0; k < R; k++)
            if (k < nrows) put_out(a.out + row0 + k, tot[k]);
      } else {
        if (rj == 0 && row_ok) put_out(a.out + row0 + rk, v);
      }
    }
    BLK_MARK(bs, 3);
    LAYER_MARK(6);
    px_finish();
    if constexpr (SYNC == SYNC_WAIT)
      if (t == 0) block_count_done(bcount, bs.done_n, bs.done, bs.epoch);
    return;
  }
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

  LAYER_MARK(5);
  if constexpr (GELU) {
#pragma unroll
    for (int k = 0; k < R; k++) {
      const float s = wave_sum(acc[k]);
      if (lane == 0) s_rows[w * R + k] = s;
    }
    __syncthreads();
    constexpr int H = RW * R / 2;  // hidden units of this work-group
    pxs += gelu_out<H>(a, bid, s_rows, t, fout, tout);
  } else {
#pragma unroll
    for (int k = 0; k < R; k++) {
      const float s = wave_sum(acc[k]);
      if (lane == 0 && k < nrows) put_out(a.out + row0 + k, s);
    }
  }
  LAYER_MARK(6);
  px_finish();
  if constexpr (SYNC == SYNC_WAIT)
    if (t == 0) block_count_done(bcount, bs.done_n, bs.done, bs.epoch);
}


}  // namespace

}  // namespace llmi
