// Development micro-benchmark of the exact engine's GEMV roles (k_exact.hip compiled in with -DXL_TRACE):
// 4B Gemma-3 shapes, random weights/activations, 20 launches each timed by events, plus the median over
// work-groups of the phase clocks of the last launch (s_memtime cycles from the work-group's start):
//   1 operands in LDS, 2 chain 1 done, 3 h written, 4 chain 2 done, 5 activation (XE) built, 6 rows done.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DXL_TRACE -I llm_inference_amd/csrc \
//        scripts/dev/xl_bench.hip -o scripts/dev/xl_bench
#include "../../llm_inference_amd/csrc/k_exact.hip"

namespace llmi {
void dev_free(void* p) { (void)hipFree(p); }  // (libllmi's cached allocator, k_session.hip; not linked here)
void* dev_alloc(size_t b) {
  void* p = nullptr;
  (void)hipMalloc(&p, b);
  return p;
}
}  // namespace llmi

#include <algorithm>
#include <cstring>
#include <cstdio>
#include <random>
#include <vector>

using namespace llmi;

static DevWeight rand_q4(int rows, int cols, std::mt19937& g) {
  DevWeight w;
  w.type = T_Q4_0;
  w.rows = rows;
  w.cols = cols;
  const size_t nb = (size_t)rows * cols / 32;
  std::vector<uint8_t> q(nb * 16);
  std::vector<uint16_t> d(nb);
  for (auto& b : q) b = (uint8_t)g();
  for (auto& x : d) x = 0x2000 + (g() & 0x3FF);  // small positive f16 scales
  LLMI_HIP(hipMalloc(&w.qs, q.size()));
  LLMI_HIP(hipMalloc(&w.d, d.size() * 2));
  LLMI_HIP(hipMemcpy(w.qs, q.data(), q.size(), hipMemcpyHostToDevice));
  LLMI_HIP(hipMemcpy(w.d, d.data(), d.size() * 2, hipMemcpyHostToDevice));
  w.bytes = nb * 18;
  return w;
}

static float* rand_vec(int n, std::mt19937& g, float sc) {
  std::normal_distribution<float> N(0.0f, sc);
  std::vector<float> h(n);
  for (auto& x : h) x = N(g);
  float* d;
  LLMI_HIP(hipMalloc(&d, n * 4 + 64));
  LLMI_HIP(hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice));
  return d;
}

static void run(const char* name, const XlWeight& w, const XlArgs& a, int role) {
  hipEvent_t e0, e1;
  LLMI_HIP(hipEventCreate(&e0));
  LLMI_HIP(hipEventCreate(&e1));
  for (int i = 0; i < 3; i++) launch_exact_gemv(w, a, role, 0);
  LLMI_HIP(hipDeviceSynchronize());
  const int reps = 20;
  LLMI_HIP(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; i++) launch_exact_gemv(w, a, role, 0);
  LLMI_HIP(hipEventRecord(e1, 0));
  LLMI_HIP(hipEventSynchronize(e1));
  float ms = 0;
  LLMI_HIP(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> tr(8192 * 8);
  LLMI_HIP(hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(g_xl_trace), tr.size() * 8));
  const int nwg = std::min(8192, (w.rows + 63) / 64 * 4);
  std::printf("%-10s %8.2f us/launch  phases (median cycles from WG start):", name, ms * 1000.0 / reps);
  for (int ph = 1; ph <= 6; ph++) {
    std::vector<long long> v;
    for (int b = 0; b < nwg; b++) {
      const unsigned long long t0 = tr[b * 8], t = tr[b * 8 + ph];
      if (t0 && t && t >= t0) v.push_back((long long)(t - t0));
    }
    if (v.empty()) { std::printf("  %d:-", ph); continue; }
    std::sort(v.begin(), v.end());
    std::printf("  %d:%lld", ph, v[v.size() / 2]);
  }
  std::printf("\n");
  std::fflush(stdout);
  std::vector<unsigned long long> z(8192 * 8, 0);
  LLMI_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_xl_trace), z.data(), z.size() * 8));
}

#define XL_MARK_NL(ph) do { } while (0)
// the round-4 first cut of the accumulate kernel (per-lane V loads), for the A/B
namespace llmi {
namespace {
template <int HD>
__global__ __launch_bounds__((HD / 64 + 1) * 64) void xattn_accum_kernel_old(XAttnArgs a) {
  constexpr int NWV = HD / 64, T = (NWV + 1) * 64;
  constexpr int KPT = XA_CH / 256;  // keys per scan thread (threads 0..255)
  __shared__ double s_sc[XA_CH];
  __shared__ __attribute__((aligned(16))) float s_e[XA_CH];   // e per key
  __shared__ __attribute__((aligned(16))) float s_pe[XA_CH];  // pe per key
  __shared__ uint32_t s_up[XA_CH / 32];
  __shared__ double s_tmax[256];
  __shared__ float s_sacc;
  const int h = blockIdx.x, t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int n_keys = *a.d_pos + 1;
  const int hkv = h / (a.n_head / a.n_head_kv);
  const uint16_t* vb = a.v_cache + (size_t)hkv * a.max_ctx * HD + wave * 64 + lane;
  const double* sc_in = a.scores + (size_t)h * a.max_ctx;
  XL_MARK(0);
  double run_max = -INFINITY;
  uint16_t v16 = 0;  // f32_to_f16(0.0f)
  float s_acc = 0.0f;
  for (int c0 = 0; c0 < n_keys; c0 += XA_CH) {
    const int nk = min(XA_CH, n_keys - c0);
    for (int i = t; i < nk; i += T)
      s_sc[i] = a.softcap > 0.0f ? llmi_glibc::softcap_score(sc_in[c0 + i], a.softcap) : sc_in[c0 + i];
    for (int i = t; i < XA_CH / 32; i += T) s_up[i] = 0u;
    __syncthreads();
    XL_MARK(1);
    double tmax = -INFINITY;
    if (t < 256) {
#pragma unroll
      for (int k = 0; k < KPT; k++) {
        const int j = t * KPT + k;
        if (j < nk) tmax = fmax(tmax, s_sc[j]);
      }
      s_tmax[t] = tmax;
    }
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // inclusive prefix max over the 256 segments (max is exact)
      const double v = (t < 256 && t >= o) ? s_tmax[t - o] : -INFINITY;
      __syncthreads();
      if (t < 256) s_tmax[t] = fmax(s_tmax[t], v);
      __syncthreads();
    }
    XL_MARK(2);
    if (t < 256) {
      double pm = fmax(run_max, t > 0 ? s_tmax[t - 1] : -INFINITY);  // max of every key before this segment
#pragma unroll
      for (int k = 0; k < KPT; k++) {
        const int j = t * KPT + k;
        if (j >= nk) break;
        const double score = s_sc[j];
        const float prev = (float)pm;  // the reference's max_score before key j
        if (score > (double)prev) {    // model.cpp:520-532
          s_e[j] = 1.0f;
          s_pe[j] = llmi_glibc::expf(prev - (float)score);
          atomicOr(&s_up[j >> 5], 1u << (j & 31));
        } else {
          s_e[j] = llmi_glibc::expf((float)(score - (double)prev));
          s_pe[j] = 1.0f;
        }
        pm = fmax(pm, score);
      }
    }
    run_max = fmax(run_max, s_tmax[255]);
    __syncthreads();
    XL_MARK(3);
    if (wave < NWV) {  // this lane's head dim: vec_scale_f16 when the max moved, then vec_mad_f16 (ops.cpp:1084-1099)
      const uint16_t* vp = vb + (size_t)c0 * HD;
      // V of 32 keys per batch, the next batch's loads issued before this one is summed (clamped keys past the
      // chunk are loaded but never summed)
      uint32_t va[32], vn[32];  // one f16 per register (low half): the mad8 asm reads them as they are
#pragma unroll
      for (int u = 0; u < 32; u++) va[u] = vp[(size_t)min(u, nk - 1) * HD];
      for (int j0 = 0; j0 < nk; j0 += 32) {
#pragma unroll
        for (int u = 0; u < 32; u++) vn[u] = vp[(size_t)min(j0 + 32 + u, nk - 1) * HD];
        // the batch's max moves (wave-uniform, a scalar branch per key) and e values (broadcast LDS reads)
        const uint32_t up = __builtin_amdgcn_readfirstlane(s_up[j0 >> 5]);
        const int m = __builtin_amdgcn_readfirstlane(min(32, nk - j0));
        float e[32];
#pragma unroll
        for (int u4 = 0; u4 < 8; u4++) {
          const float4 q = reinterpret_cast<const float4*>(s_e + j0)[u4];
          e[4 * u4] = q.x; e[4 * u4 + 1] = q.y; e[4 * u4 + 2] = q.z; e[4 * u4 + 3] = q.w;
        }
        // each step rounds to f32 (the fma), then to f16 (the conversion as its own instruction: fused by the
        // compiler into v_fma_mixlo_f16 it would round once, another f16 whenever the f32 value is a midpoint)
        if (up == 0 && m == 32) {  // the common batch: the max did not move, 32 straight fma + round steps
          uint32_t acc = v16;
#pragma unroll
          for (int u = 0; u < 32; u += 8) xa_mad8(acc, va + u, e + u);
          v16 = (uint16_t)acc;
        } else {
#pragma unroll
          for (int u = 0; u < 32; u++) {
            if (u < m) {
              if (up & (1u << u)) v16 = cvt_f16_rne((float)__builtin_bit_cast(_Float16, v16) * s_pe[j0 + u]);
              v16 = cvt_f16_rne(fmaf((float)__builtin_bit_cast(_Float16, (uint16_t)va[u]), e[u], (float)__builtin_bit_cast(_Float16, v16)));
            }
          }
        }
#pragma unroll
        for (int u = 0; u < 32; u++) va[u] = vn[u];
      }
    } else {  // s_acc = s_acc * pe + e, keys in order (model.cpp:540)
      for (int j0 = 0; j0 < nk; j0 += 4) {
        const float4 e4 = reinterpret_cast<const float4*>(s_e + j0)[0];
        const float4 p4 = reinterpret_cast<const float4*>(s_pe + j0)[0];
        const float ev[4] = {e4.x, e4.y, e4.z, e4.w}, pv[4] = {p4.x, p4.y, p4.z, p4.w};
#pragma unroll
        for (int u = 0; u < 4; u++)
          if (j0 + u < nk) s_acc = s_acc * pv[u] + ev[u];
      }
    }
    XL_MARK(4);
    __syncthreads();  // the chunk's LDS is reused by the next one
    XL_MARK(5);
  }
  if (wave == NWV && lane == 0) s_sacc = s_acc == 0.0f ? 0.0f : 1.0f / s_acc;
  __syncthreads();
  if (wave < NWV) {
    const int d = wave * 64 + lane;
    const float o = h2f(v16) * s_sacc;  // model.cpp:543-547
    a.out[(size_t)h * HD + d] = o;
    q8_block_store(o, true, a.xq + ((size_t)h * HD + wave * 64) / 32 + (lane >> 5), lane & 31);
  }
}

template <int HD>
__global__ __launch_bounds__((HD / 64 + 1) * 64) void xattn_accum_kernel_noload(XAttnArgs a) {
  constexpr int NWV = HD / 64, T = (NWV + 1) * 64;
  constexpr int KPT = XA_CH / 256;  // keys per scan thread (threads 0..255)
  __shared__ double s_sc[XA_CH];
  __shared__ __attribute__((aligned(16))) float s_e[XA_CH];   // e per key
  __shared__ __attribute__((aligned(16))) float s_pe[XA_CH];  // pe per key
  __shared__ uint32_t s_up[XA_CH / 32];
  __shared__ double s_tmax[256];
  __shared__ float s_sacc;
  const int h = blockIdx.x, t = threadIdx.x, wave = t >> 6, lane = t & 63;
  const int n_keys = *a.d_pos + 1;
  const int hkv = h / (a.n_head / a.n_head_kv);
  const uint16_t* vb = a.v_cache + (size_t)hkv * a.max_ctx * HD + wave * 64 + lane;
  const double* sc_in = a.scores + (size_t)h * a.max_ctx;
  XL_MARK_NL(0);
  double run_max = -INFINITY;
  uint16_t v16 = 0;  // f32_to_f16(0.0f)
  float s_acc = 0.0f;
  for (int c0 = 0; c0 < n_keys; c0 += XA_CH) {
    const int nk = min(XA_CH, n_keys - c0);
    for (int i = t; i < nk; i += T)
      s_sc[i] = a.softcap > 0.0f ? llmi_glibc::softcap_score(sc_in[c0 + i], a.softcap) : sc_in[c0 + i];
    for (int i = t; i < XA_CH / 32; i += T) s_up[i] = 0u;
    __syncthreads();
    XL_MARK_NL(1);
    double tmax = -INFINITY;
    if (t < 256) {
#pragma unroll
      for (int k = 0; k < KPT; k++) {
        const int j = t * KPT + k;
        if (j < nk) tmax = fmax(tmax, s_sc[j]);
      }
      s_tmax[t] = tmax;
    }
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // inclusive prefix max over the 256 segments (max is exact)
      const double v = (t < 256 && t >= o) ? s_tmax[t - o] : -INFINITY;
      __syncthreads();
      if (t < 256) s_tmax[t] = fmax(s_tmax[t], v);
      __syncthreads();
    }
    XL_MARK_NL(2);
    if (t < 256) {
      double pm = fmax(run_max, t > 0 ? s_tmax[t - 1] : -INFINITY);  // max of every key before this segment
#pragma unroll
      for (int k = 0; k < KPT; k++) {
        const int j = t * KPT + k;
        if (j >= nk) break;
        const double score = s_sc[j];
        const float prev = (float)pm;  // the reference's max_score before key j
        if (score > (double)prev) {    // model.cpp:520-532
          s_e[j] = 1.0f;
          s_pe[j] = llmi_glibc::expf(prev - (float)score);
          atomicOr(&s_up[j >> 5], 1u << (j & 31));
        } else {
          s_e[j] = llmi_glibc::expf((float)(score - (double)prev));
          s_pe[j] = 1.0f;
        }
        pm = fmax(pm, score);
      }
    }
    run_max = fmax(run_max, s_tmax[255]);
    __syncthreads();
    XL_MARK_NL(3);
    if (wave < NWV) {  // this lane's head dim: vec_scale_f16 when the max moved, then vec_mad_f16 (ops.cpp:1084-1099)
      const uint16_t* vp = vb + (size_t)c0 * HD;
      // V of 32 keys per batch, the next batch's loads issued before this one is summed (clamped keys past the
      // chunk are loaded but never summed)
      uint32_t va[32], vn[32];  // one f16 per register (low half): the mad8 asm reads them as they are
#pragma unroll
      for (int u = 0; u < 32; u++) va[u] = vp[(size_t)min(u, nk - 1) * HD];
      for (int j0 = 0; j0 < nk; j0 += 32) {
#pragma unroll
        for (int u = 0; u < 32; u++) vn[u] = va[u] ^ 1u;  // (timing variant: no V loads in the loop)
        // the batch's max moves (wave-uniform, a scalar branch per key) and e values (broadcast LDS reads)
        const uint32_t up = __builtin_amdgcn_readfirstlane(s_up[j0 >> 5]);
        const int m = __builtin_amdgcn_readfirstlane(min(32, nk - j0));
        float e[32];
#pragma unroll
        for (int u4 = 0; u4 < 8; u4++) {
          const float4 q = reinterpret_cast<const float4*>(s_e + j0)[u4];
          e[4 * u4] = q.x; e[4 * u4 + 1] = q.y; e[4 * u4 + 2] = q.z; e[4 * u4 + 3] = q.w;
        }
        // each step rounds to f32 (the fma), then to f16 (the conversion as its own instruction: fused by the
        // compiler into v_fma_mixlo_f16 it would round once, another f16 whenever the f32 value is a midpoint)
        if (up == 0 && m == 32) {  // the common batch: the max did not move, 32 straight fma + round steps
          uint32_t acc = v16;
#pragma unroll
          for (int u = 0; u < 32; u += 8) xa_mad8(acc, va + u, e + u);
          v16 = (uint16_t)acc;
        } else {
#pragma unroll
          for (int u = 0; u < 32; u++) {
            if (u < m) {
              if (up & (1u << u)) v16 = cvt_f16_rne((float)__builtin_bit_cast(_Float16, v16) * s_pe[j0 + u]);
              v16 = cvt_f16_rne(fmaf((float)__builtin_bit_cast(_Float16, (uint16_t)va[u]), e[u], (float)__builtin_bit_cast(_Float16, v16)));
            }
          }
        }
#pragma unroll
        for (int u = 0; u < 32; u++) va[u] = vn[u];
      }
    } else {  // s_acc = s_acc * pe + e, keys in order (model.cpp:540)
      for (int j0 = 0; j0 < nk; j0 += 4) {
        const float4 e4 = reinterpret_cast<const float4*>(s_e + j0)[0];
        const float4 p4 = reinterpret_cast<const float4*>(s_pe + j0)[0];
        const float ev[4] = {e4.x, e4.y, e4.z, e4.w}, pv[4] = {p4.x, p4.y, p4.z, p4.w};
#pragma unroll
        for (int u = 0; u < 4; u++)
          if (j0 + u < nk) s_acc = s_acc * pv[u] + ev[u];
      }
    }
    XL_MARK_NL(4);
    __syncthreads();  // the chunk's LDS is reused by the next one
    XL_MARK_NL(5);
  }
  if (wave == NWV && lane == 0) s_sacc = s_acc == 0.0f ? 0.0f : 1.0f / s_acc;
  __syncthreads();
  if (wave < NWV) {
    const int d = wave * 64 + lane;
    const float o = h2f(v16) * s_sacc;  // model.cpp:543-547
    a.out[(size_t)h * HD + d] = o;
    q8_block_store(o, true, a.xq + ((size_t)h * HD + wave * 64) / 32 + (lane >> 5), lane & 31);
  }
}

}  // namespace
}  // namespace llmi

template <typename K>
static void time_launch(const char* name, K launch, int reps = 20) {
  hipEvent_t e0, e1;
  LLMI_HIP(hipEventCreate(&e0));
  LLMI_HIP(hipEventCreate(&e1));
  for (int i = 0; i < 3; i++) launch();
  LLMI_HIP(hipDeviceSynchronize());
  LLMI_HIP(hipEventRecord(e0, 0));
  for (int i = 0; i < reps; i++) launch();
  LLMI_HIP(hipEventRecord(e1, 0));
  LLMI_HIP(hipEventSynchronize(e1));
  float ms = 0;
  LLMI_HIP(hipEventElapsedTime(&ms, e0, e1));
  std::printf("%-24s %8.2f us/launch\n", name, ms * 1000.0 / reps);
  std::fflush(stdout);
}

// the PLAIN role at 4 or 8 lanes per row (down: 2560 rows of 320 blocks)
template <int LPR, int NCH>
static void plain_variant(const char* name, const XlWeight& w, const XlArgs& a) {
  const size_t lds = (size_t)w.nb * 64 + (size_t)w.nb * 4;
  const int rpg = 64 / LPR;
  time_launch(name, [&] {
    hipLaunchKernelGGL((exact_gemv_kernel<1, XL_PLAIN, 1, NCH, LPR>), dim3((w.rows + rpg - 1) / rpg), dim3(64), lds, 0,
                       w.qs, w.d, w.rows, w.nb, a);
  });
}

// the split PLAIN kernel against exact_gemv_kernel's PLAIN role: bit-identical rows
static void split_check(const char* name, const XlWeight& w, const XlArgs& a) {
  std::vector<float> o1(w.rows), o2(w.rows);
  const size_t lds = (size_t)w.nb * 64 + (size_t)w.nb * 4;
  hipLaunchKernelGGL((exact_gemv_kernel<1, XL_PLAIN, 1, 4, 4>), dim3(w.rows / 16), dim3(64), lds, 0, w.qs, w.d, w.rows, w.nb, a);
  LLMI_HIP(hipMemcpy(o1.data(), a.out, w.rows * 4, hipMemcpyDeviceToHost));
  LLMI_HIP(hipMemset(a.out, 0, w.rows * 4));
  launch_exact_gemv(w, a, XL_PLAIN, 0);
  LLMI_HIP(hipMemcpy(o2.data(), a.out, w.rows * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int i = 0; i < w.rows; i++) bad += std::memcmp(&o1[i], &o2[i], 4) != 0;
  std::printf("%s split vs serial-lane kernel: %d of %d rows differ (row 0: %.6g %.6g)\n", name, bad, w.rows, o1[0], o2[0]);
}

// the exact attention of one 4B layer at a given position (random K / V history, q|k|v row, norms, rope)
static void phases(const char* what, int H);
static void phases_quiet();
static void attn_bench(std::mt19937& g, int pos) {
  const int H = 8, HK = 4, HD = 256, MC = 4096;
  XAttnArgs x;
  x.qkv = rand_vec((H + 2 * HK) * HD, g, 1.0f);
  x.k_off = H * HD;
  x.v_off = (H + HK) * HD;
  x.n_head = H;
  x.n_head_kv = HK;
  x.head_dim = HD;
  x.q_norm_w = rand_vec(HD, g, 0.3f);
  x.k_norm_w = rand_vec(HD, g, 0.3f);
  x.rope_cs = rand_vec(MC * HD, g, 0.7f);
  x.attn_scale = 0.0625f;
  x.eps = 1e-6;
  const size_t kvn = (size_t)HK * MC * HD;
  std::vector<uint16_t> hk(kvn);
  std::normal_distribution<float> N(0.0f, 1.0f);
  for (auto& v : hk) { const _Float16 hv = (_Float16)N(g); std::memcpy(&v, &hv, 2); }
  LLMI_HIP(hipMalloc(&x.k_cache, kvn * 2));
  LLMI_HIP(hipMalloc(&x.v_cache, kvn * 2));
  LLMI_HIP(hipMemcpy(x.k_cache, hk.data(), kvn * 2, hipMemcpyHostToDevice));
  {  // the per-key exactness words (exact.h XAttnArgs::kmeta) of the random K rows
    std::vector<uint32_t> km((size_t)HK * MC);
    for (size_t r = 0; r < (size_t)HK * MC; r++) {
      int code = 31;
      uint32_t mag = 0;
      for (int d = 0; d < HD; d++) {
        const uint16_t b = hk[r * HD + d];
        if (b & 0x7FFF) code = std::min(code, std::max((b >> 10) & 0x1F, 1));
        mag = std::max(mag, (uint32_t)(b & 0x7FFF));
      }
      km[r] = ((uint32_t)code << 16) | mag;
    }
    LLMI_HIP(hipMalloc(&x.kmeta, km.size() * 4));
    LLMI_HIP(hipMemcpy(x.kmeta, km.data(), km.size() * 4, hipMemcpyHostToDevice));
  }
  for (auto& v : hk) { const _Float16 hv = (_Float16)N(g); std::memcpy(&v, &hv, 2); }
  LLMI_HIP(hipMemcpy(x.v_cache, hk.data(), kvn * 2, hipMemcpyHostToDevice));
  {  // the tiled copy the scores kernel maintains (exact.h XAttnArgs::vt)
    x.vt_stride = MC;
    std::vector<uint16_t> vt(kvn);
    for (int kv = 0; kv < HK; kv++)
      for (int p = 0; p < MC; p++)
        for (int d = 0; d < HD; d++)
          vt[(((size_t)kv * (HD / 64) + d / 64) * (MC / 32) + p / 32) * 2048 + ((p & 31) >> 3) * 512 + (d & 63) * 8 +
             (p & 7)] = hk[((size_t)kv * MC + p) * HD + d];
    LLMI_HIP(hipMalloc(&x.vt, kvn * 2));
    LLMI_HIP(hipMemcpy(x.vt, vt.data(), kvn * 2, hipMemcpyHostToDevice));
  }
  x.max_ctx = MC;
  int* dp;
  LLMI_HIP(hipMalloc(&dp, 4));
  LLMI_HIP(hipMemcpy(dp, &pos, 4, hipMemcpyHostToDevice));
  x.d_pos = dp;
  LLMI_HIP(hipMalloc(&x.scores, (size_t)H * MC * 8));
  LLMI_HIP(hipMalloc(&x.out, (size_t)H * HD * 4));
  LLMI_HIP(hipMalloc(&x.xq, (size_t)H * HD / 32 * sizeof(XBlock)));
  char nm[64];
  std::snprintf(nm, sizeof nm, "attn both (pos %d)", pos);
  time_launch(nm, [&] { launch_exact_attn(x, 0); });
  phases_quiet();
  std::snprintf(nm, sizeof nm, "attn scores (pos %d)", pos);
  time_launch(nm, [&] { hipLaunchKernelGGL(xattn_scores_kernel<256>, dim3(H, XA_NSPLIT + 1), dim3(64), 0, 0, x); });
  phases("scores (all WGs)", H * (XA_NSPLIT + 1));
  std::snprintf(nm, sizeof nm, "attn accum (pos %d)", pos);
  time_launch(nm, [&] { hipLaunchKernelGGL(xattn_accum_kernel<256>, dim3(H), dim3(320), 0, 0, x); });
  phases("accum", H);
  std::vector<uint32_t> o_new((size_t)H * HD), o_old((size_t)H * HD);
  LLMI_HIP(hipMemcpy(o_new.data(), x.out, o_new.size() * 4, hipMemcpyDeviceToHost));
  {  // the same launch with every V load inside the first 4-KB tile (L1 hits): the V fetch's share
    const int st = x.vt_stride;
    x.vt_stride = 32;
    std::snprintf(nm, sizeof nm, "attn accum cheapV (pos %d)", pos);
    time_launch(nm, [&] { hipLaunchKernelGGL(xattn_accum_kernel<256>, dim3(H), dim3(320), 0, 0, x); });
    phases("accum cheapV", H);
    x.vt_stride = st;
  }
  std::snprintf(nm, sizeof nm, "attn accum old (pos %d)", pos);
  time_launch(nm, [&] { hipLaunchKernelGGL(xattn_accum_kernel_old<256>, dim3(H), dim3(320), 0, 0, x); });
  LLMI_HIP(hipMemcpy(o_old.data(), x.out, o_old.size() * 4, hipMemcpyDeviceToHost));
  {
    int bad = 0;
    for (size_t i = 0; i < o_new.size(); i++) bad += o_new[i] != o_old[i];
    std::printf("   accum vs the round-4 kernel (pos %d): %d of %zu outputs differ\n", pos, bad, o_new.size());
  }
  std::snprintf(nm, sizeof nm, "attn accum no-V (pos %d)", pos);
  time_launch(nm, [&] { hipLaunchKernelGGL(xattn_accum_kernel_noload<256>, dim3(H), dim3(320), 0, 0, x); });
  phases("accum old", H);
}

static void phases_quiet() {
  std::vector<unsigned long long> z(8192 * 8, 0);
  LLMI_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_xl_trace), z.data(), z.size() * 8));
}
// phase clocks of the last launch, median over the heads' work-groups
static void phases(const char* what, int H) {
  {
    std::vector<unsigned long long> tr(8192 * 8);
    LLMI_HIP(hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(g_xl_trace), tr.size() * 8));
    std::printf("   %s phases (cycles): ", what);
    for (int ph = 1; ph <= 5; ph++) {
      std::vector<long long> v;
      for (int b = 0; b < H; b++)
        if (tr[b * 8] && tr[b * 8 + ph]) v.push_back((long long)(tr[b * 8 + ph] - tr[b * 8]));
      std::sort(v.begin(), v.end());
      std::printf(" %d:%lld", ph, v.empty() ? -1LL : v[v.size() / 2]);
    }
    std::printf("\n");
    std::vector<unsigned long long> z(8192 * 8, 0);
    LLMI_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_xl_trace), z.data(), z.size() * 8));
  }
}

// dependent-chain latency of the accumulate's step shapes: one wave, 1024 steps, cycles per step
__device__ unsigned long long g_lat[8];
template <int MODE>
__global__ __launch_bounds__(64) void lat_kernel(float e, uint32_t v) {
  uint32_t a = threadIdx.x, b = threadIdx.x + 7;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 1024; i++) {
    if (MODE == 0)
      asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]\n\tv_cvt_f16_f32_e32 %0, %0" : "+v"(a) : "v"(v), "v"(e));
    else if (MODE == 1)
      asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(a) : "v"(v), "v"(e));
    else if (MODE == 2)
      asm volatile("v_cvt_f16_f32_e32 %0, %0" : "+v"(a));
    else if (MODE == 3)
      asm volatile("v_fma_mix_f32 %0, %2, %3, %0 op_sel_hi:[1,0,1]\n\tv_fma_mix_f32 %1, %2, %3, %1 op_sel_hi:[1,0,1]\n\t"
                   "v_cvt_f16_f32_e32 %0, %0\n\tv_cvt_f16_f32_e32 %1, %1"
                   : "+v"(a), "+v"(b) : "v"(v), "v"(e));
    else if (MODE == 4)
      asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(a) : "v"(v), "v"(e));
    else if (MODE == 5)
      asm volatile("v_fma_mixlo_f16 %0, %1, %2, %0 op_sel_hi:[1,0,1]" : "+v"(a) : "v"(v), "v"(e));
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) g_lat[MODE] = t1 - t0 + (a + b == 12345u ? 1 : 0);
}
// f64: the scores kernel's element step (f16 -> f32 -> f64, fma) as one dependent chain (MODE 0) or four (1)
__device__ unsigned long long g_lat64[4];
template <int MODE>
__global__ __launch_bounds__(64) void lat64_kernel(const uint32_t* kw, double q) {
  double a0 = threadIdx.x, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  uint32_t w = kw[threadIdx.x];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < 256; i++) {
    w = w * 1664525u + 1013904223u;  // (independent of the chain)
    const double x = (double)h2f((uint16_t)(w & 0x7BFF)), y = (double)h2f((uint16_t)((w >> 16) & 0x7BFF));
    if (MODE == 0) {
      a0 = fma(x, q, a0);
      a0 = fma(y, q, a0);
    } else if (MODE == 1) {
      a0 = fma(x, q, a0);
      a1 = fma(y, q, a1);
      i++;
      w = w * 1664525u + 1013904223u;
      const double x2 = (double)h2f((uint16_t)(w & 0x7BFF)), y2 = (double)h2f((uint16_t)((w >> 16) & 0x7BFF));
      a2 = fma(x2, q, a2);
      a3 = fma(y2, q, a3);
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) g_lat64[MODE] = t1 - t0 + (a0 + a1 + a2 + a3 == 1.2345 ? 1 : 0);
}
static void latency_bench() {
  const char* nm[] = {"fma_mix+cvt", "fma_f32", "cvt_f16", "2 chains fma_mix+cvt", "fma_mix", "fma_mixlo"};
  hipLaunchKernelGGL(lat_kernel<0>, dim3(1), dim3(64), 0, 0, 0.5f, 0x3c00u);
  hipLaunchKernelGGL(lat_kernel<1>, dim3(1), dim3(64), 0, 0, 0.5f, 0x3c00u);
  hipLaunchKernelGGL(lat_kernel<2>, dim3(1), dim3(64), 0, 0, 0.5f, 0x3c00u);
  hipLaunchKernelGGL(lat_kernel<3>, dim3(1), dim3(64), 0, 0, 0.5f, 0x3c00u);
  hipLaunchKernelGGL(lat_kernel<4>, dim3(1), dim3(64), 0, 0, 0.5f, 0x3c00u);
  hipLaunchKernelGGL(lat_kernel<5>, dim3(1), dim3(64), 0, 0, 0.5f, 0x3c00u);
  LLMI_HIP(hipDeviceSynchronize());
  unsigned long long l[8];
  LLMI_HIP(hipMemcpyFromSymbol(l, HIP_SYMBOL(g_lat), sizeof l));
  for (int m = 0; m < 6; m++) std::printf("latency %-22s %6.2f cycles/step\n", nm[m], l[m] / 1024.0);
  uint32_t* kw;
  LLMI_HIP(hipMalloc(&kw, 256));
  LLMI_HIP(hipMemset(kw, 0x11, 256));
  hipLaunchKernelGGL(lat64_kernel<0>, dim3(1), dim3(64), 0, 0, kw, 0.37);
  hipLaunchKernelGGL(lat64_kernel<1>, dim3(1), dim3(64), 0, 0, kw, 0.37);
  LLMI_HIP(hipDeviceSynchronize());
  unsigned long long l64[4];
  LLMI_HIP(hipMemcpyFromSymbol(l64, HIP_SYMBOL(g_lat64), sizeof l64));
  std::printf("f64 element step, one chain  %6.2f cycles/element\n", l64[0] / 512.0);
  std::printf("f64 element step, four chains %6.2f cycles/element\n", l64[1] / 512.0);
}

// the norm chain variants alone: 256 threads, 2560 random floats per work-group in LDS, cycles + fallbacks
template <int V>
__global__ __launch_bounds__(256) void sumsq_kernel(const float* x, unsigned long long* cyc, float* res, unsigned* fb) {
  __shared__ __attribute__((aligned(16))) float s[2560];
  __shared__ float s_out;
  for (int i = threadIdx.x; i < 2560; i += 256) s[i] = x[(size_t)blockIdx.x * 2560 + i];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  float r;
  if (V == 0) r = xl_chain_spec<4>(s, 2560, fb);
  else if (V == 1) r = xl_chain_spec2<4>(s, 2560, fb);
  else if (V == 3) r = xl_chain_spec_fast<4>(s, 2560);
  else {
    if (threadIdx.x < 64) { const float v = xl_chain(s, 2560); if (threadIdx.x == 0) s_out = v; }
    __syncthreads();
    r = s_out;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) { cyc[blockIdx.x] = t1 - t0; res[blockIdx.x] = r; }
}
static void sumsq_bench(std::mt19937& g) {
  const int NB = 64;
  float* x = rand_vec(NB * 2560, g, 1.0f);
  unsigned long long* cyc; float* res; unsigned* fb;
  LLMI_HIP(hipMalloc(&cyc, NB * 8)); LLMI_HIP(hipMalloc(&res, NB * 4)); LLMI_HIP(hipMalloc(&fb, 4));
  // (a 16-segment x 2-candidate form with spec_fast's costs measured 5.5K vs 5.3K cycles: not kept)
  std::vector<float> r[4];
  const char* nm[] = {"spec<4> (8 segs)", "spec2<4> (16 segs x 2)", "serial", "spec_fast<4> (8 segs)"};
  for (int v = 0; v < 4; v++) {
    LLMI_HIP(hipMemset(fb, 0, 4));
    for (int rep = 0; rep < 2; rep++) {
      if (v == 0) hipLaunchKernelGGL(sumsq_kernel<0>, dim3(NB), dim3(256), 0, 0, x, cyc, res, fb);
      if (v == 1) hipLaunchKernelGGL(sumsq_kernel<1>, dim3(NB), dim3(256), 0, 0, x, cyc, res, fb);
      if (v == 2) hipLaunchKernelGGL(sumsq_kernel<2>, dim3(NB), dim3(256), 0, 0, x, cyc, res, fb);
      if (v == 3) hipLaunchKernelGGL(sumsq_kernel<3>, dim3(NB), dim3(256), 0, 0, x, cyc, res, fb);
    }
    LLMI_HIP(hipDeviceSynchronize());
    std::vector<unsigned long long> c(NB);
    r[v].resize(NB);
    unsigned f;
    LLMI_HIP(hipMemcpy(c.data(), cyc, NB * 8, hipMemcpyDeviceToHost));
    LLMI_HIP(hipMemcpy(r[v].data(), res, NB * 4, hipMemcpyDeviceToHost));
    LLMI_HIP(hipMemcpy(&f, fb, 4, hipMemcpyDeviceToHost));
    std::sort(c.begin(), c.end());
    std::printf("sumsq %-24s median %llu cycles (min %llu max %llu), fallbacks %u over 2 x %d chains\n", nm[v], c[NB / 2],
                c[0], c[NB - 1], f, NB);
  }
  int bad = 0;
  for (int i = 0; i < NB; i++)
    bad += (std::memcmp(&r[0][i], &r[2][i], 4) != 0) + (std::memcmp(&r[1][i], &r[2][i], 4) != 0) +
           (std::memcmp(&r[3][i], &r[2][i], 4) != 0);
  std::printf("sumsq variants vs serial: %d mismatches\n", bad);
}

int main() {
  latency_bench();
  {
    std::mt19937 g0(7);
    sumsq_bench(g0);
  }
  std::mt19937 g(1);
  const int E = 2560, F = 10240;
  DevWeight wq = rand_q4(4096, E, g), wgate = rand_q4(F, E, g), wup = rand_q4(F, E, g), wd = rand_q4(E, F, g);
  XlSrc sq; sq.w[sq.n++] = &wq;
  XlSrc sgu; sgu.w[sgu.n++] = &wgate; sgu.w[sgu.n++] = &wup; sgu.gelu32 = true;
  XlSrc sd; sd.w[sd.n++] = &wd;
  XlWeight xq = make_xl_weight(sq, 0), xgu = make_xl_weight(sgu, 0), xd = make_xl_weight(sd, 0);
  float *y = rand_vec(E, g, 1.0f), *r0 = rand_vec(E, g, 1.0f), *r1 = rand_vec(E, g, 1.0f), *wp = rand_vec(E, g, 0.3f),
        *wn = rand_vec(E, g, 0.3f), *out = rand_vec(F * 2, g, 1.0f), *hid = rand_vec(F, g, 1.0f);
  XBlock *hq, *xb;
  LLMI_HIP(hipMalloc(&hq, F / 32 * sizeof(XBlock)));
  LLMI_HIP(hipMalloc(&xb, F / 32 * sizeof(XBlock)));
  LLMI_HIP(hipMemset(xb, 0, F / 32 * sizeof(XBlock)));
  XlArgs pre;
  pre.y = y; pre.w_post = wp; pre.resid_in = r0; pre.resid_out = r1; pre.w_next = wn; pre.n = E; pre.eps = 1e-6;
  pre.out = out;
  run("qkv PRE", xq, pre, XL_PRE);
  {  // the split-row PRE (SPR 16) against the 64-row form: bit-identical q|k|v rows
    std::vector<float> o1(xq.rows), o2(xq.rows);
    const size_t lds = (size_t)xq.nb * 64 + (size_t)xq.nb * 4 + (size_t)2 * pre.n * 4;
    hipLaunchKernelGGL((exact_gemv_kernel<4, XL_PRE, 3, 2>), dim3(xq.rows / 64), dim3(256), lds, 0, xq.qs, xq.d, xq.rows,
                       xq.nb, pre);
    LLMI_HIP(hipMemcpy(o1.data(), pre.out, xq.rows * 4, hipMemcpyDeviceToHost));
    LLMI_HIP(hipMemset(pre.out, 0, xq.rows * 4));
    hipLaunchKernelGGL((exact_gemv_kernel<4, XL_PRE, 3, 2, 4, 16>), dim3(xq.rows / 16), dim3(256), lds, 0, xq.qs, xq.d,
                       xq.rows, xq.nb, pre);
    LLMI_HIP(hipGetLastError());
    LLMI_HIP(hipMemcpy(o2.data(), pre.out, xq.rows * 4, hipMemcpyDeviceToHost));
    int bad = 0, first = -1;
    for (int i = 0; i < xq.rows; i++)
      if (std::memcmp(&o1[i], &o2[i], 4) != 0) { bad++; if (first < 0) first = i; }
    std::printf("qkv split vs 64-row PRE: %d of %d rows differ (first %d: %.6g vs %.6g)\n", bad, xq.rows, first,
                first >= 0 ? o1[first] : 0.f, first >= 0 ? o2[first] : 0.f);
  }
  XlArgs gu = pre;
  gu.out = nullptr; gu.hid = hid; gu.hq = hq;
  run("gate_up", xgu, gu, XL_GELU);
  XlArgs dn;
  dn.xb = hq; dn.out = out;
  run("down", xd, dn, XL_PLAIN);
  plain_variant<4, 4>("down LPR4 NCH4", xd, dn);
  split_check("down", xd, dn);
  {  // the o projection's shape (2560 x 2048)
    DevWeight wo = rand_q4(E, 2048, g);
    XlSrc so; so.w[so.n++] = &wo;
    XlWeight xo = make_xl_weight(so, 0);
    XlArgs oa;
    oa.xb = hq; oa.out = out;
    run("o", xo, oa, XL_PLAIN);
    plain_variant<4, 4>("o LPR4 NCH4 (old)", xo, oa);
    split_check("o", xo, oa);
  }
  plain_variant<8, 4>("down LPR8 NCH4", xd, dn);
  plain_variant<8, 2>("down LPR8 NCH2", xd, dn);
  attn_bench(g, 1);
  attn_bench(g, 64);
  attn_bench(g, 600);
  attn_bench(g, 2000);
  return 0;
}
