// Development micro-benchmark of the exact engine's GEMV roles (k_exact.hip compiled in with -DXL_TRACE):
// 4B Gemma-3 shapes, random weights/activations, 20 launches each timed by events, plus the median over
// work-groups of the phase clocks of the last launch (s_memtime cycles from the work-group's start):
//   1 operands in LDS, 2 chain 1 done, 3 h written, 4 chain 2 done, 5 activation (XE) built, 6 rows done.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DXL_TRACE -I llm_inference_amd/csrc \
//        scripts/dev/xl_bench.hip -o scripts/dev/xl_bench
#include "../../llm_inference_amd/csrc/k_exact.hip"

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

// the exact attention of one 4B layer at a given position (random K / V history, q|k|v row, norms, rope)
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
  for (auto& v : hk) { const _Float16 hv = (_Float16)N(g); std::memcpy(&v, &hv, 2); }
  LLMI_HIP(hipMemcpy(x.v_cache, hk.data(), kvn * 2, hipMemcpyHostToDevice));
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
  std::snprintf(nm, sizeof nm, "attn scores (pos %d)", pos);
  time_launch(nm, [&] { hipLaunchKernelGGL(xattn_scores_kernel<256>, dim3(H, XA_NSPLIT), dim3(64), 0, 0, x); });
  std::snprintf(nm, sizeof nm, "attn accum (pos %d)", pos);
  time_launch(nm, [&] { hipLaunchKernelGGL(xattn_accum_kernel<256>, dim3(H), dim3(320), 0, 0, x); });
}

int main() {
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
  XlArgs gu = pre;
  gu.out = nullptr; gu.hid = hid; gu.hq = hq;
  run("gate_up", xgu, gu, XL_GELU);
  XlArgs dn;
  dn.xb = hq; dn.out = out;
  run("down", xd, dn, XL_PLAIN);
  plain_variant<4, 4>("down LPR4 NCH4", xd, dn);
  plain_variant<8, 4>("down LPR8 NCH4", xd, dn);
  plain_variant<8, 2>("down LPR8 NCH2", xd, dn);
  attn_bench(g, 600);
  attn_bench(g, 2000);
  return 0;
}
