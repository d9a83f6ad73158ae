// k_session.hip -- weight upload/repack and the fused glue kernels of the
// decode step (residual + norms, GELU + quantize, argmax, token feedback).
#include "session_kernels.h"
#include "spec_chain.h"

#include <mutex>
#include <unordered_map>
#include <vector>

namespace llmi {

// ---------------------------------------------------------------------------
// weight upload: GGUF blocks -> device SoA layout (kernels.h)
// ---------------------------------------------------------------------------
__global__ void repack_q4_0_kernel(const uint8_t* __restrict__ src, size_t n_blocks, uint4* __restrict__ qs,
                                   uint16_t* __restrict__ d) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_blocks) return;
  const uint8_t* b = src + i * 18;
  d[i] = (uint16_t)(b[0] | (b[1] << 8));
  uint32_t w[4];
#pragma unroll
  for (int k = 0; k < 4; k++)
    w[k] = (uint32_t)b[2 + 4 * k] | ((uint32_t)b[3 + 4 * k] << 8) | ((uint32_t)b[4 + 4 * k] << 16) |
           ((uint32_t)b[5 + 4 * k] << 24);
  qs[i] = make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ void repack_q8_0_kernel(const uint8_t* __restrict__ src, size_t n_blocks, uint4* __restrict__ qs,
                                   uint16_t* __restrict__ d) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_blocks) return;
  const uint8_t* b = src + i * 34;
  d[i] = (uint16_t)(b[0] | (b[1] << 8));
  uint32_t w[8];
#pragma unroll
  for (int k = 0; k < 8; k++)
    w[k] = (uint32_t)b[2 + 4 * k] | ((uint32_t)b[3 + 4 * k] << 8) | ((uint32_t)b[4 + 4 * k] << 16) |
           ((uint32_t)b[5 + 4 * k] << 24);
  qs[2 * i] = make_uint4(w[0], w[1], w[2], w[3]);
  qs[2 * i + 1] = make_uint4(w[4], w[5], w[6], w[7]);
}

size_t gguf_bytes(uint32_t type, size_t rows, size_t cols) {
  switch (type) {
    case T_F32: return rows * cols * 4;
    case T_F16: case T_BF16: return rows * cols * 2;
    case T_Q4_0: return rows * (cols / 32) * 18;
    case T_Q5_0: return rows * (cols / 32) * 22;
    case T_Q8_0: return rows * (cols / 32) * 34;
    case T_Q4_K: return rows * (cols / 256) * 144;
    case T_Q6_K: return rows * (cols / 256) * 210;
    default: return 0;
  }
}

bool gemv_type_supported(uint32_t type) {
  return type == T_Q4_0 || type == T_Q8_0 || type == T_F16 || type == T_Q4_K || type == T_Q6_K || type == T_Q5_0 ||
         type == T_BF16;
}

// Device memory of the sessions.  (1) While a session is being CONSTRUCTED and
// another is alive, released memory does not go back to reuse: with several sessions constructed together in one
// process (the one-GPU tensor-parallel group), memory one session freed and another reallocated at the same time
// was read wrong on its first use -- one word of a weight row, right on every later read (a one-GPU 4-rank group:
// 8 of 23 lifetimes; 0 of 2,868 with the frees held back, scripts/dev/tp_diag.py).  Such frees wait in a
// graveyard released when the last construction ends (round 6: was the last session's end, which let a
// long-lived session plus repeatedly created and closed ones grow device memory without bound).  (2) Released blocks stay mapped: they are kept by size and handed to the next
// allocation of that size instead of hipFree + hipMalloc (a 4-rank group constructed after a whole-model session
// closed still read 0.012-off logits once in a full suite run: the same signature); the cache is returned to
// the allocator when an allocation fails or it exceeds kCacheCap.
namespace {
std::mutex g_mem_mu;
int g_live_sessions = 0;
int g_constructing = 0;            // sessions between session_live(+1) and session_constructed()
std::vector<void*> g_graveyard;
size_t g_grave_bytes = 0;
std::unordered_map<void*, size_t> g_sizes;       // live blocks from dev_alloc: rounded size
std::unordered_multimap<size_t, void*> g_cache;  // released blocks, still mapped
size_t g_cached = 0;
constexpr size_t kGran = 64 << 10, kCacheCap = (size_t)48 << 30;

void flush_cache_locked() {
  for (auto& kv : g_cache) (void)hipFree(kv.second);
  g_cache.clear();
  g_cached = 0;
}
// LLMI_DEV_CACHE=0: released blocks go straight back through hipFree (the cache is a speed measure -- repeated
// session creation without remapping -- not the correctness fix: tests/test_tp.py runs the concurrent-construction
// case with it off)
bool cache_off() {
  const char* e = getenv("LLMI_DEV_CACHE");
  return e && e[0] == '0';
}
void release_locked(void* p) {  // (no other session alive)
  auto it = g_sizes.find(p);
  if (it == g_sizes.end() || cache_off()) {  // not from dev_alloc, or the cache off
    if (it != g_sizes.end()) g_sizes.erase(it);
    (void)hipFree(p);
    return;
  }
  g_cache.emplace(it->second, p);
  g_cached += it->second;
  g_sizes.erase(it);
  if (g_cached > kCacheCap) flush_cache_locked();
}
}  // namespace

void* dev_alloc(size_t bytes) {
  const size_t sz = (bytes + kGran - 1) / kGran * kGran;
  std::lock_guard<std::mutex> lk(g_mem_mu);
  auto it = g_cache.find(sz);
  if (it != g_cache.end()) {
    void* p = it->second;
    g_cache.erase(it);
    g_cached -= sz;
    g_sizes[p] = sz;
    return p;
  }
  void* p = nullptr;
  if (hipMalloc(&p, sz) != hipSuccess) {  // out of memory: the cached blocks back to the allocator, once
    (void)hipGetLastError();
    flush_cache_locked();
    LLMI_HIP(hipMalloc(&p, sz));
  }
  g_sizes[p] = sz;
  return p;
}

namespace {
void flush_graveyard_locked() {
  for (void* p : g_graveyard) release_locked(p);
  g_graveyard.clear();
  g_grave_bytes = 0;
}
}  // namespace

void dev_free(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_mem_mu);
  if (g_constructing > 0 && g_live_sessions > 1) {
    g_graveyard.push_back(p);
    auto it = g_sizes.find(p);
    g_grave_bytes += it != g_sizes.end() ? it->second : 0;
  } else {
    release_locked(p);
  }
}

void session_live(int delta) {
  std::lock_guard<std::mutex> lk(g_mem_mu);
  g_live_sessions += delta;
  if (delta > 0) g_constructing += delta;
  if (g_constructing == 0 || g_live_sessions == 0) flush_graveyard_locked();
}

void session_constructed(bool ok) {  // the end of a constructor (ok) or of a failed one (its release ran first)
  std::lock_guard<std::mutex> lk(g_mem_mu);
  if (g_constructing > 0) g_constructing--;
  if (g_constructing == 0) flush_graveyard_locked();
  (void)ok;
}

void dev_mem_stats(size_t* live, size_t* cached, size_t* grave) {
  std::lock_guard<std::mutex> lk(g_mem_mu);
  size_t n = 0;
  for (const auto& kv : g_sizes) n += kv.second;
  *live = n;
  *cached = g_cached;
  *grave = g_grave_bytes;
}

// Upload `rows` rows of a GGUF weight (host bytes in block layout) to the
// device, appending after `dst_row0` rows of an existing allocation `w`
// (used to fuse q|k|v and gate|up into one GEMV).  w must be pre-allocated.
void upload_rows(DevWeight& w, int dst_row0, const void* host, int rows, hipStream_t s) {
  const size_t bytes = gguf_bytes(w.type, rows, w.cols);
  if (w.type == T_Q4_0 || w.type == T_Q8_0) {
    const int nb = w.cols / 32;
    const size_t nblk = (size_t)rows * nb;
    void* tmp = nullptr;
    tmp = dev_alloc(bytes);
    LLMI_HIP(hipMemcpyAsync(tmp, host, bytes, hipMemcpyHostToDevice, s));
    const size_t b0 = (size_t)dst_row0 * nb;
    if (w.type == T_Q4_0)
      hipLaunchKernelGGL(repack_q4_0_kernel, dim3((nblk + 255) / 256), dim3(256), 0, s, (const uint8_t*)tmp, nblk,
                         (uint4*)w.qs + b0, w.d + b0);
    else
      hipLaunchKernelGGL(repack_q8_0_kernel, dim3((nblk + 255) / 256), dim3(256), 0, s, (const uint8_t*)tmp, nblk,
                         (uint4*)w.qs + 2 * b0, w.d + b0);
    LLMI_HIP(hipGetLastError());
    LLMI_HIP(hipStreamSynchronize(s));
    dev_free(tmp);
  } else {
    const size_t off = gguf_bytes(w.type, dst_row0, w.cols);
    LLMI_HIP(hipMemcpyAsync((uint8_t*)w.qs + off, host, bytes, hipMemcpyHostToDevice, s));
    LLMI_HIP(hipStreamSynchronize(s));
  }
}

DevWeight alloc_weight(uint32_t type, int rows, int cols, size_t slack) {
  if (!gemv_type_supported(type))
    throw std::runtime_error("mat_vec_mul: unsupported tensor type " + std::to_string(type));
  DevWeight w;
  w.type = type;
  w.rows = rows;
  w.cols = cols;
  w.bytes = gguf_bytes(type, rows, cols);
  if (type == T_Q4_0 || type == T_Q8_0) {
    const size_t nblk = (size_t)rows * (cols / 32);
    w.qs = dev_alloc(nblk * (type == T_Q4_0 ? 16 : 32) + slack);
    w.d = static_cast<uint16_t*>(dev_alloc(nblk * 2 + slack));
  } else {
    w.qs = dev_alloc(w.bytes + slack);
  }
  return w;
}

__global__ void slab_permute_kernel(const uint4* __restrict__ qs, const uint16_t* __restrict__ d, int rows, int nb,
                                    uint4* __restrict__ qs2, uint16_t* __restrict__ d2) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // source block (row-major)
  if (i >= (size_t)rows * nb) return;
  const int r = (int)(i / nb), b = (int)(i % nb);
  const size_t j = ((size_t)(b >> 3) * rows + r) * 8 + (b & 7);
  qs2[j] = qs[i];
  d2[j] = d[i];
}

void to_slab_layout(DevWeight& w, hipStream_t s) {
  if (w.type != T_Q4_0 || w.cols % 256 != 0 || w.slab) throw std::runtime_error("to_slab_layout: Q4_0, cols % 256");
  const int nb = w.cols / 32;
  const size_t nblk = (size_t)w.rows * nb;
  void* q2 = nullptr;
  uint16_t* d2 = nullptr;
  q2 = dev_alloc(nblk * 16 + 64);
  d2 = static_cast<uint16_t*>(dev_alloc(nblk * 2 + 64));
  hipLaunchKernelGGL(slab_permute_kernel, dim3((nblk + 255) / 256), dim3(256), 0, s, (const uint4*)w.qs, w.d, w.rows,
                     nb, (uint4*)q2, d2);
  LLMI_HIP(hipGetLastError());
  LLMI_HIP(hipStreamSynchronize(s));
  dev_free(w.qs);
  dev_free(w.d);
  w.qs = q2;
  w.d = d2;
  w.slab = 1;
}

void free_weight(DevWeight& w) {
  dev_free(w.qs);
  dev_free(w.d);
  dev_free(w.kdd);
  dev_free(w.kqh);
  w.qs = nullptr;
  w.d = nullptr;
  w.kdd = nullptr;
  w.kqh = nullptr;
}

// ---- GGUF K-quant rows -> the kq layout (kernels.h), one thread per sub-block
__device__ __forceinline__ void kq_scale_min(int j, const uint8_t* q, int& d, int& m) {  // get_scale_min_k4 (ops.cpp)
  if (j < 4) {
    d = q[j] & 63;
    m = q[j + 4] & 63;
  } else {
    d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
    m = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
  }
}

// destination of source super-block sbk (row-major: row * nsb + s): itself, or
// slab-major (s * rows + row: super-block s of every row together)
__device__ __forceinline__ size_t kq_dst(size_t sbk, int rows, int nsb) {
  if (!rows) return sbk;
  return (sbk % nsb) * rows + sbk / nsb;
}

__global__ void repack_q4_k_kernel(const uint8_t* __restrict__ src, size_t n_sub, uint4* __restrict__ qs,
                                   uint16_t* __restrict__ sc, uint32_t* __restrict__ dd, int slab_rows, int nsb) {
  const size_t u0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;  // sub-block (row-major: row * nsub + j)
  if (u0 >= n_sub) return;
  const size_t sbk = u0 / 8, dsb = kq_dst(sbk, slab_rows, nsb), u = dsb * 8 + u0 % 8;
  const int j = (int)(u0 % 8);
  const uint8_t* b = src + sbk * 144;
  const uint8_t* q = b + 16 + 32 * (j / 2);
  const int sh = (j & 1) * 4;
  uint32_t w[4];
  for (int k = 0; k < 4; k++) {
    uint32_t v = 0;
    for (int i = 0; i < 4; i++) {
      const int e = 4 * k + i;  // byte e: element e (low nibble), element 16 + e (high nibble)
      v |= (uint32_t)(((q[e] >> sh) & 0xF) | (((q[16 + e] >> sh) & 0xF) << 4)) << (8 * i);
    }
    w[k] = v;
  }
  qs[u] = make_uint4(w[0], w[1], w[2], w[3]);
  int d6, m6;
  kq_scale_min(j, b + 4, d6, m6);
  sc[u] = (uint16_t)(d6 | (m6 << 8));
  if (j == 0) dd[dsb] = (uint32_t)b[0] | ((uint32_t)b[1] << 8) | ((uint32_t)b[2] << 16) | ((uint32_t)b[3] << 24);
}

__global__ void repack_q6_k_kernel(const uint8_t* __restrict__ src, size_t n_sub, uint4* __restrict__ qs,
                                   uint16_t* __restrict__ sc, uint32_t* __restrict__ dd, uint2* __restrict__ qh,
                                   int slab_rows, int nsb) {
  const size_t u0 = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (u0 >= n_sub) return;
  const size_t sbk = u0 / 8, dsb = kq_dst(sbk, slab_rows, nsb), u = dsb * 8 + u0 % 8;
  const int m = (int)(u0 % 8), n = m / 4, jq = m % 4;
  const uint8_t* b = src + sbk * 210;
  const uint8_t* ql = b + 64 * n + 32 * (jq & 1);
  const uint8_t* qhb = b + 128 + 32 * n;
  auto q6 = [&](int l) {  // element l of the sub-block, 0..63
    return ((ql[l] >> (4 * (jq >> 1))) & 0xF) | (((qhb[l] >> (2 * jq)) & 3) << 4);
  };
  uint32_t w[4];
  uint32_t h[2] = {0u, 0u};
  for (int k = 0; k < 4; k++) {
    uint32_t v = 0;
    for (int i = 0; i < 4; i++) {
      const int e = 4 * k + i;
      const int lo = q6(e), hi = q6(16 + e);
      v |= (uint32_t)((lo & 0xF) | ((hi & 0xF) << 4)) << (8 * i);
      h[0] |= (uint32_t)(lo >> 4) << (8 * i + 2 * k);
      h[1] |= (uint32_t)(hi >> 4) << (8 * i + 2 * k);
    }
    w[k] = v;
  }
  qs[u] = make_uint4(w[0], w[1], w[2], w[3]);
  qh[u] = make_uint2(h[0], h[1]);
  const uint8_t* scb = b + 192 + 8 * n + 2 * jq;
  sc[u] = (uint16_t)(scb[0] | (scb[1] << 8));
  if (m == 0) dd[dsb] = (uint32_t)b[208] | ((uint32_t)b[209] << 8);
}

void to_kq_layout(DevWeight& w, hipStream_t s, int slab) {
  if ((w.type != T_Q4_K && w.type != T_Q6_K) || w.kq || w.cols % 256) throw std::runtime_error("to_kq_layout: weight");
  const size_t nsb = (size_t)w.rows * (w.cols / 256), nsub = nsb * 8;
  const int srows = slab ? w.rows : 0, rsb = w.cols / 256;
  uint4* qs;
  uint16_t* sc;
  uint32_t* dd;
  uint2* qh = nullptr;
  qs = static_cast<uint4*>(dev_alloc(nsub * 16 + 64));
  sc = static_cast<uint16_t*>(dev_alloc(nsub * 2 + 64));
  dd = static_cast<uint32_t*>(dev_alloc(nsb * 4 + 64));
  const dim3 grid((unsigned)((nsub + 255) / 256));
  if (w.type == T_Q4_K) {
    hipLaunchKernelGGL(repack_q4_k_kernel, grid, dim3(256), 0, s, (const uint8_t*)w.qs, nsub, qs, sc, dd, srows, rsb);
  } else {
    qh = static_cast<uint2*>(dev_alloc(nsub * 8 + 64));
    hipLaunchKernelGGL(repack_q6_k_kernel, grid, dim3(256), 0, s, (const uint8_t*)w.qs, nsub, qs, sc, dd, qh, srows, rsb);
  }
  LLMI_HIP(hipGetLastError());
  LLMI_HIP(hipStreamSynchronize(s));
  dev_free(w.qs);
  w.qs = qs;
  w.d = sc;
  w.kdd = dd;
  w.kqh = qh;
  w.kq = 1;
  w.slab = slab ? 1 : 0;
}

// ---------------------------------------------------------------------------
// block-wide sum helper (<= 1024 threads), fixed order
// ---------------------------------------------------------------------------
__device__ float block_sum(float v, float* sh) {
  const int t = threadIdx.x, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if ((t & 63) == 0) sh[t >> 6] = v;
  __syncthreads();
  float tot = 0.0f;
  for (int i = 0; i < nw; i++) tot += sh[i];
  return tot;
}

// serial (reference-order) sum of squares: sum = fma(v, v, sum) in index order
__device__ float serial_sumsq(const float* x, int n, float* sh) {
  __shared__ float s_r;
  if (threadIdx.x == 0) {
    float sum = 0.0f;
    for (int i = 0; i < n; i++) sum = fmaf(x[i], x[i], sum);
    s_r = sum;
  }
  __syncthreads();
  const float r = s_r;
  __syncthreads();
  (void)sh;
  return r;
}

__device__ __forceinline__ float rms_scale(float sum, int n, double eps) {  // ops.cpp:37-38
  return 1.0f / sqrtf((float)((double)(sum / (float)n) + eps));
}

// ---------------------------------------------------------------------------
// Fused residual step (model.cpp:843-858 / 915-924 + next run_norm):
//   a = rms_norm(y) * w_post             (post_attention / post_ffw norm)
//   h = resid + a ; resid = h            (residual add)
//   xn = rms_norm(h) * w_next            (ffn_norm / next layer attn_norm /
//                                         output_norm)
// One block of 1024 threads, every operand prefetched into registers up front
// (one memory round trip), n <= 8192.  Also emits the next GEMV's activation:
// Q8_0 blocks (quantize_row_q8_0 semantics) and/or f16-rounded x (logits).
// ---------------------------------------------------------------------------
constexpr int NORM_EPT = 8;  // elements per thread (n <= 8192)

// Q8_K of one 256-element super-block (quantize_row_q8_k, ops.cpp:142-178,
// as quantize_q8_k_kernel): a group of 256 threads (threadIdx.x / 256) reads
// element threadIdx.x % 256 of xs.  Every thread of the block calls it (two
// block-wide barriers); groups with active == false only take part in them.
__device__ void q8k_group(const float* xs, bool active, uint8_t* blk, float* s_ax, int* s_ix) {
  const int t = threadIdx.x, tl = t & 255, lane = t & 63, w = t >> 6, g4 = (t >> 8) * 4;
  const float v = active ? xs[tl] : 0.0f;
  float ax = fabsf(v);
  int ix = tl;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {  // max |x|, first index on ties (strict > scan)
    const float oa = __shfl_xor(ax, o);
    const int oi = __shfl_xor(ix, o);
    if (oa > ax || (oa == ax && oi < ix)) { ax = oa; ix = oi; }
  }
  if (lane == 0) { s_ax[w] = ax; s_ix[w] = ix; }
  __syncthreads();
  float amax = s_ax[g4];
  int imax = s_ix[g4];
  for (int k = 1; k < 4; k++)
    if (s_ax[g4 + k] > amax || (s_ax[g4 + k] == amax && s_ix[g4 + k] < imax)) { amax = s_ax[g4 + k]; imax = s_ix[g4 + k]; }
  __syncthreads();  // s_ax / s_ix free for the next call
  if (!active) return;  // no barriers below
  if (amax == 0.0f) {  // ops.cpp:158-163
    blk[4 + tl] = 0;
    if (tl < 16) { blk[260 + 2 * tl] = 0; blk[261 + 2 * tl] = 0; }
    if (tl == 0) *reinterpret_cast<float*>(blk) = 0.0f;
    return;
  }
  const float iscale = -127.f / xs[imax];
  int q = nearest_int_fma(iscale, v);
  q = q < -128 ? -128 : (q > 127 ? 127 : q);
  blk[4 + tl] = (uint8_t)(int8_t)q;
  int sum = q;  // 16-lane group sums -> bsums
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
  if ((tl & 15) == 0) {
    const int16_t s16 = (int16_t)sum;
    blk[260 + 2 * (tl >> 4)] = (uint8_t)(s16 & 0xFF);
    blk[261 + 2 * (tl >> 4)] = (uint8_t)((uint16_t)s16 >> 8);
  }
  if (tl == 0) *reinterpret_cast<float*>(blk) = 1.0f / iscale;
}

// s_h: n floats of LDS (free again: callers are past their last use of it).
// Q8_0 blocks: x staged in LDS, one DPP quad per block (q8_block_quad, bit-identical to the one-thread
// q8_block_serial this used: 27B's 168 blocks as serial 32-element chains made the launch 5.8 us)
__device__ __forceinline__ void norm_outputs(const float (&xv)[NORM_EPT], int n, const NormOut& out, float* s_h) {
  const int t = threadIdx.x;
  __syncthreads();  // s_h reuse
#pragma unroll
  for (int k = 0; k < NORM_EPT; k++) {
    const int i = t + k * 1024;
    if (i < n) {
      out.xn[i] = xv[k];
      s_h[i] = xv[k];
      if (out.x16) out.x16[i] = f2h_ggml(xv[k]);
    }
  }
  if (out.q8) {
    __syncthreads();
    const int sub = t & 3;
    for (int b = t >> 2; b < n / 32; b += 256) {  // whole quads in or out together
      const float4 f0 = reinterpret_cast<const float4*>(s_h + 32 * b + 8 * sub)[0];
      const float4 f1 = reinterpret_cast<const float4*>(s_h + 32 * b + 8 * sub)[1];
      const float v[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
      q8_block_quad(v, sub, out.q8 + b);
    }
  }
  if (out.q8k) {  // one wave per Q8_K super-block (n % 256 == 0: host-checked), no block barriers
    __syncthreads();
    const int lane = t & 63;
    for (int sb = t >> 6; sb < n / 256; sb += 16) {
      const float* xs = s_h + sb * 256;
      uint8_t* blk = out.q8k + (size_t)sb * 292;
      float v[4], ax = -1.0f;
      int ix = 0;
#pragma unroll
      for (int k = 0; k < 4; k++) {  // element lane + 64 k; first index of the max |x| (strict > scan)
        v[k] = xs[lane + 64 * k];
        if (fabsf(v[k]) > ax) { ax = fabsf(v[k]); ix = lane + 64 * k; }
      }
#pragma unroll
      for (int o = 32; o >= 1; o >>= 1) {
        const float oa = __shfl_xor(ax, o);
        const int oi = __shfl_xor(ix, o);
        if (oa > ax || (oa == ax && oi < ix)) { ax = oa; ix = oi; }
      }
      if (ax == 0.0f) {  // ops.cpp:158-163
#pragma unroll
        for (int k = 0; k < 4; k++) blk[4 + lane + 64 * k] = 0;
        if (lane < 32) blk[260 + lane] = 0;
        if (lane == 0) *reinterpret_cast<float*>(blk) = 0.0f;
        continue;
      }
      const float iscale = -127.f / xs[ix];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        int q = nearest_int_fma(iscale, v[k]);
        q = q < -128 ? -128 : (q > 127 ? 127 : q);
        blk[4 + lane + 64 * k] = (uint8_t)(int8_t)q;
        int sum = q;  // elements 64 k + 16 (lane / 16) .. + 15: bsums[4 k + lane / 16]
#pragma unroll
        for (int o = 8; o >= 1; o >>= 1) sum += __shfl_xor(sum, o);
        if ((lane & 15) == 0) {
          const int16_t s16 = (int16_t)sum;
          const int j = 4 * k + (lane >> 4);
          blk[260 + 2 * j] = (uint8_t)(s16 & 0xFF);
          blk[261 + 2 * j] = (uint8_t)((uint16_t)s16 >> 8);
        }
      }
      if (lane == 0) *reinterpret_cast<float*>(blk) = 1.0f / iscale;
    }
  }
  if (out.scr) {  // the screening's x16 blocks from the same f16 roundings (screen_prep_kernel's arithmetic)
    __shared__ double s_l1[256];  // n <= 8192: at most 256 blocks, one quad each
    __syncthreads();  // s_h holds xv
    const int b = t >> 2, sub = t & 3;
    if (b < n / 32) {
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; i++) v[i] = h2f(f2h_ggml(s_h[32 * b + 8 * sub + i]));
      const double l1 = screen_prep_quad(v, sub, n, out.scr + b);
      if (sub == 0) s_l1[b] = l1;
    }
    __syncthreads();
    if (t < 64) screen_prep_total(s_l1, n / 32, out.scr, out.scr_mkey);
  }
}

template <bool EXACT>
__device__ __forceinline__ float sumsq_regs(const float (&v)[NORM_EPT], int n, float* s_h, float* sh) {
  if (EXACT) {  // stage, then the reference's serial fma chain (ops.cpp:33-36): speculative over the block's first
    // 4 waves where n splits into 8 segments of whole float4s (round 5: one thread's chain of dependent LDS loads
    // was ~25K cycles per 2560-term norm), bit-identical (spec_chain.h)
#pragma unroll
    for (int k = 0; k < NORM_EPT; k++)
      if (threadIdx.x + k * 1024 < n) s_h[threadIdx.x + k * 1024] = v[k];
    __syncthreads();
    if (n % 32 == 0 && n / 32 <= 192) return xl_chain_spec_fast<4, 1024>(s_h, n);
    return serial_sumsq(s_h, n, sh);
  }
  float sq = 0.0f;
#pragma unroll
  for (int k = 0; k < NORM_EPT; k++) sq = fmaf(v[k], v[k], sq);
  return block_sum(sq, sh);
}

template <bool EXACT>
__global__ __launch_bounds__(1024) void residual_norm_kernel(const float* __restrict__ y,
                                                             const float* __restrict__ w_post,
                                                             float* __restrict__ resid,
                                                             const float* __restrict__ w_next, NormOut out, int n,
                                                             double eps, float post_scale) {
  extern __shared__ float s_h[];  // [n]: exact-mode sum staging, then the Q8_0 staging
  __shared__ float sh[16];
  const int t = threadIdx.x;
  float yv[NORM_EPT], rv[NORM_EPT], wp[NORM_EPT], wn[NORM_EPT];
#pragma unroll
  for (int k = 0; k < NORM_EPT; k++) {
    const int i = t + k * 1024;
    const bool ok = i < n;
    yv[k] = ok ? y[i] : 0.0f;
    rv[k] = ok ? resid[i] : 0.0f;
    wp[k] = (ok && w_post) ? w_post[i] : 0.0f;
    wn[k] = ok ? w_next[i] : 0.0f;
  }
  const float sc1 = rms_scale(sumsq_regs<EXACT>(yv, n, s_h, sh), n, eps);
  float hv[NORM_EPT];
#pragma unroll
  for (int k = 0; k < NORM_EPT; k++) {
    const int i = t + k * 1024;
    const float a = w_post ? (sc1 * yv[k]) * wp[k] : yv[k];
    hv[k] = rv[k] + a;
    if (post_scale != 1.0f) hv[k] = hv[k] * post_scale;  // Gemma-4 layer output scale (model.cpp:968-977)
    if (i < n) resid[i] = hv[k];
  }
  if (EXACT) __syncthreads();  // s_h reuse
  const float sc2 = rms_scale(sumsq_regs<EXACT>(hv, n, s_h, sh), n, eps);
  float xv[NORM_EPT];
#pragma unroll
  for (int k = 0; k < NORM_EPT; k++) xv[k] = (sc2 * hv[k]) * wn[k];
  norm_outputs(xv, n, out, s_h);
}

void launch_residual_norm(const float* y, const float* w_post, float* resid, const float* w_next, const NormOut& out,
                          int n, double eps, bool exact, hipStream_t s, float post_scale) {
  if (n > 1024 * NORM_EPT) throw std::runtime_error("residual_norm: n_embd > 8192");
  if (exact)
    hipLaunchKernelGGL(residual_norm_kernel<true>, dim3(1), dim3(1024), (size_t)n * 4, s, y, w_post, resid, w_next, out,
                       n, eps, post_scale);
  else
    hipLaunchKernelGGL(residual_norm_kernel<false>, dim3(1), dim3(1024), (size_t)n * 4, s, y, w_post, resid, w_next,
                       out, n, eps, post_scale);
  LLMI_HIP(hipGetLastError());
}

// Gemma-4 per-layer inputs, second half of project_per_layer_inputs
// (model.cpp:676-701): per layer l, nx = rms_norm(proj[l]) (ops.cpp:28-43),
// inp[l] = (nx * nw + inp[l]) * (1 / sqrt(2)).  proj was scaled by
// 1/sqrt(n_embd) by the caller (model.cpp:651-652).  One 256-thread block per layer.
template <bool EXACT>
__global__ __launch_bounds__(256) void ple_combine_kernel(const float* __restrict__ proj, const float* __restrict__ nw,
                                                          float* __restrict__ inp, int ep, double eps) {
  __shared__ float sh[16];
  const float* p = proj + (size_t)blockIdx.x * ep;
  float* d = inp + (size_t)blockIdx.x * ep;
  float sum;
  if (EXACT) {
    sum = serial_sumsq(p, ep, sh);
  } else {
    float sq = 0.0f;
    for (int i = threadIdx.x; i < ep; i += blockDim.x) sq = fmaf(p[i], p[i], sq);
    sum = block_sum(sq, sh);
  }
  const float sc = rms_scale(sum, ep, eps);
  const float is = 1.0f / sqrtf(2.0f);
  for (int i = threadIdx.x; i < ep; i += blockDim.x) {
    const float nx = sc * p[i];
    d[i] = (nx * nw[i] + d[i]) * is;
  }
}

void launch_ple_combine(const float* proj, const float* nw, float* inp, int n_layer, int n_epl, double eps, bool exact,
                        hipStream_t s) {
  if (exact)
    hipLaunchKernelGGL(ple_combine_kernel<true>, dim3(n_layer), dim3(256), 0, s, proj, nw, inp, n_epl, eps);
  else
    hipLaunchKernelGGL(ple_combine_kernel<false>, dim3(n_layer), dim3(256), 0, s, proj, nw, inp, n_epl, eps);
  LLMI_HIP(hipGetLastError());
}

__global__ void softcap_kernel(float* x, int n, float cap) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) x[i] = cap * llmi_glibc::tanhf(x[i] / cap);
}
void launch_softcap(float* x, int n, float cap, hipStream_t s) {
  hipLaunchKernelGGL(softcap_kernel, dim3((n + 255) / 256), dim3(256), 0, s, x, n, cap);
  LLMI_HIP(hipGetLastError());
}

// embedding row * sqrt(n_embd) (model.cpp:240-344) + first attn_norm
template <bool EXACT>
__global__ __launch_bounds__(1024) void embed_norm_kernel(uint32_t type, const uint8_t* __restrict__ table,
                                                          size_t row_bytes, const int32_t* __restrict__ d_token,
                                                          float emb_scale, float* __restrict__ resid,
                                                          const float* __restrict__ w, float* __restrict__ xn, int n,
                                                          double eps);

// ---------------------------------------------------------------------------
// GELU(tanh)(gate) * up (model.cpp:892-899) fused with quantize_row_q8_0 of the
// result (ops.cpp:116-139) for the down projection: one 32-lane half-wave per
// Q8_0 block.  Also writes the f32 hidden vector (parity/debug).  Bit-exact
// GELU (glibc tanhf): this launch serves exact mode and the ops.h surface.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gelu_quant_kernel(const float* __restrict__ gu, int n, float* __restrict__ hid,
                                                         XBlock* __restrict__ xb) {
  const int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const bool ok = gl < n;
  const float v = ok ? gelu_mul1<true>(gu[gl], gu[n + gl]) : 0.0f;  // the unfused / exact path: glibc tanhf
  if (ok) hid[gl] = v;
  if (xb != nullptr) q8_block_store(v, ok && (gl >> 5) < n / 32, xb + (ok ? (gl >> 5) : 0), gl & 31);
}

// the same with the GELU output's Q8_K super-blocks (one block = one super-block)
__global__ __launch_bounds__(256) void gelu_quant_k_kernel(const float* __restrict__ gu, int n, float* __restrict__ hid,
                                                           uint8_t* __restrict__ q8k) {
  __shared__ float s_x[256];
  __shared__ float s_ax[4];
  __shared__ int s_ix[4];
  const int gl = blockIdx.x * 256 + threadIdx.x;
  const float v = gelu_mul1<true>(gu[gl], gu[n + gl]);
  hid[gl] = v;
  s_x[threadIdx.x] = v;
  __syncthreads();
  q8k_group(s_x, true, q8k + (size_t)blockIdx.x * 292, s_ax, s_ix);
}

void launch_gelu_quant(const float* gu, int n, float* hid, const Q8Act* q8, hipStream_t s, uint8_t* q8k) {
  if (q8k) {
    if (n % 256 || q8) throw std::runtime_error("gelu_quant: Q8_K output needs n % 256 == 0 and no Q8_0 output");
    hipLaunchKernelGGL(gelu_quant_k_kernel, dim3(n / 256), dim3(256), 0, s, gu, n, hid, q8k);
  } else {
    hipLaunchKernelGGL(gelu_quant_kernel, dim3((n + 255) / 256), dim3(256), 0, s, gu, n, hid, q8 ? q8->xb : nullptr);
  }
  LLMI_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// argmax (first maximal index, main.cpp:193-194) folded into a 64-bit key
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void argmax_kernel(const float* __restrict__ x, int n,
                                                      unsigned long long* __restrict__ key) {
  unsigned long long best = 0;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const unsigned long long k = argmax_key(x[i], (uint32_t)i);
    best = k > best ? k : best;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const unsigned long long other = __shfl_xor(best, o);
    best = other > best ? other : best;
  }
  if ((threadIdx.x & 63) == 0) atomicMax(key, best);
}

void launch_argmax(const float* x, int n, unsigned long long* key, hipStream_t s) {
  hipLaunchKernelGGL(argmax_kernel, dim3(64), dim3(1024), 0, s, x, n, key);
  LLMI_HIP(hipGetLastError());
}

// token feedback: next token = argmax, pos += 1, record, reset key.  With
// row-sharded logits key q holds the best of vocabulary
// rows [q * shard, (q + 1) * shard) by local index; the winner is re-keyed by
// global index so ties resolve to the lowest id, as the whole-vocab argmax.
// The buffers are distinct (__restrict__) and every load is issued before the first store: one memory
// round trip instead of three dependent ones (the single thread's launch was ~4.2 us).
__global__ void finalize_token_kernel(unsigned long long* __restrict__ keys, int n_keys, int shard,
                                      int32_t* __restrict__ d_token, int32_t* __restrict__ d_pos,
                                      int32_t* __restrict__ ring, int32_t* __restrict__ ring_idx, int ring_cap) {
  unsigned long long best = keys[0];
  const int pos = *d_pos, i = *ring_idx;
  keys[0] = 0;
  for (int q = 1; q < n_keys; q++) {
    const unsigned long long k = keys[q];
    keys[q] = 0;
    if (k == 0) continue;
    const uint32_t gi = (uint32_t)q * (uint32_t)shard + argmax_key_index(k);
    const unsigned long long kg = (k & 0xFFFFFFFF00000000ull) | (0xFFFFFFFFu - gi);
    if (kg > best) best = kg;
  }
  // no key at all (every logit NaN: no row compared as a maximum): token 0 rather than an index past the table
  const uint32_t tok = best ? argmax_key_index(best) : 0u;
  *d_token = (int32_t)tok;
  *d_pos = pos + 1;
  if (i < ring_cap) ring[i] = (int32_t)tok;
  *ring_idx = i + 1;
}

void launch_finalize_token(unsigned long long* keys, int n_keys, int shard, int32_t* d_token, int32_t* d_pos,
                           int32_t* ring, int32_t* ring_idx, int ring_cap, hipStream_t s) {
  hipLaunchKernelGGL(finalize_token_kernel, dim3(1), dim3(1), 0, s, keys, n_keys, shard, d_token, d_pos, ring,
                     ring_idx, ring_cap);
  LLMI_HIP(hipGetLastError());
}

// the token loop's per-token inputs as kernel arguments (no host staging buffer, so no stream sync and no
// pinned-memory copy between the step-graph replays)
__global__ void set_token_pos_kernel(int32_t* d_token, int32_t* d_pos, int32_t* ring_idx, int token, int pos, int reset) {
  *d_token = token;
  *d_pos = pos;
  if (reset) *ring_idx = 0;
}
void launch_set_token_pos(int32_t* d_token, int32_t* d_pos, int32_t* ring_idx, int token, int pos, bool reset,
                          hipStream_t s) {
  hipLaunchKernelGGL(set_token_pos_kernel, dim3(1), dim3(1), 0, s, d_token, d_pos, ring_idx, token, pos, reset ? 1 : 0);
  LLMI_HIP(hipGetLastError());
}

// ---------------------------------------------------------------------------
// embedding lookup + scale + first attn_norm, in one block
// ---------------------------------------------------------------------------
__device__ float deq_embed(uint32_t type, const uint8_t* row, int i);

template <bool EXACT>
__global__ __launch_bounds__(1024) void embed_norm_kernel(uint32_t type, const uint8_t* __restrict__ table,
                                                          size_t row_bytes, const int32_t* __restrict__ d_token,
                                                          float emb_scale, float* __restrict__ resid,
                                                          const float* __restrict__ w, NormOut out, int n,
                                                          double eps) {
  extern __shared__ float s_h[];  // [n]: exact-mode sum staging, then the Q8_0 staging
  __shared__ float sh[16];
  const int t = threadIdx.x;
  const uint8_t* row = table + (size_t)(*d_token) * row_bytes;
  float ev[NORM_EPT], wv[NORM_EPT];
#pragma unroll
  for (int k = 0; k < NORM_EPT; k++) {
    const int i = t + k * 1024;
    const bool ok = i < n;
    ev[k] = ok ? deq_embed(type, row, i) * emb_scale : 0.0f;
    wv[k] = ok ? w[i] : 0.0f;
    if (ok) resid[i] = ev[k];
  }
  const float sc = rms_scale(sumsq_regs<EXACT>(ev, n, s_h, sh), n, eps);
  float xv[NORM_EPT];
#pragma unroll
  for (int k = 0; k < NORM_EPT; k++) xv[k] = (sc * ev[k]) * wv[k];
  norm_outputs(xv, n, out, s_h);
}

__device__ float deq_embed(uint32_t type, const uint8_t* row, int i) {
  switch (type) {
    case T_F16: return h2f(reinterpret_cast<const uint16_t*>(row)[i]);
    case T_F32: return reinterpret_cast<const float*>(row)[i];
    case T_Q8_0: {
      const uint8_t* b = row + (i / 32) * 34;
      return h2f((uint16_t)(b[0] | (b[1] << 8))) * (float)(int8_t)b[2 + (i & 31)];
    }
    default: return 0.0f;  // Q6_K/Q4_K/Q5_0 tables use launch_dequantize_rows + rms_norm
  }
}

// The decode loop's token feedback and the next step's embed_norm in one launch (the step graph then starts at
// layer 0): thread 0 runs finalize_token_kernel's selection and bookkeeping, the token reaches the work-group
// through LDS, and the embedding row + scale + first attn_norm follow as embed_norm_kernel computes them.
template <bool EXACT>
__global__ __launch_bounds__(1024) void finalize_embed_norm_kernel(
    unsigned long long* __restrict__ keys, int n_keys, int shard, int32_t* __restrict__ d_token,
    int32_t* __restrict__ d_pos, int32_t* __restrict__ ring, int32_t* __restrict__ ring_idx, int ring_cap,
    uint32_t type, const uint8_t* __restrict__ table, size_t row_bytes, float emb_scale, float* __restrict__ resid,
    const float* __restrict__ w, NormOut out, int n, double eps) {
  extern __shared__ float s_h[];
  __shared__ float sh[16];
  __shared__ int s_tok;
  const int t = threadIdx.x;
  float wv[NORM_EPT];
#pragma unroll
  for (int k = 0; k < NORM_EPT; k++) wv[k] = t + k * 1024 < n ? w[t + k * 1024] : 0.0f;
  if (t == 0) {
    unsigned long long best = keys[0];
    const int pos = *d_pos, i = *ring_idx;
    keys[0] = 0;
    for (int q = 1; q < n_keys; q++) {
      const unsigned long long k = keys[q];
      keys[q] = 0;
      if (k == 0) continue;
      const uint32_t gi = (uint32_t)q * (uint32_t)shard + argmax_key_index(k);
      const unsigned long long kg = (k & 0xFFFFFFFF00000000ull) | (0xFFFFFFFFu - gi);
      if (kg > best) best = kg;
    }
    const uint32_t tok = best ? argmax_key_index(best) : 0u;  // no key (NaN logits): a valid row, not 2^32 - 1
    *d_token = (int32_t)tok;
    *d_pos = pos + 1;
    if (i < ring_cap) ring[i] = (int32_t)tok;
    *ring_idx = i + 1;
    s_tok = (int)tok;
  }
  __syncthreads();
  const uint8_t* row = table + (size_t)s_tok * row_bytes;
  float ev[NORM_EPT];
#pragma unroll
  for (int k = 0; k < NORM_EPT; k++) {
    const int i = t + k * 1024;
    const bool ok = i < n;
    ev[k] = ok ? deq_embed(type, row, i) * emb_scale : 0.0f;
    if (ok) resid[i] = ev[k];
  }
  const float sc = rms_scale(sumsq_regs<EXACT>(ev, n, s_h, sh), n, eps);
  float xv[NORM_EPT];
#pragma unroll
  for (int k = 0; k < NORM_EPT; k++) xv[k] = (sc * ev[k]) * wv[k];
  norm_outputs(xv, n, out, s_h);
}

void launch_finalize_embed_norm(unsigned long long* keys, int n_keys, int shard, int32_t* d_token, int32_t* d_pos,
                                int32_t* ring, int32_t* ring_idx, int ring_cap, uint32_t type, const uint8_t* table,
                                size_t row_bytes, float emb_scale, float* resid, const float* w, const NormOut& out,
                                int n, double eps, bool exact, hipStream_t s) {
  if (n > 1024 * NORM_EPT) throw std::runtime_error("embed_norm: n_embd > 8192");
  if (type != T_F16 && type != T_F32 && type != T_Q8_0) throw std::runtime_error("finalize_embed_norm: table type");
  if (exact)
    hipLaunchKernelGGL(finalize_embed_norm_kernel<true>, dim3(1), dim3(1024), (size_t)n * 4, s, keys, n_keys, shard,
                       d_token, d_pos, ring, ring_idx, ring_cap, type, table, row_bytes, emb_scale, resid, w, out, n,
                       eps);
  else
    hipLaunchKernelGGL(finalize_embed_norm_kernel<false>, dim3(1), dim3(1024), (size_t)n * 4, s, keys, n_keys, shard,
                       d_token, d_pos, ring, ring_idx, ring_cap, type, table, row_bytes, emb_scale, resid, w, out, n,
                       eps);
  LLMI_HIP(hipGetLastError());
}

void launch_embed_norm(uint32_t type, const uint8_t* table, size_t row_bytes, const int32_t* d_token,
                       float emb_scale, float* resid, const float* w, const NormOut& out, int n, double eps,
                       bool exact, hipStream_t s) {
  if (n > 1024 * NORM_EPT) throw std::runtime_error("embed_norm: n_embd > 8192");
  if (exact)
    hipLaunchKernelGGL(embed_norm_kernel<true>, dim3(1), dim3(1024), (size_t)n * 4, s, type, table, row_bytes, d_token,
                       emb_scale, resid, w, out, n, eps);
  else
    hipLaunchKernelGGL(embed_norm_kernel<false>, dim3(1), dim3(1024), (size_t)n * 4, s, type, table, row_bytes, d_token,
                       emb_scale, resid, w, out, n, eps);
  LLMI_HIP(hipGetLastError());
}

}  // namespace llmi
