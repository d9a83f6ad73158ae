// ops_mi355x.cpp -- drop-in replacement for the reference's ops.cpp.
//
// Implements every function declared in the reference's ops.h (ops.h:38-107)
// with the SAME signatures on top of the C ABI of libllmi.so
// (include/llmi.h), so model.cpp, gguf.cpp and their callers compile
// unchanged.  Build it in place of ops.cpp in the `:ops` cc_library
// (INTEGRATION.md); it needs the reference's own ops.h / gguf.h / tensor.h on
// the include path and links libllmi.so.
//
// Semantics kept from the reference:
//  * results are complete on return (the reference's fork/join, ops.cpp:450);
//  * `o` is resized by the callee (ops.cpp:200, 464, ...);
//  * size mismatches and unsupported types throw std::runtime_error with the
//    reference's messages (ops.cpp:196-198, 953-954); rms_norm with eps <= 0
//    throws instead of exit(1) (ops.cpp:29-32);
//  * numerics: LLMI_EXACT (bit-identical to the AVX2 kernels) unless
//    LLMI_OPS_FAST=1 is set in the environment.
// Weights are uploaded to the GPU once per tensor, keyed by their mmap pointer
// (GGUFFile::get_tensor_data, gguf.cpp:354-356) or, for the F16 logits copy,
// by the Model-owned vector's data pointer; later calls move only x and o.
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "gguf.h"
#include "llmi.h"
#include "ops.h"

namespace {

uint32_t flags() {
  static const uint32_t f = getenv("LLMI_OPS_FAST") ? 0u : LLMI_EXACT;
  return f;
}

void check(int rc) {
  if (rc != LLMI_OK) throw std::runtime_error(llmi_last_error());
}

struct WeightKey {
  const void* p;
  uint32_t type;
  size_t rows, cols;
  bool operator==(const WeightKey& o) const { return p == o.p && type == o.type && rows == o.rows && cols == o.cols; }
};
struct WeightKeyHash {
  size_t operator()(const WeightKey& k) const {
    return std::hash<const void*>()(k.p) ^ (k.rows * 1315423911u) ^ (k.cols << 7) ^ k.type;
  }
};

// Content fingerprint of a weight's bytes: a buffer freed and reallocated at
// the same address with other contents (model_test.cpp:394/410/463 builds
// several Models from heap vectors in one process) gets a new upload instead
// of the previous tensor's device copy.  Buffers up to FULL_HASH_BYTES are
// hashed WHOLE (every byte: an edit anywhere is seen); larger ones (the
// reference mmaps them read-only, gguf.cpp:130-149, so they cannot change in
// place) are hashed over 4096 evenly spaced 64-byte windows plus the length --
// callers that rewrite a large weight in place must call
// llmi_ops_flush_weights().
constexpr size_t FULL_HASH_BYTES = (size_t)64 << 20;

uint64_t hash_words(const uint8_t* p, size_t n, uint64_t h) {  // 4 independent lanes, 8-byte words
  uint64_t a = h, b = h ^ 0x9E3779B97F4A7C15ull, c = h ^ 0xC2B2AE3D27D4EB4Full, d = h ^ 0x165667B19E3779F9ull;
  size_t i = 0;
  auto mix = [](uint64_t x, uint64_t w) {
    x ^= w * 0x87C37B91114253D5ull;
    x = (x << 31) | (x >> 33);
    return x * 0x4CF5AD432745937Full;
  };
  for (; i + 32 <= n; i += 32) {
    uint64_t w[4];
    std::memcpy(w, p + i, 32);
    a = mix(a, w[0]);
    b = mix(b, w[1]);
    c = mix(c, w[2]);
    d = mix(d, w[3]);
  }
  for (; i < n; i++) a = mix(a, p[i]);
  return mix(mix(mix(a, b), c), d);
}

uint64_t fingerprint(const void* data, size_t bytes) {
  const uint8_t* p = static_cast<const uint8_t*>(data);
  const uint64_t h0 = 1469598103934665603ull ^ bytes;
  if (bytes <= FULL_HASH_BYTES) return hash_words(p, bytes, h0);
  constexpr size_t win = 64, n = 4096;
  uint64_t h = h0;
  for (size_t i = 0; i < n; i++) h = hash_words(p + (bytes - win) * i / (n - 1), win, h);
  return h;
}

size_t weight_bytes(uint32_t type, size_t rows, size_t cols) {
  switch (type) {
    case 2: return rows * cols / 32 * 18;    // Q4_0
    case 6: return rows * cols / 32 * 22;    // Q5_0
    case 8: return rows * cols / 32 * 34;    // Q8_0
    case 12: return rows * cols / 256 * 144; // Q4_K
    case 14: return rows * cols / 256 * 210; // Q6_K
    default: return rows * cols * 2;         // F16 / BF16
  }
}

struct Cached {
  llmi_weight* w;
  uint64_t fp;
};

std::mutex g_cache_mu;
std::unordered_map<WeightKey, Cached, WeightKeyHash> g_cache;

llmi_weight* cached_weight(uint32_t type, const void* data, size_t rows, size_t cols) {
  std::lock_guard<std::mutex> lock(g_cache_mu);
  const WeightKey key{data, type, rows, cols};
  const uint64_t fp = fingerprint(data, weight_bytes(type, rows, cols));
  auto it = g_cache.find(key);
  if (it != g_cache.end()) {
    if (it->second.fp == fp) return it->second.w;
    llmi_weight_destroy(it->second.w);  // same address, other contents: stale
    g_cache.erase(it);
  }
  llmi_weight* w = nullptr;
  check(llmi_weight_create(type, data, rows, cols, &w));
  g_cache.emplace(key, Cached{w, fp});
  return w;
}

void gemv(std::vector<float>& o, uint32_t type, const void* data, size_t rows, size_t cols,
          const std::vector<float>& x) {
  if (x.size() != cols) throw std::runtime_error("mat_vec_mul: input vector size mismatch");
  llmi_weight* w = cached_weight(type, data, rows, cols);
  o.resize(rows);
  check(llmi_weight_mat_vec_mul(w, x.data(), x.size(), o.data(), flags()));
}

void gemv_tensor(std::vector<float>& o, const TensorInfo& t, const GGUFFile& f, const std::vector<float>& x,
                 uint32_t expect_type) {
  if (expect_type != 0xFFFFFFFFu && t.tensor_type != expect_type)
    throw std::runtime_error("mat_vec_mul: unexpected tensor type " + std::to_string(t.tensor_type));
  gemv(o, t.tensor_type, f.get_tensor_data(t), (size_t)t.shape[1], (size_t)t.shape[0], x);
}

// tensor_3 [tokens][heads][dim] <-> one contiguous buffer
std::vector<float> flatten(const tensor_3& t, size_t& n0, size_t& n1, size_t& n2) {
  n0 = t.size();
  n1 = n0 ? t[0].size() : 0;
  n2 = n1 ? t[0][0].size() : 0;
  std::vector<float> f(n0 * n1 * n2);
  for (size_t a = 0; a < n0; a++)
    for (size_t b = 0; b < n1; b++) std::memcpy(&f[(a * n1 + b) * n2], t[a][b].data(), n2 * sizeof(float));
  return f;
}
void unflatten(const std::vector<float>& f, tensor_3& t, size_t n0, size_t n1, size_t n2) {
  for (size_t a = 0; a < n0; a++)
    for (size_t b = 0; b < n1; b++) std::memcpy(t[a][b].data(), &f[(a * n1 + b) * n2], n2 * sizeof(float));
}

}  // namespace

// Drops every cached device weight (e.g. after a GGUFFile is unmapped);
// extern "C" so a host that owns the model lifetime can call it.
extern "C" void llmi_ops_flush_weights(void) {
  std::lock_guard<std::mutex> lock(g_cache_mu);
  for (auto& kv : g_cache) llmi_weight_destroy(kv.second.w);
  g_cache.clear();
}

void init_ops(int /*n_threads*/) { check(llmi_init_ops(0)); }  // ops.cpp:21-24: device 0 instead of a pool

void mat_vec_mul_fp16(std::vector<float>& o, const std::vector<uint16_t>& w, const std::vector<float>& x,
                      size_t n_rows, size_t n_cols) {
  gemv(o, 1 /* F16 */, w.data(), n_rows, n_cols, x);
}

void vec_scale_f16(tensor_f16_1& y, float v) { check(llmi_vec_scale_f16(y.data(), y.size(), v)); }

void vec_mad_f16(tensor_f16_1& y, const tensor_f16_1& x, float v) {
  if (x.size() != y.size()) throw std::runtime_error("vec_mad_f16: size mismatch");
  check(llmi_vec_mad_f16(y.data(), x.data(), y.size(), v));
}

void mat_vec_mul(std::vector<float>& o, const TensorInfo& w, const GGUFFile& f, const std::vector<float>& x) {
  gemv_tensor(o, w, f, x, 0xFFFFFFFFu);  // type dispatch happens in llmi_weight_create (ops.cpp:940-954)
}
void mat_vec_mul_q4_0(std::vector<float>& o, const TensorInfo& w, const GGUFFile& f, const std::vector<float>& x) {
  gemv_tensor(o, w, f, x, 2);
}
void mat_vec_mul_q4_k(std::vector<float>& o, const TensorInfo& w, const GGUFFile& f, const std::vector<float>& x) {
  gemv_tensor(o, w, f, x, 12);
}
void mat_vec_mul_q6_k(std::vector<float>& o, const TensorInfo& w, const GGUFFile& f, const std::vector<float>& x) {
  gemv_tensor(o, w, f, x, 14);
}
void mat_vec_mul_q8_0(std::vector<float>& o, const TensorInfo& w, const GGUFFile& f, const std::vector<float>& x) {
  gemv_tensor(o, w, f, x, 8);
}
void mat_vec_mul_q5_0(std::vector<float>& o, const TensorInfo& w, const GGUFFile& f, const std::vector<float>& x) {
  gemv_tensor(o, w, f, x, 6);
}
void mat_vec_mul_bf16(std::vector<float>& o, const TensorInfo& w, const GGUFFile& f, const std::vector<float>& x) {
  gemv_tensor(o, w, f, x, 30);
}

static void deq(uint32_t type, std::vector<float>& o, const uint8_t* blocks, size_t n_cols) {
  o.resize(n_cols);
  check(llmi_dequantize_row(type, blocks, n_cols, o.data()));
}
void dequantize_q4_k_row(std::vector<float>& o, const uint8_t* b, size_t n) { deq(12, o, b, n); }
void dequantize_q6_k_row(std::vector<float>& o, const uint8_t* b, size_t n) { deq(14, o, b, n); }
void dequantize_q8_0_row(std::vector<float>& o, const uint8_t* b, size_t n) { deq(8, o, b, n); }
void dequantize_q5_0_row(std::vector<float>& o, const uint8_t* b, size_t n) { deq(6, o, b, n); }

void rms_norm(std::vector<float>& o, const std::vector<float>& x, double eps) {
  o.resize(x.size());
  check(llmi_rms_norm(o.data(), x.data(), x.size(), eps, flags()));
}

void softmax(std::vector<float>& x) { check(llmi_softmax(x.data(), x.size())); }

void rope(tensor_3& t, int n_rot, float base, float freq_scale, int pos) {
  size_t n0, n1, n2;
  std::vector<float> f = flatten(t, n0, n1, n2);
  if (f.empty()) return;
  check(llmi_rope(f.data(), n0, n1, n2, n_rot, base, freq_scale, pos));
  unflatten(f, t, n0, n1, n2);
}

void scale(tensor_3& t, float s) {
  size_t n0, n1, n2;
  std::vector<float> f = flatten(t, n0, n1, n2);
  if (f.empty()) return;
  check(llmi_scale(f.data(), f.size(), s));
  unflatten(f, t, n0, n1, n2);
}

void quantize_row_q8_0(const std::vector<float>& x, std::vector<BlockQ8_0>& y, size_t size) {
  static_assert(sizeof(BlockQ8_0) == 34, "BlockQ8_0 layout (ops.h:89-92)");
  y.resize(size / 32);
  check(llmi_quantize_row_q8_0(x.data(), size, y.data()));
}

void quantize_row_q8_k(const std::vector<float>& x, std::vector<block_q8_K>& y, size_t size) {
  static_assert(sizeof(block_q8_K) == 292, "block_q8_K layout (ops.h:98-102)");
  y.resize(size / 256);
  check(llmi_quantize_row_q8_k(x.data(), size, y.data()));
}
