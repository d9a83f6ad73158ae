// ref_capi.cpp -- extern "C" binding over the REFERENCE implementation.
//
// TEST INFRASTRUCTURE ONLY.  This file is ours; it is compiled together with
// the reference's own sources (/root/reference/{ops,gguf,model}.cpp, never
// copied into this repo) by oracle/Makefile into oracle/_ref/libllmref.so.
// It lets tests/golden/gen_golden.py (and bench.py's cpu_baseline leg) call
// the reference's real ops.h / Model API through ctypes:
//   ref_mat_vec_mul     -> mat_vec_mul            ops.cpp:933-956
//   ref_mat_vec_mul_fp16-> mat_vec_mul_fp16       ops.cpp:455-612
//   ref_quantize_*      -> quantize_row_q8_0/_k   ops.cpp:116-178
//   ref_model_*         -> GGUFFile + Model::forward gguf.cpp:265, model.cpp:706
// Weight matrices are wrapped in a one-tensor in-memory GGUF exactly like the
// reference's own tests do (ops_test.cpp:96-136).
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include <iostream>

#include "gguf.h"
#include "model.h"
#include "ops.h"

bool verbose_g = false;  // defined by main.cpp in the reference binary

static std::string g_err;

static std::vector<uint8_t> one_tensor_gguf(uint32_t type, const void* data, size_t bytes,
                                            uint64_t n_cols, uint64_t n_rows) {
  std::vector<uint8_t> buf(256 + bytes);
  size_t off = 0;
  GGUFHeader h = {GGUF_MAGIC, GGUF_VERSION, 1, 0};
  memcpy(buf.data() + off, &h, sizeof h); off += sizeof h;
  const char* name = "w";
  uint64_t nl = 1; memcpy(buf.data() + off, &nl, 8); off += 8;
  memcpy(buf.data() + off, name, 1); off += 1;
  uint32_t dims = 2; memcpy(buf.data() + off, &dims, 4); off += 4;
  uint64_t shape[2] = {n_cols, n_rows}; memcpy(buf.data() + off, shape, 16); off += 16;
  memcpy(buf.data() + off, &type, 4); off += 4;
  uint64_t toff = 0; memcpy(buf.data() + off, &toff, 8); off += 8;
  const size_t ds = (off + 31) & ~size_t(31);
  memcpy(buf.data() + ds, data, bytes);
  buf.resize(ds + bytes);
  return buf;
}

extern "C" {

const char* ref_last_error() { return g_err.c_str(); }
// --verbose of main.cpp:39-51: the model's VERBOSE print_tensor dumps go to stdout
void ref_set_verbose(int on) {
  verbose_g = on != 0;
  std::cout.flush();
}
void ref_flush() { std::cout.flush(); }
void ref_init_ops(int n_threads) { init_ops(n_threads); }
float ref_f16_to_f32(uint16_t h) { return f16_to_f32(h); }
uint16_t ref_f32_to_f16(float f) { return f32_to_f16(f); }

void ref_quantize_row_q8_0(const float* x, size_t n, uint8_t* y) {
  std::vector<float> xv(x, x + n);
  std::vector<BlockQ8_0> out;
  quantize_row_q8_0(xv, out, n);
  memcpy(y, out.data(), out.size() * sizeof(BlockQ8_0));
}

void ref_quantize_row_q8_k(const float* x, size_t n, uint8_t* y) {
  std::vector<float> xv(x, x + n);
  std::vector<block_q8_K> out;
  quantize_row_q8_k(xv, out, n);
  memcpy(y, out.data(), out.size() * sizeof(block_q8_K));
}

// W in GGUF block layout, row-major, n_rows x n_cols; returns 0 or -1.
int ref_mat_vec_mul(uint32_t type, const void* w, size_t w_bytes, size_t n_rows, size_t n_cols,
                    const float* x, float* o) {
  try {
    std::vector<float> xv(x, x + n_cols), ov;
    if (type == (uint32_t)GGUFTensorType::F16) {
      std::vector<uint16_t> wv((const uint16_t*)w, (const uint16_t*)w + n_rows * n_cols);
      mat_vec_mul_fp16(ov, wv, xv, n_rows, n_cols);
    } else {
      auto buf = one_tensor_gguf(type, w, w_bytes, n_cols, n_rows);
      GGUFFile f(buf.data(), buf.size());
      mat_vec_mul(ov, f.get_tensor_infos()[0], f, xv);
    }
    memcpy(o, ov.data(), n_rows * sizeof(float));
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

// A prepared GEMV for timing the reference's kernels alone (the bench's
// GEMV-only CPU baseline): the one-tensor GGUF (or the F16 vector) is built
// once, then ref_gemv_run calls mat_vec_mul / mat_vec_mul_fp16 on it.
struct RefGemv {
  uint32_t type;
  size_t rows, cols;
  std::vector<uint8_t> buf;
  GGUFFile* f = nullptr;
  std::vector<uint16_t> w16;
  std::vector<float> x, o;
};

void* ref_gemv_prepare(uint32_t type, const void* w, size_t w_bytes, size_t n_rows, size_t n_cols) {
  try {
    auto* g = new RefGemv{type, n_rows, n_cols};
    if (type == (uint32_t)GGUFTensorType::F16) {
      g->w16.assign((const uint16_t*)w, (const uint16_t*)w + n_rows * n_cols);
    } else {
      g->buf = one_tensor_gguf(type, w, w_bytes, n_cols, n_rows);
      g->f = new GGUFFile(g->buf.data(), g->buf.size());
    }
    g->x.resize(n_cols);
    return g;
  } catch (const std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
}

int ref_gemv_run(void* h, const float* x, float* o) {
  auto* g = (RefGemv*)h;
  try {
    memcpy(g->x.data(), x, g->cols * sizeof(float));
    if (g->f) mat_vec_mul(g->o, g->f->get_tensor_infos()[0], *g->f, g->x);
    else mat_vec_mul_fp16(g->o, g->w16, g->x, g->rows, g->cols);
    if (o) memcpy(o, g->o.data(), g->rows * sizeof(float));
    return 0;
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

void ref_gemv_free(void* h) {
  auto* g = (RefGemv*)h;
  delete g->f;
  delete g;
}

int ref_dequantize_row(uint32_t type, const void* blocks, size_t n_cols, float* o) {
  std::vector<float> ov;
  const uint8_t* p = (const uint8_t*)blocks;
  switch ((GGUFTensorType)type) {
    case GGUFTensorType::Q4_K: dequantize_q4_k_row(ov, p, n_cols); break;
    case GGUFTensorType::Q6_K: dequantize_q6_k_row(ov, p, n_cols); break;
    case GGUFTensorType::Q8_0: dequantize_q8_0_row(ov, p, n_cols); break;
    case GGUFTensorType::Q5_0: dequantize_q5_0_row(ov, p, n_cols); break;
    default: g_err = "unsupported"; return -1;
  }
  memcpy(o, ov.data(), n_cols * sizeof(float));
  return 0;
}

void ref_rms_norm(float* o, const float* x, size_t n, double eps) {
  std::vector<float> xv(x, x + n), ov(n);
  rms_norm(ov, xv, eps);
  memcpy(o, ov.data(), n * sizeof(float));
}

void ref_softmax(float* x, size_t n) {
  std::vector<float> xv(x, x + n);
  softmax(xv);
  memcpy(x, xv.data(), n * sizeof(float));
}

// t: [n_tokens][n_heads][head_dim], in place
void ref_rope(float* t, size_t n_tokens, size_t n_heads, size_t head_dim, int n_rot, float base,
              float scale, int pos) {
  tensor_3 tt(n_tokens, tensor_2(n_heads, tensor_1(head_dim)));
  for (size_t a = 0; a < n_tokens; a++)
    for (size_t h = 0; h < n_heads; h++)
      memcpy(tt[a][h].data(), t + (a * n_heads + h) * head_dim, head_dim * 4);
  rope(tt, n_rot, base, scale, pos);
  for (size_t a = 0; a < n_tokens; a++)
    for (size_t h = 0; h < n_heads; h++)
      memcpy(t + (a * n_heads + h) * head_dim, tt[a][h].data(), head_dim * 4);
}

void ref_vec_scale_f16(uint16_t* y, size_t n, float v) {
  tensor_f16_1 yv(y, y + n);
  vec_scale_f16(yv, v);
  memcpy(y, yv.data(), n * 2);
}

void ref_vec_mad_f16(uint16_t* y, const uint16_t* x, size_t n, float v) {
  tensor_f16_1 yv(y, y + n), xv(x, x + n);
  vec_mad_f16(yv, xv, v);
  memcpy(y, yv.data(), n * 2);
}

struct RefModel {
  GGUFFile* f;
  Model* m;
};

// The gguf bytes must outlive the model (the reference borrows them).
void* ref_model_create(const uint8_t* gguf, size_t size) {
  try {
    RefModel* r = new RefModel;
    r->f = new GGUFFile(gguf, size);
    r->m = new Model(*r->f);
    return r;
  } catch (const std::exception& e) {
    g_err = e.what();
    return nullptr;
  }
}

int ref_model_forward(void* h, const int* tokens, int n_tokens, int pos, float* logits) {
  try {
    RefModel* r = (RefModel*)h;
    std::vector<int> tv(tokens, tokens + n_tokens);
    auto res = r->m->forward(tv, pos);
    memcpy(logits, res[0].data(), res[0].size() * sizeof(float));
    return (int)res[0].size();
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
}

int ref_model_tokenize(void* h, const char* prompt, int chat, int* out, int max_out) {
  RefModel* r = (RefModel*)h;
  auto t = r->m->tokenize(prompt, chat != 0);
  for (int i = 0; i < (int)t.size() && i < max_out; i++) out[i] = t[i];
  return (int)t.size();
}

void ref_model_destroy(void* h) {
  RefModel* r = (RefModel*)h;
  delete r->m;
  delete r->f;
  delete r;
}

}  // extern "C"
