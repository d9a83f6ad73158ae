// capi.cpp -- extern "C" entry points of include/llmi.h.
//
// Error contract: no C++ exception crosses the ABI; every call returns an
// llmi_status and stores the message (the reference's own wording where it
// has one) for llmi_last_error().
#include <cmath>
#include <mutex>
#include <vector>

#include "session.h"

using namespace llmi;

namespace {

thread_local std::string g_err;

struct Ctx {
  int device = -1;
  hipStream_t stream = nullptr;
  // orders a caller stream against this context's scratch (device-pointer GEMV)
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  // grow-only scratch for the host-pointer ops API
  std::vector<std::pair<void*, size_t>> bufs;
  void* get(int slot, size_t bytes) {
    if ((int)bufs.size() <= slot) bufs.resize(slot + 1, {nullptr, 0});
    auto& b = bufs[slot];
    if (b.second < bytes) {
      if (b.first) LLMI_HIP(hipFree(b.first));
      LLMI_HIP(hipMalloc(&b.first, bytes + 256));
      b.second = bytes;
    }
    return b.first;
  }
};

Ctx& ctx() {
  static thread_local Ctx c;
  if (c.device < 0) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) throw status_error(LLMI_E_NODEV, "no HIP device");
    c.device = 0;
    LLMI_HIP(hipSetDevice(0));
    LLMI_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
  }
  return c;
}

template <typename F>
int guard(F&& f) {
  try {
    f();
    return LLMI_OK;
  } catch (const status_error& e) {
    g_err = e.what();
    return e.code;
  } catch (const hip_error& e) {
    g_err = e.what();
    return LLMI_E_HIP;
  } catch (const gguf_error& e) {
    g_err = e.what();
    return LLMI_E_GGUF;
  } catch (const std::exception& e) {
    g_err = e.what();
    return std::string(e.what()).find("unsupported tensor type") != std::string::npos ? LLMI_E_TYPE : LLMI_E_ARG;
  }
}

const char* type_fn(uint32_t t) {
  switch (t) {
    case T_Q4_0: return "mat_vec_mul_q4_0";
    case T_Q4_K: return "mat_vec_mul_q4_k";
    case T_Q6_K: return "mat_vec_mul_q6_k";
    case T_Q8_0: return "mat_vec_mul_q8_0";
    case T_Q5_0: return "mat_vec_mul_q5_0";
    case T_BF16: return "mat_vec_mul_bf16";
    case T_F16: return "mat_vec_mul_fp16";
    default: return "mat_vec_mul";
  }
}

void check_shape(uint32_t type, size_t n_rows, size_t n_cols, size_t x_len) {
  if (!gemv_type_supported(type))
    throw status_error(LLMI_E_TYPE, "mat_vec_mul: unsupported tensor type " + std::to_string(type));
  if (x_len != n_cols) throw status_error(LLMI_E_SIZE, std::string(type_fn(type)) + ": input vector size mismatch");
  const size_t blk = (type == T_Q4_K || type == T_Q6_K) ? 256 : (type == T_F16 || type == T_BF16) ? 1 : 32;
  if (n_cols % blk) throw status_error(LLMI_E_SIZE, std::string(type_fn(type)) + ": n_cols not a block multiple");
  if (n_rows > (size_t)INT32_MAX || n_cols > (size_t)INT32_MAX)
    throw status_error(LLMI_E_SIZE, "matrix too large");
}

// activation for weight type `t` from device x (scratch slots 10..13)
ActBuf make_act(Ctx& c, uint32_t t, const float* x_dev, int n, hipStream_t s) {
  ActBuf a;
  a.xf = x_dev;
  if (t == T_Q4_0 || t == T_Q8_0) {
    a.q8.xb = (XBlock*)c.get(10, (size_t)(n / 32 + 1) * sizeof(XBlock));
    a.q8.nb = n / 32;
    launch_quantize_q8_0(x_dev, n, a.q8, s);
  } else if (t == T_Q4_K || t == T_Q6_K) {
    a.q8k = (uint8_t*)c.get(13, (size_t)(n / 256 + 1) * 292);
    launch_quantize_q8_k(x_dev, n, a.q8k, s);
  } else if (t == T_F16) {
    a.x16 = (uint16_t*)c.get(14, (size_t)n * 2);
    launch_round_f16(x_dev, n, a.x16, s);
  }
  return a;
}

}  // namespace

struct llmi_weight {
  DevWeight w;
};
struct llmi_session {
  Session* s;
};

extern "C" {

const char* llmi_last_error(void) { return g_err.c_str(); }
int llmi_version(void) { return 1; }

int llmi_init_ops(int device) {
  return guard([&] {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
      throw status_error(LLMI_E_NODEV, "no HIP device " + std::to_string(device));
    Ctx& c = ctx();
    if (c.device != device) {
      if (c.stream) LLMI_HIP(hipStreamDestroy(c.stream));
      for (auto& b : c.bufs)
        if (b.first) (void)hipFree(b.first);
      c.bufs.clear();
      c.device = device;
      LLMI_HIP(hipSetDevice(device));
      LLMI_HIP(hipStreamCreateWithFlags(&c.stream, hipStreamNonBlocking));
    }
  });
}

int llmi_weight_create(uint32_t type, const void* w, size_t n_rows, size_t n_cols, llmi_weight** out) {
  return guard([&] {
    if (!w || !out) throw status_error(LLMI_E_ARG, "null pointer");
    check_shape(type, n_rows, n_cols, n_cols);
    Ctx& c = ctx();
    auto* h = new llmi_weight;
    try {
      h->w = alloc_weight(type, (int)n_rows, (int)n_cols);
      upload_rows(h->w, 0, w, (int)n_rows, c.stream);
    } catch (...) {
      free_weight(h->w);
      delete h;
      throw;
    }
    *out = h;
  });
}

void llmi_weight_destroy(llmi_weight* w) {
  if (!w) return;
  free_weight(w->w);
  delete w;
}

int llmi_weight_mat_vec_mul_dev(const llmi_weight* w, const float* x_dev, float* o_dev, uint32_t flags,
                                void* stream) {
  return guard([&] {
    if (!w || !x_dev || !o_dev) throw status_error(LLMI_E_ARG, "null pointer");
    check_shape(w->w.type, w->w.rows, w->w.cols, w->w.cols);
    Ctx& c = ctx();
    hipStream_t s = stream ? (hipStream_t)stream : c.stream;
    // the activation goes through this thread's scratch slots, which the
    // host-pointer calls use on c.stream: a caller stream first waits for
    // c.stream's earlier work, and c.stream then waits for this call, so calls
    // on any mix of streams touch the scratch one at a time
    if (s != c.stream) {
      if (!c.ev_in) {
        LLMI_HIP(hipEventCreateWithFlags(&c.ev_in, hipEventDisableTiming));
        LLMI_HIP(hipEventCreateWithFlags(&c.ev_out, hipEventDisableTiming));
      }
      LLMI_HIP(hipEventRecord(c.ev_in, c.stream));
      LLMI_HIP(hipStreamWaitEvent(s, c.ev_in, 0));
    }
    ActBuf a = make_act(c, w->w.type, x_dev, w->w.cols, s);
    launch_gemv(w->w, a, o_dev, (flags & LLMI_EXACT) ? GEMV_EXACT : GEMV_FAST, s);
    if (s != c.stream) {
      LLMI_HIP(hipEventRecord(c.ev_out, s));
      LLMI_HIP(hipStreamWaitEvent(c.stream, c.ev_out, 0));
    }
  });
}

int llmi_weight_mat_vec_mul(const llmi_weight* w, const float* x, size_t x_len, float* o, uint32_t flags) {
  return guard([&] {
    if (!w || !x || !o) throw status_error(LLMI_E_ARG, "null pointer");
    check_shape(w->w.type, w->w.rows, w->w.cols, x_len);
    Ctx& c = ctx();
    float* xd = (float*)c.get(0, x_len * 4);
    float* od = (float*)c.get(1, (size_t)w->w.rows * 4);
    LLMI_HIP(hipMemcpyAsync(xd, x, x_len * 4, hipMemcpyHostToDevice, c.stream));
    ActBuf a = make_act(c, w->w.type, xd, (int)x_len, c.stream);
    launch_gemv(w->w, a, od, (flags & LLMI_EXACT) ? GEMV_EXACT : GEMV_FAST, c.stream);
    LLMI_HIP(hipMemcpyAsync(o, od, (size_t)w->w.rows * 4, hipMemcpyDeviceToHost, c.stream));
    LLMI_HIP(hipStreamSynchronize(c.stream));
  });
}

int llmi_mat_vec_mul(uint32_t type, const void* w, size_t n_rows, size_t n_cols, const float* x, size_t x_len,
                     float* o, uint32_t flags) {
  return guard([&] {
    if (!w || !x || !o) throw status_error(LLMI_E_ARG, "null pointer");
    check_shape(type, n_rows, n_cols, x_len);
    if (n_rows == 0) return;
    llmi_weight* h = nullptr;
    int rc = llmi_weight_create(type, w, n_rows, n_cols, &h);
    if (rc) throw status_error(rc, g_err);
    rc = llmi_weight_mat_vec_mul(h, x, x_len, o, flags);
    llmi_weight_destroy(h);
    if (rc) throw status_error(rc, g_err);
  });
}

int llmi_quantize_row_q8_0(const float* x, size_t n, void* y) {
  return guard([&] {
    if (n % 32) throw status_error(LLMI_E_SIZE, "quantize_row_q8_0: size % 32 != 0");
    Ctx& c = ctx();
    float* xd = (float*)c.get(0, n * 4);
    Q8Act q;
    q.xb = (XBlock*)c.get(10, (n / 32 + 1) * sizeof(XBlock));
    q.nb = (int)(n / 32);
    LLMI_HIP(hipMemcpyAsync(xd, x, n * 4, hipMemcpyHostToDevice, c.stream));
    launch_quantize_q8_0(xd, (int)n, q, c.stream);
    std::vector<XBlock> xb(n / 32);
    LLMI_HIP(hipMemcpyAsync(xb.data(), q.xb, n / 32 * sizeof(XBlock), hipMemcpyDeviceToHost, c.stream));
    LLMI_HIP(hipStreamSynchronize(c.stream));
    uint8_t* out = (uint8_t*)y;  // BlockQ8_0 {f16 d; i8 qs[32]} (ops.h:89-92)
    for (size_t b = 0; b < n / 32; b++) {
      const _Float16 dh = (_Float16)xb[b].d;  // exact: d holds an f16 value
      std::memcpy(out + b * 34, &dh, 2);
      std::memcpy(out + b * 34 + 2, &xb[b].lo, 32);
    }
  });
}

int llmi_quantize_row_q8_k(const float* x, size_t n, void* y) {
  return guard([&] {
    if (n % 256) throw status_error(LLMI_E_SIZE, "quantize_row_q8_k: size % 256 != 0");
    Ctx& c = ctx();
    float* xd = (float*)c.get(0, n * 4);
    uint8_t* yd = (uint8_t*)c.get(13, n / 256 * 292);
    LLMI_HIP(hipMemcpyAsync(xd, x, n * 4, hipMemcpyHostToDevice, c.stream));
    launch_quantize_q8_k(xd, (int)n, yd, c.stream);
    LLMI_HIP(hipMemcpyAsync(y, yd, n / 256 * 292, hipMemcpyDeviceToHost, c.stream));
    LLMI_HIP(hipStreamSynchronize(c.stream));
  });
}

int llmi_dequantize_row(uint32_t type, const void* blocks, size_t n_cols, float* o) {
  return guard([&] {
    if (type != T_Q4_K && type != T_Q6_K && type != T_Q8_0 && type != T_Q5_0 && type != T_F16 && type != T_F32)
      throw status_error(LLMI_E_TYPE, "dequantize: unsupported tensor type " + std::to_string(type));
    Ctx& c = ctx();
    const size_t rb = gguf_bytes(type, 1, n_cols);
    uint8_t* bd = (uint8_t*)c.get(2, rb);
    float* od = (float*)c.get(1, n_cols * 4);
    int32_t* idd = (int32_t*)c.get(3, 4);
    LLMI_HIP(hipMemcpyAsync(bd, blocks, rb, hipMemcpyHostToDevice, c.stream));
    LLMI_HIP(hipMemsetAsync(idd, 0, 4, c.stream));
    launch_dequantize_rows(type, bd, rb, idd, 1, (int)n_cols, 1.0f, od, c.stream);
    LLMI_HIP(hipMemcpyAsync(o, od, n_cols * 4, hipMemcpyDeviceToHost, c.stream));
    LLMI_HIP(hipStreamSynchronize(c.stream));
  });
}

int llmi_rms_norm(float* o, const float* x, size_t n, double eps, uint32_t flags) {
  return guard([&] {
    if (eps <= 0) throw status_error(LLMI_E_ARG, "Error: eps must be > 0 in rms_norm.");  // ops.cpp:29-32
    Ctx& c = ctx();
    float* xd = (float*)c.get(0, n * 4);
    float* od = (float*)c.get(1, n * 4);
    LLMI_HIP(hipMemcpyAsync(xd, x, n * 4, hipMemcpyHostToDevice, c.stream));
    launch_rms_norm(xd, nullptr, od, (int)n, 1, eps, (flags & LLMI_EXACT) != 0, c.stream);
    LLMI_HIP(hipMemcpyAsync(o, od, n * 4, hipMemcpyDeviceToHost, c.stream));
    LLMI_HIP(hipStreamSynchronize(c.stream));
  });
}

int llmi_softmax(float* x, size_t n) {
  return guard([&] {
    Ctx& c = ctx();
    float* xd = (float*)c.get(0, n * 4);
    LLMI_HIP(hipMemcpyAsync(xd, x, n * 4, hipMemcpyHostToDevice, c.stream));
    launch_softmax(xd, (int)n, c.stream);
    LLMI_HIP(hipMemcpyAsync(x, xd, n * 4, hipMemcpyDeviceToHost, c.stream));
    LLMI_HIP(hipStreamSynchronize(c.stream));
  });
}

int llmi_rope(float* t, size_t n_tokens, size_t n_heads, size_t head_dim, int n_rot, float freq_base,
              float freq_scale, int pos) {
  return guard([&] {
    if (n_rot <= 0 || (size_t)n_rot > head_dim || n_rot % 2)
      throw status_error(LLMI_E_ARG, "rope: invalid n_rot");
    if (n_tokens == 0 || n_heads == 0) return;
    Ctx& c = ctx();
    const int half = n_rot / 2;
    std::vector<float> cs(n_tokens * half * 2);  // ops.cpp:79-83, host glibc
    for (size_t tk = 0; tk < n_tokens; tk++)
      for (int i = 0; i < half; i++) {
        const float freq = 1.0f / powf(freq_base, (float)(2 * i) / (float)n_rot);
        const float val = ((float)(uint32_t)(pos + (uint32_t)tk) * freq) / freq_scale;
        cs[(tk * half + i) * 2] = cosf(val);
        cs[(tk * half + i) * 2 + 1] = sinf(val);
      }
    const size_t n = n_tokens * n_heads * head_dim;
    float* td = (float*)c.get(0, n * 4);
    float* csd = (float*)c.get(4, cs.size() * 4);
    LLMI_HIP(hipMemcpyAsync(td, t, n * 4, hipMemcpyHostToDevice, c.stream));
    LLMI_HIP(hipMemcpyAsync(csd, cs.data(), cs.size() * 4, hipMemcpyHostToDevice, c.stream));
    launch_rope(td, (int)(n_tokens * n_heads), (int)head_dim, n_rot, csd, (int)n_heads, c.stream);
    LLMI_HIP(hipMemcpyAsync(t, td, n * 4, hipMemcpyDeviceToHost, c.stream));
    LLMI_HIP(hipStreamSynchronize(c.stream));
  });
}

int llmi_scale(float* t, size_t n, float sc) {
  return guard([&] {
    Ctx& c = ctx();
    float* td = (float*)c.get(0, n * 4);
    LLMI_HIP(hipMemcpyAsync(td, t, n * 4, hipMemcpyHostToDevice, c.stream));
    launch_scale(td, (int)n, sc, c.stream);
    LLMI_HIP(hipMemcpyAsync(t, td, n * 4, hipMemcpyDeviceToHost, c.stream));
    LLMI_HIP(hipStreamSynchronize(c.stream));
  });
}

int llmi_vec_scale_f16(uint16_t* y, size_t n, float v) {
  return guard([&] {
    Ctx& c = ctx();
    uint16_t* yd = (uint16_t*)c.get(0, n * 2);
    LLMI_HIP(hipMemcpyAsync(yd, y, n * 2, hipMemcpyHostToDevice, c.stream));
    launch_vec_scale_f16(yd, (int)n, v, c.stream);
    LLMI_HIP(hipMemcpyAsync(y, yd, n * 2, hipMemcpyDeviceToHost, c.stream));
    LLMI_HIP(hipStreamSynchronize(c.stream));
  });
}

int llmi_vec_mad_f16(uint16_t* y, const uint16_t* x, size_t n, float v) {
  return guard([&] {
    Ctx& c = ctx();
    uint16_t* yd = (uint16_t*)c.get(0, n * 2);
    uint16_t* xd = (uint16_t*)c.get(1, n * 2);
    LLMI_HIP(hipMemcpyAsync(yd, y, n * 2, hipMemcpyHostToDevice, c.stream));
    LLMI_HIP(hipMemcpyAsync(xd, x, n * 2, hipMemcpyHostToDevice, c.stream));
    launch_vec_mad_f16(yd, xd, (int)n, v, c.stream);
    LLMI_HIP(hipMemcpyAsync(y, yd, n * 2, hipMemcpyDeviceToHost, c.stream));
    LLMI_HIP(hipStreamSynchronize(c.stream));
  });
}

int llmi_attention(const float* q, const uint16_t* k, const uint16_t* v, int n_head, int n_head_kv, int n_keys,
                   int head_dim, float* out, uint32_t flags) {
  return guard([&] {
    if (n_head <= 0 || n_head_kv <= 0 || n_head % n_head_kv || n_keys <= 0 || head_dim <= 0 || head_dim > 256 ||
        head_dim % 8)
      throw status_error(LLMI_E_ARG, "attention: invalid shape");
    Ctx& c = ctx();
    const size_t nq = (size_t)n_head * head_dim, nkv = (size_t)n_head_kv * n_keys * head_dim;
    const int nsplit = ATTN_NSPLIT;
    float* qd = (float*)c.get(0, nq * 4);
    float* od = (float*)c.get(1, nq * 4);
    uint16_t* kd = (uint16_t*)c.get(2, nkv * 2);
    uint16_t* vd = (uint16_t*)c.get(3, nkv * 2);
    float* pd = (float*)c.get(4, (size_t)n_head * nsplit * (head_dim + 2) * 4);
    int32_t* posd = (int32_t*)c.get(5, 4);
    const int32_t pos = n_keys - 1;
    LLMI_HIP(hipMemcpyAsync(qd, q, nq * 4, hipMemcpyHostToDevice, c.stream));
    LLMI_HIP(hipMemcpyAsync(kd, k, nkv * 2, hipMemcpyHostToDevice, c.stream));
    LLMI_HIP(hipMemcpyAsync(vd, v, nkv * 2, hipMemcpyHostToDevice, c.stream));
    LLMI_HIP(hipMemcpyAsync(posd, &pos, 4, hipMemcpyHostToDevice, c.stream));
    unsigned* td = (unsigned*)c.get(6, (size_t)n_head_kv * 4);
    LLMI_HIP(hipMemsetAsync(td, 0, (size_t)n_head_kv * 4, c.stream));
    AttnArgs a{qd, kd, vd, n_head, n_head_kv, head_dim, n_keys, posd, pd, od, td, nullptr};
    launch_attention(a, (flags & LLMI_EXACT) != 0, c.stream);
    LLMI_HIP(hipMemcpyAsync(out, od, nq * 4, hipMemcpyDeviceToHost, c.stream));
    LLMI_HIP(hipStreamSynchronize(c.stream));
  });
}

int llmi_gelu_mul(const float* gate, const float* up, size_t n, float* out) {
  return guard([&] {
    Ctx& c = ctx();
    float* gd = (float*)c.get(0, n * 8);
    float* od = (float*)c.get(1, n * 4);
    LLMI_HIP(hipMemcpyAsync(gd, gate, n * 4, hipMemcpyHostToDevice, c.stream));
    LLMI_HIP(hipMemcpyAsync(gd + n, up, n * 4, hipMemcpyHostToDevice, c.stream));
    launch_gelu_quant(gd, (int)n, od, nullptr, c.stream);
    LLMI_HIP(hipMemcpyAsync(out, od, n * 4, hipMemcpyDeviceToHost, c.stream));
    LLMI_HIP(hipStreamSynchronize(c.stream));
  });
}

// ---- session ----
int llmi_session_create(const void* gguf, size_t size, const llmi_session_opts* opts, llmi_session** out) {
  return guard([&] {
    if (!gguf || !out) throw status_error(LLMI_E_ARG, "null pointer");
    llmi_session_opts o{0, 0, 4096, 0, 0, 1, nullptr, nullptr};
    if (opts) o = *opts;
    auto* h = new llmi_session{nullptr};
    try {
      h->s = new Session((const uint8_t*)gguf, size, o);
    } catch (...) {
      delete h;
      throw;
    }
    *out = h;
  });
}

void llmi_session_destroy(llmi_session* s) {
  if (!s) return;
  delete s->s;
  delete s;
}

int llmi_session_forward(llmi_session* s, const int32_t* tokens, int n_tokens, int pos, float* logits,
                         int32_t* argmax) {
  return guard([&] { s->s->forward(tokens, n_tokens, pos, logits, argmax); });
}

int llmi_session_dump(llmi_session* s, const int32_t* tokens, int n_tokens, int pos, const char* path) {
  return guard([&] { s->s->forward_dump(tokens, n_tokens, pos, path); });
}

int llmi_session_trace(llmi_session* s, const int32_t* tokens, int n_tokens, int pos, uint32_t flags,
                       llmi_trace_fn fn, void* user) {
  return guard([&] {
    if (!s || !tokens || !fn) throw status_error(LLMI_E_ARG, "null pointer");
    s->s->forward_trace(tokens, n_tokens, pos, (flags & 1u) != 0, fn, user);
  });
}

int llmi_session_generate(llmi_session* s, int32_t first, int pos, int n_steps, int32_t* out_tokens) {
  return guard([&] {
    s->s->enqueue(first, pos, n_steps);
    s->s->sync(out_tokens, n_steps);
  });
}

int llmi_session_enqueue(llmi_session* s, int32_t first, int pos, int n_steps) {
  return guard([&] { s->s->enqueue(first, pos, n_steps); });
}

int llmi_session_sync(llmi_session* s, int32_t* out_tokens, int n) {
  return guard([&] { s->s->sync(out_tokens, n); });
}

int llmi_tp_unique_id(void* out) {
  return guard([&] {
    if (!out) throw status_error(LLMI_E_ARG, "null pointer");
    rccl_unique_id(out);
  });
}

int llmi_tp_group_create(int size, llmi_tp_group** out) {
  return guard([&] {
    if (!out || size < 1) throw status_error(LLMI_E_ARG, "tp group: size < 1");
    *out = reinterpret_cast<llmi_tp_group*>(new LocalGroup(size));
  });
}

void llmi_tp_group_destroy(llmi_tp_group* g) { delete reinterpret_cast<LocalGroup*>(g); }

static_assert(LLMI_PEER_HANDLE_BYTES == PEER_HANDLE_BYTES, "peer handle size");

int llmi_session_peer_handle(const llmi_session* s, void* out) {
  return guard([&] {
    if (!s || !out) throw status_error(LLMI_E_ARG, "peer handle: null argument");
    s->s->peer_handle(out);
  });
}

int llmi_session_peer_connect(llmi_session* s, const void* handles) {
  return guard([&] {
    if (!s) throw status_error(LLMI_E_ARG, "peer connect: null session");
    s->s->peer_connect(handles);
  });
}

int llmi_selftest(int which, unsigned long long* out) {
  return guard([&] {
    if (!out) throw status_error(LLMI_E_ARG, "null pointer");
    if (which == 0) {
      exact_selftest_f16(out);
    } else if (which == 1) {
      unsigned r[2];
      exact_selftest_chain(r);
      out[0] = r[0];
      out[1] = r[1];
    } else if (which == 2) {
      size_t live = 0, cached = 0, grave = 0;
      dev_mem_stats(&live, &cached, &grave);
      out[0] = live;
      out[1] = cached;
      out[2] = grave;
    } else {
      throw status_error(LLMI_E_ARG, "selftest: unknown test");
    }
  });
}

int llmi_session_get_info(const llmi_session* s, llmi_session_info* info) {
  return guard([&] { s->s->info(info); });
}

int llmi_session_time_kernel(llmi_session* s, int which, int reps, double* us, double* bytes) {
  return guard([&] { s->s->time_kernel(which, reps, us, bytes); });
}

}  // extern "C"
