/*
 * llmi_oracle.c -- CPU restatement of the reference decode path.
 *
 * TEST INFRASTRUCTURE ONLY (see llmi_oracle.h).  Parity status: PINNED --
 * tests/test_oracle_golden.py checks every function below bit-for-bit against
 * fixtures produced by the reference itself (oracle/_ref/libllmref.so, built
 * from /root/reference/{ops,gguf,model}.cpp with the reference's own flags by
 * oracle/Makefile; generator tests/golden/gen_golden.py), and the model
 * forward additionally against the reference's own ModelTest golden logits
 * (model_test.cpp:426-459).
 *
 * Compiled with -ffp-contract=off: every fused multiply-add that the
 * reference's compiler emits (verified in its disassembly) is an explicit
 * fmaf() here; every other operation is a separately rounded IEEE op.
 */
#define _GNU_SOURCE
#include "llmi_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static __thread char g_err[256];
const char* orc_last_error(void) { return g_err; }
#define ORC_FAIL(...) (snprintf(g_err, sizeof g_err, __VA_ARGS__), -1)

/* ------------------------------------------------------------------ */
/* fp16 <-> fp32, ggml bit-exact (gguf.cpp:22-113)                     */
/* ------------------------------------------------------------------ */
static inline float f_from_bits(uint32_t w) { float f; memcpy(&f, &w, 4); return f; }
static inline uint32_t f_to_bits(float f) { uint32_t w; memcpy(&w, &f, 4); return w; }

float orc_f16_to_f32(uint16_t h) {  /* gguf.cpp:40-66 */
  const uint32_t w = (uint32_t)h << 16;
  const uint32_t sign = w & 0x80000000u;
  const uint32_t two_w = w + w;
  const float normalized = f_from_bits((two_w >> 4) + (0xE0u << 23)) * 0x1.0p-112f;
  const float denormalized = f_from_bits((two_w >> 17) | (126u << 23)) - 0.5f;
  const uint32_t r = sign | (two_w < (1u << 27) ? f_to_bits(denormalized) : f_to_bits(normalized));
  return f_from_bits(r);
}

uint16_t orc_f32_to_f16(float f) {  /* gguf.cpp:68-95 */
  float base = (fabsf(f) * 0x1.0p+112f) * 0x1.0p-110f;
  const uint32_t w = f_to_bits(f);
  const uint32_t shl1_w = w + w;
  const uint32_t sign = w & 0x80000000u;
  uint32_t bias = shl1_w & 0xFF000000u;
  if (bias < 0x71000000u) bias = 0x71000000u;
  base = f_from_bits((bias >> 1) + 0x07800000u) + base;
  const uint32_t bits = f_to_bits(base);
  const uint32_t exp_bits = (bits >> 13) & 0x00007C00u;
  const uint32_t mant_bits = bits & 0x00000FFFu;
  const uint32_t nonsign = exp_bits + mant_bits;
  return (uint16_t)((sign >> 16) | (shl1_w > 0xFF000000u ? 0x7E00u : nonsign));
}

float orc_bf16_to_f32(uint16_t h) { return f_from_bits((uint32_t)h << 16); } /* gguf.cpp:395-402 */

static float g_f16_table[65536];
static pthread_once_t g_table_once = PTHREAD_ONCE_INIT;
static void table_init(void) {  /* gguf.cpp:104-113 */
  for (int i = 0; i < 65536; i++) g_f16_table[i] = orc_f16_to_f32((uint16_t)i);
}
static inline float F16(uint16_t h) { return g_f16_table[h]; }
static inline uint16_t rd16(const uint8_t* p) { uint16_t v; memcpy(&v, p, 2); return v; }

size_t orc_row_bytes(uint32_t type, size_t n) {
  switch (type) {
    case ORC_F32: return n * 4;
    case ORC_F16: case ORC_BF16: return n * 2;
    case ORC_Q4_0: return n / 32 * 18;
    case ORC_Q5_0: return n / 32 * 22;
    case ORC_Q8_0: return n / 32 * 34;
    case ORC_Q4_K: return n / 256 * 144;
    case ORC_Q6_K: return n / 256 * 210;
    default: return 0;
  }
}

/* ------------------------------------------------------------------ */
/* activation quantizers                                               */
/* ------------------------------------------------------------------ */
/* nearest_int (ops.cpp:107-113); the reference's compiler fuses the
 * preceding product into the magic add: bits(fmaf(a, b, 1.5*2^23)). */
static inline int nearest_int_fma(float a, float b) {
  const float v = fmaf(a, b, 12582912.f);
  return (int)(f_to_bits(v) & 0x007fffff) - 0x00400000;
}

void orc_quantize_row_q8_0(const float* x, size_t n, uint8_t* y) {  /* ops.cpp:116-139 */
  pthread_once(&g_table_once, table_init);
  for (size_t i = 0; i < n / 32; i++) {
    float amax = 0.0f;
    for (int j = 0; j < 32; j++) {
      const float v = fabsf(x[i * 32 + j]);
      if (amax < v) amax = v;
    }
    const float d = amax / 127.0f;
    const float id = d != 0.0f ? 1.0f / d : 0.0f;
    uint8_t* blk = y + i * 34;
    const uint16_t dh = orc_f32_to_f16(d);
    memcpy(blk, &dh, 2);
    for (int j = 0; j < 32; j++) blk[2 + j] = (uint8_t)(int8_t)nearest_int_fma(x[i * 32 + j], id);
  }
}

void orc_quantize_row_q8_k(const float* x, size_t n, uint8_t* y) {  /* ops.cpp:142-178 */
  for (size_t i = 0; i < n / 256; i++) {
    uint8_t* blk = y + i * 292;  /* {f32 d; i8 qs[256]; i16 bsums[16]} */
    const float* xb = x + i * 256;
    float max = 0, amax = 0;
    for (int j = 0; j < 256; ++j) {
      const float ax = fabsf(xb[j]);
      if (ax > amax) { amax = ax; max = xb[j]; }
    }
    if (amax == 0.0f) { memset(blk, 0, 292); continue; }
    const float iscale = -127.f / max;
    int8_t* qs = (int8_t*)(blk + 4);
    for (int j = 0; j < 256; ++j) {
      int v = nearest_int_fma(iscale, xb[j]);
      qs[j] = (int8_t)(v < -128 ? -128 : (v > 127 ? 127 : v));
    }
    for (int j = 0; j < 16; ++j) {
      int s = 0;
      for (int ii = 0; ii < 16; ++ii) s += qs[j * 16 + ii];
      const int16_t s16 = (int16_t)s;
      memcpy(blk + 260 + 2 * j, &s16, 2);
    }
    const float d = 1.0f / iscale;
    memcpy(blk, &d, 4);
  }
}

/* ------------------------------------------------------------------ */
/* row kernels (one output row each)                                   */
/* ------------------------------------------------------------------ */
/* Q4_0 x Q8_0, AVX2 path ops.cpp:364-399: 8 lane accumulators, lane j holds
 * the integer dot of elements 4j..4j+3 (elements 0..15 = low nibbles of
 * qs[0..15], 16..31 = high nibbles), acc_j = fma(d_w*d_x, isum_j, acc_j),
 * horizontal sum hsum_float_8 (ops.cpp:324-330). */
static float row_q4_0(const uint8_t* w, const uint8_t* xq, size_t nb) {
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (size_t b = 0; b < nb; b++) {
    const uint8_t* wb = w + b * 18;
    const uint8_t* xb = xq + b * 34;
    const float d = F16(rd16(wb)) * F16(rd16(xb));
    const int8_t* q8 = (const int8_t*)(xb + 2);
    for (int j = 0; j < 8; j++) {
      int isum = 0;
      for (int e = 4 * j; e < 4 * j + 4; e++) {
        const int nib = e < 16 ? (wb[2 + e] & 0x0F) : (wb[2 + e - 16] >> 4);
        isum += (nib - 8) * q8[e];
      }
      acc[j] = fmaf(d, (float)isum, acc[j]);
    }
  }
  return ((acc[0] + acc[4]) + (acc[2] + acc[6])) + ((acc[1] + acc[5]) + (acc[3] + acc[7]));
}

/* F16, AVX2+F16C path ops.cpp:541-586 (x pre-rounded to f16 by the caller) */
static float row_f16(const uint16_t* w, const uint16_t* x16, size_t n) {
  const size_t np = n & ~(size_t)31;
  float s[4][8];
  memset(s, 0, sizeof s);
  for (size_t k = 0; k < np; k += 32)
    for (int l = 0; l < 4; l++)
      for (int m = 0; m < 8; m++)
        s[l][m] = fmaf(F16(w[k + 8 * l + m]), F16(x16[k + 8 * l + m]), s[l][m]);
  float v[8], t[4];
  for (int m = 0; m < 8; m++) v[m] = (s[0][m] + s[1][m]) + (s[2][m] + s[3][m]);
  for (int m = 0; m < 4; m++) t[m] = v[m] + v[m + 4];
  float r = (t[0] + t[1]) + (t[2] + t[3]);
  for (size_t k = np; k < n; ++k) r = fmaf(F16(w[k]), F16(x16[k]), r);
  return r;
}

/* Q8_0 x Q8_0, ops.cpp:806-824 */
static float row_q8_0(const uint8_t* w, const uint8_t* xq, size_t nb) {
  float sum = 0.0f;
  for (size_t b = 0; b < nb; b++) {
    const int8_t* wq = (const int8_t*)(w + b * 34 + 2);
    const int8_t* xqs = (const int8_t*)(xq + b * 34 + 2);
    int dot = 0;
    for (int i = 0; i < 32; i++) dot += wq[i] * xqs[i];
    sum = fmaf((float)dot * F16(rd16(w + b * 34)), F16(rd16(xq + b * 34)), sum);
  }
  return sum;
}

static inline void scale_min_k4(int j, const uint8_t* q, uint8_t* d, uint8_t* m) {  /* ops.cpp:633-641 */
  if (j < 4) { *d = q[j] & 63; *m = q[j + 4] & 63; }
  else { *d = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4); *m = (q[j + 4] >> 4) | ((q[j - 0] >> 6) << 4); }
}

/* Q4_K x Q8_K, ops.cpp:643-691 */
static float row_q4_k(const uint8_t* w, const uint8_t* xk, size_t nb) {
  float sum = 0.0f;
  for (size_t b = 0; b < nb; b++) {
    const uint8_t* blk = w + b * 144;  /* {f16 d; f16 dmin; u8 scales[12]; u8 qs[128]} */
    const uint8_t* xb = xk + b * 292;
    float xd; memcpy(&xd, xb, 4);
    const float d = F16(rd16(blk)) * xd;
    const float mn = F16(rd16(blk + 2)) * xd;
    const uint8_t* sc = blk + 4;
    const uint8_t* q4 = blk + 16;
    const int8_t* q8 = (const int8_t*)(xb + 4);
    int16_t bs[16]; memcpy(bs, xb + 260, 32);
    int is = 0;
    for (int j = 0; j < 256; j += 64) {
      uint8_t s, m;
      scale_min_k4(is + 0, sc, &s, &m);
      float d1 = d * (float)s, m1 = mn * (float)m;
      int a = 0;
      for (int l = 0; l < 32; ++l) a += (q4[l] & 0xF) * q8[l];
      sum = sum + fmaf((float)a, d1, -(m1 * (float)(bs[is * 2] + bs[is * 2 + 1])));
      scale_min_k4(is + 1, sc, &s, &m);
      d1 = d * (float)s; m1 = mn * (float)m;
      a = 0;
      for (int l = 0; l < 32; ++l) a += (q4[l] >> 4) * q8[l + 32];
      sum = sum + fmaf((float)a, d1, -(m1 * (float)(bs[(is + 1) * 2] + bs[(is + 1) * 2 + 1])));
      q4 += 32; q8 += 64; is += 2;
    }
  }
  return sum;
}

/* Q6_K x Q8_K, ops.cpp:727-770 */
static float row_q6_k(const uint8_t* w, const uint8_t* xk, size_t nb) {
  float sum = 0.0f;
  for (size_t b = 0; b < nb; b++) {
    const uint8_t* blk = w + b * 210;  /* {u8 ql[128]; u8 qh[64]; i8 scales[16]; f16 d} */
    const uint8_t* xb = xk + b * 292;
    float xd; memcpy(&xd, xb, 4);
    const float d = F16(rd16(blk + 208)) * xd;
    const uint8_t* ql = blk;
    const uint8_t* qh = blk + 128;
    const int8_t* sc = (const int8_t*)(blk + 192);
    const int8_t* xq = (const int8_t*)(xb + 4);
    for (int n = 0; n < 256; n += 128) {
      int32_t part = 0;
      for (int l = 0; l < 32; ++l) {
        const int is = l / 16;
        const int8_t q1 = (int8_t)((ql[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
        const int8_t q2 = (int8_t)((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
        const int8_t q3 = (int8_t)((ql[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
        const int8_t q4 = (int8_t)((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
        part += sc[is + 0] * q1 * xq[l + 0];
        part += sc[is + 2] * q2 * xq[l + 32];
        part += sc[is + 4] * q3 * xq[l + 64];
        part += sc[is + 6] * q4 * xq[l + 96];
      }
      sum = fmaf((float)part, d, sum);
      ql += 64; qh += 32; sc += 8; xq += 128;
    }
  }
  return sum;
}

/* Q5_0 x f32 (no activation quantization), ops.cpp:856-879 */
static float row_q5_0(const uint8_t* w, const float* x, size_t nb) {
  float sum = 0.0f;
  for (size_t b = 0; b < nb; b++) {
    const uint8_t* blk = w + b * 22;  /* {f16 d; u8 qh[4]; u8 qs[16]} packed */
    const float d = F16(rd16(blk));
    uint32_t qh; memcpy(&qh, blk + 2, 4);
    for (int i = 0; i < 16; ++i) {
      const uint8_t ql = blk[6 + i];
      const int q0 = (ql & 0x0F) | (((qh >> (i + 0)) & 1) << 4);
      const int q1 = (ql >> 4) | (((qh >> (i + 16)) & 1) << 4);
      sum = fmaf(d * (float)(q0 - 16), x[b * 32 + i + 0], sum);
      sum = fmaf(d * (float)(q1 - 16), x[b * 32 + i + 16], sum);
    }
  }
  return sum;
}

/* BF16 x f32, ops.cpp:908-917 */
static float row_bf16(const uint16_t* w, const float* x, size_t n) {
  float sum = 0.0f;
  for (size_t c = 0; c < n; ++c) sum = fmaf(orc_bf16_to_f32(w[c]), x[c], sum);
  return sum;
}

/* ------------------------------------------------------------------ */
/* GEMV driver: contiguous row chunks per thread (ops.cpp:439-450)      */
/* ------------------------------------------------------------------ */
typedef struct {
  uint32_t type; const uint8_t* w; size_t row_bytes, n_cols, r0, r1;
  const void* xprep; const float* x; float* o;
} gemv_job;

static void* gemv_worker(void* arg) {
  gemv_job* j = (gemv_job*)arg;
  for (size_t r = j->r0; r < j->r1; r++) {
    const uint8_t* wr = j->w + r * j->row_bytes;
    float v = 0.0f;
    switch (j->type) {
      case ORC_Q4_0: v = row_q4_0(wr, (const uint8_t*)j->xprep, j->n_cols / 32); break;
      case ORC_Q8_0: v = row_q8_0(wr, (const uint8_t*)j->xprep, j->n_cols / 32); break;
      case ORC_Q4_K: v = row_q4_k(wr, (const uint8_t*)j->xprep, j->n_cols / 256); break;
      case ORC_Q6_K: v = row_q6_k(wr, (const uint8_t*)j->xprep, j->n_cols / 256); break;
      case ORC_Q5_0: v = row_q5_0(wr, j->x, j->n_cols / 32); break;
      case ORC_BF16: v = row_bf16((const uint16_t*)wr, j->x, j->n_cols); break;
      case ORC_F16: v = row_f16((const uint16_t*)wr, (const uint16_t*)j->xprep, j->n_cols); break;
    }
    j->o[r] = v;
  }
  return NULL;
}

static void gemv_run(uint32_t type, const void* w, size_t rb, size_t n_rows, size_t n_cols, const void* xprep,
                     const float* x, float* o, int n_threads);

int orc_mat_vec_mul(uint32_t type, const void* w, size_t n_rows, size_t n_cols,
                    const float* x, float* o, int n_threads) {
  pthread_once(&g_table_once, table_init);
  const size_t rb = orc_row_bytes(type, n_cols);
  if (rb == 0 || type == ORC_F32) return ORC_FAIL("mat_vec_mul: unsupported tensor type %u", type);
  void* xprep = NULL;
  if (type == ORC_Q4_0 || type == ORC_Q8_0) {
    xprep = malloc(n_cols / 32 * 34 + 1);
    orc_quantize_row_q8_0(x, n_cols, (uint8_t*)xprep);
  } else if (type == ORC_Q4_K || type == ORC_Q6_K) {
    xprep = malloc(n_cols / 256 * 292 + 1);
    orc_quantize_row_q8_k(x, n_cols, (uint8_t*)xprep);
  } else if (type == ORC_F16) {  /* ops.cpp:542-551: x -> f16, RNE */
    uint16_t* x16 = (uint16_t*)malloc(n_cols * 2 + 2);
    for (size_t j = 0; j < n_cols; j++) x16[j] = orc_f32_to_f16(x[j]);
    xprep = x16;
  }
  gemv_run(type, w, rb, n_rows, n_cols, xprep, x, o, n_threads);
  free(xprep);
  return 0;
}

/* The Q4_0 / Q8_0 row loops of mat_vec_mul (ops.cpp:364-399, 806-824) on an
 * activation that is ALREADY a row of 34-B BlockQ8_0 (ops.h:89-92): the
 * op-level tests feed the device's own quantized inputs (prefill GEMM). */
int orc_mat_vec_mul_q8(uint32_t type, const void* w, size_t n_rows, size_t n_cols, const void* xq, float* o,
                       int n_threads) {
  pthread_once(&g_table_once, table_init);
  if (type != ORC_Q4_0 && type != ORC_Q8_0) return ORC_FAIL("mat_vec_mul_q8: type %u is not Q4_0/Q8_0", type);
  gemv_run(type, w, orc_row_bytes(type, n_cols), n_rows, n_cols, xq, NULL, o, n_threads);
  return 0;
}

static void gemv_run(uint32_t type, const void* w, size_t rb, size_t n_rows, size_t n_cols, const void* xprep,
                     const float* x, float* o, int n_threads) {
  if (n_threads < 1) n_threads = 1;
  const size_t chunk = (n_rows + n_threads - 1) / n_threads;
  gemv_job jobs[256];
  pthread_t th[256];
  int nj = 0;
  for (int t = 0; t < n_threads && t < 256; t++) {
    const size_t s = t * chunk, e = s + chunk < n_rows ? s + chunk : n_rows;
    if (s >= e) break;
    jobs[nj] = (gemv_job){type, (const uint8_t*)w, rb, n_cols, s, e, xprep, x, o};
    nj++;
  }
  if (nj == 1) gemv_worker(&jobs[0]);
  else {
    for (int t = 0; t < nj; t++) pthread_create(&th[t], NULL, gemv_worker, &jobs[t]);
    for (int t = 0; t < nj; t++) pthread_join(th[t], NULL);
  }
}

int orc_dequantize_row(uint32_t type, const void* blocks, size_t n_cols, float* o) {
  pthread_once(&g_table_once, table_init);
  const uint8_t* p = (const uint8_t*)blocks;
  switch (type) {
    case ORC_F32: memcpy(o, p, n_cols * 4); return 0;
    case ORC_F16: for (size_t i = 0; i < n_cols; i++) o[i] = F16(rd16(p + 2 * i)); return 0;
    case ORC_Q8_0:  /* ops.cpp:1045-1059 */
      for (size_t b = 0; b < n_cols / 32; b++) {
        const float d = F16(rd16(p + b * 34));
        for (int i = 0; i < 32; i++) o[b * 32 + i] = d * (float)(int8_t)p[b * 34 + 2 + i];
      }
      return 0;
    case ORC_Q5_0:  /* ops.cpp:1061-1082 */
      for (size_t b = 0; b < n_cols / 32; b++) {
        const uint8_t* blk = p + b * 22;
        const float d = F16(rd16(blk));
        uint32_t qh; memcpy(&qh, blk + 2, 4);
        for (int i = 0; i < 16; i++) {
          const uint8_t ql = blk[6 + i];
          const int q0 = (ql & 0x0F) | (((qh >> (i + 0)) & 1) << 4);
          const int q1 = (ql >> 4) | (((qh >> (i + 16)) & 1) << 4);
          o[b * 32 + i] = d * (float)(q0 - 16);
          o[b * 32 + i + 16] = d * (float)(q1 - 16);
        }
      }
      return 0;
    case ORC_Q4_K:  /* ops.cpp:958-1003 */
      for (size_t b = 0; b < n_cols / 256; b++) {
        const uint8_t* blk = p + b * 144;
        const float d = F16(rd16(blk)), mn = F16(rd16(blk + 2));
        const uint8_t* q4 = blk + 16;
        int is = 0;
        for (int j = 0; j < 256; j += 64) {
          uint8_t s, m;
          scale_min_k4(is + 0, blk + 4, &s, &m);
          float d1 = d * (float)s, m1 = mn * (float)m;
          for (int l = 0; l < 32; ++l) o[b * 256 + is * 32 + l] = fmaf(d1, (float)(q4[l] & 0xF), -m1);
          scale_min_k4(is + 1, blk + 4, &s, &m);
          d1 = d * (float)s; m1 = mn * (float)m;
          for (int l = 0; l < 32; ++l) o[b * 256 + (is + 1) * 32 + l] = fmaf(d1, (float)(q4[l] >> 4), -m1);
          q4 += 32; is += 2;
        }
      }
      return 0;
    case ORC_Q6_K: {  /* ops.cpp:1005-1043 */
      size_t col = 0;
      for (size_t b = 0; b < n_cols / 256; b++) {
        const uint8_t* blk = p + b * 210;
        const float d = F16(rd16(blk + 208));
        const uint8_t* ql = blk; const uint8_t* qh = blk + 128;
        const int8_t* sc = (const int8_t*)(blk + 192);
        for (int n = 0; n < 256; n += 128) {
          for (int l = 0; l < 32; ++l) {
            const int is = l / 16;
            const int8_t q1 = (int8_t)((ql[l + 0] & 0xF) | (((qh[l] >> 0) & 3) << 4)) - 32;
            const int8_t q2 = (int8_t)((ql[l + 32] & 0xF) | (((qh[l] >> 2) & 3) << 4)) - 32;
            const int8_t q3 = (int8_t)((ql[l + 0] >> 4) | (((qh[l] >> 4) & 3) << 4)) - 32;
            const int8_t q4 = (int8_t)((ql[l + 32] >> 4) | (((qh[l] >> 6) & 3) << 4)) - 32;
            o[col + l + 0] = d * (float)sc[is + 0] * (float)q1;
            o[col + l + 32] = d * (float)sc[is + 2] * (float)q2;
            o[col + l + 64] = d * (float)sc[is + 4] * (float)q3;
            o[col + l + 96] = d * (float)sc[is + 6] * (float)q4;
          }
          col += 128; ql += 64; qh += 32; sc += 8;
        }
      }
      return 0;
    }
    default: return ORC_FAIL("dequantize: unsupported type %u", type);
  }
}

/* ------------------------------------------------------------------ */
/* small ops                                                           */
/* ------------------------------------------------------------------ */
int orc_rms_norm(float* o, const float* x, size_t n, double eps) {  /* ops.cpp:28-43 */
  if (eps <= 0) return ORC_FAIL("Error: eps must be > 0 in rms_norm.");
  float sum = 0.0f;
  for (size_t i = 0; i < n; i++) sum = fmaf(x[i], x[i], sum);
  const float mean = sum / (float)n;
  const float s = 1.0f / sqrtf((float)((double)mean + eps));
  for (size_t i = 0; i < n; i++) o[i] = s * x[i];
  return 0;
}

void orc_softmax(float* x, size_t n) {  /* ops.cpp:45-62 */
  float mx = x[0];
  for (size_t i = 0; i < n; i++) if (x[i] > mx) mx = x[i];
  float sum = 0.0f;
  for (size_t i = 0; i < n; i++) { x[i] = expf(x[i] - mx); sum += x[i]; }
  for (size_t i = 0; i < n; i++) x[i] /= sum;
}

void orc_rope(float* t, size_t n_tokens, size_t n_heads, size_t head_dim, int n_rot,
              float base, float freq_scale, int pos) {  /* ops.cpp:67-95 */
  for (uint32_t tk = 0; tk < n_tokens; ++tk) {
    for (int i = 0; i < n_rot / 2; ++i) {
      const float freq = 1.0f / powf(base, (float)(2 * i) / (float)n_rot);
      const float val = ((float)(uint32_t)(pos + tk) * freq) / freq_scale;
      float s, c;
      sincosf(val, &s, &c);
      for (size_t h = 0; h < n_heads; ++h) {
        float* v = t + (tk * n_heads + h) * head_dim;
        const float v0 = v[i], v1 = v[i + n_rot / 2];
        v[i] = fmaf(v0, c, -(v1 * s));
        v[i + n_rot / 2] = fmaf(v0, s, v1 * c);
      }
    }
  }
}

void orc_scale(float* t, size_t n, float s) { for (size_t i = 0; i < n; i++) t[i] *= s; } /* ops.cpp:97-105 */

void orc_vec_scale_f16(uint16_t* y, size_t n, float v) {  /* ops.cpp:1084-1089 */
  pthread_once(&g_table_once, table_init);
  for (size_t i = 0; i < n; i++) y[i] = orc_f32_to_f16(F16(y[i]) * v);
}

void orc_vec_mad_f16(uint16_t* y, const uint16_t* x, size_t n, float v) {  /* ops.cpp:1091-1099 */
  pthread_once(&g_table_once, table_init);
  for (size_t i = 0; i < n; i++) y[i] = orc_f32_to_f16(fmaf(F16(x[i]), v, F16(y[i])));
}

void orc_gelu_mul(float* o, const float* gate, const float* up, size_t n) {  /* model.cpp:892-899 */
  const float c = sqrtf((float)(2.0 / M_PI));
  for (size_t j = 0; j < n; j++) {
    const float x = gate[j];
    const float inner = x + ((0.044715f * x) * x) * x;
    const float g = (0.5f * x) * (1.0f + tanhf(c * inner));
    o[j] = g * up[j];
  }
}

/* the attention logit soft-cap (model.cpp:511-513): score is a double, the cap a float, so
 * score / cap is a double division, tanhf takes its float rounding, and cap * tanhf(...) is a float
 * product stored back into the double */
static inline double softcap_score(double score, float cap) {
  return cap > 0.0f ? (double)(cap * tanhf((float)(score / (double)cap))) : score;
}

void orc_attn_head_cap(const float* q, const uint16_t* k, const uint16_t* v, size_t n_keys,
                       size_t hd, float cap, float* out) {  /* model.cpp:481-547 (ALiBi 0) */
  pthread_once(&g_table_once, table_init);
  uint16_t* vacc = (uint16_t*)malloc(hd * 2);
  uint16_t* q16 = (uint16_t*)malloc(hd * 2);
  const uint16_t z = orc_f32_to_f16(0.0f);
  for (size_t i = 0; i < hd; i++) { vacc[i] = z; q16[i] = orc_f32_to_f16(q[i]); }
  float s_acc = 0.0f, max_score = -INFINITY;
  for (size_t t = 0; t < n_keys; t++) {
    double score = 0.0;
    for (size_t i = 0; i < hd; i++) score += (double)(F16(k[t * hd + i]) * F16(q16[i]));
    score = softcap_score(score, cap);
    const float prev_max = max_score;
    float e, pe;
    if (score > (double)prev_max) {
      max_score = (float)score;
      e = 1.0f;
      pe = expf(prev_max - max_score);
      orc_vec_scale_f16(vacc, hd, pe);
    } else {
      e = expf((float)(score - (double)max_score));
      pe = 1.0f;
    }
    orc_vec_mad_f16(vacc, v + t * hd, hd, e);
    s_acc = s_acc * pe + e;
  }
  const float inv = s_acc == 0.0f ? 0.0f : 1.0f / s_acc;
  for (size_t i = 0; i < hd; i++) out[i] = F16(vacc[i]) * inv;
  free(vacc); free(q16);
}

void orc_attn_head(const float* q, const uint16_t* k, const uint16_t* v, size_t n_keys, size_t hd, float* out) {
  orc_attn_head_cap(q, k, v, n_keys, hd, 0.0f, out);
}

/* NOT the reference: the same attention in float64 math (no f16 V
 * accumulator rounding).  Used only to pin the fast GPU path, whose fp32
 * split-K accumulation is closer to exact math than the reference itself
 * (whose f16 accumulator carries ~1e-3 absolute error). */
void orc_attn_head_f64_cap(const float* q, const uint16_t* k, const uint16_t* v, size_t n_keys, size_t hd,
                           float cap, float* out) {
  pthread_once(&g_table_once, table_init);
  double* s = (double*)malloc(sizeof(double) * n_keys);
  double mx = -INFINITY, l = 0.0;
  for (size_t t = 0; t < n_keys; t++) {
    double sc = 0.0;
    for (size_t i = 0; i < hd; i++) sc += (double)F16(k[t * hd + i]) * (double)F16(orc_f32_to_f16(q[i]));
    if (cap > 0.0f) sc = (double)cap * tanh(sc / (double)cap);
    s[t] = sc;
    if (sc > mx) mx = sc;
  }
  for (size_t t = 0; t < n_keys; t++) { s[t] = exp(s[t] - mx); l += s[t]; }
  for (size_t i = 0; i < hd; i++) {
    double a = 0.0;
    for (size_t t = 0; t < n_keys; t++) a += s[t] * (double)F16(v[t * hd + i]);
    out[i] = (float)(a / l);
  }
  free(s);
}

void orc_attn_head_f64(const float* q, const uint16_t* k, const uint16_t* v, size_t n_keys, size_t hd, float* out) {
  orc_attn_head_f64_cap(q, k, v, n_keys, hd, 0.0f, out);
}

/* ------------------------------------------------------------------ */
/* minimal GGUF v3 reader (gguf.cpp:195-304)                           */
/* ------------------------------------------------------------------ */
typedef struct { char name[96]; uint32_t ndim; uint64_t shape[4]; uint32_t type; uint64_t off; } orc_tensor;

typedef struct { const uint8_t* p; size_t n, pos; int err; } rdr;
static int rd(rdr* r, void* dst, size_t n) {
  if (r->pos + n > r->n) { r->err = 1; return -1; }
  memcpy(dst, r->p + r->pos, n); r->pos += n; return 0;
}
static uint64_t rd_u64(rdr* r) { uint64_t v = 0; rd(r, &v, 8); return v; }
static uint32_t rd_u32(rdr* r) { uint32_t v = 0; rd(r, &v, 4); return v; }

typedef struct { int kind; double num; uint32_t u32; const uint8_t* str; size_t slen;
                 uint32_t arr_type; uint64_t arr_n; size_t arr_pos; } gval;

static int skip_value(rdr* r, uint32_t type, gval* out);
static int skip_value(rdr* r, uint32_t type, gval* out) {
  static const int sz[] = {1, 1, 2, 2, 4, 4, 4, 1, 0, 0, 8, 8, 8};
  if (out) { memset(out, 0, sizeof *out); out->kind = (int)type; }
  if (type == 8) {
    uint64_t l = rd_u64(r);
    if (r->pos + l > r->n) { r->err = 1; return -1; }
    if (out) { out->str = r->p + r->pos; out->slen = l; }
    r->pos += l; return 0;
  }
  if (type == 9) {
    const uint32_t et = rd_u32(r); const uint64_t cnt = rd_u64(r);
    if (out) { out->arr_type = et; out->arr_n = cnt; out->arr_pos = r->pos; }
    for (uint64_t i = 0; i < cnt && !r->err; i++) skip_value(r, et, NULL);
    return r->err ? -1 : 0;
  }
  if (type > 12) { r->err = 1; return -1; }
  uint8_t buf[8] = {0};
  if (rd(r, buf, sz[type])) return -1;
  if (out) {
    switch (type) {
      case 0: out->num = buf[0]; break; case 1: out->num = (int8_t)buf[0]; break;
      case 2: { uint16_t v; memcpy(&v, buf, 2); out->num = v; } break;
      case 3: { int16_t v; memcpy(&v, buf, 2); out->num = v; } break;
      case 4: { uint32_t v; memcpy(&v, buf, 4); out->num = v; } break;
      case 5: { int32_t v; memcpy(&v, buf, 4); out->num = v; } break;
      case 6: { float v; memcpy(&v, buf, 4); out->num = v; } break;
      case 7: out->num = buf[0] != 0; break;
      case 10: { uint64_t v; memcpy(&v, buf, 8); out->num = (double)v; } break;
      case 11: { int64_t v; memcpy(&v, buf, 8); out->num = (double)v; } break;
      case 12: { double v; memcpy(&v, buf, 8); out->num = v; } break;
    }
    memcpy(&out->u32, buf, 4);
  }
  return 0;
}

#define ORC_MAX_LAYERS 128
typedef struct {
  int attn_norm, q, k, v, o, q_norm, k_norm, post_attn_norm, ffn_norm, gate, up, down, post_ffw_norm;
  int out_scale, ple_gate, ple_proj, ple_post_norm;  /* Gemma-4 (model.cpp:215-228) */
} orc_layer;

struct orc_model {
  const uint8_t* base; size_t size, data_start;
  orc_tensor* t; int nt;
  int n_layer, n_embd, n_ff, n_head, n_head_kv, hd_k, hd_v, hd_k_swa, hd_v_swa;
  float eps_f; float rope_base; float attn_scale; float final_softcap, attn_softcap;
  int n_swa; uint8_t swa[ORC_MAX_LAYERS];
  orc_layer L[ORC_MAX_LAYERS];
  int tok_embd, out_norm, vocab;
  int gemma4, n_epl, kv_from;                     /* model.cpp:117-166: per-layer embd width, shared-KV start */
  int ple_table, ple_model_proj, ple_proj_norm;   /* model.cpp:181-188 */
  int n_threads, max_ctx, n_cached, attn_f64;
  uint16_t* kc[ORC_MAX_LAYERS]; uint16_t* vc[ORC_MAX_LAYERS];
};

static int key_eq(const uint8_t* k, size_t kl, const char* a, const char* b) {
  const size_t la = strlen(a), lb = b ? strlen(b) : 0;
  return kl == la + lb && memcmp(k, a, la) == 0 && (lb == 0 || memcmp(k + la, b, lb) == 0);
}

static const uint8_t* tdata(const orc_model* m, int ti) { return m->base + m->data_start + m->t[ti].off; }

orc_model* orc_model_create(const uint8_t* g, size_t size, int n_threads, int max_ctx) {
  pthread_once(&g_table_once, table_init);
  orc_model* m = (orc_model*)calloc(1, sizeof *m);
  m->base = g; m->size = size; m->n_threads = n_threads < 1 ? 1 : n_threads;
  m->max_ctx = max_ctx;
  rdr r = {g, size, 0, 0};
  if (rd_u32(&r) != 0x46554747u) { ORC_FAIL("Invalid GGUF magic number"); free(m); return NULL; }
  rd_u32(&r);
  const uint64_t nt = rd_u64(&r), nkv = rd_u64(&r);
  /* pass 1: architecture name */
  char arch[64] = {0};
  const size_t kv_start = r.pos;
  for (uint64_t i = 0; i < nkv && !r.err; i++) {
    const uint64_t kl = rd_u64(&r); const uint8_t* k = g + r.pos; r.pos += kl;
    const uint32_t ty = rd_u32(&r); gval v; skip_value(&r, ty, &v);
    if (key_eq(k, kl, "general.architecture", NULL) && ty == 8 && v.slen < sizeof arch) memcpy(arch, v.str, v.slen);
  }
  r.pos = kv_start;
  int have[16] = {0};
  m->hd_k = -1; m->hd_k_swa = -1; m->hd_v = -1; m->hd_v_swa = -1;
  for (uint64_t i = 0; i < nkv && !r.err; i++) {
    const uint64_t kl = rd_u64(&r); const uint8_t* k = g + r.pos; r.pos += kl;
    const uint32_t ty = rd_u32(&r); gval v; skip_value(&r, ty, &v);
    if (kl <= strlen(arch) || memcmp(k, arch, strlen(arch)) != 0 || k[strlen(arch)] != '.') continue;
    const uint8_t* s = k + strlen(arch) + 1; const size_t sl = kl - strlen(arch) - 1;
#define KEY(str) key_eq(s, sl, str, NULL)
    if (KEY("block_count")) { m->n_layer = (int)v.u32; have[0] = 1; }
    else if (KEY("embedding_length")) { m->n_embd = (int)v.u32; have[1] = 1; }
    else if (KEY("feed_forward_length")) { m->n_ff = (int)v.u32; have[2] = 1; }
    else if (KEY("attention.head_count")) { m->n_head = (int)v.u32; have[3] = 1; }
    else if (KEY("attention.head_count_kv")) { m->n_head_kv = (int)v.u32; have[4] = 1; }
    else if (KEY("attention.layer_norm_rms_epsilon")) { memcpy(&m->eps_f, &v.u32, 4); have[5] = 1; }
    else if (KEY("rope.freq_base")) { memcpy(&m->rope_base, &v.u32, 4); have[6] = 1; }
    else if (KEY("attention.key_length")) m->hd_k = (int)v.u32;
    else if (KEY("attention.key_length_swa")) m->hd_k_swa = (int)v.u32;
    else if (KEY("attention.value_length")) m->hd_v = (int)v.u32;
    else if (KEY("attention.value_length_swa")) m->hd_v_swa = (int)v.u32;
    else if (KEY("attention.logit_softcapping")) memcpy(&m->attn_softcap, &v.u32, 4);
    else if (KEY("embedding_length_per_layer") || KEY("embedding_length_per_layer_input")) {
      if (KEY("embedding_length_per_layer") || m->n_epl == 0) m->n_epl = (int)v.u32;  /* model.cpp:148-157 */
    } else if (KEY("attention.shared_kv_layers")) m->kv_from = -(int)v.u32 - 2;   /* resolved below */
    else if (KEY("final_logit_softcapping") || KEY("attention.final_logit_softcapping")) {
      if (KEY("attention.final_logit_softcapping")) memcpy(&m->final_softcap, &v.u32, 4);
    } else if (KEY("attention.sliding_window_pattern") && ty == 9) {
      rdr a = {g, size, v.arr_pos, 0};
      for (uint64_t e = 0; e < v.arr_n && e < ORC_MAX_LAYERS; e++) {
        gval ev; skip_value(&a, v.arr_type, &ev); m->swa[e] = ev.u32 & 0xFF ? 1 : 0; m->n_swa++;
      }
    }
#undef KEY
  }
  for (int i = 0; i < 7; i++)
    if (!have[i]) { ORC_FAIL("Failed to find required metadata key #%d", i); free(m); return NULL; }
  if (m->n_layer > ORC_MAX_LAYERS) { ORC_FAIL("too many layers"); free(m); return NULL; }
  /* model.cpp:93-120 */
  if (m->hd_k < 0) m->hd_k = m->n_embd / m->n_head;
  if (m->hd_k_swa < 0) m->hd_k_swa = m->hd_k;
  if (m->hd_v < 0) m->hd_v = m->hd_k;
  if (m->hd_v_swa < 0) m->hd_v_swa = m->hd_v;
  m->attn_scale = 1.0f / sqrtf((float)m->hd_k);
  m->gemma4 = strcmp(arch, "gemma4") == 0;
  if (m->gemma4) m->attn_scale = 1.0f;                       /* model.cpp:119-122 */
  m->kv_from = m->kv_from <= -2 ? m->n_layer - (-m->kv_from - 2) : -1;  /* model.cpp:159-166 */
  if (m->hd_k != m->hd_v || m->hd_k_swa != m->hd_v_swa) {  /* run_attn dots over n_embd_head_v */
    ORC_FAIL("key_length != value_length is not supported"); free(m); return NULL;
  }
  /* tensor infos */
  m->t = (orc_tensor*)calloc(nt ? nt : 1, sizeof(orc_tensor)); m->nt = (int)nt;
  m->tok_embd = m->out_norm = -1;
  m->ple_table = m->ple_model_proj = m->ple_proj_norm = -1;
  for (int l = 0; l < ORC_MAX_LAYERS; l++) memset(&m->L[l], 0xff, sizeof(orc_layer));
  for (uint64_t i = 0; i < nt && !r.err; i++) {
    orc_tensor* T = &m->t[i];
    const uint64_t nl = rd_u64(&r);
    const size_t cl = nl < sizeof T->name - 1 ? nl : sizeof T->name - 1;
    memcpy(T->name, g + r.pos, cl); r.pos += nl;
    T->ndim = rd_u32(&r);
    for (uint32_t d = 0; d < T->ndim; d++) { const uint64_t v = rd_u64(&r); if (d < 4) T->shape[d] = v; }
    T->type = rd_u32(&r); T->off = rd_u64(&r);
  }
  if (r.err) { ORC_FAIL("Read beyond end of file"); orc_model_destroy(m); return NULL; }
  m->data_start = (r.pos + 31) & ~(size_t)31;
  for (int i = 0; i < m->nt; i++) {  /* model.cpp:169-238 */
    const char* n = m->t[i].name;
    if (!strcmp(n, "token_embd.weight")) m->tok_embd = i;
    else if (!strcmp(n, "output_norm.weight")) m->out_norm = i;
    else if (!strcmp(n, "token_embd_per_layer.weight") || !strcmp(n, "per_layer_token_embd.weight")) m->ple_table = i;
    else if (!strcmp(n, "per_layer_model_proj.weight")) m->ple_model_proj = i;
    else if (!strcmp(n, "per_layer_proj_norm.weight")) m->ple_proj_norm = i;
    else if (!strncmp(n, "blk.", 4)) {
      char* end; const long li = strtol(n + 4, &end, 10);
      if (*end != '.' || li < 0 || li >= m->n_layer) continue;
      const char* p = end + 1; orc_layer* L = &m->L[li];
      if (!strcmp(p, "attn_norm.weight")) L->attn_norm = i;
      else if (!strcmp(p, "attn_q.weight")) L->q = i;
      else if (!strcmp(p, "attn_k.weight")) L->k = i;
      else if (!strcmp(p, "attn_v.weight")) L->v = i;
      else if (!strcmp(p, "attn_output.weight")) L->o = i;
      else if (!strcmp(p, "ffn_norm.weight")) L->ffn_norm = i;
      else if (!strcmp(p, "ffn_gate.weight")) L->gate = i;
      else if (!strcmp(p, "ffn_up.weight")) L->up = i;
      else if (!strcmp(p, "ffn_down.weight")) L->down = i;
      else if (!strcmp(p, "post_attention_norm.weight") || !strcmp(p, "attn_post_norm.weight")) L->post_attn_norm = i;
      else if (!strcmp(p, "post_ffw_norm.weight") || !strcmp(p, "ffn_post_norm.weight")) L->post_ffw_norm = i;
      else if (!strcmp(p, "attn_k_norm.weight")) L->k_norm = i;
      else if (!strcmp(p, "attn_q_norm.weight")) L->q_norm = i;
      else if (!strcmp(p, "out_scale.weight") || !strcmp(p, "layer_output_scale.weight")) L->out_scale = i;
      else if (!strcmp(p, "per_layer_inp_gate.weight") || !strcmp(p, "inp_gate.weight")) L->ple_gate = i;
      else if (!strcmp(p, "per_layer_proj.weight") || !strcmp(p, "proj.weight")) L->ple_proj = i;
      else if (!strcmp(p, "per_layer_post_norm.weight") || !strcmp(p, "post_norm.weight")) L->ple_post_norm = i;
    }
  }
  if (m->tok_embd < 0 || m->out_norm < 0) { ORC_FAIL("missing token_embd/output_norm"); orc_model_destroy(m); return NULL; }
  m->vocab = (int)m->t[m->tok_embd].shape[1];
  /* shared KV (model.cpp:832-835): layer l >= kv_from reads kv_from-2 (SWA) or
     kv_from-1 (global); the source must be of the same kind (same head dims) */
  for (int l = m->kv_from < 0 ? m->n_layer : m->kv_from; l < m->n_layer; l++) {
    const int sw = l < m->n_swa ? m->swa[l] : (l % 6 < 5), src = m->kv_from - (sw ? 2 : 1);
    const int ssw = src >= 0 ? (src < m->n_swa ? m->swa[src] : (src % 6 < 5)) : -1;
    if (ssw != sw) { ORC_FAIL("shared-KV layer %d reads layer %d of another attention kind", l, src); orc_model_destroy(m); return NULL; }
  }
  for (int l = 0; l < m->n_layer; l++) {
    const int hd = m->hd_k > m->hd_k_swa ? m->hd_k : m->hd_k_swa;
    const int hv = m->hd_v > m->hd_v_swa ? m->hd_v : m->hd_v_swa;
    m->kc[l] = (uint16_t*)calloc((size_t)max_ctx * m->n_head_kv * hd, 2);
    m->vc[l] = (uint16_t*)calloc((size_t)max_ctx * m->n_head_kv * hv, 2);
  }
  return m;
}

void orc_model_destroy(orc_model* m) {
  if (!m) return;
  for (int l = 0; l < m->n_layer && l < ORC_MAX_LAYERS; l++) { free(m->kc[l]); free(m->vc[l]); }
  free(m->t); free(m);
}

int orc_model_vocab(const orc_model* m) { return m->vocab; }
void orc_model_set_attn_f64(orc_model* m, int on) { m->attn_f64 = on; }

static int mm(const orc_model* m, int ti, const float* x, float* o) {
  const orc_tensor* T = &m->t[ti];
  return orc_mat_vec_mul(T->type, tdata(m, ti), T->shape[1], T->shape[0], x, o, m->n_threads);
}

/* run_norm with weight: model.cpp:346-423 (weight read as f32 from file) */
static void norm_w(const orc_model* m, int wi, const float* x, float* o, size_t n) {
  orc_rms_norm(o, x, n, (double)m->eps_f);
  const float* w = (const float*)tdata(m, wi);
  for (size_t j = 0; j < n; j++) o[j] = o[j] * w[j];
}

int orc_model_forward(orc_model* m, const int* tokens, int T, int pos, float* logits) {
  if (T <= 0) return ORC_FAIL("no tokens");
  if (pos + T > m->max_ctx) return ORC_FAIL("context overflow");
  const int E = m->n_embd;
  const orc_tensor* te = &m->t[m->tok_embd];
  const size_t te_row = orc_row_bytes(te->type, te->shape[0]);
  float* hs = (float*)malloc(sizeof(float) * T * E);
  const float emb_scale = sqrtf((float)E);  /* model.cpp:336-344 */
  for (int t = 0; t < T; t++) {
    if (orc_dequantize_row(te->type, tdata(m, m->tok_embd) + (size_t)tokens[t] * te_row, E, hs + t * E)) {
      free(hs); return -1;
    }
    for (int j = 0; j < E; j++) hs[t * E + j] *= emb_scale;
  }
  size_t mx = (size_t)(m->n_ff > E ? m->n_ff : E);
  for (int l = 0; l < m->n_layer; l++) {
    const orc_layer* L = &m->L[l];
    const size_t r[] = {m->t[L->q].shape[1], L->k >= 0 ? m->t[L->k].shape[1] : 0, L->v >= 0 ? m->t[L->v].shape[1] : 0,
                        m->t[L->o].shape[1], m->t[L->gate].shape[1], m->t[L->down].shape[1]};
    for (int i = 0; i < 6; i++) if (r[i] > mx) mx = r[i];
  }
  /* Gemma-4 per-layer inputs (model.cpp:568-704): [T][n_layer][n_epl] */
  const int NL = m->n_layer, EP = m->n_epl;
  float* inp_pl = NULL;
  if (m->ple_table >= 0) {
    const orc_tensor* pt = &m->t[m->ple_table];
    const size_t row_el = (size_t)EP * NL, row_b = orc_row_bytes(pt->type, row_el);
    const float sc = sqrtf((float)EP);
    inp_pl = (float*)malloc(sizeof(float) * T * row_el);
    float* proj = (float*)malloc(sizeof(float) * row_el);
    float* nx = (float*)malloc(sizeof(float) * EP);
    for (int t = 0; t < T; t++) {
      float* row = inp_pl + (size_t)t * row_el;
      if (orc_dequantize_row(pt->type, tdata(m, m->ple_table) + (size_t)tokens[t] * row_b, row_el, row)) {
        free(hs); free(inp_pl); free(proj); free(nx); return -1;
      }
      for (size_t i = 0; i < row_el; i++) row[i] *= sc;
    }
    if (m->ple_model_proj >= 0) {
      const float ps = 1.0f / sqrtf((float)E), is = 1.0f / sqrtf(2.0f);
      const float* nw = (const float*)tdata(m, m->ple_proj_norm);
      for (int t = 0; t < T; t++) {
        mm(m, m->ple_model_proj, hs + (size_t)t * E, proj);
        for (size_t i = 0; i < row_el; i++) proj[i] *= ps;
        for (int l = 0; l < NL; l++) {
          orc_rms_norm(nx, proj + (size_t)l * EP, EP, (double)m->eps_f);
          float* d = inp_pl + (size_t)t * row_el + (size_t)l * EP;
          for (int i = 0; i < EP; i++) d[i] = (nx[i] * nw[i] + d[i]) * is;
        }
      }
    }
    free(proj); free(nx);
  }
  float* xn = (float*)malloc(sizeof(float) * mx);
  float* qv = (float*)malloc(sizeof(float) * T * mx);
  float* kv = (float*)malloc(sizeof(float) * T * mx);
  float* vv = (float*)malloc(sizeof(float) * T * mx);
  float* att = (float*)malloc(sizeof(float) * T * mx);
  float* tmp = (float*)malloc(sizeof(float) * mx);
  float* g = (float*)malloc(sizeof(float) * mx);
  float* u = (float*)malloc(sizeof(float) * mx);
  float* hb = (float*)malloc(sizeof(float) * T * mx);
  int rc = 0;
  for (int l = 0; l < m->n_layer && rc == 0; l++) {
    const orc_layer* L = &m->L[l];
    const int is_swa = l < m->n_swa ? m->swa[l] : (l % 6 < 5);  /* model.cpp:723-729 */
    const float base = is_swa ? 10000.0f : m->rope_base;
    const int hk = is_swa ? m->hd_k_swa : m->hd_k, hv = is_swa ? m->hd_v_swa : m->hd_v;
    const int H = m->n_head, HK = m->n_head_kv;
    /* shared KV (model.cpp:775-777, 832-835): the last layers read an earlier layer's cache */
    const int has_kv = m->kv_from < 0 || l < m->kv_from;
    const int src = has_kv ? l : m->kv_from - (is_swa ? 2 : 1);
    for (int t = 0; t < T; t++) {
      norm_w(m, L->attn_norm, hs + t * E, xn, E);
      rc |= mm(m, L->q, xn, tmp); memcpy(qv + (size_t)t * H * hk, tmp, sizeof(float) * H * hk);
      if (has_kv) {
        rc |= mm(m, L->k, xn, tmp); memcpy(kv + (size_t)t * HK * hk, tmp, sizeof(float) * HK * hk);
        rc |= mm(m, L->v, xn, tmp); memcpy(vv + (size_t)t * HK * hv, tmp, sizeof(float) * HK * hv);
      }
    }
    /* per-head q/k norms (model.cpp:762,792), rope, q scale (model.cpp:767) */
    for (int t = 0; t < T; t++) {
      for (int h = 0; h < H; h++) { float* p = qv + ((size_t)t * H + h) * hk; norm_w(m, L->q_norm, p, tmp, hk); memcpy(p, tmp, 4 * hk); }
      if (has_kv)
        for (int h = 0; h < HK; h++) { float* p = kv + ((size_t)t * HK + h) * hk; norm_w(m, L->k_norm, p, tmp, hk); memcpy(p, tmp, 4 * hk); }
      if (has_kv && m->gemma4)  /* V RMSNorm without weight (model.cpp:813-829) */
        for (int h = 0; h < HK; h++) { float* p = vv + ((size_t)t * HK + h) * hv; orc_rms_norm(tmp, p, hv, (double)m->eps_f); memcpy(p, tmp, 4 * hv); }
    }
    orc_rope(qv, T, H, hk, hk, base, 1.0f, pos);
    orc_scale(qv, (size_t)T * H * hk, m->attn_scale);
    if (has_kv) {
      orc_rope(kv, T, HK, hk, hk, base, 1.0f, pos);
      /* KV append as f16 (model.cpp:442-474): cache [pos][kvh][hd] */
      for (int t = 0; t < T; t++)
        for (int h = 0; h < HK; h++) {
          for (int i = 0; i < hk; i++) m->kc[l][((size_t)(pos + t) * HK + h) * hk + i] = orc_f32_to_f16(kv[((size_t)t * HK + h) * hk + i]);
          for (int i = 0; i < hv; i++) m->vc[l][((size_t)(pos + t) * HK + h) * hv + i] = orc_f32_to_f16(vv[((size_t)t * HK + h) * hv + i]);
        }
    }
    /* attention (model.cpp:478-550): gather per-kv-head contiguous history */
    {
      const int nk_max = pos + T;
      uint16_t* kh = (uint16_t*)malloc(2 * (size_t)nk_max * hk);
      uint16_t* vh = (uint16_t*)malloc(2 * (size_t)nk_max * hv);
      for (int t = 0; t < T; t++)
        for (int h = 0; h < H; h++) {
          const int hkv = h / (H / HK);
          const int nk = pos + t + 1;
          for (int tk = 0; tk < nk; tk++) {
            memcpy(kh + (size_t)tk * hk, &m->kc[src][((size_t)tk * HK + hkv) * hk], 2 * hk);
            memcpy(vh + (size_t)tk * hv, &m->vc[src][((size_t)tk * HK + hkv) * hv], 2 * hv);
          }
          (m->attn_f64 ? orc_attn_head_f64_cap : orc_attn_head_cap)(qv + ((size_t)t * H + h) * hk, kh, vh, nk, hv,
                                                                    m->attn_softcap, att + ((size_t)t * H + h) * hv);
        }
      free(kh); free(vh);
    }
    for (int t = 0; t < T && rc == 0; t++) {
      rc |= mm(m, L->o, att + (size_t)t * H * hv, tmp);
      if (L->post_attn_norm >= 0) { norm_w(m, L->post_attn_norm, tmp, xn, E); memcpy(tmp, xn, 4 * E); }
      for (int j = 0; j < E; j++) hs[t * E + j] += tmp[j];
    }
    for (int t = 0; t < T && rc == 0; t++) {
      norm_w(m, L->ffn_norm, hs + t * E, xn, E);
      rc |= mm(m, L->gate, xn, g);
      rc |= mm(m, L->up, xn, u);
      const int F = (int)m->t[L->gate].shape[1];
      orc_gelu_mul(hb, g, u, F);
      rc |= mm(m, L->down, hb, tmp);
      if (L->post_ffw_norm >= 0) { norm_w(m, L->post_ffw_norm, tmp, xn, E); memcpy(tmp, xn, 4 * E); }
      for (int j = 0; j < E; j++) hs[t * E + j] += tmp[j];
      if (inp_pl) {  /* per-layer embedding (model.cpp:926-966) */
        float* h = hs + (size_t)t * E;
        rc |= mm(m, L->ple_gate, h, g);
        orc_gelu_mul(u, g, inp_pl + (size_t)t * EP * NL + (size_t)l * EP, EP);
        rc |= mm(m, L->ple_proj, u, tmp);
        orc_rms_norm(xn, tmp, E, (double)m->eps_f);
        const float* pw = (const float*)tdata(m, L->ple_post_norm);
        for (int j = 0; j < E; j++) h[j] += xn[j] * pw[j];
      }
      if (L->out_scale >= 0) {  /* layer output scale (model.cpp:968-977) */
        const float os = *(const float*)tdata(m, L->out_scale);
        for (int j = 0; j < E; j++) hs[t * E + j] *= os;
      }
    }
  }
  if (rc == 0) {  /* final norm on last token + logits (model.cpp:983-1041) */
    norm_w(m, m->out_norm, hs + (size_t)(T - 1) * E, xn, E);
    rc = orc_mat_vec_mul(te->type, tdata(m, m->tok_embd), te->shape[1], te->shape[0], xn, logits, m->n_threads);
    if (rc == 0 && m->final_softcap > 0.0f)
      for (int i = 0; i < m->vocab; i++) logits[i] = m->final_softcap * tanhf(logits[i] / m->final_softcap);
  }
  free(hs); free(xn); free(qv); free(kv); free(vv); free(att); free(tmp); free(g); free(u); free(hb); free(inp_pl);
  return rc;
}
