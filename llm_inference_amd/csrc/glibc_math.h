// glibc_math.h -- bit-exact device restatements of the two libm functions the
// reference's decode arithmetic calls per element: expf (attention softmax,
// model.cpp:510-521) and tanhf (GELU, model.cpp:892-899).
//
// The reference is linked against the host's glibc 2.35 libm (Ubuntu 22.04,
// the image both the build container and the GPU box run).  expf is an ifunc
// whose FMA variant runs on every AVX2+FMA host (__expf_fma: the
// exp2f-table algorithm with fused multiply-adds, read off its disassembly);
// tanhf / expm1f are the plain SSE fdlibm code (no contraction).  The
// constants below are the ones in that libm's .rodata (address-for-address
// checked with llvm-objdump), and tests/test_glibc_math.py compares these
// functions, compiled for the host with the same source, against the host's
// libm over every float in the ranges the model can produce.  Only exact mode
// (LLMI_EXACT) uses them; the fast kernels keep the device intrinsics.
#pragma once

#include <stdint.h>
#include <string.h>

#if defined(__HIPCC__)
#define LLMI_HD __host__ __device__ __forceinline__
#else
#define LLMI_HD static inline
#endif

namespace llmi_glibc {

LLMI_HD uint32_t fbits(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
}
LLMI_HD float bitsf(uint32_t u) {
  float f;
  memcpy(&f, &u, 4);
  return f;
}
LLMI_HD double bitsd(uint64_t u) {
  double d;
  memcpy(&d, &u, 8);
  return d;
}
LLMI_HD uint64_t dbits(double d) {
  uint64_t u;
  memcpy(&u, &d, 8);
  return u;
}

// __exp2f_data.tab: bits of 2^(i/32) minus i << 47 (glibc e_exp2f_data.c)
#define LLMI_EXP2F_TAB                                                                            \
  {0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull, \
   0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull, \
   0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull, \
   0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull, \
   0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull, \
   0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull, \
   0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull, \
   0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull}
#if defined(__HIPCC__)
__device__ __constant__ static const uint64_t kExp2fTabDev[32] = LLMI_EXP2F_TAB;
#endif
static const uint64_t kExp2fTabHost[32] = LLMI_EXP2F_TAB;
#undef LLMI_EXP2F_TAB

LLMI_HD uint64_t exp2f_tab(int i) {
#if defined(__HIP_DEVICE_COMPILE__)
  return kExp2fTabDev[i];
#else
  return kExp2fTabHost[i];
#endif
}

// glibc 2.35 __expf_fma (sysdeps/ieee754/flt-32/e_expf.c built with -mfma):
//   kd = fma(InvLn2N, x, SHIFT); ki = bits(kd); kd -= SHIFT;
//   r = fma(InvLn2N, x, -kd); s = double(tab[ki % 32] + (ki << 47));
//   y = fma(fma(C0, r, C1), r*r, fma(C2, r, 1)) * s;  return (float)y
// (tab: the 32 entries of exp2f_tab, e.g. staged in LDS by a kernel that calls this per element)
LLMI_HD float expf_tab(float x, const uint64_t* tab) {
  const uint32_t abstop = (fbits(x) >> 20) & 0x7ff;
  if (abstop > 0x42a) {                             // |x| >= 88 or NaN (top12(88.0f) = 0x42b)
    if (fbits(x) == 0xff800000u) return 0.0f;       // -inf
    if (abstop > 0x7f7) return x + x;               // +inf / NaN
    if (x > bitsf(0x42b17217u)) return bitsf(0x7f800000u);  // overflow (x > 0x1.62e42ep6)
    if (x < bitsf(0xc2cff1b4u)) return 0.0f;        // underflow (x < -0x1.9fe368p6)
    if (x < bitsf(0xc2ce8ecfu)) return bitsf(0x00000001u);  // __math_may_uflowf: 0x1.4p-75f squared = 2^-149
  }
  const double InvLn2N = bitsd(0x40471547652b82feull);  // 0x1.71547652b82fep+5
  const double SHIFT = bitsd(0x4338000000000000ull);    // 0x1.8p+52
  const double C0 = bitsd(0x3ebc6af84b912394ull);       // 0x1.c6af84b912394p-20
  const double C1 = bitsd(0x3f2ebfce50fac4f3ull);       // 0x1.ebfce50fac4f3p-13
  const double C2 = bitsd(0x3f962e42ff0c52d6ull);       // 0x1.62e42ff0c52d6p-6
  const double xd = (double)x;
  double kd = __builtin_fma(InvLn2N, xd, SHIFT);
  const uint64_t ki = dbits(kd);
  kd -= SHIFT;
  const double r = __builtin_fma(InvLn2N, xd, -kd);
  const uint64_t t = tab[ki & 31] + (ki << 47);
  const double s = bitsd(t);
  const double z = __builtin_fma(C0, r, C1);
  const double r2 = r * r;
  const double y1 = __builtin_fma(C2, r, 1.0);
  const double y = __builtin_fma(z, r2, y1) * s;
  return (float)y;
}
LLMI_HD float expf(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return expf_tab(x, kExp2fTabDev);
#else
  return expf_tab(x, kExp2fTabHost);
#endif
}

// glibc 2.35 __expm1f (sysdeps/ieee754/flt-32/s_expm1f.c, fdlibm; SSE, no FMA)
LLMI_HD float expm1f(float x) {
  const float one = 1.0f, huge = bitsf(0x7149f2cau), tiny = bitsf(0x0da24260u);
  const float o_threshold = bitsf(0x42b17180u), ln2_hi = bitsf(0x3f317180u), ln2_lo = bitsf(0x3717f7d1u),
              invln2 = bitsf(0x3fb8aa3bu);
  const float Q1 = bitsf(0xbd088889u), Q2 = bitsf(0x3ad00d01u), Q3 = bitsf(0xb8a670cdu), Q4 = bitsf(0x36867e54u),
              Q5 = bitsf(0xb457edbbu);
  uint32_t hx = fbits(x);
  const uint32_t xsb = hx & 0x80000000u;
  hx &= 0x7fffffffu;
  float hi, lo, c = 0.0f, t, e, y;
  int k;
  if (hx >= 0x4195b844u) {  // |x| >= 27 ln2
    if (hx >= 0x42b17218u) {
      if (hx > 0x7f800000u) return x + x;
      if (hx == 0x7f800000u) return xsb == 0 ? x : -1.0f;
      if (x > o_threshold) return huge * huge;
    }
    if (xsb != 0) return tiny - one;
  }
  if (hx > 0x3eb17218u) {      // |x| > 0.5 ln2
    if (hx < 0x3f851592u) {    // and |x| < 1.5 ln2
      if (xsb == 0) {
        hi = x - ln2_hi;
        lo = ln2_lo;
        k = 1;
      } else {
        hi = x + ln2_hi;
        lo = -ln2_lo;
        k = -1;
      }
    } else {
      k = (int)(invln2 * x + (xsb == 0 ? 0.5f : -0.5f));
      t = (float)k;
      hi = x - t * ln2_hi;
      lo = t * ln2_lo;
    }
    x = hi - lo;
    c = (hi - x) - lo;
  } else if (hx < 0x33000000u) {  // |x| < 2^-25
    return x;
  } else {
    k = 0;
  }
  const float hfx = 0.5f * x;
  const float hxs = x * hfx;
  const float r1 = one + hxs * (Q1 + hxs * (Q2 + hxs * (Q3 + hxs * (Q4 + hxs * Q5))));
  t = 3.0f - r1 * hfx;
  e = hxs * ((r1 - t) / (6.0f - x * t));
  if (k == 0) return x - (x * e - hxs);
  e = x * (e - c) - c;
  e -= hxs;
  if (k == -1) return 0.5f * (x - e) - 0.5f;
  if (k == 1) {
    if (x < -0.25f) return -2.0f * (e - (x + 0.5f));
    return one + 2.0f * (x - e);
  }
  if (k <= -2 || k > 56) {  // exp(x) - 1 ~ exp(x)
    y = one - (e - x);
    y = bitsf(fbits(y) + ((uint32_t)k << 23));
    return y - one;
  }
  if (k < 23) {
    t = bitsf(0x3f800000u - (0x1000000u >> k));  // 1 - 2^-k
    y = t - (e - x);
  } else {
    t = bitsf((uint32_t)(0x7f - k) << 23);  // 2^-k
    y = x - (e + t);
    y += one;
  }
  return bitsf(fbits(y) + ((uint32_t)k << 23));
}

// glibc 2.35 __tanhf (sysdeps/ieee754/flt-32/s_tanhf.c, fdlibm)
LLMI_HD float tanhf(float x) {
  const uint32_t jx = fbits(x), ix = jx & 0x7fffffffu;
  if (ix > 0x7f7fffffu) return (jx >> 31) == 0 ? 1.0f / x + 1.0f : 1.0f / x - 1.0f;
  float z;
  if (ix < 0x41b00000u) {     // |x| < 22
    if (ix == 0) return x;
    if (ix < 0x24000000u) return x * (1.0f + x);  // |x| < 2^-55
    const float ax = bitsf(ix);
    if (ix >= 0x3f800000u) {  // |x| >= 1
      const float t = expm1f(ax + ax);
      z = 1.0f - 2.0f / (t + 2.0f);
    } else {
      const float t = expm1f(-2.0f * ax);
      z = -t / (t + 2.0f);
    }
  } else {
    z = 1.0f - bitsf(0x0da24260u);  // 1 - tiny
  }
  return (jx >> 31) == 0 ? z : -z;
}

// the attention logit soft-cap (model.cpp:511-513): the double score over the float cap is a double division,
// tanhf takes its float rounding, and the float product cap * tanhf(...) goes back into the double
LLMI_HD double softcap_score(double score, float cap) { return (double)(cap * tanhf((float)(score / (double)cap))); }

}  // namespace llmi_glibc
