// exact_math.hpp — IEEE-exact restatements of the three libm/libgcc routines the
// reference's hot path calls with non-basic arithmetic, for use in gfx950
// device code (and compiled on the host by the CPU tests to pin them).
//
//   kml_hypot  — |z| as computed by std::abs(std::complex<double>) -> cabs ->
//                glibc 2.35 hypot (sysdeps/ieee754/dbl-64/e_hypot.c, the
//                non-FMA kernel of Borges' "An Improved Algorithm for
//                hypot(a,b)", MyHypot3 with a one-step correction).  Used by
//                KMeans::Run (src/kmeans.cc:18, :53, :76).
//   kml_cdiv   — complex division as std::complex<double> operator/ lowers to
//                libgcc __divdc3: Smith's algorithm (scale by the larger of
//                |c|,|d|), with the libgcc-12 alternative ordering when the
//                ratio is subnormal.  Used by src/kmeans.cc:25, :59-62, :66 and
//                src/simulator.cc:145.  The RMIN/RBIG pre-scalings of libgcc
//                multiply every operand by the same power of two and therefore
//                do not change the quotient for the finite, non-extreme values
//                this path divides (cluster sums, received symbols,
//                constellation points).
//   kml_exp    — glibc >= 2.28 exp (sysdeps/ieee754/dbl-64/e_exp.c, the
//                table-driven algorithm of ARM optimized-routines: N = 128,
//                degree-5 polynomial), in the contraction pattern of the x86-64
//                FMA ifunc variant (__exp_fma) that glibc selects on every
//                FMA-capable host — the one the reference's demapper calls
//                (lib/lab/src/modemlinearsystem.cc:61).  The 2^(k/128) table is
//                regenerated from first principles (tools/gen_exp_table.py).
//   kml_log    — glibc >= 2.28 log (sysdeps/ieee754/dbl-64/e_log.c, ARM
//                optimized-routines: N = 128 table, degree-6 polynomial, a
//                degree-12 one near 1), again in the contraction pattern of the
//                FMA ifunc variant (__log_fma).  Used by the soft syndrome
//                metric (src/kmcodec.cc:155).  Table from tools/gen_log_table.py.
//   kml_cmul   — std::complex<double> operator* as GCC expands it without
//                -ffast-math: (ac - bd, ad + bc), and libgcc __muldc3's
//                recovery of infinities when both parts are NaN.
//
// Everything here uses only IEEE-754 basic operations and sqrt, which are
// correctly rounded on x86-64 and, on gfx950, through kml_div (division;
// hipcc's '/' is not correctly rounded everywhere, exact_div.hpp) and the
// hardware's add/mul/fma/sqrt, so host and device produce the same bits.
// Divisions by powers of two are exact either way and keep '/'.  Compile
// with -ffp-contract=off.
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define KML_HD __host__ __device__ __forceinline__
#define KML_HD_COLD static __host__ __device__ __noinline__
#else
#define KML_HD inline
#define KML_HD_COLD static inline
#endif

#include <cmath>
#include <cstdint>

#include "exp_table.hpp"
#include "log_table.hpp"
#if defined(__HIPCC__)
#include "exact_div.hpp"
#endif

namespace kml {

// RN(a / b): the host's IEEE division, and on the device exact_div.hpp div_rn
// (hipcc's f64 '/' is not correctly rounded everywhere), its rare path inline
// (k-means: few division sites, and a call would raise its registers).
KML_HD double kml_div(double a, double b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return div_rn<true>(a, b);
#else
  return a / b;
#endif
}

struct cplx {
  double re, im;
};

KML_HD double hypot_kernel(double ax, double ay) {
  // requires ax >= ay >= 0 and no overflow/underflow when squaring
  double h = sqrt(ax * ax + ay * ay);
  double t1, t2;
  if (h <= 2.0 * ay) {
    double delta = h - ay;
    t1 = ax * (2.0 * delta - ax);
    t2 = (delta - 2.0 * (ax - ay)) * delta;
  } else {
    double delta = h - ax;
    t1 = 2.0 * delta * (ax - 2.0 * ay);
    t2 = (4.0 * delta - ay) * ay + delta * delta;
  }
  h -= kml_div(t1 + t2, 2.0 * h);
  return h;
}

KML_HD double kml_hypot(double x, double y) {
  const double SCALE = 0x1p-600;
  const double LARGE_VAL = 0x1p+511;
  const double TINY_VAL = 0x1p-511;
  const double EPS = 0x1p-54;
  if (!std::isfinite(x) || !std::isfinite(y)) {
    if (std::isinf(x) || std::isinf(y)) return INFINITY;
    return x + y;
  }
  x = fabs(x);
  y = fabs(y);
  double ax = x < y ? y : x;
  double ay = x < y ? x : y;
  if (ax > LARGE_VAL) {
    if (ay <= ax * EPS) return ax + ay;
    return hypot_kernel(ax * SCALE, ay * SCALE) / SCALE;
  }
  if (ay < TINY_VAL) {
    if (ax >= ay / EPS) return ax + ay;
    return hypot_kernel(ax / SCALE, ay / SCALE) * SCALE;
  }
  if (ay <= ax * EPS) return ax + ay;
  return hypot_kernel(ax, ay);
}

KML_HD cplx kml_cdiv(cplx n, cplx dd) {
  const double a = n.re, b = n.im, c = dd.re, d = dd.im;
  const double RMIN = 2.2250738585072014e-308;  // DBL_MIN
  double denom, ratio, x, y;
  if (fabs(c) < fabs(d)) {
    ratio = kml_div(c, d);
    denom = (c * ratio) + d;
    if (fabs(ratio) > RMIN) {
      x = kml_div((a * ratio) + b, denom);
      y = kml_div((b * ratio) - a, denom);
    } else {
      x = kml_div((c * kml_div(a, d)) + b, denom);
      y = kml_div((c * kml_div(b, d)) - a, denom);
    }
  } else {
    ratio = kml_div(d, c);
    denom = (d * ratio) + c;
    if (fabs(ratio) > RMIN) {
      x = kml_div((b * ratio) + a, denom);
      y = kml_div(b - (a * ratio), denom);
    } else {
      x = kml_div(a + (d * kml_div(b, c)), denom);
      y = kml_div(b - (d * kml_div(a, c)), denom);
    }
  }
  // C99 Annex G recovery of infinities and zeros (what __divdc3 does when
  // both parts came out NaN), e.g. a cluster sum divided by a zero count.
  if (std::isnan(x) && std::isnan(y)) {
    if (c == 0.0 && d == 0.0 && (!std::isnan(a) || !std::isnan(b))) {
      x = copysign(INFINITY, c) * a;
      y = copysign(INFINITY, c) * b;
    } else if ((std::isinf(a) || std::isinf(b)) && std::isfinite(c) && std::isfinite(d)) {
      const double a1 = copysign(std::isinf(a) ? 1.0 : 0.0, a);
      const double b1 = copysign(std::isinf(b) ? 1.0 : 0.0, b);
      x = INFINITY * (a1 * c + b1 * d);
      y = INFINITY * (b1 * c - a1 * d);
    } else if ((std::isinf(c) || std::isinf(d)) && std::isfinite(a) && std::isfinite(b)) {
      const double c1 = copysign(std::isinf(c) ? 1.0 : 0.0, c);
      const double d1 = copysign(std::isinf(d) ? 1.0 : 0.0, d);
      x = 0.0 * (a * c1 + b * d1);
      y = 0.0 * (b * c1 - a * d1);
    }
  }
  return cplx{x, y};
}

KML_HD uint64_t as_u64(double x) { return __builtin_bit_cast(uint64_t, x); }
KML_HD double as_f64(uint64_t x) { return __builtin_bit_cast(double, x); }

KML_HD uint64_t exp_tab(int i) {
#if defined(__HIP_DEVICE_COMPILE__)
  return kExpTabDev[i];
#else
  return kExpTabHost[i];
#endif
}

// FMA selects the contraction pattern of the FMA-compiled glibc variant.
template <bool FMA>
KML_HD double exp_special(double tmp, uint64_t sbits, uint64_t ki) {
  double scale, y;
  if ((ki & 0x80000000) == 0) {  // k > 0: the exponent of scale may have overflowed by <= 460
    sbits -= 1009ull << 52;
    scale = as_f64(sbits);
    y = 0x1p1009 * (FMA ? fma(scale, tmp, scale) : scale + scale * tmp);
    return y;
  }
  sbits += 1022ull << 52;  // k < 0: careful rounding into the subnormal range
  scale = as_f64(sbits);
  // scale*tmp has two uses here and is not fused in the FMA build
  const double st = scale * tmp;
  y = scale + st;
  if (y < 1.0) {
    double hi, lo;
    lo = scale - y + st;
    hi = 1.0 + y;
    lo = 1.0 - hi + y + lo;
    y = (hi + lo) - 1.0;
    if (y == 0.0) y = 0.0;
  }
  return 0x1p-1022 * y;
}

template <bool FMA>
KML_HD double kml_exp_t(double x) {
  const double InvLn2N = 0x1.71547652b82fep0 * 128;
  const double Shift = 0x1.8p52;
  const double NegLn2hiN = -0x1.62e42fefa0000p-8;
  const double NegLn2loN = -0x1.cf79abc9e3b3ap-47;
  const double C2 = 0x1.ffffffffffdbdp-2, C3 = 0x1.555555555543cp-3;
  const double C4 = 0x1.55555cf172b91p-5, C5 = 0x1.1111167a4d017p-7;
  const uint32_t top_tiny = (uint32_t)(as_u64(0x1p-54) >> 52);
  const uint32_t top_512 = (uint32_t)(as_u64(512.0) >> 52);
  const uint32_t top_1024 = (uint32_t)(as_u64(1024.0) >> 52);
  const uint32_t top_inf = (uint32_t)(as_u64(INFINITY) >> 52);
  uint32_t abstop = (uint32_t)(as_u64(x) >> 52) & 0x7ff;
  if (abstop - top_tiny >= top_512 - top_tiny) {
    if (abstop - top_tiny >= 0x80000000u) return 1.0 + x;  // tiny |x| (incl. 0)
    if (abstop >= top_1024) {
      if (as_u64(x) == as_u64(-INFINITY)) return 0.0;
      if (abstop >= top_inf) return 1.0 + x;
      if (as_u64(x) >> 63) return 0x1p-767 * 0x1p-767;  // underflow
      return 0x1p769 * 0x1p769;                          // overflow
    }
    abstop = 0;  // large |x|: special-cased below
  }
  double kd = FMA ? fma(InvLn2N, x, Shift) : InvLn2N * x + Shift;
  const uint64_t ki = as_u64(kd);
  kd -= Shift;
  const double r = FMA ? fma(kd, NegLn2loN, fma(kd, NegLn2hiN, x)) : x + kd * NegLn2hiN + kd * NegLn2loN;
  const int idx = (int)(2 * (ki % 128));
  const uint64_t top = ki << (52 - 7);
  const double tail = as_f64(exp_tab(idx));
  const uint64_t sbits = exp_tab(idx + 1) + top;
  const double r2 = r * r;
  double tmp;
  if (FMA)
    tmp = fma(r2 * r2, fma(r, C5, C4), fma(r2, fma(r, C3, C2), tail + r));
  else
    tmp = tail + r + r2 * (C2 + r * C3) + r2 * r2 * (C4 + r * C5);
  if (abstop == 0) return exp_special<FMA>(tmp, sbits, ki);
  const double scale = as_f64(sbits);
  return FMA ? fma(scale, tmp, scale) : scale + scale * tmp;
}

KML_HD double kml_exp(double x) { return kml_exp_t<true>(x); }

KML_HD double log_tab(int i) {
#if defined(__HIP_DEVICE_COMPILE__)
  return as_f64(kLogTabDev[i]);
#else
  return as_f64(kLogTabHost[i]);
#endif
}

template <bool FMA>
KML_HD double kml_log_t(double x) {
  const double A[5] = {KML_LOG_POLY_INIT};
  const double B[11] = {KML_LOG_POLY1_INIT};
  const double Ln2hi = 0x1.62e42fefa3800p-1, Ln2lo = 0x1.ef35793c76730p-45;
  const uint64_t OFF = 0x3fe6000000000000ull;
  uint64_t ix = as_u64(x);
  const uint32_t top = (uint32_t)(ix >> 48);
  const uint64_t LO = as_u64(1.0 - 0x1p-4), HI = as_u64(1.0 + 0x1.09p-4);
  if (ix - LO < HI - LO) {  // close to 1
    if (ix == as_u64(1.0)) return 0.0;
    const double r = x - 1.0;
    const double r2 = r * r;
    const double r3 = r * r2;
    double p;  // y = r3 * p
    if (FMA) {
      const double p3 = fma(r3, B[10], fma(r2, B[9], fma(r, B[8], B[7])));
      const double p2 = fma(r3, p3, fma(r2, B[6], fma(r, B[5], B[4])));
      p = fma(r3, p2, fma(r2, B[3], fma(r, B[2], B[1])));
    } else {
      p = B[1] + r * B[2] + r2 * B[3] + r3 * (B[4] + r * B[5] + r2 * B[6] + r3 * (B[7] + r * B[8] + r2 * B[9] + r3 * B[10]));
    }
    double w = r * 0x1p27;
    const double rhi = r + w - w;
    const double rlo = r - rhi;
    w = rhi * rhi * B[0];
    const double hi = r + w;
    double lo = r - hi + w;
    lo = FMA ? fma(B[0] * rlo, rhi + r, lo) : lo + B[0] * rlo * (rhi + r);
    // y = r3*p; y += lo; y += hi — the FMA build fuses the first add
    const double y = FMA ? fma(r3, p, lo) : r3 * p + lo;
    return y + hi;
  }
  if (top - 0x0010 >= 0x7ff0 - 0x0010) {
    if (ix * 2 == 0) return -1.0 / 0.0;        // log(+-0) = -inf, divide-by-zero
    if (ix == as_u64(INFINITY)) return x;    // log(inf) = inf
    if ((top & 0x8000) || (top & 0x7ff0) == 0x7ff0) return (x - x) / (x - x);  // negative or NaN
    ix = as_u64(x * 0x1p52);                 // subnormal: normalise
    ix -= 52ull << 52;
  }
  const uint64_t tmp = ix - OFF;
  const int i = (int)((tmp >> (52 - 7)) % 128);
  const int k = (int)((int64_t)tmp >> 52);
  const uint64_t iz = ix - (tmp & (0xfffull << 52));
  const double invc = log_tab(4 * i), logc = log_tab(4 * i + 1);
  const double z = as_f64(iz);
  double r;
  if (FMA)
    r = fma(z, invc, -1.0);
  else
    r = (z - log_tab(4 * i + 2) - log_tab(4 * i + 3)) * invc;
  const double kd = (double)k;
  const double w = FMA ? fma(kd, Ln2hi, logc) : kd * Ln2hi + logc;
  const double hi = w + r;
  const double lo = FMA ? fma(kd, Ln2lo, w - hi + r) : w - hi + r + kd * Ln2lo;
  const double r2 = r * r;
  if (FMA) {
    const double p = fma(r2, fma(r, A[4], A[3]), fma(r, A[2], A[1]));
    return fma(r * r2, p, fma(r2, A[0], lo)) + hi;
  }
  return lo + r2 * A[0] + r * r2 * (A[1] + r * A[2] + r2 * (A[3] + r * A[4])) + hi;
}

KML_HD double kml_log(double x) { return kml_log_t<true>(x); }

// libgcc __muldc3's Annex G recovery of infinities that the naive product
// computed as NaN + i NaN (reached only then; out of line: rare)
KML_HD_COLD cplx kml_cmul_recover(double a, double b, double c, double d) {
  const double ac = a * c, bd = b * d, ad = a * d, bc = b * c;
  bool recalc = false;
  if (std::isinf(a) || std::isinf(b)) {  // the first factor is infinite: box it, NaNs of the other to 0
    a = copysign(std::isinf(a) ? 1.0 : 0.0, a);
    b = copysign(std::isinf(b) ? 1.0 : 0.0, b);
    if (std::isnan(c)) c = copysign(0.0, c);
    if (std::isnan(d)) d = copysign(0.0, d);
    recalc = true;
  }
  if (std::isinf(c) || std::isinf(d)) {  // the second factor is infinite
    c = copysign(std::isinf(c) ? 1.0 : 0.0, c);
    d = copysign(std::isinf(d) ? 1.0 : 0.0, d);
    if (std::isnan(a)) a = copysign(0.0, a);
    if (std::isnan(b)) b = copysign(0.0, b);
    recalc = true;
  }
  if (!recalc && (std::isinf(ac) || std::isinf(bd) || std::isinf(ad) || std::isinf(bc))) {  // overflow: NaNs to 0
    if (std::isnan(a)) a = copysign(0.0, a);
    if (std::isnan(b)) b = copysign(0.0, b);
    if (std::isnan(c)) c = copysign(0.0, c);
    if (std::isnan(d)) d = copysign(0.0, d);
    recalc = true;
  }
  if (!recalc) return cplx{ac - bd, ad + bc};
  return cplx{INFINITY * (a * c - b * d), INFINITY * (a * d + b * c)};
}

// std::complex<double> operator* as GCC compiles it without -ffast-math:
// (ac - bd, ad + bc), and __muldc3 when both parts are NaN.
KML_HD cplx kml_cmul(cplx a, cplx b) {
  const double x = a.re * b.re - a.im * b.im, y = a.re * b.im + a.im * b.re;
  if (std::isnan(x) && std::isnan(y)) return kml_cmul_recover(a.re, a.im, b.re, b.im);
  return cplx{x, y};
}

}  // namespace kml
