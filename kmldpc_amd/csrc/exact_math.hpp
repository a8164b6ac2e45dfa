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
//   kml_cmul   — std::complex<double> operator* as GCC expands it without
//                -ffast-math: (ac - bd, ad + bc); the __muldc3 fallback is
//                reached only when both parts are NaN.
//
// Everything here uses only IEEE-754 basic operations and sqrt, which are
// correctly rounded on gfx950 and on x86-64, so host and device produce the
// same bits.  Compile with -ffp-contract=off.
#pragma once

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define KML_HD __host__ __device__ __forceinline__
#else
#define KML_HD inline
#endif

#include <cmath>
#include <cstdint>

namespace kml {

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
  h -= (t1 + t2) / (2.0 * h);
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
    ratio = c / d;
    denom = (c * ratio) + d;
    if (fabs(ratio) > RMIN) {
      x = ((a * ratio) + b) / denom;
      y = ((b * ratio) - a) / denom;
    } else {
      x = ((c * (a / d)) + b) / denom;
      y = ((c * (b / d)) - a) / denom;
    }
  } else {
    ratio = d / c;
    denom = (d * ratio) + c;
    if (fabs(ratio) > RMIN) {
      x = ((b * ratio) + a) / denom;
      y = (b - (a * ratio)) / denom;
    } else {
      x = (a + (d * (b / c))) / denom;
      y = (b - (d * (a / c))) / denom;
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

KML_HD cplx kml_cmul(cplx a, cplx b) { return cplx{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }

}  // namespace kml
