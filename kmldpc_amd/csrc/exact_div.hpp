// exact_div.hpp — correctly rounded double division on gfx950.
//
// The reference divides with x86-64 `divsd`: RN(n / s) for every operand pair.
// gfx950 has no f64 divide instruction, and hipcc's f64 '/' (v_div_scale,
// v_rcp_f64, two Newton steps, the Markstein tail, v_div_fmas, v_div_fixup) is
// NOT correctly rounded everywhere: its refined reciprocal is one ulp low for
// s = 1 - k 2^-53 (k = 3, 5, ..., 13), and e.g. 0x1.6666666666663p-1 /
// 0x1.ffffffffffffbp-1 comes out one ulp low (tools/probe/cn_div_candidates.py,
// tests/test_gpu_parity.py::test_exact_division_*).  Everything here is
// provably RN(n / s).
//
// 1. dd_quot + dd_check (the decoders' FAST VN divisions, demap_common.hpp):
//    y0 = v_rcp_f64(s), whose relative error e0 the ISA documents as at most
//    2^29 ulp = 2^-23 (tests/test_gpu_parity.py::test_hardware_reciprocal_error
//    measures it on the device).  Shipped form (KML_DD_NEWTON = 1): one Newton
//    step y1 = y0 + y0 RN(1 - s y0), e1 = RN(1 - s y1) (fma), |e1| <= e0^2 +
//    2^-53 < 2^-45, hi = y1, ylo = RN(e1 y1), yk = RN(y1 (1 + 2^-40)).
//    y1 + e1 y1 = (1 - e1^2) / s.  Alternative (KML_DD_NEWTON = 0, one
//    instruction less per pair but measured 2.7 % slower on the headline BP
//    kernel: its yk waits on ylo): hi = y0, e = RN(1 - s y0),
//    ylo = RN(y0 RN(e + e^2)), yk = RN(y0 (1 + 2^-40) + ylo); y0 (1 + e* + e*^2)
//    = (1 - e*^3) / s.  Either way y0 + ylo (resp. y1 + ylo) is within 2^-67 of
//    1/s, and
//        q = fma(n, hi, RN(n ylo))
//    rounds a value within 2^-66 relative of n/s once: q is a FAITHFUL
//    rounding of n/s (one of its two neighbours).  Premise: e0 <= 2^-23 (the
//    ISA's bound, which test_hardware_reciprocal_error asserts on the device
//    and tests/test_division_model.py replays adversarially as +-2^-23 in
//    exact rational arithmetic, both forms).  The argument itself has slack:
//    the Newton form needs e0 <= 2^-20.1 (F > 1 below needs |e1| < 2^-40.2),
//    the Newton-free form e0 <= 2^-22.3 (its e*^3 <= 2^-67).
//    The check: r = fma(-q, s, n) is exact (q faithful; n = 0 or n >= 2^-969,
//    s and q normal), r = s (n/s - q).  With yk as above,
//        t = fma(r, yk, q) = RN(q + (n/s - q) F),  F = s yk = (1 + d)(1 + 2^-40) + eps',
//    |eps'| <= 2^-52, so 1 < F < 1 + 2^-39 (the fma forms r yk exactly, and t
//    rounds once).  If q != RN(n/s),
//    |n/s - q| exceeds half the gap g between q and its neighbour towards n/s
//    (g = ulp(q), or ulp(q)/2 below a power of two; n/s is never exactly a
//    midpoint: s times a 54-bit odd significand has more than 53 bits), so
//    q + (n/s - q) F lies strictly beyond that midpoint and t != q.
//    Contrapositive: t == q proves q == RN(n/s).  A correct q is flagged only
//    when n/s lies within 2^-39 of half a gap from the midpoint.  BP's
//    saturated messages make such quotients recur (e.g. n0 = 1/4 + 3 ulp,
//    s = 1/2 - 2^-55: n/s within 2^-50 of a midpoint, measured by
//    tools/div_stats.py), so the decoders settle a flagged quotient in place
//    with dd_fix (q faithful: RN(n/s) is q or its neighbour, told apart by
//    their exact residuals) instead of redoing the codeword; the demapper
//    reruns the symbol on the exact path.
//    Cost per normalisation pair: v_rcp_f64 + 5 shared (4 without the Newton
//    step) + 5 per quotient (+ the fix, rare).
//
// 2. div_rn (every other division: the decoders' exact re-decode, the
//    non-FAST demap, k-means): any operands.  Finite normal operands with
//    2^-969 <= |n| < 2^1000, 2^-1000 <= |s| < 2^1000 and a normal quotient:
//    q from dd_quot (faithful, above), r = fma(-q, s, n) exact, and q is
//    replaced by its neighbour qn towards n/s when |fma(-qn, s, n)| < |r|
//    (both residuals exact, |residual| = |s| * distance to n/s; no ties).
//    Zeros, infinities and NaNs: hipcc's '/' (its special-case handling is
//    IEEE-754's, and the NaN payloads are the ones the parity tests pinned).
//    Other finite nonzero operands (subnormal or extreme): div_soft, an
//    integer long division of the significands with round-to-nearest-even
//    onto the normal or subnormal grid.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace kml {

// The double-double reciprocal and the proof's scaled reciprocal:
//   KML_DD_NEWTON = 1 (shipped): hi = y1 = y0 + y0 RN(1 - s y0), lo = RN(e1 y1)
//                                with e1 = RN(1 - s y1), k = RN(y1 (1 + 2^-40));
//   KML_DD_NEWTON = 0:           hi = y0, lo = RN(y0 RN(e + e^2)) with
//                                e = RN(1 - s y0), k = RN(y0 (1 + 2^-40) + lo).
struct DdRcp {
  double hi, lo, k;
};

#ifndef KML_DD_NEWTON
#define KML_DD_NEWTON 1
#endif
__device__ __forceinline__ DdRcp dd_rcp(double s) {
  const double y0 = __builtin_amdgcn_rcp(s);
#if KML_DD_NEWTON  // (A/B) round 3's first form: one Newton step, y1 + RN(e1 y1), yk = RN(y1 (1 + 2^-40))
  const double y1 = fma(y0, fma(-y0, s, 1.0), y0);
  const double e1 = fma(-y1, s, 1.0);
  return {y1, e1 * y1, y1 * (1.0 + 0x1p-40)};
#else
  const double e = fma(-y0, s, 1.0);
  const double lo = y0 * fma(e, e, e);
  return {y0, lo, fma(y0, 1.0 + 0x1p-40, lo)};
#endif
}

__device__ __forceinline__ double dd_quot(double n, const DdRcp &y) { return fma(n, y.hi, n * y.lo); }

// true when q == RN(n / s) is proven (see 1. above)
__device__ __forceinline__ bool dd_check(double n, double s, double q, const DdRcp &y) {
  return fma(fma(-q, s, n), y.k, q) == q;
}

// RN(n / s) from a faithful q that dd_check could not prove: q or its
// neighbour towards n / s, whichever has the smaller residual (both residuals
// exact in dd_check's domain, |residual| = |s| * distance to n / s; no ties).
__device__ __forceinline__ double dd_fix(double n, double s, double q) {
  const double r = fma(-q, s, n);
  const long long step = ((r > 0.0) == (s > 0.0)) == (q > 0.0) ? 1 : -1;
  const double qn = __longlong_as_double(__double_as_longlong(q) + step);
  return fabs(fma(-qn, s, n)) < fabs(r) ? qn : q;
}

// Integer long division for finite nonzero n, s (any magnitude): RN(n / s).
__device__ __forceinline__ double div_soft(double n, double s) {
  const uint64_t bn = (uint64_t)__double_as_longlong(n), bs = (uint64_t)__double_as_longlong(s);
  const uint64_t sign = (bn ^ bs) & 0x8000000000000000ull;
  constexpr uint64_t kMant = (1ull << 52) - 1;
  int en = (int)((bn >> 52) & 0x7FF), es = (int)((bs >> 52) & 0x7FF);
  uint64_t mn = bn & kMant, ms = bs & kMant;
  // value = m * 2^(e - 1075) with m in [2^52, 2^53) after normalisation
  if (en) mn |= 1ull << 52; else en = 1;
  if (es) ms |= 1ull << 52; else es = 1;
  {
    const int zn = __clzll((long long)mn) - 11, zs = __clzll((long long)ms) - 11;
    mn <<= zn;
    en -= zn;
    ms <<= zs;
    es -= zs;
  }
  int e = en - es;  // n / s = (mn / ms) 2^e
  if (mn < ms) {
    mn <<= 1;
    --e;
  }
  // Q = floor((mn / ms) 2^53) in [2^53, 2^54), sticky = remainder != 0
  uint64_t Q = 0, rem = mn;
  for (int i = 0; i < 54; ++i) {
    const bool ge = rem >= ms;
    Q = (Q << 1) | (ge ? 1ull : 0ull);
    if (ge) rem -= ms;
    rem <<= 1;
  }
  const bool sticky = rem != 0;
  uint64_t out;
  if (e >= -1022) {  // normal: significand Q >> 1, round bit Q & 1
    uint64_t S = Q >> 1;
    if ((Q & 1) && (sticky || (S & 1))) ++S;
    if (S >> 53) {
      S >>= 1;
      ++e;
    }
    if (e > 1023) return __longlong_as_double((long long)(sign | 0x7FF0000000000000ull));
    out = ((uint64_t)(e + 1023) << 52) | (S & kMant);
  } else {  // subnormal grid 2^-1074: N = (mn / ms) 2^(e + 1074) = Q 2^(e + 1021)
    const int sh = -(e + 1021);  // >= 2
    if (sh > 55) {
      out = 0;  // below half the smallest subnormal
    } else {
      const uint64_t N = Q >> sh;
      const bool rbit = (Q >> (sh - 1)) & 1;
      const bool st = sticky || (Q & ((1ull << (sh - 1)) - 1)) != 0;
      out = N + ((rbit && (st || (N & 1))) ? 1 : 0);  // may carry into the smallest normal
    }
  }
  return __longlong_as_double((long long)(sign | out));
}

// RN(n / s) outside div_rn's fast domain: zeros, infinities and NaNs (IEEE
// cases: hipcc's '/'), else the integer long division.
__device__ __forceinline__ double div_rn_rare(double n, double s) {
  const double an = fabs(n), as = fabs(s);
  if (!(an > 0.0) || !(as > 0.0) || an == INFINITY || as == INFINITY) return n / s;  // 0, inf, NaN: IEEE cases
  return div_soft(n, s);
}
// Out of line: inlined at every division site of the exact kernels it
// multiplied their code size past the instruction cache.
__device__ __noinline__ double div_rn_cold(double n, double s) { return div_rn_rare(n, s); }

// RN(n / s) for any operands (see 2. above).  INLINE_RARE: the rare path
// inline too (a kernel with few division sites, where a call's register
// convention would cost more than the code: k-means).
template <bool INLINE_RARE = false>
__device__ __forceinline__ double div_rn(double n, double s) {
  const double an = fabs(n), as = fabs(s);
  if (__builtin_expect((an >= 0x1p-969) & (an < 0x1p1000) & (as >= 0x1p-1000) & (as < 0x1p1000), 1)) {
    const DdRcp y = dd_rcp(s);
    double q = dd_quot(n, y);
    const double aq = fabs(q);
    if (__builtin_expect((aq >= 0x1p-1020) & (aq < 0x1p1020), 1)) {
      // the neighbour of q towards n / s (whose sign is r's times s's): an
      // exact residual of 0 keeps q (|fma(-qn, s, n)| > 0)
      const double r = fma(-q, s, n);
      const long long step = ((r > 0.0) == (s > 0.0)) == (q > 0.0) ? 1 : -1;
      const double qn = __longlong_as_double(__double_as_longlong(q) + step);
      return fabs(fma(-qn, s, n)) < fabs(r) ? qn : q;
    }
  }
  if constexpr (INLINE_RARE) return div_rn_rare(n, s);
  else return div_rn_cold(n, s);
}

// div_rn with the divisor's reciprocal taken by the caller (y = dd_rcp(s),
// e.g. once for several quotients by one divisor, or ahead of the numerator):
// the same operations on the same values.
template <bool INLINE_RARE = false>
__device__ __forceinline__ double div_rn_y(double n, double s, const DdRcp &y) {
  const double an = fabs(n), as = fabs(s);
  if (__builtin_expect((an >= 0x1p-969) & (an < 0x1p1000) & (as >= 0x1p-1000) & (as < 0x1p1000), 1)) {
    double q = dd_quot(n, y);
    const double aq = fabs(q);
    if (__builtin_expect((aq >= 0x1p-1020) & (aq < 0x1p1020), 1)) {
      const double r = fma(-q, s, n);
      const long long step = ((r > 0.0) == (s > 0.0)) == (q > 0.0) ? 1 : -1;
      const double qn = __longlong_as_double(__double_as_longlong(q) + step);
      return fabs(fma(-qn, s, n)) < fabs(r) ? qn : q;
    }
  }
  if constexpr (INLINE_RARE) return div_rn_rare(n, s);
  else return div_rn_cold(n, s);
}

}  // namespace kml
