// bp_common.hpp — device helpers shared by the BP kernels.
#pragma once
#include <hip/hip_runtime.h>

#include "exact_div.hpp"

namespace kml {

constexpr double kSmallestProb = 1.0e-12;  // lib/lab/include/utility.h:12

// LDS accesses through precomputed 32-bit LDS addresses.  `smem + off` with a
// runtime `off` makes hipcc emit a v_add_u32 of the dynamic-LDS base before
// every ds_read / ds_write (it does not fold the base into the offset field);
// a kernel that keeps absolute LDS addresses in its registers addresses with
// the register directly.
typedef __attribute__((address_space(3))) unsigned char lds_byte;
typedef double dbl2 __attribute__((ext_vector_type(2)));  // 16-byte LDS slot (ds_write_b128)
__device__ __forceinline__ unsigned lds_addr(const void *p) {
  return (unsigned)(size_t)(const lds_byte *)p;
}
template <class T>
__device__ __forceinline__ T lds_ld(unsigned a) {
  return *(const __attribute__((address_space(3))) T *)(size_t)a;
}
template <class T>
__device__ __forceinline__ void lds_st(unsigned a, T v) {
  *(__attribute__((address_space(3))) T *)(size_t)a = v;
}

// Workgroup OR of a predicate with one barrier: each wave's lane 0 stores the
// wave's ballot to its own LDS word, and after the barrier every lane ORs the
// NW words (vector loads).  (__syncthreads_or goes through a two-barrier
// library reduction: ~650 more cycles per call at 12 waves.)  The words need
// no reset: a wave rewrites its word only after a later barrier that every
// reader of the previous values has passed — callers must place one between
// two calls (the BP kernels' VN-phase barrier).
template <int NW>
__device__ __forceinline__ int wg_any(int pred, int *wflags) {
  static_assert(NW % 4 == 0 && NW <= 16, "wave flags are read as int4");
  const int any = __ballot(pred) != 0;
  if ((threadIdx.x & 63) == 0) wflags[threadIdx.x >> 6] = any;
  __syncthreads();
  int r = 0;
#pragma unroll
  for (int w = 0; w < NW; w += 4) {
    const int4 v = *reinterpret_cast<const int4 *>(wflags + w);
    r |= v.x | v.y | v.z | v.w;
  }
  return r;
}

// Two workgroup ORs with one barrier (same rules as wg_any): bit 0 = OR of
// p0, bit 1 = OR of p1.
template <int NW>
__device__ __forceinline__ int wg_any2(int p0, int p1, int *wflags) {
  static_assert(NW % 4 == 0 && NW <= 16, "wave flags are read as int4");
  const int any = (__ballot(p0) != 0 ? 1 : 0) | (__ballot(p1) != 0 ? 2 : 0);
  if ((threadIdx.x & 63) == 0) wflags[threadIdx.x >> 6] = any;
  __syncthreads();
  int r = 0;
#pragma unroll
  for (int w = 0; w < NW; w += 4) {
    const int4 v = *reinterpret_cast<const int4 *>(wflags + w);
    r |= v.x | v.y | v.z | v.w;
  }
  return r;
}

template <int NW>
__device__ __forceinline__ int wg_all(int pred, int *wflags) {
  return !wg_any<NW>(!pred, wflags);
}

// hipcc's reciprocal refinement of an f64 '/': v_rcp_f64 and two Newton steps.
// Used only by the div probe (tests) to show where it is not RN(1/s).
__device__ __forceinline__ double rcp_refine(double s) {
  double r = __builtin_amdgcn_rcp(s);
  double e = fma(-r, s, 1.0);
  r = fma(r, e, r);
  e = fma(-r, s, 1.0);
  return fma(r, e, r);
}

// The reciprocal of a sum within 2^-40 of 1, correctly rounded.  Every
// normalisation sum of the CN phase is one (s = (s0 + s1)(m0 + m1) of two
// normalised pairs, within a few ulps of 1), and so is the VN phase's last
// backward step, whose t is the normalised forward state itself (beta = 1).  With u = 1 - s (exact),
// 1/s = 1 + u + u^2 + ..., which rounds to 1 + u, except that when 1 + u is a
// midpoint (s < 1 an odd multiple of 2^-53 below 1) the positive u^2 term
// rounds it up; 1 + (u + 2^-80) reproduces both (u + 2^-80 is exact, and
// 2^-80 breaks exactly the ties u^2 breaks).  So rcp_near1(s) = RN(1/s): two
// instructions instead of a quarter-rate v_rcp_f64 and four fmas.  With a correctly
// rounded reciprocal the division tail (m = RN(n r), q = fma(fma(-s, m, n), r,
// m)) is off only when n / s lies within 2^-51 ulp of a rounding midpoint;
// tools/verify_cn_division.py enumerates every such n for |s - 1| <= 64 ulp
// and evaluates the tail exactly: it always rounds to RN(n / s).  hipcc's
// refinement is NOT RN(1/s) on six of these s (s = 1 - k 2^-53, k = 3, 5, ...,
// 13: one ulp low), and hipcc's '/' then misrounds three significands (the
// GPU test test_cn_reciprocal_exhaustive shows both).
constexpr double kNearOne = 0x1p-40;
#ifndef KML_CN_RANGE_CHECK
#define KML_CN_RANGE_CHECK 0
#endif
// Two instructions: X * Y = 1 + 2^-78 exactly (X = 1 + 2^-26, Y = 1 - 2^-26 +
// 2^-52), so fma(X, Y, 1 - s) is RN(1 + u + 2^-78) with one rounding — the
// same tie-breaking as 1 + (u + 2^-80) without the third add.
__device__ __forceinline__ double rcp_near1(double s) { return fma(0x1.0000004p+0, 0x1.ffffff8000002p-1, 1.0 - s); }
// (see rcp_cn_rows for why the range check is off by default)
__device__ __forceinline__ double rcp_cn(double s) {
  double r = rcp_near1(s);
#if KML_CN_RANGE_CHECK
  if (__builtin_expect(!(fabs(1.0 - s) <= kNearOne), 0)) r = rcp_refine(s);
#endif
  return r;
}

// Reciprocals of the R sums of one CN step (R independent rows): the near-one
// formula, or — when any sum of the lane is out of its range (not seen in a
// CN phase) — hipcc's refinement for all R, as the other FAST divisions use.
// One branch per step keeps the R rows' chains in one scheduling region.
//
// The range check is provably redundant on the FAST path: a CN sum is
// RN(n0 + n1) with n0 = RN(RN(s0 m0) + RN(s1 m1)), n1 likewise, where (s0, s1)
// and (m0, m1) are quotient pairs of one normalisation (each pair sums to
// 1 within 2 ulps: RN(x0/S) + RN(x1/S) with S = RN(x0 + x1)) or the boundary
// state (1, 0); the few roundings keep |s - 1| <= 16 * 2^-53 = 2^-49, far
// inside 2^-40 (products that underflow are tiny beside the sum's dominant
// terms).  KML_CN_RANGE_CHECK=1 builds keep it anyway (A/B, debugging).
template <int R>
__device__ __forceinline__ void rcp_cn_rows(const double (&s)[R], double (&r)[R]) {
#pragma unroll
  for (int i = 0; i < R; ++i) r[i] = rcp_near1(s[i]);
#if KML_CN_RANGE_CHECK
  bool ok = true;
#pragma unroll
  for (int i = 0; i < R; ++i) ok = ok & (fabs(1.0 - s[i]) <= kNearOne);
  if (__builtin_expect(!ok, 0)) {
#pragma unroll
    for (int i = 0; i < R; ++i) r[i] = rcp_refine(s[i]);
  }
#endif
}
// n / s from a reciprocal r of s that is exact for it (FAST division tail).
__device__ __forceinline__ double qdiv_r(double n, double s, double r) {
  const double m = n * r;
  return fma(fma(-m, s, n), r, m);
}

// One CN step's normalisations for R rows: the c2v quotients clip(t0 / ts)
// and the chain states (n0, n1) / (n0 + n1) (binaryldpccodec.cc:241-266), the
// sums' reciprocals from rcp_cn_rows on the FAST path, div_rn else.
template <int R, bool FAST>
__device__ __forceinline__ void cn_c2v_rows(const double (&t0)[R], const double (&ts)[R], double (&q)[R]);
template <int R, bool FAST>
__device__ __forceinline__ void cn_norm_rows(const double (&n0)[R], const double (&n1)[R], double (&s0)[R],
                                             double (&s1)[R]);

// q0 = RN(n0 / s) and q1 = RN(n1 / s) (binaryldpccodec.cc:177-273 divide
// with x86 divsd).
//   FAST, CN: s within 2^-49 of 1 (every CN-phase sum and the VN phase's
//     unit-beta step): the near-one reciprocal and the division tail, exact by
//     exhaustive enumeration (rcp_near1).
//   FAST, VN: exact_div.hpp dd_quot — faithful always, and proven correctly
//     rounded by dd_check; a quotient the check cannot prove (n/s next to a
//     rounding midpoint: rare, but BP's saturated messages repeat such
//     quotients) is settled by dd_fix, its neighbour's exact residual.  So
//     every FAST VN quotient is RN(n/s) and sus stays as the caller set it
//     (div2 keeps the flag for the kernels' redo machinery).  The FAST
//     path runs only for codewords whose priors pass fast_prior_ok (on codes
//     with column degree <= 23), which keeps every nonzero numerator at or
//     above 2^-961 and every sum and quotient normal ("Division"),
//     inside dd_check's domain.
//   !FAST: div_rn (any operands).
// Diagnostic build (-DKML_DIV_STATS=1, `make variant`): counts of the FAST
// VN divisions' failed premises and checks per translation unit, and the
// operands of the first 64 failures ([0] pairs seen (per wave), [1] !ok,
// [2] q0 unproven, [3] q1 unproven, [4] max |e0| bits (v_rcp_f64), [8 + 5 i ..] samples:
// n0, n1, s, q0, q1).  Read by kml_debug_div_stats.
#ifndef KML_DIV_STATS
#define KML_DIV_STATS 0
#endif
#if KML_DIV_STATS
static __device__ unsigned long long kml_div_stats[8 + 5 * 64];
__device__ __noinline__ void div_stats_record(bool ok, bool c0, bool c1, double n0, double n1, double s, double q0,
                                              double q1) {
  const unsigned long long all = __ballot(1), bok = __ballot(!ok), b0 = __ballot(!c0), b1 = __ballot(!c1);
  if ((threadIdx.x & 63) == __builtin_ctzll(all)) {
    atomicAdd(&kml_div_stats[0], (unsigned long long)__popcll(all));
    if (bok) atomicAdd(&kml_div_stats[1], (unsigned long long)__popcll(bok));
    if (b0) atomicAdd(&kml_div_stats[2], (unsigned long long)__popcll(b0));
    if (b1) atomicAdd(&kml_div_stats[3], (unsigned long long)__popcll(b1));
  }
  {
    const DdRcp y = dd_rcp(s);
    const double e = fabs(fma(-y.hi, s, 1.0));
    atomicMax(&kml_div_stats[4], (unsigned long long)__double_as_longlong(e));
  }
  if (!(ok & c0 & c1)) {
    const unsigned long long i = atomicAdd(&kml_div_stats[5], 1ull);
    if (i < 64) {
      double *d = reinterpret_cast<double *>(&kml_div_stats[8 + 5 * i]);
      d[0] = n0;
      d[1] = n1;
      d[2] = s;
      d[3] = q0;
      d[4] = q1;
    }
  }
}
#define KML_DIV_STATS_ACCESSOR(NAME)                                                                   \
  extern "C" int NAME(unsigned long long *out, int reset) {                                            \
    hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(kml::kml_div_stats), sizeof(kml::kml_div_stats)); \
    if (reset) {                                                                                       \
      static unsigned long long zero[8 + 5 * 64];                                                      \
      hipMemcpyToSymbol(HIP_SYMBOL(kml::kml_div_stats), zero, sizeof(zero));                           \
    }                                                                                                  \
    return e == hipSuccess ? 0 : -1;                                                                   \
  }
#endif

// KML_DIV_NOPROOF = 1 (A/B measurement builds only, `make variant`): the FAST
// VN quotients skip dd_check / dd_fix, i.e. faithful but unproven — the price
// of the proof per kernel family, never a shipped build (the parity tests fail).
#ifndef KML_DIV_NOPROOF
#define KML_DIV_NOPROOF 0
#endif
// DEFER (FAST VN only): a quotient the check cannot prove is left faithful and
// sets sus, for a caller that then reruns the whole column with DEFER = false
// (one rare branch per column instead of one per normalisation).
template <bool FAST, bool CN = false, bool DEFER = false>
__device__ __forceinline__ void div2(double n0, double n1, double s, double &q0, double &q1, bool &sus) {
  if constexpr (!FAST) {
    q0 = div_rn(n0, s);
    q1 = div_rn(n1, s);
  } else if constexpr (CN) {
    const double r = rcp_cn(s);
    q0 = qdiv_r(n0, s, r);
    q1 = qdiv_r(n1, s, r);
  } else {
    const DdRcp y = dd_rcp(s);
    q0 = dd_quot(n0, y);
    q1 = dd_quot(n1, y);
#if KML_DIV_NOPROOF  // (A/B measurement builds only: faithful, NOT proven correctly rounded)
    return;
#endif
    const bool c0 = dd_check(n0, s, q0, y), c1 = dd_check(n1, s, q1, y);
#if KML_DIV_STATS
    div_stats_record(true, c0, c1, n0, n1, s, q0, q1);
#endif
    if constexpr (DEFER) {
      sus |= !((int)c0 & (int)c1);
    } else if (__builtin_expect(!((int)c0 & (int)c1), 0)) {  // n/s next to a rounding midpoint: rare
      if (!c0) q0 = dd_fix(n0, s, q0);
      if (!c1) q1 = dd_fix(n1, s, q1);
    }
  }
}
// the CN phase's form (near-one sums: nothing to prove at run time)
template <bool FAST, bool CN>
__device__ __forceinline__ void div2(double n0, double n1, double s, double &q0, double &q1) {
  static_assert(CN, "VN divisions carry a suspect flag");
  bool unused = false;
  div2<FAST, CN>(n0, n1, s, q0, q1, unused);
}

// n0 / s for the CN phase (near-one sums on the FAST path)
template <bool FAST, bool CN = true>
__device__ __forceinline__ double div1(double n0, double s) {
  static_assert(CN, "div1 is the CN phase's division");
  if constexpr (!FAST) return div_rn(n0, s);
  else return qdiv_r(n0, s, rcp_cn(s));
}

// The first backward step of a column multiplies beta = (1, 1) by the c2v pair
// (c0, RN(1 - c0)) and normalises by s = RN(c0 + RN(1 - c0)).  For c0 in [0, 1]
// s is exactly 1: for c0 >= 1/2, 1 - c0 is exact (Sterbenz); for c0 < 1/2 the
// rounding error of 1 - c0 (in (1/2, 1]) is at most 2^-54, so the exact sum lies
// in [1 - 2^-54, 1 + 2^-54], which rounds to 1 (1 - 2^-54 is a tie, broken to
// the even 1).  Division by 1 is exact, so the FAST kernels take beta =
// (c0, RN(1 - c0)) directly; c2v messages are always clipped to
// [1e-12, 1 - 1e-12] or 0.5 on the FAST path.

// Prior values for which the FAST division path is exact (see div2): +0, 1,
// and q with q >= lo and 1 - q >= lo, lo = fast_prior_lo(dv_max) =
// 2^(40 dv_max - 960).  Every quantity a FAST decode divides is a product of a
// prior component and at most dv_max c2v components (each >= 1e-12 > 2^-40,
// ProbClip), renormalised along the way (which only raises it), so it is 0 or
// at least lo 2^(-40 dv_max) (1 - 2^-50) >= 2^-961 > 2^-969: inside the
// residual-exactness domain of dd_check and of the near-one CN division.
// -0.0 is excluded: with every prior >= +0 no message is ever -0, which makes
// the x*1.0 / (1,0)-state identities used on the FAST path exact.
__device__ __forceinline__ double fast_prior_lo(int dv_max) {
  return __longlong_as_double((long long)(63 + 40 * dv_max) << 52);  // 2^(40 dv_max - 960)
}
__device__ __forceinline__ bool fast_prior_ok(double q, double lo) {
  return (q == 0.0 && __double_as_longlong(q) == 0) || q == 1.0 || (q >= lo && 1.0 - q >= lo);
}

// lo = 2^-40 at dv_max = 23; beyond it no prior but 0 and 1 would qualify
constexpr int kFastMaxColumnDegree = 23;

// ProbClip of a c2v message (binaryldpccodec.cc:260-263).  On the FAST path the
// value is finite (no NaN), where min(max(q, lo), hi) is the same two tests.
template <bool FAST>
__device__ __forceinline__ double clip_c2v(double q) {
  if constexpr (FAST) {
    return fmin(fmax(q, kSmallestProb), 1.0 - kSmallestProb);
  } else {
    if (q > 1.0 - kSmallestProb) q = 1.0 - kSmallestProb;
    if (q < kSmallestProb) q = kSmallestProb;
    return q;
  }
}

template <int R, bool FAST>
__device__ __forceinline__ void cn_c2v_rows(const double (&t0)[R], const double (&ts)[R], double (&q)[R]) {
  if constexpr (FAST) {
    double rc[R];
    rcp_cn_rows<R>(ts, rc);
#pragma unroll
    for (int i = 0; i < R; ++i) q[i] = clip_c2v<true>(qdiv_r(t0[i], ts[i], rc[i]));
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) q[i] = clip_c2v<false>(div_rn(t0[i], ts[i]));
  }
}
template <int R, bool FAST>
__device__ __forceinline__ void cn_norm_rows(const double (&n0)[R], const double (&n1)[R], double (&s0)[R],
                                             double (&s1)[R]) {
  double ns[R];
#pragma unroll
  for (int i = 0; i < R; ++i) ns[i] = n0[i] + n1[i];
  if constexpr (FAST) {
    double rc[R];
    rcp_cn_rows<R>(ns, rc);
#pragma unroll
    for (int i = 0; i < R; ++i) {
      s0[i] = qdiv_r(n0[i], ns[i], rc[i]);
      s1[i] = qdiv_r(n1[i], ns[i], rc[i]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      s0[i] = div_rn(n0[i], ns[i]);
      s1[i] = div_rn(n1[i], ns[i]);
    }
  }
}

// Hard decision of a column from the un-normalised posterior (n0, n1):
// the reference compares RN(n0/s) > RN(n1/s) with s = n0 + n1
// (binaryldpccodec.cc:186-194).  When n0 and n1 differ by more than 2^-48
// relative, the rounded quotients are ordered like n0, n1 (RN is monotone and
// the gap exceeds an ulp); only then is the division skipped (FAST path, all
// values finite and >= +0).
template <bool FAST>
__device__ __forceinline__ int hard_decision(double n0, double n1, bool &sus) {
  if constexpr (FAST) {
    const double g = 1.0 + 0x1p-48;
    if (n0 > n1 * g) return 0;
    if (n1 > n0 * g) return 1;
  }
  double a0, a1;
  div2<FAST>(n0, n1, n0 + n1, a0, a1, sus);
  return (a0 > a1) ? 0 : 1;
}

// SourceSink::CntErr (sourcesink.cc:29-47) of one codeword's info bits against
// its packed source word array ref[Kw]: Σ popcount(packed(uu_hat) ^ ref).
// Wave w of the workgroup packs words w, w + T/64, ... with one ballot each
// (lane j holds bit 64w + j, zero past K), so the 64-step serial pack of the
// one-thread-per-word form leaves the codeword's tail.  cch holds 0/1 hard
// decisions; bit i sits at cch[pos ? pos[off + i] : off + i].  Returns the
// wave's count on lane 0, 0 on the other lanes.
template <int T>
__device__ __forceinline__ int count_info_errors(const unsigned char *cch, const int *pos, int off, int K, int Kw,
                                                 const uint64_t *ref, int tid) {
  const int lane = tid & 63;
  int errs = 0;
  for (int w = tid >> 6; w < Kw; w += T / 64) {
    const int i = w * 64 + lane;
    int bit = 0;
    if (i < K) bit = cch[pos ? pos[off + i] : off + i];
    const uint64_t word = __ballot(bit);
    if (lane == 0) errs += __popcll(word ^ ref[w]);
  }
  return errs;
}

}  // namespace kml
