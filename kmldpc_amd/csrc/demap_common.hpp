// demap_common.hpp — the soft demapper of one symbol, shared by demap.hip and
// the BP kernels that fuse the demapper into their prologue.
//
//   ModemLinearSystem::SoftAWGNDemodulation (lib/lab/src/modemlinearsystem.cc:51-79)
//   followed by Modem::DeMapping with bitLin = 0.5 (lib/lab/src/modem.cc:23-79;
//   KmCodec::DeMapping sets bit_l_in_ = 0.5, src/kmcodec.cc:96-98), in the
//   reference's operation order, exp = kml_exp (glibc-exact).
#pragma once
#include "bp_common.hpp"
#include "exact_math.hpp"

namespace kml {

__device__ __forceinline__ double prob_clip(double v) {  // utility.cc:18-26
  if (v < kSmallestProb) return kSmallestProb;
  if (v > 1.0 - kSmallestProb) return 1.0 - kSmallestProb;
  return v;
}

// FAST quotient n / s with its proof (exact_div.hpp dd_quot / dd_check): ok
// is cleared when the quotient is not proven correctly rounded, and the caller
// then reruns the symbol on the exact path.
__device__ __forceinline__ double qdiv(double n, double s, const DdRcp &r, bool &ok) {
  const double q = dd_quot(n, r);
  ok &= dd_check(n, s, q, r);
  return q;
}

// Constellation points staged in LDS by the calling kernel (cons_lds); CP is
// the pointer type the demap helpers read them through.
typedef const __attribute__((address_space(3))) double *lds_cons;

// The exp table (kExpTabDev, 128 (tail, scale bits) pairs) staged in LDS by the
// calling kernel: one ds_read_b128 per exp instead of two scattered global loads.
typedef const __attribute__((address_space(3))) uint64_t *lds_exptab;
__device__ __forceinline__ void stage_exp_table(uint64_t *dst) {  // dst: a __shared__ array
  for (int i = threadIdx.x; i < 256; i += blockDim.x) dst[i] = kExpTabDev[i];
}
// Bank-private form (ES = kExpBanked u64 per entry): 16 copies of the table,
// entry i of copy L at byte 256 i + 16 L, and lane L (mod 16) reads copy L
// (the base pointer it passes is dst + 2 (lane & 15)).  A ds_read_b128 is
// serviced 16 lanes per pass, one 4-bank group per lane, so the random table
// indices of a wave's exps no longer collide on banks (32 KB of LDS; the
// 64QAM demap_kernel).
constexpr int kExpBanked = 32;
__device__ __forceinline__ void stage_exp_table_banked(uint64_t *dst) {  // dst: a __shared__ array of 4096
  for (int i = threadIdx.x; i < 128 * 16; i += blockDim.x) {
    const int e = i >> 4, L = i & 15;
    dst[e * kExpBanked + 2 * L] = kExpTabDev[2 * e];
    dst[e * kExpBanked + 2 * L + 1] = kExpTabDev[2 * e + 1];
  }
}

// glibc's exp (kml_exp_t<true>) on its main path only: exact for x == 0 and
// for 2^-54 <= |x| < 512, where glibc takes no special case (x == 0 gives
// fma(1, 0, 1) = 1 here, as glibc's 1 + x).  exp_core_ok says whether x is in
// that domain; callers fall back to kml_exp outside it.
__device__ __forceinline__ bool exp_core_ok(double x) {
  const double a = fabs(x);  // branch-free: (2^-54 <= |x| < 512) or x == 0
  return ((a >= 0x1p-54) & (a < 512.0)) | (x == 0.0);
}
template <int ES = 2>  // u64 per table entry: 2 (stage_exp_table) or kExpBanked
__device__ __forceinline__ double exp_core(double x, lds_exptab tab) {
  const double InvLn2N = 0x1.71547652b82fep0 * 128;
  const double Shift = 0x1.8p52;
  const double NegLn2hiN = -0x1.62e42fefa0000p-8;
  const double NegLn2loN = -0x1.cf79abc9e3b3ap-47;
  const double C2 = 0x1.ffffffffffdbdp-2, C3 = 0x1.555555555543cp-3;
  const double C4 = 0x1.55555cf172b91p-5, C5 = 0x1.1111167a4d017p-7;
  double kd = fma(InvLn2N, x, Shift);
  const uint64_t ki = as_u64(kd);
  kd -= Shift;
  const double r = fma(kd, NegLn2loN, fma(kd, NegLn2hiN, x));
  const int idx = (int)(ES * (ki % 128));
  const double tail = as_f64(tab[idx]);
  const uint64_t sbits = tab[idx + 1] + (ki << (52 - 7));
  const double r2 = r * r;
  const double tmp = fma(r2 * r2, fma(r, C5, C4), fma(r2, fma(r, C3, C2), tail + r));
  const double scale = as_f64(sbits);
  return fma(scale, tmp, scale);
}

// P0 for the MB bits of one symbol.  FAST: the divisions by var, by the
// exponential sum, by the prior-weighted sum and by q0 + q1 share one
// double-double reciprocal each, and every quotient carries its proof
// (qdiv, exact_div.hpp); returns false, with out[] unset, when an operand
// leaves the proof's domain or a quotient is not proven, and the caller reruns
// the symbol with div_rn (FAST = false, always true).  The domain:
//   * var in [2^-64, 2^64] and every squared distance n_k in [2^-512, 2^512]
//     (n_k = 0, a symbol exactly on a point, falls back);
//   * the exponential sum lies in [1, KC] (its largest term is exp(0) = 1);
//     a term below 2^-969 is outside the proof's domain, but its quotient and
//     RN's are both far below 1e-12, so ProbClip maps both to 1e-12 whatever
//     the check says;
//   * the sum of the clipped terms in [2^-64, 2^64] (at least w / KC, or 1 / KC
//     unweighted, see below): the terms (>= w * 1e-12) and q0, q1 (>= 1e-14,
//     q0 + q1 ~ 2) are inside.
// LEAN (default): ProbClip once and, FAST, the sum without the prior weight
// (below; the same bits).  The fused QPSK prologue of bp_regular keeps the
// reference's sequence (LEAN = false): there the lean form measured 0.45 %
// slower on the headline kernel (profiles/r04_ab15_summary.txt).
// ROT (FAST only): cons holds the points already multiplied by the channel,
// (cr hr - ci hi, cr hi + ci hr) in the reference's operation order
// (demap_kernel stages them per codeword), and hr, hi are unused: the same
// values, 6 fewer operations per point.
#ifndef KML_DEMAP_MX_NMIN  // (A/B) 0: the running maximum of the reference's loop
#define KML_DEMAP_MX_NMIN 1
#endif
template <int MB, bool FAST, class CP, int ES = 2, bool LEAN = true, bool ROT = false>
__device__ __forceinline__ bool demap_symbol_t(CP cons, lds_exptab etab, double yr, double yi, double hr,
                                               double hi, double var, double *out) {
  static_assert(!ROT || FAST, "pre-rotated points: FAST path only");
  constexpr int KC = 1 << MB;
  // opaque per call: the constellation's LDS loads must not be hoisted out of
  // the caller's symbol loop (64QAM: 128 doubles held live across it)
  asm volatile("" : "+v"(cons), "+v"(etab));
  double pr[KC];
  double mx = 0.0;
  double nmin = 0.0, nmax = 0.0;
  bool dok = true;  // every FAST quotient proven correctly rounded
  DdRcp rv{};
  if (FAST) rv = dd_rcp(var);
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const double cr = cons[2 * k], ci = cons[2 * k + 1];
    double sr = ROT ? cr : cr * hr - ci * hi;  // symbol *= theta_h
    double si = ROT ? ci : cr * hi + ci * hr;
    sr = sr - yr;  // symbol -= yy
    si = si - yi;
    const double n = sr * sr + si * si;
    double d;
    if (FAST) {
      nmin = k == 0 ? n : fmin(nmin, n);
      nmax = k == 0 ? n : fmax(nmax, n);
      d = qdiv(n, var, rv, dok);
    } else {
      d = div_rn(n, var);
    }
    pr[k] = -d;
    if (!(FAST && KML_DEMAP_MX_NMIN) && (k == 0 || mx < pr[k])) mx = pr[k];  // *max_element
  }
  // FAST: *max_element = -RN(nmin / var): every d_k = RN(n_k / var) once the
  // proofs pass, and RN(x / var) is non-decreasing in x (var > 0), so the
  // largest -d_k is -RN(min n_k / var), proven like the others (no
  // per-point running maximum)
  if (FAST && KML_DEMAP_MX_NMIN) mx = -qdiv(nmin, var, rv, dok);
  if (FAST && !(dok && nmin >= 0x1p-512 && nmax <= 0x1p512 && var >= 0x1p-64 && var <= 0x1p64)) return false;
  double sum = 0.0;
  bool eok = true;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const double x = pr[k] - mx;
    if (FAST) {  // glibc's main path (exp_core), the rest falls back
      eok &= exp_core_ok(x);
      pr[k] = exp_core<ES>(x, etab);
    } else {
      pr[k] = kml_exp(x);  // glibc exp, bit-exact (exact_math.hpp)
    }
    sum += pr[k];
  }
  if (FAST && !(eok && sum >= 1.0 && sum <= (double)KC)) return false;
  // normalise + ProbClip (modemlinearsystem.cc:240-246), ProbClip again (modem.cc:27)
  double w = 1.0;  // prod over bits of bitLin (= 0.5) or 1 - bitLin (= 0.5)
#pragma unroll
  for (int j = 0; j < MB; ++j) w *= 0.5;
  DdRcp rs{};
  if (FAST) rs = dd_rcp(sum);
  double sum2 = 0.0;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    bool ok_k = true;
    const double qk = FAST ? qdiv(pr[k], sum, rs, ok_k) : div_rn(pr[k], sum);
    // a faithful quotient below 1e-12 has RN's clip: RN is it or its upper
    // neighbour, at most 1e-12 (terms below 2^-969, outside the check's domain)
    if (FAST) dok &= ok_k | (qk < kSmallestProb);
    // ProbClip twice in the reference (modemlinearsystem.cc:240-246, then
    // modem.cc:27): the clip is idempotent (NaN included), so once
    pr[k] = LEAN ? prob_clip(qk) : prob_clip(prob_clip(qk));
    // FAST: the prior weight w = 2^-MB scales every term and hence every
    // partial sum of sum2 exactly (all normal: terms >= 1e-12), so the
    // quotients pr[k] / sum2 below are the same without it
    if (!(FAST && LEAN)) pr[k] = w * pr[k];
    sum2 += pr[k];
  }
  if (FAST && !(dok && sum2 >= 0x1p-64 && sum2 <= 0x1p64)) return false;
  DdRcp rs2{};
  if (FAST) rs2 = dd_rcp(sum2);
#pragma unroll
  for (int k = 0; k < KC; ++k) pr[k] = FAST ? qdiv(pr[k], sum2, rs2, dok) : div_rn(pr[k], sum2);
  // per-bit sums in ascending k (modem.cc:58-70); one bit at a time keeps two
  // accumulators live next to the KC probabilities
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    double q0 = 0.0, q1 = 0.0;
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      if (((k >> (MB - 1 - j)) & 1) == 0)
        q0 += pr[k];
      else
        q1 += pr[k];
    }
    q0 /= 0.5;
    q1 /= (1.0 - 0.5);
    const double t = q0 + q1;
    if constexpr (FAST) {
      const DdRcp rt = dd_rcp(t);
      out[j] = prob_clip(qdiv(q0, t, rt, dok));
    } else {
      out[j] = prob_clip(div_rn(q0, t));
    }
  }
  return dok;
}

// Every kernel that demaps runs demap_symbol_t<MB, true> (FAST, proven) in a
// FAST kernel and hands the symbols (or codewords) it cannot prove to an EXACT
// kernel that runs demap_symbol_t<MB, false>: inlined side by side, the exact
// path (div_rn, kml_exp) doubled the FAST kernels' registers and code, the
// 64QAM demapper's past 300 KB (instruction-cache bound).

// Hard decisions rr_j = (P0_j > 0.5) of one symbol's MB bits (the metric's
// kmcodec.cc:111-115) screened in single precision: returns false when some bit
// is too close to call, and the caller then runs the exact demap_symbol.
// P0_j > 0.5 iff Q0_j > Q1_j, where Q_b = sum over the points whose label bit j
// is b of c_k = ProbClip(exp(a_k) / sum exp(a)), a_k = dmin - d_k (the common
// factors w and 1 / sum2 cancel, and ProbClip of the final quotient does not
// move it across 0.5).  The screen compares instead the unclipped, unnormalised
// sums q_b = sum of exp(a_k) (one scale factor, sum exp(a), is common to both):
//   * d_k is formed in double in log2 units, f_k = RN_f32(d_k log2 e), and the
//     symbol is screened only when fmin = min f_k <= 64; a term that is not
//     negligible has f_k <= fmin + 58 < 128, so its f_k is within 2^-18 of the
//     exact value (the double arithmetic adds < 2^-30: the expanded form below
//     M <= 2^20, checked; the direct form is the reference's own |c_k h - y|^2
//     times 1 / var log2 e, 2^-51 relative);
//   * e_k = v_exp_f32(fmin - f_k): the subtraction rounds once (< 2^-19 for
//     |.| < 64) and v_exp_f32 is within 1 ulp, so e_k = 2^(dmin log2 e - d_k
//     log2 e + dlt) (1 +- 2^-23) with |dlt| < 2^-17 beyond the error of fmin,
//     which is a factor common to every term: relative to each other the terms
//     are within 1e-5, and the float sums add < 65 * 2^-24 relative;
//   * the clips: ProbClip's floor 1e-12 adds at most 2^6 * 1e-12 to a
//     normalised Q, and the ceiling 1 only removes rounding; the smaller side of
//     a decided bit is compared with the larger, which holds at least half of
//     the total, so both move its ratio by < 1e-9.
// A bit is decided only when one sum exceeds the other by 2^-12 (2.4e-4)
// relative, against < 4e-5 of accumulated error (the reference's own rounding
// is below 1e-13).  Terms with a_k below -88 flush to 0 here and clip to 1e-12
// there: covered by the clip bound.
// 16QAM and up: d_k = |c_k|^2 A - 2 Re(c_k B) + |y|^2 / var with A = |h|^2 / var
// and B = h conj(y) / var, three fmas per point from the staged
// (|c_k|^2, 2 Re c_k, 2 Im c_k) (scr; the reference's form costs nine);
// M = cbound (A + |Br| + |Bi|) + |y|^2 / var bounds every partial result.  QPSK
// and 8-point sets keep the direct form |c_k h - y|^2 / var (there the setup
// outweighs the saving, measured 0.96 -> 0.99 ms per 32768 QPSK codewords).
template <int MB, class CP>
__device__ __forceinline__ bool hard_bits_screen(CP cons, CP scr, double cbound, double yr, double yi, double hr,
                                                 double hi, double inv_var, unsigned &bits) {
  constexpr int KC = 1 << MB;
  constexpr bool kExpand = MB >= 4;
  asm volatile("" : "+v"(scr));  // opaque per call: no hoisting of the point loads out of the caller's loop
  const double iv = inv_var * 1.4426950408889634;  // 1 / var in log2 units
  double A = 0.0, Br = 0.0, Bi = 0.0, Y = 0.0;
  if constexpr (kExpand) {
    A = (hr * hr + hi * hi) * iv;
    Br = (hr * yr + hi * yi) * iv;  // Re(h conj(y)) / var
    Bi = (hi * yr - hr * yi) * iv;  // Im(h conj(y)) / var
    Y = (yr * yr + yi * yi) * iv;
    // cbound >= max(max |c_k|^2, 2 max(|Re c_k|, |Im c_k|))
    if (!(cbound * (A + fabs(Br) + fabs(Bi)) + Y <= 0x1p20)) return false;
  }
  float e[KC];  // f_k, then exp2(fmin - f_k) in place
  float fmin = INFINITY;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    double d;
    if constexpr (kExpand) {
      d = fma(scr[3 * k], A, fma(-scr[3 * k + 1], Br, fma(scr[3 * k + 2], Bi, Y)));
    } else {
      const double cr = cons[2 * k], ci = cons[2 * k + 1];
      const double sr = cr * hr - ci * hi - yr;
      const double si = cr * hi + ci * hr - yi;
      d = (sr * sr + si * si) * iv;
    }
    e[k] = (float)d;
    fmin = fminf(fmin, e[k]);
  }
  if (!(fmin <= 64.f)) return false;  // (NaN too)
  float q0[MB], q1[MB];
#pragma unroll
  for (int j = 0; j < MB; ++j) q0[j] = q1[j] = 0.f;
  // 16QAM and up: q1_j = total - q0_j (half the label-sum adds).  Its error
  // is at most 2^-24 (KC + 1) total beside q0_j's; a wrong call needs the true
  // sums ordered the other way, where the smaller-labelled sum is at least
  // total / 2, so the extra error stays below 2^-17 relative to the sums
  // compared, far inside the 2^-12 margin.
#ifndef KML_SCREEN_COMPLEMENT
#define KML_SCREEN_COMPLEMENT 1
#endif
  constexpr bool kComplement = KML_SCREEN_COMPLEMENT && MB >= 4;
  float tot = 0.f;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const float c = __builtin_amdgcn_exp2f(fmin - e[k]);
    if (kComplement) tot += c;
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      if (((k >> (MB - 1 - j)) & 1) == 0)
        q0[j] += c;
      else if (!kComplement)
        q1[j] += c;
    }
  }
  if (kComplement) {
#pragma unroll
    for (int j = 0; j < MB; ++j) q1[j] = tot - q0[j];
  }
  constexpr float g = 1.f + 0x1p-12f;
  unsigned b = 0;
#pragma unroll
  for (int j = 0; j < MB; ++j) {
    if (q0[j] > q1[j] * g)
      b |= 1u << j;
    else if (!(q1[j] > q0[j] * g))
      return false;
  }
  bits = b;
  return true;
}

}  // namespace kml
