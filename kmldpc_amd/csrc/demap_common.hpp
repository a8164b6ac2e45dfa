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

// P0 for the MB bits of one symbol.
template <int MB>
__device__ __forceinline__ void demap_symbol(const double *__restrict__ cons, double yr, double yi, double hr, double hi,
                                             double var, double *out) {
  constexpr int KC = 1 << MB;
  double pr[KC];
  double mx = 0.0;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    const double cr = cons[2 * k], ci = cons[2 * k + 1];
    double sr = cr * hr - ci * hi;  // symbol *= theta_h
    double si = cr * hi + ci * hr;
    sr = sr - yr;  // symbol -= yy
    si = si - yi;
    const double d = (sr * sr + si * si) / var;
    pr[k] = -d;
    if (k == 0 || mx < pr[k]) mx = pr[k];  // *max_element
  }
  double sum = 0.0;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    pr[k] = kml_exp(pr[k] - mx);  // glibc exp, bit-exact (exact_math.hpp)
    sum += pr[k];
  }
  // normalise + ProbClip (modemlinearsystem.cc:240-246), ProbClip again (modem.cc:27)
  double w = 1.0;  // prod over bits of bitLin (= 0.5) or 1 - bitLin (= 0.5)
#pragma unroll
  for (int j = 0; j < MB; ++j) w *= 0.5;
  double sum2 = 0.0;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    pr[k] = prob_clip(prob_clip(pr[k] / sum));
    pr[k] = w * pr[k];
    sum2 += pr[k];
  }
#pragma unroll
  for (int k = 0; k < KC; ++k) pr[k] /= sum2;
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
    out[j] = prob_clip(q0 / (q0 + q1));
  }
}


}  // namespace kml
