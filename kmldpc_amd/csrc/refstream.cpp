// refstream.cpp — the reference's host random sources, for runs that must see
// the reference's own frames ("identical RNG seeds"):
//
//   lab::CLCRandNum (lib/lab/src/randnum.cc:4-92): Park-Miller minimal standard
//     generator (A = 48271, M = 2^31 - 1) with Schrage's decomposition,
//     u = state / M, and Marsaglia's polar method for normals.  SetSeed(-1)
//     gives state 17 (the other SetSeed modes read the clock or stdin).
//   lab::CWHRandNum (randnum.cc:95-166): Wichmann-Hill, three small LCGs summed
//     mod 1, same polar method.  SetSeed(-1) gives (13, 37, 91).
//   lab::SourceSink::GetBitStr / GetSymStr (sourcesink.cc:5-19).
//   kml_ref_frames: Simulator::run_blocks' draw order per codeword
//     (simulator.cc:118-130): K uniforms for the bits, one polar pair for h
//     (scaled by sqrt(0.5)), one polar pair per symbol for the noise, with the
//     encoder, the MSB-first mapping (modem.cc:12-21) and y = x*h + n*(sigma/sqrt2)
//     (modemlinearsystem.cc:38-48) in std::complex<double> arithmetic.
//
// These are inherently sequential streams and run on the host; the GPU
// throughput path uses the counter-based generator in framegen.hip instead.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/kmldpc_amd.h"
#include "code.hpp"
#include "modem.hpp"

namespace {

constexpr int64_t kA = 48271, kM = 2147483647, kQ = kM / kA, kR = kM % kA;

double lcg_uniform(int64_t &state) {
  const int tmp = (int)(kA * (state % kQ) - kR * (state / kQ));
  state = tmp >= 0 ? tmp : tmp + kM;
  return state / (double)kM;
}

double wh_uniform(int32_t *s) {
  s[0] = 171 * s[0] % 30269;
  s[1] = 172 * s[1] % 30307;
  s[2] = 170 * s[2] % 30323;
  double u = s[0] / 30269.0 + s[1] / 30307.0 + s[2] / 30323.0;
  return u - (int)u;
}

template <class U>
void polar(U uniform, double *nn, int len) {
  double x1, x2, w;
  for (int t = 0; 2 * t + 1 < len; t++) {
    w = 2.0;
    while (w > 1.0) {
      x1 = 2.0 * uniform() - 1.0;
      x2 = 2.0 * uniform() - 1.0;
      w = x1 * x1 + x2 * x2;
    }
    w = std::sqrt(-2.0 * std::log(w) / w);
    nn[2 * t] = x1 * w;
    nn[2 * t + 1] = x2 * w;
  }
  if (len % 2 == 1) {
    w = 2.0;
    while (w > 1.0) {
      x1 = 2.0 * uniform() - 1.0;
      x2 = 2.0 * uniform() - 1.0;
      w = x1 * x1 + x2 * x2;
    }
    w = std::sqrt(-2.0 * std::log(w) / w);
    nn[len - 1] = x1 * w;
  }
}

}  // namespace

extern "C" {

double kml_lcg_uniform(int64_t *state) { return lcg_uniform(*state); }

void kml_lcg_normal(int64_t *state, double *nn, int len) {
  polar([&] { return lcg_uniform(*state); }, nn, len);
}

double kml_wh_uniform(int32_t *xyz) { return wh_uniform(xyz); }

void kml_wh_normal(int32_t *xyz, double *nn, int len) {
  polar([&] { return wh_uniform(xyz); }, nn, len);
}

void kml_get_bit_str(int64_t *state, uint8_t *uu, int len) {
  for (int t = 0; t < len; t++) uu[t] = lcg_uniform(*state) < 0.5 ? 0 : 1;
}

void kml_get_sym_str(int64_t *state, int32_t *uu, int qary, int len) {
  for (int t = 0; t < len; t++) {
    uu[t] = qary;
    while (uu[t] == qary) uu[t] = (int)(qary * lcg_uniform(*state));
  }
}

}  // extern "C"

// needs the context internals (code + modem): defined in capi.cpp through this hook
namespace kml {
int ref_frames(const LdpcCode &code, const Modem &modem, int64_t *state, double snr, int n, uint8_t *uu_out,
               double *h_out, double *y_out) {
  const int K = code.K, S = code.cc_len / modem.bits;
  double var, sigma, ns;
  channel_constants(snr, var, sigma, ns);
  std::vector<uint8_t> cc(code.cc_len);
  const double s5 = std::sqrt(0.5);
  for (int b = 0; b < n; b++) {
    uint8_t *uu = uu_out + (size_t)b * K;
    kml_get_bit_str(state, uu, K);
    code.encode(uu, cc.data());
    if (!code.active) memset(uu, 0, K);  // the inactive Encoder zeroes uu too (binaryldpccodec.cc:157-158)
    double h[2];
    kml_lcg_normal(state, h, 2);
    const double hr = h[0] * s5, hi = h[1] * s5;
    h_out[2 * b] = hr;
    h_out[2 * b + 1] = hi;
    double *y = y_out + (size_t)b * 2 * S;
    for (int j = 0; j < S; j++) {
      int idx = 0;
      for (int q = 0; q < modem.bits; q++) idx = (idx << 1) + cc[(size_t)j * modem.bits + q];
      const double xr = modem.pts[2 * idx], xi = modem.pts[2 * idx + 1];
      double nz[2];
      kml_lcg_normal(state, nz, 2);
      const double tr = xr * hr - xi * hi, ti = xr * hi + xi * hr;
      const double sr = nz[0] * ns - nz[1] * 0.0, si = nz[0] * 0.0 + nz[1] * ns;
      y[2 * j] = tr + sr;
      y[2 * j + 1] = ti + si;
    }
  }
  return KML_OK;
}
}  // namespace kml
