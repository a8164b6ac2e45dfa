// framegen.hip — synthetic y = h*x + w frames generated on the GPU.
//
// Throughput counterpart of the reference's per-codeword frame generation
// (src/simulator.cc:118-130): SourceSink::GetBitStr (lib/lab/src/sourcesink.cc:5-10),
// the dense systematic encoder (lib/lab/src/binaryldpccodec.cc:144-162 /
// binary5gldpccodec.cc:86-109), Modem::Mapping (lib/lab/src/modem.cc:12-21) and
// ModemLinearSystem::PartitionHAWGNSystem (lib/lab/src/modemlinearsystem.cc:38-48)
// with h ~ CN(0,1) per codeword (simulator.cc:121-123).
//
// The reference draws from one sequential Park-Miller stream, which cannot be
// split across 10^5 concurrent codewords, so this path uses a counter-based
// Philox4x32-10 generator keyed by (seed, global codeword index): frames are
// independent of the batch size and of the number of GPUs (weak-scaling
// invariant), and BER/FER are checked against the reference within Monte-Carlo
// confidence.  Bit-exact parity runs feed the reference's own frames instead.
#include <cstdlib>

#include "kernels.hpp"

namespace kml {

namespace {

struct u32x4 {
  uint32_t x, y, z, w;
};

// Philox4x32-10 (Salmon et al., SC'11).
__device__ __forceinline__ u32x4 philox(u32x4 ctr, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * ctr.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * ctr.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    ctr = u32x4{hi1 ^ ctr.y ^ k0, lo1, hi0 ^ ctr.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return ctr;
}

enum : uint32_t { STREAM_BITS = 1, STREAM_H = 2, STREAM_NOISE = 3 };

__device__ __forceinline__ u32x4 draw(unsigned long long seed, unsigned long long cw, uint32_t stream, uint32_t idx) {
  return philox(u32x4{(uint32_t)cw, (uint32_t)(cw >> 32), stream, idx}, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// uniform in (0, 1]
__device__ __forceinline__ double u01(uint32_t hi, uint32_t lo) {
  const uint64_t v = ((uint64_t)hi << 32 | lo) >> 11;
  return (double)(v + 1) * 0x1p-53;
}

// Box-Muller pair of standard normals
__device__ __forceinline__ double2 gauss2(u32x4 r) {
  const double u1 = u01(r.x, r.y), u2 = u01(r.z, r.w);
  const double rad = sqrt(-2.0 * log(u1));
  double sn, cs;
  sincospi(2.0 * u2, &sn, &cs);
  return make_double2(rad * cs, rad * sn);
}

// one thread per 64-bit word of info bits
__global__ void source_kernel(int K, int Kw, int B, unsigned long long seed, unsigned long long first_cw, int active,
                              uint64_t *__restrict__ uu) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)B * Kw) return;
  const int cw = (int)(gid / Kw), w = (int)(gid - (long long)cw * Kw);
  uint64_t word = 0;
  if (active) {  // Encoder() zeroes uu when the encoder is inactive (binaryldpccodec.cc:157-158)
    const u32x4 r = draw(seed, first_cw + cw, STREAM_BITS, (uint32_t)(w >> 1));
    word = (w & 1) ? ((uint64_t)r.w << 32 | r.z) : ((uint64_t)r.y << 32 | r.x);
    const int nb = K - w * 64;
    if (nb < 64) word &= (1ull << nb) - 1;
  }
  uu[gid] = word;
}

// one lane per transmitted bit; a wavefront packs 64 bits with a ballot
__global__ __launch_bounds__(256) void encode_kernel(DevCode c, int B, int Cw, const uint64_t *__restrict__ uu,
                                                     uint64_t *__restrict__ cc) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long per_cw = (long long)Cw * 64;
  const int cw = (int)(gid / per_cw);
  const int i = (int)(gid - (long long)cw * per_cw);
  if (cw >= B) return;  // whole wavefronts exit together (per_cw is a multiple of 64)
  const uint64_t *u = uu + (long long)cw * c.Kw;
  int bit = 0;
  if (i < c.cc_len && c.active) {
    int info = -1, par = -1;
    if (!c.is5g) {  // cc = [parity(chk) | info(K)]
      if (i < c.chk)
        par = i;
      else
        info = i - c.chk;
    } else {  // [info(K) | parity] without the first 2Z bits
      const int f = i + c.punct;
      if (f < c.K)
        info = f;
      else
        par = f - c.K;
    }
    if (info >= 0) {
      bit = (int)((u[info >> 6] >> (info & 63)) & 1u);
    } else {
      const uint64_t *row = c.enc_info + (long long)par * c.Kw;
      uint64_t acc = 0;
      for (int w = 0; w < c.Kw; ++w) acc ^= row[w] & u[w];
      bit = __popcll(acc) & 1;
    }
  }
  const uint64_t mask = __ballot(bit);
  if ((threadIdx.x & 63) == 0) cc[(long long)cw * Cw + (i >> 6)] = mask;
}

// The parity part of the same encoder for codes whose parity and info runs
// start on 64-bit word boundaries of cc (PEG2304, PEG8064, 5G BG2 K960): a
// workgroup takes 64 parity rows x kEncCw codewords.  The rows' generator
// words are staged in LDS transposed (word w of row r at [w][r]: lane r reads
// consecutive addresses), the codewords' info words likewise ([cw][w], one
// broadcast per word); lane r of a wave forms parity bit r of one codeword
// per pass (AND / XOR over Kw words, popcount parity) and the wave packs the
// 64 bits with a ballot.  Each generator word is read from HBM once per
// kEncCw codewords instead of once per codeword, and every global access is
// coalesced (the one-lane-per-bit encode_kernel reads 64 rows per load).
constexpr int kEncCw = 64;
__global__ __launch_bounds__(256) void encode_parity_kernel(DevCode c, int B, int Cw, int par_word,
                                                            const uint64_t *__restrict__ uu,
                                                            uint64_t *__restrict__ cc) {
  extern __shared__ uint64_t es[];
  const int Kw = c.Kw;
  uint64_t *gt = es;            // [Kw][64]
  uint64_t *us = es + Kw * 64;  // [kEncCw][Kw]
  const int r0 = blockIdx.x * 64, c0 = blockIdx.y * kEncCw;
  const int ncw = min(kEncCw, B - c0);
  for (int idx = threadIdx.x; idx < 64 * Kw; idx += blockDim.x) {
    const int r = idx / Kw, w = idx - r * Kw;
    gt[w * 64 + r] = r0 + r < c.chk ? c.enc_info[(long long)(r0 + r) * Kw + w] : 0ull;
  }
  for (int idx = threadIdx.x; idx < ncw * Kw; idx += blockDim.x) us[idx] = uu[(long long)c0 * Kw + idx];
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int k = wave; k < ncw; k += blockDim.x / 64) {
    const uint64_t *u = us + k * Kw;
    uint64_t a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    int w = 0;
    for (; w + 4 <= Kw; w += 4) {
      a0 ^= gt[(w + 0) * 64 + lane] & u[w + 0];
      a1 ^= gt[(w + 1) * 64 + lane] & u[w + 1];
      a2 ^= gt[(w + 2) * 64 + lane] & u[w + 2];
      a3 ^= gt[(w + 3) * 64 + lane] & u[w + 3];
    }
    for (; w < Kw; ++w) a0 ^= gt[w * 64 + lane] & u[w];
    const int bit = __popcll(a0 ^ a1 ^ a2 ^ a3) & 1;
    const uint64_t mask = __ballot(bit);
    if (lane == 0) cc[(long long)(c0 + k) * Cw + par_word + blockIdx.x] = mask;
  }
}

// the info part of cc for the same codes: a word-aligned copy of uu's words
// [info_word0, info_word0 + n) to cc words [cc_word0, ...)
__global__ void encode_info_kernel(int B, int Kw, int Cw, int info_word0, int cc_word0, int n,
                                   const uint64_t *__restrict__ uu, uint64_t *__restrict__ cc) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)B * n) return;
  const int cw = (int)(gid / n), w = (int)(gid - (long long)cw * n);
  cc[(long long)cw * Cw + cc_word0 + w] = uu[(long long)cw * Kw + info_word0 + w];
}

// one thread per symbol: Mapping + y = x*h + n*(sigma/sqrt2)
__global__ __launch_bounds__(256) void channel_kernel(int bits, const double *__restrict__ cons, int S, int Cw, int B,
                                                      unsigned long long seed, unsigned long long first_cw,
                                                      double noise_scale, const uint64_t *__restrict__ cc,
                                                      double2 *__restrict__ y, double2 *__restrict__ hout) {
  const long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (gid >= (long long)B * S) return;
  const int cw = (int)(gid / S), j = (int)(gid - (long long)cw * S);
  const double2 g = gauss2(draw(seed, first_cw + cw, STREAM_H, 0));
  const double s5 = sqrt(0.5);
  const double hr = g.x * s5, hi = g.y * s5;
  if (j == 0) hout[cw] = make_double2(hr, hi);
  const uint64_t *c = cc + (long long)cw * Cw;
  int idx = 0;
  for (int b = 0; b < bits; ++b) {  // MSB-first label (modem.cc:14-17)
    const int pos = j * bits + b;
    idx = (idx << 1) + (int)((c[pos >> 6] >> (pos & 63)) & 1u);
  }
  const double xr = cons[2 * idx], xi = cons[2 * idx + 1];
  const double2 n = gauss2(draw(seed, first_cw + cw, STREAM_NOISE, (uint32_t)j));
  const double tr = xr * hr - xi * hi, ti = xr * hi + xi * hr;
  const double sr = n.x * noise_scale - n.y * 0.0, si = n.x * 0.0 + n.y * noise_scale;
  y[gid] = make_double2(tr + sr, ti + si);
}

}  // namespace

hipError_t launch_framegen(const DevCode &c, int bits, const double *cons, const FrameLaunch &f, hipStream_t s) {
  if (f.B == 0) return hipSuccess;
  const int Cw = (c.cc_len + 63) / 64;
  const int S = c.cc_len / bits;
  {
    const long long n = (long long)f.B * c.Kw;
    hipLaunchKernelGGL(source_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c.K, c.Kw, f.B, f.seed,
                       f.first_cw, c.active, f.uu_bits);
  }
  // word-aligned layout: PEG cc = [parity(chk) | info(K)]; 5G cc = info bits
  // [punct, K) then the parity bits (the first 2Z info bits are punctured)
  const int info_cc0 = c.is5g ? 0 : c.chk, par_cc0 = c.is5g ? c.K - c.punct : 0;
  const int info_u0 = c.is5g ? c.punct : 0, ninfo = c.is5g ? c.K - c.punct : c.K;
  const int npar = c.cc_len - ninfo;  // transmitted parity bits (rows 0..npar-1 of the generator)
  const size_t elds = sizeof(uint64_t) * ((size_t)c.Kw * 64 + (size_t)kEncCw * c.Kw);
  const bool aligned = c.active && npar > 0 && npar <= c.chk && npar % 64 == 0 && info_cc0 % 64 == 0 &&
                       par_cc0 % 64 == 0 && info_u0 % 64 == 0 && ninfo % 64 == 0 &&
                       (c.is5g ? par_cc0 + npar == c.cc_len : info_cc0 == npar) && elds <= 64 * 1024;
  if (aligned && !getenv("KML_ENCODE_LANE")) {
    hipLaunchKernelGGL(encode_parity_kernel, dim3((unsigned)(npar / 64), (unsigned)((f.B + kEncCw - 1) / kEncCw)),
                       dim3(256), elds, s, c, f.B, Cw, par_cc0 / 64, f.uu_bits, f.cc_bits);
    const long long n = (long long)f.B * (ninfo / 64);
    hipLaunchKernelGGL(encode_info_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, f.B, c.Kw, Cw,
                       info_u0 / 64, info_cc0 / 64, ninfo / 64, f.uu_bits, f.cc_bits);
  } else {
    const long long n = (long long)f.B * Cw * 64;
    hipLaunchKernelGGL(encode_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, c, f.B, Cw, f.uu_bits,
                       f.cc_bits);
  }
  {
    const long long n = (long long)f.B * S;
    hipLaunchKernelGGL(channel_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, bits, cons, S, Cw, f.B,
                       f.seed, f.first_cw, f.noise_scale, f.cc_bits, f.y, f.h);
  }
  return hipGetLastError();
}

}  // namespace kml
