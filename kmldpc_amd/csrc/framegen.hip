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
  {
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
