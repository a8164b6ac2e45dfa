// demap.hip — soft demapper, blind-candidate metric and error counting.
//
//   demap_kernel     ModemLinearSystem::SoftAWGNDemodulation
//                    (lib/lab/src/modemlinearsystem.cc:51-79) followed by
//                    Modem::DeMapping with bitLin = 0.5 (lib/lab/src/modem.cc:23-79;
//                    KmCodec::DeMapping sets bit_l_in_ = 0.5, src/kmcodec.cc:96-98).
//                    One thread per (codeword, symbol); the K-point loops run in
//                    ascending k like the reference's sequential sums.
//   cand_metric      KmCodec::GetMetrics + Metric with metric_type = false on a
//                    PEG code (src/kmcodec.cc:122-142, :105-119): per codeword and
//                    rotated estimate, count unsatisfied checks of rr = (P0 > 0.5);
//                    argmin with first-minimum tie break (:59-65).  One workgroup
//                    per codeword; hard decisions staged in LDS.
//   select_kernel    the same argmin for the BP-based metrics (5G, :157-160).
//   count_bytes      SourceSink::CntErr (lib/lab/src/sourcesink.cc:29-47).
//
// Numerics: every operation is the reference's IEEE operation in the
// reference's order; exp() is kml_exp, a bit-exact restatement of the glibc exp
// the reference calls (the ROCm device exp differs from it in the last bit on
// ~6% of inputs), so P0 is bit-identical to the CPU path.
#include <algorithm>

#include "demap_common.hpp"
#include "kernels.hpp"

namespace kml {

namespace {

template <int MB>
__global__ __launch_bounds__(256) void demap_kernel(const double *__restrict__ cons, const double2 *__restrict__ y,
                                                    int S, int reps, const double2 *__restrict__ h, int h_stride,
                                                    const int32_t *__restrict__ h_sel, double var, int B,
                                                    double *__restrict__ p0) {
  __shared__ double cl[2 << MB];  // the constellation, read with uniform LDS loads
  __shared__ uint64_t etab[256];
  for (int k = threadIdx.x; k < (2 << MB); k += blockDim.x) cl[k] = cons[k];
  stage_exp_table(etab);
  __syncthreads();
  // grid-stride over the symbols: the LDS staging above is paid once per
  // workgroup, not once per 256 symbols
  const long long n = (long long)B * S;
  for (long long gid = (long long)blockIdx.x * blockDim.x + threadIdx.x; gid < n;
       gid += (long long)gridDim.x * blockDim.x) {
    const int ent = (int)(gid / S);
    const int j = (int)(gid - (long long)ent * S);
    const double2 hh = h[(long long)ent * h_stride + (h_sel ? h_sel[ent] : 0)];
    const double2 yy = y[(long long)(ent / reps) * S + j];
    double out[MB];
    demap_symbol<MB>((lds_cons)cl, (lds_exptab)etab, yy.x, yy.y, hh.x, hh.y, var, out);
#pragma unroll
    for (int b = 0; b < MB; ++b) p0[gid * MB + b] = out[b];
  }
}

// One workgroup per codeword: hard decisions of the candidates into LDS, then
// the unsatisfied-check counts.  The (candidate, symbol) pairs are flattened
// over the workgroup; each symbol's decisions come from the single-precision
// screen (hard_bits_screen) unless a bit is too close to call, in which case
// the exact demapper decides.
template <int MB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MB >= 6 ? 3 : 1))) void cand_metric_kernel(DevCode c, const double *__restrict__ cons,
                                                          const double2 *__restrict__ y, int S,
                                                          const double2 *__restrict__ h4, int nc, double var,
                                                          double inv_var, double *__restrict__ metrics,
                                                          int32_t *__restrict__ chosen) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int *cnt = reinterpret_cast<int *>(smem);  // 4 counters + the undecided flag
  unsigned char *hb = smem + 32;             // [4][cc_len]
  constexpr bool kRescan = MB >= 5;
  const int cw = blockIdx.x;
  const int tid = threadIdx.x;
  __shared__ double cl[2 << MB];
  __shared__ uint64_t etab[256];
  for (int k = tid; k < (2 << MB); k += blockDim.x) cl[k] = cons[k];
  stage_exp_table(etab);
  if (tid < 5) cnt[tid] = 0;
  __syncthreads();
  const double2 *yy = y + (long long)cw * S;
  for (int i = tid; i < nc * S; i += blockDim.x) {
    const int q = i / S, j = i - q * S;
    const double2 v = yy[j];
    const double2 hh = h4[(long long)cw * nc + q];
    unsigned bits;
    if (!hard_bits_screen<MB>((lds_cons)cl, v.x, v.y, hh.x, hh.y, inv_var, bits)) {
      if (kRescan) {
        hb[q * c.cc_len + j * MB] = 2;  // undecided: the exact pass below
        cnt[4] = 1;
        continue;
      }
      double out[MB];
      demap_symbol<MB>((lds_cons)cl, (lds_exptab)etab, v.x, v.y, hh.x, hh.y, var, out);
      bits = 0;
#pragma unroll
      for (int b = 0; b < MB; ++b) bits |= (out[b] > 0.5 ? 1u : 0u) << b;  // kmcodec.cc:111-115
    }
#pragma unroll
    for (int b = 0; b < MB; ++b) hb[q * c.cc_len + j * MB + b] = (bits >> b) & 1;
  }
  __syncthreads();
  if (kRescan && cnt[4]) {  // 64QAM: the exact demapper in a pass of its own
                            // keeps its registers out of the screening loop's
    for (int i = tid; i < nc * S; i += blockDim.x) {
      const int q = i / S, j = i - q * S;
      if (hb[q * c.cc_len + j * MB] != 2) continue;
      const double2 v = yy[j];
      const double2 hh = h4[(long long)cw * nc + q];
      double out[MB];
      demap_symbol<MB>((lds_cons)cl, (lds_exptab)etab, v.x, v.y, hh.x, hh.y, var, out);
#pragma unroll
      for (int b = 0; b < MB; ++b) hb[q * c.cc_len + j * MB + b] = out[b] > 0.5 ? 1 : 0;  // kmcodec.cc:111-115
    }
  }
  __syncthreads();
  int local[4] = {0, 0, 0, 0};
  for (int r = tid; r < c.M; r += blockDim.x) {
    int p[4] = {0, 0, 0, 0};
    for (int e = c.row_ptr[r]; e < c.row_ptr[r + 1]; ++e) {
      const int col = c.row_col[e];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (q < nc) p[q] ^= hb[q * c.cc_len + col];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) local[q] += p[q];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (local[q]) atomicAdd(&cnt[q], local[q]);
  __syncthreads();
  if (tid == 0) {
    int best = 0;
    for (int q = 0; q < 4; ++q) {
      metrics[(long long)cw * 4 + q] = q < nc ? fabs((double)cnt[q]) : 0.0;
      if (q < nc && cnt[q] < cnt[best]) best = q;
    }
    chosen[cw] = best;
  }
}

__global__ void select_kernel(const int32_t *__restrict__ pc, int nc, int B, double *__restrict__ metrics,
                              int32_t *__restrict__ chosen) {
  const int cw = blockIdx.x * blockDim.x + threadIdx.x;
  if (cw >= B) return;
  int best = 0;
  for (int q = 0; q < 4; ++q) {
    metrics[(long long)cw * 4 + q] = q < nc ? fabs((double)pc[(long long)cw * nc + q]) : 0.0;
    if (q < nc && pc[(long long)cw * nc + q] < pc[(long long)cw * nc + best]) best = q;
  }
  chosen[cw] = best;
}

// SourceSink::CntErr (sourcesink.cc:29-47) of byte decisions uh (NULL = all
// zero) against bit-packed reference words; one wave per codeword.
__global__ __launch_bounds__(64) void count_packed_kernel(const uint64_t *__restrict__ ref, int Kw, int K,
                                                          const uint8_t *__restrict__ uh, long long uh_stride, int B,
                                                          int32_t *__restrict__ cw_err,
                                                          unsigned long long *__restrict__ counters) {
  const int cw = blockIdx.x;
  const int lane = threadIdx.x;
  int errs = 0;
  for (int w = lane; w < Kw; w += 64) {
    uint64_t word = 0;
    const int base = w * 64;
    const int nb = min(64, K - base);
    if (uh)
      for (int j = 0; j < nb; ++j) word |= (uint64_t)(uh[(long long)cw * uh_stride + base + j] & 1) << j;
    errs += __popcll(word ^ ref[(long long)cw * Kw + w]);
  }
  for (int off = 32; off > 0; off >>= 1) errs += __shfl_xor(errs, off);
  if (lane == 0) {
    if (cw_err) cw_err[cw] = errs;
    atomicAdd(&counters[CNT_ERR_BIT], (unsigned long long)errs);
    atomicAdd(&counters[CNT_ERR_BLK], errs > 0 ? 1ull : 0ull);
    atomicAdd(&counters[CNT_TOT_BIT], (unsigned long long)K);
    atomicAdd(&counters[CNT_TOT_BLK], 1ull);
  }
}

__global__ void count_bytes_kernel(const uint8_t *__restrict__ uu, const uint8_t *__restrict__ uh, int K, int B,
                                   unsigned long long *counters) {
  // one workgroup per codeword
  __shared__ int errs;
  const int cw = blockIdx.x;
  if (threadIdx.x == 0) errs = 0;
  __syncthreads();
  int e = 0;
  for (int i = threadIdx.x; i < K; i += blockDim.x) e += (uu[(long long)cw * K + i] != uh[(long long)cw * K + i]);
  if (e) atomicAdd(&errs, e);
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(&counters[CNT_ERR_BIT], (unsigned long long)errs);
    atomicAdd(&counters[CNT_ERR_BLK], errs > 0 ? 1ull : 0ull);
    atomicAdd(&counters[CNT_TOT_BIT], (unsigned long long)K);
    atomicAdd(&counters[CNT_TOT_BLK], 1ull);
  }
}

// KmCodec::Metric, soft branch (src/kmcodec.cc:150-156): L = sum_{j<M} log(syn[j])
// accumulated in row order from 0.0 like the reference's loop, with the
// glibc-exact log.  One wave per entry (list[i] or i); entries whose decode ran
// no CN phase (iters == 0) keep their L (the caller resolves them as stale).
__global__ __launch_bounds__(64) void soft_sum_kernel(const double *__restrict__ syn, int M,
                                                      const int32_t *__restrict__ iters,
                                                      const int32_t *__restrict__ list, double *__restrict__ L) {
  extern __shared__ double lg[];
  const int e = list ? list[blockIdx.x] : (int)blockIdx.x;
  if (iters && iters[e] == 0) return;
  const double *s = syn + (long long)e * M;
  for (int j = threadIdx.x; j < M; j += 64) lg[j] = kml_log(s[j]);
  __syncthreads();
  if (threadIdx.x == 0) {
    double acc = 0.0;
    for (int j = 0; j < M; ++j) acc += lg[j];
    L[e] = acc;
  }
}

}  // namespace

hipError_t launch_soft_sum(const double *syn, int M, const int32_t *iters, const int32_t *list, int n, double *L,
                           hipStream_t s) {
  if (n == 0) return hipSuccess;
  const size_t lds = sizeof(double) * (size_t)M;
  if (lds > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute((const void *)soft_sum_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                       (int)lds);
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(soft_sum_kernel, dim3(n), dim3(64), lds, s, syn, M, iters, list, L);
  return hipGetLastError();
}

hipError_t launch_demap(int bits, const double *cons, const double2 *y, int S, int reps, const double2 *h,
                        int h_stride, const int32_t *h_sel, double var, int B, double *p0, hipStream_t s) {
  const long long n = (long long)B * S;
  if (n == 0) return hipSuccess;
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  // small constellations: 8 workgroups per CU, grid-stride; 64QAM (three
  // waves per SIMD, long symbols): one symbol per thread
  const long long wg = (n + 255) / 256;
  const dim3 grid((unsigned)(bits >= 5 ? wg : std::min<long long>(wg, 8LL * ncu))), blk(256);
  switch (bits) {
    case 1: hipLaunchKernelGGL(demap_kernel<1>, grid, blk, 0, s, cons, y, S, reps, h, h_stride, h_sel, var, B, p0); break;
    case 2: hipLaunchKernelGGL(demap_kernel<2>, grid, blk, 0, s, cons, y, S, reps, h, h_stride, h_sel, var, B, p0); break;
    case 3: hipLaunchKernelGGL(demap_kernel<3>, grid, blk, 0, s, cons, y, S, reps, h, h_stride, h_sel, var, B, p0); break;
    case 4: hipLaunchKernelGGL(demap_kernel<4>, grid, blk, 0, s, cons, y, S, reps, h, h_stride, h_sel, var, B, p0); break;
    case 6: hipLaunchKernelGGL(demap_kernel<6>, grid, blk, 0, s, cons, y, S, reps, h, h_stride, h_sel, var, B, p0); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_cand_metric(const DevCode &c, int bits, const double *cons, const double2 *y, int S,
                              const double2 *h4, int nc, double var, int B, double *metrics, int32_t *chosen,
                              hipStream_t s) {
  if (B == 0) return hipSuccess;
  if (nc < 1 || nc > 4) return hipErrorInvalidValue;
  const size_t lds = 32 + 4 * (size_t)c.cc_len;
  const dim3 grid(B), blk(256);
  switch (bits) {
#define KML_CM(MBV)                                                                                          \
  case MBV: {                                                                                                \
    hipError_t e = hipFuncSetAttribute((const void *)cand_metric_kernel<MBV>,                                \
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                \
    if (e != hipSuccess) return e;                                                                           \
    hipLaunchKernelGGL(cand_metric_kernel<MBV>, grid, blk, lds, s, c, cons, y, S, h4, nc, var, 1.0 / var, metrics, \
                       chosen);                                                                              \
    break;                                                                                                   \
  }
    KML_CM(1)
    KML_CM(2)
    KML_CM(3)
    KML_CM(4)
    KML_CM(6)
#undef KML_CM
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_select(const int32_t *parity_cnt, int nc, int B, double *metrics, int32_t *chosen, hipStream_t s) {
  if (B == 0) return hipSuccess;
  hipLaunchKernelGGL(select_kernel, dim3((B + 255) / 256), dim3(256), 0, s, parity_cnt, nc, B, metrics, chosen);
  return hipGetLastError();
}

hipError_t launch_count_packed(const uint64_t *ref, int Kw, int K, const uint8_t *uh, long long uh_stride, int B,
                               int32_t *cw_err, unsigned long long *counters, hipStream_t s) {
  if (B == 0) return hipSuccess;
  hipLaunchKernelGGL(count_packed_kernel, dim3(B), dim3(64), 0, s, ref, Kw, K, uh, uh_stride, B, cw_err, counters);
  return hipGetLastError();
}

hipError_t launch_count_bytes(const uint8_t *uu, const uint8_t *uu_hat, int K, int B, unsigned long long *counters,
                              hipStream_t s) {
  if (B == 0) return hipSuccess;
  hipLaunchKernelGGL(count_bytes_kernel, dim3(B), dim3(256), 0, s, uu, uu_hat, K, B, counters);
  return hipGetLastError();
}

}  // namespace kml
