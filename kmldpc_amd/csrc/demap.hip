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
#include <cmath>
#include <cstdlib>
#include <algorithm>

#include "demap_common.hpp"
#include "kernels.hpp"

namespace kml {

namespace {

// FAST (EXACT = false): every symbol on the proven FAST path; a symbol it
// cannot prove gets the sentinel p0 = -1 in its first bit and its index on the
// defer list (d.idx, up to d.cap entries; the count runs on past the cap).
// EXACT: the listed symbols on the exact path (div_rn, kml_exp), or, when the
// list overflowed, every symbol carrying the sentinel.
// 64QAM: the 64 probabilities of a symbol stay in registers (280 VGPRs
// unconstrained, one wave per SIMD); KML_DEMAP64_WAVES caps the kernel so that
// several waves per SIMD hide the exp table loads and the dependent chains
// (A/B) 1: the 64QAM demap_kernel reads bank-private copies of the exp table
// (demap_common.hpp stage_exp_table_banked).  Measured: 0.89 ms per 4096
// PEG8064 codewords against 0.87 with the plain table (profiles/r04_ab2_summary.txt):
// the bank conflicts were not on the kernel's critical path.
#ifndef KML_EXPTAB_BANKED
#define KML_EXPTAB_BANKED 0
#endif
// Round 4: 64QAM at 3 waves per SIMD (168 VGPRs: 37 spilled, as many as at
// 256), 16QAM at 4 (128 VGPRs, 2 spilled): 0.87 -> 0.84 ms and 0.295 -> 0.291
// ms per 4096 PEG8064 / 16384 BG2 codewords (profiles/r04_ab17_summary.txt)
#ifndef KML_DEMAP64_WAVES
#define KML_DEMAP64_WAVES 3
#endif
#ifndef KML_DEMAP16_WAVES
#define KML_DEMAP16_WAVES 4
#endif
template <int MB, bool EXACT, bool ROT = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MB >= 6 ? KML_DEMAP64_WAVES : MB == 4 ? KML_DEMAP16_WAVES : 1))) void demap_kernel(const double *__restrict__ cons, const double2 *__restrict__ y,
                                                    int S, int reps, const double2 *__restrict__ h, int h_stride,
                                                    const int32_t *__restrict__ h_sel, double var, int B,
                                                    double *__restrict__ p0, DemapDefer d) {
  __shared__ double cl[2 << MB];  // the constellation, read with uniform LDS loads
  // the exp table: bank-private copies for 64QAM (64 exps per symbol), the
  // plain table otherwise (demap_common.hpp stage_exp_table_banked)
  constexpr int ES = (MB >= 6 && KML_EXPTAB_BANKED) ? kExpBanked : 2;
  __shared__ uint64_t etab[ES == 2 ? 256 : 128 * kExpBanked];
  // ROT (64QAM, FAST, one symbol per thread, S >= 256: launch_demap): the
  // points times the channel of the (at most two) codewords of this
  // workgroup's symbols, formed once per workgroup instead of once per symbol
  static_assert(!ROT || !EXACT, "ROT: the FAST instance only");
  __shared__ double crot[ROT ? 4 << MB : 2];
  const long long n = (long long)B * S;
  long long todo = n;
  bool listed = false;
  if constexpr (EXACT) {
    const unsigned cnt = *d.cnt;
    if (cnt == 0) return;
    listed = cnt <= (unsigned)d.cap;
    if (listed) todo = cnt;
  }
  for (int k = threadIdx.x; k < (2 << MB); k += blockDim.x) cl[k] = cons[k];
  if constexpr (ES == 2)
    stage_exp_table(etab);
  else
    stage_exp_table_banked(etab);
  const int ent0 = (int)((long long)blockIdx.x * blockDim.x / S);
  if (ROT)
    for (int t = threadIdx.x; t < (2 << MB); t += blockDim.x) {
      const int e = ent0 + (t >> MB), k = t & ((1 << MB) - 1);
      if (e >= B) break;
      const double2 hh = h[(long long)e * h_stride + (h_sel ? h_sel[e] : 0)];
      const double cr = cons[2 * k], ci = cons[2 * k + 1];
      crot[2 * t] = cr * hh.x - ci * hh.y;  // the reference's symbol *= theta_h (demap_symbol_t)
      crot[2 * t + 1] = cr * hh.y + ci * hh.x;
    }
  __syncthreads();
  const lds_exptab et = (lds_exptab)etab + (ES == 2 ? 0 : 2 * (threadIdx.x & 15));
  // grid-stride over the symbols: the LDS staging above is paid once per
  // workgroup, not once per 256 symbols
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < todo; i += (long long)gridDim.x * blockDim.x) {
    const long long gid = listed ? (long long)(unsigned)d.idx[i] : i;
    if (EXACT && !listed && !(p0[gid * MB] < 0.0)) continue;
    const int ent = (int)(gid / S);
    const int j = (int)(gid - (long long)ent * S);
    const double2 hh = h[(long long)ent * h_stride + (h_sel ? h_sel[ent] : 0)];
    const double2 yy = y[(long long)(ent / reps) * S + j];
    double out[MB] = {};  // defined for the unconditional stores below
    bool ok = true;
    if constexpr (EXACT)
      demap_symbol_t<MB, false>((lds_cons)cl, (lds_exptab)etab, yy.x, yy.y, hh.x, hh.y, var, out);
    else if (ROT)
      ok = demap_symbol_t<MB, true, lds_cons, ES, true, ROT>((lds_cons)crot + ((ent - ent0) << (MB + 1)), et, yy.x,
                                                              yy.y, hh.x, hh.y, var, out);
    else
      ok = demap_symbol_t<MB, true, lds_cons, ES>((lds_cons)cl, et, yy.x, yy.y, hh.x, hh.y, var, out);
    // stored unconditionally: an unproven symbol gets the sentinel p0 = -1 in
    // its first bit (a P0 is in [1e-12, 1 - 1e-12]) and the EXACT instance
    // rewrites all its bits; no branch around the stores, so the outputs are
    // not spilled across a divergent join (64QAM: 48 B per symbol of scratch)
    if (!EXACT) out[0] = ok ? out[0] : -1.0;
#pragma unroll
    for (int b = 0; b < MB; ++b) p0[gid * MB + b] = out[b];
    if (!ok) {
      const unsigned k = atomicAdd(d.cnt, 1u);
      if (k < (unsigned)d.cap) d.idx[k] = (int32_t)gid;
    }
    if (ROT) break;  // one symbol per thread: no loop state held across the symbol
  }
}

// One codeword: hard decisions of its candidates into LDS, then the
// unsatisfied-check counts.  The (candidate, symbol) pairs are flattened over
// the workgroup; each symbol's decisions come from the single-precision screen
// (hard_bits_screen) unless a bit is too close to call, in which case the
// demapper decides: the FAST one (EXACT = false), which leaves the codeword to
// the EXACT kernel when it cannot prove a symbol (returns false, nothing
// written), or the exact one.
// 64QAM: the undecided (candidate, symbol) pairs are listed in LDS (up to
// kRescanCap; past it the second pass scans every pair for the mark), so the
// exact demapper runs on a dense list — one pass for the ~0.25 % undecided
// pairs of a codeword instead of one per wave-iteration that holds one.
constexpr int kRescanCap = 256;
template <int MB, bool EXACT>
__device__ __forceinline__ bool cand_metric_cw(int cw, const DevCode &c, const double2 *__restrict__ y, int S,
                                               const double2 *__restrict__ h4, int nc, double var, double inv_var,
                                               double *__restrict__ metrics, int32_t *__restrict__ chosen,
                                               unsigned char *smem, lds_cons cl, lds_exptab etab, lds_cons scr,
                                               double scb) {
  int *cnt = reinterpret_cast<int *>(smem);  // 4 counters, the undecided count, the unproven flag
  unsigned char *hb = smem + 32;             // [cc_len][4]: column-major, a row's parity of all candidates in one word
  int *und = reinterpret_cast<int *>(smem + 32 + ((4 * (size_t)c.cc_len + 3) & ~(size_t)3));  // [kRescanCap]
  constexpr bool kRescan = MB >= 5;
  const int tid = threadIdx.x;
  if (tid < 6) cnt[tid] = 0;
  __syncthreads();
  const double2 *yy = y + (long long)cw * S;
  // (candidate q, symbol j) of pair i = q S + j, advanced without a division
  int q = tid / S, j = tid - q * S;
  for (int i = tid; i < nc * S; i += blockDim.x, j += blockDim.x) {
    while (j >= S) {
      j -= S;
      ++q;
    }
    const double2 v = yy[j];
    const double2 hh = h4[(long long)cw * nc + q];
    unsigned bits;
    if (!hard_bits_screen<MB>(cl, scr, scb, v.x, v.y, hh.x, hh.y, inv_var, bits)) {
      if (kRescan) {
        hb[(j * MB) * 4 + q] = 2;  // undecided: the demap pass below
        const int u = atomicAdd(&cnt[4], 1);
        if (u < kRescanCap) und[u] = i;
        continue;
      }
      double out[MB];
      if constexpr (EXACT) {
        demap_symbol_t<MB, false>(cl, etab, v.x, v.y, hh.x, hh.y, var, out);
      } else if (!demap_symbol_t<MB, true>(cl, etab, v.x, v.y, hh.x, hh.y, var, out)) {
        cnt[5] = 1;
        continue;
      }
      bits = 0;
#pragma unroll
      for (int b = 0; b < MB; ++b) bits |= (out[b] > 0.5 ? 1u : 0u) << b;  // kmcodec.cc:111-115
    }
#pragma unroll
    for (int b = 0; b < MB; ++b) hb[(j * MB + b) * 4 + q] = (bits >> b) & 1;
  }
  __syncthreads();
  if (kRescan && cnt[4]) {  // 64QAM: the demapper in a pass of its own keeps its
                            // registers out of the screening loop's
    const int nu = cnt[4];
    const bool listed = nu <= kRescanCap;
    for (int u = tid; u < (listed ? nu : nc * S); u += blockDim.x) {
      const int i = listed ? und[u] : u;
      const int q = i / S, j = i - q * S;
      if (hb[(j * MB) * 4 + q] != 2) continue;
      const double2 v = yy[j];
      const double2 hh = h4[(long long)cw * nc + q];
      double out[MB];
      if constexpr (EXACT) {
        demap_symbol_t<MB, false>(cl, etab, v.x, v.y, hh.x, hh.y, var, out);
      } else if (!demap_symbol_t<MB, true>(cl, etab, v.x, v.y, hh.x, hh.y, var, out)) {
        cnt[5] = 1;
        continue;
      }
#pragma unroll
      for (int b = 0; b < MB; ++b) hb[(j * MB + b) * 4 + q] = out[b] > 0.5 ? 1 : 0;  // kmcodec.cc:111-115
    }
  }
  __syncthreads();
  if (!EXACT && cnt[5]) return false;  // uniform: every thread read the flag after the barrier
  int local[4] = {0, 0, 0, 0};
  const unsigned *hb32 = reinterpret_cast<const unsigned *>(hb);
#ifndef KML_CM_ROW6  // (A/B) 0: the generic row loop
#define KML_CM_ROW6 1
#endif
  if (KML_CM_ROW6 && c.regular && c.dc_max == 6) {  // (PEG codes) row r's edges at 6 r: three independent 8-byte loads
    for (int r = tid; r < c.M; r += blockDim.x) {
      const int2 *rc = reinterpret_cast<const int2 *>(c.row_col + 6 * r);  // 8-byte aligned (256-aligned base)
      const int2 e0 = rc[0], e1 = rc[1], e2 = rc[2];
      const unsigned p = hb32[e0.x] ^ hb32[e0.y] ^ hb32[e1.x] ^ hb32[e1.y] ^ hb32[e2.x] ^ hb32[e2.y];
#pragma unroll
      for (int q = 0; q < 4; ++q) local[q] += (p >> (8 * q)) & 1;
    }
  } else {
    for (int r = tid; r < c.M; r += blockDim.x) {
      unsigned p = 0;  // byte q: candidate q's parity (bytes of candidates >= nc unused)
      for (int e = c.row_ptr[r]; e < c.row_ptr[r + 1]; ++e) p ^= hb32[c.row_col[e]];
#pragma unroll
      for (int q = 0; q < 4; ++q) local[q] += (p >> (8 * q)) & 1;
    }
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
  __syncthreads();  // cnt and hb are reused by the next codeword
  return true;
}

// FAST: one workgroup per codeword, unproven codewords onto the defer list
// (at most B entries: d.cap >= B).  EXACT: the listed codewords, grid-stride.
template <int MB, bool EXACT>
// Minimum waves per SIMD of the metric kernel: <= 4-point sets 8 (64 VGPRs;
// 10 spilled, on the inline demap of undecided symbols only): QPSK 0.79 -> 0.66
// ms per 32768 codewords against the unconstrained 88 VGPRs / 5 waves (6 waves:
// 0.73; profiles/r04_ab9_summary.txt); 64QAM 4 (128 VGPRs: the 64 screen terms
// fit, the spills sit in the undecided list's exact demap): 0.73 -> 0.70 ms per
// 4096 PEG8064 codewords against 3 (r04_ab10_summary.txt).
#ifndef KML_CM_SMALL_WAVES
#define KML_CM_SMALL_WAVES 8
#endif
#ifndef KML_CM_BIG_WAVES
#define KML_CM_BIG_WAVES 4
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MB >= 6 ? KML_CM_BIG_WAVES : MB <= 2 ? KML_CM_SMALL_WAVES : 1))) void cand_metric_kernel(
    DevCode c, const double *__restrict__ cons, const double2 *__restrict__ y, int S, const double2 *__restrict__ h4,
    int nc, double var, double inv_var, double *__restrict__ metrics, int32_t *__restrict__ chosen, DemapDefer d) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ double cl[2 << MB];
  __shared__ double scr[3 << MB];  // the screen's (|c_k|^2, 2 Re c_k, 2 Im c_k)
  __shared__ double scb;           // the screen's bound on the constellation (hard_bits_screen)
  __shared__ uint64_t etab[256];
  unsigned todo = 1;
  if constexpr (EXACT) {
    todo = *d.cnt;
    if (blockIdx.x >= todo) return;
  }
  for (int k = threadIdx.x; k < (2 << MB); k += blockDim.x) cl[k] = cons[k];
  for (int k = threadIdx.x; k < (1 << MB); k += blockDim.x) {
    const double cr = cons[2 * k], ci = cons[2 * k + 1];
    scr[3 * k] = cr * cr + ci * ci;
    scr[3 * k + 1] = 2.0 * cr;
    scr[3 * k + 2] = 2.0 * ci;
  }
  if (threadIdx.x == 0) {  // max(max |c|^2, 2 max(|Re c|, |Im c|)), rounded up
    double b = 0.0;
    for (int k = 0; k < (1 << MB); ++k) {
      const double cr = cons[2 * k], ci = cons[2 * k + 1];
      b = fmax(b, fmax(cr * cr + ci * ci, 2.0 * fmax(fabs(cr), fabs(ci))));
    }
    scb = b * (1.0 + 0x1p-40);
  }
  stage_exp_table(etab);
  __syncthreads();
  if constexpr (EXACT) {
    for (unsigned i = blockIdx.x; i < todo; i += gridDim.x)
      cand_metric_cw<MB, true>(d.idx[i], c, y, S, h4, nc, var, inv_var, metrics, chosen, smem, (lds_cons)cl,
                               (lds_exptab)etab, (lds_cons)scr, scb);
  } else {
    const int cw = blockIdx.x;
    if (!cand_metric_cw<MB, false>(cw, c, y, S, h4, nc, var, inv_var, metrics, chosen, smem, (lds_cons)cl,
                                   (lds_exptab)etab, (lds_cons)scr, scb) &&
        threadIdx.x == 0)
      d.idx[atomicAdd(d.cnt, 1u)] = cw;
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
                        int h_stride, const int32_t *h_sel, double var, int B, double *p0, const DemapDefer &d,
                        hipStream_t s) {
  const long long n = (long long)B * S;
  if (n == 0) return hipSuccess;
  if (n > 0x7FFFFFFFLL || !d.idx || !d.cnt || d.cap < 1) return hipErrorInvalidValue;  // int32 symbol indices
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  // small constellations: 8 workgroups per CU, grid-stride; 64QAM (long
  // symbols): one symbol per thread
  const long long wg = (n + 255) / 256;
  const dim3 grid((unsigned)(bits >= 5 ? wg : std::min<long long>(wg, 8LL * ncu))), blk(256);
  const dim3 xgrid((unsigned)std::min<long long>(wg, 2LL * ncu));  // the exact pass: few symbols, or a scan
  hipError_t e = hipMemsetAsync(d.cnt, 0, sizeof(unsigned), s);
  if (e != hipSuccess) return e;
  switch (bits) {
#define KML_DM(MBV)                                                                                              \
  case MBV:                                                                                                      \
    hipLaunchKernelGGL((demap_kernel<MBV, false>), grid, blk, 0, s, cons, y, S, reps, h, h_stride, h_sel, var, B, \
                       p0, d);                                                                                   \
    hipLaunchKernelGGL((demap_kernel<MBV, true>), xgrid, blk, 0, s, cons, y, S, reps, h, h_stride, h_sel, var, B, \
                       p0, d);                                                                                   \
    break;
    KML_DM(1)
    KML_DM(2)
    KML_DM(3)
    KML_DM(4)
    case 6:
      // one symbol per thread and S >= 256: a workgroup's symbols span at most
      // two codewords, whose rotated points it stages (demap_kernel ROT)
      if (S >= 256)
        hipLaunchKernelGGL((demap_kernel<6, false, true>), grid, blk, 0, s, cons, y, S, reps, h, h_stride, h_sel, var,
                           B, p0, d);
      else
        hipLaunchKernelGGL((demap_kernel<6, false>), grid, blk, 0, s, cons, y, S, reps, h, h_stride, h_sel, var, B, p0,
                           d);
      hipLaunchKernelGGL((demap_kernel<6, true>), xgrid, blk, 0, s, cons, y, S, reps, h, h_stride, h_sel, var, B, p0, d);
      break;
#undef KML_DM
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_cand_metric(const DevCode &c, int bits, const double *cons, const double2 *y, int S,
                              const double2 *h4, int nc, double var, int B, double *metrics, int32_t *chosen,
                              const DemapDefer &d, hipStream_t s) {
  if (B == 0) return hipSuccess;
  if (nc < 1 || nc > 4) return hipErrorInvalidValue;
  if (!d.idx || !d.cnt || d.cap < B) return hipErrorInvalidValue;  // every codeword may defer
  const size_t lds = 32 + ((4 * (size_t)c.cc_len + 3) & ~(size_t)3) + (bits >= 5 ? 4 * (size_t)kRescanCap : 0);
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  const dim3 grid(B), xgrid((unsigned)std::min(B, 2 * ncu)), blk(256);
  // KML_CM_NOSCREEN=1 (tests): a NaN 1 / var fails every screen (hard_bits_screen
  // returns false), so every (candidate, symbol) takes the demapper
  double iv = 1.0 / var;
  if (const char *ev = getenv("KML_CM_NOSCREEN"))
    if (ev[0] == '1') iv = NAN;
  hipError_t e = hipMemsetAsync(d.cnt, 0, sizeof(unsigned), s);
  if (e != hipSuccess) return e;
  switch (bits) {
#define KML_CM(MBV)                                                                                             \
  case MBV: {                                                                                                   \
    e = hipFuncSetAttribute((const void *)cand_metric_kernel<MBV, false>,                                       \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                              \
    if (e == hipSuccess)                                                                                        \
      e = hipFuncSetAttribute((const void *)cand_metric_kernel<MBV, true>,                                      \
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);                            \
    if (e != hipSuccess) return e;                                                                              \
    hipLaunchKernelGGL((cand_metric_kernel<MBV, false>), grid, blk, lds, s, c, cons, y, S, h4, nc, var, iv,       \
                       metrics, chosen, d);                                                                     \
    hipLaunchKernelGGL((cand_metric_kernel<MBV, true>), xgrid, blk, lds, s, c, cons, y, S, h4, nc, var, iv,      \
                       metrics, chosen, d);                                                                     \
    break;                                                                                                      \
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
