// bp_static.hip — the LDS-resident BP decoder with a static thread -> column /
// row assignment (the production kernel for codes whose message state fits in
// LDS: PEG2304, 5G BG2 K960).
//
// Same arithmetic as bp.hip (bit-exact restatement of
// lib/lab/src/binaryldpccodec.cc:165-278 / binary5gldpccodec.cc:112-232); what
// changes is how the work meets the hardware:
//   * every thread owns RV fixed columns and RC fixed rows for the whole
//     launch; their slot ids, degrees and (for the parity check) column ids are
//     read once per workgroup into registers, so an iteration touches no
//     global memory at all (P0 is read into registers once per codeword);
//   * inside a phase each thread first gathers all message slots of all its
//     columns (rows), then runs the independent chains back to back, then
//     scatters the results: RV (RC) independent dependency chains per thread
//     give the scheduler instruction-level parallelism to hide the fp64
//     division latency;
//   * the two quotients of every normalisation share one reciprocal
//     refinement (div2 in bp_common.hpp), bit-identical to two IEEE divisions
//     for the value ranges the caller validates per codeword.
#include "bp_common.hpp"
#include "kernels.hpp"

namespace kml {

namespace {

constexpr int kRedBytes = 16;

template <int T, int RV, int RC, int DV, int DC, bool REG, bool SYN, bool FAST>
__device__ __forceinline__ void decode_cw(const DevCode &c, const BpLaunch &a, int cw, double2 *slots,
                                          unsigned char *cch, const int (&vcol)[RV], const int (&vdeg)[RV],
                                          const int (&vslot)[RV][DV], const double (&pv)[RV], const int (&crow)[RC],
                                          const int (&cbase)[RC], const int (&cdeg)[RC], const int (&ccol)[RC][DC],
                                          int &iter_out, bool &conv_out) {
  int iter = 0;
  bool conv = false;
  for (; iter < a.iter_count; ++iter) {
    // ------------------------------------------------------------ VN phase
    {
      double c0s[RV][DV];
#pragma unroll
      for (int r = 0; r < RV; ++r)
#pragma unroll
        for (int k = 0; k < DV; ++k) c0s[r][k] = (k < (REG ? (vcol[r] >= 0 ? DV : 0) : vdeg[r])) ? slots[vslot[r][k]].x : 0.5;
#pragma unroll
      for (int r = 0; r < RV; ++r) {
        if (REG && vcol[r] < 0) continue;  // wave-uniform (only the tail round can be partial)
        const int d = REG ? DV : vdeg[r];
        double a0 = pv[r], a1 = 1.0 - pv[r];
        double al0[DV], al1[DV];
#pragma unroll
        for (int k = 0; k < DV; ++k) {
          al0[k] = a0;
          al1[k] = a1;
          if (k < d) {
            const double c0 = c0s[r][k];
            const double n0 = a0 * c0;
            const double n1 = a1 * (1.0 - c0);
            div2<FAST>(n0, n1, n0 + n1, a0, a1);
          }
        }
        if (vcol[r] >= 0) cch[vcol[r]] = (a0 > a1) ? 0 : 1;
        double b0 = 1.0, b1 = 1.0;
#pragma unroll
        for (int k = DV - 1; k >= 0; --k) {
          if (k < d) {
            const double t0 = al0[k] * b0;
            const double t1 = al1[k] * b1;
            double q0, q1;
            div2<FAST>(t0, t1, t0 + t1, q0, q1);
            slots[vslot[r][k]] = make_double2(q0, q1);  // all of this phase's loads are done
            if (k > 0) {
              const double c0 = c0s[r][k];
              const double n0 = b0 * c0;
              const double n1 = b1 * (1.0 - c0);
              div2<FAST>(n0, n1, n0 + n1, b0, b1);
            }
          }
        }
      }
    }
    __syncthreads();

    // ------------------------------------------------ early-stop parity check
    int fail = 0;
#pragma unroll
    for (int r = 0; r < RC; ++r) {
      int p = 0;
#pragma unroll
      for (int k = 0; k < DC; ++k)
        if (k < cdeg[r]) p ^= cch[ccol[r][k]];
      fail |= p;
    }
    if (!__syncthreads_or(fail)) {
      conv = true;
      break;
    }

    // ------------------------------------------------------------ CN phase
    {
      double v0[RC][DC], v1[RC][DC];
#pragma unroll
      for (int r = 0; r < RC; ++r)
#pragma unroll
        for (int k = 0; k < DC; ++k) {
          double2 m = make_double2(0.5, 0.5);
          if (k < (REG ? (crow[r] >= 0 ? DC : 0) : cdeg[r])) m = slots[cbase[r] + k];
          v0[r][k] = m.x;
          v1[r][k] = m.y;
        }
#pragma unroll
      for (int r = 0; r < RC; ++r) {
        if (REG && crow[r] < 0) continue;
        const int d = REG ? DC : cdeg[r];
        double al0[DC], al1[DC];
        double a0 = 1.0, a1 = 0.0;
#pragma unroll
        for (int k = 0; k < DC; ++k) {
          al0[k] = a0;
          al1[k] = a1;
          if (k < d && (SYN || k + 1 < d)) {
            const double n0 = a0 * v0[r][k] + a1 * v1[r][k];
            const double n1 = a0 * v1[r][k] + a1 * v0[r][k];
            div2<FAST>(n0, n1, n0 + n1, a0, a1);
          }
        }
        if constexpr (SYN)
          if (crow[r] >= 0) a.syn[(long long)cw * c.M + crow[r]] = a0;
        double b0 = 1.0, b1 = 0.0;
#pragma unroll
        for (int k = DC - 1; k >= 0; --k) {
          if (k < d) {
            const double t0 = al0[k] * b0 + al1[k] * b1;
            const double t1 = al0[k] * b1 + al1[k] * b0;
            double q = div1<FAST>(t0, t0 + t1);
            if (q > 1.0 - kSmallestProb) q = 1.0 - kSmallestProb;
            if (q < kSmallestProb) q = kSmallestProb;
            slots[cbase[r] + k].x = q;
            if (k > 0) {
              const double n0 = b0 * v0[r][k] + b1 * v1[r][k];
              const double n1 = b0 * v1[r][k] + b1 * v0[r][k];
              div2<FAST>(n0, n1, n0 + n1, b0, b1);
            }
          }
        }
      }
    }
    __syncthreads();
  }
  iter_out = iter;
  conv_out = conv;
}

template <int T, int RV, int RC, int DV, int DC, bool REG, bool SYN>
__global__ __launch_bounds__(T) void bp_static_kernel(DevCode c, BpLaunch a, unsigned int *queue, int fast_allowed) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  double2 *slots = reinterpret_cast<double2 *>(smem);
  int *red = reinterpret_cast<int *>(smem + (size_t)c.E * 16);
  unsigned char *cch = smem + (size_t)c.E * 16 + kRedBytes;

  // static assignment (read once per workgroup)
  int vcol[RV], vdeg[RV], vslot[RV][DV];
#pragma unroll
  for (int r = 0; r < RV; ++r) {
    const int idx = r * T + tid;
    vcol[r] = -1;
    vdeg[r] = 0;
    if (idx < c.N) {
      const int v = c.vn_order[idx];
      const int b = c.col_ptr[v];
      vcol[r] = v;
      vdeg[r] = c.col_ptr[v + 1] - b;
#pragma unroll
      for (int k = 0; k < DV; ++k) vslot[r][k] = (k < vdeg[r]) ? c.col_slot[b + k] : 0;
    } else {
#pragma unroll
      for (int k = 0; k < DV; ++k) vslot[r][k] = 0;
    }
  }
  int crow[RC], cbase[RC], cdeg[RC], ccol[RC][DC];
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int idx = r * T + tid;
    crow[r] = -1;
    cbase[r] = 0;
    cdeg[r] = 0;
    if (idx < c.M) {
      const int row = c.cn_order[idx];
      crow[r] = row;
      cbase[r] = c.row_ptr[row];
      cdeg[r] = c.row_ptr[row + 1] - cbase[r];
    }
#pragma unroll
    for (int k = 0; k < DC; ++k) ccol[r][k] = (k < cdeg[r]) ? c.row_col[cbase[r] + k] : 0;
  }

  for (;;) {
    __syncthreads();
    if (tid == 0) {
      red[3] = (int)atomicAdd(queue, 1u);
      red[0] = 0;
      red[1] = 0;
    }
    __syncthreads();
    const int entry = red[3];
    if (entry >= a.B) break;
    const int cw = a.cw_idx ? a.cw_idx[entry] : entry;
    const double *p0 = a.p0 + (long long)cw * a.p0_stride;
    if (a.p0_sel) p0 += (long long)a.p0_sel[cw] * a.p0_sel_stride;

    double pv[RV];
    bool ok = true;
#pragma unroll
    for (int r = 0; r < RV; ++r) {
      pv[r] = (vcol[r] >= c.punct) ? p0[vcol[r] - c.punct] : 0.5;  // punctured prior (binary5gldpccodec.cc:126-129)
      ok = ok && fast_prior_ok(pv[r]);
    }
    for (int e = tid; e < c.E; e += T) slots[e].x = 0.5;  // InitMsg
    const bool fast = __syncthreads_and(ok ? 1 : 0) && fast_allowed;

    int iter = 0;
    bool conv = false;
    if (fast)
      decode_cw<T, RV, RC, DV, DC, REG, SYN, true>(c, a, cw, slots, cch, vcol, vdeg, vslot, pv, crow, cbase, cdeg, ccol,
                                             iter, conv);
    else
      decode_cw<T, RV, RC, DV, DC, REG, SYN, false>(c, a, cw, slots, cch, vcol, vdeg, vslot, pv, crow, cbase, cdeg, ccol,
                                              iter, conv);

    // ---------------- epilogue (same contract as bp.hip)
    if (a.iter_count > 0) {
      if (a.uu_hat) {
        uint8_t *u = a.uu_hat + (long long)cw * c.K;
        for (int i = tid; i < c.K; i += T) u[i] = cch[i + c.info_off];
      }
      if (a.cc_hat) {
        uint8_t *o = a.cc_hat + (long long)cw * c.N;
        for (int v = tid; v < c.N; v += T) o[v] = cch[v];
      }
      if (a.parity_cnt) {
        int cnt = 0;
#pragma unroll
        for (int r = 0; r < RC; ++r) {
          int p = 0;
#pragma unroll
          for (int k = 0; k < DC; ++k)
            if (k < cdeg[r]) p ^= cch[ccol[r][k]];
          cnt += p;
        }
        if (cnt) atomicAdd(&red[0], cnt);
      }
      if (a.ref_bits) {
        const uint64_t *ref = a.ref_bits + (long long)cw * c.Kw;
        int errs = 0;
        for (int w = tid; w < c.Kw; w += T) {
          uint64_t word = 0;
          const int base = w * 64;
          const int nb = min(64, c.K - base);
          for (int j = 0; j < nb; ++j) word |= (uint64_t)cch[c.info_off + base + j] << j;
          errs += __popcll(word ^ ref[w]);
        }
        if (errs) atomicAdd(&red[1], errs);
      }
    }
    __syncthreads();
    if (tid == 0) {
      if (a.ret) a.ret[cw] = iter + (iter < a.max_iter);
      if (a.parity_cnt) a.parity_cnt[cw] = red[0];
      if (a.cw_err && a.ref_bits) a.cw_err[cw] = a.iter_count > 0 ? red[1] : 0;
      if (a.iters) a.iters[cw] = iter;
      if (a.counters) {
        const unsigned long long vn = conv ? (unsigned long long)iter + 1 : (unsigned long long)iter;
        atomicAdd(&a.counters[CNT_VN_PHASES], vn);
        atomicAdd(&a.counters[CNT_CN_PHASES], (unsigned long long)iter);
        if (conv) atomicAdd(&a.counters[CNT_CONVERGED], 1ull);
        if (a.ref_bits && a.iter_count > 0) {
          const int errs = red[1];
          atomicAdd(&a.counters[CNT_ERR_BIT], (unsigned long long)errs);
          atomicAdd(&a.counters[CNT_ERR_BLK], errs > 0 ? 1ull : 0ull);
          atomicAdd(&a.counters[CNT_TOT_BIT], (unsigned long long)c.K);
          atomicAdd(&a.counters[CNT_TOT_BLK], 1ull);
        }
      }
    }
  }
}

template <int T, int RV, int RC, int DV, int DC, bool REG, bool SYN>
hipError_t launch_static_t(const DevCode &c, const BpLaunch &a, hipStream_t s, int fast_allowed) {
  auto kern = bp_static_kernel<T, RV, RC, DV, DC, REG, SYN>;
  const size_t lds = (size_t)c.E * 16 + kRedBytes + (size_t)c.N;
  hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  long long grid = ncu;
  if (grid > a.B) grid = a.B;
  e = hipMemsetAsync(a.queue, 0, sizeof(unsigned int), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(T), lds, s, c, a, a.queue, fast_allowed);
  return hipGetLastError();
}

constexpr int kStaticThreads = 768;

}  // namespace

// Returns hipErrorNotSupported when the static kernel has no instantiation for
// this code (the caller then uses the generic kernel).
hipError_t launch_bp_static(const DevCode &c, const BpLaunch &a, hipStream_t s) {
  constexpr int T = kStaticThreads;
  const int rv = (c.N + T - 1) / T, rc = (c.M + T - 1) / T;
  const int fast = c.dv_max <= kFastMaxColumnDegree ? 1 : 0;
  if ((long long)c.E * 16 + kRedBytes + c.N > 160 * 1024) return hipErrorNotSupported;
  if (rv <= 3 && rc <= 2) {
    // regular (3,6) code: every column has degree 3 and every row degree 6
    if (c.regular && c.dv_max == 3 && c.dc_max == 6)
      return a.syn ? launch_static_t<T, 3, 2, 3, 6, true, true>(c, a, s, fast)
                   : launch_static_t<T, 3, 2, 3, 6, true, false>(c, a, s, fast);
    if (c.dv_max <= 3 && c.dc_max <= 6)
      return a.syn ? launch_static_t<T, 3, 2, 3, 6, false, true>(c, a, s, fast)
                   : launch_static_t<T, 3, 2, 3, 6, false, false>(c, a, s, fast);
  }
  return hipErrorNotSupported;
}

}  // namespace kml
