// bp_irregular.hip — BP decoder for irregular codes whose message state fits
// in LDS (5G BG2 K960: 7,392 edges, column degrees {1,2,3,4,5,7,9}, row
// degrees {4,5,6,8,10}).
//
// Arithmetic: bit-exact restatement of lab::Binary5GLDPCCodec::Decoder /
// lab::BinaryLDPCCodec::Decoder (lib/lab/src/binary5gldpccodec.cc:112-232,
// binaryldpccodec.cc:165-278), like the other BP kernels; the punctured 5G
// columns get the prior (0.5, 1 - 0.5) (binary5gldpccodec.cc:126-129).
//
// Mapping (one workgroup of T threads per CU, persistent over codewords):
//   * message slots (16 B per edge), the codeword's priors and the
//     column->slot table (u16) in LDS;
//   * thread t owns vn positions r*T + t and half-rows r*T + t; the planner
//     sorts columns and rows by degree, so a wave almost always runs one
//     degree, and every degree has its own fully unrolled instance (the chain
//     states stay in registers);
//   * check rows are split over lane pairs exactly like bp_regular.hip: the
//     even lane runs the forward trellis, the odd lane the backward one, DPP
//     swaps exchange the chain states, each lane finishes half of the row's
//     c2v messages (for an odd degree the even lane also takes the middle
//     edge, from the two states both lanes hold at that step);
//   * the shared-reciprocal exact division (bp_common.hpp) on codewords whose
//     priors qualify.
#include "bp_common.hpp"
#include "kernels.hpp"

namespace kml {

namespace {

constexpr int kRedBytes = 16;

__device__ __forceinline__ double swap_pair(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  const int lo2 = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, false);
  const int hi2 = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi2, lo2);
}
__device__ __forceinline__ int swap_pair_i(int x) { return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false); }

// One column of degree D (binaryldpccodec.cc:177-213).
template <int D, bool FAST>
__device__ __forceinline__ void vn_column(double2 *slots, const unsigned short *cs, double p, unsigned char *hard) {
  double c0s[D];
#pragma unroll
  for (int k = 0; k < D; ++k) c0s[k] = slots[cs[k]].x;
  double a0 = p, a1 = 1.0 - p, al0[D], al1[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    al0[k] = a0;
    al1[k] = a1;
    const double n0 = a0 * c0s[k];
    const double n1 = a1 * (1.0 - c0s[k]);
    if (k + 1 < D)
      div2<FAST>(n0, n1, n0 + n1, a0, a1);
    else
      *hard = (unsigned char)hard_decision<FAST>(n0, n1);
  }
  double b0 = 1.0, b1 = 1.0;
#pragma unroll
  for (int k = D - 1; k >= 0; --k) {
    const bool unit = FAST && k == D - 1;  // beta = (1, 1)
    const double t0 = unit ? al0[k] : al0[k] * b0;
    const double t1 = unit ? al1[k] : al1[k] * b1;
    double q0, q1;
    div2<FAST>(t0, t1, t0 + t1, q0, q1);
    slots[cs[k]] = make_double2(q0, q1);
    if (k > 0) {
      const double c0 = c0s[k];
      if (unit) {  // (c0, 1 - c0) / (c0 + (1 - c0)): the sum rounds to exactly 1 (bp_common.hpp)
        b0 = c0;
        b1 = 1.0 - c0;
      } else {
        div2<FAST>(b0 * c0, b1 * (1.0 - c0), b0 * c0 + b1 * (1.0 - c0), b0, b1);
      }
    }
  }
}

// Half of a check row of degree D (binaryldpccodec.cc:235-275), streamed step
// by step; returns the forward state past the last edge (syndrom_soft) on the
// even lane when SYN.
template <int D, bool SYN, bool FAST>
__device__ __forceinline__ double cn_half(double2 *slots, int base, int odd) {
  constexpr int S = (D + 1) / 2;  // states kept: x[0..S)
  double x0[S], x1[S];
  double s0 = 1.0, s1 = 0.0;
#pragma unroll
  for (int st = 0; st < D; ++st) {
    const bool advance = SYN || st + 1 < D;
    double m0 = 0.0, m1 = 0.0;
    if (advance) {
      const double2 m = slots[base + (odd ? D - 1 - st : st)];
      m0 = m.x;
      m1 = m.y;
    }
    if (st < S) {
      x0[st] = s0;
      x1[st] = s1;
    }
    if ((D & 1) && st == (D - 1) / 2) {  // middle edge: both states are current here
      const double y0 = swap_pair(s0), y1 = swap_pair(s1);
      const double t0 = s0 * y0 + s1 * y1;
      const double t1 = s0 * y1 + s1 * y0;
      const double q = clip_c2v<FAST>(div1<FAST>(t0, t0 + t1));
      if (!odd) slots[base + st].x = q;
    }
    if (st >= S) {
      // c2v of edge (odd ? st : D-1-st) from (own state at D-1-st, partner state now)
      const double y0 = swap_pair(s0), y1 = swap_pair(s1);
      const double o0 = x0[D - 1 - st], o1 = x1[D - 1 - st];
      const bool unit = FAST && st == D - 1;  // own state is the boundary (1, 0)
      const double t0 = unit ? y0 : o0 * y0 + o1 * y1;
      const double t1 = unit ? y1 : o0 * y1 + o1 * y0;
      slots[base + (odd ? st : D - 1 - st)].x = clip_c2v<FAST>(div1<FAST>(t0, t0 + t1));
    }
    if (advance) {
      const bool unit = FAST && st == 0;
      const double n0 = unit ? m0 : s0 * m0 + s1 * m1;
      const double n1 = unit ? m1 : s0 * m1 + s1 * m0;
      div2<FAST>(n0, n1, n0 + n1, s0, s1);
    }
  }
  return s0;
}

// falling wave priorities over a phase's rounds (see bp_regular.hip)
__device__ __forceinline__ void set_prio(int p) {
  switch (p) {
    case 3: __builtin_amdgcn_s_setprio(3); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    default: __builtin_amdgcn_s_setprio(0); break;
  }
}

template <bool FAST>
__device__ __forceinline__ void vn_any(int d, double2 *slots, const unsigned short *cs, double p, unsigned char *h) {
  switch (d) {
    case 1: vn_column<1, FAST>(slots, cs, p, h); break;
    case 2: vn_column<2, FAST>(slots, cs, p, h); break;
    case 3: vn_column<3, FAST>(slots, cs, p, h); break;
    case 4: vn_column<4, FAST>(slots, cs, p, h); break;
    case 5: vn_column<5, FAST>(slots, cs, p, h); break;
    case 6: vn_column<6, FAST>(slots, cs, p, h); break;
    case 7: vn_column<7, FAST>(slots, cs, p, h); break;
    case 8: vn_column<8, FAST>(slots, cs, p, h); break;
    default: vn_column<9, FAST>(slots, cs, p, h); break;
  }
}

template <bool SYN, bool FAST>
__device__ __forceinline__ double cn_any(int d, double2 *slots, int base, int odd) {
  switch (d) {
    case 2: return cn_half<2, SYN, FAST>(slots, base, odd);
    case 3: return cn_half<3, SYN, FAST>(slots, base, odd);
    case 4: return cn_half<4, SYN, FAST>(slots, base, odd);
    case 5: return cn_half<5, SYN, FAST>(slots, base, odd);
    case 6: return cn_half<6, SYN, FAST>(slots, base, odd);
    case 7: return cn_half<7, SYN, FAST>(slots, base, odd);
    case 8: return cn_half<8, SYN, FAST>(slots, base, odd);
    case 9: return cn_half<9, SYN, FAST>(slots, base, odd);
    default: return cn_half<10, SYN, FAST>(slots, base, odd);
  }
}

template <int T, int RV, int RC, bool SYN, bool FAST>
__device__ __forceinline__ void decode_irr(const DevCode &c, const BpLaunch &a, int cw, double2 *slots,
                                           const unsigned short *cslot, const double *p0s, unsigned char *cch, int odd,
                                           int &iter_out, bool &conv_out) {
  const int tid = threadIdx.x;
  int iter = 0;
  bool conv = false;
  for (; iter < a.iter_count; ++iter) {
    // VN rounds: per-round column data from the (cached) planner arrays and
    // the LDS priors, so nothing is indexed by round in registers
#pragma unroll 1
    for (int r = 0; r < RV; ++r) {
      set_prio(3 - r);
      const int pos = r * T + tid;
      if (pos < c.N) {
        const int v = c.vn_order[pos];
        const int b = c.col_ptr[v];
        const double pr = v >= c.punct ? p0s[v - c.punct] : 0.5;  // :126-134
        vn_any<FAST>(c.col_ptr[v + 1] - b, slots, cslot + b, pr, &cch[v]);
      }
    }
    __syncthreads();

    int fail = 0;
#pragma unroll 1
    for (int r = 0; r < RC; ++r) {
      const int q = (r * T + tid) >> 1;
      int p = 0, d = 0;
      if (q < c.M) {
        const int row = c.cn_order[q];
        const int base = c.row_ptr[row];
        d = c.row_ptr[row + 1] - base;
        const int lo = odd ? (d + 1) / 2 : 0, hi = odd ? d : (d + 1) / 2;
        for (int k = lo; k < hi; ++k) p ^= cch[c.row_col[base + k]];
      }
      const int full = p ^ swap_pair_i(p);
      if (d > 0) fail |= full;
    }
    // the OR over the workgroup is folded into the CN phase's closing barrier
    // (speculative CN, as in bp_regular.hip); syndromes are kept until the
    // phase is known to count
    double sv[RC];
#pragma unroll
    for (int r = 0; r < RC; ++r) {
      set_prio(2 - r);
      const int q = (r * T + tid) >> 1;
      sv[r] = 0.0;
      if (q < c.M) {  // both lanes of a pair agree
        const int row = c.cn_order[q];
        const int base = c.row_ptr[row];
        sv[r] = cn_any<SYN, FAST>(c.row_ptr[row + 1] - base, slots, base, odd);
      }
    }
    if (!__syncthreads_or(fail)) {
      conv = true;
      break;
    }
    if constexpr (SYN) {
#pragma unroll
      for (int r = 0; r < RC; ++r) {
        const int q = (r * T + tid) >> 1;
        if (q < c.M && !odd) a.syn[(long long)cw * c.M + c.cn_order[q]] = sv[r];  // alpha past the last edge (:274)
      }
    }
  }
  iter_out = iter;
  conv_out = conv;
}

template <int T, int RV, int RC, bool SYN>
__global__ __launch_bounds__(T) void bp_irregular_kernel(DevCode c, BpLaunch a, unsigned int *queue, int fast_allowed) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int odd = tid & 1;
  double2 *slots = reinterpret_cast<double2 *>(smem);
  double *p0s = reinterpret_cast<double *>(smem + (size_t)c.E * 16);
  unsigned short *cslot = reinterpret_cast<unsigned short *>(smem + (size_t)c.E * 16 + (size_t)c.cc_len * 8);
  int *red = reinterpret_cast<int *>(smem + (size_t)c.E * 18 + (size_t)c.cc_len * 8);
  unsigned char *cch = smem + (size_t)c.E * 18 + (size_t)c.cc_len * 8 + kRedBytes;

  for (int e = tid; e < c.E; e += T) cslot[e] = (unsigned short)c.col_slot[e];

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

    bool ok = true;
    for (int i = tid; i < c.cc_len; i += T) {
      const double q = p0[i];
      p0s[i] = q;
      ok = ok && fast_prior_ok(q);
    }
    for (int e = tid; e < c.E; e += T) slots[e].x = 0.5;  // InitMsg
    const bool fast = __syncthreads_and(ok ? 1 : 0) && fast_allowed;

    int iter = 0;
    bool conv = false;
    if (fast)
      decode_irr<T, RV, RC, SYN, true>(c, a, cw, slots, cslot, p0s, cch, odd, iter, conv);
    else
      decode_irr<T, RV, RC, SYN, false>(c, a, cw, slots, cslot, p0s, cch, odd, iter, conv);

    if (a.iter_count > 0) {
      if (a.uu_hat) {
        uint8_t *u = a.uu_hat + (long long)cw * c.K;
        for (int i = tid; i < c.K; i += T) u[i] = cch[i + c.info_off];
      }
      if (a.cc_hat) {
        uint8_t *o = a.cc_hat + (long long)cw * c.N;
        for (int v = tid; v < c.N; v += T) o[v] = cch[v];
      }
      if (a.parity_cnt) {  // ParityCheck(cc_hat) (:281-300)
        int cnt = 0;
        for (int r = tid; r < c.M; r += T) {
          int p = 0;
          for (int e = c.row_ptr[r]; e < c.row_ptr[r + 1]; ++e) p ^= cch[c.row_col[e]];
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

template <int T, int RV, int RC, bool SYN>
hipError_t launch_irr_t(const DevCode &c, const BpLaunch &a, hipStream_t s, int fast_allowed) {
  auto kern = bp_irregular_kernel<T, RV, RC, SYN>;
  const size_t lds = (size_t)c.E * 18 + (size_t)c.cc_len * 8 + kRedBytes + (size_t)c.N;
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

}  // namespace

hipError_t launch_bp_irregular(const DevCode &c, const BpLaunch &a, hipStream_t s) {
  constexpr int T = 768, RV = 3, RC = 3;
  if ((long long)c.E * 18 + 8LL * c.cc_len + kRedBytes + c.N > 160 * 1024 || c.E > 65535) return hipErrorNotSupported;
  if (!c.irr_ok || c.N > RV * T || 2 * c.M > RC * T) return hipErrorNotSupported;
  const int fast = c.dv_max <= kFastMaxColumnDegree ? 1 : 0;
  return a.syn ? launch_irr_t<T, RV, RC, true>(c, a, s, fast) : launch_irr_t<T, RV, RC, false>(c, a, s, fast);
}

}  // namespace kml
