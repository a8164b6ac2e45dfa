// bp.hip — probability-domain sum-product LDPC decoder for gfx950.
//
// Restates lab::BinaryLDPCCodec::Decoder (lib/lab/src/binaryldpccodec.cc:165-278)
// and lab::Binary5GLDPCCodec::Decoder (lib/lab/src/binary5gldpccodec.cc:112-232)
// bit-exactly: same IEEE operations in the same order, fp64, no contraction
// (built with -ffp-contract=off), correctly rounded division.
//
// Design (MI355X-first, not a translation of the linked-list walk):
//   * one workgroup decodes one codeword at a time and pulls the next codeword
//     from a device-wide dequeue counter when it finishes (early-terminating
//     codewords free their CU immediately: no batch-wide straggler wait);
//   * the whole message state of a codeword is ONE 16-byte slot per edge held in
//     LDS: between a CN phase and the next VN phase the slot holds c2v0
//     (c2v1 = 1 - c2v0 is recomputed, exactly as the reference stores it,
//     binaryldpccodec.cc:264); between a VN phase and the CN phase it holds the
//     (v2c0, v2c1) pair.  Every column / row reads all its slots before writing
//     them, and columns / rows own disjoint slots, so the update is in place.
//     PEG2304: 6912 x 16 B = 108 KiB, 5G BG2: 115.5 KiB -> fits the 160 KiB LDS;
//     larger codes (PEG8064, 378 KiB) use the same slots in a per-workgroup
//     global scratch (L2 / Infinity-Cache resident);
//   * slots are stored in the reference's row traversal order, so a CN thread
//     reads its row as contiguous 16-byte LDS words; VN threads gather their
//     column's slots through col_slot;
//   * the early-stop parity check is a workgroup OR-reduction
//     (__syncthreads_or), the reference stops at the first failing row but the
//     boolean is the same.
//
// Compulsory-traffic accounting is accumulated in the counter
// block: executed VN and CN phases per launch.
#include <cstdlib>

#include "bp_common.hpp"
#include "kernels.hpp"

namespace kml {

namespace {

constexpr int kLdsBytes = 160 * 1024;
constexpr int kRedBytes = 16;

template <int T>
__device__ __forceinline__ int dequeue(unsigned int *queue, int *red) {
  __syncthreads();
  if (threadIdx.x == 0) {
    red[3] = (int)atomicAdd(queue, 1u);
    red[0] = 0;
    red[1] = 0;
  }
  __syncthreads();
  return red[3];
}

template <int DV, int DC, bool LDS, bool SYN, int T>
__global__ __launch_bounds__(T) void bp_kernel(DevCode c, BpLaunch a, unsigned int *queue) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int E = c.E, N = c.N, M = c.M;
  double2 *slots;
  int *red;
  unsigned char *cch;
  if constexpr (LDS) {
    slots = reinterpret_cast<double2 *>(smem);
    red = reinterpret_cast<int *>(smem + (size_t)E * 16);
    cch = smem + (size_t)E * 16 + kRedBytes;
  } else {
    slots = a.gslots + (size_t)blockIdx.x * E;
    red = reinterpret_cast<int *>(smem);
    cch = smem + kRedBytes;
  }

  for (;;) {
    const int entry = dequeue<T>(queue, red);
    if (entry >= a.B) break;
    const int cw = a.cw_idx ? a.cw_idx[entry] : entry;
    const double *p0 = a.p0 + (long long)cw * a.p0_stride;
    if (a.p0_sel) p0 += (long long)a.p0_sel[cw] * a.p0_sel_stride;

    // InitMsg (binaryldpccodec.cc:302-314): c2v = (0.5, 0.5)
    for (int e = tid; e < E; e += T) slots[e].x = 0.5;
    __syncthreads();

    int iter = 0;
    bool conv = false;
    for (; iter < a.iter_count; ++iter) {
      // ---------------- VN phase (binaryldpccodec.cc:177-213)
      for (int idx = tid; idx < N; idx += T) {
        const int v = c.vn_order[idx];
        const int b = c.col_ptr[v];
        const int d = c.col_ptr[v + 1] - b;
        double a0, a1;
        if (v < c.punct) {  // binary5gldpccodec.cc:126-129
          a0 = 0.5;
          a1 = 1.0 - 0.5;
        } else {
          const double q = p0[v - c.punct];
          a0 = q;
          a1 = 1.0 - q;
        }
        int es[DV];
        double c0s[DV], al0[DV], al1[DV];
#pragma unroll
        for (int k = 0; k < DV; ++k) {
          if (k < d) {
            const int e = c.col_slot[b + k];
            es[k] = e;
            const double c0 = slots[e].x;
            c0s[k] = c0;
            al0[k] = a0;
            al1[k] = a1;
            const double n0 = a0 * c0;
            const double n1 = a1 * (1.0 - c0);
            const double s = n0 + n1;
            a0 = div_rn(n0, s);
            a1 = div_rn(n1, s);
          }
        }
        cch[v] = (a0 > a1) ? 0 : 1;  // :190-194
        double b0 = 1.0, b1 = 1.0;
#pragma unroll
        for (int k = DV - 1; k >= 0; --k) {
          if (k < d) {
            const double t0 = al0[k] * b0;
            const double t1 = al1[k] * b1;
            const double s = t0 + t1;
            slots[es[k]] = make_double2(div_rn(t0, s), div_rn(t1, s));
            if (k > 0) {  // the head's beta (k == 0) is dead
              const double c0 = c0s[k];
              const double n0 = b0 * c0;
              const double n1 = b1 * (1.0 - c0);
              const double s2 = n0 + n1;
              b0 = div_rn(n0, s2);
              b1 = div_rn(n1, s2);
            }
          }
        }
      }
      __syncthreads();

      // ---------------- parity check (binaryldpccodec.cc:218-232)
      int fail = 0;
      for (int r = tid; r < M && !fail; r += T) {
        int p = 0;
        const int rb = c.row_ptr[r], re = c.row_ptr[r + 1];
        for (int e = rb; e < re; ++e) p ^= cch[c.row_col[e]];
        fail = p;
      }
      if (!__syncthreads_or(fail)) {
        conv = true;
        break;
      }

      // ---------------- CN phase (binaryldpccodec.cc:235-275)
      for (int idx = tid; idx < M; idx += T) {
        const int r = c.cn_order[idx];
        const int b = c.row_ptr[r];
        const int d = c.row_ptr[r + 1] - b;
        double v0[DC], v1[DC], al0[DC], al1[DC];
        double a0 = 1.0, a1 = 0.0;
#pragma unroll
        for (int k = 0; k < DC; ++k) {
          if (k < d) {
            const double2 m = slots[b + k];
            v0[k] = m.x;
            v1[k] = m.y;
            al0[k] = a0;
            al1[k] = a1;
            if (SYN || k + 1 < d) {  // alpha past the last edge only feeds syndrom_soft
              const double n0 = a0 * m.x + a1 * m.y;
              const double n1 = a0 * m.y + a1 * m.x;
              const double s = n0 + n1;
              a0 = div_rn(n0, s);
              a1 = div_rn(n1, s);
            }
          }
        }
        double b0 = 1.0, b1 = 0.0;
#pragma unroll
        for (int k = DC - 1; k >= 0; --k) {
          if (k < d) {
            const double t0 = al0[k] * b0 + al1[k] * b1;
            const double t1 = al0[k] * b1 + al1[k] * b0;
            const double s = t0 + t1;
            double q = div_rn(t0, s);  // t1/s is dead (:259 overwritten at :264)
            if (q > 1.0 - kSmallestProb) q = 1.0 - kSmallestProb;
            if (q < kSmallestProb) q = kSmallestProb;
            slots[b + k].x = q;
            if (k > 0) {
              const double n0 = b0 * v0[k] + b1 * v1[k];
              const double n1 = b0 * v1[k] + b1 * v0[k];
              const double s2 = n0 + n1;
              b0 = div_rn(n0, s2);
              b1 = div_rn(n1, s2);
            }
          }
        }
        if constexpr (SYN) a.syn[(long long)cw * M + r] = a0;  // :274
      }
      __syncthreads();
    }

    // ---------------- epilogue
    if (a.iter_count > 0) {
      if (a.uu_hat) {
        uint8_t *u = a.uu_hat + (long long)cw * c.K;
        for (int i = tid; i < c.K; i += T) u[i] = cch[i + c.info_off];  // :214-216
      }
      if (a.cc_hat) {
        uint8_t *o = a.cc_hat + (long long)cw * N;
        for (int v = tid; v < N; v += T) o[v] = cch[v];
      }
      if (a.parity_cnt) {  // ParityCheck(cc_hat) (:281-300)
        int cnt = 0;
        for (int r = tid; r < M; r += T) {
          int p = 0;
          for (int e = c.row_ptr[r]; e < c.row_ptr[r + 1]; ++e) p ^= cch[c.row_col[e]];
          cnt += p;
        }
        if (cnt) atomicAdd(&red[0], cnt);
      }
      if (a.ref_bits) {  // SourceSink::CntErr (sourcesink.cc:29-47)
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
      if (a.ret) a.ret[cw] = iter + (iter < a.max_iter);  // :277
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

constexpr int kThreads = 512;

template <int DV, int DC, bool LDS, bool SYN>
hipError_t launch_t(const DevCode &c, const BpLaunch &a, unsigned int *queue, hipStream_t s) {
  auto kern = bp_kernel<DV, DC, LDS, SYN, kThreads>;
  const size_t lds = LDS ? (size_t)c.E * 16 + kRedBytes + (size_t)c.N : kRedBytes + (size_t)c.N;
  hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  int per_cu = 1;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kThreads, lds) != hipSuccess || per_cu < 1)
    per_cu = 1;
  long long grid = (long long)ncu * per_cu;
  if (!LDS) {
    const long long cap = a.gslots_cap / (c.E > 0 ? c.E : 1);
    if (grid > cap) grid = cap;
    if (grid < 1) return hipErrorInvalidValue;
  }
  if (grid > a.B) grid = a.B;
  e = hipMemsetAsync(queue, 0, sizeof(unsigned int), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(kThreads), lds, s, c, a, queue);
  return hipGetLastError();
}

template <bool LDS, bool SYN>
hipError_t dispatch_deg(const DevCode &c, const BpLaunch &a, unsigned int *queue, hipStream_t s, const char **err) {
  if (c.dv_max <= 3 && c.dc_max <= 6) return launch_t<3, 6, LDS, SYN>(c, a, queue, s);
  if (c.dv_max <= 12 && c.dc_max <= 12) return launch_t<12, 12, LDS, SYN>(c, a, queue, s);
  if (c.dv_max <= 32 && c.dc_max <= 32) return launch_t<32, 32, LDS, SYN>(c, a, queue, s);
  if (err) *err = "node degree above 32 is not supported by the BP kernel";
  return hipErrorInvalidValue;
}

}  // namespace

namespace {
// KML_BP_KERNEL=generic forces the generic kernel (A/B measurements).
int kernel_variant() {
  static int v = -1;
  if (v < 0) {
    const char *e = getenv("KML_BP_KERNEL");
    v = (e && e[0] == 'g') ? 1 : 0;
  }
  return v;
}
}  // namespace

bool bp_uses_lds(const DevCode &c) { return (long long)c.E * 16 + kRedBytes + c.N <= kLdsBytes; }

long long bp_gslots_needed(const DevCode &c) {
  if (bp_uses_lds(c)) return 0;
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  return (long long)ncu * 4 * c.E;  // up to 4 resident workgroups per CU
}

hipError_t launch_bp(const DevCode &c, const BpLaunch &a, hipStream_t s, const char **err, const char **family) {
  if (a.B <= 0) return hipSuccess;
  if (a.iter_count < 0) {
    if (err) *err = "iter_count must be >= 0";
    return hipErrorInvalidValue;
  }
  unsigned int *queue = a.queue;
  if (!queue) {
    if (err) *err = "dequeue counter missing";
    return hipErrorInvalidValue;
  }
  const bool lds = bp_uses_lds(c);
  // kernel families, most specialised first: regular PEG2304-class (LDS),
  // irregular with degrees <= 9 / 10 (LDS), cooperative regular (L2), generic
  const int variant = kernel_variant();  // 0 auto, 1 generic
  if (lds && variant == 0) {
    hipError_t e = launch_bp_regular(c, a, s);
    if (e != hipErrorNotSupported) {
      if (family) *family = "bp_regular_kernel";
      return e;
    }
  }
  if (lds && variant == 0) {
    hipError_t e = launch_bp_irregular(c, a, s);
    if (e != hipErrorNotSupported) {
      if (family) *family = "bp_irregular_kernel";
      return e;
    }
  }
  if (!lds && variant == 0) {
    hipError_t e = launch_bp_coop(c, a, s);
    if (e != hipErrorNotSupported) {
      if (family) *family = bp_coop_family(c);
      return e;
    }
  }
  if (!lds && (a.gslots == nullptr || a.gslots_cap < c.E)) {
    if (err) *err = "global slot workspace missing";
    return hipErrorInvalidValue;
  }
  const bool syn = a.syn != nullptr;
  if (family) *family = "bp_kernel";
  if (lds) return syn ? dispatch_deg<true, true>(c, a, queue, s, err) : dispatch_deg<true, false>(c, a, queue, s, err);
  return syn ? dispatch_deg<false, true>(c, a, queue, s, err) : dispatch_deg<false, false>(c, a, queue, s, err);
}

int bp_fast_mode(const DevCode &c) {
  if (c.dv_max > kFastMaxColumnDegree) return 0;
  if (const char *e = getenv("KML_NO_FAST"))
    if (e[0] == '1') return 0;
  int m = 1;
  if (const char *e = getenv("KML_FORCE_REDO"))
    if (e[0] == '1') m |= 2;
  return m;
}

}  // namespace kml
