// kmeans.hip — the blind channel estimate of the receive path.
//
// Restates kmldpc::KMeans::Run (src/kmeans.cc:15-84) as the simulator uses it
// (src/simulator.cc:136-148), including its load-bearing quirks:
//   * idxCount / idxSum are clear()ed and then written through operator[]
//     (kmeans.cc:33-34): the storage survives, so cluster counts and sums
//     ACCUMULATE over iterations;
//   * absValues.clear() (kmeans.cc:65) makes the re-projection always take
//     cluster 0 (max_element over an empty range);
//   * convergence is exact equality of every cluster with the previous
//     iteration's (kmeans.cc:47-56), and tempClusters starts at zero;
//   * |z| is glibc hypot, '/' is __divdc3 Smith division, '*' is the naive
//     complex product (exact_math.hpp).
// Only cluster 0's running sum/count is ever read back, so the assignment only
// has to decide, per symbol, whether cluster 0 is the FIRST minimum of the K
// distances (kmeans.cc:41-44).
//
// MI355X mapping.  The production path is km_wave_kernel (one wave per
// codeword, the whole Run in one launch; described at its definition).  The
// two-launch form below (KML_KMEANS=split, A/B and S > 4096) runs one k-means
// iteration as two launches:
//   km_assign  one thread per (codeword, symbol): the K distances are screened
//              with squared norms d2 = dr*dr + di*di (relative error <= 3 ulp of
//              the exact |.|^2 of the same rounded dr, di; glibc hypot is
//              within 1 ulp of the exact |.|), so "cluster 0 is the strict
//              unique minimum" / "some k beats cluster 0" is decided exactly
//              whenever the d2 margin exceeds 1e-12 relative; inside that band
//              the glibc-exact hypot decides, with the reference's first-minimum
//              rule.  Non-finite or extreme d2 take the exact path.  The
//              cluster points c[k]*h_hat are computed once per workgroup into
//              LDS.  Membership bits are packed with a wavefront ballot.
//   km_update  one LANE per codeword: walks the membership bits in ascending
//              symbol order and adds the members' y to the running cluster-0
//              sum — a sequential floating-point chain whose rounding is part
//              of the result, so the parallelism comes from 64 codewords per
//              wavefront — then the exact convergence test and the update
//              (Smith divisions).
// km_init (first max of |y|, same screening) and km_final (h_hat and the 4
// rotated candidates) are lane-per-codeword.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "bp_common.hpp"
#include "exact_math.hpp"
#include "kernels.hpp"

namespace kml {

namespace {

constexpr double kTieBand = 1e-12;
constexpr double kD2Lo = 1e-290, kD2Hi = 1e290;

__device__ __forceinline__ bool d2_ok(double d) { return d >= kD2Lo && d <= kD2Hi; }

// first max of |y_j| over j (kmeans.cc:17-22)
__device__ int first_max_abs(const double2 *yy, int S) {
  double best = -1.0;
  bool exact = false;
  for (int j = 0; j < S; ++j) {
    const double2 v = yy[j];
    const double d = v.x * v.x + v.y * v.y;
    if (!d2_ok(d) && !(d == 0.0)) exact = true;
    if (d > best) best = d;
  }
  if (!exact && best > 0.0) {
    // candidates: d2 within the tie band of the maximum; the first exact max wins
    int mi = -1;
    double hb = 0.0;
    for (int j = 0; j < S; ++j) {
      const double2 v = yy[j];
      const double d = v.x * v.x + v.y * v.y;
      if (d >= best * (1.0 - kTieBand)) {
        const double h = kml_hypot(v.x, v.y);
        if (mi < 0 || hb < h) {
          hb = h;
          mi = j;
        }
      }
    }
    return mi;
  }
  // exact reference loop
  int mi = 0;
  double hb = kml_hypot(yy[0].x, yy[0].y);
  for (int j = 1; j < S; ++j) {
    const double h = kml_hypot(yy[j].x, yy[j].y);
    if (hb < h) {
      hb = h;
      mi = j;
    }
  }
  return mi;
}

__global__ void km_init_kernel(const double *__restrict__ cons, const double2 *__restrict__ y, int S, int B,
                               KmState *__restrict__ st) {
  const int cw = blockIdx.x * blockDim.x + threadIdx.x;
  if (cw >= B) return;
  const double2 *yy = y + (long long)cw * S;
  const int mi = first_max_abs(yy, S);
  const cplx hat = kml_cdiv(cplx{yy[mi].x, yy[mi].y}, cplx{cons[0], cons[1]});  // kmeans.cc:25
  KmState s;
  s.hat = make_double2(hat.re, hat.im);
  s.prev = make_double2(0.0, 0.0);
  s.sum = make_double2(0.0, 0.0);
  s.cnt = 0;
  s.it = 0;
  s.done = 0;
  s.have_prev = 0;
  st[cw] = s;
}

// Is cluster 0 the first minimum of |c_k*hat - y| over k?  (kmeans.cc:41-44)
template <int KC>
__device__ __forceinline__ bool member0(const double2 *cl, double yr, double yi) {
  double d0 = 0.0, m1 = 0.0;
  bool fin = true;
#pragma unroll 8
  for (int k = 0; k < KC; ++k) {
    const double2 c = cl[k];
    const double dr = c.x - yr, di = c.y - yi;
    const double d = dr * dr + di * di;
    if (k == 0)
      d0 = d;
    else if (k == 1 || d < m1)
      m1 = d;
    fin = fin && d2_ok(d);
  }
  if (fin) {
    if (d0 < m1 * (1.0 - kTieBand)) return true;
    if (d0 > m1 * (1.0 + kTieBand)) return false;
    // near tie: glibc-exact distances of the contenders decide
    const double h0 = kml_hypot(cl[0].x - yr, cl[0].y - yi);
    for (int k = 1; k < KC; ++k) {
      const double dr = cl[k].x - yr, di = cl[k].y - yi;
      const double d = dr * dr + di * di;
      if (d <= d0 * (1.0 + kTieBand))
        if (kml_hypot(dr, di) < h0) return false;
    }
    return true;
  }
  // exact reference loop (non-finite or extreme magnitudes)
  double hmin = kml_hypot(cl[0].x - yr, cl[0].y - yi);
  int kmin = 0;
  for (int k = 1; k < KC; ++k) {
    const double h = kml_hypot(cl[k].x - yr, cl[k].y - yi);
    if (h < hmin) {
      hmin = h;
      kmin = k;
    }
  }
  return kmin == 0;
}

// grid: one workgroup per codeword; the workgroup's waves sweep its symbols in
// 64-symbol words.
template <int KC>
__global__ __launch_bounds__(256) void km_assign_kernel(const double *__restrict__ cons, const double2 *__restrict__ y,
                                                        int S, int Sw, const KmState *__restrict__ st,
                                                        uint64_t *__restrict__ mem) {
  __shared__ double2 cl[KC];
  const int cw = blockIdx.x;
  const KmState s = st[cw];
  if (s.done) return;  // uniform per workgroup
  const cplx hat{s.hat.x, s.hat.y};
  for (int k = threadIdx.x; k < KC; k += blockDim.x) {
    const cplx p = kml_cmul(cplx{cons[2 * k], cons[2 * k + 1]}, hat);  // clusters_[k] = c[k] * hatH
    cl[k] = make_double2(p.re, p.im);
  }
  __syncthreads();
  const double2 *yy = y + (long long)cw * S;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int w = wave; w < Sw; w += nw) {
    const int j = w * 64 + lane;
    bool m = false;
    if (j < S) {
      const double2 v = yy[j];
      m = member0<KC>(cl, v.x, v.y);
    }
    const uint64_t bits = __ballot(m);
    if (lane == 0) mem[(long long)cw * Sw + w] = bits;
  }
}

template <int KC>
__global__ void km_update_kernel(const double *__restrict__ cons, const double2 *__restrict__ y, int S, int Sw,
                                 int iters, int B, KmState *__restrict__ st, const uint64_t *__restrict__ mem) {
  const int cw = blockIdx.x * blockDim.x + threadIdx.x;
  if (cw >= B) return;
  KmState s = st[cw];
  if (s.done) return;
  const double2 *yy = y + (long long)cw * S;
  const uint64_t *mm = mem + (long long)cw * Sw;
  // cumulative cluster-0 count and sum, ascending symbol order (kmeans.cc:36-46)
  double sr = s.sum.x, si = s.sum.y;
  int cnt = s.cnt;
  for (int w = 0; w < Sw; ++w) {
    uint64_t bits = mm[w];
    while (bits) {
      const int j = w * 64 + __builtin_ctzll(bits);
      bits &= bits - 1;
      const double2 v = yy[j];
      sr = sr + v.x;
      si = si + v.y;
      cnt++;
    }
  }
  s.sum = make_double2(sr, si);
  s.cnt = cnt;
  // convergence: every cluster equals the previous iteration's (kmeans.cc:47-56)
  const cplx hat{s.hat.x, s.hat.y}, prev{s.prev.x, s.prev.y};
  bool same = true;
  for (int k = 0; k < KC && same; ++k) {
    const cplx ck{cons[2 * k], cons[2 * k + 1]};
    const cplx a = kml_cmul(ck, hat);
    const cplx b = s.have_prev ? kml_cmul(ck, prev) : cplx{0.0, 0.0};
    same = (a.re == b.re) && (a.im == b.im);
  }
  s.it++;
  if (same) {
    s.done = 1;
  } else {
    s.prev = s.hat;
    s.have_prev = 1;
    const cplx c0{cons[0], cons[1]};
    const cplx m0 = kml_cdiv(cplx{sr, si}, cplx{(double)cnt, 0.0});  // kmeans.cc:59-62
    const cplx nh = kml_cdiv(m0, c0);                                  // kmeans.cc:64-71
    s.hat = make_double2(nh.re, nh.im);
    if (s.it >= iters) s.done = 1;
  }
  st[cw] = s;
}

__global__ void km_final_kernel(const double *__restrict__ cons, const double *__restrict__ rot, int B,
                                const KmState *__restrict__ st, double2 *__restrict__ h_hat,
                                double2 *__restrict__ h4, double2 *__restrict__ hat_out) {
  const int cw = blockIdx.x * blockDim.x + threadIdx.x;
  if (cw >= B) return;
  if (hat_out) hat_out[cw] = st[cw].hat;
  const cplx c0{cons[0], cons[1]};
  const cplx hat{st[cw].hat.x, st[cw].hat.y};
  const cplx hh = kml_cdiv(kml_cmul(c0, hat), c0);  // simulator.cc:145
  h_hat[cw] = make_double2(hh.re, hh.im);
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // simulator.cc:146-148
    const cplx r = kml_cmul(hh, cplx{rot[2 * j], rot[2 * j + 1]});
    h4[(long long)cw * 4 + j] = make_double2(r.re, r.im);
  }
}

// ---------------------------------------------------------------------------
// The whole KMeans::Run in one launch (km_wave_kernel, below).  Each codeword
// is a chain of dependent iterations, so the iterations skip the work whose
// outcome is already known, exactly:
//   * convergence (kmeans.cc:47-56) compares clusters_ = c_k * hatH with the
//     previous iteration's; lanes k < KC compute both at the iteration START
//     (the cluster points the assignment needs anyway), so a converged
//     iteration breaks before its assignment (whose sums the reference
//     discards: only hatH is read after the loop);
//   * incremental assignment: when a symbol is assigned, the gap between its
//     distance to cluster 0 and to the nearest other cluster gives a margin g
//     (a lower bound of the true gap, with the fp64 rounding of the screened
//     squared distances and of glibc hypot folded in).  A later hatH moves
//     cluster k by at most |c_k| |hatH' - hatH| plus the rounding of the two
//     complex products, so while 2 Cmax (D(t) - D(ref)) < g — D the running
//     sum of the per-iteration bounds |dh| + 2^-48 (|h| + |h'|), rounded up,
//     norms by norm2_up — the symbol's decision cannot change.  A 64-symbol
//     word is re-assigned when any of its symbols may have changed: each word
//     keeps the minimum over its symbols of T = D(ref) + g / (2 Cmax) (float,
//     rounded down);
//   * the members' list is rebuilt only when some word's membership bits
//     changed, and then only the words whose members or offset changed;
//   * the cumulative-mean division by (cnt, 0) and the division by c[0] take
//     __divdc3's own branch with the constant parts hoisted (exact: same
//     operations on the same values).
// Round 4's two-wave form (km_fused_kernel: y staged in LDS, two waves per
// codeword, 8 per CU) ran 3.50 ms per 32768 PEG2304/QPSK codewords; the
// one-wave kernel runs 2.39 ms and took 64QAM over too.
constexpr int kMaxS = 4096;  // 64-symbol words in the lanes of one wave

// Phase timing (stamps build, -DKML_STAMPS=1; tools/km_stamps.py): thread 0's
// s_memtime deltas summed over workgroups, plus event counts.
#ifndef KML_STAMPS
#define KML_STAMPS 0
#endif
enum { KS_PRO, KS_CLUSTERS, KS_ASSIGN, KS_COMPACT, KS_SUM, KS_ITERS, KS_WORDS, KS_COMPACTIONS, KS_CW, KS_UPDATE, KS_STEPS,
       KS_WEAK, KS_SLOTS = 16 };
__device__ unsigned long long kml_km_stamps[KS_SLOTS];
#if KML_STAMPS
// accumulated in thread 0's registers, flushed once per workgroup (KM_FLUSH)
#define KM_STAMP(i)                                                \
  do {                                                             \
    if (tid == 0) {                                                \
      const unsigned long long _t = __builtin_amdgcn_s_memtime();  \
      km_acc[(i)] += _t - km_prev;                                 \
      km_prev = _t;                                                \
    }                                                              \
  } while (0)
#define KM_COUNT(i, v) \
  do {                 \
    if (tid == 0) km_acc[(i)] += (unsigned long long)(v); \
  } while (0)
#else
#define KM_STAMP(i) \
  do {              \
  } while (0)
#define KM_COUNT(i, v) \
  do {                 \
  } while (0)
#endif

__device__ __forceinline__ double wave_max(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}
// wave minimum by DPP (quad swaps, row mirrors, row broadcasts 15 / 31: no
// LDS round trips), the result read from lane 63
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_min_step(float v) {
  const float o = __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, ROWS, 0xF, false));
  return fminf(v, o);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_add_step_i(int v) {
  return v + __builtin_amdgcn_update_dpp(0, v, CTRL, ROWS, 0xF, false);
}
__device__ __forceinline__ int wave_inclusive_scan_i(int v) {
  v = dpp_add_step_i<0x111, 0xF>(v);  // row_shr:1
  v = dpp_add_step_i<0x112, 0xF>(v);  // row_shr:2
  v = dpp_add_step_i<0x114, 0xF>(v);  // row_shr:4
  v = dpp_add_step_i<0x118, 0xF>(v);  // row_shr:8
  v = dpp_add_step_i<0x142, 0xA>(v);  // row_bcast:15 into rows 1, 3
  v = dpp_add_step_i<0x143, 0xC>(v);  // row_bcast:31 into rows 2, 3
  return v;
}
__device__ __forceinline__ float wave_min_f(float v) {
  v = dpp_min_step<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
  v = dpp_min_step<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
  v = dpp_min_step<0x141, 0xF>(v);  // row_half_mirror
  v = dpp_min_step<0x140, 0xF>(v);  // row_mirror: every lane holds its row's minimum
  v = dpp_min_step<0x142, 0xA>(v);  // row_bcast:15 into rows 1, 3
  v = dpp_min_step<0x143, 0xC>(v);  // row_bcast:31 into rows 2, 3
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 63));
}

// The same sum computed by a whole wave (binade-segmented integer scans;
// tools/probe/km_scan_model.py is a CPU model of exactly these steps, checked
// against the sequential sum on adversarial inputs).  While the running sum
// stays in one binade [2^(e-1), 2^e) (magnitude; sign sg), every rounded add
// is a move on the fixed grid u = 2^(e-53): with A = |acc| / u (an integer in
// [2^52, 2^53)) and X = sg x / u (exact ldexp), RN(acc + x) = sg (A + rint(X)) u
// unless X is a tie (frac 0.5: the parity of the result decides) or the result
// leaves the binade.  Each lane takes kScanPer consecutive elements, rounds
// them to the grid (v_rndne), sums them locally, and a DPP exclusive scan of
// the lane totals gives every prefix A + P.  All elements before the first one
// that is large (|X| >= 2^51: keeps every partial sum of valid elements below
// 2^53, hence exact) or whose prefix leaves [2^52 + 1, 2^53 - 1] (then the
// exact sum lies inside the binade, where RN is the grid rounding) are exact;
// that element is added with a real fp64 add and the scan resumes after it.
// Ties do not stop the scan: they count floor(X), and afterwards, in element
// order, each tie whose corrected prefix is odd rounds up (ties to even),
// adding 1 to every later prefix (kScanMargin keeps the range test valid
// under those corrections).  A zero or non-finite sum, and runs after an
// early exit, are added one by one.  On MI355X a dependent f64 add chain
// costs ~40 cycles per element here (LDS index + value loads, other waves on
// the SIMD); a step costs about 50 dependent instructions.
// elements per lane per step: 5 covers a QPSK cluster-0 list (~286) in one
// step; measured per 32768 PEG2304/QPSK codewords: 4 -> 3.42 ms, 5 -> 3.31 ms,
// 8 -> 3.89 ms (longer in-lane chains and registers)
#ifndef KML_KM_SCAN_PER
#define KML_KM_SCAN_PER 5
#endif
constexpr int kScanPer = KML_KM_SCAN_PER;
constexpr double kScanMargin = 64.0;      // grid steps kept from the binade ends: room for the tie corrections
constexpr int kScanMaxTies = 32;          // ties resolved in one step (each moves later prefixes by <= 1)
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_add_step(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROWS, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROWS, 0xF, false);
  return v + __hiloint2double(hi, lo);
}
// sum over the lanes below this one (exact where those sums are)
__device__ __forceinline__ double wave_exclusive_scan(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x138, 0xF, 0xF, false);  // wave_shr:1
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x138, 0xF, 0xF, false);
  v = __hiloint2double(hi, lo);
  v = dpp_add_step<0x111, 0xF>(v);  // row_shr:1
  v = dpp_add_step<0x112, 0xF>(v);  // row_shr:2
  v = dpp_add_step<0x114, 0xF>(v);  // row_shr:4
  v = dpp_add_step<0x118, 0xF>(v);  // row_shr:8: prefix within each row of 16
  v = dpp_add_step<0x142, 0xA>(v);  // row_bcast:15 into rows 1, 3
  v = dpp_add_step<0x143, 0xC>(v);  // row_bcast:31 into rows 2, 3
  return v;
}
__device__ __forceinline__ double lane_d(double v, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), l),
                          __builtin_amdgcn_readlane(__double2loint(v), l));
}
__device__ __forceinline__ uint64_t lane_u64(uint64_t v, int l) {
  return ((uint64_t)(unsigned)__builtin_amdgcn_readlane((int)(v >> 32), l) << 32) |
         (unsigned)__builtin_amdgcn_readlane((int)v, l);
}
// One step of the scan, split in two phases so that a wave can run the real
// and the imaginary chain side by side: scan_a is straight-line (grid values,
// the lane totals' DPP scan, the prefixes and the exit tests), scan_b the
// wave-uniform tail (first exit, ties, the new sum).
struct ScanStep {
  double T[kScanPer];  // A + prefix through element k of this lane
  double A, sg;
  int e;
  unsigned bigm, tiem, hardm;
};
__device__ __forceinline__ void scan_a(double acc, const double (&x)[kScanPer], int c, int lane, ScanStep &s) {
  s.e = __builtin_amdgcn_frexp_exp(acc);  // |acc| in [2^(e-1), 2^e)
  s.sg = acc < 0.0 ? -1.0 : 1.0;
  s.A = __builtin_amdgcn_ldexp(fabs(acc), 53 - s.e);
  s.bigm = 0;
  s.tiem = 0;
  double run = 0.0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    const double X = __builtin_amdgcn_ldexp(s.sg * x[k], 53 - s.e);
    const double fl = floor(X);
    const bool big = !(fabs(X) < 0x1p51);
    const bool tie = !big && (X - fl) == 0.5;
    s.bigm |= (big ? 1u : 0u) << k;
    s.tiem |= (tie ? 1u : 0u) << k;
    // a tie counts its lower neighbour; the parity pass adds 1 where it rounds up
    run = run + (big ? 0.0 : (tie ? fl : rint(X)));
    s.T[k] = run;
  }
  const double E = wave_exclusive_scan(run);
  const int kl = min(max(c - kScanPer * lane, 0), kScanPer);  // this lane's elements
  s.hardm = 0;
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    s.T[k] = s.A + (E + s.T[k]);
    const bool hard =
        k < kl && (((s.bigm >> k) & 1u) || !(s.T[k] >= 0x1p52 + kScanMargin && s.T[k] <= 0x1p53 - kScanMargin));
    s.hardm |= (hard ? 1u : 0u) << k;
  }
}
// The step's result: the new sum, the elements consumed (adv) and the length
// of a one-by-one run to follow (seq).
__device__ __forceinline__ double scan_b(ScanStep &s, const double (&x)[kScanPer], int c, int lane, int &adv, int &seq) {
  const int pos0 = kScanPer * lane;  // this lane's positions in the step
  int fh = c;  // the first element that must be added for real
  {
    const uint64_t hb = __ballot(s.hardm != 0);
    if (hb) {
      const int lf = __builtin_ctzll(hb);
      fh = kScanPer * lf + __builtin_amdgcn_readlane(__builtin_ctz(s.hardm | (1u << kScanPer)), lf);
    }
  }
  // ties before fh, in order: round half to even on the corrected prefix
  {
    unsigned tm = 0;
#pragma unroll
    for (int k = 0; k < kScanPer; ++k)
      if (pos0 + k < fh) tm |= s.tiem & (1u << k);
    int nt = 0;
    for (uint64_t tb = __ballot(tm != 0); tb; tb = __ballot(tm != 0)) {  // wave-uniform
      const int lt = __builtin_ctzll(tb);
      const int kt = __builtin_ctz((unsigned)__builtin_amdgcn_readlane((int)tm, lt));
      const int q = kScanPer * lt + kt;
      if (nt == kScanMaxTies) {  // too many ties for the margin: this one is added for real
        fh = q;
        break;
      }
      ++nt;
      // (every selection below reads the arrays at static indices: a
      // selection by a run-time index is lowered to a scratch array)
      double Tq = 0.0;
#pragma unroll
      for (int k = 0; k < kScanPer; ++k) {
        const double tk = lane_d(s.T[k], lt);
        Tq = kt == k ? tk : Tq;
      }
      if ((long long)Tq & 1) {  // odd: the tie rounds up, and so does every later prefix
#pragma unroll
        for (int k = 0; k < kScanPer; ++k)
          if (pos0 + k >= q) s.T[k] += 1.0;
      }
      if (lane == lt) tm &= ~(1u << kt);
    }
  }
  if (fh == c) {
    // the last element's prefix: that lane's last prefix (positions past c
    // hold zeros, which move no prefix, and every tie correction moves them all)
    adv = c;
    return s.sg * __builtin_amdgcn_ldexp(lane_d(s.T[kScanPer - 1], (c - 1) / kScanPer), s.e - 53);
  }
  const int lf = fh / kScanPer, fk = fh % kScanPer;
  double Tpre = 0.0, xf = 0.0;  // lane lf's prefix before position fk and its element fk
#pragma unroll
  for (int k = 0; k < kScanPer; ++k) {
    const double xk = lane_d(x[k], lf), tk = lane_d(s.T[k], lf);
    xf = fk == k ? xk : xf;
    Tpre = fk - 1 == k ? tk : Tpre;
  }
  // the prefix before fh: the previous element's (in this lane or the lane below), or A
  double Tp = fk > 0 ? Tpre : s.A;
  if (fk == 0 && lf > 0) Tp = lane_d(s.T[kScanPer - 1], lf - 1);
  double acc = s.sg * __builtin_amdgcn_ldexp(Tp, s.e - 53);
  acc = acc + xf;  // the exiting / large element, rounded for real
  adv = fh + 1;
  if (fh < 16) seq = 32;  // exits close together: a short one-by-one run
  return acc;
}
// one by one, lane-major element order: a run after an early exit (seq), or
// the first element onto a zero / non-finite sum
__device__ __forceinline__ double seq_run(double acc, const double (&x)[kScanPer], int c, int &adv, int &seq) {
  const int mm = seq > 0 ? min(seq, c) : 1;
  for (int l = 0; l * kScanPer < mm; ++l) {
#pragma unroll
    for (int k = 0; k < kScanPer; ++k)
      if (l * kScanPer + k < mm) acc = acc + lane_d(x[k], l);
  }
  seq = seq > 0 ? seq - mm : 0;
  adv = mm;
  return acc;
}
__device__ __forceinline__ bool scan_ok(double acc, int seq) { return seq == 0 && acc != 0.0 && isfinite(acc); }

// One chain (comp 0: real, 1: imaginary) over the LDS value list.
__device__ __forceinline__ double ordered_sum_vals1(double acc, const double2 *vals, int comp, int n, int lane,
                                                    int &steps) {
  int i = 0, seq = 0;
  const double *vv = reinterpret_cast<const double *>(vals) + comp;
  while (i < n) {  // wave-uniform
    ++steps;
    const int c = min(64 * kScanPer, n - i);
    double x[kScanPer];
#pragma unroll
    for (int k = 0; k < kScanPer; ++k) {
      const int j = i + kScanPer * lane + k;
      const double v = vv[2 * min(j, n - 1)];
      x[k] = j < n ? v : 0.0;
    }
    int adv;
    if (!scan_ok(acc, seq)) {
      acc = seq_run(acc, x, c, adv, seq);
    } else {
      ScanStep st;
      scan_a(acc, x, c, lane, st);
      acc = scan_b(st, x, c, lane, adv, seq);
    }
    i += adv;
  }
  return acc;
}

// An upper bound of the Euclidean norm sqrt(a^2 + b^2): the fp64 form (at most
// a few ulps off, v_sqrt_f64 included) times 1 + 1e-14, or |a| + |b| where a
// square could under- or overflow (and for NaN input, NaN as before).  The
// drift bound of the incremental assignment takes |c_k| and |hatH' - hatH| in
// this norm (round 4 took |re| + |im| for both: up to 2x looser for QPSK).
__device__ __forceinline__ double norm2_up(double a, double b) {
  const double m = fmax(fabs(a), fabs(b));
  if (!(m >= 0x1p-500 && m <= 0x1p500)) return fabs(a) + fabs(b);
  return sqrt(a * a + b * b) * (1.0 + 1e-14);
}

// Lower bound of |sqrt(hi) - sqrt(lo)| (true distances of the fp cluster
// points) from the screened squared distances lo <= hi (screen0):
//   sqrt(hi) - sqrt(lo) = (hi - lo) / (sqrt(hi) + sqrt(lo)) >= (hi - lo) / (2 sqrt(hi)).
// The fp64 d2 values are within 2^-50 relative of the exact squares, hence
// the 1e-13 (hi + lo) term; the float conversion and v_rsq_f32 are within
// 2^-22 relative, hence 0.5 (1 - 1e-5); the final 1e-13 (hi + 1) >= 2e-13
// sqrt(hi) term absorbs glibc hypot's rounding at the later comparison.
// 0 outside the float range (the symbol is then re-assigned every iteration).

// the tie-band / exact decision out of line (rare; keeps the hot loop's
// registers free)
#ifndef KML_KM_OUTLINE
#define KML_KM_OUTLINE 1
#endif
#if KML_KM_OUTLINE
#define KM_SLOW __noinline__
#else
#define KM_SLOW __forceinline__
#endif
template <int KC>
__device__ KM_SLOW bool member0_slow(const double2 *cl, double yr, double yi) {
  return member0<KC>(cl, yr, yi);
}

// The assignment's screen, branch-free: returns whether it decided; then m is
// "cluster 0 is the first minimum" (member0) and g its margin (the bound
// above), else the caller runs member0_slow (g = 0).  The range test d2_ok of every
// distance is taken on the high dwords as unsigned integers (NaN and inf
// included): hi(d) > hi(1e-290) and hi(d) < hi(1e290) imply 1e-290 < d <
// 1e290, so the screen decides only where member0's screen does, with the
// same operations on the same values (elsewhere the exact decision, g = 0).
constexpr unsigned kD2HiLo = 0x03b8f2b0u;  // high dword of 1e-290
constexpr unsigned kD2HiHi = 0x7c2485ceu;  // high dword of 1e290
template <int KC>
__device__ __forceinline__ bool screen0(const double2 *cl, double yr, double yi, bool &m, double &g) {
  double d0 = 0.0, m1 = 0.0;
  unsigned hmin = 0xffffffffu, hmax = 0u;
#pragma unroll 8
  for (int k = 0; k < KC; ++k) {
    const double2 c = cl[k];
    const double dr = c.x - yr, di = c.y - yi;
    const double d = dr * dr + di * di;
    const unsigned h = (unsigned)__double2hiint(d);
    hmin = min(hmin, h);
    hmax = max(hmax, h);
    if (k == 0)
      d0 = d;
    else if (k == 1)
      m1 = d;
    else
      m1 = fmin(m1, d);  // no NaN reaches a decided screen
  }
  const bool in = d0 < m1 * (1.0 - kTieBand);
  const bool out = d0 > m1 * (1.0 + kTieBand);
  const double lo = in ? d0 : m1, hi = in ? m1 : d0;
  // dist_margin(lo, hi), branch-free
  const double num = (hi - lo) - 1e-13 * (hi + lo);
  const double q = num * (double)__builtin_amdgcn_rsqf((float)hi) * (0.5 * (1.0 - 1e-5)) - 1e-13 * (hi + 1.0);
  g = (lo >= 1e-30 && hi <= 1e30 && q > 0.0) ? q : 0.0;
  m = in;
  return hmin > kD2HiLo && hmax < kD2HiHi && (in || out);
}

__device__ KM_SLOW cplx cdiv_slow(cplx n, cplx dd) { return kml_cdiv(n, dd); }

// A symbol's drift threshold D + g / (2 Cmax), rounded down: the (1 - 2^-20)
// factor covers the float conversion's rounding in the normal range; below
// FLT_MIN (where a denormal's relative rounding error is unbounded) it is 0,
// i.e. the symbol is re-assigned next iteration; past the float range a finite
// 2^127.
__device__ __forceinline__ float km_threshold(double drift, double g, double inv2c) {
  const double td = (drift + g * inv2c) * (1.0 - 0x1p-20);
  return td < 0x1p-126 ? 0.0f : td < 0x1p127 ? (float)td : 0x1p127f;
}

// Threshold tiers of the incremental assignment (KML_KM_WEAK): a word's few
// symbols closest to a decision boundary (the kKmWeak smallest thresholds) are
// re-assigned on their own, gathered from several words into one pass, while
// the drift stays below the word's other thresholds; the whole word is
// re-assigned only when it reaches those.  A CPU model of the rule
// (PEG2304 / QPSK, 2 dB) re-assigns 2.6 instead of 6.2 whole words per
// iteration, plus ~10 weak symbols in one gathered pass.
#ifndef KML_KM_WEAK
#define KML_KM_WEAK 1
#endif
#ifndef KML_KM_WEAK_K  // weak symbols per word (<= 4: packed 7-bit lane indices)
#define KML_KM_WEAK_K 3
#endif
constexpr int kKmWeak = KML_KM_WEAK_K;

// kml_cdiv(n, {c, 0}) for a count c >= 1: __divdc3's |c| >= |d| branch with
// ratio = 0 / c = 0 and denom = 0 * 0 + c = c, where fabs(ratio) > DBL_MIN is
// false, gives x = (a + 0 * (b / c)) / c and y = (b - 0 * (a / c)) / c, which
// are a / c and b / c for finite nonzero a, b (the zero terms only matter for
// signed zeros).  Anything else takes the full restatement.  yc = dd_rcp(c),
// taken before the sums are known.
__device__ __forceinline__ cplx cdiv_count(double a, double b, int cnt, const DdRcp &yc) {
  const double c = (double)cnt;
  if (cnt > 0 && a != 0.0 && b != 0.0 && isfinite(a) && isfinite(b))
    return cplx{div_rn_y<true>(a, c, yc), div_rn_y<true>(b, c, yc)};
  return cdiv_slow(cplx{a, b}, cplx{c, 0.0});
}

// kml_cdiv(n, c0) with c0 fixed for the launch: the branch, ratio, denom and
// denom's reciprocal depend on c0 only and are hoisted (the same operations on
// the same values).
struct CdivConst {
  double ratio, denom;
  DdRcp yd;
  int mode;  // 1: |c| < |d|, 2: |c| >= |d|, 0: the DBL_MIN branch (full restatement)
};
__device__ __forceinline__ CdivConst cdiv_prepare(cplx dd) {
  const double RMIN = 2.2250738585072014e-308;
  const double c = dd.re, d = dd.im;
  CdivConst k;
  if (fabs(c) < fabs(d)) {
    k.ratio = kml_div(c, d);
    k.denom = (c * k.ratio) + d;
    k.mode = 1;
  } else {
    k.ratio = kml_div(d, c);
    k.denom = (d * k.ratio) + c;
    k.mode = 2;
  }
  if (!(fabs(k.ratio) > RMIN)) k.mode = 0;
  k.yd = dd_rcp(k.denom);
  return k;
}
__device__ __forceinline__ cplx cdiv_const(cplx n, cplx dd, const CdivConst &k) {
  double x, y;
  if (k.mode == 1) {
    x = div_rn_y<true>((n.re * k.ratio) + n.im, k.denom, k.yd);
    y = div_rn_y<true>((n.im * k.ratio) - n.re, k.denom, k.yd);
  } else if (k.mode == 2) {
    x = div_rn_y<true>((n.im * k.ratio) + n.re, k.denom, k.yd);
    y = div_rn_y<true>(n.im - (n.re * k.ratio), k.denom, k.yd);
  } else {
    return cdiv_slow(n, dd);
  }
  if (isnan(x) && isnan(y)) return cdiv_slow(n, dd);  // the Annex G recovery cases
  return cplx{x, y};
}

// ---------------------------------------------------------------------------
// One wave (and one workgroup) per codeword: the production k-means.  There
// is no LDS copy of y: the symbols are read where they lie (HBM, then L2 /
// Infinity Cache for the iterations' re-reads: coalesced 64-symbol words for
// the assignment and the rebuilds); a word's membership bits and drift
// threshold live in the registers of lane = word (S <= 4096); LDS holds the
// cluster-0 members' VALUES in ascending symbol order (capacity S/3; a larger
// cluster 0, seen only on degenerate inputs, is summed straight from the
// words), the cluster points, the constellation and the launch constants
// (6.3 KB per PEG2304/QPSK codeword).  Residency is set by registers (6 waves
// per SIMD) and there is no workgroup barrier at all.  The real and the
// imaginary chains are summed by the same wave one after the other (both in
// one scan step measured slower: more registers).
// Member list in per-word segments (KML_KM_SEG): word w's members in
// ascending order, then -0.0 fillers up to its capacity (members at the last
// layout + kKmSlack).  x + (-0.0) == x for every x (signed zeros, infinities
// and NaNs included), so the ordered sum over the list equals the sum over the
// members, and a word whose members change rewrites its own segment only —
// the compacted list shifted every later word (a CPU model of the PEG2304 /
// QPSK trajectories: 6.2 -> 3.4 words reloaded per iteration for 6 % more
// scanned elements, tools/probe/km_seg_model.py; measured 2.41 -> 2.28 ms per
// 32,768 blind PEG2304 codewords, slack 2: 2.39 ms — the list passes 320
// elements, one scan step).
#ifndef KML_KM_SEG
#define KML_KM_SEG 1
#endif
#ifndef KML_KM_SLACK
#define KML_KM_SLACK 1
#endif
constexpr int kKmSlack = KML_KM_SLACK;
#ifndef KML_KM_WAVE_OCC
#define KML_KM_WAVE_OCC 6  // waves per SIMD (registers <= 512 / OCC): 6 (80 VGPRs, 9 spilled) 2.75 ms, 5 3.04, 4 3.31
#endif
#ifndef KML_KM_CAPMUL  // member-list capacity S * CAPMUL / CAPDIV (A/B with the occupancy)
#define KML_KM_CAPMUL 1
#endif
#ifndef KML_KM_CAPDIV
#define KML_KM_CAPDIV 3
#endif
// Codewords (waves) per workgroup.  One: a workgroup's LDS is released when its
// own codeword ends, not with the slowest of four (iteration counts vary), and
// the dispatcher refills the CU per codeword: blind PEG2304 2.69 ms with four,
// 2.59 with two, 2.44 with one (profiles/r05_ab5_summary.txt).
#ifndef KML_KM_WPG
#define KML_KM_WPG 1
#endif
constexpr int kWaveWpg = KML_KM_WPG;
struct KmWaveLds {
  int cap, off_cl, stride;
};
__host__ __device__ constexpr KmWaveLds km_wave_lds(int S, int KC) {
  const int cap = ((S * KML_KM_CAPMUL + KML_KM_CAPDIV - 1) / KML_KM_CAPDIV + 7) & ~7;  // (A/B) larger clusters: the fallback sum
  const int off_cl = 16 * cap;
  // then the cluster points [KC], the constellation [KC] and the launch
  // constants (KmWaveConst): kept in LDS, not in registers across the loop
  return KmWaveLds{cap, off_cl, off_cl + 32 * KC + 64};
}
struct KmWaveConst {
  double ratio, denom, yd_hi, yd_lo, yd_k, inv2c;
  int mode;
};

template <int KC>
__global__ __launch_bounds__(64 * kWaveWpg) __attribute__((amdgpu_waves_per_eu(KML_KM_WAVE_OCC))) void km_wave_kernel(
    const double *__restrict__ cons, const double *__restrict__ rot, const double2 *__restrict__ y, int S, int iters,
    int B, double2 *__restrict__ h_hat, double2 *__restrict__ h4, double2 *__restrict__ hat_out, int incremental,
    int scan) {
  extern __shared__ __attribute__((aligned(16))) unsigned char kmem[];
  const KmWaveLds L = km_wave_lds(S, KC);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cw = blockIdx.x * kWaveWpg + wave;
  if (cw >= B) return;  // wave-uniform; the waves of a workgroup never wait for each other
  double2 *vals = reinterpret_cast<double2 *>(kmem + wave * L.stride);           // [cap] the members' symbols, in order
  double2 *cl = reinterpret_cast<double2 *>(kmem + wave * L.stride + L.off_cl);  // [KC] cluster points
  // (plain LDS pointers: the loop's LDS stores may alias them, so the values
  // are reloaded where used instead of being held in registers)
  double2 *cs = cl + KC;                                              // [KC] constellation points
  KmWaveConst *kc = reinterpret_cast<KmWaveConst *>(cl + 2 * KC);
  const int Sw = (S + 63) / 64;
  // segments pay off where a word holds many members (QPSK / 4PSK: ~16 of 64);
  // for 16 and 64 points the fillers would lengthen the scanned list by 25 % /
  // 100 % (64QAM measured 0.48 -> 0.49 ms), so those keep the compacted list
  constexpr bool kSeg = KML_KM_SEG && KC <= 4;
#if KML_STAMPS
  unsigned long long km_prev = __builtin_amdgcn_s_memtime();
  unsigned long long km_acc[KS_WEAK + 1] = {};
  KM_COUNT(KS_CW, 1);
#endif
  const double2 *yy = y + (long long)cw * S;

  // ---- first max |y| (kmeans.cc:17-22), screened like first_max_abs: one
  // pass keeps each lane's largest squared norm (first index) and its second
  // largest; when no lane holds two symbols inside the tie band of the
  // maximum, the band's candidates are the lanes' maxima and one exact hypot
  // each decides (else the band is rescanned)
  int mi;
  {
    double d1 = -1.0, d2 = -1.0;
    int j1 = 0;
    bool ex = false;
#pragma unroll 6
    for (int j = lane; j < S; j += 64) {
      const double2 v = yy[j];
      const double d = v.x * v.x + v.y * v.y;
      if (!d2_ok(d) && !(d == 0.0)) ex = true;
      if (d > d1) {
        d2 = d1;
        d1 = d;
        j1 = j;
      } else if (d > d2) {
        d2 = d;
      }
    }
    const double best = wave_max(d1);
    const double band = best * (1.0 - kTieBand);
    if (__ballot(ex) == 0 && best > 0.0 && __ballot(d2 >= band) == 0) {
      const bool cand = d1 >= band;
      const double h = cand ? kml_hypot(yy[j1].x, yy[j1].y) : -1.0;
      const double hb = wave_max(h);
      mi = wave_min_i(cand && h == hb ? j1 : 0x7fffffff);
    } else if (__ballot(ex) == 0 && best > 0.0) {
      double hb = -1.0;  // max exact |y| among the band's candidates
      for (int j = lane; j < S; j += 64) {
        const double2 v = yy[j];
        if (v.x * v.x + v.y * v.y >= band) hb = fmax(hb, kml_hypot(v.x, v.y));
      }
      hb = wave_max(hb);
      int jm = 0x7fffffff;  // the first index attaining it
      for (int j = lane; j < S; j += 64) {
        const double2 v = yy[j];
        if (v.x * v.x + v.y * v.y >= band && kml_hypot(v.x, v.y) == hb) jm = min(jm, j);
      }
      mi = wave_min_i(jm);
    } else {  // the reference loop, sequentially (non-finite / extreme / all-zero input)
      int m = 0;
      if (lane == 0) {
        double h0 = kml_hypot(yy[0].x, yy[0].y);
        for (int j = 1; j < S; ++j) {
          const double h = kml_hypot(yy[j].x, yy[j].y);
          if (h0 < h) {
            h0 = h;
            m = j;
          }
        }
      }
      mi = __builtin_amdgcn_readlane(m, 0);
    }
  }
  const cplx c0{cons[0], cons[1]};
  cplx hat = kml_cdiv(cplx{yy[mi].x, yy[mi].y}, c0);  // kmeans.cc:25
  {
    const CdivConst c0k = cdiv_prepare(c0);
    // 1 / (2 Cmax), rounded down (Cmax >= max |c_k|, norm2_up)
    double cb = 0.0;
    for (int k = 0; k < KC; ++k) cb = fmax(cb, norm2_up(cons[2 * k], cons[2 * k + 1]));
    if (lane == 0) {
      kc->ratio = c0k.ratio;
      kc->denom = c0k.denom;
      kc->yd_hi = c0k.yd.hi;
      kc->yd_lo = c0k.yd.lo;
      kc->yd_k = c0k.yd.k;
      kc->inv2c = cb > 0.0 ? (0.5 / cb) * (1.0 - 1e-12) : 0.0;
      kc->mode = c0k.mode;
    }
    if (lane < KC) {
      cs[lane].x = cons[2 * lane];
      cs[lane].y = cons[2 * lane + 1];
    }
  }
  cplx hprev = hat;  // the previous iteration's hatH (clusters_ of the previous iteration: c[k] hprev)
  double drift = 0.0;  // D, the same value in every lane
  double sr = 0.0, si = 0.0;  // cumulative cluster-0 sum (kmeans.cc:33-34, 46)
  int cnt = 0, nmem = 0;
  // lane w < Sw: word w's membership bits and its threshold min(D(ref) + g / (2 Cmax)); -1: assign
  uint64_t wb = 0;
  float wt = -1.0f;
#if KML_KM_WEAK
  // tiers (KML_KM_WEAK): wt is the minimum threshold of the word's kKmWeak weak
  // symbols (packed 7-bit lane indices in wk, bit 6 = none), wt2 that of the others
  float wt2 = -1.0f;
  unsigned wk = 0;
#endif
  uint64_t wb_list = 0;  // lane w: word w's bits and list offset at the last rebuild
  // kSeg: lane w: word w's segment of the value list, offset << 16 | capacity
  // (members + kKmSlack -0.0 fillers, at most 64); nlist: the list's length
  int seg = 0, nlist = 0;
  bool listok = false;
  int excl_list = 0;  // (!kSeg) lane w: word w's list offset at the last rebuild
  const double *yv = reinterpret_cast<const double *>(yy);
  __builtin_amdgcn_wave_barrier();
  KM_STAMP(KS_PRO);
  for (int it = 0; it < iters; ++it) {
    // clusters_[k] = c[k] * hatH and the convergence test against tempClusters
    // (kmeans.cc:26-28 / 72-74, 47-56), lanes k < KC
    {
      bool same = true;
      if (lane < KC) {
        const cplx ck{cs[lane].x, cs[lane].y};
        const cplx p = kml_cmul(ck, hat);
        const cplx pk = it > 0 ? kml_cmul(ck, hprev) : cplx{0.0, 0.0};  // tempClusters: the previous clusters_
        cl[lane] = make_double2(p.re, p.im);
        same = (p.re == pk.re) && (p.im == pk.im);
      }
      const bool conv = __ballot(!same) == 0;
      __builtin_amdgcn_wave_barrier();  // the cluster stores precede the loads below (LDS in order per wave)
      KM_STAMP(KS_CLUSTERS);
      if (conv) break;  // the reference breaks after an assignment it then discards
    }
    KM_COUNT(KS_ITERS, 1);
    {
      const double dd = norm2_up(hat.re - hprev.re, hat.im - hprev.im) +
                        0x1p-48 * (fabs(hat.re) + fabs(hat.im) + fabs(hprev.re) + fabs(hprev.im));
      drift = (drift + dd) * (1.0 + 0x1p-50);
      hprev = hat;
    }
    // assignment (kmeans.cc:36-46) of the words whose decisions the drift may
    // have changed; two words per pass (independent loads, screens and minima)
    int chg = 0;
#if KML_KM_WEAK
    {
      // a full pass over the words whose other symbols' thresholds the drift
      // reached; a gathered pass over the weak symbols of the words where only
      // theirs were reached
      uint64_t need = __ballot(lane < Sw && (!incremental || !(drift < (double)wt2)));
      uint64_t weakw = incremental ? __ballot(lane < Sw && !(drift < (double)wt) && drift < (double)wt2) : 0ull;
      // one pass per flagged word, then passes over up to 21 words' weak
      // symbols (kKmWeak = 3 entries each); the passes share one screen
      while (need | weakw) {  // wave-uniform
        const bool full = need != 0;
        int q = 0, src = 0, b = 0, nw = 0;
        uint64_t chunk = 0;
        if (full) {
          q = __builtin_ctzll(need);
          need &= need - 1;
          b = lane;
        } else {
          const int rank = __popcll(weakw & ((1ull << lane) - 1));
          chunk = __ballot(((weakw >> lane) & 1) && rank < 64 / kKmWeak);
          weakw &= ~chunk;
          // entry i = kKmWeak n + jj: the jj-th weak symbol of the n-th word of the chunk
          for (uint64_t c = chunk; c; c &= c - 1, ++nw)  // scalar loop over the chunk's words
            if (lane / kKmWeak == nw) src = __builtin_ctzll(c);
          const unsigned pk = (unsigned)__shfl((int)wk, src);
          b = lane < kKmWeak * nw ? (int)((pk >> (7 * (lane % kKmWeak))) & 0x7F) : 64;
          q = src;
        }
        const int sym = q * 64 + b;
        const bool valid = b < 64 && sym < S;  // (weak symbols are always valid lanes)
        const double2 v = yy[valid ? sym : 0];
        bool m = false;
        double g = 0.0;
        const bool dec = screen0<KC>(cl, v.x, v.y, m, g);
        if (__ballot(valid && !dec))
          if (valid && !dec) {  // tie band / range: the exact decision
            m = member0_slow<KC>(cl, v.x, v.y);
            g = 0.0;
          }
        float tt = valid ? km_threshold(drift, g, kc->inv2c) : INFINITY;
        if (!full) {  // back to the word lanes: the threshold with the decision in its sign bit
          const float r = m ? -tt : tt;
          const bool mine = (chunk >> lane) & 1;
          const int base = kKmWeak * __popcll(chunk & ((1ull << lane) - 1));
          float nt = INFINITY;
          uint64_t nb = wb;
#pragma unroll
          for (int jj = 0; jj < kKmWeak; ++jj) {
            const float rj = __shfl(r, base + jj);
            const int bj = (int)((wk >> (7 * jj)) & 0x7F);
            if (mine && bj < 64) {
              nt = fminf(nt, fabsf(rj));
              nb = (nb & ~(1ull << bj)) | ((uint64_t)(__float_as_uint(rj) >> 31) << bj);
            }
          }
          if (__ballot(mine && nb != wb)) chg = 1;
          if (mine) {
            wb = nb;
            wt = nt;
          }
          KM_COUNT(KS_WEAK, 1);
          continue;
        }
        // the kKmWeak smallest thresholds (first lane on ties) are the weak
        // symbols; the rest's minimum is wt2
        float t1 = INFINITY;
        unsigned wkp = 0;
#pragma unroll
        for (int jj = 0; jj < kKmWeak; ++jj) {
          const float mj = wave_min_f(tt);
          const uint64_t at = __ballot(tt == mj);
          const int lj = mj < INFINITY ? __builtin_ctzll(at) : 64;  // 64: none
          if (jj == 0) t1 = mj;
          wkp |= (unsigned)(lj & 0x7F) << (7 * jj);
          if (lane == lj) tt = INFINITY;
        }
        const float t2 = wave_min_f(tt);
        const uint64_t bits = __ballot(valid && m);
        if (it == 0 || bits != lane_u64(wb, q)) chg = 1;
        if (lane == q) {
          wb = bits;
          wt = t1;
          wt2 = t2;
          wk = wkp;
        }
        KM_COUNT(KS_WORDS, 1);
      }
    }
#else
    {
      uint64_t need = __ballot(lane < Sw && (!incremental || !(drift < (double)wt)));
      while (need) {  // wave-uniform, one flagged word per pass
        const int q = __builtin_ctzll(need);
        need &= need - 1;
        const double2 v = yy[min(q * 64 + lane, S - 1)];
        const bool valid = q * 64 + lane < S;
        bool m;
        double g;
        const bool dec = screen0<KC>(cl, v.x, v.y, m, g);
        if (__ballot(valid && !dec))
          if (valid && !dec) {  // tie band / range: the exact decision
            m = member0_slow<KC>(cl, v.x, v.y);
            g = 0.0;
          }
        // D + g / (2 Cmax), rounded down: the (1 - 2^-20) factor covers the
        // float conversion's rounding in the normal range; below FLT_MIN (where
        // a denormal's relative rounding error is unbounded) the threshold is 0,
        // i.e. the word is re-assigned next iteration; past the float range a
        // finite 2^127
        const double td = (drift + g * kc->inv2c) * (1.0 - 0x1p-20);
        const float t = wave_min_f(valid ? (td < 0x1p-126 ? 0.0f : td < 0x1p127 ? (float)td : 0x1p127f) : INFINITY);
        const uint64_t bits = __ballot(valid && m);
        if (it == 0 || bits != lane_u64(wb, q)) chg = 1;
        if (lane == q) {
          wb = bits;
          wt = t;
        }
        KM_COUNT(KS_WORDS, 1);
      }
    }
#endif
    KM_STAMP(KS_ASSIGN);
    if (kSeg && chg) {  // members changed: rewrite the changed words' segments (coalesced loads, lanes = symbols)
      KM_COUNT(KS_COMPACTIONS, 1);
      const int c = __popcll(wb);
      nmem = __builtin_amdgcn_readlane(wave_inclusive_scan_i(c), 63);
      // a new layout at the first iteration, after an overflowing list, or when
      // a word outgrew its segment: every segment sized to its members + slack
      const bool full = it == 0 || !listok || __ballot(lane < Sw && c > (seg & 0xFFFF)) != 0;
      if (full) {
        const int nc = lane < Sw ? min(c + kKmSlack, 64) : 0;
        const int incl = wave_inclusive_scan_i(nc);
        seg = ((incl - nc) << 16) | nc;
        nlist = __builtin_amdgcn_readlane(incl, 63);
        listok = nlist <= L.cap;
      }
      uint64_t need = listok ? __ballot(lane < Sw && (full || wb != wb_list)) : 0ull;
      wb_list = wb;
      while (need) {  // wave-uniform, six words' loads in flight
        int qs[6];
#pragma unroll
        for (int u = 0; u < 6; ++u) {
          qs[u] = need ? __builtin_ctzll(need) : -1;
          need &= need - 1;
        }
        double2 v[6];
#pragma unroll
        for (int u = 0; u < 6; ++u) v[u] = yy[min((qs[u] < 0 ? qs[0] : qs[u]) * 64 + lane, S - 1)];
#pragma unroll
        for (int u = 0; u < 6; ++u)
          if (qs[u] >= 0) {
            const uint64_t bits = lane_u64(wb, qs[u]);
            const int so = __builtin_amdgcn_readlane(seg, qs[u]), off = so >> 16, cw = so & 0xFFFF;
            if ((bits >> lane) & 1) vals[off + __popcll(bits & ((1ull << lane) - 1))] = v[u];
            // the segment's tail: -0.0, the exact identity of the ordered sum
            if (lane >= __popcll(bits) && lane < cw) vals[off + lane] = make_double2(-0.0, -0.0);
          }
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (!kSeg && chg) {  // members changed: rebuild the value list (word by word, coalesced loads, lanes = symbols)
      KM_COUNT(KS_COMPACTIONS, 1);
      const int c = __popcll(wb);
      const int incl = wave_inclusive_scan_i(c);
      const int excl = incl - c;
      // only the words whose members or list offset changed are rewritten (the
      // others' segments hold their values already); all of them after an
      // overflowing list (its tail was never written)
      const bool full = it == 0 || nmem > L.cap;
      uint64_t need = __ballot(lane < Sw && (full || wb != wb_list || excl != excl_list));
      nmem = __builtin_amdgcn_readlane(incl, 63);
      wb_list = wb;
      excl_list = excl;
      while (need) {  // wave-uniform, six words' loads in flight
        int qs[6];
#pragma unroll
        for (int u = 0; u < 6; ++u) {
          qs[u] = need ? __builtin_ctzll(need) : -1;
          need &= need - 1;
        }
        double2 v[6];
#pragma unroll
        for (int u = 0; u < 6; ++u) v[u] = yy[min((qs[u] < 0 ? qs[0] : qs[u]) * 64 + lane, S - 1)];
#pragma unroll
        for (int u = 0; u < 6; ++u)
          if (qs[u] >= 0) {
            const uint64_t bits = lane_u64(wb, qs[u]);
            const int p = __builtin_amdgcn_readlane(excl, qs[u]) + __popcll(bits & ((1ull << lane) - 1));
            if (((bits >> lane) & 1) && p < L.cap) vals[p] = v[u];
          }
      }
      __builtin_amdgcn_wave_barrier();
    }
    KM_STAMP(KS_COMPACT);
    const int n = nmem;
    cnt += n;
    const bool fromwords = kSeg ? !listok : n > L.cap;
    const int nscan = kSeg ? nlist : n;
    if (fromwords) {  // more members than the list holds (degenerate input): straight from the words
      double acc = lane == 0 ? sr : si;  // lane 0: real chain, lane 1: imaginary chain, ascending j
      for (int w = 0; w < Sw; ++w) {
        const uint64_t bits = lane_u64(wb, w);
        if (lane < 2)
          for (uint64_t b = bits; b; b &= b - 1) acc = acc + yv[2 * (w * 64 + __builtin_ctzll(b)) + lane];
      }
      sr = lane_d(acc, 0);
      si = lane_d(acc, 1);
    } else if (scan) {
      int steps = 0;
      sr = ordered_sum_vals1(sr, vals, 0, nscan, lane, steps);  // the real chain, then the imaginary one
      si = ordered_sum_vals1(si, vals, 1, nscan, lane, steps);
      KM_COUNT(KS_STEPS, steps);
    } else {  // lane 0: real chain, lane 1: imaginary chain
      double acc = lane == 0 ? sr : si;
      if (lane < 2)
        for (int i = 0; i < nscan; ++i) acc = acc + reinterpret_cast<const double *>(vals)[2 * i + lane];
      sr = lane_d(acc, 0);
      si = lane_d(acc, 1);
    }
    KM_STAMP(KS_SUM);
    {
      const DdRcp yc = dd_rcp((double)cnt);
      const cplx m0 = cdiv_count(sr, si, cnt, yc);  // kmeans.cc:59-62
      CdivConst c0k;
      c0k.ratio = kc->ratio;
      c0k.denom = kc->denom;
      c0k.yd = DdRcp{kc->yd_hi, kc->yd_lo, kc->yd_k};
      c0k.mode = kc->mode;
      hat = cdiv_const(m0, c0, c0k);  // kmeans.cc:64-71
    }
    KM_STAMP(KS_UPDATE);
  }
#if KML_STAMPS
  if (tid == 0)
    for (int i = 0; i <= KS_WEAK; ++i) atomicAdd(&kml_km_stamps[i], km_acc[i]);
#endif
  if (lane == 0) {
    if (hat_out) hat_out[cw] = make_double2(hat.re, hat.im);  // the final hatH (clusters_ = c[k] * hatH)
    const cplx hh = kml_cdiv(kml_cmul(c0, hat), c0);  // simulator.cc:145
    h_hat[cw] = make_double2(hh.re, hh.im);
    for (int j = 0; j < 4; ++j) {  // simulator.cc:146-148
      const cplx r = kml_cmul(hh, cplx{rot[2 * j], rot[2 * j + 1]});
      h4[(long long)cw * 4 + j] = make_double2(r.re, r.im);
    }
  }
}

template <int KC>
bool run_kmeans_wave(const double *cons, const double *rot, const double2 *y, int S, int iters, int B,
                     double2 *h_hat, double2 *h4, double2 *hat_out, hipStream_t s, hipError_t &err) {
  const size_t lds = (size_t)kWaveWpg * km_wave_lds(S, KC).stride;
  if (S > kMaxS || lds > 160 * 1024) return false;
  if (const char *e = getenv("KML_KMEANS")) {  // A/B switch: "wave" (default) or "split" (the two-launch form)
    if (!strcmp(e, "split")) return false;
    if (strcmp(e, "wave") != 0) {
      static bool warned = false;
      if (!warned) fprintf(stderr, "kmldpc_amd: KML_KMEANS=%s is not a k-means kernel (wave, split); running wave\n", e);
      warned = true;
    }
  }
  err = hipFuncSetAttribute((const void *)km_wave_kernel<KC>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (err != hipSuccess) return true;
  int incremental = 1, scan = 1;
  if (const char *e = getenv("KML_KM_INCR")) incremental = e[0] != '0';
  if (const char *e = getenv("KML_KM_SCAN")) scan = e[0] != '0';
  hipLaunchKernelGGL(km_wave_kernel<KC>, dim3((B + kWaveWpg - 1) / kWaveWpg), dim3(64 * kWaveWpg), lds, s, cons, rot,
                     y, S, iters, B, h_hat, h4, hat_out, incremental, scan);
  err = hipGetLastError();
  return true;
}

template <int KC>
hipError_t run_kmeans(const double *cons, const double *rot, const double2 *y, int S, int iters, int B,
                      KmState *st, uint64_t *mem, double2 *h_hat, double2 *h4, double2 *hat_out, hipStream_t s) {
  hipError_t ferr = hipSuccess;
  if (run_kmeans_wave<KC>(cons, rot, y, S, iters, B, h_hat, h4, hat_out, s, ferr)) return ferr;
  const int Sw = (S + 63) / 64;
  const dim3 lanes((B + 63) / 64), l64(64);
  hipLaunchKernelGGL(km_init_kernel, lanes, l64, 0, s, cons, y, S, B, st);
  const int threads = Sw >= 4 ? 256 : 64 * Sw;
  for (int it = 0; it < iters; ++it) {
    hipLaunchKernelGGL(km_assign_kernel<KC>, dim3(B), dim3(threads), 0, s, cons, y, S, Sw, st, mem);
    hipLaunchKernelGGL(km_update_kernel<KC>, lanes, l64, 0, s, cons, y, S, Sw, iters, B, st, mem);
  }
  hipLaunchKernelGGL(km_final_kernel, lanes, l64, 0, s, cons, rot, B, st, h_hat, h4, hat_out);
  return hipGetLastError();
}

}  // namespace

size_t kmeans_workspace_bytes(int S, int B) {
  return (size_t)B * sizeof(KmState) + (size_t)B * ((S + 63) / 64) * sizeof(uint64_t) + 256;
}

hipError_t launch_kmeans(int Kc, const double *cons, const double *rot, const double2 *y, int S, int iters, int B,
                         double2 *h_hat, double2 *h4, void *ws, hipStream_t s, double2 *hat_out) {
  if (B == 0) return hipSuccess;
  KmState *st = reinterpret_cast<KmState *>(ws);
  uint64_t *mem = reinterpret_cast<uint64_t *>(reinterpret_cast<char *>(ws) + (size_t)B * sizeof(KmState));
  switch (Kc) {
    case 2: return run_kmeans<2>(cons, rot, y, S, iters, B, st, mem, h_hat, h4, hat_out, s);
    case 4: return run_kmeans<4>(cons, rot, y, S, iters, B, st, mem, h_hat, h4, hat_out, s);
    case 8: return run_kmeans<8>(cons, rot, y, S, iters, B, st, mem, h_hat, h4, hat_out, s);
    case 16: return run_kmeans<16>(cons, rot, y, S, iters, B, st, mem, h_hat, h4, hat_out, s);
    case 64: return run_kmeans<64>(cons, rot, y, S, iters, B, st, mem, h_hat, h4, hat_out, s);
    default: return hipErrorInvalidValue;
  }
}

// KMeans::clusters() and idx() after Run (include/kmeans.h:18-19): the final
// clusters_ = c[k] * hatH and the closing assignment loop (kmeans.cc:76-83),
// idx_[i] = the FIRST k minimising glibc hypot(clusters_[k] - data_[i]).  The
// simulator computes idx and drops it (simulator.cc:142); it is what
// KMeans::DumpToMat writes (kmeans.cc:99-109).  One thread per symbol; the
// squared-norm screen of member0 with the exact hypot decision inside the tie
// band, the reference loop for non-finite / extreme values.
namespace {
template <int KC>
__device__ int first_argmin(const double2 *cl, double yr, double yi) {
  double dm = 0.0;
  int km = 0;
  bool fin = true;
  for (int k = 0; k < KC; ++k) {
    const double dr = cl[k].x - yr, di = cl[k].y - yi;
    const double d = dr * dr + di * di;
    if (k == 0 || d < dm) {
      dm = d;
      km = k;
    }
    fin = fin && d2_ok(d);
  }
  if (fin) {
    int ties = 0;
    for (int k = 0; k < KC; ++k) {
      const double dr = cl[k].x - yr, di = cl[k].y - yi;
      ties += (dr * dr + di * di <= dm * (1.0 + kTieBand)) ? 1 : 0;
    }
    if (ties == 1) return km;  // every other squared distance is > dm (1 + 1e-12): hypot orders them alike
    double hb = 0.0;
    int kb = -1;
    for (int k = 0; k < KC; ++k) {  // the band's contenders, exactly, first minimum
      const double dr = cl[k].x - yr, di = cl[k].y - yi;
      if (dr * dr + di * di <= dm * (1.0 + kTieBand)) {
        const double h = kml_hypot(dr, di);
        if (kb < 0 || h < hb) {
          hb = h;
          kb = k;
        }
      }
    }
    return kb;
  }
  double hb = kml_hypot(cl[0].x - yr, cl[0].y - yi);  // the reference loop
  int kb = 0;
  for (int k = 1; k < KC; ++k) {
    const double h = kml_hypot(cl[k].x - yr, cl[k].y - yi);
    if (h < hb) {
      hb = h;
      kb = k;
    }
  }
  return kb;
}

template <int KC>
__global__ __launch_bounds__(256) void km_state_kernel(const double *__restrict__ cons, const double2 *__restrict__ y,
                                                       int S, const double2 *__restrict__ hat,
                                                       double2 *__restrict__ clusters, int *__restrict__ idx) {
  __shared__ double2 cl[KC];
  const int cw = blockIdx.x;  // codewords in x (up to 2^31 - 1), symbol blocks in y
  const cplx h{hat[cw].x, hat[cw].y};
  for (int k = threadIdx.x; k < KC; k += blockDim.x) {
    const cplx p = kml_cmul(cplx{cons[2 * k], cons[2 * k + 1]}, h);  // kmeans.cc:72-74
    cl[k] = make_double2(p.re, p.im);
    if (blockIdx.y == 0 && clusters) clusters[(long long)cw * KC + k] = cl[k];
  }
  __syncthreads();
  const int j = blockIdx.y * blockDim.x + threadIdx.x;
  if (j >= S || !idx) return;
  const double2 v = y[(long long)cw * S + j];
  idx[(long long)cw * S + j] = first_argmin<KC>(cl, v.x, v.y);
}
}  // namespace

hipError_t launch_kmeans_state(int Kc, const double *cons, const double2 *y, int S, int B, const double2 *hat,
                               double2 *clusters, int *idx, hipStream_t s) {
  if (B == 0) return hipSuccess;
  if ((S + 255) / 256 > 65535) return hipErrorInvalidValue;
  const dim3 grid(B, (S + 255) / 256), blk(256);
  switch (Kc) {
    case 2: hipLaunchKernelGGL(km_state_kernel<2>, grid, blk, 0, s, cons, y, S, hat, clusters, idx); break;
    case 4: hipLaunchKernelGGL(km_state_kernel<4>, grid, blk, 0, s, cons, y, S, hat, clusters, idx); break;
    case 8: hipLaunchKernelGGL(km_state_kernel<8>, grid, blk, 0, s, cons, y, S, hat, clusters, idx); break;
    case 16: hipLaunchKernelGGL(km_state_kernel<16>, grid, blk, 0, s, cons, y, S, hat, clusters, idx); break;
    case 64: hipLaunchKernelGGL(km_state_kernel<64>, grid, blk, 0, s, cons, y, S, hat, clusters, idx); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Probe for the device restatements of hypot / complex division / exp (tests).
namespace {
__global__ void math_probe_kernel(const double *in, int n, double *out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double a = in[4 * i], b = in[4 * i + 1], c = in[4 * i + 2], d = in[4 * i + 3];
  out[4 * i] = kml_hypot(a, b);
  const cplx q = kml_cdiv(cplx{a, b}, cplx{c, d});
  out[4 * i + 1] = q.re;
  out[4 * i + 2] = q.im;
  out[4 * i + 3] = kml_exp(a);
}

__global__ void log_probe_kernel(const double *in, int n, double *out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = kml_log(in[i]);
}

__global__ void div_probe_kernel(const double *in, int n, double *out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double n0 = in[3 * i], n1 = in[3 * i + 1], s = in[3 * i + 2];
  double q0, q1, c0, c1;
  bool sus = false;
  div2<true>(n0, n1, s, q0, q1, sus);  // the FAST VN form: dd_quot + dd_check
  const DdRcp y = dd_rcp(s);
  const int flags = (dd_check(n0, s, q0, y) ? 0 : 1) | (dd_check(n1, s, q1, y) ? 0 : 2);
  div2<true, true>(n0, n1, s, c0, c1);
  double *o = out + 12 * (long long)i;
  o[0] = q0;
  o[1] = q1;
  o[2] = div_rn(n0, s);
  o[3] = div_rn(n1, s);
  o[4] = c0;
  o[5] = c1;
  o[6] = rcp_near1(s);
  o[7] = rcp_refine(s);
  o[8] = n0 / s;  // hipcc's '/'
  o[9] = n1 / s;
  o[10] = (double)(flags | (sus ? 4 : 0));
  o[11] = fabs(fma(-__builtin_amdgcn_rcp(s), s, 1.0));  // e0 (exact_div.hpp: documented <= 2^-23)
}
}  // namespace

extern "C" int kml_debug_km_stamps(unsigned long long *out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(kml::kml_km_stamps), sizeof(kml::kml_km_stamps));
  if (reset) {
    unsigned long long zero[KS_SLOTS] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(kml::kml_km_stamps), zero, sizeof(zero));
  }
  return e == hipSuccess ? 0 : -3;
}

hipError_t launch_div_probe(const double *in, int n, double *out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(div_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, n, out);
  return hipGetLastError();
}

hipError_t launch_log_probe(const double *in, int n, double *out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(log_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, n, out);
  return hipGetLastError();
}

hipError_t launch_math_probe(const double *in, int n, double *out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(math_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, n, out);
  return hipGetLastError();
}

}  // namespace kml
