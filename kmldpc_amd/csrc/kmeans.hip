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
// MI355X mapping — one k-means iteration is two launches:
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
#include <cstdlib>

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
                                double2 *__restrict__ h4) {
  const int cw = blockIdx.x * blockDim.x + threadIdx.x;
  if (cw >= B) return;
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
// Fused k-means: one workgroup per codeword runs the whole KMeans::Run.  The
// symbols are staged in LDS once; each iteration assigns in parallel (same
// screening as km_assign, 64-symbol words by ballot), compacts the cluster-0
// members' values into LDS in ascending symbol order, and two lanes run the
// re / im accumulation chains in that order (the reference's sequential sum,
// software-pipelined so the adds, not the LDS latency, set its pace); lane 0
// then tests convergence and updates h_hat.  One launch instead of two per
// iteration, and y is read from HBM once.
constexpr int kFusedT = 256;
constexpr int kFusedMaxW = 64;  // 64-symbol words: S <= 4096

__device__ __forceinline__ double wave_max(double v) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ int wave_min_i(int v) {
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o));
  return v;
}

// acc + x[0] + x[2] + ... + x[2(n-1)] in that order (stride 2: one component
// of a double2 array).
__device__ __forceinline__ double ordered_sum(double acc, const double *x, int n) {
  int i = 0;
  for (; i + 4 <= n; i += 4) {
    const double a0 = x[2 * i], a1 = x[2 * i + 2], a2 = x[2 * i + 4], a3 = x[2 * i + 6];
    acc = acc + a0;
    acc = acc + a1;
    acc = acc + a2;
    acc = acc + a3;
  }
  for (; i < n; ++i) acc = acc + x[2 * i];
  return acc;
}

template <int KC>
__global__ __launch_bounds__(kFusedT) void km_fused_kernel(const double *__restrict__ cons,
                                                           const double *__restrict__ rot,
                                                           const double2 *__restrict__ y, int S, int iters,
                                                           double2 *__restrict__ h_hat, double2 *__restrict__ h4) {
  extern __shared__ __attribute__((aligned(16))) unsigned char kmem[];
  double2 *ys = reinterpret_cast<double2 *>(kmem);  // [S] symbols
  double2 *ym = ys + S;                              // [S] compacted cluster-0 members
  __shared__ double2 cl[KC];
  __shared__ uint64_t wbits[kFusedMaxW];
  __shared__ int wpos[kFusedMaxW + 1];
  __shared__ double red_d[kFusedT / 64];
  __shared__ int red_i[kFusedT / 64];
  __shared__ double2 s_hat;
  __shared__ int s_done, s_exact;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int NW = kFusedT / 64;
  const int cw = blockIdx.x;
  const int Sw = (S + 63) / 64;
  const double2 *yy = y + (long long)cw * S;
  for (int j = tid; j < S; j += kFusedT) ys[j] = yy[j];
  if (tid == 0) s_exact = 0;
  __syncthreads();

  // ---- first max |y| (kmeans.cc:17-22), screened like first_max_abs
  double best = -1.0;
  bool ex = false;
  for (int j = tid; j < S; j += kFusedT) {
    const double2 v = ys[j];
    const double d = v.x * v.x + v.y * v.y;
    if (!d2_ok(d) && !(d == 0.0)) ex = true;
    if (d > best) best = d;
  }
  best = wave_max(best);
  const bool wex = __ballot(ex) != 0;
  if (lane == 0) {
    red_d[wave] = best;
    if (wex) s_exact = 1;
  }
  __syncthreads();
  best = red_d[0];
  for (int w = 1; w < NW; ++w) best = fmax(best, red_d[w]);
  int mi;
  if (!s_exact && best > 0.0) {
    double hb = -1.0;  // max exact |y| among the band's candidates
    for (int j = tid; j < S; j += kFusedT) {
      const double2 v = ys[j];
      if (v.x * v.x + v.y * v.y >= best * (1.0 - kTieBand)) hb = fmax(hb, kml_hypot(v.x, v.y));
    }
    hb = wave_max(hb);
    __syncthreads();
    if (lane == 0) red_d[wave] = hb;
    __syncthreads();
    hb = red_d[0];
    for (int w = 1; w < NW; ++w) hb = fmax(hb, red_d[w]);
    int jm = 0x7fffffff;  // the first index attaining it
    for (int j = tid; j < S; j += kFusedT) {
      const double2 v = ys[j];
      if (v.x * v.x + v.y * v.y >= best * (1.0 - kTieBand) && kml_hypot(v.x, v.y) == hb) jm = min(jm, j);
    }
    jm = wave_min_i(jm);
    if (lane == 0) red_i[wave] = jm;
    __syncthreads();
    mi = red_i[0];
    for (int w = 1; w < NW; ++w) mi = min(mi, red_i[w]);
  } else {  // the reference loop, sequentially (non-finite / extreme / all-zero input)
    if (tid == 0) {
      int m = 0;
      double h0 = kml_hypot(ys[0].x, ys[0].y);
      for (int j = 1; j < S; ++j) {
        const double h = kml_hypot(ys[j].x, ys[j].y);
        if (h0 < h) {
          h0 = h;
          m = j;
        }
      }
      red_i[0] = m;
    }
    __syncthreads();
    mi = red_i[0];
  }
  const cplx c0{cons[0], cons[1]};
  cplx hat = kml_cdiv(cplx{ys[mi].x, ys[mi].y}, c0);  // kmeans.cc:25
  cplx prev{0.0, 0.0};
  bool have_prev = false;
  double sr = 0.0, si = 0.0;  // cumulative cluster-0 sum (kmeans.cc:33-34, 46)
  int cnt = 0;
  for (int it = 0; it < iters; ++it) {
    for (int k = tid; k < KC; k += kFusedT) {
      const cplx p = kml_cmul(cplx{cons[2 * k], cons[2 * k + 1]}, hat);  // clusters_[k] = c[k] * hatH
      cl[k] = make_double2(p.re, p.im);
    }
    __syncthreads();
    // assignment: is cluster 0 the first minimum?  (kmeans.cc:36-46)
    for (int w = wave; w < Sw; w += NW) {
      const int j = w * 64 + lane;
      const bool m = j < S && member0<KC>(cl, ys[j].x, ys[j].y);
      const uint64_t bits = __ballot(m);
      if (lane == 0) wbits[w] = bits;
    }
    __syncthreads();
    if (tid < 64) {  // word offsets: exclusive prefix of the popcounts (Sw <= 64)
      int c = tid < Sw ? __popcll(wbits[tid]) : 0;
      int x = c;
      for (int o = 1; o < 64; o <<= 1) {
        const int t = __shfl_up(x, o);
        if (lane >= o) x += t;
      }
      wpos[tid] = x - c;
      if (tid == 63) wpos[kFusedMaxW] = x;
    }
    __syncthreads();
    for (int w = wave; w < Sw; w += NW) {
      const uint64_t bits = wbits[w];
      if ((bits >> lane) & 1) ym[wpos[w] + __popcll(bits & ((1ull << lane) - 1))] = ys[w * 64 + lane];
    }
    __syncthreads();
    const int n = wpos[kFusedMaxW];
    if (tid < 2) {  // lane 0: real chain, lane 1: imaginary chain, ascending j
      const double acc = ordered_sum(tid == 0 ? sr : si, reinterpret_cast<const double *>(ym) + tid, n);
      const double other = __shfl_xor(acc, 1);
      sr = tid == 0 ? acc : other;
      si = tid == 0 ? other : acc;
      cnt += n;
      if (tid == 0) {
        // convergence: every cluster equals the previous iteration's (kmeans.cc:47-56)
        bool same = true;
        for (int k = 0; k < KC && same; ++k) {
          const cplx ck{cons[2 * k], cons[2 * k + 1]};
          const cplx a = kml_cmul(ck, hat);
          const cplx b = have_prev ? kml_cmul(ck, prev) : cplx{0.0, 0.0};
          same = (a.re == b.re) && (a.im == b.im);
        }
        int done = 0;
        if (same) {
          done = 1;
        } else {
          prev = hat;
          have_prev = true;
          const cplx m0 = kml_cdiv(cplx{sr, si}, cplx{(double)cnt, 0.0});  // kmeans.cc:59-62
          hat = kml_cdiv(m0, c0);                                         // kmeans.cc:64-71
        }
        s_hat = make_double2(hat.re, hat.im);
        s_done = done;
      }
    }
    __syncthreads();
    hat = cplx{s_hat.x, s_hat.y};
    if (s_done) break;
  }
  if (tid == 0) {
    const cplx hh = kml_cdiv(kml_cmul(c0, hat), c0);  // simulator.cc:145
    h_hat[cw] = make_double2(hh.re, hh.im);
    for (int j = 0; j < 4; ++j) {  // simulator.cc:146-148
      const cplx r = kml_cmul(hh, cplx{rot[2 * j], rot[2 * j + 1]});
      h4[(long long)cw * 4 + j] = make_double2(r.re, r.im);
    }
  }
}

template <int KC>
bool run_kmeans_fused(const double *cons, const double *rot, const double2 *y, int S, int iters, int B,
                      double2 *h_hat, double2 *h4, hipStream_t s, hipError_t &err) {
  const size_t lds = 2 * sizeof(double2) * (size_t)S;
  if (S > 64 * kFusedMaxW || lds > 128 * 1024) return false;
  if (const char *e = getenv("KML_KMEANS"))
    if (e[0] == 's') return false;  // KML_KMEANS=split: the two-launch form (A/B)
  err = hipFuncSetAttribute((const void *)km_fused_kernel<KC>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (err != hipSuccess) return true;
  hipLaunchKernelGGL(km_fused_kernel<KC>, dim3(B), dim3(kFusedT), lds, s, cons, rot, y, S, iters, h_hat, h4);
  err = hipGetLastError();
  return true;
}

template <int KC>
hipError_t run_kmeans(const double *cons, const double *rot, const double2 *y, int S, int iters, int B,
                      KmState *st, uint64_t *mem, double2 *h_hat, double2 *h4, hipStream_t s) {
  hipError_t ferr = hipSuccess;
  if (run_kmeans_fused<KC>(cons, rot, y, S, iters, B, h_hat, h4, s, ferr)) return ferr;
  const int Sw = (S + 63) / 64;
  const dim3 lanes((B + 63) / 64), l64(64);
  hipLaunchKernelGGL(km_init_kernel, lanes, l64, 0, s, cons, y, S, B, st);
  const int threads = Sw >= 4 ? 256 : 64 * Sw;
  for (int it = 0; it < iters; ++it) {
    hipLaunchKernelGGL(km_assign_kernel<KC>, dim3(B), dim3(threads), 0, s, cons, y, S, Sw, st, mem);
    hipLaunchKernelGGL(km_update_kernel<KC>, lanes, l64, 0, s, cons, y, S, Sw, iters, B, st, mem);
  }
  hipLaunchKernelGGL(km_final_kernel, lanes, l64, 0, s, cons, rot, B, st, h_hat, h4);
  return hipGetLastError();
}

}  // namespace

size_t kmeans_workspace_bytes(int S, int B) {
  return (size_t)B * sizeof(KmState) + (size_t)B * ((S + 63) / 64) * sizeof(uint64_t) + 256;
}

hipError_t launch_kmeans(int Kc, const double *cons, const double *rot, const double2 *y, int S, int iters, int B,
                         double2 *h_hat, double2 *h4, void *ws, hipStream_t s) {
  if (B == 0) return hipSuccess;
  KmState *st = reinterpret_cast<KmState *>(ws);
  uint64_t *mem = reinterpret_cast<uint64_t *>(reinterpret_cast<char *>(ws) + (size_t)B * sizeof(KmState));
  switch (Kc) {
    case 2: return run_kmeans<2>(cons, rot, y, S, iters, B, st, mem, h_hat, h4, s);
    case 4: return run_kmeans<4>(cons, rot, y, S, iters, B, st, mem, h_hat, h4, s);
    case 8: return run_kmeans<8>(cons, rot, y, S, iters, B, st, mem, h_hat, h4, s);
    case 16: return run_kmeans<16>(cons, rot, y, S, iters, B, st, mem, h_hat, h4, s);
    case 64: return run_kmeans<64>(cons, rot, y, S, iters, B, st, mem, h_hat, h4, s);
    default: return hipErrorInvalidValue;
  }
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
  double q0, q1, r0, r1, c0, c1;
  div2<true>(n0, n1, s, q0, q1);
  div2<false>(n0, n1, s, r0, r1);
  div2<true, true>(n0, n1, s, c0, c1);
  double *o = out + 8 * (long long)i;
  o[0] = q0;
  o[1] = q1;
  o[2] = r0;
  o[3] = r1;
  o[4] = c0;
  o[5] = c1;
  o[6] = rcp_near1(s);
  o[7] = rcp_refine(s);
}
}  // namespace

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
