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
// Only cluster 0's running sum/count is ever read back, so that is all we keep;
// the per-symbol assignment still evaluates every cluster to find the first
// minimum (kmeans.cc:41-44).
//
// Mapping: one LANE per codeword.  The cluster-0 sum is a sequential
// floating-point chain in ascending symbol order (its rounding is part of the
// result), so the parallelism has to come from independent codewords, not from
// splitting a codeword's symbols.  A wavefront carries 64 independent chains.
#include "bp_common.hpp"
#include "exact_math.hpp"
#include "kernels.hpp"

namespace kml {

namespace {

template <int KC>
__global__ __launch_bounds__(64) void kmeans_kernel(const double *__restrict__ cons, const double *__restrict__ rot,
                                                    const double2 *__restrict__ y, int S, int iters, int B,
                                                    double2 *__restrict__ h_hat, double2 *__restrict__ h4) {
  const int cw = blockIdx.x * blockDim.x + threadIdx.x;
  if (cw >= B) return;
  const double2 *yy = y + (long long)cw * S;
  const cplx c0{cons[0], cons[1]};

  // first max of |y| (kmeans.cc:17-22)
  int mi = 0;
  double best = kml_hypot(yy[0].x, yy[0].y);
  for (int j = 1; j < S; ++j) {
    const double2 v = yy[j];
    const double a = kml_hypot(v.x, v.y);
    if (best < a) {
      best = a;
      mi = j;
    }
  }
  cplx hat = kml_cdiv(cplx{yy[mi].x, yy[mi].y}, c0);  // kmeans.cc:25
  cplx prev{0.0, 0.0};
  bool have_prev = false;  // tempClusters starts as zeros
  long long cnt0 = 0;
  double s0r = 0.0, s0i = 0.0;
  for (int it = 0; it < iters; ++it) {
    for (int j = 0; j < S; ++j) {
      const double2 v = yy[j];
      const cplx cl0 = kml_cmul(c0, hat);
      double dmin = kml_hypot(cl0.re - v.x, cl0.im - v.y);
      int kmin = 0;
#pragma unroll 4
      for (int k = 1; k < KC; ++k) {
        const cplx cl = kml_cmul(cplx{cons[2 * k], cons[2 * k + 1]}, hat);
        const double d = kml_hypot(cl.re - v.x, cl.im - v.y);
        if (d < dmin) {  // min_element: first minimum
          dmin = d;
          kmin = k;
        }
      }
      if (kmin == 0) {
        cnt0++;
        s0r = s0r + v.x;
        s0i = s0i + v.y;
      }
    }
    bool same = true;  // kmeans.cc:47-56
    for (int k = 0; k < KC && same; ++k) {
      const cplx ck{cons[2 * k], cons[2 * k + 1]};
      const cplx cl = kml_cmul(ck, hat);
      const cplx tp = have_prev ? kml_cmul(ck, prev) : cplx{0.0, 0.0};
      same = (cl.re == tp.re) && (cl.im == tp.im);
    }
    if (same) break;
    prev = hat;
    have_prev = true;
    const cplx cl0 = kml_cdiv(cplx{s0r, s0i}, cplx{(double)(int)cnt0, 0.0});  // kmeans.cc:59-62
    hat = kml_cdiv(cl0, c0);                                                 // kmeans.cc:64-71
  }
  const cplx hh = kml_cdiv(kml_cmul(c0, hat), c0);  // simulator.cc:145
  h_hat[cw] = make_double2(hh.re, hh.im);
#pragma unroll
  for (int j = 0; j < 4; ++j) {  // simulator.cc:146-148
    const cplx r = kml_cmul(hh, cplx{rot[2 * j], rot[2 * j + 1]});
    h4[(long long)cw * 4 + j] = make_double2(r.re, r.im);
  }
}

}  // namespace

hipError_t launch_kmeans(int Kc, const double *cons, const double *rot, const double2 *y, int S, int iters, int B,
                         double2 *h_hat, double2 *h4, hipStream_t s) {
  if (B == 0) return hipSuccess;
  const dim3 grid((B + 63) / 64), blk(64);
  switch (Kc) {
    case 2: hipLaunchKernelGGL(kmeans_kernel<2>, grid, blk, 0, s, cons, rot, y, S, iters, B, h_hat, h4); break;
    case 4: hipLaunchKernelGGL(kmeans_kernel<4>, grid, blk, 0, s, cons, rot, y, S, iters, B, h_hat, h4); break;
    case 8: hipLaunchKernelGGL(kmeans_kernel<8>, grid, blk, 0, s, cons, rot, y, S, iters, B, h_hat, h4); break;
    case 16: hipLaunchKernelGGL(kmeans_kernel<16>, grid, blk, 0, s, cons, rot, y, S, iters, B, h_hat, h4); break;
    case 64: hipLaunchKernelGGL(kmeans_kernel<64>, grid, blk, 0, s, cons, rot, y, S, iters, B, h_hat, h4); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// Probe for the device restatements of hypot / complex division (tests).
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
__global__ void div_probe_kernel(const double *in, int n, double *out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double n0 = in[3 * i], n1 = in[3 * i + 1], s = in[3 * i + 2];
  double q0, q1, r0, r1;
  div2<true>(n0, n1, s, q0, q1);
  div2<false>(n0, n1, s, r0, r1);
  out[4 * i] = q0;
  out[4 * i + 1] = q1;
  out[4 * i + 2] = r0;
  out[4 * i + 3] = r1;
}
}  // namespace

hipError_t launch_div_probe(const double *in, int n, double *out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(div_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, n, out);
  return hipGetLastError();
}

hipError_t launch_math_probe(const double *in, int n, double *out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(math_probe_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, n, out);
  return hipGetLastError();
}

}  // namespace kml
