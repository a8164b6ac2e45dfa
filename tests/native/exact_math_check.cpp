// Pins kmldpc_amd/csrc/exact_math.hpp against glibc hypot, libgcc __divdc3 and
// std::complex<double> operator* (inline product + libgcc __muldc3) — the
// routines the reference calls.  Built and run by tests/test_host.py.
#include <cmath>
#include <complex>
#include <cstdio>
#include <cstdlib>
#include <random>
#include "../../kmldpc_amd/csrc/exact_math.hpp"

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 2000000;
  std::mt19937_64 g(12345);
  std::normal_distribution<double> nd(0.0, 1.0);
  std::uniform_real_distribution<double> ud(-30, 30);
  long bad_h = 0, bad_d = 0;
  for (long i = 0; i < n; i++) {
    double s = std::exp2(ud(g) * (i % 7 == 0 ? 10 : 1));
    double x = nd(g) * s, y = nd(g) * (i % 3 == 0 ? s : 1.0);
    if (i % 11 == 0) y = x * (1 + 1e-9 * nd(g));
    if (i % 13 == 0) y = 0.0;
    double h1 = std::hypot(x, y), h2 = kml::kml_hypot(x, y);
    if (!(h1 == h2)) { if (bad_h < 5) printf("hypot %a %a: %a vs %a\n", x, y, h1, h2); bad_h++; }
    double a = nd(g) * s, b = nd(g), c = nd(g), d = nd(g) * (i % 5 == 0 ? 0.0 : 1.0);
    if (i % 17 == 0) c = 0.0;
    if (i % 19 == 0) { c = (double)(1 + i % 300); d = 0.0; }
    std::complex<double> q = std::complex<double>(a, b) / std::complex<double>(c, d);
    kml::cplx r = kml::kml_cdiv({a, b}, {c, d});
    bool same = (q.real() == r.re || (q.real() != q.real() && r.re != r.re)) &&
                (q.imag() == r.im || (q.imag() != q.imag() && r.im != r.im));
    if (!same) { if (bad_d < 5) printf("cdiv (%a,%a)/(%a,%a): (%a,%a) vs (%a,%a)\n", a, b, c, d, q.real(), q.imag(), r.re, r.im); bad_d++; }
  }
  // complex products, with infinities, NaNs, zeros and overflow among the operands
  const double sp[] = {0.0, -0.0, 1.0, -2.5, 1e300, -1e300, 1e-300, INFINITY, -INFINITY, NAN, -NAN};
  const int nsp = sizeof(sp) / sizeof(sp[0]);
  long bad_m = 0, nm = 0;
  auto same_d = [](double u, double v) {
    return (u != u && v != v) || (u == v && std::signbit(u) == std::signbit(v));
  };
  auto check_mul = [&](double a, double b, double c, double d) {
    volatile double va = a, vb = b, vc = c, vd = d;  // no constant folding of the library product
    const std::complex<double> q = std::complex<double>(va, vb) * std::complex<double>(vc, vd);
    const kml::cplx r = kml::kml_cmul({a, b}, {c, d});
    ++nm;
    if (!same_d(q.real(), r.re) || !same_d(q.imag(), r.im)) {
      if (bad_m < 5) printf("cmul (%a,%a)*(%a,%a): (%a,%a) vs (%a,%a)\n", a, b, c, d, q.real(), q.imag(), r.re, r.im);
      bad_m++;
    }
  };
  for (int i = 0; i < nsp; i++)
    for (int j = 0; j < nsp; j++)
      for (int k = 0; k < nsp; k++)
        for (int l = 0; l < nsp; l++) check_mul(sp[i], sp[j], sp[k], sp[l]);
  for (long i = 0; i < n / 4; i++) {
    const double s = std::exp2(ud(g) * 10);
    check_mul(nd(g) * s, nd(g), nd(g) * s, nd(g) * (i % 5 == 0 ? 0.0 : 1.0));
  }
  printf("n=%ld hypot_mismatch=%ld cdiv_mismatch=%ld cmul_mismatch=%ld (of %ld)\n", n, bad_h, bad_d, bad_m, nm);
  return (bad_h || bad_d || bad_m) ? 1 : 0;
}
