// Pins kmldpc_amd/csrc/exact_math.hpp against glibc hypot and libgcc __divdc3
// (the routines the reference calls).  Built and run by tests/test_host.py.
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
  printf("n=%ld hypot_mismatch=%ld cdiv_mismatch=%ld\n", n, bad_h, bad_d);
  return (bad_h || bad_d) ? 1 : 0;
}
