// Pins kml_exp (kmldpc_amd/csrc/exact_math.hpp) against the host glibc exp.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include "../../kmldpc_amd/csrc/exact_math.hpp"

int main(int argc, char **argv) {
  long n = argc > 1 ? atol(argv[1]) : 2000000;
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> u(-40.0, 0.0), w(-760.0, 720.0), t(-1e-10, 1e-10), s(-746.0, -700.0);
  long bad_f = 0, bad_n = 0;
  for (long i = 0; i < n; i++) {
    double x = (i % 4 == 0) ? w(g) : (i % 97 == 0 ? t(g) : (i % 5 == 1 ? s(g) : u(g)));
    if (i % 1001 == 0) x = -std::ldexp(1.0, -(int)(i % 70));
    volatile double xv = x;
    double ref = std::exp(xv);
    double a = kml::kml_exp_t<true>(x), b = kml::kml_exp_t<false>(x);
    if (!(a == ref)) { if (bad_f < 5) printf("fma   x=%a ref=%a got=%a\n", x, ref, a); bad_f++; }
    if (!(b == ref)) bad_n++;
  }
  printf("n=%ld exp_fma_mismatch=%ld exp_nofma_mismatch=%ld\n", n, bad_f, bad_n);
  return bad_f ? 1 : 0;
}
