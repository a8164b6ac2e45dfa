// Pins kml_log (kmldpc_amd/csrc/exact_math.hpp) against the host glibc log.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include "../../kmldpc_amd/csrc/exact_math.hpp"

static bool same(double a, double b) { return memcmp(&a, &b, 8) == 0 || (std::isnan(a) && std::isnan(b)); }

int main(int argc, char **argv) {
  long n = argc > 1 ? atol(argv[1]) : 2000000;
  std::mt19937_64 g(11);
  std::uniform_real_distribution<double> e(-45.0, 1.0), near1(-0x1p-4, 0x1.09p-4), wide(-1070.0, 1023.0);
  long bad_f = 0, bad_n = 0;
  for (long i = 0; i < n; i++) {
    double x;
    switch (i % 5) {
      case 0: x = std::exp2(e(g)); break;          // probabilities (syndrom_soft in (0, 1])
      case 1: x = 1.0 + near1(g); break;           // the close-to-1 branch
      case 2: x = std::exp2(wide(g)); break;       // every exponent incl. subnormals
      case 3: x = 1e-12 + (1.0 - 2e-12) * std::generate_canonical<double, 53>(g); break;
      default: { uint64_t b = g() & 0x7fffffffffffffffull; memcpy(&x, &b, 8); }  // raw bit patterns
    }
    if (i < 8) {
      const double sp[8] = {0.0, -0.0, 1.0, INFINITY, -1.0, NAN, 4.9e-324, 1.0 - 0x1p-53};
      x = sp[i];
    }
    volatile double xv = x;
    double ref = std::log(xv);
    double a = kml::kml_log_t<true>(x), b = kml::kml_log_t<false>(x);
    if (!same(a, ref)) { if (bad_f < 5) printf("fma   x=%a ref=%a got=%a\n", x, ref, a); bad_f++; }
    if (!same(b, ref)) bad_n++;
  }
  printf("n=%ld log_fma_mismatch=%ld log_nofma_mismatch=%ld\n", n, bad_f, bad_n);
  return bad_f ? 1 : 0;
}
