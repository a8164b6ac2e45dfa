#include "modem.hpp"

#include <cmath>
#include <complex>
#include <cstdlib>
#include <fstream>
#include <sstream>

namespace kml {

bool Modem::load(const std::string &path, std::string &err) {
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) {
    err = "Cannot open " + path;
    return false;
  }
  std::string tok;
  int out_len = 0;
  if (!(f >> tok >> bits >> tok >> out_len >> tok) || bits <= 0 || bits > 8) {
    err = "bad constellation header in " + path;
    return false;
  }
  Kc = 1 << bits;
  pts.assign(2 * Kc, 0.0);
  double energies = 0;
  for (int i = 0; i < Kc; i++) {
    int dec = 0, acc = 0;
    if (!(f >> dec)) {
      err = "truncated constellation file " + path;
      return false;
    }
    for (int j = 0; j < bits; j++) {
      int b = 0;
      if (!(f >> b)) {
        err = "truncated constellation file " + path;
        return false;
      }
      acc = (acc << 1) + b;
    }
    if (dec != acc || dec != i) {
      err = std::to_string(dec) + " is not the binary expression of " + std::to_string(acc);
      return false;
    }
    double re = 0, im = 0;
    if (!(f >> re >> im)) {
      err = "bad point in " + path;
      return false;
    }
    pts[2 * i] = re;
    pts[2 * i + 1] = im;
    energies += std::pow(std::abs(std::complex<double>(re, im)), 2);
  }
  energies /= Kc;
  const double s = std::sqrt(energies);
  for (int i = 0; i < 2 * Kc; i++) pts[i] /= s;
  return true;
}

void channel_constants(double snr, double &var, double &sigma, double &noise_scale) {
  var = std::pow(10.0, -0.1 * (snr));
  sigma = std::sqrt(var);
  noise_scale = sigma / 1.4142135623730950488016;  // sigma_ / kSqrt2 (modemlinearsystem.cc:45)
}

void rotation_factors(double *rot) {
  const double kPi = 3.14159265358979;
  for (int j = 0; j < 4; j++) {
    std::complex<double> r = std::exp(std::complex<double>(0, (kPi / 2) * (double)j));
    rot[2 * j] = r.real();
    rot[2 * j + 1] = r.imag();
  }
}

}  // namespace kml
