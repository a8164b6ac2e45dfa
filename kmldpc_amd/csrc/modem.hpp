// modem.hpp — constellation file loader (lib/lab/src/modem.cc:87-129) and the
// host-side channel constants the reference derives with glibc.
#pragma once
#include <string>
#include <vector>

namespace kml {

struct Modem {
  int bits = 0;  // input_len_ (bits per symbol)
  int Kc = 0;    // symbol_num_ = 2^bits
  std::vector<double> pts;  // 2*Kc, normalised to unit mean energy (modem.cc:122-128)

  // Validates the labels exactly like modem.cc:113-118 (label bits MSB-first
  // must equal the row index).
  bool load(const std::string &path, std::string &err);
};

// var = 10^(-snr/10), sigma = sqrt(var)  (src/simulator.cc:74-75); snr is Es/N0.
void channel_constants(double snr, double &var, double &sigma, double &noise_scale);
// exp(i*kPi/2*j), j=0..3, with the reference's truncated kPi (utility.h:10,
// simulator.cc:147); rot[2*j], rot[2*j+1].
void rotation_factors(double *rot);

}  // namespace kml
