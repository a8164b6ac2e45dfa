// Reference harness — TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Compiled by oracle/Makefile directly against the reference sources under
// /root/reference (when present) into oracle/_ref/ref_harness.  It drives the
// reference's own public API through the per-codeword loop of
// Simulator::run_blocks (kmldpc/src/simulator.cc:116-167) with a fixed seed
// (CLCRandNum::SetSeed(-1) -> state 17, lab/src/randnum.cc:9-11) and dumps every
// intermediate that the MI355X build must reproduce:
//   uu, cc, true_h, y, k-means h_hat, the 4 phase-candidate metrics, the chosen
//   candidate, P0 = demapper output for the chosen h, the BP return value,
//   cc_hat, syndrom_soft, uu_hat (via KmCodec::Decoder) and the error count.
// The output is a flat little-endian record stream consumed by
// tests/golden/make_golden.py.  Nothing here is copied from the reference; the
// harness only calls its public methods.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "binary5gldpccodec.h"
#include "binaryldpccodec.h"
#include "kmcodec.h"
#include "kmeans.h"
#include "log.h"
#include "modemlinearsystem.h"
#include "randnum.h"
#include "sourcesink.h"
#include "toml.hpp"
#include "utility.h"

static void put(FILE *f, const void *p, size_t n) { fwrite(p, 1, n, f); }
static void put_i32(FILE *f, int32_t v) { put(f, &v, 4); }
static void put_f64(FILE *f, double v) { put(f, &v, 8); }
static void put_bits(FILE *f, const int *v, int n) {
  std::vector<uint8_t> b(n);
  for (int i = 0; i < n; i++) b[i] = (uint8_t)v[i];
  put(f, b.data(), n);
}

int main(int argc, char **argv) {
  if (argc < 5) {
    fprintf(stderr, "usage: %s config.toml snr n_codewords out.bin [mode]\n", argv[0]);
    fprintf(stderr, "  mode: frames (default) | simulate | soft | softhist | rng | kmstate\n");
    return 2;
  }
  const std::string cfg = argv[1];
  const double snr = atof(argv[2]);
  const int ncw = atoi(argv[3]);
  const std::string out_path = argv[4];
  const std::string mode = argc > 5 ? argv[5] : "frames";

  // Log::log_stream(bool) casts the stream to TeeStream* (lab/src/log.cc:71-75),
  // so a TeeStream must be installed; both ends go to a null sink.
  std::ofstream null1("/dev/null"), null2("/dev/null");
  lab::logger::TeeStream tee(null1, null2);
  lab::logger::Log::get().set_log_stream(tee);
  lab::logger::Log::get().set_log_level(lab::logger::Info);

  lab::CLCRandNum::Get().SetSeed(-1);
  lab::CWHRandNum::Get().SetSeed(-1);

  if (mode == "rng") {
    // The host random sources with SetSeed(-1): CLCRandNum / CWHRandNum
    // uniforms and normals, SourceSink::GetSymStr / GetBitStr.
    FILE *f = fopen(out_path.c_str(), "wb");
    if (!f) return 1;
    const int n = ncw;
    for (int i = 0; i < n; i++) put_f64(f, lab::CLCRandNum::Get().Uniform());
    for (int i = 0; i < n; i++) put_f64(f, lab::CWHRandNum::Get().Uniform());
    std::vector<double> nn(n + 1);
    lab::CLCRandNum::Get().Normal(nn.data(), n + 1);  // odd length: the single-value tail
    for (int i = 0; i <= n; i++) put_f64(f, nn[i]);
    lab::CWHRandNum::Get().Normal(nn.data(), n + 1);
    for (int i = 0; i <= n; i++) put_f64(f, nn[i]);
    lab::SourceSink ss;
    std::vector<int> sym(n), bits(n);
    ss.GetSymStr(sym.data(), 16, n);
    for (int i = 0; i < n; i++) put_i32(f, sym[i]);
    ss.GetSymStr(sym.data(), 3, n);
    for (int i = 0; i < n; i++) put_i32(f, sym[i]);
    ss.GetBitStr(bits.data(), n);
    for (int i = 0; i < n; i++) put_i32(f, bits[i]);
    fclose(f);
    return 0;
  }

  std::ifstream ifs(cfg, std::ios_base::binary);
  if (!ifs.is_open()) {
    fprintf(stderr, "cannot open %s\n", cfg.c_str());
    return 1;
  }
  auto args = toml::parse(ifs);

  const bool known_h = toml::find<bool>(toml::find(args, "decoder"), "true_h_arg");
  const bool is5g = toml::find<bool>(toml::find(args, "xcodec"), "5gldpc");

  KmCodec codec(args);
  const int K = codec.uu_len();
  const int N = codec.cc_len();
  lab::ModemLinearSystem mls(args, N);
  double var = pow(10.0, -0.1 * snr);
  double sigma = sqrt(var);
  mls.set_sigma(sigma);
  mls.set_var(var);

  // A directly constructed codec of the same kind exposes the BP internals
  // (return value, cc_hat, syndrom_soft) for the chosen P0.
  // (not built in simulate mode: its H load + SystemMatrixH takes about a
  // minute on one core for PEG8064, and simulate needs only the KmCodec)
  lab::BinaryLDPCCodec *direct = nullptr;
  if (mode == "simulate")
    direct = nullptr;
  else if (is5g)
    direct = new lab::Binary5GLDPCCodec(args);
  else
    direct = new lab::BinaryLDPCCodec(args);
  const int Nint = !direct ? N : (is5g ? N + 0 : direct->code_len());
  const int M = direct ? direct->num_row() : 0;
  const int max_iter = direct ? direct->max_iter() : toml::find<int>(toml::find(args, "ldpc"), "max_iter");

  FILE *f = fopen(out_path.c_str(), "wb");
  if (!f) return 1;
  int S = (int)mls.GetRecvSymbol().size();
  auto cons = mls.constellations();
  int Kc = (int)cons.size();
  // header
  put_i32(f, 0x4B4D4C31);  // 'KML1'
  put_i32(f, K);
  put_i32(f, N);
  put_i32(f, S);
  put_i32(f, M);
  put_i32(f, Kc);
  put_i32(f, known_h ? 1 : 0);
  put_i32(f, is5g ? 1 : 0);
  put_i32(f, max_iter);
  put_i32(f, ncw);
  put_f64(f, snr);
  for (auto &c : cons) {
    put_f64(f, c.real());
    put_f64(f, c.imag());
  }

  if (mode == "simulate") {
    // The reference's own counters path: SourceSink::CntErr per codeword.
    lab::SourceSink ssink;
    ssink.ClrCnt();
    std::vector<int> uu(K), cc(N), uu_hat(K);
    std::vector<int32_t> cw_errs;  // per-codeword error bits (for the BER sigma)
    // wall time of the loop (construction excluded), split into frame
    // generation (source, encoder, channel) and the receive (k-means, Decoder,
    // CntErr): bench.py's single-core reference rate
    double t_gen = 0, t_rx = 0;
    for (int i = 0; i < ncw; i++) {
      const auto t0 = std::chrono::steady_clock::now();
      ssink.GetBitStr(uu.data(), K);
      codec.Encoder(uu.data(), cc.data());
      std::complex<double> true_h;
      lab::CLCRandNum::Get().Normal(true_h);
      true_h *= sqrt(0.5);
      std::vector<std::complex<double>> gh(1, true_h);
      mls.PartitionModemLSystem(cc.data(), gh);
      const auto t1 = std::chrono::steady_clock::now();
      std::vector<std::complex<double>> h_hats;
      if (known_h) {
        h_hats.push_back(true_h);
      } else {
        auto constellations = mls.constellations();
        auto received = mls.GetRecvSymbol();
        kmldpc::KMeans km(received, constellations, 20);
        km.Run();
        auto cl = km.clusters();
        std::complex<double> h_hat = cl[0] / constellations[0];
        for (size_t j = 0; j < 4; j++)
          h_hats.push_back(h_hat * exp(std::complex<double>(0, (lab::kPi / 2) * j)));
      }
      codec.Decoder(mls, h_hats, uu_hat.data());
      ssink.CntErr(uu.data(), uu_hat.data(), K, 1);
      const auto t2 = std::chrono::steady_clock::now();
      t_gen += std::chrono::duration<double>(t1 - t0).count();
      t_rx += std::chrono::duration<double>(t2 - t1).count();
      int e = 0;
      for (int k = 0; k < K; k++) e += uu[k] != uu_hat[k];
      cw_errs.push_back(e);
    }
    put_i32(f, (int32_t)ssink.tot_blk());
    put_i32(f, (int32_t)ssink.err_blk());
    // err_bit is private; recompute from BER exactly: ber = err_bit / tot_bit
    double ber = ssink.ber();
    put_f64(f, ber);
    put_f64(f, ssink.fer());
    for (int32_t e : cw_errs) put_i32(f, e);
    fclose(f);
    fprintf(stderr, "{\"codewords\": %d, \"gen_seconds\": %.6f, \"receive_seconds\": %.6f}\n", ncw, t_gen, t_rx);
    return 0;
  }

  if (mode == "kmstate") {
    // KMeans::clusters() and KMeans::idx() after Run (include/kmeans.h:18-19)
    // on the simulator's frames (simulator.cc:116-142): per codeword y,
    // clusters[Kc], idx[S].
    std::vector<int> uu(K), cc(N);
    for (int i = 0; i < ncw; i++) {
      lab::SourceSink ssink;
      ssink.GetBitStr(uu.data(), K);
      codec.Encoder(uu.data(), cc.data());
      std::complex<double> true_h;
      lab::CLCRandNum::Get().Normal(true_h);
      true_h *= sqrt(0.5);
      std::vector<std::complex<double>> gh(1, true_h);
      mls.PartitionModemLSystem(cc.data(), gh);
      auto constellations = mls.constellations();
      auto received = mls.GetRecvSymbol();
      kmldpc::KMeans km(received, constellations, 20);
      km.Run();
      auto cl = km.clusters();
      auto idx = km.idx();
      put_f64(f, true_h.real());
      put_f64(f, true_h.imag());
      for (auto &v : received) {
        put_f64(f, v.real());
        put_f64(f, v.imag());
      }
      for (auto &v : cl) {
        put_f64(f, v.real());
        put_f64(f, v.imag());
      }
      for (int v : idx) put_i32(f, v);
    }
    fclose(f);
    delete direct;
    return 0;
  }

  if (mode == "soft" || mode == "softhist") {
    // Soft syndrome metric ([xcodec] metric_type = true).  The metric depends
    // on the codec's syndrom_soft_ history (rows are only rewritten when a CN
    // phase runs), so the call sequence must be exactly the simulator's:
    //   soft     : KmCodec::Decoder only (simulator.cc:164); the candidate
    //              metrics and the chosen index are recovered from the codec's
    //              own log records ("Hhat = ... Metric = %.14f", "hatIndex = ").
    //   softhist : KmCodec::GetHistogramData only (histogram mode,
    //              simulator.cc:155); metrics are returned exactly, and uu_hat
    //              is what the last metric decode left.
    std::ostringstream cap;
    std::ofstream null3("/dev/null");
    lab::logger::TeeStream tee2(cap, null3);
    lab::logger::Log::get().set_log_stream(tee2);
    std::vector<int> uu(K), cc(N), uu_hat(K, 0);
    for (int i = 0; i < ncw; i++) {
      lab::SourceSink ssink;
      ssink.GetBitStr(uu.data(), K);
      codec.Encoder(uu.data(), cc.data());
      std::complex<double> true_h;
      lab::CLCRandNum::Get().Normal(true_h);
      true_h *= sqrt(0.5);
      std::vector<std::complex<double>> gh(1, true_h);
      mls.PartitionModemLSystem(cc.data(), gh);
      auto y = mls.GetRecvSymbol();
      std::vector<std::complex<double>> h_hats;
      std::complex<double> h_hat(0, 0);
      if (known_h) {
        h_hats.push_back(true_h);
      } else {
        auto constellations = mls.constellations();
        kmldpc::KMeans km(y, constellations, 20);
        km.Run();
        auto cl = km.clusters();
        h_hat = cl[0] / constellations[0];
        for (size_t j = 0; j < 4; j++)
          h_hats.push_back(h_hat * exp(std::complex<double>(0, (lab::kPi / 2) * j)));
      }
      std::vector<double> metrics(4, 0.0);
      int chosen = 0;
      cap.str("");
      cap.clear();
      if (mode == "softhist") {
        auto m = codec.GetHistogramData(mls, h_hats, uu_hat.data());
        for (size_t j = 0; j < m.size(); j++) metrics[j] = m[j];
        chosen = (int)std::distance(m.begin(), std::min_element(m.begin(), m.end()));
      } else {
        codec.Decoder(mls, h_hats, uu_hat.data());
        std::string line;
        std::istringstream in(cap.str());
        int j = 0;
        while (std::getline(in, line)) {
          size_t k = line.find("Metric = ");
          if (k != std::string::npos && j < 4) metrics[j++] = fabs(strtod(line.c_str() + k + 9, nullptr));
          k = line.find("hatIndex = ");
          if (k != std::string::npos) chosen = atoi(line.c_str() + k + 11);
        }
      }
      int errs = 0;
      for (int t = 0; t < K; t++) errs += (uu[t] != uu_hat[t]);
      put_bits(f, uu.data(), K);
      put_f64(f, true_h.real());
      put_f64(f, true_h.imag());
      for (auto &v : y) {
        put_f64(f, v.real());
        put_f64(f, v.imag());
      }
      put_f64(f, h_hat.real());
      put_f64(f, h_hat.imag());
      for (int j = 0; j < 4; j++) put_f64(f, metrics[j]);
      put_i32(f, chosen);
      put_bits(f, uu_hat.data(), K);
      put_i32(f, errs);
    }
    fclose(f);
    delete direct;
    return 0;
  }

  std::vector<int> uu(K), cc(N), uu_hat(K), uu_hat2(K);
  std::vector<double> p0(N), bitin(N, 0.5);
  for (int i = 0; i < ncw; i++) {
    lab::SourceSink ssink;  // GetBitStr only draws from the RNG singleton
    ssink.GetBitStr(uu.data(), K);
    codec.Encoder(uu.data(), cc.data());
    std::complex<double> true_h;
    lab::CLCRandNum::Get().Normal(true_h);
    true_h *= sqrt(0.5);
    std::vector<std::complex<double>> gh(1, true_h);
    mls.PartitionModemLSystem(cc.data(), gh);
    auto y = mls.GetRecvSymbol();

    std::vector<std::complex<double>> h_hats;
    std::complex<double> h_hat(0, 0);
    std::vector<double> metrics(4, 0.0);
    int chosen = 0;
    if (known_h) {
      h_hats.push_back(true_h);
    } else {
      auto constellations = mls.constellations();
      auto received = mls.GetRecvSymbol();
      kmldpc::KMeans km(received, constellations, 20);
      km.Run();
      auto cl = km.clusters();
      h_hat = cl[0] / constellations[0];
      for (size_t j = 0; j < 4; j++)
        h_hats.push_back(h_hat * exp(std::complex<double>(0, (lab::kPi / 2) * j)));
      metrics = codec.GetHistogramData(mls, h_hats, uu_hat2.data());
      chosen = (int)std::distance(metrics.begin(), std::min_element(metrics.begin(), metrics.end()));
    }
    codec.Decoder(mls, h_hats, uu_hat.data());

    // P0 for the chosen candidate, then a direct decode for the internals.
    std::vector<std::pair<int, std::complex<double>>> th = {{0, h_hats[chosen]}};
    for (int t = 0; t < N; t++) bitin[t] = 0.5;
    mls.DeMapping(th, bitin.data(), p0.data());
    int ret = direct->Decoder(p0.data(), uu_hat2.data(), max_iter);

    int errs = 0;
    for (int t = 0; t < K; t++) errs += (uu[t] != uu_hat[t]);

    put_bits(f, uu.data(), K);
    put_bits(f, cc.data(), N);
    put_f64(f, true_h.real());
    put_f64(f, true_h.imag());
    for (auto &v : y) {
      put_f64(f, v.real());
      put_f64(f, v.imag());
    }
    put_f64(f, h_hat.real());
    put_f64(f, h_hat.imag());
    for (int j = 0; j < 4; j++) put_f64(f, metrics[j]);
    put_i32(f, chosen);
    put(f, p0.data(), sizeof(double) * N);
    put_i32(f, ret);
    int nint = is5g ? N + 0 : Nint;
    (void)nint;
    // cc_hat has num_col entries (internal length, incl. punctured columns for 5G)
    int ncol = 0;
    {
      // num_col is not exposed; for PEG it equals code_len, for 5G it is
      // N + 2Z which equals M + K.
      ncol = is5g ? (M + K) : direct->code_len();
    }
    put_i32(f, ncol);
    put_bits(f, direct->cc_hat(), ncol);
    put(f, direct->syndrom_soft(), sizeof(double) * M);
    put_bits(f, uu_hat.data(), K);
    put_bits(f, uu_hat2.data(), K);
    put_i32(f, errs);
  }
  fclose(f);
  delete direct;
  return 0;
}
