// Reference-side shims: what a trganda/kmldpc maintainer adds to the reference
// tree to route its hot path through libkmldpc_amd.so (the MI355X build).
// Header-only; compiles against the reference's own headers
// (kmldpc/include, kmldpc/lib/lab/include, kmldpc/lib/toml11) plus
// include/kmldpc_amd.h, and links libkmldpc_amd.so.  Pinned by
// tests/test_integration.py (compile + link here) and
// tests/test_gpu_integration.py (the shims against the reference's CPU classes
// on the GPU box, oracle/shim_check.cc).
//
//   GpuBinaryLDPCCodec    overrides  virtual int lab::BinaryLDPCCodec::Decoder(const double*, int*, int)
//                                    (lib/lab/include/binaryldpccodec.h:20)
//   GpuBinary5GLDPCCodec  overrides  lab::Binary5GLDPCCodec::Decoder (lib/lab/include/binary5gldpccodec.h:17)
//   GpuKmCodec            same call as void KmCodec::Decoder(lab::ModemLinearSystem&,
//                                    const std::vector<std::complex<double>>& h_hats, int* uu_hat)
//                                    (include/kmcodec.h:23-25; not virtual in the reference, so the
//                                    simulator's `KmCodec` type becomes `GpuKmCodec` at its use sites)
//   gpu_kmeans_h_hats     KMeans(received, constellations, 20).Run(); clusters()[0] / c[0] and its
//                         4 rotations (include/kmeans.h:14-22, src/simulator.cc:136-148)
//   GpuKMeans             the kmldpc::KMeans interface (include/kmeans.h:12-32): Run, clusters,
//                         idx and DumpToMat (which the reference only has with matio)
#ifndef KMLDPC_AMD_GPU_CODECS_HPP
#define KMLDPC_AMD_GPU_CODECS_HPP

#include <complex>
#include <cstdint>
#include <cstdlib>
#include <string>
#include <vector>

#include "binary5gldpccodec.h"
#include "binaryldpccodec.h"
#include "kmldpc_amd.h"
#include "log.h"
#include "modemlinearsystem.h"
#include "toml.hpp"

namespace kml_lab {

// The reference's error convention: log an ERROR and exit(-1)
// (binaryldpccodec.cc:77-80, modem.cc:89-92).
inline void check(kml_ctx *ctx, int rc) {
  if (rc != KML_OK) {
    lab::logger::ERROR(std::string("kmldpc_amd: ") + (ctx ? kml_last_error(ctx) : "no context"), true);
    exit(-1);
  }
}

inline kml_ctx *open_ctx(const std::string &config_path, int device) {
  if (kml_abi_version() != KML_ABI_VERSION) {  // a library built from another header (kml_dims' array length, ...)
    lab::logger::ERROR("kmldpc_amd: library ABI " + std::to_string(kml_abi_version()) + ", header ABI " +
                           std::to_string(KML_ABI_VERSION) + ": rebuild against the library's include/kmldpc_amd.h",
                       true);
    exit(-1);
  }
  kml_ctx *ctx = nullptr;
  const int rc = kml_create(config_path.c_str(), nullptr, device, &ctx);
  if (rc != KML_OK) {
    lab::logger::ERROR(std::string("kmldpc_amd: ") + (ctx ? kml_last_error(ctx) : "kml_create failed"), true);
    exit(-1);
  }
  return ctx;
}

// Drop-in subclass of the reference's BP codec.  Same constructor argument
// (the parsed config.toml) plus the config path and a HIP device; Decoder has
// the reference contract: M2V[code_len] = P(bit = 0), uu_hat[code_dim],
// return iter + (iter < max_iter); cc_hat() and syndrom_soft() are updated as
// the CPU decoder updates them (syndrom_soft rows only when a CN phase runs).
// Encoder, ParityCheck and the accessors stay the reference's.
template <class Base>
class GpuLdpcCodec : public Base {
 public:
  GpuLdpcCodec(const toml::value &args, const std::string &config_path, int device = 0)
      : Base(args), ctx_(open_ctx(config_path, device)) {
    check(ctx_, kml_dims(ctx_, dims_));
  }
  // From an existing CPU codec (the reference's copy constructor, binaryldpccodec.h:14):
  // skips a second H load + SystemMatrixH elimination, which takes about a minute
  // on one core for PEG8064.  (Not for Binary5GLDPCCodec, whose copy the
  // reference itself avoids: kmcodec.cc:8-11.)
  GpuLdpcCodec(const Base &cpu, const std::string &config_path, int device = 0)
      : Base(cpu), ctx_(open_ctx(config_path, device)) {
    check(ctx_, kml_dims(ctx_, dims_));
  }
  GpuLdpcCodec(const GpuLdpcCodec &) = delete;
  GpuLdpcCodec &operator=(const GpuLdpcCodec &) = delete;
  ~GpuLdpcCodec() override { kml_destroy(ctx_); }

  int Decoder(const double *M2V, int *uu_hat, int iter_count) override {
    const int K = dims_[KML_DIM_K], ncol = dims_[KML_DIM_NCOL], M = dims_[KML_DIM_M];
    u_.resize(K);
    cch_.resize(ncol);
    syn_.assign(this->syndrom_soft_, this->syndrom_soft_ + M);
    int32_t ret = 0;
    check(ctx_, kml_bp_decode(ctx_, M2V, 1, iter_count, u_.data(), &ret, cch_.data(), syn_.data(), 0));
    for (int i = 0; i < K; i++) uu_hat[i] = u_[i];
    for (int i = 0; i < ncol; i++) this->cc_hat_[i] = cch_[i];
    for (int i = 0; i < M; i++) this->syndrom_soft_[i] = syn_[i];
    return ret;
  }

  // Batched form for callers that gather codewords: M2V[B][code_len] -> uu_hat[B][code_dim].
  void DecodeBatch(const double *M2V, int B, uint8_t *uu_hat, int32_t *ret) {
    check(ctx_, kml_bp_decode(ctx_, M2V, B, this->max_iter(), uu_hat, ret, nullptr, nullptr, 0));
  }

  kml_ctx *context() const { return ctx_; }

 private:
  kml_ctx *ctx_;
  int32_t dims_[KML_DIM_COUNT] = {};
  std::vector<uint8_t> u_, cch_;
  std::vector<double> syn_;
};

using GpuBinaryLDPCCodec = GpuLdpcCodec<lab::BinaryLDPCCodec>;
using GpuBinary5GLDPCCodec = GpuLdpcCodec<lab::Binary5GLDPCCodec>;

// KmCodec::Decoder on the GPU: the same arguments (the modem/channel state
// holding the received symbols, the caller's channel estimates, uu_hat).  One
// estimate: demap + BP; several (the simulator's 4 k-means rotations): the
// syndrome metric per candidate ([xcodec] metric_type / 5gldpc as configured),
// the first minimum, demap with it, BP (kmcodec.cc:54-72).  The noise variance
// is the simulator's var = 10^(-snr/10) (simulator.cc:73-76): call set_snr
// where the simulator calls mls.set_var.  DecodeBatch takes B frames at once.
class GpuKmCodec {
 public:
  GpuKmCodec(const std::string &config_path, int device = 0) : ctx_(open_ctx(config_path, device)) {
    check(ctx_, kml_dims(ctx_, dims_));
  }
  GpuKmCodec(const GpuKmCodec &) = delete;
  GpuKmCodec &operator=(const GpuKmCodec &) = delete;
  ~GpuKmCodec() { kml_destroy(ctx_); }

  void set_snr(double snr) { snr_ = snr; }
  int uu_len() const { return dims_[KML_DIM_K]; }
  int cc_len() const { return dims_[KML_DIM_CCLEN]; }

  void Decoder(lab::ModemLinearSystem &mls, const std::vector<std::complex<double>> &h_hats, int *uu_hat) {
    const std::vector<std::complex<double>> &rx = mls.GetRecvSymbol();
    const int K = uu_len(), nc = (int)h_hats.size();
    std::vector<uint8_t> u(K);
    int32_t chosen = 0;
    // std::complex<double> is layout-compatible with double[2] (re, im)
    check(ctx_, kml_decode_candidates(ctx_, reinterpret_cast<const double *>(rx.data()),
                                      reinterpret_cast<const double *>(h_hats.data()), nc, snr_, 1, u.data(), &chosen,
                                      metrics_, nullptr, 0));
    last_chosen_ = chosen;
    for (int i = 0; i < K; i++) uu_hat[i] = u[i];
  }

  // B frames: y[B][S] received symbols, h_hats[B][nc] estimates, uu_hat[B][K].
  void DecodeBatch(const std::complex<double> *y, const std::complex<double> *h_hats, int nc, int B,
                   uint8_t *uu_hat, int32_t *chosen = nullptr) {
    check(ctx_, kml_decode_candidates(ctx_, reinterpret_cast<const double *>(y),
                                      reinterpret_cast<const double *>(h_hats), nc, snr_, B, uu_hat, chosen, nullptr,
                                      nullptr, 0));
  }

  // GetMetrics of the last Decoder call with several estimates (the reference
  // logs these as "Hhat = ... Metric"); metrics()[last_chosen()] is the minimum.
  const double *metrics() const { return metrics_; }
  int last_chosen() const { return last_chosen_; }
  kml_ctx *context() const { return ctx_; }

 private:
  kml_ctx *ctx_;
  int32_t dims_[KML_DIM_COUNT] = {};
  double snr_ = 0.0;
  double metrics_[4] = {};
  int last_chosen_ = 0;
};

// The simulator's blind channel estimate on the GPU: KMeans(received,
// constellations, 20).Run(), h_hat = clusters()[0] / constellations[0], and
// h_hat * exp(i*kPi/2*j), j = 0..3 (simulator.cc:136-148).
inline std::vector<std::complex<double>> gpu_kmeans_h_hats(kml_ctx *ctx, const std::vector<std::complex<double>> &rx,
                                                           int iters = 20) {
  std::vector<std::complex<double>> h4(4);
  check(ctx, kml_kmeans(ctx, reinterpret_cast<const double *>(rx.data()), 1, iters, nullptr,
                        reinterpret_cast<double *>(h4.data()), 0));
  return h4;
}

// kmldpc::KMeans with the same calls (include/kmeans.h:14-22): the context's
// constellation is the one the reference passes in (mls.constellations()).
class GpuKMeans {
 public:
  GpuKMeans(kml_ctx *ctx, std::vector<std::complex<double>> &data, std::vector<std::complex<double>> &constellations,
            int iter)
      : ctx_(ctx), data_(data), constellations_(constellations), iter_(iter),
        clusters_(constellations.size()), idx_(data.size()) {}
  void Run() {
    check(ctx_, kml_kmeans_state(ctx_, reinterpret_cast<const double *>(data_.data()), 1, iter_,
                                 reinterpret_cast<double *>(clusters_.data()), idx_.data(), 0));
  }
  std::vector<std::complex<double>> clusters() { return clusters_; }
  std::vector<int> idx() { return std::vector<int>(idx_.begin(), idx_.end()); }
  // KMeans::DumpToMat (src/kmeans.cc:99-109): append = the 4 candidates + the true H
  void DumpToMat(std::string &filename, std::vector<std::complex<double>> &append) {
    if (append.size() < 5 ||
        kml_kmeans_dump_mat(filename.c_str(), reinterpret_cast<const double *>(data_.data()), (int)data_.size(),
                            reinterpret_cast<const double *>(clusters_.data()), idx_.data(),
                            reinterpret_cast<const double *>(constellations_.data()), (int)constellations_.size(),
                            reinterpret_cast<const double *>(append.data())) != KML_OK) {
      lab::logger::ERROR("Creating file failed, file name is " + filename, true);  // lab/src/mat.cc:21-24
      exit(-1);
    }
  }

 private:
  kml_ctx *ctx_;
  std::vector<std::complex<double>> data_, constellations_, clusters_;
  std::vector<int32_t> idx_;
  int iter_;
};

}  // namespace kml_lab

#endif
