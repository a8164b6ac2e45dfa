// Shim check — TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Compiled by oracle/Makefile against the reference sources under
// /root/reference (when present) and linked with kmldpc_amd/libkmldpc_amd.so
// into oracle/_ref/shim_check.  It runs the reference's per-codeword loop
// (Simulator::run_blocks, kmldpc/src/simulator.cc:116-167, seed 17) and feeds
// every codeword both to the reference's own CPU classes and to the drop-in
// shims of integration/kmldpc_gpu_codecs.hpp:
//   lab::BinaryLDPCCodec::Decoder  vs  GpuBinaryLDPCCodec::Decoder   (ret, uu_hat, cc_hat, syndrom_soft)
//   KmCodec::Decoder               vs  GpuKmCodec::Decoder          (uu_hat)
//   KMeans + rotations             vs  gpu_kmeans_h_hats            (the 4 candidates, bitwise)
// and prints one JSON line of mismatch counts.  Needs a GPU (run by
// tests/test_gpu_integration.py on the GPU box; only compiled here).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <string>
#include <vector>

#include "kmcodec.h"
#include "kmeans.h"
#include "kmldpc_gpu_codecs.hpp"
#include "sourcesink.h"

int main(int argc, char **argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s config.toml snr n_codewords\n", argv[0]);
    return 2;
  }
  const std::string cfg = argv[1];
  const double snr = atof(argv[2]);
  const int ncw = atoi(argv[3]);
  std::ofstream null1("/dev/null"), null2("/dev/null");
  lab::logger::TeeStream tee(null1, null2);
  lab::logger::Log::get().set_log_stream(tee);
  lab::logger::Log::get().set_log_level(lab::logger::Info);
  lab::CLCRandNum::Get().SetSeed(-1);

  std::ifstream ifs(cfg, std::ios_base::binary);
  if (!ifs.is_open()) return 1;
  auto args = toml::parse(ifs);
  const bool known_h = toml::find<bool>(toml::find(args, "decoder"), "true_h_arg");
  const bool is5g = toml::find<bool>(toml::find(args, "xcodec"), "5gldpc");

  KmCodec ref_km(args);
  kml_lab::GpuKmCodec gpu_km(cfg, 0);
  gpu_km.set_snr(snr);
  std::unique_ptr<lab::BinaryLDPCCodec> ref_bp, gpu_bp;
  if (is5g) {
    ref_bp.reset(new lab::Binary5GLDPCCodec(args));
    gpu_bp.reset(new kml_lab::GpuBinary5GLDPCCodec(args, cfg, 0));
  } else {  // the GPU codec copies the CPU one (no second SystemMatrixH elimination)
    auto *cpu = new lab::BinaryLDPCCodec(args);
    ref_bp.reset(cpu);
    gpu_bp.reset(new kml_lab::GpuBinaryLDPCCodec(*cpu, cfg, 0));
  }
  const int K = ref_km.uu_len(), N = ref_km.cc_len();
  int32_t dims[KML_DIM_COUNT];
  kml_lab::check(gpu_km.context(), kml_dims(gpu_km.context(), dims));
  const int ncol = dims[KML_DIM_NCOL];  // cc_hat_ length: code_len_ (PEG), code_len_no_puncture_ (5G)
  const int M = ref_bp->num_row();
  lab::ModemLinearSystem mls(args, N);
  const double var = pow(10.0, -0.1 * snr);
  mls.set_sigma(sqrt(var));
  mls.set_var(var);
  lab::SourceSink ssink;
  std::vector<int> uu(K), cc(N), uu_ref(K), uu_gpu(K), b_ref(K), b_gpu(K);
  std::vector<double> bit_in(N, 0.5), m2v(N);
  int mm_km = 0, mm_bp_ret = 0, mm_bp_uu = 0, mm_bp_cc = 0, mm_bp_syn = 0, mm_cand = 0, mm_kmstate = 0, err_ref = 0,
      err_gpu = 0;
  for (int i = 0; i < ncw; i++) {
    ssink.GetBitStr(uu.data(), K);
    ref_km.Encoder(uu.data(), cc.data());
    std::complex<double> true_h;
    lab::CLCRandNum::Get().Normal(true_h);
    true_h *= sqrt(0.5);
    std::vector<std::complex<double>> gh(1, true_h);
    mls.PartitionModemLSystem(cc.data(), gh);
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
      for (size_t j = 0; j < 4; j++) h_hats.push_back(h_hat * exp(std::complex<double>(0, (lab::kPi / 2) * j)));
      auto g4 = kml_lab::gpu_kmeans_h_hats(gpu_km.context(), mls.GetRecvSymbol());
      if (memcmp(g4.data(), h_hats.data(), sizeof(double) * 8) != 0) mm_cand++;
      kml_lab::GpuKMeans gkm(gpu_km.context(), received, constellations, 20);
      gkm.Run();
      auto gcl = gkm.clusters();
      if (gcl != cl || gkm.idx() != km.idx()) mm_kmstate++;
      if (i == 0) {  // KMeans::DumpToMat of the first codeword (append = candidates + true H)
        std::string fn = "kmeans0.mat";
        std::vector<std::complex<double>> app(h_hats);
        app.push_back(true_h);
        gkm.DumpToMat(fn, app);
      }
    }
    // the whole receive step
    ref_km.Decoder(mls, h_hats, uu_ref.data());
    gpu_km.Decoder(mls, h_hats, uu_gpu.data());
    if (uu_ref != uu_gpu) mm_km++;
    for (int k = 0; k < K; k++) {
      err_ref += uu[k] != uu_ref[k];
      err_gpu += uu[k] != uu_gpu[k];
    }
    // the BP codec alone, on the demapper output for the first estimate
    std::vector<std::pair<int, std::complex<double>>> theta = {{0, h_hats[0]}};
    mls.DeMapping(theta, bit_in.data(), m2v.data());
    const int r1 = ref_bp->Decoder(m2v.data(), b_ref.data(), ref_bp->max_iter());
    const int r2 = gpu_bp->Decoder(m2v.data(), b_gpu.data(), gpu_bp->max_iter());
    if (r1 != r2) mm_bp_ret++;
    if (b_ref != b_gpu) mm_bp_uu++;
    if (memcmp(ref_bp->cc_hat(), gpu_bp->cc_hat(), sizeof(int) * ncol) != 0) mm_bp_cc++;
    if (memcmp(ref_bp->syndrom_soft(), gpu_bp->syndrom_soft(), sizeof(double) * M) != 0) mm_bp_syn++;
  }
  printf("{\"codewords\": %d, \"K\": %d, \"known\": %d, \"is5g\": %d, \"kmcodec_uu_mismatch\": %d, "
         "\"candidate_mismatch\": %d, \"bp_ret_mismatch\": %d, \"bp_uu_mismatch\": %d, \"bp_cc_hat_mismatch\": %d, "
         "\"bp_syndrom_soft_mismatch\": %d, \"kmeans_state_mismatch\": %d, \"err_bit_ref\": %d, "
         "\"err_bit_gpu\": %d}\n",
         ncw, K, known_h ? 1 : 0, is5g ? 1 : 0, mm_km, mm_cand, mm_bp_ret, mm_bp_uu, mm_bp_cc, mm_bp_syn, mm_kmstate,
         err_ref, err_gpu);
  return 0;
}
