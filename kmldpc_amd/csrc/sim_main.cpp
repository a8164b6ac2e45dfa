// sim_main.cpp — `kmldpc_sim`, the drop-in for the reference executable
// (kmldpc/kmldpc.cpp): reads config.toml (or argv[1]), runs the SNR sweep of
// Simulator::Simulate (src/simulator.cc:24-67) on one GPU through the C ABI, and
// prints the reference's console lines (timestamped [INFO] records, per-point
// progress every 100 blocks, the BER / FER result tables, total time), teeing
// them to logs/<time>-kmldpc.logger when a logs/ directory exists.
//
// Differences, by design: the SNR points run one after another on the GPU
// (the reference runs them on concurrent threads, interleaving their progress
// lines); frames come from the counter-based GPU generator, so the numbers are
// statistically, not bitwise, equal to a reference run (bitwise parity of the
// receive path is established on the reference's own frames, tests/); the
// per-codeword debug records the reference writes only to the log file
// ("Generated H", "Hhat = ... Metric", "hatIndex") are not produced.
//
// Environment: KML_DEVICE (GPU ordinal, default 0), KML_BATCH (codewords per
// GPU round, default 32768), KML_SEED (frame seed, default 0 like
// CLCRandNum::SetSeed(0) in kmldpc.cpp:22).
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <sys/stat.h>
#include <vector>

#include "../../include/kmldpc_amd.h"

namespace {

FILE *g_log = nullptr;

std::string now_string() {  // Log::get_time (log.cc:77-87)
  std::time_t t = std::time(nullptr);
  char buf[50] = {0};
  strftime(buf, sizeof buf, "%Y-%m-%d %H:%M:%S", localtime(&t));
  return buf;
}

void emit(const char *tag, const std::string &msg) {
  const std::string line = "[" + now_string() + "]" + tag + msg + "\n";
  fputs(line.c_str(), stdout);
  fflush(stdout);
  if (g_log) {
    fputs(line.c_str(), g_log);
    fflush(g_log);
  }
}
void info(const std::string &m) { emit(" \x1b[32;1m[INFO]\x1b[0m ", m); }
void error(const std::string &m) { emit(" \x1b[31;1m[ERROR]\x1b[0m ", m); }

std::string fmt(const char *f, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, f);
  vsnprintf(buf, sizeof buf, f, ap);
  va_end(ap);
  return buf;
}

// SourceSink::PrintResult (sourcesink.cc:50-65): zero-filled width-7 counters,
// 14-digit BER / FER.
void print_result(double snr, const uint64_t *c) {
  const double ber = c[2] ? (double)c[0] / (double)c[2] : 0.0;
  const double fer = c[3] ? (double)c[1] / (double)c[3] : 0.0;
  info(fmt("SNR = %03.3f Total blk = %07llu Error blk = %07llu Error bit = %07llu BER = %.14f FER = %.14f", snr,
           (unsigned long long)c[3], (unsigned long long)c[1], (unsigned long long)c[0], ber, fer));
}

struct Progress {
  double snr;
};
void on_progress(const uint64_t *c, void *user) { print_result(static_cast<Progress *>(user)->snr, c); }

std::string dir_of(const std::string &p) {
  const size_t k = p.find_last_of('/');
  return k == std::string::npos ? std::string(".") : p.substr(0, k);
}

// std::to_string(double) == "%f"
std::string hist_name(double snr) { return "histogram_" + fmt("%f", snr) + ".txt"; }

}  // namespace

int main(int argc, char **argv) {
  const auto begin = std::chrono::steady_clock::now();
  struct stat st;
  if (stat("logs", &st) == 0 && S_ISDIR(st.st_mode)) {
    const std::string name = "logs/" + now_string() + "-kmldpc.logger";
    g_log = fopen(name.c_str(), "w");
  }
  info("Start simulation");
  const std::string cfg = argc > 1 ? argv[1] : "config.toml";
  {
    FILE *f = fopen(cfg.c_str(), "rb");
    if (!f) {
      error("Encouter error while opening config.toml");  // kmldpc.cpp:36 (sic)
      info("Simulation done");
      return 0;
    }
    fclose(f);
  }
  const int device = getenv("KML_DEVICE") ? atoi(getenv("KML_DEVICE")) : 0;
  const int batch = getenv("KML_BATCH") ? atoi(getenv("KML_BATCH")) : 32768;
  const uint64_t seed = getenv("KML_SEED") ? strtoull(getenv("KML_SEED"), nullptr, 10) : 0;
  kml_ctx *ctx = nullptr;
  if (kml_create(cfg.c_str(), dir_of(cfg).c_str(), device, &ctx) != KML_OK) {
    error(ctx ? kml_last_error(ctx) : "kml_create failed");
    kml_destroy(ctx);
    return 255;  // the reference exits with -1 on setup errors
  }
  double f[3];
  int64_t n[10];
  kml_run_config(ctx, f, n);
  const double min_snr = f[0], max_snr = f[1], step_snr = f[2];
  info(n[4] ? "Using 5G LDPC." : "Using traditional LDPC.");  // kmcodec.cc:27,32
  info(fmt("[%.3f,%.3f,%.3f]", min_snr, step_snr, max_snr));  // simulator.cc:16-18
  info(fmt("[MAX_ERROR_BLK = %lld,MAX_BLK = %lld]", (long long)n[0], (long long)n[1]));
  const unsigned long points = (unsigned long)((max_snr - min_snr) / step_snr + 1);
  std::vector<double> snrs, ber, fer;
  int rc = KML_OK;
  for (unsigned long i = 0; i < points && rc == KML_OK; i++) {
    const double snr = min_snr + step_snr * i;
    kml_point_cfg pc{};
    pc.snr = snr;
    pc.rank = 0;
    pc.world = 1;
    pc.batch = batch > 0 ? batch : 32768;
    pc.max_blocks = n[1] > 0 ? (uint64_t)n[1] : 0;
    pc.max_err = n[0] > 0 ? (uint64_t)n[0] : 0;
    pc.report_every = 100;
    const std::string hist = hist_name(snr);
    pc.hist_path = n[7] ? hist.c_str() : nullptr;
    Progress pr{snr};
    uint64_t c[4] = {0, 0, 0, 0};
    const uint64_t point_seed = seed ^ (0x9E3779B97F4A7C15ull * (uint64_t)(i + 1));
    rc = kml_sim_point(ctx, &pc, point_seed, nullptr, nullptr, on_progress, &pr, c);
    if (rc != KML_OK) {
      error(kml_last_error(ctx));
      break;
    }
    print_result(snr, c);  // Simulator::run's final PrintResult
    snrs.push_back(snr);
    ber.push_back(c[2] ? (double)c[0] / (double)c[2] : 0.0);
    fer.push_back(c[3] ? (double)c[1] / (double)c[3] : 0.0);
  }
  if (rc == KML_OK) {
    info("BER Result");
    for (size_t i = 0; i < snrs.size(); i++) info(fmt("%03.3f %.14f", snrs[i], ber[i]));
    info("FER Result");
    for (size_t i = 0; i < snrs.size(); i++) info(fmt("%03.3f %.14f", snrs[i], fer[i]));
  }
  kml_destroy(ctx);
  info("Simulation done");
  const auto end = std::chrono::steady_clock::now();
  long long ms = std::chrono::duration_cast<std::chrono::milliseconds>(end - begin).count();
  const long long mins = ms / 60000, secs = ms / 1000 - mins * 60;
  ms -= mins * 60 * 1000;
  info(fmt("Total time cost: %lldmin:%lldsec:%lldms", mins, secs, ms));
  if (g_log) fclose(g_log);
  return rc == KML_OK ? 0 : 1;
}
