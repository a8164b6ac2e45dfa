// Host-code exercise for the AddressSanitizer / UndefinedBehaviorSanitizer build
// (tests/test_host.py::test_host_code_under_sanitizers): the planner, the config
// parser, the constellation loader and the reference-stream frame generator run
// on the reference's data files AND on malformed inputs (truncated / garbage
// files, broken TOML), so every error path is walked with the sanitizers on.
// Prints "san_errors=0" on success (the sanitizers themselves abort on a finding).
//   host_san_check <data dir> <scratch dir>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "code.hpp"
#include "config.hpp"
#include "layout.hpp"
#include "modem.hpp"

namespace kml {
int ref_frames(const LdpcCode &code, const Modem &modem, int64_t *state, double snr, int n, uint8_t *uu_out,
               double *h_out, double *y_out);
}
using namespace kml;

static int errors = 0;
#define CHECK(c, msg)                                   \
  do {                                                  \
    if (!(c)) {                                         \
      ++errors;                                         \
      printf("FAIL %s: %s\n", #c, std::string(msg).c_str()); \
    }                                                   \
  } while (0)

static std::string slurp(const std::string &p) {
  std::ifstream f(p, std::ios::binary);
  std::stringstream ss;
  ss << f.rdbuf();
  return ss.str();
}

static void spit(const std::string &p, const std::string &s) {
  std::ofstream f(p, std::ios::binary);
  f << s;
}

// A code that loads must encode to H-codewords: the syndrome of the encoded
// internal codeword is zero on every row (PEG: cc is the internal codeword).
static void check_code(const std::string &path, bool is5g, const Modem &modem, int64_t seed) {
  for (int active = 0; active < 2; active++) {
    LdpcCode L;
    std::string err;
    CHECK(L.load(path, is5g, active != 0, false, err), path + ": " + err);
    if (!err.empty()) continue;
    std::vector<uint8_t> uu(L.K), cc(L.cc_len);
    uint32_t x = 12345u + active;
    for (int rep = 0; rep < 4; rep++) {
      for (int i = 0; i < L.K; i++) {
        x = x * 1664525u + 1013904223u;
        uu[i] = (x >> 31) & 1;
      }
      L.encode(uu.data(), cc.data());
      if (!is5g) {
        int bad = 0;
        for (int r = 0; r < L.M; r++) {
          int s = 0;
          for (int e = L.row_ptr[r]; e < L.row_ptr[r + 1]; e++) s ^= cc[L.row_col[e]];
          bad += s;
        }
        CHECK(bad == 0, path + " syndrome rows " + std::to_string(bad));
      }
    }
    // plans the kernels use (their own checks are in plan_check.cpp)
    if (L.dv_max == 3 && L.N <= 4096) {
      RegularLayout rl;
      plan_regular_layout(L, 1024, rl);
    }
    if (is5g) {
      IrregularPlan ip;
      plan_irregular(L, kIrrThreads, kIrrVnPairMax, kIrrCnPairMax, ip);
    }
    if (L.N > 4096) {
      PartitionPlan pp;
      plan_partition(L, 4, pp);
    }
    // the reference's frame stream through the host encoder and mapper
    if (L.cc_len % modem.bits == 0) {
      const int n = 3, S = L.cc_len / modem.bits;
      std::vector<uint8_t> fu((size_t)n * L.K);
      std::vector<double> h(2 * n), y((size_t)2 * n * S);
      int64_t st = seed;
      CHECK(ref_frames(L, modem, &st, 2.0, n, fu.data(), h.data(), y.data()) == 0, path);
    }
  }
  // error paths: missing file, truncated file, garbage
  const std::string text = slurp(path);
  const std::string cuts[] = {"", text.substr(0, text.size() / 3), text.substr(0, 7), "x y z\n1 2\n",
                              "-5 3\n1 1\n", "4 2\n1 2\n1 1 1 1\n9 9\n"};
  for (const std::string &c : cuts) {
    const std::string p = path + ".bad";
    spit(p, c);
    LdpcCode L;
    std::string err;
    L.load(p, is5g, true, false, err);  // must return (either way) without a sanitizer finding
  }
  LdpcCode L;
  std::string err;
  CHECK(!L.load(path + ".missing", is5g, true, false, err), "missing file accepted");
}

static void check_modem(const std::string &path) {
  Modem m;
  std::string err;
  CHECK(m.load(path, err), path + ": " + err);
  CHECK(m.Kc == (1 << m.bits) && (int)m.pts.size() == 2 * m.Kc, path);
  const std::string text = slurp(path);
  const std::string cuts[] = {"", text.substr(0, text.size() / 2), "2\n0 0 1.0\n", "99\n", "garbage\n"};
  for (const std::string &c : cuts) {
    spit(path + ".bad", c);
    Modem b;
    b.load(path + ".bad", err);
  }
}

static void check_config(const std::string &scratch, const std::string &data) {
  // the reference's config.toml keys (src/simulator.cc, config.cpp load_run_config)
  const char *good =
      "# comment\n[range]\nminimum_snr = 1.5\nmaximum_snr = 2\nstep_snr = 0.5\nmaximum_error_number = 100\n"
      "maximum_block_number = 1_000\nthread_block_number = 10\n[decoder]\ntrue_h_arg = true\n[xcodec]\n"
      "5gldpc = false\nmetric_type = false\nmetric_iter = 5\n[histogram]\nenable = false\n[ldpc]\nmax_iter = 20\n"
      "active = true\nmatrix_file = \"PEG2304regular0.5.txt\"\n[modem]\nmodem_file = \"2bits_QPSK.txt\"\n";
  Config c;
  std::string err;
  CHECK(c.parse_string(good, err), err);
  double f = 0;
  long long i = 0;
  bool b = false;
  std::string s;
  CHECK(c.get_float("range", "minimum_snr", f, err) && f == 1.5, err);
  CHECK(c.get_int("range", "maximum_block_number", i, err) && i == 1000, err);
  CHECK(c.get_bool("decoder", "true_h_arg", b, err) && b, err);
  CHECK(c.get_string("ldpc", "matrix_file", s, err) && s == "PEG2304regular0.5.txt", err);
  CHECK(!c.get_int("ldpc", "matrix_file", i, err), "string read as int");
  CHECK(!c.get_bool("nope", "x", b, err), "missing table read");
  spit(scratch + "/config.toml", good);
  RunConfig rc;
  CHECK(load_run_config(scratch + "/config.toml", data, rc, err), err);
  const std::string deep(1000, '[');
  const char *bad[] = {"[range", "[range]\nx = \"unterminated\n", "[a]\n= 3\n", "[a]\nx = 99999999999999999999999\n",
                       "[a]\nx = 1e99999\n", "[a]\nx = tru\n", "[a]\nx\n", "[a]\nx = [1, 2\n", "\"\n", "[]\n",
                       "[a]\nx = 'lit'\ny = \"\\u00e9\\n\"\n", deep.c_str(), "[a]\nx = -\n",
                       "[a]\nx = 0x\n", "[a]\nx = 1.\n", "[a]\nx = .5\n", "[a]\nx = \"a\" # c\nx = 2\n"};
  for (const char *t : bad) {
    Config d;
    d.parse_string(t, err);  // must return without a sanitizer finding
  }
  spit(scratch + "/bad.toml", std::string(good).replace(std::string(good).find("1.5"), 3, "\"a\""));
  CHECK(!load_run_config(scratch + "/bad.toml", data, rc, err), "bad run config accepted");
}

int main(int argc, char **argv) {
  if (argc < 3) {
    printf("usage: host_san_check <data dir> <scratch dir>\n");
    return 2;
  }
  const std::string data = argv[1], scratch = argv[2];
  const char *modems[] = {"2bits_QPSK.txt", "2bits_4PSK.txt", "4bit_16QAM_Gray.txt", "6bits_64QAM_Gray.txt"};
  for (const char *m : modems) {
    // copy into scratch so the truncated variants land there
    spit(scratch + "/" + m, slurp(data + "/" + m));
    check_modem(scratch + "/" + m);
  }
  Modem qpsk, qam16, qam64;
  std::string err;
  qpsk.load(data + "/2bits_QPSK.txt", err);
  qam16.load(data + "/4bit_16QAM_Gray.txt", err);
  qam64.load(data + "/6bits_64QAM_Gray.txt", err);
  const char *codes[] = {"PEG2304regular0.5.txt", "5GLDPCBG2a3_R12_K960.txt", "PEG8064regular0.5.txt"};
  const Modem *cm[] = {&qpsk, &qam16, &qam64};
  for (int k = 0; k < 3; k++) {
    spit(scratch + "/" + codes[k], slurp(data + "/" + codes[k]));
    check_code(scratch + "/" + codes[k], k == 1, *cm[k], -1 - k);
  }
  check_config(scratch, data);
  printf("san_errors=%d\n", errors);
  return errors != 0;
}
