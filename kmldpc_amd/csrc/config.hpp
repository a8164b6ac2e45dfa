// config.hpp — the config.toml subset the reference reads.
//
// The reference parses config.toml with toml11 v3.5.0 and reads these keys with
// toml::find<T> (src/simulator.cc:7-15, src/kmcodec.cc:22-25,
// lib/lab/src/binaryldpccodec.cc:70-73, lib/lab/src/modem.cc:6-7,
// src/simulator.cc:33-34).  We parse exactly that subset: [section] headers,
// `key = value` with booleans, integers, floats and basic strings, and `#`
// comments.  Unlike toml11 an integer is accepted where a float is expected.
#pragma once
#include <map>
#include <string>

namespace kml {

struct TomlValue {
  enum Kind { Bool, Int, Float, String } kind = String;
  bool b = false;
  long long i = 0;
  double f = 0.0;
  std::string s;
};

class Config {
 public:
  // Returns false and fills err on a syntax error.
  bool parse_file(const std::string &path, std::string &err);
  bool parse_string(const std::string &text, std::string &err);

  bool has(const std::string &sec, const std::string &key) const;
  // Typed getters: return false + err when missing or of the wrong type.
  bool get_bool(const std::string &sec, const std::string &key, bool &out, std::string &err) const;
  bool get_int(const std::string &sec, const std::string &key, long long &out, std::string &err) const;
  bool get_float(const std::string &sec, const std::string &key, double &out, std::string &err) const;
  bool get_string(const std::string &sec, const std::string &key, std::string &out, std::string &err) const;

 private:
  std::map<std::string, std::map<std::string, TomlValue>> tables_;
  const TomlValue *find(const std::string &sec, const std::string &key, std::string &err) const;
};

// The full set of keys a kmldpc run uses, with the reference's meaning.
struct RunConfig {
  // [range]
  double min_snr = 0, max_snr = 0, step_snr = 1;
  long long max_err_blk = 0, max_num_blk = 0, thread_num_blk = 0;
  // [decoder]
  bool known_h = false;
  // [xcodec]
  bool is5g = false, metric_soft = false;
  int metric_iter = 5;
  // [histogram]
  bool histogram = false;
  // [ldpc]
  int max_iter = 20;
  bool active = true;
  std::string matrix_file;
  // [modem]
  std::string modem_file;
};

// Reads every key above.  Missing [range]/[decoder]/[histogram] sections are
// allowed (codec-only use); [xcodec], [ldpc] and [modem] are required.
// Relative file paths are resolved against base_dir when it is non-empty
// (the reference resolves them against the CWD).
bool load_run_config(const std::string &path, const std::string &base_dir, RunConfig &rc, std::string &err);

}  // namespace kml
