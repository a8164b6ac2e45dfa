#include "config.hpp"

#include <cerrno>
#include <cstdlib>
#include <fstream>
#include <sstream>

namespace kml {

static std::string trim(const std::string &s) {
  size_t a = 0, b = s.size();
  while (a < b && (s[a] == ' ' || s[a] == '\t' || s[a] == '\r')) a++;
  while (b > a && (s[b - 1] == ' ' || s[b - 1] == '\t' || s[b - 1] == '\r')) b--;
  return s.substr(a, b - a);
}

// Strip a trailing comment that is not inside a string.
static std::string strip_comment(const std::string &s) {
  bool in_str = false;
  for (size_t i = 0; i < s.size(); i++) {
    if (s[i] == '"' && (i == 0 || s[i - 1] != '\\')) in_str = !in_str;
    if (s[i] == '#' && !in_str) return s.substr(0, i);
  }
  return s;
}

static bool parse_value(const std::string &raw, TomlValue &v, std::string &err) {
  std::string t = trim(raw);
  if (t.empty()) {
    err = "empty value";
    return false;
  }
  if (t == "true" || t == "false") {
    v.kind = TomlValue::Bool;
    v.b = (t == "true");
    return true;
  }
  if (t[0] == '"') {
    if (t.size() < 2 || t.back() != '"') {
      err = "unterminated string: " + t;
      return false;
    }
    std::string out;
    for (size_t i = 1; i + 1 < t.size(); i++) {
      if (t[i] == '\\' && i + 2 < t.size()) {
        char n = t[++i];
        out += (n == 'n') ? '\n' : (n == 't') ? '\t' : n;
      } else {
        out += t[i];
      }
    }
    v.kind = TomlValue::String;
    v.s = out;
    return true;
  }
  if (t[0] == '\'') {
    if (t.size() < 2 || t.back() != '\'') {
      err = "unterminated literal string: " + t;
      return false;
    }
    v.kind = TomlValue::String;
    v.s = t.substr(1, t.size() - 2);
    return true;
  }
  std::string num;
  for (char ch : t)
    if (ch != '_') num += ch;
  bool is_float = num.find_first_of(".eE") != std::string::npos || num == "inf" || num == "+inf" ||
                  num == "-inf" || num == "nan";
  char *end = nullptr;
  errno = 0;
  if (is_float) {
    v.f = strtod(num.c_str(), &end);
    v.kind = TomlValue::Float;
  } else {
    v.i = strtoll(num.c_str(), &end, 10);
    v.kind = TomlValue::Int;
  }
  if (!end || *end != '\0' || errno) {
    err = "bad value: " + t;
    return false;
  }
  return true;
}

bool Config::parse_string(const std::string &text, std::string &err) {
  std::istringstream in(text);
  std::string line, section;
  int lineno = 0;
  while (std::getline(in, line)) {
    lineno++;
    std::string t = trim(strip_comment(line));
    if (t.empty()) continue;
    if (t[0] == '[') {
      if (t.back() != ']') {
        err = "line " + std::to_string(lineno) + ": bad table header";
        return false;
      }
      section = trim(t.substr(1, t.size() - 2));
      tables_[section];
      continue;
    }
    size_t eq = t.find('=');
    if (eq == std::string::npos) {
      err = "line " + std::to_string(lineno) + ": expected key = value";
      return false;
    }
    std::string key = trim(t.substr(0, eq));
    if (key.size() >= 2 && key.front() == '"' && key.back() == '"') key = key.substr(1, key.size() - 2);
    TomlValue v;
    std::string verr;
    if (!parse_value(t.substr(eq + 1), v, verr)) {
      err = "line " + std::to_string(lineno) + ": " + verr;
      return false;
    }
    tables_[section][key] = v;
  }
  return true;
}

bool Config::parse_file(const std::string &path, std::string &err) {
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) {
    err = "cannot open config " + path;
    return false;
  }
  std::stringstream ss;
  ss << f.rdbuf();
  return parse_string(ss.str(), err);
}

bool Config::has(const std::string &sec, const std::string &key) const {
  auto it = tables_.find(sec);
  return it != tables_.end() && it->second.count(key);
}

const TomlValue *Config::find(const std::string &sec, const std::string &key, std::string &err) const {
  auto it = tables_.find(sec);
  if (it == tables_.end()) {
    err = "missing table [" + sec + "]";
    return nullptr;
  }
  auto jt = it->second.find(key);
  if (jt == it->second.end()) {
    err = "missing key " + sec + "." + key;
    return nullptr;
  }
  return &jt->second;
}

bool Config::get_bool(const std::string &sec, const std::string &key, bool &out, std::string &err) const {
  const TomlValue *v = find(sec, key, err);
  if (!v) return false;
  if (v->kind != TomlValue::Bool) {
    err = sec + "." + key + " must be a boolean";
    return false;
  }
  out = v->b;
  return true;
}

bool Config::get_int(const std::string &sec, const std::string &key, long long &out, std::string &err) const {
  const TomlValue *v = find(sec, key, err);
  if (!v) return false;
  if (v->kind != TomlValue::Int) {
    err = sec + "." + key + " must be an integer";
    return false;
  }
  out = v->i;
  return true;
}

bool Config::get_float(const std::string &sec, const std::string &key, double &out, std::string &err) const {
  const TomlValue *v = find(sec, key, err);
  if (!v) return false;
  if (v->kind == TomlValue::Float)
    out = v->f;
  else if (v->kind == TomlValue::Int)
    out = (double)v->i;
  else {
    err = sec + "." + key + " must be a number";
    return false;
  }
  return true;
}

bool Config::get_string(const std::string &sec, const std::string &key, std::string &out, std::string &err) const {
  const TomlValue *v = find(sec, key, err);
  if (!v) return false;
  if (v->kind != TomlValue::String) {
    err = sec + "." + key + " must be a string";
    return false;
  }
  out = v->s;
  return true;
}

static std::string resolve(const std::string &base, const std::string &p) {
  if (p.empty() || p[0] == '/' || base.empty()) return p;
  return base + "/" + p;
}

bool load_run_config(const std::string &path, const std::string &base_dir, RunConfig &rc, std::string &err) {
  Config c;
  if (!c.parse_file(path, err)) return false;
  long long t = 0;
  // [xcodec] kmcodec.cc:22-25
  if (!c.get_bool("xcodec", "5gldpc", rc.is5g, err)) return false;
  if (!c.get_bool("xcodec", "metric_type", rc.metric_soft, err)) return false;
  if (!c.get_int("xcodec", "metric_iter", t, err)) return false;
  rc.metric_iter = (int)t;
  // [ldpc] binaryldpccodec.cc:70-73
  if (!c.get_int("ldpc", "max_iter", t, err)) return false;
  rc.max_iter = (int)t;
  if (!c.get_bool("ldpc", "active", rc.active, err)) return false;
  if (!c.get_string("ldpc", "matrix_file", rc.matrix_file, err)) return false;
  // [modem] modem.cc:6-7
  if (!c.get_string("modem", "modem_file", rc.modem_file, err)) return false;
  rc.matrix_file = resolve(base_dir, rc.matrix_file);
  rc.modem_file = resolve(base_dir, rc.modem_file);
  std::string e2;
  // [range] simulator.cc:7-13 (optional for codec-only contexts)
  if (c.has("range", "minimum_snr")) {
    if (!c.get_float("range", "minimum_snr", rc.min_snr, err)) return false;
    if (!c.get_float("range", "maximum_snr", rc.max_snr, err)) return false;
    if (!c.get_float("range", "step_snr", rc.step_snr, err)) return false;
    if (!c.get_int("range", "maximum_error_number", rc.max_err_blk, err)) return false;
    if (!c.get_int("range", "maximum_block_number", rc.max_num_blk, err)) return false;
    if (!c.get_int("range", "thread_block_number", rc.thread_num_blk, err)) return false;
  }
  if (c.has("decoder", "true_h_arg") && !c.get_bool("decoder", "true_h_arg", rc.known_h, err)) return false;
  if (c.has("histogram", "enable") && !c.get_bool("histogram", "enable", rc.histogram, err)) return false;
  return true;
}

}  // namespace kml
