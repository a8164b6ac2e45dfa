#include "code.hpp"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>

namespace kml {

namespace {

// Whitespace tokenizer with fscanf("%s"/"%d") semantics.
struct Tokens {
  std::string buf;
  size_t pos = 0;
  bool next(std::string &tok) {
    while (pos < buf.size() && isspace((unsigned char)buf[pos])) pos++;
    if (pos >= buf.size()) return false;
    size_t b = pos;
    while (pos < buf.size() && !isspace((unsigned char)buf[pos])) pos++;
    tok.assign(buf, b, pos - b);
    return true;
  }
  bool next_int(long &v) {
    std::string t;
    if (!next(t)) return false;
    char *end = nullptr;
    v = strtol(t.c_str(), &end, 10);
    return end && *end == '\0';
  }
};

// Dense GF(2) matrix, rows bit-packed little-endian in 64-bit words.
struct BitMat {
  int rows = 0, cols = 0, W = 0;
  std::vector<uint64_t> w;
  void init(int r, int c) {
    rows = r;
    cols = c;
    W = (c + 63) >> 6;
    w.assign((size_t)r * W, 0);
  }
  uint64_t *row(int i) { return w.data() + (size_t)i * W; }
  const uint64_t *row(int i) const { return w.data() + (size_t)i * W; }
  bool get(int i, int j) const { return (row(i)[j >> 6] >> (j & 63)) & 1u; }
  void set(int i, int j) { row(i)[j >> 6] |= 1ull << (j & 63); }
  void swap_rows(int a, int b) {
    if (a != b) std::swap_ranges(row(a), row(a) + W, row(b));
  }
  void swap_cols(int a, int b) {
    const uint64_t ma = 1ull << (a & 63), mb = 1ull << (b & 63);
    const int wa = a >> 6, wb = b >> 6;
    for (int i = 0; i < rows; i++) {
      uint64_t *r = row(i);
      const bool x = (r[wa] & ma) != 0, y = (r[wb] & mb) != 0;
      if (x != y) {
        r[wa] ^= ma;
        r[wb] ^= mb;
      }
    }
  }
  // row m ^= row i over word range [w0, w1)
  void xor_into(int m, int i, int w0, int w1) {
    uint64_t *d = row(m);
    const uint64_t *s = row(i);
    for (int k = w0; k < w1; k++) d[k] ^= s[k];
  }
};

// SystemMatrixH, PEG flavour (binaryldpccodec.cc:386-431).
int eliminate_forward(BitMat &A, std::vector<int32_t> &perm) {
  const int M = A.rows, N = A.cols;
  int chk = 0;
  for (int i = 0; i < M; i++) {
    int pr = -1, pc = -1;
    for (int jj = i; jj < N && pr < 0; jj++)
      for (int ii = i; ii < M; ii++)
        if (A.get(ii, jj)) {
          pr = ii;
          pc = jj;
          break;
        }
    if (pr < 0) break;
    chk++;
    A.swap_rows(i, pr);
    if (pc != i) {
      std::swap(perm[i], perm[pc]);
      A.swap_cols(i, pc);
    }
    // row i is zero left of column i (those columns are already reduced)
    const int w0 = i >> 6;
    for (int m = 0; m < M; m++)
      if (m != i && A.get(m, i)) A.xor_into(m, i, w0, A.W);
  }
  return chk;
}

// SystemMatrixH, 5G flavour (binary5gldpccodec.cc:281-325): pivots placed at
// column i + N - M, searched right-to-left / bottom-to-top.
int eliminate_backward(BitMat &A, std::vector<int32_t> &perm) {
  const int M = A.rows, N = A.cols;
  int chk = 0;
  for (int i = M - 1; i >= 0; --i) {
    const int c = i + N - M;
    int pr = -1, pc = -1;
    for (int jj = c; jj >= 0 && pr < 0; --jj)
      for (int ii = i; ii >= 0; --ii)
        if (A.get(ii, jj)) {
          pr = ii;
          pc = jj;
          break;
        }
    if (pr < 0) break;
    chk++;
    A.swap_rows(i, pr);
    if (pc != c) {
      std::swap(perm[c], perm[pc]);
      A.swap_cols(c, pc);
    }
    // row i is zero right of column c
    const int w1 = (c >> 6) + 1;
    for (int m = M - 1; m >= 0; --m)
      if (m != i && A.get(m, c)) A.xor_into(m, i, 0, w1);
  }
  return chk;
}

}  // namespace

bool LdpcCode::load(const std::string &path, bool is5g_, bool active_, bool reversed_rows, std::string &err) {
  std::ifstream f(path, std::ios::binary);
  if (!f.is_open()) {
    err = "Cannot open " + path;  // binaryldpccodec.cc:77-80 logs and exit(-1)s
    return false;
  }
  Tokens tk;
  {
    std::stringstream ss;
    ss << f.rdbuf();
    tk.buf = ss.str();
  }
  is5g = is5g_;
  active = active_;
  std::string tok;
  long m = 0, n = 0, rank = 0, z = 0;
  if (!tk.next(tok) || !tk.next_int(m) || !tk.next_int(n) || !tk.next_int(rank) || (is5g && !tk.next_int(z)) ||
      !tk.next(tok) || m <= 0 || n <= 0) {
    err = "bad H-matrix header in " + path;
    return false;
  }
  M = (int)m;
  N = (int)n;
  Z = is5g ? (int)z : 0;
  std::vector<std::vector<int32_t>> file_rows(M);
  for (int i = 0; i < M; i++) {
    long rno = 0, deg = 0;
    if (!tk.next_int(rno) || !tk.next_int(deg) || deg < 0) {
      err = "bad row " + std::to_string(i) + " in " + path;
      return false;
    }
    for (long j = 0; j < deg; j++) {
      long c = 0;
      if (!tk.next_int(c) || c < 0 || c >= N) {
        err = "bad column index in row " + std::to_string(i) + " of " + path;
        return false;
      }
      file_rows[i].push_back((int32_t)c);
    }
  }

  perm.resize(N);
  for (int j = 0; j < N; j++) perm[j] = j;
  row_ptr.assign(M + 1, 0);
  row_col.clear();
  BitMat H;
  H.init(M, N);
  for (int i = 0; i < M; i++)
    for (int c : file_rows[i]) H.set(i, c);

  if (active) {
    BitMat A = H;
    chk = is5g ? eliminate_backward(A, perm) : eliminate_forward(A, perm);
    // graph of H[:, perm], rows listed by descending new column
    std::vector<int32_t> inv(N);
    for (int j = 0; j < N; j++) inv[perm[j]] = j;
    for (int i = 0; i < M; i++) {
      std::vector<int32_t> cols;
      const uint64_t *r = H.row(i);
      for (int w = 0; w < H.W; w++)
        for (uint64_t x = r[w]; x; x &= x - 1) cols.push_back(inv[(w << 6) + __builtin_ctzll(x)]);
      std::sort(cols.begin(), cols.end(), std::greater<int32_t>());
      row_col.insert(row_col.end(), cols.begin(), cols.end());
      row_ptr[i + 1] = (int32_t)row_col.size();
    }
    K = N - chk;
    Kw = (K + 63) >> 6;
    enc_info.assign((size_t)chk * Kw, 0);
    const int c0 = is5g ? 0 : chk;  // first info column
    for (int t = 0; t < chk; t++)
      for (int j = 0; j < K; j++)
        if (A.get(t, c0 + j)) enc_info[(size_t)t * Kw + (j >> 6)] |= 1ull << (j & 63);
  } else {
    chk = (int)rank;  // code_chk_ straight from the file header
    for (int i = 0; i < M; i++) {
      for (auto it = file_rows[i].rbegin(); it != file_rows[i].rend(); ++it) row_col.push_back(*it);
      row_ptr[i + 1] = (int32_t)row_col.size();
    }
    K = N - chk;
    Kw = (K + 63) >> 6;
    enc_info.clear();
  }
  if (reversed_rows)
    for (int i = 0; i < M; i++) std::reverse(row_col.begin() + row_ptr[i], row_col.begin() + row_ptr[i + 1]);
  E = (int)row_col.size();

  // column lists: descending row index
  col_ptr.assign(N + 1, 0);
  for (int e = 0; e < E; e++) col_ptr[row_col[e] + 1]++;
  for (int j = 0; j < N; j++) col_ptr[j + 1] += col_ptr[j];
  col_slot.assign(E, 0);
  {
    std::vector<int32_t> fill(col_ptr.begin() + 1, col_ptr.end());
    for (int i = 0; i < M; i++)
      for (int e = row_ptr[i]; e < row_ptr[i + 1]; e++) col_slot[--fill[row_col[e]]] = e;
  }
  dv_max = dc_max = 0;
  for (int j = 0; j < N; j++) dv_max = std::max(dv_max, col_ptr[j + 1] - col_ptr[j]);
  for (int i = 0; i < M; i++) dc_max = std::max(dc_max, row_ptr[i + 1] - row_ptr[i]);
  vn_order.resize(N);
  cn_order.resize(M);
  for (int j = 0; j < N; j++) vn_order[j] = j;
  for (int i = 0; i < M; i++) cn_order[i] = i;
  std::stable_sort(vn_order.begin(), vn_order.end(), [&](int a, int b) {
    return (col_ptr[a + 1] - col_ptr[a]) > (col_ptr[b + 1] - col_ptr[b]);
  });
  std::stable_sort(cn_order.begin(), cn_order.end(), [&](int a, int b) {
    return (row_ptr[a + 1] - row_ptr[a]) > (row_ptr[b + 1] - row_ptr[b]);
  });

  punct = is5g ? 2 * Z : 0;
  cc_len = N - punct;
  info_off = is5g ? 0 : chk;
  return true;
}

void LdpcCode::encode(const uint8_t *uu, uint8_t *cc) const {
  if (!active) {
    memset(cc, 0, cc_len);
    return;
  }
  std::vector<uint64_t> u(Kw, 0);
  for (int j = 0; j < K; j++)
    if (uu[j] & 1) u[j >> 6] |= 1ull << (j & 63);
  std::vector<uint8_t> par(chk);
  for (int t = 0; t < chk; t++) {
    uint64_t acc = 0;
    for (int w = 0; w < Kw; w++) acc ^= enc_info[(size_t)t * Kw + w] & u[w];
    par[t] = (uint8_t)(__builtin_popcountll(acc) & 1);
  }
  if (!is5g) {
    for (int t = 0; t < chk; t++) cc[t] = par[t];
    for (int j = 0; j < K; j++) cc[chk + j] = uu[j] & 1;
  } else {
    for (int i = 0; i < cc_len; i++) {
      const int f = i + punct;
      cc[i] = f < K ? (uu[f] & 1) : par[f - K];
    }
  }
}

}  // namespace kml
