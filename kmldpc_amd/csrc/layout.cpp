// layout.cpp — see layout.hpp.
#include "layout.hpp"

#include <algorithm>
#include <cmath>
#include <memory>
#include <mutex>

namespace kml {

namespace {

struct Xorshift {
  uint64_t s;
  uint64_t next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  }
  double uniform() { return (double)(next() >> 11) * 0x1p-53; }
};

}  // namespace

static void plan_uncached(const LdpcCode &L, RegularLayout &out);

// The plan is a pure function of the graph; contexts on the same code (tests,
// one context per rank) reuse it instead of re-running the annealing (~1 s).
void plan_regular_layout(const LdpcCode &L, int T, RegularLayout &out) {
  struct Entry {
    std::vector<int32_t> row_col, col_slot, cn_order;
    int T;
    RegularLayout plan;
  };
  static std::mutex mu;
  static std::vector<std::unique_ptr<Entry>> cache;
  std::lock_guard<std::mutex> g(mu);
  for (auto &e : cache)
    if (e->T == T && e->row_col == L.row_col && e->col_slot == L.col_slot && e->cn_order == L.cn_order) {
      out = e->plan;
      return;
    }
  auto e = std::make_unique<Entry>();
  e->row_col = L.row_col;
  e->col_slot = L.col_slot;
  e->cn_order = L.cn_order;
  e->T = T;
  plan_uncached(L, e->plan);
  out = e->plan;
  if (cache.size() >= 8) cache.erase(cache.begin());
  cache.push_back(std::move(e));
}

// Positions are grouped by wave (64 consecutive positions) whatever T is.
static void plan_uncached(const LdpcCode &L, RegularLayout &out) {
  const int N = L.N, dv = L.dv_max;
  // CN position of each row -> half bit h(row) = (position >> 2) & 1
  std::vector<int> row_pos(L.M);
  for (int i = 0; i < L.M; i++) row_pos[L.cn_order[i]] = i;
  std::vector<int> slot_h(L.E);
  for (int i = 0; i < L.M; i++)
    for (int e = L.row_ptr[i]; e < L.row_ptr[i + 1]; e++) slot_h[e] = (row_pos[i] >> 2) & 1;
  out.c2v_addr.resize(L.E);
  for (int e = 0; e < L.E; e++) out.c2v_addr[e] = L.col_slot[e] * 16 + 8 * slot_h[L.col_slot[e]];

  // bank bins per (column, k): ds_write_b128 of the slot (8-lane groups, 8 bins
  // of 16 B mod 128 B) and ds_read_b64 of the c2v half (32-lane halves, 32 bins
  // of 8 B mod 256 B)
  std::vector<uint8_t> wb((size_t)N * dv), rb((size_t)N * dv);
  for (int j = 0; j < N; j++)
    for (int k = 0; k < dv; k++) {
      const int e = L.col_ptr[j] + std::min(k, L.col_ptr[j + 1] - L.col_ptr[j] - 1);
      const int a = out.c2v_addr[e];
      wb[(size_t)j * dv + k] = (uint8_t)((L.col_slot[e]) & 7);
      rb[(size_t)j * dv + k] = (uint8_t)((a >> 3) & 31);
    }

  std::vector<int32_t> &ord = out.order;
  ord.assign(L.vn_order.begin(), L.vn_order.end());
  const int nW = (N + 7) / 8, nR = (N + 31) / 32;
  std::vector<uint16_t> wc((size_t)nW * dv * 8, 0), rc((size_t)nR * dv * 32, 0);
  std::vector<int> wmax((size_t)nW * dv, 0), rmax((size_t)nR * dv, 0);
  auto wcnt = [&](int g, int k) { return &wc[((size_t)g * dv + k) * 8]; };
  auto rcnt = [&](int g, int k) { return &rc[((size_t)g * dv + k) * 32]; };
  auto gmax = [](const uint16_t *c, int n) {
    int m = 0;
    for (int i = 0; i < n; i++) m = std::max(m, (int)c[i]);
    return m;
  };
  for (int p = 0; p < N; p++)
    for (int k = 0; k < dv; k++) {
      wcnt(p / 8, k)[wb[(size_t)ord[p] * dv + k]]++;
      rcnt(p / 32, k)[rb[(size_t)ord[p] * dv + k]]++;
    }
  long long cost = 0;
  for (int g = 0; g < nW; g++)
    for (int k = 0; k < dv; k++) cost += (wmax[(size_t)g * dv + k] = gmax(wcnt(g, k), 8)) - 1;
  for (int g = 0; g < nR; g++)
    for (int k = 0; k < dv; k++) cost += (rmax[(size_t)g * dv + k] = gmax(rcnt(g, k), 32)) - 1;
  out.cost_initial = cost;

  // swaps only between columns of equal degree (the kernel assigns columns to
  // positions in degree order; the regular kernel has one degree)
  Xorshift rng{0x9E3779B97F4A7C15ull};
  const long long iters = 1000LL * N * dv;
  double temp = 1.0;
  const double cool = std::pow(0.05, 1.0 / (double)iters);
  auto move = [&](int p, int col, int sign) {
    for (int k = 0; k < dv; k++) {
      wcnt(p / 8, k)[wb[(size_t)col * dv + k]] += sign;
      rcnt(p / 32, k)[rb[(size_t)col * dv + k]] += sign;
    }
  };
  auto group_delta = [&](int a, int b, bool commit) {
    long long d = 0;
    for (int k = 0; k < dv; k++) {
      const int ga = a / 8, gb = b / 8;
      int m = gmax(wcnt(ga, k), 8);
      d += m - wmax[(size_t)ga * dv + k];
      if (commit) wmax[(size_t)ga * dv + k] = m;
      if (gb != ga) {
        m = gmax(wcnt(gb, k), 8);
        d += m - wmax[(size_t)gb * dv + k];
        if (commit) wmax[(size_t)gb * dv + k] = m;
      }
      const int ra = a / 32, rb2 = b / 32;
      m = gmax(rcnt(ra, k), 32);
      d += m - rmax[(size_t)ra * dv + k];
      if (commit) rmax[(size_t)ra * dv + k] = m;
      if (rb2 != ra) {
        m = gmax(rcnt(rb2, k), 32);
        d += m - rmax[(size_t)rb2 * dv + k];
        if (commit) rmax[(size_t)rb2 * dv + k] = m;
      }
    }
    return d;
  };
  for (long long it = 0; it < iters; it++, temp *= cool) {
    const int a = (int)(rng.next() % (uint64_t)N), b = (int)(rng.next() % (uint64_t)N);
    if (a / 8 == b / 8) continue;
    const int ca = ord[a], cb = ord[b];
    if (L.col_ptr[ca + 1] - L.col_ptr[ca] != L.col_ptr[cb + 1] - L.col_ptr[cb]) continue;
    move(a, ca, -1);
    move(b, cb, -1);
    move(a, cb, +1);
    move(b, ca, +1);
    const long long d = group_delta(a, b, false);
    if (d <= 0 || rng.uniform() < std::exp(-(double)d / temp)) {
      group_delta(a, b, true);
      std::swap(ord[a], ord[b]);
      cost += d;
    } else {
      move(a, cb, -1);
      move(b, ca, -1);
      move(a, ca, +1);
      move(b, cb, +1);
    }
  }
  out.cost_final = cost;
  out.pos.assign(N, 0);
  for (int p = 0; p < N; p++) out.pos[ord[p]] = p;
}

}  // namespace kml
