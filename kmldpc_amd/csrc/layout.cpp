// layout.cpp — see layout.hpp.
#include "layout.hpp"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <thread>

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
  // Physical slot of the j-th edge of a row (row_ptr order): rows are stored in
  // CN position order, and within a row the edges the even lane reads
  // (j < dc/2, ascending) and the odd lane reads (j >= dc/2, descending)
  // alternate, so at step st the pair reads slots 2st and 2st+1 of its row
  // (slots 2(dc-1-st)+1 and 2(dc-1-st) once st >= dc/2): per-lane base registers
  // plus immediate offsets, and conflict-free ds_read_b128 / ds_write_b64 groups
  // (consecutive positions).
  const int dc = L.dc_max;
  std::vector<int> slot_h(L.E), phys(L.E);
  for (int i = 0; i < L.M; i++)
    for (int e = L.row_ptr[i]; e < L.row_ptr[i + 1]; e++) {
      const int j = e - L.row_ptr[i];
      slot_h[e] = (row_pos[i] >> 2) & 1;
      phys[e] = row_pos[i] * dc + (j < dc / 2 ? 2 * j : 2 * (dc - 1 - j) + 1);
    }
  out.c2v_addr.resize(L.E);
  for (int e = 0; e < L.E; e++) out.c2v_addr[e] = phys[L.col_slot[e]] * 16 + 8 * slot_h[L.col_slot[e]];

  // bank bins per (column, k): ds_write_b128 of the slot (8-lane groups, 8 bins
  // of 16 B mod 128 B) and ds_read_b64 of the c2v half (32-lane halves, 32 bins
  // of 8 B mod 256 B)
  std::vector<uint8_t> wb((size_t)N * dv), rb((size_t)N * dv);
  for (int j = 0; j < N; j++)
    for (int k = 0; k < dv; k++) {
      const int e = L.col_ptr[j] + std::min(k, L.col_ptr[j + 1] - L.col_ptr[j] - 1);
      const int a = out.c2v_addr[e];
      wb[(size_t)j * dv + k] = (uint8_t)((a >> 4) & 7);
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

namespace kml {

namespace {

// Capacity-bounded majority assignment: every item goes to the part holding
// most of its neighbours, strongest preferences first, each part taking at
// most `cap` items (ties broken by a seeded random key).
void assign_majority(const std::vector<int32_t> &ptr, const std::vector<int32_t> &nbr,
                     const std::vector<int32_t> &nbr_part, int G, int cap, Xorshift &rng,
                     std::vector<int32_t> &part) {
  const int n = (int)ptr.size() - 1;
  struct Cand {
    int cnt;
    uint32_t key;
    int item, g;
  };
  std::vector<Cand> cand;
  cand.reserve((size_t)n * G);
  std::vector<int> cnt(G);
  for (int i = 0; i < n; i++) {
    std::fill(cnt.begin(), cnt.end(), 0);
    for (int e = ptr[i]; e < ptr[i + 1]; e++) cnt[nbr_part[nbr[e]]]++;
    for (int g = 0; g < G; g++) cand.push_back({cnt[g], (uint32_t)rng.next(), i, g});
  }
  std::sort(cand.begin(), cand.end(), [](const Cand &a, const Cand &b) {
    return a.cnt != b.cnt ? a.cnt > b.cnt : a.key < b.key;
  });
  part.assign(n, -1);
  std::vector<int> load(G, 0);
  for (const Cand &c : cand)
    if (part[c.item] < 0 && load[c.g] < cap) {
      part[c.item] = c.g;
      load[c.g]++;
    }
}

// The VN phase's LDS bank model (bp_regular's, above): position p's column
// stores its k-th v2c slot with ds_write_b128 (8-lane groups: 8 bins of 16 B
// mod 128 B, bin wb) and reads its k-th c2v with ds_read_b64 (32-lane halves:
// 32 bins of 8 B mod 256 B, bin rb).  Anneals the column order ord[lo, hi)
// (all columns of one degree) against the summed excess group maxima.
// Returns (initial cost, final cost).
std::pair<long long, long long> anneal_vn_order(std::vector<int32_t> &ord, int lo, int hi, int dv,
                                                const std::vector<uint8_t> &wb, const std::vector<uint8_t> &rb,
                                                uint64_t seed, long long iters) {
  const int n = hi - lo;
  const int nW = (n + 7) / 8, nR = (n + 31) / 32;
  std::vector<uint16_t> wc((size_t)nW * dv * 8, 0), rc((size_t)nR * dv * 32, 0);
  std::vector<int> wmax((size_t)nW * dv, 0), rmax((size_t)nR * dv, 0);
  auto wcnt = [&](int g, int k) { return &wc[((size_t)g * dv + k) * 8]; };
  auto rcnt = [&](int g, int k) { return &rc[((size_t)g * dv + k) * 32]; };
  auto gmax = [](const uint16_t *c, int m) {
    int x = 0;
    for (int i = 0; i < m; i++) x = std::max(x, (int)c[i]);
    return x;
  };
  for (int p = 0; p < n; p++)
    for (int k = 0; k < dv; k++) {
      wcnt(p / 8, k)[wb[(size_t)ord[lo + p] * dv + k]]++;
      rcnt(p / 32, k)[rb[(size_t)ord[lo + p] * dv + k]]++;
    }
  long long cost = 0;
  for (int g = 0; g < nW; g++)
    for (int k = 0; k < dv; k++) cost += (wmax[(size_t)g * dv + k] = gmax(wcnt(g, k), 8)) - 1;
  for (int g = 0; g < nR; g++)
    for (int k = 0; k < dv; k++) cost += (rmax[(size_t)g * dv + k] = gmax(rcnt(g, k), 32)) - 1;
  const long long c0 = cost;
  Xorshift rng{seed};
  double temp = 1.0;
  const double cool = std::pow(0.05, 1.0 / (double)std::max(iters, 1LL));
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
    const int a = (int)(rng.next() % (uint64_t)n), b = (int)(rng.next() % (uint64_t)n);
    if (a / 8 == b / 8) continue;
    const int ca = ord[lo + a], cb = ord[lo + b];
    move(a, ca, -1);
    move(b, cb, -1);
    move(a, cb, +1);
    move(b, ca, +1);
    const long long d = group_delta(a, b, false);
    if (d <= 0 || rng.uniform() < std::exp(-(double)d / temp)) {
      group_delta(a, b, true);
      std::swap(ord[lo + a], ord[lo + b]);
      cost += d;
    } else {
      move(a, cb, -1);
      move(b, ca, -1);
      move(a, ca, +1);
      move(b, cb, +1);
    }
  }
  return {c0, cost};
}

}  // namespace

// Cut refinement of the balanced G-way partition (rows and columns of the
// Tanner graph; a cut edge is one whose row and column sit in different
// members, i.e. one mailbox entry of bp_part_kernel).  The BFS seeding and
// majority relabelling below reach a local optimum of "relabel one side given
// the other"; this escapes it by simulated annealing over single-node moves (a
// row or column to a member one of its neighbours is in), with member sizes
// kept within +-kSlack of MG / NG, then a repair to exact balance (the
// cheapest moves) and a greedy same-type swap polish.  kChains chains with
// fixed seeds run in parallel threads and the lowest cut wins (ties: the
// lowest chain), so the plan does not depend on timing or the host.
// PEG8064 at G = 4: 6,602 -> ~5,480 cut edges (27.3 % -> 22.7 % of 24,192).
struct PartRefiner {
  const std::vector<int32_t> &row_ptr, &row_cols, &col_ptr, &col_rows;
  int G, MG, NG;
  long long run(std::vector<int32_t> &R, std::vector<int32_t> &C, long long iters, uint64_t seed) const {
    constexpr int kSlack = 16;
    const int M = (int)row_ptr.size() - 1, N = (int)col_ptr.size() - 1;
    std::vector<int> rcnt((size_t)M * G, 0), ccnt((size_t)N * G, 0), rload(G, 0), cload(G, 0);
    long long cut = 0;
    for (int i = 0; i < M; i++) {
      rload[R[i]]++;
      for (int e = row_ptr[i]; e < row_ptr[i + 1]; e++) rcnt[(size_t)i * G + C[row_cols[e]]]++;
    }
    for (int j = 0; j < N; j++) {
      cload[C[j]]++;
      for (int e = col_ptr[j]; e < col_ptr[j + 1]; e++) {
        ccnt[(size_t)j * G + R[col_rows[e]]]++;
        cut += R[col_rows[e]] != C[j];
      }
    }
    auto mv_row = [&](int x, int a, int b) {
      for (int e = row_ptr[x]; e < row_ptr[x + 1]; e++) {
        const int j = row_cols[e];
        ccnt[(size_t)j * G + a]--;
        ccnt[(size_t)j * G + b]++;
      }
      R[x] = b;
      rload[a]--;
      rload[b]++;
    };
    auto mv_col = [&](int x, int a, int b) {
      for (int e = col_ptr[x]; e < col_ptr[x + 1]; e++) {
        const int i = col_rows[e];
        rcnt[(size_t)i * G + a]--;
        rcnt[(size_t)i * G + b]++;
      }
      C[x] = b;
      cload[a]--;
      cload[b]++;
    };
    Xorshift rng{seed};
    const double lT0 = std::log(1.0), lT1 = std::log(0.15);
    double acc[64];
    for (long long t = 0; t < iters; t++) {
      if ((t & 1023) == 0) {
        const double T = std::exp(lT0 + (lT1 - lT0) * (double)t / (double)iters);
        for (int d = 0; d < 64; d++) acc[d] = std::exp(-d / T);
      }
      const uint64_t r = rng.next();
      if (r & 1) {
        const int x = (int)((r >> 1) % (uint64_t)M), a = R[x];
        const int b = C[row_cols[row_ptr[x] + (int)((r >> 33) % (uint64_t)(row_ptr[x + 1] - row_ptr[x]))]];
        if (b == a || rload[b] >= MG + kSlack || rload[a] <= MG - kSlack) continue;
        const int d = rcnt[(size_t)x * G + a] - rcnt[(size_t)x * G + b];
        if (d <= 0 || rng.uniform() < acc[std::min(d, 63)]) {
          mv_row(x, a, b);
          cut += d;
        }
      } else {
        const int x = (int)((r >> 1) % (uint64_t)N), a = C[x];
        const int b = R[col_rows[col_ptr[x] + (int)((r >> 33) % (uint64_t)(col_ptr[x + 1] - col_ptr[x]))]];
        if (b == a || cload[b] >= NG + kSlack || cload[a] <= NG - kSlack) continue;
        const int d = ccnt[(size_t)x * G + a] - ccnt[(size_t)x * G + b];
        if (d <= 0 || rng.uniform() < acc[std::min(d, 63)]) {
          mv_col(x, a, b);
          cut += d;
        }
      }
    }
    // exact balance: the cheapest move from an overfull member to an underfull one
    for (int side = 0; side < 2; side++) {
      std::vector<int> &load = side ? cload : rload;
      const int cap = side ? NG : MG, n = side ? N : M;
      for (;;) {
        int over = -1, under = -1;
        for (int g = 0; g < G; g++) {
          if (load[g] > cap) over = g;
          if (load[g] < cap) under = g;
        }
        if (over < 0) break;
        int bx = -1, bd = 1 << 30;
        for (int x = 0; x < n; x++) {
          if ((side ? C[x] : R[x]) != over) continue;
          const int d = side ? ccnt[(size_t)x * G + over] - ccnt[(size_t)x * G + under]
                             : rcnt[(size_t)x * G + over] - rcnt[(size_t)x * G + under];
          if (d < bd) {
            bd = d;
            bx = x;
          }
        }
        if (side)
          mv_col(bx, over, under);
        else
          mv_row(bx, over, under);
        cut += bd;
      }
    }
    // greedy polish: improving swaps of two rows (or two columns) of different
    // members; rows are not adjacent to rows, so the two moves' gains add
    for (int pass = 0; pass < 4; pass++) {
      const long long before = cut;
      for (long long t = 0; t < 4 * (long long)(M + N) * G; t++) {
        const uint64_t r = rng.next();
        if (r & 1) {
          const int x = (int)((r >> 1) % (uint64_t)M), y = (int)((r >> 32) % (uint64_t)M), a = R[x], b = R[y];
          if (a == b) continue;
          const int d = rcnt[(size_t)x * G + a] - rcnt[(size_t)x * G + b] + rcnt[(size_t)y * G + b] - rcnt[(size_t)y * G + a];
          if (d < 0) {
            mv_row(x, a, b);
            mv_row(y, b, a);
            cut += d;
          }
        } else {
          const int x = (int)((r >> 1) % (uint64_t)N), y = (int)((r >> 32) % (uint64_t)N), a = C[x], b = C[y];
          if (a == b) continue;
          const int d = ccnt[(size_t)x * G + a] - ccnt[(size_t)x * G + b] + ccnt[(size_t)y * G + b] - ccnt[(size_t)y * G + a];
          if (d < 0) {
            mv_col(x, a, b);
            mv_col(y, b, a);
            cut += d;
          }
        }
      }
      if (cut == before) break;
    }
    return cut;
  }
};

#ifndef KML_PART_ANNEAL  // (A/B) 0: members' columns in index order
#define KML_PART_ANNEAL 1
#endif

static bool plan_partition_uncached(const LdpcCode &L, int G, PartitionPlan &out);

// Cached like plan_regular_layout: a pure function of the graph, and the
// annealing takes ~1 s.
bool plan_partition(const LdpcCode &L, int G, PartitionPlan &out) {
  struct Entry {
    std::vector<int32_t> row_col, col_slot;
    int G;
    bool ok;
    PartitionPlan plan;
  };
  static std::mutex mu;
  static std::vector<std::unique_ptr<Entry>> cache;
  std::lock_guard<std::mutex> g(mu);
  for (auto &e : cache)
    if (e->G == G && e->row_col == L.row_col && e->col_slot == L.col_slot) {
      out = e->plan;
      return e->ok;
    }
  auto e = std::make_unique<Entry>();
  e->row_col = L.row_col;
  e->col_slot = L.col_slot;
  e->G = G;
  e->ok = plan_partition_uncached(L, G, e->plan);
  out = e->plan;
  const bool ok = e->ok;
  if (cache.size() >= 4) cache.erase(cache.begin());
  cache.push_back(std::move(e));
  return ok;
}

static bool plan_partition_uncached(const LdpcCode &L, int G, PartitionPlan &out) {
  const int M = L.M, N = L.N, E = L.E;
  if (G <= 0 || M % G || N % G || !L.dv_max || !L.dc_max) return false;
  for (int j = 0; j < N; j++)
    if (L.col_ptr[j + 1] - L.col_ptr[j] != L.dv_max) return false;
  for (int i = 0; i < M; i++)
    if (L.row_ptr[i + 1] - L.row_ptr[i] != L.dc_max) return false;
  const int MG = M / G, NG = N / G, dc = L.dc_max, dv = L.dv_max;
  // slot -> row
  std::vector<int32_t> slot_row(E);
  for (int i = 0; i < M; i++)
    for (int e = L.row_ptr[i]; e < L.row_ptr[i + 1]; e++) slot_row[e] = i;
  // column adjacency (rows) and row adjacency (columns)
  std::vector<int32_t> col_rows(E), row_cols(L.row_col.begin(), L.row_col.end());
  for (int e = 0; e < E; e++) col_rows[e] = slot_row[L.col_slot[e]];

  // initial row parts: breadth-first order over the Tanner graph, cut in G runs
  std::vector<int32_t> rpart(M, -1), cpart;
  {
    std::vector<int32_t> order;
    order.reserve(M);
    std::vector<char> seen_r(M, 0), seen_c(N, 0);
    for (int s = 0; s < M; s++) {
      if (seen_r[s]) continue;
      size_t head = order.size();
      order.push_back(s);
      seen_r[s] = 1;
      while (head < order.size()) {
        const int r = order[head++];
        for (int e = L.row_ptr[r]; e < L.row_ptr[r + 1]; e++) {
          const int c = row_cols[e];
          if (seen_c[c]) continue;
          seen_c[c] = 1;
          for (int f = L.col_ptr[c]; f < L.col_ptr[c + 1]; f++) {
            const int r2 = col_rows[f];
            if (!seen_r[r2]) {
              seen_r[r2] = 1;
              order.push_back(r2);
            }
          }
        }
      }
    }
    for (int k = 0; k < M; k++) rpart[order[k]] = (int32_t)((long long)k * G / M);
  }
  auto cut_of = [&](const std::vector<int32_t> &rp, const std::vector<int32_t> &cp) {
    long long n = 0;
    for (int j = 0; j < N; j++)
      for (int e = L.col_ptr[j]; e < L.col_ptr[j + 1]; e++) n += rp[col_rows[e]] != cp[j];
    return n;
  };
  Xorshift rng{0xC2B2AE3D27D4EB4Full};
  long long best = -1;
  std::vector<int32_t> best_r, best_c;
  for (int it = 0; it < 40; it++) {
    assign_majority(L.col_ptr, col_rows, rpart, G, NG, rng, cpart);
    const long long cc = cut_of(rpart, cpart);
    if (best < 0 || cc < best) {
      best = cc;
      best_r = rpart;
      best_c = cpart;
    }
    assign_majority(L.row_ptr, row_cols, cpart, G, MG, rng, rpart);
  }
  // refinement (PartRefiner above); KML_PART_REFINE=0 keeps the relabelling's
  // plan (A/B), KML_PART_REFINE_ITERS sets the annealing steps per chain
  const char *ref_env = getenv("KML_PART_REFINE");
  if (!(ref_env && ref_env[0] == '0')) {
    constexpr int kChains = 4;
    long long iters = 150000000LL;
    if (const char *e = getenv("KML_PART_REFINE_ITERS")) iters = std::max(0LL, atoll(e));
    const PartRefiner pr{L.row_ptr, row_cols, L.col_ptr, col_rows, G, MG, NG};
    std::vector<std::vector<int32_t>> rs(kChains, best_r), cs(kChains, best_c);
    std::vector<long long> cut(kChains, -1);
    std::vector<std::thread> th;
    for (int k = 0; k < kChains; k++)
      th.emplace_back([&, k] { cut[k] = pr.run(rs[k], cs[k], iters, 0x243F6A8885A308D3ull * (uint64_t)(k + 1)); });
    for (auto &t : th) t.join();
    for (int k = 0; k < kChains; k++)
      if (cut[k] < best) {
        best = cut[k];
        best_r = rs[k];
        best_c = cs[k];
      }
  }

  // member orders: rows by index, columns by index (annealed below)
  out.G = G;
  out.MG = MG;
  out.NG = NG;
  out.vn.clear();
  out.cn.clear();
  for (int g = 0; g < G; g++) {
    for (int j = 0; j < N; j++)
      if (best_c[j] == g) out.vn.push_back(j);
    for (int i = 0; i < M; i++)
      if (best_r[i] == g) out.cn.push_back(i);
  }
  std::vector<int32_t> row_at(M);
  for (int p = 0; p < M; p++) row_at[out.cn[p]] = p;
  const int EG = MG * dc;

  // cut edges, sorted by (row owner, partitioned row slot)
  struct Cut {
    int R, S, slot, col, k;
  };
  std::vector<Cut> cuts;
  for (int p = 0; p < N; p++) {
    const int j = out.vn[p];
    for (int e = L.col_ptr[j], k = 0; e < L.col_ptr[j + 1]; e++, k++) {
      const int s = L.col_slot[e], r = slot_row[s];
      if (best_r[r] != best_c[j]) cuts.push_back({best_r[r], best_c[j], row_at[r] * dc + (s - L.row_ptr[r]), j, k});
    }
  }
  std::sort(cuts.begin(), cuts.end(), [](const Cut &a, const Cut &b) {
    return a.R != b.R ? a.R < b.R : a.slot < b.slot;
  });
  out.ncut = (int)cuts.size();
  {
    std::vector<char> pair((size_t)G * G, 0);
    for (const Cut &c : cuts) pair[(size_t)c.R * G + c.S] = 1;
    out.all_pairs = true;
    for (int r = 0; r < G; r++)
      for (int q = 0; q < G; q++)
        if (r != q && !pair[(size_t)r * G + q]) out.all_pairs = false;
  }
  if (out.ncut >= (1 << 15)) return false;  // packed (x << 16) entries
  std::vector<std::vector<int32_t>> xr(G), xc(G);
  std::vector<int> mirror_of(cuts.size());
  for (size_t x = 0; x < cuts.size(); x++) {
    const Cut &c = cuts[x];
    xr[c.R].push_back((int32_t)((x << 16) | (uint32_t)(c.slot - c.R * EG)));
    mirror_of[x] = (int)xc[c.S].size();
    xc[c.S].push_back((int32_t)((x << 16) | (uint32_t)(EG + mirror_of[x])));
  }
  out.mirror_max = 0;
  out.xr.clear();
  out.xc.clear();
  out.xr_ptr.assign(1, 0);
  out.xc_ptr.assign(1, 0);
  for (int g = 0; g < G; g++) {
    out.mirror_max = std::max(out.mirror_max, (int)xc[g].size());
    if (EG + (int)xc[g].size() >= (1 << 16)) return false;
    out.xr.insert(out.xr.end(), xr[g].begin(), xr[g].end());
    out.xc.insert(out.xc.end(), xc[g].begin(), xc[g].end());
    out.xr_ptr.push_back((int32_t)out.xr.size());
    out.xc_ptr.push_back((int32_t)out.xc.size());
  }
  // per-edge LDS addresses of the VN phase, per column: own row slot, or the
  // mirror slot
  std::vector<int32_t> caddr((size_t)N * dv, 0), cvx((size_t)N * dv, -1);
  for (int j = 0; j < N; j++) {
    const int g = best_c[j];
    for (int e = L.col_ptr[j], k = 0; e < L.col_ptr[j + 1]; e++, k++) {
      const int s = L.col_slot[e], r = slot_row[s];
      if (best_r[r] == g) caddr[(size_t)j * dv + k] = ((row_at[r] - g * MG) * dc + (s - L.row_ptr[r])) * 16;
    }
  }
  for (size_t x = 0; x < cuts.size(); x++) {
    caddr[(size_t)cuts[x].col * dv + cuts[x].k] = (EG + mirror_of[x]) * 16;
    cvx[(size_t)cuts[x].col * dv + cuts[x].k] = (int32_t)x;
  }
  // the columns' lane positions within each member: annealed against the VN
  // phase's bank conflicts (write bins of the slot, read bins of the c2v half:
  // bp_coop.hip part_c2v_half — bit 2 of the row for row slots, of the slot
  // index for mirror slots)
  // each member's INTERIOR columns (every edge's row its own) last, so the
  // boundary columns, whose v2c the partners wait for, are stored first; the
  // annealing below keeps the two runs apart (a VN phase split around the c2v
  // receive, interior columns first, measured slower: 8.75 vs 8.20 ms per 4096
  // PEG8064 codewords, profiles/r05_ab2_summary.txt)
  std::vector<int> nbound(G, NG);
  const char *il_env = getenv("KML_PART_INTERIOR_LAST");  // (A/B) 0: columns in index order
  for (int g = 0; g < G && !(il_env && il_env[0] == '0'); g++) {
    auto interior = [&](int j) {
      for (int e = L.col_ptr[j]; e < L.col_ptr[j + 1]; e++)
        if (best_r[col_rows[e]] != g) return false;
      return true;
    };
    auto first = out.vn.begin() + (size_t)g * NG, last = first + NG;
    nbound[g] = (int)(std::stable_partition(first, last, [&](int j) { return !interior(j); }) - first);
  }
  out.interior = 0;
  for (int g = 0; g < G; g++) out.interior += NG - nbound[g];
  if (KML_PART_ANNEAL) {
    std::vector<uint8_t> wb((size_t)N * dv), rb((size_t)N * dv);
    for (int j = 0; j < N; j++)
      for (int k = 0; k < dv; k++) {
        const int a = caddr[(size_t)j * dv + k], sl = a >> 4;
        const int half = sl < EG ? ((sl / dc) >> 2) & 1 : (sl >> 2) & 1;
        wb[(size_t)j * dv + k] = (uint8_t)((a >> 4) & 7);
        rb[(size_t)j * dv + k] = (uint8_t)(((a + 8 * half) >> 3) & 31);
      }
    out.anneal_initial = out.anneal_final = 0;
    for (int g = 0; g < G; g++)
      for (int part = 0; part < 2; part++) {
        const int lo = g * NG + (part ? nbound[g] : 0), hi = part ? (g + 1) * NG : g * NG + nbound[g];
        if (hi - lo < 2) continue;
        const auto c = anneal_vn_order(out.vn, lo, hi, dv, wb, rb, 0x9E3779B97F4A7C15ull + (uint64_t)(2 * g + part),
                                       300LL * (hi - lo) * dv);
        out.anneal_initial += c.first;
        out.anneal_final += c.second;
      }
  }
  out.pos.assign(N, 0);
  for (int p = 0; p < N; p++) out.pos[out.vn[p]] = p;
  out.vaddr.assign((size_t)N * dv, 0);
  out.vx.assign((size_t)N * dv, -1);
  for (int p = 0; p < N; p++)
    for (int k = 0; k < dv; k++) {
      out.vaddr[(size_t)p * dv + k] = caddr[(size_t)out.vn[p] * dv + k];
      out.vx[(size_t)p * dv + k] = cvx[(size_t)out.vn[p] * dv + k];
    }
  out.rx.assign(M, 0);
  for (size_t x = 0; x < cuts.size(); x++) {
    const int P = cuts[x].slot / dc, e = cuts[x].slot % dc;  // plan row index, edge position in the row
    if (!(out.rx[P] & 0xFF)) out.rx[P] = (int32_t)(x << 8);
    out.rx[P] |= 1 << e;
  }
  return true;
}

}  // namespace kml

namespace kml {

namespace {

// One wave's worth of items (64 columns, or 32 rows) for one round.
#ifndef KML_IRR_PARTIAL_PAIRS
#define KML_IRR_PARTIAL_PAIRS 1
#endif

struct WaveItems {
  std::vector<int32_t> a, b;  // a: the (first) items; b: the second items of a pair wave
  double cost = 0;
};

// items[d] = the items of degree d.  cost(d) models one item's VALU work.
// Returns false when the items do not fit W pair waves + W single waves.
bool plan_rounds(std::vector<std::vector<int32_t>> items, int per_wave, int W, int pair_max, double (*cost)(int),
                 std::vector<WaveItems> &pairs, std::vector<WaveItems> &singles) {
  const int dmax = (int)items.size() - 1;
  pairs.clear();
  singles.clear();
  // pair waves from the highest degrees (up to pair_max): 2 * per_wave items of one degree
  for (int d = std::min(dmax, pair_max); d >= 0 && (int)pairs.size() < W; --d)
    while ((int)items[d].size() >= 2 * per_wave && (int)pairs.size() < W) {
      WaveItems w;
      w.a.assign(items[d].begin(), items[d].begin() + per_wave);
      w.b.assign(items[d].begin() + per_wave, items[d].begin() + 2 * per_wave);
      items[d].erase(items[d].begin(), items[d].begin() + 2 * per_wave);
      w.cost = 2 * per_wave * cost(d);
      pairs.push_back(std::move(w));
    }
  // leftover pair slots take a partial pair wave of one degree (at least half
  // a wave of pairs, lowest degrees first), so that fewer single waves mix
  // two degrees (a mixed wave runs both degrees' code paths)
  if (KML_IRR_PARTIAL_PAIRS)
    for (int d = 0; d <= std::min(dmax, pair_max) && (int)pairs.size() < W; ++d) {
      const int np = (int)items[d].size() / 2;
      if (np < per_wave / 2 || np >= per_wave) continue;
      WaveItems w;
      w.a.assign(items[d].begin(), items[d].begin() + np);
      w.b.assign(items[d].begin() + np, items[d].begin() + 2 * np);
      items[d].erase(items[d].begin(), items[d].begin() + 2 * np);
      w.cost = 2 * np * cost(d);
      pairs.push_back(std::move(w));
    }
  // the rest as single waves, highest degree first; a partial wave is topped up
  // with the next degree's items (a mixed wave)
  WaveItems cur;
  for (int d = dmax; d >= 0; --d)
    for (int32_t it : items[d]) {
      cur.a.push_back(it);
      cur.cost += cost(d);
      if ((int)cur.a.size() == per_wave) {
        singles.push_back(std::move(cur));
        cur = WaveItems();
      }
    }
  if (!cur.a.empty()) singles.push_back(std::move(cur));
  return (int)singles.size() <= W;
}

// Place pair waves and single waves on lane waves 0..W-1 so that the SIMD
// totals (wave w on SIMD w % 4) are balanced: longest-processing-time first,
// each SIMD taking W/4 pair waves and W/4 single waves.
void place_waves(const std::vector<WaveItems> &pairs, const std::vector<WaveItems> &singles, int W,
                 std::vector<int> &pair_of, std::vector<int> &single_of) {
  const int per = W / 4;
  std::vector<double> load(4, 0.0);
  std::vector<std::vector<int>> simd_waves(4);
  for (int w = 0; w < W; ++w) simd_waves[w % 4].push_back(w);
  pair_of.assign(W, -1);
  single_of.assign(W, -1);
  auto lpt = [&](const std::vector<WaveItems> &v, std::vector<int> &of) {
    std::vector<int> idx(v.size());
    for (size_t i = 0; i < v.size(); ++i) idx[i] = (int)i;
    std::stable_sort(idx.begin(), idx.end(), [&](int x, int y) { return v[x].cost > v[y].cost; });
    std::vector<int> used(4, 0);
    for (int i : idx) {
      int best = -1;
      for (int s = 0; s < 4; ++s)
        if (used[s] < per && (best < 0 || load[s] < load[best])) best = s;
      of[simd_waves[best][used[best]++]] = i;
      load[best] += v[i].cost;
    }
  };
  lpt(pairs, pair_of);
  lpt(singles, single_of);
}

// div2 steps of a column (forward d-1, backward 2d-1); a degree-1 column's
// FAST v2c needs none (bp_irregular.hip vn_cols), only its hard decision
#ifndef KML_IRR_VN_COST1
#define KML_IRR_VN_COST1 2.0
#endif
double vn_cost(int d) { return d == 1 ? KML_IRR_VN_COST1 : 3.0 * d - 1.0; }
double cn_cost(int d) { return 1.5 * d; }        // per half-row: advances + half the c2v outputs

}  // namespace

bool plan_irregular(const LdpcCode &L, int T, int vn_pair_max, int cn_pair_max, IrregularPlan &out) {
  if (T % 256) return false;
  const int W = T / 64;
  std::vector<std::vector<int32_t>> cols(L.dv_max + 1), rows(L.dc_max + 1);
  for (int32_t v : L.vn_order) cols[L.col_ptr[v + 1] - L.col_ptr[v]].push_back(v);
  for (int32_t r : L.cn_order) rows[L.row_ptr[r + 1] - L.row_ptr[r]].push_back(r);
  std::vector<WaveItems> vp, vs, cp, cs;
  if (!plan_rounds(cols, 64, W, vn_pair_max, vn_cost, vp, vs) ||
      !plan_rounds(rows, 32, W, cn_pair_max, cn_cost, cp, cs))
    return false;
  std::vector<int> vp_of, vs_of, cp_of, cs_of;
  place_waves(vp, vs, W, vp_of, vs_of);
  place_waves(cp, cs, W, cp_of, cs_of);
  out.vn.assign(3 * T, -1);
  out.cn.assign(3 * T / 2, -1);
  for (int w = 0; w < W; ++w) {
    if (vp_of[w] >= 0)
      for (size_t l = 0; l < vp[vp_of[w]].a.size(); ++l) {  // (a partial pair wave leaves lanes idle)
        out.vn[w * 64 + l] = vp[vp_of[w]].a[l];
        out.vn[T + w * 64 + l] = vp[vp_of[w]].b[l];
      }
    if (vs_of[w] >= 0)
      for (size_t l = 0; l < vs[vs_of[w]].a.size(); ++l) out.vn[2 * T + w * 64 + l] = vs[vs_of[w]].a[l];
    if (cp_of[w] >= 0)
      for (size_t l = 0; l < cp[cp_of[w]].a.size(); ++l) {
        out.cn[w * 32 + l] = cp[cp_of[w]].a[l];
        out.cn[T / 2 + w * 32 + l] = cp[cp_of[w]].b[l];
      }
    if (cs_of[w] >= 0)
      for (size_t l = 0; l < cs[cs_of[w]].a.size(); ++l) out.cn[T + w * 32 + l] = cs[cs_of[w]].a[l];
  }
  // slot blocks (kIrrCnStride), one per wave and round, in plan order
  std::vector<int32_t> slot_of(L.E, -1);
  out.cn_base.assign(3 * T / 2, -1);
  int next = 0;
  for (int r = 0; r < 3; ++r)
    for (int w = 0; w < W; ++w) {
      const int p0 = r * (T / 2) + w * 32;
      int dw = 0;
      for (int pi = 0; pi < 32; ++pi) {
        const int row = out.cn[p0 + pi];
        if (row >= 0) dw = std::max(dw, L.row_ptr[row + 1] - L.row_ptr[row]);
      }
      for (int pi = 0; pi < 32; ++pi) {
        const int row = out.cn[p0 + pi];
        if (row < 0) continue;
        out.cn_base[p0 + pi] = next + pi;
        for (int e = L.row_ptr[row]; e < L.row_ptr[row + 1]; ++e)
          slot_of[e] = next + pi + (e - L.row_ptr[row]) * kIrrCnStride;
      }
      next += dw * kIrrCnStride;
    }
  for (int32_t s : slot_of)
    if (s < 0) return false;
  out.n_slots = next;
  out.col_slot.resize(L.E);
  for (int e = 0; e < L.E; ++e) out.col_slot[e] = slot_of[L.col_slot[e]];
  return true;
}

}  // namespace kml

