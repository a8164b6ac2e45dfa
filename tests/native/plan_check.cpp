// Host checks of the kernels' placement plans (layout.cpp) on the reference's
// H files: every plan is a valid assignment of columns / rows / slots to lanes
// with the properties the kernels rely on.  Prints "plan_errors=0" on success.
//   plan_check <PEG2304 H> <BG2 H> <PEG8064 H>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <string>
#include <vector>

#include "code.hpp"
#include "layout.hpp"

using namespace kml;

static int errors = 0;
#define CHECK(c, ...)                 \
  do {                                \
    if (!(c)) {                       \
      ++errors;                       \
      if (errors < 20) {              \
        printf("FAIL %s: ", #c);      \
        printf(__VA_ARGS__);          \
        printf("\n");                 \
      }                               \
    }                                 \
  } while (0)

static bool load(LdpcCode &L, const char *path, bool is5g) {
  std::string err;
  if (!L.load(path, is5g, true, false, err)) {
    printf("load %s: %s\n", path, err.c_str());
    return false;
  }
  return true;
}

static int col_deg(const LdpcCode &L, int v) { return L.col_ptr[v + 1] - L.col_ptr[v]; }
static int row_deg(const LdpcCode &L, int r) { return L.row_ptr[r + 1] - L.row_ptr[r]; }

// bp_regular.hip: rows in CN-position order with the lane pair's edges
// interleaved; each edge's c2v byte address names its own slot and half.
static void check_regular(const LdpcCode &L) {
  RegularLayout P;
  plan_regular_layout(L, 768, P);
  CHECK((int)P.order.size() == L.N, "order size %zu", P.order.size());
  std::vector<int> seen(L.N, 0);
  for (int v : P.order) seen[v]++;
  for (int v = 0; v < L.N; v++) CHECK(seen[v] == 1, "column %d placed %d times", v, seen[v]);
  for (int p = 0; p < L.N; p++) CHECK(P.pos[P.order[p]] == p, "pos of position %d", p);
  std::vector<int> row_pos(L.M);
  for (int i = 0; i < L.M; i++) row_pos[L.cn_order[i]] = i;
  std::set<int> slots;
  for (int e = 0; e < L.E; e++) {  // e: a column-order edge; col_slot[e] = its row-order slot
    const int s = L.col_slot[e];
    int row = 0;
    while (L.row_ptr[row + 1] <= s) row++;
    const int j = s - L.row_ptr[row], dc = row_deg(L, row);
    const int phys = row_pos[row] * dc + (j < dc / 2 ? 2 * j : 2 * (dc - 1 - j) + 1);
    const int a = P.c2v_addr[e];
    CHECK(a / 16 == phys, "edge %d slot %d != %d", e, a / 16, phys);
    CHECK((a & 8) == 8 * ((row_pos[row] >> 2) & 1), "edge %d half", e);
    slots.insert(a / 16);
  }
  CHECK((int)slots.size() == L.E, "distinct slots %zu", slots.size());
  printf("regular: bank-conflict cost %lld -> %lld\n", P.cost_initial, P.cost_final);
}

// bp_irregular.hip: three rounds, pairs of equal degree (up to the limits) in
// rounds 0-1, every column / row exactly once, one degree per paired wave.
static void check_irregular(const LdpcCode &L) {
  const int T = kIrrThreads;
  IrregularPlan P;
  CHECK(plan_irregular(L, T, kIrrVnPairMax, kIrrCnPairMax, P), "plan_irregular failed");
  if (P.vn.empty()) return;
  CHECK((int)P.vn.size() == 3 * T && (int)P.cn.size() == 3 * T / 2, "sizes");
  std::vector<int> cs(L.N, 0), rs(L.M, 0);
  for (int v : P.vn)
    if (v >= 0) cs[v]++;
  for (int r : P.cn)
    if (r >= 0) rs[r]++;
  for (int v = 0; v < L.N; v++) CHECK(cs[v] == 1, "column %d placed %d times", v, cs[v]);
  for (int r = 0; r < L.M; r++) CHECK(rs[r] == 1, "row %d placed %d times", r, rs[r]);
  for (int t = 0; t < T; t++) {
    const int a = P.vn[t], b = P.vn[T + t];
    CHECK((a < 0) == (b < 0), "lane %d half-empty pair", t);
    if (a >= 0) {
      CHECK(col_deg(L, a) == col_deg(L, b), "lane %d pair degrees", t);
      CHECK(col_deg(L, a) <= kIrrVnPairMax, "lane %d pair degree %d", t, col_deg(L, a));
      CHECK(col_deg(L, a) == col_deg(L, P.vn[(t & ~63)]) || P.vn[t & ~63] < 0, "wave of lane %d mixes degrees", t);
    }
  }
  for (int q = 0; q < T / 2; q++) {
    const int a = P.cn[q], b = P.cn[T / 2 + q];
    CHECK((a < 0) == (b < 0), "pair %d half-empty", q);
    if (a >= 0) {
      CHECK(row_deg(L, a) == row_deg(L, b), "pair %d row degrees", q);
      CHECK(row_deg(L, a) <= kIrrCnPairMax, "pair %d row degree %d", q, row_deg(L, a));
    }
  }
  // slot blocks: edge e of the row at a lane pair sits at cn_base + e * kIrrCnStride,
  // every edge has its own slot, and the column-ordered table points at the same slots
  CHECK((int)P.cn_base.size() == 3 * T / 2 && (int)P.col_slot.size() == L.E, "slot table sizes");
  std::vector<int> owner(P.n_slots, -1), slot_of(L.E, -1);
  for (int q = 0; q < 3 * T / 2; q++) {
    const int r = P.cn[q];
    CHECK((r < 0) == (P.cn_base[q] < 0), "pair position %d base", q);
    if (r < 0) continue;
    for (int e = L.row_ptr[r]; e < L.row_ptr[r + 1]; e++) {
      const int s = P.cn_base[q] + (e - L.row_ptr[r]) * kIrrCnStride;
      CHECK(s >= 0 && s < P.n_slots && owner[s] < 0, "edge %d slot %d", e, s);
      if (s >= 0 && s < P.n_slots) owner[s] = e;
      slot_of[e] = s;
    }
  }
  for (int e = 0; e < L.E; e++) CHECK(P.col_slot[e] == slot_of[L.col_slot[e]], "column edge %d slot", e);
  printf("irregular: plan ok for T=%d, %d slots for %d edges\n", T, P.n_slots, L.E);
}

// bp_part_kernel: members own whole column / row blocks; every edge's LDS
// address of the column side is a row slot of the owner or one of its mirrors.
static void check_partition(const LdpcCode &L) {
  PartitionPlan P;
  CHECK(plan_partition(L, 4, P), "plan_partition failed");
  if (P.vn.empty()) return;
  std::vector<int> cs(L.N, 0), rs(L.M, 0);
  for (int v : P.vn) cs[v]++;
  for (int r : P.cn) rs[r]++;
  for (int v = 0; v < L.N; v++) CHECK(cs[v] == 1, "column %d placed %d times", v, cs[v]);
  for (int r = 0; r < L.M; r++) CHECK(rs[r] == 1, "row %d placed %d times", r, rs[r]);
  const int nslots = P.MG * L.dc_max + P.mirror_max;
  for (size_t i = 0; i < P.vaddr.size(); i++)
    CHECK(P.vaddr[i] >= 0 && P.vaddr[i] < nslots * 16, "vaddr %zu = %d", i, P.vaddr[i]);
  // tagged exchange: a row's cut edges have consecutive mailbox indices from
  // rx's first index, in row order; vx names the same index from the column side
  std::vector<int> seen_x(P.ncut, 0);
  const int EG = P.MG * L.dc_max;
  for (int m = 0; m < P.G; m++)
    for (int q = P.xr_ptr[m]; q < P.xr_ptr[m + 1]; q++) {
      const int x = P.xr[q] >> 16, slot = P.xr[q] & 0xFFFF;  // member-local row slot
      const int Pr = m * P.MG + slot / L.dc_max, e = slot % L.dc_max;
      const int mask = P.rx[Pr] & 0xFF;
      CHECK((mask >> e) & 1, "row %d edge %d not in its cut mask", Pr, e);
      const int want = (P.rx[Pr] >> 8) + __builtin_popcount(mask & ((1 << e) - 1));
      CHECK(x == want, "row %d edge %d: x %d, rx gives %d", Pr, e, x, want);
      seen_x[x]++;
    }
  long long nvx = 0;
  for (size_t i = 0; i < P.vx.size(); i++)
    if (P.vx[i] >= 0) {
      ++nvx;
      CHECK(P.vx[i] < P.ncut, "vx %zu = %d", i, P.vx[i]);
      CHECK(P.vaddr[i] >= EG * 16, "cut edge %zu addressed to a row slot", i);
    }
  CHECK(nvx == P.ncut, "vx names %lld cut edges of %d", nvx, P.ncut);
  // exact balance (member m owns vn[m NG, (m+1) NG) and cn[m MG, (m+1) MG)):
  // every uncut edge of a column addresses a row slot of its own member whose
  // row holds that column
  const int NG = P.NG, dv = L.dv_max, dc = L.dc_max;
  CHECK(NG * P.G == L.N && P.MG * P.G == L.M, "member sizes %d %d", NG, P.MG);
  for (int p = 0; p < L.N; p++)
    for (int k = 0; k < dv; k++) {
      if (P.vx[(size_t)p * dv + k] >= 0) continue;
      const int sl = P.vaddr[(size_t)p * dv + k] / 16, r = P.cn[(p / NG) * P.MG + sl / dc];
      bool has = false;
      for (int e = L.row_ptr[r]; e < L.row_ptr[r + 1]; e++) has |= L.row_col[e] == P.vn[p];
      CHECK(has, "column position %d edge %d: row %d of member %d does not hold it", p, k, r, p / NG);
    }
  // the refined cut (layout.cpp PartRefiner; the relabelling alone: 6,602)
  if (!getenv("KML_PART_REFINE") || getenv("KML_PART_REFINE")[0] != '0')
    CHECK(P.ncut <= (getenv("KML_PART_REFINE_ITERS") ? 6602 : 5700), "cut %d edges", P.ncut);
  for (int x = 0; x < P.ncut; x++) CHECK(seen_x[x] == 1, "mailbox index %d received %d times", x, seen_x[x]);
  printf("partition: %d of %d edges cut, mirror_max %d\n", P.ncut, L.E, P.mirror_max);
}

int main(int argc, char **argv) {
  if (argc < 4) return 2;
  LdpcCode a, b, c;
  if (!load(a, argv[1], false) || !load(b, argv[2], true) || !load(c, argv[3], false)) return 2;
  check_regular(a);
  check_irregular(b);
  check_partition(c);
  printf("plan_errors=%d\n", errors);
  return errors ? 1 : 0;
}
