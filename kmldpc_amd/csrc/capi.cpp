// capi.cpp — the C ABI (include/kmldpc_amd.h) over the host planner and the
// gfx950 kernels.  One context = one GPU + one HIP stream + one code/modem.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/kmldpc_amd.h"
#include "code.hpp"
#include "comm.hpp"
#include "config.hpp"
#include "kernels.hpp"
#include "layout.hpp"
#include "modem.hpp"

namespace kml {
int ref_frames(const LdpcCode &code, const Modem &modem, int64_t *state, double snr, int n, uint8_t *uu_out,
               double *h_out, double *y_out);
}

namespace {

struct DBuf {
  void *p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(bytes, 256);
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T *as() const {
    return reinterpret_cast<T *>(p);
  }
};

struct Pending {
  std::string stage;
  hipEvent_t ev0, ev1;
  int cnt_slot;  // counter-arena slot for "bp" launches (-1 otherwise)
  double fixed_bytes;
};

struct Stat {
  int64_t launches = 0;
  double ms = 0, bytes = 0, flops = 0;
};

constexpr int kArenaSlots = 1024;

}  // namespace

struct kml_ctx {
  int device = 0;
  const char *bp_family = nullptr;  // kernel family of the last BP launch
  hipStream_t stream = nullptr;
  hipStream_t cstream = nullptr;  // host-buffer frame uploads (kml_decode_frames' chunked path), made on first use
  kml::RunConfig rc;
  kml::LdpcCode code;
  kml::Modem modem;
  kml::DevCode dc{};
  double rot[8];
  // resident constants
  DBuf d_graph, d_cons;
  // algorithmic fp64 flops per executed VN / CN phase ("Roofline")
  double vn_flops = 0, cn_flops = 0;
  DBuf d_arena;  // kArenaSlots x CNT_N counters
  int arena_next = 0;
  DBuf d_queue, d_gslots, d_gsync, d_gcch;
  long long gslots_cap = 0;
  int coop_groups = 0;      // cooperative BP groups (0: kernel not used)
  long long part_cut = 0;   // cut edges of the partition plan (partitioned cooperative kernel)
  bool coop_pending = false;  // a cooperative launch whose abort word is unchecked
  bool coop_this_call = false;  // the current API call made a cooperative launch (fail() settles it)
  bool coop_inherited = false;  // ... on top of an earlier call's unchecked launch (the abort word is shared)
  int inject_abort = -1;      // test hook (kml_debug_inject_abort): raise the abort after the n-th coop launch
  bool inject_fail = false;   // test hook (kml_debug_inject_abort(-2)): ... and fail that call before its sync
  kml::RcclComm *comm = nullptr;  // counter all-reduce over the ranks (kml_comm_init)
  DBuf w_comm;
  DBuf w_defer;  // BP launches: codewords the FAST kernel leaves to the exact kernel (+ count)
  DBuf w_ddefer;  // demap / candidate-metric launches: the same for symbols or codewords
  // workspaces
  DBuf w_y, w_h, w_h4, w_hhat, w_p0, w_uu, w_uh, w_uh4, w_ret, w_cch, w_syn, w_sel, w_met, w_pc, w_cnt, w_km, w_cwerr;
  // soft syndrome metric: candidate / final syndromes, iteration counts, sums, decode lists
  DBuf s_synm, s_synf, s_itm, s_itf, s_Lm, s_Lf, s_list, s_sel;
  // Sum of log(syndrom_soft) of the most recent decode that ran a CN phase on
  // this context (the reference codec's stale member array, reduced to what
  // the metric reads); -inf = the never-written (zero) array.
  double soft_state = -INFINITY;
  // resident simulation frames
  DBuf s_uu, s_cc, s_y, s_h;
  DBuf w_hc;  // caller candidates (kml_decode_candidates)
  int sim_B = 0;
  double sim_snr = 0;
  uint64_t sim_first = 0;
  // profiling
  bool prof = false;
  std::vector<Pending> pend;
  std::map<std::string, Stat> stats;
  std::string err;
};

namespace {

// An error return of a call that made a cooperative launch and will not reach
// its sync(): the launch's abort word is settled here (waited for, dropped with
// the call's error), so the next call's first launch clears it instead of
// inheriting it (a stale timeout reported against a healthy call).  A pending
// launch of an EARLIER call (kml_sim_decode with do_sync = 0) stays pending
// for its own kml_sync: when this call's launches shared its abort word
// (coop_inherited) and the word is set, it stays pending.
int fail(kml_ctx *c, int code, const std::string &msg) {
  if (c) {
    c->err = msg;
    if (c->coop_pending && c->coop_this_call) {
      bool keep = false;
      if (c->stream) {
        (void)hipStreamSynchronize(c->stream);
        if (c->coop_inherited) {
          kml::BpLaunch a;
          a.gsync = c->d_gsync.p;
          keep = kml::bp_coop_aborted(a, c->coop_groups, c->stream);
        }
      }
      c->coop_pending = keep;
      c->coop_this_call = false;
    }
  }
  return code;
}

// Every entry point that takes a context starts here: a new API call, so the
// cooperative launches fail() settles are only this call's.
inline void call_begin(kml_ctx *c) {
  if (c) c->coop_this_call = false;
}

int hip_fail(kml_ctx *c, hipError_t e, const char *what) {
  return fail(c, KML_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

#define HIPCHK(ctx, expr, what)                       \
  do {                                                \
    hipError_t _e = (expr);                           \
    if (_e != hipSuccess) return hip_fail(ctx, _e, what); \
  } while (0)

int upload_code(kml_ctx *c) {
  const kml::LdpcCode &L = c->code;
  // pack all int32 arrays + enc words into one allocation
  std::vector<size_t> off;
  size_t bytes = 0;
  auto reserve = [&](size_t n) {
    bytes = (bytes + 255) & ~size_t(255);
    off.push_back(bytes);
    bytes += n;
  };
  reserve(L.row_ptr.size() * 4);
  reserve(L.row_col.size() * 4);
  reserve(L.col_ptr.size() * 4);
  int regular = 1;
  for (int j = 0; j < L.N; j++)
    if (L.col_ptr[j + 1] - L.col_ptr[j] != L.dv_max) regular = 0;
  for (int i = 0; i < L.M; i++)
    if (L.row_ptr[i + 1] - L.row_ptr[i] != L.dc_max) regular = 0;
  const int reg_T = kml::bp_regular_threads(L.N, L.M, L.E, L.dv_max, L.dc_max, regular);
  kml::RegularLayout plan;
  if (reg_T > 0) kml::plan_regular_layout(L, reg_T, plan);
  const std::vector<int32_t> &vn_order = reg_T > 0 ? plan.order : L.vn_order;
  if (reg_T <= 0) {  // column -> vn position, used by the cooperative kernel
    plan.pos.assign(L.N, 0);
    for (int p = 0; p < L.N; p++) plan.pos[L.vn_order[p]] = p;
  }
  reserve(L.col_slot.size() * 4);
  reserve(vn_order.size() * 4);
  reserve(L.cn_order.size() * 4);
  reserve(std::max<size_t>(L.enc_info.size(), 1) * 8);
  reserve(plan.c2v_addr.size() * 4);
  reserve(plan.pos.size() * 4);
  // partition plan of the partitioned cooperative kernel (codes whose slots exceed one CU's LDS)
  kml::PartitionPlan part;
  const int part_G = kml::bp_part_group_size(L.N, L.M, L.E, L.dv_max, L.dc_max, regular);
  if (part_G > 0 && !kml::plan_partition(L, part_G, part)) part.G = 0;
  if (part.G && getenv("KML_PLAN_VERBOSE"))
    fprintf(stderr, "partition plan: G %d, %d cut edges, mirrors <= %d, VN bank model cost %lld -> %lld\n", part.G,
            part.ncut, part.mirror_max, part.anneal_initial, part.anneal_final);
  int part_xmax = 0;
  for (int m = 0; part.G && m < part.G; m++)
    part_xmax = std::max({part_xmax, part.xr_ptr[m + 1] - part.xr_ptr[m], part.xc_ptr[m + 1] - part.xc_ptr[m]});
  if (part.G && !kml::part_plan_fits(part.G, L.N, L.M, L.E, part.ncut, part.mirror_max, part_xmax)) part.G = 0;
  reserve(part.vn.size() * 4);
  reserve(part.cn.size() * 4);
  reserve(part.pos.size() * 4);
  reserve(part.vaddr.size() * 4);
  reserve(part.xr.size() * 4);
  reserve(part.xr_ptr.size() * 4);
  reserve(part.xc.size() * 4);
  reserve(part.xc_ptr.size() * 4);
  reserve(part.vx.size() * 4);
  reserve(part.rx.size() * 4);
  // round plan of the irregular-code kernel (layout.hpp IrregularPlan)
  kml::IrregularPlan irr;
  if (!regular && !kml::plan_irregular(L, kml::kIrrThreads, kml::kIrrVnPairMax, kml::kIrrCnPairMax, irr))
    irr = kml::IrregularPlan();
  reserve(irr.vn.size() * 4);
  reserve(irr.cn.size() * 4);
  reserve(irr.cn_base.size() * 4);
  reserve(irr.col_slot.size() * 4);
  HIPCHK(c, c->d_graph.ensure(bytes), "hipMalloc(graph)");
  std::vector<unsigned char> host(bytes, 0);
  auto put = [&](int i, const void *src, size_t n) {
    if (n) memcpy(host.data() + off[i], src, n);
  };
  put(0, L.row_ptr.data(), L.row_ptr.size() * 4);
  put(1, L.row_col.data(), L.row_col.size() * 4);
  put(2, L.col_ptr.data(), L.col_ptr.size() * 4);
  put(3, L.col_slot.data(), L.col_slot.size() * 4);
  put(4, vn_order.data(), vn_order.size() * 4);
  put(5, L.cn_order.data(), L.cn_order.size() * 4);
  put(6, L.enc_info.data(), L.enc_info.size() * 8);
  put(7, plan.c2v_addr.data(), plan.c2v_addr.size() * 4);
  put(8, plan.pos.data(), plan.pos.size() * 4);
  put(9, part.vn.data(), part.vn.size() * 4);
  put(10, part.cn.data(), part.cn.size() * 4);
  put(11, part.pos.data(), part.pos.size() * 4);
  put(12, part.vaddr.data(), part.vaddr.size() * 4);
  put(13, part.xr.data(), part.xr.size() * 4);
  put(14, part.xr_ptr.data(), part.xr_ptr.size() * 4);
  put(15, part.xc.data(), part.xc.size() * 4);
  put(16, part.xc_ptr.data(), part.xc_ptr.size() * 4);
  put(17, part.vx.data(), part.vx.size() * 4);
  put(18, part.rx.data(), part.rx.size() * 4);
  put(19, irr.vn.data(), irr.vn.size() * 4);
  put(20, irr.cn.data(), irr.cn.size() * 4);
  put(21, irr.cn_base.data(), irr.cn_base.size() * 4);
  put(22, irr.col_slot.data(), irr.col_slot.size() * 4);
  HIPCHK(c, hipMemcpy(c->d_graph.p, host.data(), bytes, hipMemcpyHostToDevice), "upload graph");
  unsigned char *base = c->d_graph.as<unsigned char>();
  kml::DevCode &d = c->dc;
  d.row_ptr = reinterpret_cast<const int32_t *>(base + off[0]);
  d.row_col = reinterpret_cast<const int32_t *>(base + off[1]);
  d.col_ptr = reinterpret_cast<const int32_t *>(base + off[2]);
  d.col_slot = reinterpret_cast<const int32_t *>(base + off[3]);
  d.vn_order = reinterpret_cast<const int32_t *>(base + off[4]);
  d.cn_order = reinterpret_cast<const int32_t *>(base + off[5]);
  d.enc_info = reinterpret_cast<const uint64_t *>(base + off[6]);
  d.reg_c2v = reg_T > 0 ? reinterpret_cast<const int32_t *>(base + off[7]) : nullptr;
  d.reg_pos = reinterpret_cast<const int32_t *>(base + off[8]);
  d.pt_G = part.G;
  d.pt_vn = part.G ? reinterpret_cast<const int32_t *>(base + off[9]) : nullptr;
  d.pt_cn = part.G ? reinterpret_cast<const int32_t *>(base + off[10]) : nullptr;
  d.pt_pos = part.G ? reinterpret_cast<const int32_t *>(base + off[11]) : nullptr;
  d.pt_vaddr = part.G ? reinterpret_cast<const int32_t *>(base + off[12]) : nullptr;
  d.pt_xr = part.G ? reinterpret_cast<const int32_t *>(base + off[13]) : nullptr;
  d.pt_xr_ptr = part.G ? reinterpret_cast<const int32_t *>(base + off[14]) : nullptr;
  d.pt_xc = part.G ? reinterpret_cast<const int32_t *>(base + off[15]) : nullptr;
  d.pt_xc_ptr = part.G ? reinterpret_cast<const int32_t *>(base + off[16]) : nullptr;
  d.pt_vx = part.G ? reinterpret_cast<const int32_t *>(base + off[17]) : nullptr;
  d.pt_rx = part.G ? reinterpret_cast<const int32_t *>(base + off[18]) : nullptr;
  d.irr_vn = irr.vn.empty() ? nullptr : reinterpret_cast<const int32_t *>(base + off[19]);
  d.irr_cn = irr.cn.empty() ? nullptr : reinterpret_cast<const int32_t *>(base + off[20]);
  d.irr_cn_base = irr.cn.empty() ? nullptr : reinterpret_cast<const int32_t *>(base + off[21]);
  d.irr_col_slot = irr.cn.empty() ? nullptr : reinterpret_cast<const int32_t *>(base + off[22]);
  d.irr_slots = irr.n_slots;
  d.pt_ncut = part.ncut;
  d.pt_mirror = part.mirror_max;
  d.pt_pairs = part.all_pairs ? 1 : 0;
  for (int m = 0; m < 8; m++) {
    d.pt_xr_n[m] = m < part.G ? part.xr_ptr[m + 1] - part.xr_ptr[m] : 0;
    d.pt_xc_n[m] = m < part.G ? part.xc_ptr[m + 1] - part.xc_ptr[m] : 0;
  }
  c->part_cut = part.ncut;
  d.M = L.M;
  d.N = L.N;
  d.E = L.E;
  d.K = L.K;
  d.cc_len = L.cc_len;
  d.punct = L.punct;
  d.info_off = L.info_off;
  d.chk = L.chk;
  d.Kw = L.Kw;
  d.dv_max = L.dv_max;
  d.dc_max = L.dc_max;
  d.is5g = L.is5g ? 1 : 0;
  d.active = L.active ? 1 : 0;
  d.regular = regular;
  d.irr_ok = 1;
  for (int j = 0; j < L.N; j++) {
    const int dv = L.col_ptr[j + 1] - L.col_ptr[j];
    if (dv < 1 || dv > 9) d.irr_ok = 0;
  }
  for (int i = 0; i < L.M; i++) {
    const int dc = L.row_ptr[i + 1] - L.row_ptr[i];
    if (dc < 2 || dc > 10) d.irr_ok = 0;
  }

  HIPCHK(c, c->d_cons.ensure(sizeof(double) * (c->modem.pts.size() + 8)), "hipMalloc(cons)");
  kml::rotation_factors(c->rot);
  std::vector<double> cr(c->modem.pts);
  cr.insert(cr.end(), c->rot, c->rot + 8);
  HIPCHK(c, hipMemcpy(c->d_cons.p, cr.data(), sizeof(double) * cr.size(), hipMemcpyHostToDevice), "upload cons");
  HIPCHK(c, c->d_arena.ensure(sizeof(unsigned long long) * kml::CNT_N * kArenaSlots), "hipMalloc(counters)");
  HIPCHK(c, c->d_queue.ensure(256), "hipMalloc(queue)");
  const long long need = kml::bp_gslots_needed(d);
  if (need > 0) {
    HIPCHK(c, c->d_gslots.ensure((size_t)need * sizeof(double2)), "hipMalloc(gslots)");
    c->gslots_cap = need;
  }
  c->coop_groups = kml::bp_coop_groups(d);
  if (c->coop_groups > 0) {
    HIPCHK(c, c->d_gsync.ensure(kml::bp_coop_sync_bytes(c->coop_groups)), "hipMalloc(gsync)");
    HIPCHK(c, c->d_gcch.ensure((size_t)c->coop_groups * L.N), "hipMalloc(gcch)");
  }
  return KML_OK;
}

// FP64 work of one VN / CN phase of the exact algorithm: per column of degree
// d, 68d - 23 flops; per row of degree d, 73d - 52 flops (fma = 2, mul / add /
// sub / rcp = 1; each normalisation pair = one reciprocal refinement + two
// residual corrections, the minimal exact-IEEE sequence).
void phase_flops(kml_ctx *c) {
  const kml::LdpcCode &L = c->code;
  double v = 0, r = 0;
  for (int j = 0; j < L.N; j++) v += 68.0 * (L.col_ptr[j + 1] - L.col_ptr[j]) - 23.0;
  for (int i = 0; i < L.M; i++) r += 73.0 * (L.row_ptr[i + 1] - L.row_ptr[i]) - 52.0;
  c->vn_flops = v;
  c->cn_flops = r;
}

int finish_create(kml_ctx *c) {
  std::string err;
  if (!c->code.load(c->rc.matrix_file, c->rc.is5g, c->rc.active, false, err)) return fail(c, KML_E_IO, err);
  phase_flops(c);
  if (!c->modem.load(c->rc.modem_file, err)) return fail(c, KML_E_IO, err);
  if (c->code.cc_len % c->modem.bits != 0)  // modemlinearsystem.cc:7-12
    return fail(c, KML_E_ARG, "(cc_len = " + std::to_string(c->code.cc_len) + ") % (input_len = " +
                                  std::to_string(c->modem.bits) + ") != 0");
  if (c->modem.bits != 1 && c->modem.bits != 2 && c->modem.bits != 3 && c->modem.bits != 4 && c->modem.bits != 6)
    return fail(c, KML_E_UNSUP, "bits per symbol must be 1, 2, 3, 4 or 6");
  if (c->device < 0) {  // host-only context: planner + encoder, no GPU
    kml::rotation_factors(c->rot);
    return KML_OK;
  }
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  HIPCHK(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking), "hipStreamCreate");
  return upload_code(c);
}

// ---- profiling helpers
int next_slot(kml_ctx *c) {
  int s = c->arena_next;
  c->arena_next = (c->arena_next + 1) % kArenaSlots;
  return s;
}
unsigned long long *slot_ptr(kml_ctx *c, int s) { return c->d_arena.as<unsigned long long>() + (size_t)s * kml::CNT_N; }

struct Timer {
  kml_ctx *c;
  Pending p;
  bool on;
  Timer(kml_ctx *ctx, const char *stage, int slot, double bytes) : c(ctx), on(ctx->prof) {
    if (!on) return;
    p.stage = stage;
    p.cnt_slot = slot;
    p.fixed_bytes = bytes;
    hipEventCreate(&p.ev0);
    hipEventCreate(&p.ev1);
    hipEventRecord(p.ev0, c->stream);
  }
  void stop() {
    if (!on) return;
    hipEventRecord(p.ev1, c->stream);
    c->pend.push_back(p);
    on = false;
  }
};

void drain_profile(kml_ctx *c) {
  if (c->pend.empty()) return;
  hipStreamSynchronize(c->stream);
  for (auto &p : c->pend) {
    float ms = 0;
    hipEventElapsedTime(&ms, p.ev0, p.ev1);
    Stat &s = c->stats[p.stage];
    s.launches++;
    s.ms += ms;
    double bytes = p.fixed_bytes;
    if (p.cnt_slot >= 0) {
      unsigned long long h[kml::CNT_N];
      hipMemcpy(h, slot_ptr(c, p.cnt_slot), sizeof(h), hipMemcpyDeviceToHost);
      const double E = c->code.E, N = c->code.N;
      bytes += (double)h[kml::CNT_VN_PHASES] * (24.0 * E + 9.0 * N) + (double)h[kml::CNT_CN_PHASES] * 24.0 * E;
    }
    s.bytes += bytes;
    if (p.cnt_slot >= 0) {
      unsigned long long h[kml::CNT_N];
      hipMemcpy(h, slot_ptr(c, p.cnt_slot), sizeof(h), hipMemcpyDeviceToHost);
      s.flops += (double)h[kml::CNT_VN_PHASES] * c->vn_flops + (double)h[kml::CNT_CN_PHASES] * c->cn_flops;
    }
    hipEventDestroy(p.ev0);
    hipEventDestroy(p.ev1);
  }
  c->pend.clear();
}

// Launch BP over n entries with a fresh counter slot; returns the slot.
// reuse >= 0 accumulates into that (already zeroed) slot.
int run_bp(kml_ctx *c, kml::BpLaunch a, int &slot_out, int reuse = -1) {
  const int slot = reuse >= 0 ? reuse : next_slot(c);
  if (reuse < 0)
    HIPCHK(c, hipMemsetAsync(slot_ptr(c, slot), 0, sizeof(unsigned long long) * kml::CNT_N, c->stream), "memset");
  a.counters = slot_ptr(c, slot);
  HIPCHK(c, c->w_defer.ensure(sizeof(int32_t) * ((size_t)a.B + 16)), "hipMalloc(defer list)");
  a.defer_idx = c->w_defer.as<int32_t>();
  a.defer_cnt = reinterpret_cast<unsigned *>(c->w_defer.as<int32_t>() + a.B);
  a.gslots = c->d_gslots.as<double2>();
  a.gslots_cap = c->gslots_cap;
  a.queue = c->d_queue.as<unsigned int>();
  a.gsync = c->d_gsync.p;
  a.gcch = c->d_gcch.as<uint8_t>();
  // the abort word is cleared only by the first cooperative launch after the
  // last sync(): a timeout in any launch before the check (e.g. chunk 0 of a
  // chunked host-buffer call) stays set until sync() reports it
  a.reset_abort = !c->coop_pending;
  if (c->coop_groups > 0) {
    if (!c->coop_this_call) c->coop_inherited = c->coop_pending;  // the call's first cooperative launch
    c->coop_pending = c->coop_this_call = true;
  }
  Timer t(c, "bp", slot, (double)a.B * 8.0 * c->code.cc_len);
  const char *msg = nullptr;
  hipError_t e = kml::launch_bp(c->dc, a, c->stream, &msg, &c->bp_family);
  t.stop();
  if (e != hipSuccess) return msg ? fail(c, KML_E_UNSUP, msg) : hip_fail(c, e, "bp launch");
  if (c->inject_abort >= 0 && c->coop_groups > 0 && c->inject_abort-- == 0)  // as if a group barrier timed out
  {
    HIPCHK(c, kml::bp_coop_raise_abort(a, c->coop_groups, c->stream), "inject abort");
    if (c->inject_fail) {
      c->inject_fail = false;
      return fail(c, KML_E_HIP, "injected failure after a cooperative launch (kml_debug_inject_abort)");
    }
  }
  slot_out = slot;
  return KML_OK;
}

// The FAST demappers' defer list (kernels.hpp DemapDefer): at least `need`
// entries (the candidate metric defers whole codewords: need = B).
int demap_defer(kml_ctx *c, int need, kml::DemapDefer &d) {
  const int cap = std::max(need, 65536);
  HIPCHK(c, c->w_ddefer.ensure(sizeof(int32_t) * ((size_t)cap + 16)), "hipMalloc(demap defer list)");
  d.idx = c->w_ddefer.as<int32_t>();
  d.cnt = reinterpret_cast<unsigned *>(d.idx + cap);
  d.cap = cap;
  return KML_OK;
}

// Stage a host or device input; returns a device pointer.
template <class T>
int stage_in(kml_ctx *c, DBuf &buf, const T *src, size_t n, int flags, const T *&dev) {
  if (flags & KML_DEVICE_PTRS) {
    dev = src;
    return KML_OK;
  }
  HIPCHK(c, buf.ensure(n * sizeof(T)), "hipMalloc(workspace)");
  if (n) HIPCHK(c, hipMemcpyAsync(buf.p, src, n * sizeof(T), hipMemcpyHostToDevice, c->stream), "H2D");
  dev = buf.as<T>();
  return KML_OK;
}

template <class T>
int stage_out_ptr(kml_ctx *c, DBuf &buf, T *dst, size_t n, int flags, T *&dev) {
  if (!dst) {
    dev = nullptr;
    return KML_OK;
  }
  if (flags & KML_DEVICE_PTRS) {
    dev = dst;
    return KML_OK;
  }
  HIPCHK(c, buf.ensure(n * sizeof(T)), "hipMalloc(workspace)");
  dev = buf.as<T>();
  return KML_OK;
}

template <class T>
int copy_out(kml_ctx *c, T *dst, const T *dev, size_t n, int flags) {
  if (!dst || (flags & KML_DEVICE_PTRS) || n == 0) return KML_OK;
  HIPCHK(c, hipMemcpyAsync(dst, dev, n * sizeof(T), hipMemcpyDeviceToHost, c->stream), "D2H");
  return KML_OK;
}

int sync(kml_ctx *c) {
  HIPCHK(c, hipStreamSynchronize(c->stream), "hipStreamSynchronize");
  if (c->coop_pending) {
    c->coop_pending = false;
    kml::BpLaunch a;
    a.gsync = c->d_gsync.p;
    unsigned why = 0;
    if (kml::bp_coop_aborted(a, c->coop_groups, c->stream, &why)) {
      static const char *const site[] = {"raised by the host", "group barrier", "v2c mailbox poll", "c2v mailbox poll",
                                         "early-stop flag poll"};
      const unsigned k = why >> 24;
      return fail(c, KML_E_HIP,
                  std::string("cooperative BP kernel aborted: ") + (k == 0 ? "" : "timed out at ") + (k < 5 ? site[k] : "?") +
                      (why ? ", workgroup " + std::to_string(why & 0xFFFFFFu) : std::string()));
    }
  }
  return KML_OK;
}

int need_gpu(kml_ctx *c) {
  if (c->device < 0 || !c->stream) return fail(c, KML_E_ARG, "host-only context (device < 0): no GPU operations");
  return KML_OK;
}

#define TRY(x)            \
  do {                    \
    int _r = (x);         \
    if (_r != KML_OK) return _r; \
  } while (0)

// Receive path shared by kml_decode_frames, kml_sim_decode and
// kml_sim_histogram.  All pointers are device pointers.
struct RecvIO {
  const double2 *y = nullptr;
  const double2 *true_h = nullptr;  // known channel (simulator.cc:132-133); NULL = blind
  const double2 *cand = nullptr;    // caller's candidates [B][ncand] (KmCodec::Decoder h_hats), ncand > 1
  int ncand = 0;
  uint8_t *uh = nullptr;            // uu_hat[B][K] (NULL: not kept)
  int32_t *chosen = nullptr;        // [B]
  double *met = nullptr;            // [B][4]
  int32_t *ret = nullptr;           // [B]
  double2 *hhat = nullptr;          // [B] k-means h_hat
  const uint64_t *ref_bits = nullptr;  // packed source bits for CntErr
  int32_t *cw_err = nullptr;           // [B] error bits per codeword
  // GetHistogramData instead of Decoder (simulator.cc:154-162): candidate
  // metrics only, no final decode; CntErr then sees the uu_hat left by the last
  // candidate's metric decode (5G metric), or all zeros for the hard PEG metric
  // (the reference's uu_hat buffer is uninitialised there).
  bool histogram = false;
  // soft metric stale-state rule: in the simulator (sim) the reference's codec
  // is copied per task of thread_block_number codewords, so the state restarts
  // at global indices that are multiples of it (and at the batch start);
  // kml_decode_frames carries it across calls like one KmCodec instance.
  bool sim = false;
  uint64_t first_cw = 0;
};

int soft_receive(kml_ctx *c, const RecvIO &io, double var, int B, const double2 *hc, int nc, int &bp_slot);

int receive(kml_ctx *c, const RecvIO &io, double snr, int B, int &bp_slot) {
  double var, sigma, ns;
  kml::channel_constants(snr, var, sigma, ns);
  const int S = c->code.cc_len / c->modem.bits;
  const double *cons = c->d_cons.as<double>();
  const double *rot = cons + c->modem.pts.size();
  const size_t cc = (size_t)c->code.cc_len;
  const int K = c->code.K;
  kml::BpLaunch a;
  a.B = B;
  a.iter_count = c->rc.max_iter;
  a.max_iter = c->rc.max_iter;
  a.uu_hat = io.uh;
  a.ret = io.ret;
  a.ref_bits = io.ref_bits;
  a.cw_err = io.cw_err;
  if (io.true_h && !io.histogram && kml::bp_regular_fuses_demap(c->dc, c->modem.bits)) {
    // known channel on the regular kernel: the demap runs in its prologue
    a.sym_y = io.y;
    a.sym_h = io.true_h;
    a.sym_cons = cons;
    a.sym_var = var;
    a.sym_bits = c->modem.bits;
    return run_bp(c, a, bp_slot);
  }
  if (io.true_h && !io.histogram) {  // known channel: one demap + BP
    HIPCHK(c, c->w_p0.ensure(sizeof(double) * cc * B), "hipMalloc(p0)");
    Timer t(c, "demap", -1, (double)B * S * (16.0 + 8.0 * c->modem.bits));
    kml::DemapDefer dd;
    TRY(demap_defer(c, 0, dd));
    HIPCHK(c, kml::launch_demap(c->modem.bits, cons, io.y, S, 1, io.true_h, 1, nullptr, var, B, c->w_p0.as<double>(),
                                dd, c->stream),
           "demap");
    t.stop();
    a.p0 = c->w_p0.as<double>();
    a.p0_stride = (long long)cc;
    return run_bp(c, a, bp_slot);
  }
  // candidate channel estimates: the true h (histogram on the known-H path) or
  // k-means + 4 rotations (simulator.cc:136-148)
  const double2 *hc;
  int nc;
  if (io.cand) {
    hc = io.cand;
    nc = io.ncand;
  } else if (io.true_h) {
    hc = io.true_h;
    nc = 1;
  } else {
    HIPCHK(c, c->w_h4.ensure(sizeof(double2) * 4 * B), "hipMalloc(h4)");
    double2 *hh = io.hhat;
    if (!hh) {
      HIPCHK(c, c->w_hhat.ensure(sizeof(double2) * B), "hipMalloc(hhat)");
      hh = c->w_hhat.as<double2>();
    }
    HIPCHK(c, c->w_km.ensure(kml::kmeans_workspace_bytes(S, B)), "hipMalloc(kmeans)");
    Timer t(c, "kmeans", -1, (double)B * S * 16.0);
    HIPCHK(c, kml::launch_kmeans(c->modem.Kc, cons, rot, io.y, S, 20, B, hh, c->w_h4.as<double2>(), c->w_km.p,
                                 c->stream),
           "kmeans");
    t.stop();
    hc = c->w_h4.as<double2>();
    nc = 4;
  }
  int32_t *chosen = io.chosen;
  double *met = io.met;
  if (!chosen) {
    HIPCHK(c, c->w_sel.ensure(sizeof(int32_t) * B), "hipMalloc(sel)");
    chosen = c->w_sel.as<int32_t>();
  }
  if (!met) {
    HIPCHK(c, c->w_met.ensure(sizeof(double) * 4 * B), "hipMalloc(met)");
    met = c->w_met.as<double>();
  }
  if (c->rc.metric_soft) return soft_receive(c, io, var, B, hc, nc, bp_slot);
  // histogram mode: the counters go to a fresh arena slot (read back like BP's)
  unsigned long long *hist_cnt = nullptr;
  if (io.histogram) {
    bp_slot = next_slot(c);
    hist_cnt = slot_ptr(c, bp_slot);
    HIPCHK(c, hipMemsetAsync(hist_cnt, 0, sizeof(unsigned long long) * kml::CNT_N, c->stream), "memset");
  }
  if (!c->code.is5g) {  // hard metric on the demapper output (kmcodec.cc:109-117)
    Timer t(c, "metric", -1, (double)B * nc * S * 16.0);
    kml::DemapDefer dd;
    TRY(demap_defer(c, B, dd));
    HIPCHK(c, kml::launch_cand_metric(c->dc, c->modem.bits, cons, io.y, S, hc, nc, var, B, met, chosen, dd, c->stream),
           "cand_metric");
    t.stop();
    if (io.histogram) {
      if (io.ref_bits)
        HIPCHK(c, kml::launch_count_packed(io.ref_bits, c->code.Kw, K, nullptr, 0, B, io.cw_err, hist_cnt, c->stream),
               "count");
      if (io.uh) HIPCHK(c, hipMemsetAsync(io.uh, 0, (size_t)B * K, c->stream), "memset uh");
      return KML_OK;
    }
    if (kml::bp_regular_fuses_demap(c->dc, c->modem.bits)) {  // demap with the chosen estimate in the BP prologue
      a.sym_y = io.y;
      a.sym_h = hc;
      a.sym_h_stride = nc;
      a.sym_h_sel = chosen;
      a.sym_cons = cons;
      a.sym_var = var;
      a.sym_bits = c->modem.bits;
      return run_bp(c, a, bp_slot);
    }
    HIPCHK(c, c->w_p0.ensure(sizeof(double) * cc * B), "hipMalloc(p0)");
    Timer t2(c, "demap", -1, (double)B * S * (16.0 + 8.0 * c->modem.bits));
    HIPCHK(c, kml::launch_demap(c->modem.bits, cons, io.y, S, 1, hc, nc, chosen, var, B, c->w_p0.as<double>(),
                                dd, c->stream),
           "demap");
    t2.stop();
    a.p0 = c->w_p0.as<double>();
    a.p0_stride = (long long)cc;
    return run_bp(c, a, bp_slot);
  }
  // 5G: metric = parity count after metric_iter BP iterations (kmcodec.cc:157-160)
  HIPCHK(c, c->w_p0.ensure(sizeof(double) * cc * nc * B), "hipMalloc(p0)");
  HIPCHK(c, c->w_pc.ensure(sizeof(int32_t) * nc * B), "hipMalloc(pc)");
  {
    Timer t(c, "demap", -1, (double)nc * B * S * (16.0 + 8.0 * c->modem.bits));
    kml::DemapDefer dd;
    TRY(demap_defer(c, 0, dd));
    HIPCHK(c, kml::launch_demap(c->modem.bits, cons, io.y, S, nc, hc, 1, nullptr, var, nc * B, c->w_p0.as<double>(),
                                dd, c->stream),
           "demap candidates");
    t.stop();
  }
  kml::BpLaunch m;
  m.B = nc * B;
  m.iter_count = c->rc.metric_iter;
  m.max_iter = c->rc.max_iter;
  m.p0 = c->w_p0.as<double>();
  m.p0_stride = (long long)cc;
  m.parity_cnt = c->w_pc.as<int32_t>();
  if (io.histogram) {  // keep the candidates' uu_hat: CntErr reads the last one's
    HIPCHK(c, c->w_uh4.ensure((size_t)nc * B * K), "hipMalloc(uh4)");
    m.uu_hat = c->w_uh4.as<uint8_t>();
  }
  int mslot = 0;
  TRY(run_bp(c, m, mslot));
  HIPCHK(c, kml::launch_select(c->w_pc.as<int32_t>(), nc, B, met, chosen, c->stream), "select");
  if (io.histogram) {
    const uint8_t *last = c->w_uh4.as<uint8_t>() + (size_t)(nc - 1) * K;
    if (io.ref_bits)
      HIPCHK(c, kml::launch_count_packed(io.ref_bits, c->code.Kw, K, last, (long long)nc * K, B, io.cw_err, hist_cnt,
                                         c->stream),
             "count");
    if (io.uh)
      HIPCHK(c, hipMemcpy2DAsync(io.uh, K, last, (size_t)nc * K, K, B, hipMemcpyDeviceToDevice, c->stream), "copy uh");
    return KML_OK;
  }
  a.p0 = c->w_p0.as<double>();
  a.p0_stride = (long long)cc * nc;
  a.p0_sel = chosen;
  a.p0_sel_stride = (long long)cc;
  return run_bp(c, a, bp_slot);
}

// Soft syndrome metric (kmcodec.cc:145-156 with metric_type = true): for each
// candidate, BP for metric_iter iterations, metric = |sum_j log(syndrom_soft[j])|.
// syndrom_soft is the codec's member array and is only rewritten when a CN
// phase runs, so a candidate whose decode stops at iteration 0 reads the array
// left by the most recent decode that did run one — an earlier candidate, the
// previous codeword's final decode, ... — a sequential dependency across the
// batch.  Only the sum of logs of that array matters, so the state is one
// scalar.  The candidates' decodes and sums run batched on the GPU; the host
// walks the codewords in order resolving the stale reads; a codeword's final
// decode can be skipped in that walk whenever it provably repeats its chosen
// candidate's metric decode (same trajectory up to the shorter iteration cap),
// and otherwise the walk stops at the first codeword whose choice needs it,
// decodes what is resolved so far, and resumes (one extra round per such link).
int soft_receive(kml_ctx *c, const RecvIO &io, double var, int B, const double2 *hc, int nc, int &bp_slot) {
  const int S = c->code.cc_len / c->modem.bits;
  const size_t cc = (size_t)c->code.cc_len;
  const int K = c->code.K, M = c->code.M;
  const int mit = c->rc.metric_iter, max_iter = c->rc.max_iter;
  const double *cons = c->d_cons.as<double>();
  const size_t nB = (size_t)nc * B;
  HIPCHK(c, c->w_p0.ensure(sizeof(double) * cc * nB), "hipMalloc(p0)");
  HIPCHK(c, c->s_synm.ensure(sizeof(double) * (size_t)M * nB), "hipMalloc(syn)");
  HIPCHK(c, c->s_itm.ensure(sizeof(int32_t) * nB), "hipMalloc(iters)");
  HIPCHK(c, c->s_Lm.ensure(sizeof(double) * nB), "hipMalloc(L)");
  {
    Timer t(c, "demap", -1, (double)nB * S * (16.0 + 8.0 * c->modem.bits));
    kml::DemapDefer dd;
    TRY(demap_defer(c, 0, dd));
    HIPCHK(c, kml::launch_demap(c->modem.bits, cons, io.y, S, nc, hc, 1, nullptr, var, (int)nB, c->w_p0.as<double>(),
                                dd, c->stream),
           "demap candidates");
    t.stop();
  }
  kml::BpLaunch m;
  m.B = (int)nB;
  m.iter_count = mit;
  m.max_iter = max_iter;
  m.p0 = c->w_p0.as<double>();
  m.p0_stride = (long long)cc;
  m.syn = c->s_synm.as<double>();
  m.iters = c->s_itm.as<int32_t>();
  if (io.histogram) {
    HIPCHK(c, c->w_uh4.ensure(nB * K), "hipMalloc(uh4)");
    m.uu_hat = c->w_uh4.as<uint8_t>();
  }
  int mslot = 0;
  TRY(run_bp(c, m, mslot));
  {
    Timer t(c, "metric", -1, (double)nB * M * 8.0);
    HIPCHK(c, kml::launch_soft_sum(m.syn, M, m.iters, nullptr, (int)nB, c->s_Lm.as<double>(), c->stream), "soft sum");
    t.stop();
  }
  std::vector<int32_t> itm(nB);
  std::vector<double> Lm(nB);
  HIPCHK(c, hipMemcpyAsync(itm.data(), m.iters, sizeof(int32_t) * nB, hipMemcpyDeviceToHost, c->stream), "D2H");
  HIPCHK(c, hipMemcpyAsync(Lm.data(), c->s_Lm.p, sizeof(double) * nB, hipMemcpyDeviceToHost, c->stream), "D2H");
  TRY(sync(c));

  const long long T = std::max<long long>(1, c->rc.thread_num_blk);
  auto reset_at = [&](int b) { return io.sim && (b == 0 || (long long)((io.first_cw + (uint64_t)b) % (uint64_t)T) == 0); };
  double state = io.sim ? -INFINITY : c->soft_state;
  std::vector<int32_t> chosen(B, 0);
  std::vector<double> met((size_t)4 * B, 0.0);
  // candidates of codeword b against the incoming state; returns the state after them
  auto metrics_of = [&](int b, double in) {
    double cur = in;
    for (int i = 0; i < nc; i++) {
      const size_t e = (size_t)b * nc + i;
      if (itm[e] > 0) cur = Lm[e];
      met[(size_t)b * 4 + i] = std::fabs(cur);
    }
    int best = 0;
    for (int i = 1; i < nc; i++)
      if (met[(size_t)b * 4 + i] < met[(size_t)b * 4 + best]) best = i;
    chosen[b] = best;
    return cur;
  };

  int32_t *d_chosen = io.chosen;
  if (!d_chosen) {
    HIPCHK(c, c->s_sel.ensure(sizeof(int32_t) * B), "hipMalloc(sel)");
    d_chosen = c->s_sel.as<int32_t>();
  }
  double *d_met = io.met;
  if (!d_met) {
    HIPCHK(c, c->w_met.ensure(sizeof(double) * 4 * B), "hipMalloc(met)");
    d_met = c->w_met.as<double>();
  }

  if (io.histogram) {  // GetHistogramData: metric decodes only
    for (int b = 0; b < B; b++) {
      if (reset_at(b)) state = -INFINITY;
      state = metrics_of(b, state);
    }
    if (!io.sim) c->soft_state = state;
    HIPCHK(c, hipMemcpyAsync(d_chosen, chosen.data(), sizeof(int32_t) * B, hipMemcpyHostToDevice, c->stream), "H2D");
    HIPCHK(c, hipMemcpyAsync(d_met, met.data(), sizeof(double) * 4 * B, hipMemcpyHostToDevice, c->stream), "H2D");
    bp_slot = next_slot(c);
    unsigned long long *cnt = slot_ptr(c, bp_slot);
    HIPCHK(c, hipMemsetAsync(cnt, 0, sizeof(unsigned long long) * kml::CNT_N, c->stream), "memset");
    const uint8_t *last = c->w_uh4.as<uint8_t>() + (size_t)(nc - 1) * K;
    if (io.ref_bits)
      HIPCHK(c, kml::launch_count_packed(io.ref_bits, c->code.Kw, K, last, (long long)nc * K, B, io.cw_err, cnt,
                                         c->stream),
             "count");
    if (io.uh)
      HIPCHK(c, hipMemcpy2DAsync(io.uh, K, last, (size_t)nc * K, K, B, hipMemcpyDeviceToDevice, c->stream), "copy uh");
    return sync(c);
  }

  // final decodes, in rounds
  HIPCHK(c, c->s_synf.ensure(sizeof(double) * (size_t)M * B), "hipMalloc(syn final)");
  HIPCHK(c, c->s_itf.ensure(sizeof(int32_t) * B), "hipMalloc(iters final)");
  HIPCHK(c, c->s_Lf.ensure(sizeof(double) * B), "hipMalloc(L final)");
  HIPCHK(c, c->s_list.ensure(sizeof(int32_t) * B), "hipMalloc(list)");
  kml::BpLaunch a;
  a.iter_count = max_iter;
  a.max_iter = max_iter;
  a.uu_hat = io.uh;
  a.ret = io.ret;
  a.ref_bits = io.ref_bits;
  a.cw_err = io.cw_err;
  a.p0 = c->w_p0.as<double>();
  a.p0_stride = (long long)cc * nc;
  a.p0_sel = d_chosen;
  a.p0_sel_stride = (long long)cc;
  a.syn = c->s_synf.as<double>();
  a.iters = c->s_itf.as<int32_t>();
  a.cw_idx = c->s_list.as<int32_t>();
  bp_slot = next_slot(c);
  HIPCHK(c, hipMemsetAsync(slot_ptr(c, bp_slot), 0, sizeof(unsigned long long) * kml::CNT_N, c->stream), "memset");
  std::vector<int32_t> list;
  list.reserve(B);
  int cursor = 0;
  while (cursor < B) {
    const size_t first = list.size();
    bool unknown = false;
    int pend = -1;
    double pend_cur = 0.0;
    int b = cursor;
    for (; b < B; b++) {
      if (reset_at(b)) {
        state = -INFINITY;
        unknown = false;
      }
      const bool stale_first = itm[(size_t)b * nc] <= 0;
      if (stale_first && unknown) break;  // needs the pending final decode
      const double cur = metrics_of(b, unknown ? 0.0 : state);
      list.push_back(b);
      const int mc = itm[(size_t)b * nc + chosen[b]];
      // the final decode repeats the chosen candidate's metric decode when
      // both stop at the same iteration: converged before both caps, or equal caps
      const bool same = (mc < mit && mc <= max_iter) || mit == max_iter;
      if (same) {
        state = mc > 0 ? Lm[(size_t)b * nc + chosen[b]] : cur;
        unknown = false;
      } else {
        unknown = true;
        pend = b;
        pend_cur = cur;
      }
    }
    const int n = (int)(list.size() - first);
    HIPCHK(c, hipMemcpyAsync(d_chosen, chosen.data(), sizeof(int32_t) * B, hipMemcpyHostToDevice, c->stream), "H2D");
    HIPCHK(c, hipMemcpyAsync(c->s_list.as<int32_t>() + first, list.data() + first, sizeof(int32_t) * n,
                             hipMemcpyHostToDevice, c->stream),
           "H2D list");
    a.B = n;
    a.cw_idx = c->s_list.as<int32_t>() + first;
    int slot = 0;
    TRY(run_bp(c, a, slot, bp_slot));
    if (unknown && pend >= 0) {  // the last codeword's final decode sets the state
      const int32_t *pl = c->s_list.as<int32_t>() + first + (n - 1);
      HIPCHK(c, kml::launch_soft_sum(a.syn, M, a.iters, pl, 1, c->s_Lf.as<double>(), c->stream), "soft sum");
      int32_t itf = 0;
      double Lf = 0.0;
      HIPCHK(c, hipMemcpyAsync(&itf, a.iters + pend, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream), "D2H");
      HIPCHK(c, hipMemcpyAsync(&Lf, c->s_Lf.as<double>() + pend, sizeof(double), hipMemcpyDeviceToHost, c->stream),
             "D2H");
      TRY(sync(c));
      state = itf > 0 ? Lf : pend_cur;
    }
    cursor = b;
  }
  if (!io.sim) c->soft_state = state;
  HIPCHK(c, hipMemcpyAsync(d_met, met.data(), sizeof(double) * 4 * B, hipMemcpyHostToDevice, c->stream), "H2D");
  return sync(c);
}

}  // namespace

extern "C" {

int kml_abi_version(void) { return KML_ABI_VERSION; }

int kml_create(const char *config_toml, const char *data_dir, int device, kml_ctx **out) {
  if (!out || !config_toml) return KML_E_ARG;
  *out = nullptr;
  kml_ctx *c = new kml_ctx();
  c->device = device;
  std::string err;
  if (!kml::load_run_config(config_toml, data_dir ? data_dir : "", c->rc, err)) {
    c->err = err;
    *out = c;  // keep the context so kml_last_error can report
    return KML_E_IO;
  }
  int r = finish_create(c);
  *out = c;
  return r;
}

int kml_create_explicit(const char *matrix_file, const char *modem_file, int is5g, int active, int max_iter,
                        int metric_soft, int metric_iter, int device, kml_ctx **out) {
  if (!out || !matrix_file || !modem_file) return KML_E_ARG;
  kml_ctx *c = new kml_ctx();
  c->device = device;
  c->rc.matrix_file = matrix_file;
  c->rc.modem_file = modem_file;
  c->rc.is5g = is5g != 0;
  c->rc.active = active != 0;
  c->rc.max_iter = max_iter;
  c->rc.metric_soft = metric_soft != 0;
  c->rc.metric_iter = metric_iter;
  int r = finish_create(c);
  *out = c;
  return r;
}

void kml_destroy(kml_ctx *c) {
  if (!c) return;
  if (c->stream && c->device >= 0) {
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    drain_profile(c);
    kml::rccl_destroy(c->comm);
    c->comm = nullptr;
    c->w_comm.release();
    c->w_defer.release();
    c->w_ddefer.release();
    for (DBuf *b : {&c->d_graph, &c->d_cons, &c->d_arena, &c->d_queue, &c->d_gslots, &c->d_gsync, &c->d_gcch, &c->w_y, &c->w_h, &c->w_h4,
                    &c->w_hhat, &c->w_p0, &c->w_uu, &c->w_uh, &c->w_uh4, &c->w_cwerr, &c->w_ret, &c->w_cch, &c->w_syn, &c->w_sel, &c->w_met,
                    &c->w_pc, &c->w_cnt, &c->w_km, &c->s_synm, &c->s_synf, &c->s_itm, &c->s_itf, &c->s_Lm, &c->s_Lf, &c->s_list, &c->s_sel, &c->s_uu, &c->s_cc, &c->s_y, &c->s_h, &c->w_hc})
      b->release();
    hipStreamDestroy(c->stream);
    if (c->cstream) hipStreamDestroy(c->cstream);
  }
  delete c;
}

// context-free calls (kml_comm_unique_id) report through this thread's message
static thread_local std::string g_free_err = "null context";
const char *kml_last_error(const kml_ctx *c) { return c ? c->err.c_str() : g_free_err.c_str(); }

const char *kml_bp_kernel(const kml_ctx *c) { return c && c->bp_family ? c->bp_family : ""; }

int kml_dims(const kml_ctx *c, int32_t *d) {
  if (!c || !d) return KML_E_ARG;
  const kml::LdpcCode &L = c->code;
  d[KML_DIM_M] = L.M;
  d[KML_DIM_NCOL] = L.N;
  d[KML_DIM_K] = L.K;
  d[KML_DIM_CCLEN] = L.cc_len;
  d[KML_DIM_Z] = L.Z;
  d[KML_DIM_E] = L.E;
  d[KML_DIM_CHK] = L.chk;
  d[KML_DIM_MAXITER] = c->rc.max_iter;
  d[KML_DIM_BITS] = c->modem.bits;
  d[KML_DIM_KC] = c->modem.Kc;
  d[KML_DIM_S] = c->modem.bits ? L.cc_len / c->modem.bits : 0;
  kml::DevCode tmp{};
  tmp.E = L.E;
  tmp.N = L.N;
  d[KML_DIM_BP_LDS] = kml::bp_uses_lds(tmp) ? 1 : 0;
  d[KML_DIM_PART_G] = c->dc.pt_G;
  return KML_OK;
}

int kml_code_perm(const kml_ctx *c, int32_t *perm) {
  if (!c || !perm) return KML_E_ARG;
  memcpy(perm, c->code.perm.data(), sizeof(int32_t) * c->code.perm.size());
  return KML_OK;
}

int kml_code_graph(const kml_ctx *c, int32_t *rp, int32_t *rc, int32_t *cp, int32_t *cs) {
  if (!c) return KML_E_ARG;
  const kml::LdpcCode &L = c->code;
  if (rp) memcpy(rp, L.row_ptr.data(), 4 * L.row_ptr.size());
  if (rc) memcpy(rc, L.row_col.data(), 4 * L.row_col.size());
  if (cp) memcpy(cp, L.col_ptr.data(), 4 * L.col_ptr.size());
  if (cs) memcpy(cs, L.col_slot.data(), 4 * L.col_slot.size());
  return KML_OK;
}

int kml_constellation(const kml_ctx *c, double *pts) {
  if (!c || !pts) return KML_E_ARG;
  memcpy(pts, c->modem.pts.data(), sizeof(double) * c->modem.pts.size());
  return KML_OK;
}

int kml_encode(const kml_ctx *c, const uint8_t *uu, uint8_t *cc, int B) {
  if (!c || !uu || !cc || B < 0) return KML_E_ARG;
  for (int b = 0; b < B; b++) c->code.encode(uu + (size_t)b * c->code.K, cc + (size_t)b * c->code.cc_len);
  return KML_OK;
}

int kml_bp_decode(kml_ctx *c, const double *p0, int B, int iter_count, uint8_t *uu_hat, int32_t *ret, uint8_t *cc_hat,
                  double *syn, int flags) {
  call_begin(c);
  if (!c || !p0 || B < 0 || iter_count < 0) return fail(c, KML_E_ARG, "kml_bp_decode: bad argument");
  if (B == 0) return KML_OK;
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const kml::LdpcCode &L = c->code;
  const double *d_p0;
  TRY(stage_in(c, c->w_p0, p0, (size_t)B * L.cc_len, flags, d_p0));
  uint8_t *d_uh, *d_cch;
  int32_t *d_ret;
  double *d_syn;
  TRY(stage_out_ptr(c, c->w_uh, uu_hat, (size_t)B * L.K, flags, d_uh));
  TRY(stage_out_ptr(c, c->w_ret, ret, (size_t)B, flags, d_ret));
  TRY(stage_out_ptr(c, c->w_cch, cc_hat, (size_t)B * L.N, flags, d_cch));
  TRY(stage_out_ptr(c, c->w_syn, syn, (size_t)B * L.M, flags, d_syn));
  // syndrom_soft semantics: rows not rewritten keep the caller's values
  if (syn && !(flags & KML_DEVICE_PTRS))
    HIPCHK(c, hipMemcpyAsync(d_syn, syn, sizeof(double) * B * L.M, hipMemcpyHostToDevice, c->stream), "H2D syn");
  kml::BpLaunch a;
  a.B = B;
  a.iter_count = iter_count;
  a.max_iter = c->rc.max_iter;
  a.p0 = d_p0;
  a.p0_stride = L.cc_len;
  a.uu_hat = d_uh;
  a.ret = d_ret;
  a.cc_hat = d_cch;
  a.syn = d_syn;
  int slot;
  TRY(run_bp(c, a, slot));
  // the reference writes uu_hat (and cc_hat_) only inside its iteration loop
  // (binaryldpccodec.cc:177-216): with iter_count = 0 the kernels write
  // neither, and the caller's arrays stay as they were
  if (iter_count > 0) {
    TRY(copy_out(c, uu_hat, d_uh, (size_t)B * L.K, flags));
    TRY(copy_out(c, cc_hat, d_cch, (size_t)B * L.N, flags));
  }
  TRY(copy_out(c, ret, d_ret, (size_t)B, flags));
  TRY(copy_out(c, syn, d_syn, (size_t)B * L.M, flags));
  return sync(c);
}

int kml_demap(kml_ctx *c, const double *y, const double *h, double var, int B, double *p0, int flags) {
  call_begin(c);
  if (!c || !y || !h || !p0 || B < 0) return fail(c, KML_E_ARG, "kml_demap: bad argument");
  if (B == 0) return KML_OK;
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const int S = c->code.cc_len / c->modem.bits;
  const double *d_y, *d_h;
  TRY(stage_in(c, c->w_y, y, (size_t)B * S * 2, flags, d_y));
  TRY(stage_in(c, c->w_h, h, (size_t)B * 2, flags, d_h));
  double *d_p0;
  TRY(stage_out_ptr(c, c->w_p0, p0, (size_t)B * c->code.cc_len, flags, d_p0));
  Timer t(c, "demap", -1, (double)B * S * (16.0 + 8.0 * c->modem.bits));
  kml::DemapDefer dd;
  TRY(demap_defer(c, 0, dd));
  HIPCHK(c, kml::launch_demap(c->modem.bits, c->d_cons.as<double>(), reinterpret_cast<const double2 *>(d_y), S, 1,
                              reinterpret_cast<const double2 *>(d_h), 1, nullptr, var, B, d_p0, dd, c->stream),
         "demap");
  t.stop();
  TRY(copy_out(c, p0, d_p0, (size_t)B * c->code.cc_len, flags));
  return sync(c);
}

int kml_kmeans(kml_ctx *c, const double *y, int B, int iters, double *h_hat, double *h4, int flags) {
  call_begin(c);
  if (!c || !y || B < 0 || iters < 0) return fail(c, KML_E_ARG, "kml_kmeans: bad argument");
  if (B == 0) return KML_OK;
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const int S = c->code.cc_len / c->modem.bits;
  const double *d_y;
  TRY(stage_in(c, c->w_y, y, (size_t)B * S * 2, flags, d_y));
  double *d_hh, *d_h4;
  HIPCHK(c, c->w_hhat.ensure(sizeof(double2) * B), "hipMalloc");
  HIPCHK(c, c->w_h4.ensure(sizeof(double2) * 4 * B), "hipMalloc");
  d_hh = (h_hat && (flags & KML_DEVICE_PTRS)) ? h_hat : c->w_hhat.as<double>();
  d_h4 = (h4 && (flags & KML_DEVICE_PTRS)) ? h4 : c->w_h4.as<double>();
  const double *cons = c->d_cons.as<double>();
  HIPCHK(c, c->w_km.ensure(kml::kmeans_workspace_bytes(S, B)), "hipMalloc(kmeans)");
  Timer t(c, "kmeans", -1, (double)B * S * 16.0);
  HIPCHK(c, kml::launch_kmeans(c->modem.Kc, cons, cons + c->modem.pts.size(), reinterpret_cast<const double2 *>(d_y), S,
                               iters, B, reinterpret_cast<double2 *>(d_hh), reinterpret_cast<double2 *>(d_h4),
                               c->w_km.p, c->stream),
         "kmeans");
  t.stop();
  TRY(copy_out(c, h_hat, (const double *)d_hh, (size_t)B * 2, flags));
  TRY(copy_out(c, h4, (const double *)d_h4, (size_t)B * 8, flags));
  return sync(c);
}

int kml_kmeans_state(kml_ctx *c, const double *y, int B, int iters, double *clusters, int32_t *idx, int flags) {
  call_begin(c);
  if (!c || !y || B < 0 || iters < 0) return fail(c, KML_E_ARG, "kml_kmeans_state: bad argument");
  if (B == 0) return KML_OK;
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const int S = c->code.cc_len / c->modem.bits;
  const int Kc = c->modem.Kc;
  const double *d_y;
  TRY(stage_in(c, c->w_y, y, (size_t)B * S * 2, flags, d_y));
  HIPCHK(c, c->w_hhat.ensure(sizeof(double2) * B), "hipMalloc");
  HIPCHK(c, c->w_h4.ensure(sizeof(double2) * 4 * B), "hipMalloc");
  HIPCHK(c, c->w_h.ensure(sizeof(double2) * B), "hipMalloc");  // the final hatH
  double *d_cl;
  int32_t *d_idx;
  TRY(stage_out_ptr(c, c->w_met, clusters, (size_t)B * Kc * 2, flags, d_cl));
  TRY(stage_out_ptr(c, c->w_cwerr, idx, (size_t)B * S, flags, d_idx));
  const double *cons = c->d_cons.as<double>();
  HIPCHK(c, c->w_km.ensure(kml::kmeans_workspace_bytes(S, B)), "hipMalloc(kmeans)");
  Timer t(c, "kmeans", -1, (double)B * S * 16.0);
  HIPCHK(c, kml::launch_kmeans(Kc, cons, cons + c->modem.pts.size(), reinterpret_cast<const double2 *>(d_y), S, iters, B,
                               c->w_hhat.as<double2>(), c->w_h4.as<double2>(), c->w_km.p, c->stream,
                               c->w_h.as<double2>()),
         "kmeans");
  t.stop();
  HIPCHK(c, kml::launch_kmeans_state(Kc, cons, reinterpret_cast<const double2 *>(d_y), S, B, c->w_h.as<double2>(),
                                     reinterpret_cast<double2 *>(d_cl), d_idx, c->stream),
         "kmeans_state");
  TRY(copy_out(c, clusters, (const double *)d_cl, (size_t)B * Kc * 2, flags));
  TRY(copy_out(c, idx, (const int32_t *)d_idx, (size_t)B * S, flags));
  return sync(c);
}

// ---- MAT-file level 5 writer (KMeans::DumpToMat, src/kmeans.cc:99-109) ----
// What lab::Mat does through matio (lib/lab/src/mat.cc): Mat_CreateVer(...,
// MAT_FT_DEFAULT) = a level-5 file, each variable written uncompressed
// (MAT_COMPRESSION_NONE) as an n x 1 column: WriteVector(complex) ->
// mxDOUBLE_CLASS with the complex flag (real part, then imaginary part),
// WriteVector(int32) -> mxINT32_CLASS, WriteComplex -> a 1 x 1 complex double.
namespace {
struct MatOut {
  std::string buf;
  void raw(const void *p, size_t n) { buf.append(static_cast<const char *>(p), n); }
  void u32(uint32_t v) { raw(&v, 4); }
  void pad8() {
    while (buf.size() % 8) buf.push_back('\0');
  }
  // one data element: tag (type, bytes) + data, padded to 8 bytes
  void element(uint32_t type, const void *p, size_t n) {
    u32(type);
    u32((uint32_t)n);
    raw(p, n);
    pad8();
  }
  enum { miINT8 = 1, miINT32 = 5, miUINT32 = 6, miDOUBLE = 9, miMATRIX = 14 };
  enum { mxDOUBLE_CLASS = 6, mxINT32_CLASS = 12 };
  void matrix(const char *name, uint32_t cls, bool cplx, int rows, const void *re, const void *im, size_t elem) {
    MatOut body;
    const uint32_t flags[2] = {cls | (cplx ? 0x0800u : 0u), 0u};
    body.element(miUINT32, flags, sizeof(flags));
    const int32_t dims[2] = {rows, 1};
    body.element(miINT32, dims, sizeof(dims));
    body.element(miINT8, name, strlen(name));
    const uint32_t t = cls == mxINT32_CLASS ? miINT32 : miDOUBLE;
    body.element(t, re, (size_t)rows * elem);
    if (cplx) body.element(t, im, (size_t)rows * elem);
    u32(miMATRIX);
    u32((uint32_t)body.buf.size());
    raw(body.buf.data(), body.buf.size());
  }
  void complex_vec(const char *name, const double *z, int n) {  // z interleaved (re, im)
    std::vector<double> re(n), im(n);
    for (int i = 0; i < n; ++i) {
      re[i] = z[2 * i];
      im[i] = z[2 * i + 1];
    }
    matrix(name, mxDOUBLE_CLASS, true, n, re.data(), im.data(), sizeof(double));
  }
};
}  // namespace

int kml_kmeans_dump_mat(const char *path, const double *data, int S, const double *clusters, const int32_t *idx,
                        const double *constellations, int Kc, const double *append) {
  if (!path || !data || !clusters || !idx || !constellations || !append || S < 0 || Kc < 0) return KML_E_ARG;
  MatOut m;
  char hdr[128];
  memset(hdr, ' ', sizeof(hdr));
  const char *text = "MATLAB 5.0 MAT-file, Platform: GLNXA64, Created by: kmldpc_amd (KMeans::DumpToMat)";
  memcpy(hdr, text, strlen(text));
  memset(hdr + 116, 0, 8);  // subsystem data offset: none
  const uint16_t ver = 0x0100;
  memcpy(hdr + 124, &ver, 2);
  hdr[126] = 'I';  // written little-endian: reads back as "IM"
  hdr[127] = 'M';
  m.raw(hdr, sizeof(hdr));
  m.complex_vec("data", data, S);
  m.complex_vec("cluster", clusters, Kc);
  m.matrix("idx", MatOut::mxINT32_CLASS, false, S, idx, nullptr, sizeof(int32_t));
  m.complex_vec("constellations", constellations, Kc);
  m.complex_vec("hHats", append, 4);   // append[0..3]
  m.complex_vec("realH", append + 8, 1);  // append[4] (WriteComplex: 1 x 1)
  FILE *f = fopen(path, "wb");
  if (!f) return KML_E_IO;
  const bool ok = fwrite(m.buf.data(), 1, m.buf.size(), f) == m.buf.size();
  return (fclose(f) == 0 && ok) ? KML_OK : KML_E_IO;
}

namespace {
// Codewords per chunk of the host-buffer known-channel path (KML_HOST_CHUNK;
// 0 = one piece).
int host_chunk() {
  if (const char *e = getenv("KML_HOST_CHUNK")) return atoi(e);
  return 8192;
}

// kml_decode_frames with HOST buffers, in chunks: the frames of chunk i + 1
// cross PCIe on the copy stream while chunk i decodes on the context's stream
// (which waits on the upload's event), and chunk i's outputs come back before
// chunk i + 1 is launched.  Chunks decode in order on one stream, so every
// codeword sees what it sees in one call: the known-channel and hard-metric
// decodes have no cross-codeword state (the soft metric's stale syndrom_soft_
// has; its calls stay in one piece).  Only the transfers move.  chosen /
// metrics / h_hat are the blind path's outputs (NULL on the known path).
int decode_frames_chunked(kml_ctx *c, const double *y, const double *true_h, double snr, int B, uint8_t *uu_hat,
                          int32_t *chosen, double *metrics, int32_t *ret, double *h_hat, int CH) {
  const int S = c->code.cc_len / c->modem.bits, K = c->code.K;
  const size_t ycw = (size_t)S * 2;  // doubles per codeword
  HIPCHK(c, c->w_y.ensure((size_t)B * ycw * sizeof(double)), "hipMalloc(workspace)");
  if (true_h) HIPCHK(c, c->w_h.ensure((size_t)B * 2 * sizeof(double)), "hipMalloc(workspace)");
  HIPCHK(c, c->w_uh.ensure((size_t)B * K), "hipMalloc(workspace)");
  if (ret) HIPCHK(c, c->w_ret.ensure((size_t)B * sizeof(int32_t)), "hipMalloc(workspace)");
  if (chosen) HIPCHK(c, c->w_sel.ensure((size_t)B * sizeof(int32_t)), "hipMalloc(workspace)");
  if (metrics) HIPCHK(c, c->w_met.ensure((size_t)B * 4 * sizeof(double)), "hipMalloc(workspace)");
  if (h_hat) HIPCHK(c, c->w_hhat.ensure((size_t)B * 2 * sizeof(double)), "hipMalloc(workspace)");
  if (!c->cstream) HIPCHK(c, hipStreamCreateWithFlags(&c->cstream, hipStreamNonBlocking), "hipStreamCreate");
  const int n = (B + CH - 1) / CH;
  std::vector<hipEvent_t> ev(n, nullptr);
  int rc = KML_OK;
  auto upload = [&](int i) -> int {
    const size_t b0 = (size_t)i * CH, nb = std::min<size_t>(CH, B - b0);
    HIPCHK(c, hipEventCreateWithFlags(&ev[i], hipEventDisableTiming), "hipEventCreate");
    HIPCHK(c, hipMemcpyAsync(c->w_y.as<double>() + b0 * ycw, y + b0 * ycw, nb * ycw * sizeof(double),
                             hipMemcpyHostToDevice, c->cstream), "H2D");
    if (true_h)
      HIPCHK(c, hipMemcpyAsync(c->w_h.as<double>() + b0 * 2, true_h + b0 * 2, nb * 2 * sizeof(double),
                               hipMemcpyHostToDevice, c->cstream), "H2D");
    HIPCHK(c, hipEventRecord(ev[i], c->cstream), "hipEventRecord");
    return KML_OK;
  };
  rc = upload(0);
  for (int i = 0; i < n && rc == KML_OK; ++i) {
    const size_t b0 = (size_t)i * CH;
    const int nb = (int)std::min<size_t>(CH, B - b0);
    if (hipStreamWaitEvent(c->stream, ev[i], 0) != hipSuccess) {
      rc = fail(c, KML_E_HIP, "hipStreamWaitEvent");
      break;
    }
    RecvIO io;
    io.y = reinterpret_cast<const double2 *>(c->w_y.as<double>() + b0 * ycw);
    io.true_h = true_h ? reinterpret_cast<const double2 *>(c->w_h.as<double>() + b0 * 2) : nullptr;
    io.uh = c->w_uh.as<uint8_t>() + b0 * K;
    io.ret = ret ? c->w_ret.as<int32_t>() + b0 : nullptr;
    io.chosen = chosen ? c->w_sel.as<int32_t>() + b0 : nullptr;
    io.met = metrics ? c->w_met.as<double>() + b0 * 4 : nullptr;
    io.hhat = h_hat ? reinterpret_cast<double2 *>(c->w_hhat.as<double>() + b0 * 2) : nullptr;
    int slot;
    if ((rc = receive(c, io, snr, nb, slot)) != KML_OK) break;
    if (i + 1 < n && (rc = upload(i + 1)) != KML_OK) break;  // overlaps chunk i's decode
    if (hipMemcpyAsync(uu_hat + b0 * K, io.uh, (size_t)nb * K, hipMemcpyDeviceToHost, c->stream) != hipSuccess ||
        (ret && hipMemcpyAsync(ret + b0, io.ret, sizeof(int32_t) * nb, hipMemcpyDeviceToHost, c->stream) != hipSuccess) ||
        (chosen && hipMemcpyAsync(chosen + b0, io.chosen, sizeof(int32_t) * nb, hipMemcpyDeviceToHost, c->stream) !=
                       hipSuccess) ||
        (metrics && hipMemcpyAsync(metrics + b0 * 4, io.met, sizeof(double) * 4 * nb, hipMemcpyDeviceToHost,
                                   c->stream) != hipSuccess) ||
        (h_hat && hipMemcpyAsync(h_hat + b0 * 2, io.hhat, sizeof(double) * 2 * nb, hipMemcpyDeviceToHost, c->stream) !=
                      hipSuccess)) {
      rc = fail(c, KML_E_HIP, "D2H");
      break;
    }
  }
  if (rc != KML_OK) {  // leave no upload in flight into the workspaces
    hipStreamSynchronize(c->cstream);
    hipStreamSynchronize(c->stream);
  } else {
    rc = sync(c);
  }
  for (hipEvent_t e : ev)
    if (e) hipEventDestroy(e);
  return rc;
}
}  // namespace

int kml_comm_unique_id(uint8_t *id) {
  std::string err;
  if (!id) return KML_E_ARG;
  if (kml::rccl_unique_id(id, err) == 0) return KML_OK;
  g_free_err = "kml_comm_unique_id: " + err;
  return KML_E_UNSUP;
}

int kml_comm_init(kml_ctx *c, const uint8_t *id, int world, int rank) {
  call_begin(c);
  if (!c || !id || world < 1 || rank < 0 || rank >= world) return fail(c, KML_E_ARG, "kml_comm_init: bad argument");
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  if (c->comm) return fail(c, KML_E_ARG, "kml_comm_init: the context already has a communicator");
  std::string err;
  c->comm = kml::rccl_init(id, world, rank, err);
  return c->comm ? KML_OK : fail(c, KML_E_UNSUP, err);
}

int kml_comm_size(const kml_ctx *c) { return c ? kml::rccl_size(c->comm) : 0; }

namespace {
int comm_allreduce(kml_ctx *c, void *vals, int n, bool f64) {
  call_begin(c);
  if (!c || (!vals && n > 0) || n < 0) return fail(c, KML_E_ARG, "kml_comm_allreduce: bad argument");
  if (!c->comm) return fail(c, KML_E_ARG, "kml_comm_allreduce: no communicator (kml_comm_init)");
  if (n == 0) return KML_OK;
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const size_t bytes = (size_t)n * 8;
  HIPCHK(c, c->w_comm.ensure(bytes), "hipMalloc(comm)");
  HIPCHK(c, hipMemcpyAsync(c->w_comm.p, vals, bytes, hipMemcpyHostToDevice, c->stream), "H2D");
  std::string err;
  if (kml::rccl_allreduce(c->comm, c->w_comm.p, (size_t)n, f64, c->stream, err) != 0) return fail(c, KML_E_HIP, err);
  HIPCHK(c, hipMemcpyAsync(vals, c->w_comm.p, bytes, hipMemcpyDeviceToHost, c->stream), "D2H");
  HIPCHK(c, hipStreamSynchronize(c->stream), "hipStreamSynchronize");
  return KML_OK;
}
}  // namespace

int kml_comm_allreduce_u64(kml_ctx *c, uint64_t *vals, int n) { return comm_allreduce(c, vals, n, false); }
int kml_comm_allreduce_f64(kml_ctx *c, double *vals, int n) { return comm_allreduce(c, vals, n, true); }

int kml_debug_inject_abort(kml_ctx *c, int nth) {
  call_begin(c);
  if (!c) return KML_E_ARG;
  c->inject_fail = nth == -2;
  c->inject_abort = nth == -2 ? 0 : nth;
  return KML_OK;
}

int kml_decode_frames(kml_ctx *c, const double *y, const double *true_h, double snr, int B, uint8_t *uu_hat,
                      int32_t *chosen, double *metrics, int32_t *ret, double *h_hat, int flags) {
  call_begin(c);
  if (!c || !y || !uu_hat || B < 0) return fail(c, KML_E_ARG, "kml_decode_frames: bad argument");
  if (B == 0) return KML_OK;
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  if (!(flags & (KML_DEVICE_PTRS | KML_HISTOGRAM)) && (true_h || !c->rc.metric_soft)) {
    const int CH = host_chunk();
    if (CH > 0 && B > CH) {
      if (!true_h) return decode_frames_chunked(c, y, nullptr, snr, B, uu_hat, chosen, metrics, ret, h_hat, CH);
      if (chosen) memset(chosen, 0, sizeof(int32_t) * B);  // single candidate (kmcodec.cc:66-67)
      if (metrics) memset(metrics, 0, sizeof(double) * 4 * B);
      if (h_hat) memset(h_hat, 0, sizeof(double) * 2 * B);
      return decode_frames_chunked(c, y, true_h, snr, B, uu_hat, nullptr, nullptr, ret, nullptr, CH);
    }
  }
  const int S = c->code.cc_len / c->modem.bits;
  const double *d_y, *d_h = nullptr;
  TRY(stage_in(c, c->w_y, y, (size_t)B * S * 2, flags, d_y));
  if (true_h) TRY(stage_in(c, c->w_h, true_h, (size_t)B * 2, flags, d_h));
  uint8_t *d_uh;
  int32_t *d_ch, *d_ret;
  double *d_met, *d_hh;
  TRY(stage_out_ptr(c, c->w_uh, uu_hat, (size_t)B * c->code.K, flags, d_uh));
  TRY(stage_out_ptr(c, c->w_sel, chosen, (size_t)B, flags, d_ch));
  TRY(stage_out_ptr(c, c->w_met, metrics, (size_t)B * 4, flags, d_met));
  TRY(stage_out_ptr(c, c->w_ret, ret, (size_t)B, flags, d_ret));
  TRY(stage_out_ptr(c, c->w_hhat, h_hat, (size_t)B * 2, flags, d_hh));
  int slot;
  RecvIO io;
  io.y = reinterpret_cast<const double2 *>(d_y);
  io.true_h = reinterpret_cast<const double2 *>(d_h);
  io.uh = d_uh;
  io.chosen = d_ch;
  io.met = d_met;
  io.ret = d_ret;
  io.hhat = reinterpret_cast<double2 *>(d_hh);
  io.histogram = (flags & KML_HISTOGRAM) != 0;
  TRY(receive(c, io, snr, B, slot));
  if (true_h && !io.histogram) {  // single candidate: chosen = 0, metrics unset (kmcodec.cc:66-67)
    if (chosen && !(flags & KML_DEVICE_PTRS)) memset(chosen, 0, sizeof(int32_t) * B);
    if (metrics && !(flags & KML_DEVICE_PTRS)) memset(metrics, 0, sizeof(double) * 4 * B);
    if (h_hat && !(flags & KML_DEVICE_PTRS)) memset(h_hat, 0, sizeof(double) * 2 * B);
  } else {
    TRY(copy_out(c, chosen, d_ch, (size_t)B, flags));
    TRY(copy_out(c, metrics, d_met, (size_t)B * 4, flags));
    if (true_h) {
      if (h_hat && !(flags & KML_DEVICE_PTRS)) memset(h_hat, 0, sizeof(double) * 2 * B);
    } else {
      TRY(copy_out(c, h_hat, d_hh, (size_t)B * 2, flags));
    }
  }
  TRY(copy_out(c, uu_hat, d_uh, (size_t)B * c->code.K, flags));
  if (io.histogram) {  // no final decode: no BP return value
    if (ret && !(flags & KML_DEVICE_PTRS)) memset(ret, 0, sizeof(int32_t) * B);
  } else {
    TRY(copy_out(c, ret, d_ret, (size_t)B, flags));
  }
  return sync(c);
}

int kml_decode_candidates(kml_ctx *c, const double *y, const double *h_hats, int nc, double snr, int B,
                          uint8_t *uu_hat, int32_t *chosen, double *metrics, int32_t *ret, int flags) {
  call_begin(c);
  if (!c || !y || !h_hats || !uu_hat || B < 0 || nc < 1 || nc > 4)
    return fail(c, KML_E_ARG, "kml_decode_candidates: bad argument (need 1 <= nc <= 4)");
  // one estimate: Decoder computes no metric (kmcodec.cc:66-67); GetHistogramData
  // (kmcodec.cc:75-79, KML_HISTOGRAM) computes that candidate's metric, as the
  // known-channel histogram path of kml_decode_frames does
  if (nc == 1) return kml_decode_frames(c, y, h_hats, snr, B, uu_hat, chosen, metrics, ret, nullptr, flags);
  if (B == 0) return KML_OK;
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const int S = c->code.cc_len / c->modem.bits;
  const double *d_y, *d_hc;
  TRY(stage_in(c, c->w_y, y, (size_t)B * S * 2, flags, d_y));
  TRY(stage_in(c, c->w_hc, h_hats, (size_t)B * nc * 2, flags, d_hc));
  uint8_t *d_uh;
  int32_t *d_ch, *d_ret;
  double *d_met;
  TRY(stage_out_ptr(c, c->w_uh, uu_hat, (size_t)B * c->code.K, flags, d_uh));
  TRY(stage_out_ptr(c, c->w_sel, chosen, (size_t)B, flags, d_ch));
  TRY(stage_out_ptr(c, c->w_met, metrics, (size_t)B * 4, flags, d_met));
  TRY(stage_out_ptr(c, c->w_ret, ret, (size_t)B, flags, d_ret));
  int slot;
  RecvIO io;
  io.y = reinterpret_cast<const double2 *>(d_y);
  io.cand = reinterpret_cast<const double2 *>(d_hc);
  io.ncand = nc;
  io.uh = d_uh;
  io.chosen = d_ch;
  io.met = d_met;
  io.ret = d_ret;
  io.histogram = (flags & KML_HISTOGRAM) != 0;
  TRY(receive(c, io, snr, B, slot));
  TRY(copy_out(c, chosen, d_ch, (size_t)B, flags));
  TRY(copy_out(c, metrics, d_met, (size_t)B * 4, flags));
  TRY(copy_out(c, uu_hat, d_uh, (size_t)B * c->code.K, flags));
  if (io.histogram) {
    if (ret && !(flags & KML_DEVICE_PTRS)) memset(ret, 0, sizeof(int32_t) * B);
  } else {
    TRY(copy_out(c, ret, d_ret, (size_t)B, flags));
  }
  return sync(c);
}

int kml_count_errors(kml_ctx *c, const uint8_t *uu, const uint8_t *uu_hat, int B, uint64_t *counters, int flags) {
  call_begin(c);
  if (!c || !uu || !uu_hat || !counters || B < 0) return fail(c, KML_E_ARG, "kml_count_errors: bad argument");
  if (B == 0) return KML_OK;
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const size_t n = (size_t)B * c->code.K;
  const uint8_t *d_uu, *d_uh;
  TRY(stage_in(c, c->w_uu, uu, n, flags, d_uu));
  TRY(stage_in(c, c->w_uh, uu_hat, n, flags, d_uh));
  HIPCHK(c, c->w_cnt.ensure(sizeof(unsigned long long) * kml::CNT_N), "hipMalloc");
  HIPCHK(c, hipMemsetAsync(c->w_cnt.p, 0, sizeof(unsigned long long) * kml::CNT_N, c->stream), "memset");
  HIPCHK(c, kml::launch_count_bytes(d_uu, d_uh, c->code.K, B, c->w_cnt.as<unsigned long long>(), c->stream), "count");
  unsigned long long h[kml::CNT_N];
  HIPCHK(c, hipMemcpyAsync(h, c->w_cnt.p, sizeof(h), hipMemcpyDeviceToHost, c->stream), "D2H");
  TRY(sync(c));
  for (int i = 0; i < 4; i++) counters[i] += h[i];
  return KML_OK;
}

int kml_sim_generate(kml_ctx *c, double snr, uint64_t seed, uint64_t first_cw, int B) {
  call_begin(c);
  if (!c || B < 0) return fail(c, KML_E_ARG, "kml_sim_generate: bad argument");
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const kml::LdpcCode &L = c->code;
  const int S = L.cc_len / c->modem.bits;
  const int Cw = (L.cc_len + 63) / 64;
  HIPCHK(c, c->s_uu.ensure(sizeof(uint64_t) * (size_t)B * L.Kw), "hipMalloc(sim uu)");
  HIPCHK(c, c->s_cc.ensure(sizeof(uint64_t) * (size_t)B * Cw), "hipMalloc(sim cc)");
  HIPCHK(c, c->s_y.ensure(sizeof(double2) * (size_t)B * S), "hipMalloc(sim y)");
  HIPCHK(c, c->s_h.ensure(sizeof(double2) * (size_t)B), "hipMalloc(sim h)");
  double var, sigma, ns;
  kml::channel_constants(snr, var, sigma, ns);
  kml::FrameLaunch f;
  f.B = B;
  f.seed = seed;
  f.first_cw = first_cw;
  f.noise_scale = ns;
  f.uu_bits = c->s_uu.as<uint64_t>();
  f.cc_bits = c->s_cc.as<uint64_t>();
  f.y = c->s_y.as<double2>();
  f.h = c->s_h.as<double2>();
  Timer t(c, "framegen", -1, 0.0);
  HIPCHK(c, kml::launch_framegen(c->dc, c->modem.bits, c->d_cons.as<double>(), f, c->stream), "framegen");
  t.stop();
  c->sim_B = B;
  c->sim_snr = snr;
  c->sim_first = first_cw;
  return sync(c);
}

namespace {
int sim_receive(kml_ctx *c, double snr, int blind, bool histogram, int &slot) {
  RecvIO io;
  io.y = c->s_y.as<double2>();
  io.true_h = blind ? nullptr : c->s_h.as<double2>();
  io.ref_bits = c->s_uu.as<uint64_t>();
  HIPCHK(c, c->w_cwerr.ensure(sizeof(int32_t) * (size_t)c->sim_B), "hipMalloc(cw_err)");
  io.cw_err = c->w_cwerr.as<int32_t>();
  io.histogram = histogram;
  io.sim = true;
  io.first_cw = c->sim_first;
  if (histogram) {
    HIPCHK(c, c->w_met.ensure(sizeof(double) * 4 * (size_t)c->sim_B), "hipMalloc(met)");
    io.met = c->w_met.as<double>();
  }
  return receive(c, io, snr, c->sim_B, slot);
}
}  // namespace

int kml_sim_decode(kml_ctx *c, double snr, int blind, uint64_t *counters, int do_sync) {
  call_begin(c);
  if (!c) return KML_E_ARG;
  if (!do_sync && counters) return fail(c, KML_E_ARG, "counters need sync != 0");
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const int B = c->sim_B;
  if (B == 0) return KML_OK;
  int slot = 0;
  TRY(sim_receive(c, snr, blind, false, slot));
  if (counters) {
    unsigned long long h[kml::CNT_N];
    HIPCHK(c, hipMemcpyAsync(h, slot_ptr(c, slot), sizeof(h), hipMemcpyDeviceToHost, c->stream), "D2H");
    TRY(sync(c));
    for (int i = 0; i < kml::CNT_N; i++) counters[i] = h[i];
  }
  return KML_OK;
}

int kml_sim_decode_ex(kml_ctx *c, double snr, int blind, int histogram, int32_t *cw_err, double *metrics,
                      uint64_t *counters) {
  call_begin(c);
  if (!c) return KML_E_ARG;
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const int B = c->sim_B;
  if (B == 0) {
    if (counters) memset(counters, 0, sizeof(uint64_t) * kml::CNT_N);
    return KML_OK;
  }
  int slot = 0;
  TRY(sim_receive(c, snr, blind, histogram != 0, slot));
  unsigned long long h[kml::CNT_N];
  HIPCHK(c, hipMemcpyAsync(h, slot_ptr(c, slot), sizeof(h), hipMemcpyDeviceToHost, c->stream), "D2H");
  if (cw_err)
    HIPCHK(c, hipMemcpyAsync(cw_err, c->w_cwerr.p, sizeof(int32_t) * B, hipMemcpyDeviceToHost, c->stream), "D2H");
  if (metrics) {
    if (histogram)
      HIPCHK(c, hipMemcpyAsync(metrics, c->w_met.p, sizeof(double) * 4 * B, hipMemcpyDeviceToHost, c->stream), "D2H");
    else
      memset(metrics, 0, sizeof(double) * 4 * B);
  }
  TRY(sync(c));
  if (counters)
    for (int i = 0; i < kml::CNT_N; i++) counters[i] = h[i];
  return KML_OK;
}

int kml_run_config(const kml_ctx *c, double *f, int64_t *n) {
  if (!c) return KML_E_ARG;
  const kml::RunConfig &r = c->rc;
  if (f) {
    f[0] = r.min_snr;
    f[1] = r.max_snr;
    f[2] = r.step_snr;
  }
  if (n) {
    n[0] = r.max_err_blk;
    n[1] = r.max_num_blk;
    n[2] = r.thread_num_blk;
    n[3] = r.known_h ? 1 : 0;
    n[4] = r.is5g ? 1 : 0;
    n[5] = r.metric_soft ? 1 : 0;
    n[6] = r.metric_iter;
    n[7] = r.histogram ? 1 : 0;
    n[8] = r.max_iter;
    n[9] = r.active ? 1 : 0;
  }
  return KML_OK;
}

int kml_sync(kml_ctx *c) {
  call_begin(c);
  if (!c) return KML_E_ARG;
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  return sync(c);
}

int kml_sim_load(kml_ctx *c, double snr, const uint8_t *uu, const double *y, const double *h, int B,
                 uint64_t first_cw) {
  call_begin(c);
  if (!c || B < 0 || (B > 0 && (!uu || !y || !h))) return fail(c, KML_E_ARG, "kml_sim_load: bad argument");
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const kml::LdpcCode &L = c->code;
  const int S = L.cc_len / c->modem.bits;
  HIPCHK(c, c->s_uu.ensure(sizeof(uint64_t) * (size_t)std::max(B, 1) * L.Kw), "hipMalloc(sim uu)");
  HIPCHK(c, c->s_y.ensure(sizeof(double2) * (size_t)std::max(B, 1) * S), "hipMalloc(sim y)");
  HIPCHK(c, c->s_h.ensure(sizeof(double2) * (size_t)std::max(B, 1)), "hipMalloc(sim h)");
  TRY(sync(c));
  // source bits packed as the frame generator writes them: bit i of word i/64
  std::vector<uint64_t> w((size_t)B * L.Kw, 0);
  for (int b = 0; b < B; b++)
    for (int i = 0; i < L.K; i++)
      if (uu[(size_t)b * L.K + i]) w[(size_t)b * L.Kw + (i >> 6)] |= 1ull << (i & 63);
  if (B > 0) {
    HIPCHK(c, hipMemcpy(c->s_uu.p, w.data(), w.size() * 8, hipMemcpyHostToDevice), "H2D");
    HIPCHK(c, hipMemcpy(c->s_y.p, y, sizeof(double2) * (size_t)B * S, hipMemcpyHostToDevice), "H2D");
    HIPCHK(c, hipMemcpy(c->s_h.p, h, sizeof(double2) * (size_t)B, hipMemcpyHostToDevice), "H2D");
  }
  c->sim_B = B;
  c->sim_snr = snr;
  c->sim_first = first_cw;
  return KML_OK;
}

int kml_sim_frames(kml_ctx *c, uint8_t *uu, double *y, double *h) {
  call_begin(c);
  if (!c) return KML_E_ARG;
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const kml::LdpcCode &L = c->code;
  const int B = c->sim_B, S = L.cc_len / c->modem.bits;
  TRY(sync(c));
  if (uu) {
    std::vector<uint64_t> w((size_t)B * L.Kw);
    HIPCHK(c, hipMemcpy(w.data(), c->s_uu.p, w.size() * 8, hipMemcpyDeviceToHost), "D2H");
    for (int b = 0; b < B; b++)
      for (int i = 0; i < L.K; i++) uu[(size_t)b * L.K + i] = (w[(size_t)b * L.Kw + (i >> 6)] >> (i & 63)) & 1;
  }
  if (y) HIPCHK(c, hipMemcpy(y, c->s_y.p, sizeof(double2) * (size_t)B * S, hipMemcpyDeviceToHost), "D2H");
  if (h) HIPCHK(c, hipMemcpy(h, c->s_h.p, sizeof(double2) * (size_t)B, hipMemcpyDeviceToHost), "D2H");
  return KML_OK;
}

int kml_prof_enable(kml_ctx *c, int on) {
  call_begin(c);
  if (!c) return KML_E_ARG;
  c->prof = on != 0;
  return KML_OK;
}

int kml_prof_reset(kml_ctx *c) {
  call_begin(c);
  if (!c) return KML_E_ARG;
  drain_profile(c);
  c->stats.clear();
  return KML_OK;
}

int kml_prof_read_flops(kml_ctx *c, const char *stage, double *alg_flops) {
  call_begin(c);
  if (!c || !stage || !alg_flops) return KML_E_ARG;
  if (c->device >= 0) hipSetDevice(c->device);
  drain_profile(c);
  auto it = c->stats.find(stage);
  *alg_flops = it != c->stats.end() ? it->second.flops : 0.0;
  return KML_OK;
}

int kml_prof_read(kml_ctx *c, const char *stage, int64_t *launches, double *total_ms, double *alg_bytes) {
  call_begin(c);
  if (!c || !stage) return KML_E_ARG;
  if (c->device >= 0) hipSetDevice(c->device);
  drain_profile(c);
  Stat s;
  auto it = c->stats.find(stage);
  if (it != c->stats.end()) s = it->second;
  if (launches) *launches = s.launches;
  if (total_ms) *total_ms = s.ms;
  if (alg_bytes) *alg_bytes = s.bytes;
  return KML_OK;
}

int kml_ref_frames(const kml_ctx *c, int64_t *state, double snr, int n, uint8_t *uu, double *true_h, double *y) {
  if (!c || !state || n < 0 || (n > 0 && (!uu || !true_h || !y))) return KML_E_ARG;
  return kml::ref_frames(c->code, c->modem, state, snr, n, uu, true_h, y);
}

int kml_log_probe(kml_ctx *c, const double *in, int n, double *out) {
  call_begin(c);
  if (!c || !in || !out || n < 0) return KML_E_ARG;
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const double *d_in;
  TRY(stage_in(c, c->w_y, in, (size_t)n, 0, d_in));
  HIPCHK(c, c->w_p0.ensure(sizeof(double) * (size_t)n), "hipMalloc");
  HIPCHK(c, kml::launch_log_probe(d_in, n, c->w_p0.as<double>(), c->stream), "probe");
  TRY(copy_out(c, out, (const double *)c->w_p0.as<double>(), (size_t)n, 0));
  return sync(c);
}

int kml_math_probe(kml_ctx *c, const double *in, int n, double *out) {
  call_begin(c);
  if (!c || !in || !out || n < 0) return KML_E_ARG;
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const double *d_in;
  TRY(stage_in(c, c->w_y, in, (size_t)n * 4, 0, d_in));
  HIPCHK(c, c->w_p0.ensure(sizeof(double) * 4 * (size_t)n), "hipMalloc");
  HIPCHK(c, kml::launch_math_probe(d_in, n, c->w_p0.as<double>(), c->stream), "probe");
  TRY(copy_out(c, out, (const double *)c->w_p0.as<double>(), (size_t)n * 4, 0));
  return sync(c);
}

int kml_div_probe(kml_ctx *c, const double *in, int n, double *out) {
  call_begin(c);
  if (!c || !in || !out || n < 0) return KML_E_ARG;
  TRY(need_gpu(c));
  HIPCHK(c, hipSetDevice(c->device), "hipSetDevice");
  const double *d_in;
  TRY(stage_in(c, c->w_y, in, (size_t)n * 3, 0, d_in));
  HIPCHK(c, c->w_p0.ensure(sizeof(double) * 12 * (size_t)n), "hipMalloc");
  HIPCHK(c, kml::launch_div_probe(d_in, n, c->w_p0.as<double>(), c->stream), "div probe");
  TRY(copy_out(c, out, (const double *)c->w_p0.as<double>(), (size_t)n * 12, 0));
  return sync(c);
}

}  // extern "C"
