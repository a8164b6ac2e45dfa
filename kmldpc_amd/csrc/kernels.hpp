// kernels.hpp — launch interfaces of the gfx950 kernels (host-visible).
//
// Layouts in HBM (B = codewords in the batch, codeword index slowest):
//   y       [B][S] double2      received symbols
//   h       [B] double2         per-codeword channel (true or estimated)
//   p0      [B][cc_len] double  P(bit = 0) from the demapper (decoder input)
//   uu_bits [B][Kw] u64         reference info bits, little-endian bit order
//   cc_bits [B][Cw] u64         transmitted codeword bits
//   uu_hat  [B][K] u8           decoded info bits (optional)
// Decoder message state never leaves the chip for N <= ~9k edges: it lives in
// LDS as one 16-byte slot per edge (see bp.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "layout.hpp"  // kIrrThreads, kIrrVnPairMax, kIrrCnPairMax

namespace kml {

// Device-resident code description (uploaded once per context).
struct DevCode {
  const int32_t *row_ptr, *row_col, *col_ptr, *col_slot, *vn_order, *cn_order;
  const uint64_t *enc_info;
  int M, N, E, K, cc_len, punct, info_off, chk, Kw, dv_max, dc_max, is5g, active;
  int regular;  // every column has degree dv_max and every row dc_max
  int irr_ok;   // column degrees in [1, 9] and row degrees in [2, 10] (bp_irregular.hip)
  // Round plan of bp_irregular.hip (layout.hpp IrregularPlan); null when none fits.
  const int32_t *irr_vn, *irr_cn, *irr_cn_base, *irr_col_slot;
  int irr_slots;
  // LDS placement plan of bp_regular.hip (layout.hpp); null when the code does
  // not take that kernel.  vn_order then holds the planned column order.
  const int32_t *reg_c2v;  // aligned with col_slot: byte offset of the c2v message
  const int32_t *reg_pos;  // column -> position (index into the kernel's hard-decision bytes)
  // Partition plan of the partitioned cooperative kernel (layout.hpp
  // PartitionPlan); null / 0 when the code does not take it.
  const int32_t *pt_vn, *pt_cn, *pt_pos, *pt_vaddr, *pt_xr, *pt_xr_ptr, *pt_xc, *pt_xc_ptr;
  const int32_t *pt_vx, *pt_rx;  // tagged exchange: mailbox index per column edge, per-row (first x, cut mask)
  int pt_G, pt_ncut, pt_mirror;
  int pt_pairs;                // every member receives cut-edge messages from every other member
  int pt_xr_n[8], pt_xc_n[8];  // exchange-list lengths per member (host copy, launch checks)
};

// Counter block in device memory (uint64):
enum {
  CNT_ERR_BIT = 0,
  CNT_ERR_BLK = 1,
  CNT_TOT_BIT = 2,
  CNT_TOT_BLK = 3,
  CNT_VN_PHASES = 4,
  CNT_CN_PHASES = 5,
  CNT_CONVERGED = 6,
  CNT_REDONE = 7,  // FAST decodes redone on the exact path (an unproven quotient, exact_div.hpp)
  CNT_N = 8
};

struct BpLaunch {
  int B = 0;
  int iter_count = 0, max_iter = 0;
  const double *p0 = nullptr;
  long long p0_stride = 0;       // doubles between codewords
  const int32_t *p0_sel = nullptr;  // optional per-codeword candidate: p0 += sel*p0_sel_stride
  long long p0_sel_stride = 0;
  uint8_t *uu_hat = nullptr;     // [B][K]
  int32_t *ret = nullptr;        // [B]  BinaryLDPCCodec::Decoder return value
  uint8_t *cc_hat = nullptr;     // [B][N]
  double *syn = nullptr;         // [B][M] syndrom_soft (written by CN phases only)
  int32_t *parity_cnt = nullptr; // [B] unsatisfied checks of the final cc_hat
  const uint64_t *ref_bits = nullptr;  // [B][Kw] for error counting
  unsigned long long *counters = nullptr;  // [CNT_N]
  int32_t *cw_err = nullptr;     // [B] error bits per codeword vs ref_bits (stop-rule prefix)
  int32_t *iters = nullptr;      // [B] CN phases run (= iter of the reference loop)
  // Entry e of the launch decodes codeword cw_idx[e] (NULL: e); every
  // per-codeword array above is indexed by the codeword, B counts entries.
  const int32_t *cw_idx = nullptr;
  const unsigned *B_dev = nullptr;  // when set, the entry count is *B_dev (<= B), read on the device
  // partitioned kernel's tagged launch: codewords it leaves to the barrier-exchange launch
  int32_t *defer_idx = nullptr;
  unsigned *defer_cnt = nullptr;
  // Cooperative global-slot kernel (bp_coop.hip): per-group sync blocks
  // (bp_coop_sync_bytes) and per-group hard-decision bytes (groups x N).
  void *gsync = nullptr;
  uint8_t *gcch = nullptr;
  double2 *gslots = nullptr;     // global slot scratch when E*16 exceeds LDS
  long long gslots_cap = 0;      // number of double2 available
  unsigned int *queue = nullptr; // 4-byte device dequeue counter (zeroed by the launcher)
  // Cooperative kernels: clear the abort word before the launch.  The caller
  // clears it only for the first launch after the last check (capi.cpp sync),
  // so a timeout in an earlier launch of the same API call stays visible.
  bool reset_abort = true;
  // Fused demap (bp_regular.hip only, bp_regular_fuses_demap): when sym_y is
  // set, p0 is ignored and each codeword's P0 is computed in the kernel's
  // prologue from y[B][S] and the known channel h[B] (demap_common.hpp).
  const double2 *sym_y = nullptr;
  const double2 *sym_h = nullptr;     // h of codeword cw: sym_h[cw * sym_h_stride + (sym_h_sel ? sym_h_sel[cw] : 0)]
  int sym_h_stride = 1;
  const int32_t *sym_h_sel = nullptr;  // chosen candidate (blind path)
  const double *sym_cons = nullptr;  // the normalised constellation, 2 << bits doubles
  double sym_var = 0;
  int sym_bits = 0;
};

// FAST-path mode of a BP launch: bit 0 = FAST division allowed (column degree
// <= kFastMaxColumnDegree, and not KML_NO_FAST=1: every codeword on the
// exact path); bit 1 = KML_FORCE_REDO=1 (tests: every FAST decode is treated
// as suspect and redone on the exact path, exercising the redo machinery).
int bp_fast_mode(const DevCode &c);
hipError_t launch_bp_regular(const DevCode &c, const BpLaunch &a, hipStream_t s);
// Can the regular kernel compute P0 itself (BpLaunch::sym_y) for this code and modem?
bool bp_regular_fuses_demap(const DevCode &c, int bits);
hipError_t launch_bp_irregular(const DevCode &c, const BpLaunch &a, hipStream_t s);
// Cooperative kernel for regular codes whose slots exceed the LDS: groups of
// workgroups on one XCD share a codeword.  0 groups = not applicable.
int bp_coop_groups(const DevCode &c);
size_t bp_coop_sync_bytes(int groups);
hipError_t launch_bp_coop(const DevCode &c, const BpLaunch &a, hipStream_t s);
// Group size of the partitioned cooperative kernel (0: not used); host-side,
// decides whether upload_code builds the partition plan.
int bp_part_group_size(int N, int M, int E, int dv_max, int dc_max, int regular);
// Does a partition plan (cut edges, most mirror slots of a member, longest
// exchange list) fit the partitioned kernel's LDS, scratch and tilings?
bool part_plan_fits(int G, int N, int M, int E, int ncut, int mirror_max, int xmax);
// Name of the cooperative kernel launch_bp_coop runs for this code.
const char *bp_coop_family(const DevCode &c);
bool bp_coop_aborted(const BpLaunch &a, int groups, hipStream_t s, unsigned *why = nullptr);
// Test hook: set the abort word on the stream, as a timed-out group barrier would.
hipError_t bp_coop_raise_abort(const BpLaunch &a, int groups, hipStream_t s);
// Threads per workgroup of the regular kernel for this code shape, 0 if it does
// not apply (host-side; decides whether upload_code builds the LDS plan).
int bp_regular_threads(int N, int M, int E, int dv_max, int dc_max, int regular);
// family (optional) receives the name of the kernel that was launched.
hipError_t launch_bp(const DevCode &c, const BpLaunch &a, hipStream_t s, const char **err,
                     const char **family = nullptr);
// Workspace the BP launcher needs in global-slot mode (double2 elements).
long long bp_gslots_needed(const DevCode &c);
bool bp_uses_lds(const DevCode &c);

// The FAST demappers' defer list (demap.hip): symbol indices (launch_demap,
// any cap; past it the exact pass scans for the sentinel) or codewords
// (launch_cand_metric, cap >= B), and their device-side count.
struct DemapDefer {
  int32_t *idx = nullptr;
  unsigned *cnt = nullptr;
  int cap = 0;
};
// SoftAWGNDemodulation + Modem::DeMapping with bitLin = 0.5, for `n` entries:
// entry e reads y row e / reps and channel h[e * h_stride + (h_sel ? h_sel[e] : 0)],
// writes p0 row e.  (reps = 4, h_stride = 1 demaps the 4 blind candidates.)
hipError_t launch_demap(int bits, const double *cons, const double2 *y, int S, int reps, const double2 *h,
                        int h_stride, const int32_t *h_sel, double var, int n, double *p0, const DemapDefer &d,
                        hipStream_t s);

// Hard-metric candidates for the PEG blind path (kmcodec.cc:105-119):
// for each codeword and each of its nc (1 or 4) channel estimates h4[b][j], the
// number of unsatisfied checks of rr = (P0 > 0.5).  metrics[b][4] doubles
// (entries >= nc zeroed), chosen[b] = first argmin.
hipError_t launch_cand_metric(const DevCode &c, int bits, const double *cons, const double2 *y, int S,
                              const double2 *h4, int nc, double var, int B, double *metrics, int32_t *chosen,
                              const DemapDefer &d, hipStream_t s);
// argmin over a [B][nc] parity-count table (first minimum) for the BP-based
// metrics; metrics[b][4] = |count|.
hipError_t launch_select(const int32_t *parity_cnt, int nc, int B, double *metrics, int32_t *chosen, hipStream_t s);
// Soft syndrome metric sums: L[e] = sum_j log(syn[e][j]) in row order, for
// e = list[i] (or i), i < n; skipped where iters[e] == 0.
hipError_t launch_soft_sum(const double *syn, int M, const int32_t *iters, const int32_t *list, int n, double *L,
                           hipStream_t s);
// CntErr of byte decisions (uh == NULL: all-zero decisions) against packed
// reference bits; optional per-codeword error bits.
hipError_t launch_count_packed(const uint64_t *ref, int Kw, int K, const uint8_t *uh, long long uh_stride, int B,
                               int32_t *cw_err, unsigned long long *counters, hipStream_t s);

// KMeans::Run + h_hat = clusters[0]/c[0] + 4 rotations (kmeans.hip).
struct KmState {
  double2 hat, prev, sum;  // current h_hat, previous iteration's, cumulative cluster-0 sum
  int cnt, it, done, have_prev;
};
size_t kmeans_workspace_bytes(int S, int B);
// hat_out (optional): the final hatH per codeword (clusters_ = c[k] * hatH).
hipError_t launch_kmeans(int Kc, const double *cons, const double *rot, const double2 *y, int S, int iters, int B,
                         double2 *h_hat, double2 *h4, void *ws, hipStream_t s, double2 *hat_out = nullptr);
// KMeans::clusters() / idx() from the final hatH (kmeans.cc:72-83): clusters[B][Kc], idx[B][S] (either may be null).
hipError_t launch_kmeans_state(int Kc, const double *cons, const double2 *y, int S, int B, const double2 *hat,
                               double2 *clusters, int *idx, hipStream_t s);

// GPU frame generation (counter-based Philox; statistically equivalent to the
// reference's sequential Park-Miller stream, not bit-equal).
struct FrameLaunch {
  int B = 0;
  unsigned long long seed = 0, first_cw = 0;
  double noise_scale = 0;
  uint64_t *uu_bits = nullptr;  // [B][Kw]
  uint64_t *cc_bits = nullptr;  // [B][Cw]
  double2 *y = nullptr;         // [B][S]
  double2 *h = nullptr;         // [B]
};
hipError_t launch_framegen(const DevCode &c, int bits, const double *cons, const FrameLaunch &f, hipStream_t s);

// Count mismatching bits: uu_hat bytes vs reference bits (SourceSink::CntErr).
hipError_t launch_count_bytes(const uint8_t *uu, const uint8_t *uu_hat, int K, int B, unsigned long long *counters,
                              hipStream_t s);

// Device-side self tests of the exact-math helpers (hypot, complex division).
hipError_t launch_math_probe(const double *in, int n, double *out, hipStream_t s);
hipError_t launch_log_probe(const double *in, int n, double *out, hipStream_t s);
// Device-side self test of the shared-reciprocal division (bp_common.hpp):
// in[n][3] = (n0, n1, s) -> out[n][4] = (fast q0, fast q1, IEEE q0, IEEE q1).
hipError_t launch_div_probe(const double *in, int n, double *out, hipStream_t s);

}  // namespace kml
