// bp_regular.hip — BP decoder specialised for regular (dv, dc) codes whose
// message state fits in LDS (PEG2304: dv = 3, dc = 6, 6912 edges).
//
// Arithmetic: bit-exact restatement of lab::BinaryLDPCCodec::Decoder
// (lib/lab/src/binaryldpccodec.cc:165-278), like bp.hip.
//
// Mapping onto a gfx950 CU (one workgroup of T threads per CU, all message
// slots in LDS, persistent over codewords via a dequeue counter):
//   * VN phase: thread t owns columns vn_order[r*T + t], r < RV, exactly
//     (N == RV*T): no predicates, RV independent chains per thread.
//   * CN phase: every check row is shared by an adjacent lane PAIR.  The even
//     lane runs the forward trellis (alpha, binaryldpccodec.cc:237-249) over the
//     row's v2c messages, the odd lane the backward trellis (beta, :251-273)
//     over the same messages in reverse; the lanes then swap the chain states
//     they need through one DPP quad_perm per word, and each computes half of
//     the row's c2v outputs.  c2v_k = clip(t0 / (t0 + t1)) with
//     t0 = a0*b0 + a1*b1, t1 = a0*b1 + a1*b0 is symmetric in (alpha_k, beta_k)
//     under IEEE arithmetic (products commute, the two-term sums commute), so
//     both lanes evaluate the same formula on (own state, partner state) and
//     the result is the reference's bit for bit.  2M == RC*T half-rows:
//     the CN phase has exactly as many lanes busy as the VN phase.
//   * the early-stop parity check rides on the CN phase: the VN phase leaves
//     each column's decision in the sign bit of its q1 words, each lane XORs
//     the ones of its half-row as its chain loads them, and the pair combines
//     the halves through the same DPP swap; the workgroup OR is one barrier
//     (bp_common.hpp wg_any).
//   * wave priorities: falling by step in the VN phase, by wave age in the CN
//     phase (KML_CN_AGE_PRIO).
//   * LDS placement (layout.hpp): the columns' lane assignment is annealed on
//     the host against the VN phase's bank conflicts, the hard decisions are
//     stored by lane position (contiguous byte stores), rows are stored in CN
//     position order with the lane pair's edges interleaved (the pair reads
//     slots 2st, 2st+1 of its row at step st: a per-lane base register plus an
//     immediate offset, conflict-free), and a c2v message goes to the lower or
//     upper half of its slot by bit 2 of the row's CN position.  The VN phase
//     reads it at the planned byte offset.
//   * every LDS address is kept absolute in a register (bp_common.hpp lds_ld).
#include <cstdlib>

#include <type_traits>

#include "bp_common.hpp"
#include "demap_common.hpp"
#include "kernels.hpp"

namespace kml {

namespace {

constexpr int kRedBytes = 16;

// Phase timing (stamps build, -DKML_STAMPS=1; tools/reg_stamps.py): thread 0's
// s_memtime deltas summed per workgroup in registers, flushed at the end:
// [0] queue + barrier, [1] demap / P0, [2] priors + barrier, [3] iterations,
// [4] epilogue (outputs, counts) + barrier, [5] result atomics, [6] codewords,
// [7] iterations run (CN phases).
#ifndef KML_STAMPS
#define KML_STAMPS 0
#endif
// CN-phase wave priorities: s > 0 ranks the waves by age (the youngest third
// highest) until step s, then all at 0 — the oldest waves otherwise win the
// arbiter's age tie-break and finish 1.2K cycles before the youngest (per-wave
// stamps); measured 5 (-0.7..0.9%) against falling-by-step (0), 2, 3 and 6.
#ifndef KML_CN_AGE_PRIO
#define KML_CN_AGE_PRIO 5
#endif
#ifndef KML_VN_AGE_PRIO  // (A/B) 1: VN priorities by wave age for the whole phase (measured +4%: off)
#define KML_VN_AGE_PRIO 0
#endif
// Epilogue latency (stamps: 5.4 K + 1.3 K of ~180 K cycles per codeword): the
// codeword's reference bits for CntErr go straight from global memory into LDS
// in its prologue (global_load_lds: no register holds them, the latency hides
// under the demap / prior check instead of opening the epilogue), and the
// workgroup sums its counters in LDS, flushed with one global atomic each when
// the workgroup leaves.
#ifndef KML_REG_EPI_LDS
#define KML_REG_EPI_LDS 1
#endif
// The next queue entry is taken at the start of a codeword's epilogue (thread
// 0's atomic in flight under CntErr and the epilogue's barrier) instead of
// between two barriers at the top of the loop: one barrier and the atomic's
// round trip leave the per-codeword critical path.
#ifndef KML_REG_QUEUE_EARLY
#define KML_REG_QUEUE_EARLY 1
#endif
constexpr int kRegMaxKw = 64;  // K <= N <= 2304 (bp_regular_threads): 36 words
#if KML_STAMPS
__device__ unsigned long long kml_reg_stamps[8];
// per wave (lane 0), summed over codewords: [0] VN compute, [1] VN barrier
// wait, [2] CN compute, [3] CN barrier wait (+ OR)
__device__ unsigned long long kml_reg_wave_stamps[16][4];
#define REG_WSTAMP(i)                                              \
  do {                                                             \
    if ((threadIdx.x & 63) == 0) {                                 \
      const unsigned long long _t = __builtin_amdgcn_s_memtime();  \
      ws_acc[(i)] += _t - ws_prev;                                 \
      ws_prev = _t;                                                \
    }                                                              \
  } while (0)
#define REG_STAMP(i)                                               \
  do {                                                             \
    if (tid == 0) {                                                \
      const unsigned long long _t = __builtin_amdgcn_s_memtime();  \
      rs_acc[(i)] += _t - rs_prev;                                 \
      rs_prev = _t;                                                \
    }                                                              \
  } while (0)
#else
#define REG_STAMP(i) \
  do {               \
  } while (0)
#define REG_WSTAMP(i) \
  do {                \
  } while (0)
#endif

// swap a double with the adjacent lane (quad_perm [1,0,3,2])
__device__ __forceinline__ double swap_pair(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  const int lo2 = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, false);
  const int hi2 = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi2, lo2);
}
__device__ __forceinline__ int swap_pair_i(int x) { return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false); }
// x (>= +0 or NaN) with its sign bit set to bit
__device__ __forceinline__ double with_sign(double x, int bit) {
  return __hiloint2double((__double2hiint(x) & 0x7FFFFFFF) | (bit << 31), __double2loint(x));
}

// Returns true when a FAST decode met a quotient dd_check could not prove
// correctly rounded (exact_div.hpp): the caller redoes the codeword with
// FAST = false.  The decision is taken at the CN phase's closing barrier,
// before that iteration's syndromes are written, so everything a suspect
// decode wrote (slots, decisions, syndromes of earlier iterations) is what the
// exact decode rewrites identically or overwrites.
#ifndef KML_REG_VN_COLMAJOR
#define KML_REG_VN_COLMAJOR 1
#endif
template <int T, int RV, int RC, int DV, int DC, bool SYN, bool FAST>
__device__ __forceinline__ bool decode_reg(const DevCode &c, const BpLaunch &a, int cw, unsigned char *smem,
                                           unsigned hd, const unsigned (&vaddr)[RV][DV], const double (&pv)[RV],
                                           const int (&crow)[RC], const unsigned (&rb)[RC], const unsigned (&rb2)[RC],
                                           const unsigned (&wb)[RC], int odd, int &iter_out, bool &conv_out,
                                           bool sus0 = false) {
  static_assert(DC % 2 == 0, "the lane-pair split assumes an even row degree");
  constexpr int H = DC / 2;
  __shared__ __attribute__((aligned(16))) int wflags[16];  // wg_any (bp_common.hpp)
  int iter = 0;
  bool conv = false, sus = sus0;
#if KML_STAMPS
  unsigned long long ws_acc[4] = {0, 0, 0, 0}, ws_prev = __builtin_amdgcn_s_memtime();
#endif
  for (; iter < a.iter_count; ++iter) {
    // Wave priorities (s_setprio) fall as a wave advances through a phase, so
    // the SIMD arbiter (priority, then age) favours the waves that are behind:
    // the 3 waves of a SIMD reach the barrier together instead of the oldest
    // finishing first and the youngest running its dependent chains alone.
    // Measured: per-phase end-time spread 3100 -> 500 cycles, kernel -2.5%.
#if KML_VN_AGE_PRIO
    {
      const int grp = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) / 4;  // 0 oldest .. 2 youngest
      if (grp >= 2) __builtin_amdgcn_s_setprio(3);
      else if (grp == 1) __builtin_amdgcn_s_setprio(2);
      else __builtin_amdgcn_s_setprio(1);
    }
#else
    __builtin_amdgcn_s_setprio(3);
#endif
    // The RV columns' chains are interleaved step by step in program order so
    // their dependent fma / rcp sequences overlap.  On the FAST path the
    // boundary state beta = (1, 1) is applied as the identity (x * 1.0 == x).
    {
      // InitMsg (binaryldpccodec.cc:166-170): every c2v is 0.5 before the
      // first CN phase, so iteration 0 takes the constant instead of slots
      // initialised in LDS (every slot is written before it is read)
      double c0s[RV][DV];
#pragma unroll
      for (int r = 0; r < RV; ++r)
#pragma unroll
        for (int k = 0; k < DV; ++k) c0s[r][k] = iter == 0 ? 0.5 : lds_ld<double>(vaddr[r][k]);
#if KML_REG_VN_COLMAJOR
      // one column's chains at a time (registers: see bp_coop.hip).  FAST: the
      // column's quotients unsettled (div2 DEFER), and in the rare case that
      // one of them could not be proven the column runs again settling each
      // (its slot and decision stores are rewritten before the barrier).
#pragma unroll
      for (int r = 0; r < RV; ++r) {
        auto column = [&](auto defer) -> bool {
          constexpr bool D = FAST && decltype(defer)::value;
          bool bad = false;
          double a0 = pv[r], a1 = 1.0 - pv[r], al0[DV], al1[DV];
          int hb = 0;
#pragma unroll
          for (int k = 0; k < DV; ++k) {
            al0[k] = a0;
            al1[k] = a1;
            const double c0 = c0s[r][k];
            const double n0 = a0 * c0;
            const double n1 = a1 * (1.0 - c0);
            if (k + 1 < DV)
              div2<FAST, false, D>(n0, n1, n0 + n1, a0, a1, bad);
            else {  // the posterior only feeds the hard decision
              hb = hard_decision<FAST>(n0, n1, sus);
              lds_st<unsigned char>(hd + r * T, (unsigned char)hb);
            }
          }
          double b0 = 1.0, b1 = 1.0;
#pragma unroll
          for (int k = DV - 1; k >= 0; --k) {
            const bool unit = FAST && k == DV - 1;  // beta = (1, 1)
            const double t0 = unit ? al0[k] : al0[k] * b0;
            const double t1 = unit ? al1[k] : al1[k] * b1;
            double q0, q1;
            if (unit)
              div2<FAST, true>(t0, t1, t0 + t1, q0, q1, sus);
            else
              div2<FAST, false, D>(t0, t1, t0 + t1, q0, q1, bad);
            lds_st<dbl2>(vaddr[r][k] & ~15u, dbl2{q0, with_sign(q1, hb)});
            if (k > 0) {
              const double c0 = c0s[r][k];
              if (unit) {
                b0 = c0;
                b1 = 1.0 - c0;
              } else {
                div2<FAST, false, D>(b0 * c0, b1 * (1.0 - c0), b0 * c0 + b1 * (1.0 - c0), b0, b1, bad);
              }
            }
          }
          return bad;
        };
        if (column(std::true_type{})) column(std::false_type{});
        if (r == RV / 2) __builtin_amdgcn_s_setprio(1);
      }
      __builtin_amdgcn_s_setprio(0);
    }
#else
      double a0[RV], a1[RV], al0[RV][DV], al1[RV][DV];
      int hb[RV];
#pragma unroll
      for (int r = 0; r < RV; ++r) {
        a0[r] = pv[r];
        a1[r] = 1.0 - pv[r];
      }
#pragma unroll
      for (int k = 0; k < DV; ++k)
#pragma unroll
        for (int r = 0; r < RV; ++r) {
          al0[r][k] = a0[r];
          al1[r][k] = a1[r];
          const double c0 = c0s[r][k];
          const double n0 = a0[r] * c0;
          const double n1 = a1[r] * (1.0 - c0);
          if (k + 1 < DV)
            div2<FAST>(n0, n1, n0 + n1, a0[r], a1[r], sus);
          else {  // the posterior only feeds the hard decision
            hb[r] = hard_decision<FAST>(n0, n1, sus);
            lds_st<unsigned char>(hd + r * T, (unsigned char)hb[r]);
          }
        }
      double b0[RV], b1[RV];
#pragma unroll
      for (int r = 0; r < RV; ++r) b0[r] = b1[r] = 1.0;
#if !KML_VN_AGE_PRIO
      __builtin_amdgcn_s_setprio(2);
#endif
#pragma unroll
      for (int k = DV - 1; k >= 0; --k) {
#if !KML_VN_AGE_PRIO
        if (k == DV - 2) __builtin_amdgcn_s_setprio(1);
        if (k == DV - 3) __builtin_amdgcn_s_setprio(0);
#endif
#pragma unroll
        for (int r = 0; r < RV; ++r) {
          const bool unit = FAST && k == DV - 1;  // beta = (1, 1)
          const double t0 = unit ? al0[r][k] : al0[r][k] * b0[r];
          const double t1 = unit ? al1[r][k] : al1[r][k] * b1[r];
          double q0, q1;
          if (unit)  // beta = (1, 1): t is the normalised alpha, its sum within ulps of 1 (bp_common.hpp rcp_near1)
            div2<FAST, true>(t0, t1, t0 + t1, q0, q1, sus);
          else
            div2<FAST>(t0, t1, t0 + t1, q0, q1, sus);
          // the column's decision rides in the sign bit of q1 (a probability,
          // >= +0): the CN chains that load the message collect the parity
          lds_st<dbl2>(vaddr[r][k] & ~15u, dbl2{q0, with_sign(q1, hb[r])});
          if (k > 0) {
            const double c0 = c0s[r][k];
            if (unit) {  // (c0, 1 - c0) / (c0 + (1 - c0)): the sum rounds to exactly 1 (bp_common.hpp)
              b0[r] = c0;
              b1[r] = 1.0 - c0;
            } else {
              div2<FAST>(b0[r] * c0, b1[r] * (1.0 - c0), b0[r] * c0 + b1[r] * (1.0 - c0), b0[r], b1[r], sus);
            }
          }
        }
      }
    }
#endif
    REG_WSTAMP(0);
    __syncthreads();
    REG_WSTAMP(1);

    // The early-stop parity check rides on the CN phase: in steps 0..H-1 the
    // even lane loads the row's edges [0, H) and the odd lane [H, DC), whose
    // q1 words carry the columns' decisions in their sign bits.  The OR over
    // the workgroup is folded into the CN phase's closing barrier: the CN
    // phase runs speculatively, and a converged codeword (no failing row)
    // discards it — its slots are never read again and its syndromes are only
    // written when the phase counts.
    unsigned par[RC];

    // ------------------------------------------------------------ CN phase
    double syn0[RC];
    // Step s of the even lane advances alpha over edge s, of the odd lane beta
    // over edge DC-1-s.  From step H on, the pair swaps the chain states and
    // each lane finishes one c2v per step.  Within a step every message LOAD is
    // issued before the c2v STOREs (the partner's store of this step hits the
    // slot the lane is about to read), and LDS executes a wave's operations in
    // program order.
    {
      double x0[RC][H], x1[RC][H];  // lower-half chain states, kept for the swap
      double s0[RC], s1[RC];        // current chain state
#pragma unroll
      for (int r = 0; r < RC; ++r) {
        s0[r] = 1.0;
        s1[r] = 0.0;
        par[r] = 0;
      }
#if KML_CN_AGE_PRIO  // (A/B) the youngest waves start the CN phase at the highest priority
      {
        const int grp = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) / 4;  // 0 oldest .. 2 youngest
        if (grp >= 2) __builtin_amdgcn_s_setprio(3);
        else if (grp == 1) __builtin_amdgcn_s_setprio(2);
        else __builtin_amdgcn_s_setprio(1);
      }
#else
      __builtin_amdgcn_s_setprio(2);
#endif
#pragma unroll
      for (int st = 0; st < DC; ++st) {
#if KML_CN_AGE_PRIO
        if (st == KML_CN_AGE_PRIO) __builtin_amdgcn_s_setprio(0);
#else
        if (st == 2) __builtin_amdgcn_s_setprio(1);
        if (st == 4) __builtin_amdgcn_s_setprio(0);
#endif
        const bool advance = SYN || st + 1 < DC;
        double m0[RC], m1[RC];
        if (advance) {
#pragma unroll
          for (int r = 0; r < RC; ++r) {
            // edge (odd ? DC-1-st : st): physical slot 2st+odd of the row while
            // st < H, 2(DC-1-st)+1-odd after (layout.cpp)
            const dbl2 m = st < H ? lds_ld<dbl2>(rb[r] + st * 32) : lds_ld<dbl2>(rb2[r] + (DC - 1 - st) * 32);
            if (st < H) par[r] ^= (unsigned)__double2hiint(m.y);
            m0[r] = m.x;
            m1[r] = fabs(m.y);  // clear the decision bit
          }
        }
        if (st < H) {
#pragma unroll
          for (int r = 0; r < RC; ++r) {
            x0[r][st] = s0[r];
            x1[r][st] = s1[r];
          }
        } else {
          // c2v of edge (odd ? st : DC-1-st) from (own state at DC-1-st, partner state at st)
          double t0[RC], ts[RC], q[RC];
#pragma unroll
          for (int r = 0; r < RC; ++r) {
            const double y0 = swap_pair(s0[r]);
            const double y1 = swap_pair(s1[r]);
            const double o0 = x0[r][DC - 1 - st], o1 = x1[r][DC - 1 - st];
            const bool unit = FAST && st == DC - 1;  // own state is the boundary (1, 0)
            t0[r] = unit ? y0 : o0 * y0 + o1 * y1;
            ts[r] = t0[r] + (unit ? y1 : o0 * y1 + o1 * y0);
          }
          cn_c2v_rows<RC, FAST>(t0, ts, q);  // the sums are within ulps of 1 (bp_common.hpp)
#pragma unroll
          for (int r = 0; r < RC; ++r) lds_st<double>(wb[r] + (DC - 1 - st) * 32, q[r]);
        }
        if (advance) {
          double n0[RC], n1[RC];
#pragma unroll
          for (int r = 0; r < RC; ++r) {
            const bool unit = FAST && st == 0;  // state (1, 0)
            n0[r] = unit ? m0[r] : s0[r] * m0[r] + s1[r] * m1[r];
            n1[r] = unit ? m1[r] : s0[r] * m1[r] + s1[r] * m0[r];
          }
          cn_norm_rows<RC, FAST>(n0, n1, s0, s1);
        }
      }
#pragma unroll
      for (int r = 0; r < RC; ++r) syn0[r] = s0[r];
    }
    int fail = 0;
#pragma unroll
    for (int r = 0; r < RC; ++r) {
      const int p = (int)(par[r] >> 31);
      fail |= p ^ swap_pair_i(p);
    }
    REG_WSTAMP(2);
    const int wg = FAST ? wg_any2<T / 64>(fail, sus, wflags) : wg_any<T / 64>(fail, wflags);
    REG_WSTAMP(3);
    if (FAST && (wg & 2)) {  // an unproven quotient in this VN phase: redo exactly
      iter_out = iter;
      conv_out = false;
      return true;
    }
    if (!(wg & 1)) {  // every row satisfied before this CN phase
      conv = true;
      break;
    }
    if constexpr (SYN) {
#pragma unroll
      for (int r = 0; r < RC; ++r)
        if (!odd) a.syn[(long long)cw * c.M + crow[r]] = syn0[r];  // alpha past the last edge (:274)
    }
  }
#if KML_STAMPS
  if ((threadIdx.x & 63) == 0)
    for (int i = 0; i < 4; ++i) atomicAdd(&kml_reg_wave_stamps[threadIdx.x >> 6][i], ws_acc[i]);
#endif
  iter_out = iter;
  conv_out = conv;
  return false;
}

// Dynamic LDS: E slots of 16 B, the reduction words, N hard-decision bytes,
// then (fused demap only, 16-byte aligned) the codeword's N priors.
constexpr size_t p0s_offset(int E, int N) { return ((size_t)E * 16 + kRedBytes + (size_t)N + 15) & ~(size_t)15; }
// then the info bits' positions in the decision bytes (u16, K entries), staged
// once per workgroup for the epilogue's CntErr
constexpr size_t ipos_offset(int E, int N, int DMB) {
  return DMB > 0 ? p0s_offset(E, N) + (size_t)N * 8 : (((size_t)E * 16 + kRedBytes + (size_t)N + 1) & ~(size_t)1);
}
constexpr size_t reg_lds_bytes(int E, int N, int K, int DMB) { return ipos_offset(E, N, DMB) + (size_t)K * 2; }

// EXACT = false: the FAST kernel.  It decodes every codeword whose priors
// qualify (bp_common.hpp fast_prior_ok) on the FAST path and appends the rest,
// and every codeword whose FAST decode met an unproven quotient, to the defer
// list (a.defer_idx / a.defer_cnt; no outputs, no counters for those).
// EXACT = true: decodes its entries (the defer list) on the exact path (div_rn).
// Two kernels rather than one with both paths: the exact path's registers
// would otherwise be allocated (and spilled) in the FAST kernel too.
template <int T, int RV, int RC, int DV, int DC, bool SYN, int DMB, bool EXACT>
__global__ __launch_bounds__(T) void bp_regular_kernel(DevCode c, BpLaunch a, unsigned int *queue, int fast_allowed) {
  const double plo = fast_prior_lo(c.dv_max);  // FAST prior domain (bp_common.hpp)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ __attribute__((aligned(16))) int pflags[16];  // wg_all of the FAST prior check (bp_common.hpp)
  // fused demap: the constellation and the exp table in LDS (demap_common.hpp)
  __shared__ double dcons[DMB > 0 ? (2 << DMB) : 2];
  __shared__ uint64_t detab[DMB > 0 ? 256 : 1];
  __shared__ uint64_t refw[kRegMaxKw];                  // KML_REG_EPI_LDS: this codeword's reference bits
  __shared__ unsigned long long wcnt[CNT_CONVERGED + 1];  // KML_REG_EPI_LDS: the workgroup's counters
  double *p0s = reinterpret_cast<double *>(smem + p0s_offset(c.E, c.N));
  if constexpr (DMB > 0) {
    for (int k = threadIdx.x; k < (2 << DMB); k += T) dcons[k] = a.sym_cons[k];
    stage_exp_table(detab);
  }
  constexpr int H = (DC + 1) / 2;
  const int tid = threadIdx.x;
  const int odd = tid & 1;
  int *red = reinterpret_cast<int *>(smem + (size_t)c.E * 16);
  unsigned char *cch = smem + (size_t)c.E * 16 + kRedBytes;

  const unsigned smem_a = lds_addr(smem), cch_a = lds_addr(cch);
  unsigned short *ipos = reinterpret_cast<unsigned short *>(smem + ipos_offset(c.E, c.N, DMB));
  for (int i = tid; i < c.K; i += T) ipos[i] = (unsigned short)c.reg_pos[c.info_off + i];
  int vcol[RV];
  unsigned vaddr[RV][DV];
#pragma unroll
  for (int r = 0; r < RV; ++r) {
    const int v = c.vn_order[r * T + tid];
    const int b = c.col_ptr[v];
    vcol[r] = v;
#pragma unroll
    for (int k = 0; k < DV; ++k) {
      vaddr[r][k] = smem_a + (unsigned)c.reg_c2v[b + k];
      asm volatile("" : "+v"(vaddr[r][k]));
    }
  }
  const int chalf = ((tid >> 3) & 1) * 8;  // bit 2 of the CN position (tid >> 1)
  int crow[RC], cbase[RC];
  unsigned rb[RC], rb2[RC], wb[RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int row = c.cn_order[r * (T / 2) + (tid >> 1)];
    crow[r] = row;
    cbase[r] = c.row_ptr[row];
    // the row's slots sit at its CN position, the pair's edges interleaved (layout.cpp)
    rb[r] = smem_a + (unsigned)((r * (T / 2) + (tid >> 1)) * DC + odd) * 16;
    rb2[r] = rb[r] + 16 - 32 * odd;
    wb[r] = rb[r] + chalf;
    asm volatile("" : "+v"(rb[r]), "+v"(rb2[r]), "+v"(wb[r]));
  }

#if KML_STAMPS
  unsigned long long rs_prev = __builtin_amdgcn_s_memtime(), rs_acc[8] = {};
#endif
  const int B = a.B_dev ? (int)*a.B_dev : a.B;  // the exact kernel: the FAST kernel's defer count
  const bool cnt_lds = KML_REG_EPI_LDS && a.counters;
  const bool ref_pre = KML_REG_EPI_LDS && a.ref_bits && a.iter_count > 0;  // (c.Kw <= kRegMaxKw: host check)
  if (cnt_lds && tid <= CNT_CONVERGED) wcnt[tid] = 0;  // ordered by the loop's first barrier
  if (KML_REG_QUEUE_EARLY && tid == 0) {  // the first entry; then each codeword's epilogue takes the next
    red[3] = (int)atomicAdd(queue, 1u);
    red[0] = 0;
    red[1] = 0;
  }
  for (;;) {
    __syncthreads();
    if (!KML_REG_QUEUE_EARLY) {
      if (tid == 0) {
        red[3] = (int)atomicAdd(queue, 1u);
        red[0] = 0;
        red[1] = 0;
      }
      __syncthreads();
    }
    const int entry = red[3];
    REG_STAMP(0);
    if (entry >= B) break;
    const int cw = a.cw_idx ? a.cw_idx[entry] : entry;
    if (ref_pre && tid < 2 * c.Kw)  // one dword per lane (the first waves), in flight through the prologue
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const unsigned *>(a.ref_bits + (long long)cw * c.Kw) + tid,
                                       (__attribute__((address_space(3))) void *)(reinterpret_cast<unsigned *>(refw) +
                                                                                  (tid & ~63)),
                                       4, 0, 0);
    const double *p0;
    bool dok = true;  // FAST kernel: every symbol's FAST demap proven (else the exact kernel demaps the codeword)
    if constexpr (DMB > 0) {  // ModemLinearSystem::DeMapping of this codeword into LDS
      const int S = c.cc_len / DMB;
      const double2 hh = a.sym_h[(long long)cw * a.sym_h_stride + (a.sym_h_sel ? a.sym_h_sel[cw] : 0)];
      const double2 *yy = a.sym_y + (long long)cw * S;
      for (int j = tid; j < S; j += T) {
        const double2 v = yy[j];
        double out[DMB];
        if constexpr (EXACT)
          demap_symbol_t<DMB, false, lds_cons, 2, false>((lds_cons)dcons, (lds_exptab)detab, v.x, v.y, hh.x, hh.y,
                                                          a.sym_var, out);
        else  // no exact fallback in the FAST kernel (its registers): a failing symbol defers the codeword
          dok &= demap_symbol_t<DMB, true, lds_cons, 2, false>((lds_cons)dcons, (lds_exptab)detab, v.x, v.y, hh.x,
                                                              hh.y, a.sym_var, out);
#pragma unroll
        for (int b = 0; b < DMB; ++b) p0s[j * DMB + b] = out[b];
      }
      __syncthreads();
      p0 = p0s;
    } else {
      p0 = a.p0 + (long long)cw * a.p0_stride;
      if (a.p0_sel) p0 += (long long)a.p0_sel[cw] * a.p0_sel_stride;
    }

    REG_STAMP(1);
    double pv[RV];
    bool ok = dok;
#pragma unroll
    for (int r = 0; r < RV; ++r) {
      pv[r] = (vcol[r] >= c.punct) ? p0[vcol[r] - c.punct] : 0.5;
      ok = ok && fast_prior_ok(pv[r], plo);
    }
    // the LDS writes land before wave 0 passes the next barrier (the barriers wait lgkmcnt only)
    if (ref_pre) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const bool fast = wg_all<T / 64>(ok ? 1 : 0, pflags) && (fast_allowed & 1);
    REG_STAMP(2);

    int iter = 0;
    bool conv = false;
    if constexpr (!EXACT) {
      bool defer = !fast;
      if (fast && decode_reg<T, RV, RC, DV, DC, SYN, true>(c, a, cw, smem, cch_a + tid, vaddr, pv, crow, rb, rb2, wb,
                                                           odd, iter, conv, (fast_allowed & 2) != 0)) {
        defer = true;  // an unproven quotient: the exact kernel redoes the codeword
        if (tid == 0 && a.counters) atomicAdd(&a.counters[CNT_REDONE], 1ull);
      }
      if (defer) {
        if (tid == 0) {
          a.defer_idx[atomicAdd(a.defer_cnt, 1u)] = cw;
          if (KML_REG_QUEUE_EARLY) red[3] = (int)atomicAdd(queue, 1u);  // (every thread has read red[3])
        }
        continue;
      }
    } else {
      decode_reg<T, RV, RC, DV, DC, SYN, false>(c, a, cw, smem, cch_a + tid, vaddr, pv, crow, rb, rb2, wb, odd, iter,
                                               conv);
    }

    REG_STAMP(3);
    unsigned nxt = 0;  // KML_REG_QUEUE_EARLY: the next entry, in flight through the epilogue
    if (KML_REG_QUEUE_EARLY && tid == 0) nxt = atomicAdd(queue, 1u);
#if KML_STAMPS
    if (tid == 0) {
      rs_acc[6] += 1;
      rs_acc[7] += (unsigned long long)iter;
    }
#endif
    if (a.iter_count > 0) {
      if (a.uu_hat) {
        uint8_t *u = a.uu_hat + (long long)cw * c.K;
        for (int i = tid; i < c.K; i += T) u[i] = cch[c.reg_pos[i + c.info_off]];
      }
      if (a.cc_hat) {
        uint8_t *o = a.cc_hat + (long long)cw * c.N;
        for (int v = tid; v < c.N; v += T) o[v] = cch[c.reg_pos[v]];
      }
      if (a.parity_cnt) {
        int cnt = 0;
#pragma unroll
        for (int r = 0; r < RC; ++r) {
          int p = 0;  // ParityCheck of the final decisions (once per codeword: the columns from global)
#pragma unroll
          for (int k = 0; k < H; ++k) {
            const int e = odd ? DC / 2 + k : k;
            p ^= cch[c.reg_pos[c.row_col[cbase[r] + (e < DC ? e : DC - 1)]]];
          }
          const int full = p ^ swap_pair_i(p);
          if (!odd) cnt += full;
        }
        if (cnt) atomicAdd(&red[0], cnt);
      }
      if (a.ref_bits) {  // CntErr (sourcesink.cc:29-47): two 64-bit words per wave and round, loads first
        const uint64_t *ref = a.ref_bits + (long long)cw * c.Kw;  // (KML_REG_EPI_LDS = 0)
        const int lane = tid & 63;
        int errs = 0;
        for (int w0 = tid >> 6; w0 < c.Kw; w0 += 2 * (T / 64)) {
          const int w1 = w0 + T / 64;
          const uint64_t r0 = KML_REG_EPI_LDS ? refw[w0] : ref[w0];
          const uint64_t r1 = w1 < c.Kw ? (KML_REG_EPI_LDS ? refw[w1] : ref[w1]) : 0ull;
          const int i0 = w0 * 64 + lane, i1 = w1 * 64 + lane;
          const int b0 = i0 < c.K ? cch[ipos[i0]] : 0;
          const int b1 = i1 < c.K && w1 < c.Kw ? cch[ipos[i1]] : 0;
          const uint64_t m0 = __ballot(b0), m1 = __ballot(b1);
          errs += __popcll(m0 ^ r0) + (w1 < c.Kw ? __popcll(m1 ^ r1) : 0);
        }
        if (lane == 0 && errs) atomicAdd(&red[1], errs);
      }
    }
    __syncthreads();
    REG_STAMP(4);
    if (tid == 0) {
      if (a.ret) a.ret[cw] = iter + (iter < a.max_iter);
      if (a.parity_cnt) a.parity_cnt[cw] = red[0];
      if (a.cw_err && a.ref_bits) a.cw_err[cw] = a.iter_count > 0 ? red[1] : 0;
      if (a.iters) a.iters[cw] = iter;
      if (a.counters) {
        unsigned long long *ct = cnt_lds ? wcnt : a.counters;  // (LDS: flushed at the exit)
        const unsigned long long vn = conv ? (unsigned long long)iter + 1 : (unsigned long long)iter;
        atomicAdd(&ct[CNT_VN_PHASES], vn);
        atomicAdd(&ct[CNT_CN_PHASES], (unsigned long long)iter);
        if (conv) atomicAdd(&ct[CNT_CONVERGED], 1ull);
        if (a.ref_bits && a.iter_count > 0) {
          const int errs = red[1];
          atomicAdd(&ct[CNT_ERR_BIT], (unsigned long long)errs);
          atomicAdd(&ct[CNT_ERR_BLK], errs > 0 ? 1ull : 0ull);
          atomicAdd(&ct[CNT_TOT_BIT], (unsigned long long)c.K);
          atomicAdd(&ct[CNT_TOT_BLK], 1ull);
        }
      }
      if (KML_REG_QUEUE_EARLY) {  // after the reads above; read by all after the loop's barrier
        red[3] = (int)nxt;
        red[0] = 0;
        red[1] = 0;
      }
    }
    REG_STAMP(5);
  }
  if (cnt_lds && tid == 0)  // the workgroup's sums (only thread 0 wrote them)
    for (int i = 0; i <= CNT_CONVERGED; ++i)
      if (wcnt[i]) atomicAdd(&a.counters[i], wcnt[i]);
#if KML_STAMPS
  if (tid == 0)
    for (int i = 0; i < 8; ++i) atomicAdd(&kml_reg_stamps[i], rs_acc[i]);
#endif
}

template <int T, int RV, int RC, int DV, int DC, bool SYN, int DMB, bool EXACT>
hipError_t launch_reg_one(const DevCode &c, const BpLaunch &a, hipStream_t s, int fast_allowed) {
  auto kern = bp_regular_kernel<T, RV, RC, DV, DC, SYN, DMB, EXACT>;
  const size_t lds = reg_lds_bytes(c.E, c.N, c.K, DMB);
  hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  long long grid = ncu;
  if (grid > a.B) grid = a.B;
  e = hipMemsetAsync(a.queue, 0, sizeof(unsigned int), s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(T), lds, s, c, a, a.queue, fast_allowed);
  return hipGetLastError();
}

// The FAST kernel over the batch, then the exact kernel over the codewords it
// deferred (usually none: its workgroups read a zero count and leave); with
// FAST division off, the exact kernel over the batch.
template <int T, int RV, int RC, int DV, int DC, bool SYN, int DMB>
hipError_t launch_reg_t(const DevCode &c, const BpLaunch &a, hipStream_t s, int fast_allowed) {
  const size_t lds = reg_lds_bytes(c.E, c.N, c.K, DMB);
  if (lds > 160 * 1024 || c.K > 65536 || c.N > 65536 || c.Kw > kRegMaxKw) return hipErrorNotSupported;
  if (!(fast_allowed & 1)) return launch_reg_one<T, RV, RC, DV, DC, SYN, DMB, true>(c, a, s, 0);
  if (!a.defer_idx || !a.defer_cnt) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(a.defer_cnt, 0, sizeof(unsigned), s);
  if (e != hipSuccess) return e;
  e = launch_reg_one<T, RV, RC, DV, DC, SYN, DMB, false>(c, a, s, fast_allowed);
  if (e != hipSuccess) return e;
  BpLaunch b = a;
  b.cw_idx = a.defer_idx;
  b.B_dev = a.defer_cnt;
  return launch_reg_one<T, RV, RC, DV, DC, SYN, DMB, true>(c, b, s, 0);
}

}  // namespace

int bp_regular_threads(int N, int M, int E, int dv_max, int dc_max, int regular) {
  if (!regular || (long long)E * 16 + kRedBytes + N > 160 * 1024) return 0;
  // PEG2304-class: dv 3, dc 6, N = 3*768, 2M = 3*768
  if (dv_max == 3 && dc_max == 6 && N == 3 * 768 && 2 * M == 3 * 768) return 768;
  return 0;
}

hipError_t launch_bp_regular(const DevCode &c, const BpLaunch &a, hipStream_t s) {
  if (!c.reg_c2v || bp_regular_threads(c.N, c.M, c.E, c.dv_max, c.dc_max, c.regular) != 768)
    return hipErrorNotSupported;
  const int fast = bp_fast_mode(c);
  if (a.sym_y) {
    if (!bp_regular_fuses_demap(c, a.sym_bits) || a.cw_idx || a.p0_sel) return hipErrorNotSupported;
    return a.syn ? launch_reg_t<768, 3, 3, 3, 6, true, 2>(c, a, s, fast)
                 : launch_reg_t<768, 3, 3, 3, 6, false, 2>(c, a, s, fast);
  }
  return a.syn ? launch_reg_t<768, 3, 3, 3, 6, true, 0>(c, a, s, fast)
               : launch_reg_t<768, 3, 3, 3, 6, false, 0>(c, a, s, fast);
}

#if KML_STAMPS
}  // namespace kml
extern "C" int kml_debug_reg_stamps(unsigned long long *out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(kml::kml_reg_stamps), sizeof(kml::kml_reg_stamps));
  if (e == hipSuccess)  // then the per-wave phase sums (16 x 4)
    e = hipMemcpyFromSymbol(out + 8, HIP_SYMBOL(kml::kml_reg_wave_stamps), sizeof(kml::kml_reg_wave_stamps));
  if (reset) {
    unsigned long long zero[8 + 64] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(kml::kml_reg_stamps), zero, sizeof(kml::kml_reg_stamps));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(kml::kml_reg_wave_stamps), zero, sizeof(kml::kml_reg_wave_stamps));
  }
  return e == hipSuccess ? 0 : -3;
}
namespace kml {
#endif

bool bp_regular_fuses_demap(const DevCode &c, int bits) {
  if (const char *e = getenv("KML_FUSED_DEMAP"))
    if (e[0] == '0') return false;
  return c.reg_c2v && bp_regular_threads(c.N, c.M, c.E, c.dv_max, c.dc_max, c.regular) == 768 && c.punct == 0 &&
         bits == 2 && c.cc_len % bits == 0 && reg_lds_bytes(c.E, c.N, c.K, 2) <= 160 * 1024;
}

}  // namespace kml

#if KML_DIV_STATS
KML_DIV_STATS_ACCESSOR(kml_debug_div_stats_reg)
#endif
