// bp_irregular.hip — BP decoder for irregular codes whose message state fits
// in LDS (5G BG2 K960: 7,392 edges, column degrees {1,2,3,4,5,7,9}, row
// degrees {4,5,6,8,10}).
//
// Arithmetic: bit-exact restatement of lab::Binary5GLDPCCodec::Decoder /
// lab::BinaryLDPCCodec::Decoder (lib/lab/src/binary5gldpccodec.cc:112-232,
// binaryldpccodec.cc:165-278), like the other BP kernels; the punctured 5G
// columns get the prior (0.5, 1 - 0.5) (binary5gldpccodec.cc:126-129).
//
// Mapping (one workgroup of T threads per CU, persistent over codewords):
//   * message slots (16 B per edge), the codeword's priors and the
//     column->slot table (u16) in LDS;
//   * the round plan (layout.hpp IrregularPlan) gives thread t its columns
//     and half-rows in three rounds: in rounds 0 and 1 two items of one
//     degree whose chains run interleaved (the second chain hides the first's
//     fma / rcp latency; pairs up to degree kIrrVnPairMax / kIrrCnPairMax, the
//     limit of the 168 registers of three waves per SIMD), in round 2 a single
//     item; a wave runs one degree per round, every (degree, pairing) has its
//     own fully unrolled instance (the chain states stay in registers), and
//     the waves are placed so the 4 SIMDs get balanced VALU work.  Measured
//     (BG2, 50 iterations, 16384 codewords): 25.0 ms with one item per round
//     -> 21.25 ms; pair limits 5/8: 21.75, 5/10: 21.8, 7/8: 23.2 (pairs of
//     degree 9 spill inside the loop);
//   * check rows are split over lane pairs exactly like bp_regular.hip: the
//     even lane runs the forward trellis, the odd lane the backward one, DPP
//     swaps exchange the chain states, each lane finishes half of the row's
//     c2v messages (for an odd degree the even lane also takes the middle
//     edge, from the two states both lanes hold at that step);
//   * the slots are laid out in per-wave blocks, a row's edges 32 slots apart
//     (layout.hpp kIrrCnStride), so a CN step reads contiguous runs;
//   * the VN phase leaves each column's decision in the sign bit of its v2c
//     q1 words, and the CN chains XOR the ones they load: the early-stop
//     parity costs no pass of its own, and its workgroup OR is one barrier
//     (bp_common.hpp wg_any).  Measured: 19.5 ms (round-2 start) -> 14.7 ms;
//   * the shared-reciprocal exact division (bp_common.hpp) on codewords whose
//     priors qualify.
#include "bp_common.hpp"
#include "kernels.hpp"

namespace kml {

namespace {

constexpr int kRedBytes = 16;

__device__ __forceinline__ double swap_pair(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  const int lo2 = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, false);
  const int hi2 = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi2, lo2);
}
__device__ __forceinline__ double with_sign(double x, int bit) {
  return __hiloint2double((__double2hiint(x) & 0x7FFFFFFF) | (bit << 31), __double2loint(x));
}
__device__ __forceinline__ int swap_pair_i(int x) { return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false); }

// Beta chains ahead (R <= KML_IRR_VN_BETA_EARLY_R): a column's backward
// states beta_k (binaryldpccodec.cc:199-213: beta_{D-1} = (1, 1), beta_{k-1} =
// normalise(beta_k * c2v_k)) depend on the c2v messages only, not on the
// forward alphas, so the two chains run interleaved step by step and the
// outputs normalise(alpha_k * beta_k) follow, independent of each other: the
// column's dependent chain is max(D - 1, D - 1) + 1 normalisations instead of
// (D - 1) + (D - 1) + 1.  The same operations on the same values (bit-exact),
// in another order; the betas are held (2 D more registers).  A wave holding
// the heaviest columns alone at the end of the VN phase runs latency-bound
// (profiles/r05_v4_irr_stamps.txt: waves 0-2, degree 9).
#ifndef KML_IRR_VN_BETA_EARLY_R
#define KML_IRR_VN_BETA_EARLY_R 1
#endif
template <int D, int R, bool FAST>
__device__ __forceinline__ void vn_cols_beta_early(double2 *slots, const unsigned short *const (&cs)[R],
                                                   const double (&p)[R], unsigned char *const (&hard)[R], bool &sus) {
  double c0s[R][D];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int k = 0; k < D; ++k) c0s[r][k] = slots[cs[r][k]].x;
  double a0[R], a1[R], al0[R][D], al1[R][D], be0[R][D], be1[R][D];
  int hb[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    a0[r] = p[r];
    a1[r] = 1.0 - p[r];
    be0[r][D - 1] = be1[r][D - 1] = 1.0;
  }
#pragma unroll
  for (int k = 0; k < D; ++k)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      // forward step k
      al0[r][k] = a0[r];
      al1[r][k] = a1[r];
      const double n0 = a0[r] * c0s[r][k];
      const double n1 = a1[r] * (1.0 - c0s[r][k]);
      if (k + 1 < D)
        div2<FAST>(n0, n1, n0 + n1, a0[r], a1[r], sus);
      else
        *hard[r] = (unsigned char)(hb[r] = hard_decision<FAST>(n0, n1, sus));
      // backward state j - 1 from state j and c2v_j, j = D - 1 - k
      const int j = D - 1 - k;
      if (j > 0) {
        const double c0 = c0s[r][j];
        const double b0 = be0[r][j], b1 = be1[r][j];
        if (FAST && j == D - 1) {  // beta = (1, 1): (c0, 1 - c0), its sum rounds to exactly 1 (bp_common.hpp)
          be0[r][j - 1] = c0;
          be1[r][j - 1] = 1.0 - c0;
        } else {
          div2<FAST>(b0 * c0, b1 * (1.0 - c0), b0 * c0 + b1 * (1.0 - c0), be0[r][j - 1], be1[r][j - 1], sus);
        }
      }
    }
#pragma unroll
  for (int k = D - 1; k >= 0; --k)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool unit = FAST && k == D - 1;  // beta = (1, 1)
      const double t0 = unit ? al0[r][k] : al0[r][k] * be0[r][k];
      const double t1 = unit ? al1[r][k] : al1[r][k] * be1[r][k];
      double q0, q1;
      if (unit && D == 1) {  // the prior itself (vn_cols below)
        q0 = t0;
        q1 = t1;
      } else if (unit)
        div2<FAST, true>(t0, t1, t0 + t1, q0, q1, sus);
      else
        div2<FAST>(t0, t1, t0 + t1, q0, q1, sus);
      slots[cs[r][k]] = make_double2(q0, with_sign(q1, hb[r]));
    }
}

// R columns of degree D (binaryldpccodec.cc:177-213), their chains
// interleaved step by step so the dependent fma / rcp sequences overlap.
template <int D, int R, bool FAST>
__device__ __forceinline__ void vn_cols(double2 *slots, const unsigned short *const (&cs)[R], const double (&p)[R],
                                        unsigned char *const (&hard)[R], bool &sus) {
  if constexpr (R <= KML_IRR_VN_BETA_EARLY_R && D > 2) {
    vn_cols_beta_early<D, R, FAST>(slots, cs, p, hard, sus);
    return;
  }
  double c0s[R][D];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int k = 0; k < D; ++k) c0s[r][k] = slots[cs[r][k]].x;
  double a0[R], a1[R], al0[R][D], al1[R][D];
  int hb[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    a0[r] = p[r];
    a1[r] = 1.0 - p[r];
  }
#pragma unroll
  for (int k = 0; k < D; ++k)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      al0[r][k] = a0[r];
      al1[r][k] = a1[r];
      const double n0 = a0[r] * c0s[r][k];
      const double n1 = a1[r] * (1.0 - c0s[r][k]);
      if (k + 1 < D)
        div2<FAST>(n0, n1, n0 + n1, a0[r], a1[r], sus);
      else
        *hard[r] = (unsigned char)(hb[r] = hard_decision<FAST>(n0, n1, sus));
    }
  double b0[R], b1[R];
#pragma unroll
  for (int r = 0; r < R; ++r) b0[r] = b1[r] = 1.0;
#pragma unroll
  for (int k = D - 1; k >= 0; --k)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const bool unit = FAST && k == D - 1;  // beta = (1, 1)
      const double t0 = unit ? al0[r][k] : al0[r][k] * b0[r];
      const double t1 = unit ? al1[r][k] : al1[r][k] * b1[r];
      double q0, q1;
      if (unit && D == 1) {
        // a degree-1 column's v2c is its prior (p, 1 - p) / (p + RN(1 - p)), a
        // constant of the codeword: for a FAST prior p in [0, 1] the sum is
        // exactly 1 (1 - p is exact for p >= 1/2; below, RN(1 - p) is within
        // 2^-54 of 1 - p, and p + RN(1 - p) = 1 + d with |d| <= 2^-54 rounds
        // to 1, the tie -2^-54 to the even 1), so the quotients are t0, t1
        q0 = t0;
        q1 = t1;
      } else if (unit)  // beta = (1, 1): t is the normalised alpha, its sum within ulps of 1 (bp_common.hpp rcp_near1)
        div2<FAST, true>(t0, t1, t0 + t1, q0, q1, sus);
      else
        div2<FAST>(t0, t1, t0 + t1, q0, q1, sus);
      // the column's decision rides in the sign bit of the v2c q1 (a probability,
      // so the bit is otherwise clear): the parity check reads it in row order
      slots[cs[r][k]] = make_double2(q0, with_sign(q1, hb[r]));
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

// Half of R check rows of degree D (binaryldpccodec.cc:235-275), streamed step
// by step with the R rows interleaved; sv[r] = the forward state past the
// last edge (syndrom_soft, read on the even lane) when SYN.  par[r] (bit 31)
// = the XOR of the decisions (vn_cols' sign bits) of the lane's half of the
// row, from the words the chain loads anyway: the even lane's edges
// [0, (D+1)/2), the odd lane's [(D+1)/2, D).
template <int D, int R, bool SYN, bool FAST>
__device__ __forceinline__ void cn_halves(double2 *slots, const int (&base)[R], int odd, double (&sv)[R],
                                          unsigned (&par)[R]) {
  constexpr int S = (D + 1) / 2;  // states kept: x[0..S)
  double x0[R][S], x1[R][S], s0[R], s1[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    s0[r] = 1.0;
    s1[r] = 0.0;
    par[r] = 0;
  }
#pragma unroll
  for (int st = 0; st < D; ++st) {
    const bool advance = SYN || st + 1 < D;
    double m0[R], m1[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      m0[r] = m1[r] = 0.0;
      if (advance) {
        const double2 m = slots[base[r] + (odd ? D - 1 - st : st) * kIrrCnStride];
        if (st < D - S || (st < S && !odd)) par[r] ^= (unsigned)__double2hiint(m.y);
        m0[r] = m.x;
        m1[r] = fabs(m.y);  // clear the decision bit (vn_cols)
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (st < S) {
        x0[r][st] = s0[r];
        x1[r][st] = s1[r];
      }
      if ((D & 1) && st == (D - 1) / 2) {  // middle edge: both states are current here
        const double y0 = swap_pair(s0[r]), y1 = swap_pair(s1[r]);
        const double t0 = s0[r] * y0 + s1[r] * y1;
        const double t1 = s0[r] * y1 + s1[r] * y0;
        const double q = clip_c2v<FAST>(div1<FAST, true>(t0, t0 + t1));
        if (!odd) slots[base[r] + st * kIrrCnStride].x = q;
      }
      if (st >= S) {
        // c2v of edge (odd ? st : D-1-st) from (own state at D-1-st, partner state now)
        const double y0 = swap_pair(s0[r]), y1 = swap_pair(s1[r]);
        const double o0 = x0[r][D - 1 - st], o1 = x1[r][D - 1 - st];
        const bool unit = FAST && st == D - 1;  // own state is the boundary (1, 0)
        const double t0 = unit ? y0 : o0 * y0 + o1 * y1;
        const double t1 = unit ? y1 : o0 * y1 + o1 * y0;
        slots[base[r] + (odd ? st : D - 1 - st) * kIrrCnStride].x = clip_c2v<FAST>(div1<FAST, true>(t0, t0 + t1));
      }
    }
    if (advance) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const bool unit = FAST && st == 0;
        const double n0 = unit ? m0[r] : s0[r] * m0[r] + s1[r] * m1[r];
        const double n1 = unit ? m1[r] : s0[r] * m1[r] + s1[r] * m0[r];
        div2<FAST, true>(n0, n1, n0 + n1, s0[r], s1[r]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) sv[r] = s0[r];
}

// falling wave priorities over a phase's rounds (see bp_regular.hip);
// the levels are overridable for A/B builds
#ifndef KML_IRR_PRIO_VN_PAIR
#define KML_IRR_PRIO_VN_PAIR 3
#endif
#ifndef KML_IRR_PRIO_VN_SINGLE
#define KML_IRR_PRIO_VN_SINGLE 1
#endif
#ifndef KML_IRR_PRIO_CN_PAIR
#define KML_IRR_PRIO_CN_PAIR 2
#endif
#ifndef KML_IRR_CN_AGE_PRIO
#define KML_IRR_CN_AGE_PRIO 0
#endif
#ifndef KML_IRR_PRIO_CN_SINGLE
#define KML_IRR_PRIO_CN_SINGLE 0
#endif
__device__ __forceinline__ void set_prio(int p) {
  switch (p) {
    case 3: __builtin_amdgcn_s_setprio(3); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    default: __builtin_amdgcn_s_setprio(0); break;
  }
}

// Degree dispatch.  Paired (R = 2) instances exist up to the plan's pair
// limits (kIrrVnPairMax / kIrrCnPairMax): the register budget of three waves
// per SIMD holds two interleaved chains only up to those degrees.
template <int D, int R, bool FAST>
__device__ __forceinline__ void vn_cols_if(double2 *slots, const unsigned short *const (&cs)[R], const double (&p)[R],
                                           unsigned char *const (&h)[R], bool &sus) {
  if constexpr (R == 1 || D <= kIrrVnPairMax) vn_cols<D, R, FAST>(slots, cs, p, h, sus);
}
template <int R, bool FAST>
__device__ __forceinline__ void vn_any(int d, double2 *slots, const unsigned short *const (&cs)[R], const double (&p)[R],
                                       unsigned char *const (&h)[R], bool &sus) {
  switch (d) {
    case 1: vn_cols_if<1, R, FAST>(slots, cs, p, h, sus); break;
    case 2: vn_cols_if<2, R, FAST>(slots, cs, p, h, sus); break;
    case 3: vn_cols_if<3, R, FAST>(slots, cs, p, h, sus); break;
    case 4: vn_cols_if<4, R, FAST>(slots, cs, p, h, sus); break;
    case 5: vn_cols_if<5, R, FAST>(slots, cs, p, h, sus); break;
    case 6: vn_cols_if<6, R, FAST>(slots, cs, p, h, sus); break;
    case 7: vn_cols_if<7, R, FAST>(slots, cs, p, h, sus); break;
    case 8: vn_cols_if<8, R, FAST>(slots, cs, p, h, sus); break;
    default: vn_cols_if<9, R, FAST>(slots, cs, p, h, sus); break;
  }
}

template <int D, int R, bool SYN, bool FAST>
__device__ __forceinline__ void cn_halves_if(double2 *slots, const int (&base)[R], int odd, double (&sv)[R],
                                             unsigned (&par)[R]) {
  if constexpr (R == 1 || D <= kIrrCnPairMax) cn_halves<D, R, SYN, FAST>(slots, base, odd, sv, par);
}
template <int R, bool SYN, bool FAST>
__device__ __forceinline__ void cn_any(int d, double2 *slots, const int (&base)[R], int odd, double (&sv)[R],
                                       unsigned (&par)[R]) {
  switch (d) {
    case 2: cn_halves_if<2, R, SYN, FAST>(slots, base, odd, sv, par); break;
    case 3: cn_halves_if<3, R, SYN, FAST>(slots, base, odd, sv, par); break;
    case 4: cn_halves_if<4, R, SYN, FAST>(slots, base, odd, sv, par); break;
    case 5: cn_halves_if<5, R, SYN, FAST>(slots, base, odd, sv, par); break;
    case 6: cn_halves_if<6, R, SYN, FAST>(slots, base, odd, sv, par); break;
    case 7: cn_halves_if<7, R, SYN, FAST>(slots, base, odd, sv, par); break;
    case 8: cn_halves_if<8, R, SYN, FAST>(slots, base, odd, sv, par); break;
    case 9: cn_halves_if<9, R, SYN, FAST>(slots, base, odd, sv, par); break;
    default: cn_halves_if<10, R, SYN, FAST>(slots, base, odd, sv, par); break;
  }
}

// Phase timing (stamps build, -DKML_STAMPS=1; tools/irr_stamps.py): lane 0 of
// every wave sums its s_memtime deltas per phase of an iteration; the sums are
// flushed per wave at the end of each codeword: [0] VN paired round, [1] VN
// single round, [2] VN barrier wait, [3] parity, [4] CN paired round, [5] CN
// single round, [6] CN barrier wait (+ OR), [7] iterations run.
#ifndef KML_STAMPS
#define KML_STAMPS 0
#endif
#if KML_STAMPS
__device__ unsigned long long kml_irr_stamps[kIrrThreads / 64][8];
#define IRR_STAMP(i)                                               \
  do {                                                             \
    if ((threadIdx.x & 63) == 0) {                                 \
      const unsigned long long _t = __builtin_amdgcn_s_memtime();  \
      st_acc[(i)] += _t - st_prev;                                 \
      st_prev = _t;                                                \
    }                                                              \
  } while (0)
#else
#define IRR_STAMP(i) \
  do {               \
  } while (0)
#endif

// Column / row of the lane in round r of the plan (layout.hpp IrregularPlan):
// rounds 0 and 1 pair two items of one degree, round 2 holds single items.
// Returns true when a FAST decode met an unproven quotient (exact_div.hpp):
// the caller re-initialises the slots and redoes the codeword with FAST =
// false (decided at the CN closing barrier, before that iteration's
// syndromes are written; see bp_regular.hip decode_reg).
template <int T, bool SYN, bool FAST>
__device__ __forceinline__ bool decode_irr(const DevCode &c, const BpLaunch &a, int cw, double2 *slots,
                                           const unsigned short *cslot, const double *p0s, unsigned char *cch, int odd,
                                           const int (&vcol)[3], const int (&crow)[3], int &iter_out, bool &conv_out,
                                           bool sus0 = false) {
  // Each lane's plan packed into one word per round (slot base | degree << 14
  // | column or row << 18; ~0 = no item), built once per codeword: the
  // iteration loop makes no global loads.  The words are laundered at the top
  // of every iteration so that nothing derived from them is loop-invariant
  // (left invariant, LICM hoists per-degree offsets out of the loop and spills).
  unsigned vpk[3], cpk[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    vpk[r] = ~0u;
    cpk[r] = ~0u;
    if (vcol[r] >= 0) {
      const int b = c.col_ptr[vcol[r]];
      vpk[r] = (unsigned)b | (unsigned)(c.col_ptr[vcol[r] + 1] - b) << 14 | (unsigned)vcol[r] << 18;
    }
    if (crow[r] >= 0) {
      const int b = c.irr_cn_base[r * (T / 2) + (threadIdx.x >> 1)];
      const int d = c.row_ptr[crow[r] + 1] - c.row_ptr[crow[r]];
      cpk[r] = (unsigned)b | (unsigned)d << 14 | (unsigned)crow[r] << 18;
    }
  }
  auto pbase = [](unsigned w) { return (int)(w & 0x3FFFu); };
  auto pdeg = [](unsigned w) { return (int)((w >> 14) & 15u); };
  auto pitem = [](unsigned w) { return (int)(w >> 18); };
  __shared__ __attribute__((aligned(16))) int wflags[16];  // wg_any (bp_common.hpp)
  int iter = 0;
  bool conv = false, sus = sus0;
  auto prior = [&](int v) { return v >= c.punct ? p0s[v - c.punct] : 0.5; };  // :126-134
#if KML_STAMPS
  unsigned long long st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_prev = __builtin_amdgcn_s_memtime();
#endif
  for (; iter < a.iter_count; ++iter) {
    IRR_STAMP(6);
    unsigned vp[3], cp[3];
    int od = odd;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      vp[r] = vpk[r];
      cp[r] = cpk[r];
      asm volatile("" : "+v"(vp[r]), "+v"(cp[r]));
    }
    asm volatile("" : "+v"(od));
    set_prio(KML_IRR_PRIO_VN_PAIR);
    if (vp[0] != ~0u) {  // paired round: two columns of one degree, interleaved
      const int v0 = pitem(vp[0]), v1 = pitem(vp[1]);
      const unsigned short *const cs[2] = {cslot + pbase(vp[0]), cslot + pbase(vp[1])};
      const double p[2] = {prior(v0), prior(v1)};
      unsigned char *const h[2] = {&cch[v0], &cch[v1]};
      vn_any<2, FAST>(pdeg(vp[0]), slots, cs, p, h, sus);
    }
    IRR_STAMP(0);
    set_prio(KML_IRR_PRIO_VN_SINGLE);
    if (vp[2] != ~0u) {
      const int v = pitem(vp[2]);
      const unsigned short *const cs[1] = {cslot + pbase(vp[2])};
      const double p[1] = {prior(v)};
      unsigned char *const h[1] = {&cch[v]};
      vn_any<1, FAST>(pdeg(vp[2]), slots, cs, p, h, sus);
    }
    IRR_STAMP(1);
    __syncthreads();
    IRR_STAMP(2);

    // The early-stop parity of each row comes out of the CN pass (the row
    // halves' decisions ride in the v2c sign bits the chains load); the OR
    // over the workgroup is folded into the CN phase's closing barrier
    // (speculative CN, as in bp_regular.hip); syndromes are kept until the
    // phase is known to count.
    double sv[3] = {0.0, 0.0, 0.0};
    unsigned par[3] = {0u, 0u, 0u};
    IRR_STAMP(3);
#if KML_IRR_CN_AGE_PRIO  // (A/B) the CN pair round's priority by wave age (youngest third highest)
    set_prio(1 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) * 3 / (T / 64));
#else
    set_prio(KML_IRR_PRIO_CN_PAIR);
#endif
    if (cp[0] != ~0u) {  // both lanes of a pair agree
      const int base[2] = {pbase(cp[0]), pbase(cp[1])};
      double s2[2];
      unsigned p2[2];
      cn_any<2, SYN, FAST>(pdeg(cp[0]), slots, base, od, s2, p2);
      sv[0] = s2[0];
      sv[1] = s2[1];
      par[0] = p2[0];
      par[1] = p2[1];
    }
    IRR_STAMP(4);
    set_prio(KML_IRR_PRIO_CN_SINGLE);
    if (cp[2] != ~0u) {
      const int base[1] = {pbase(cp[2])};
      double s1[1];
      unsigned p1[1];
      cn_any<1, SYN, FAST>(pdeg(cp[2]), slots, base, od, s1, p1);
      sv[2] = s1[0];
      par[2] = p1[0];
    }
    int fail = 0;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      const int p = (int)(par[r] >> 31);
      const int full = p ^ swap_pair_i(p);
      if (cp[r] != ~0u) fail |= full;
    }
    IRR_STAMP(5);
    const int wg = FAST ? wg_any2<T / 64>(fail, sus, wflags) : wg_any<T / 64>(fail, wflags);
    if (FAST && (wg & 2)) {  // an unproven quotient in this VN phase: redo exactly
      iter_out = iter;
      conv_out = false;
      return true;
    }
    if (!(wg & 1)) {
      conv = true;
      break;
    }
    if constexpr (SYN) {
#pragma unroll
      for (int r = 0; r < 3; ++r)
        if (cp[r] != ~0u && !od) a.syn[(long long)cw * c.M + pitem(cp[r])] = sv[r];  // alpha past the last edge (:274)
    }
  }
  IRR_STAMP(6);
#if KML_STAMPS
  if ((threadIdx.x & 63) == 0) {
    st_acc[7] = iter;
    for (int i = 0; i < 8; ++i) atomicAdd(&kml_irr_stamps[threadIdx.x >> 6][i], st_acc[i]);
  }
#endif
  iter_out = iter;
  conv_out = conv;
  return false;
}

// EXACT = false: the FAST kernel (defers non-FAST and suspect codewords);
// EXACT = true: the exact path over the defer list (see bp_regular.hip).
template <int T, bool SYN, bool EXACT>
__global__ __launch_bounds__(T) void bp_irregular_kernel(DevCode c, BpLaunch a, unsigned int *queue, int fast_allowed) {
  const double plo = fast_prior_lo(c.dv_max);  // FAST prior domain (bp_common.hpp)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  __shared__ __attribute__((aligned(16))) int pflags[16];  // wg_all of the FAST prior check (bp_common.hpp)
  const int tid = threadIdx.x;
  const int odd = tid & 1;
  double2 *slots = reinterpret_cast<double2 *>(smem);
  const size_t sb = (size_t)c.irr_slots * 16;  // slot blocks (layout.hpp kIrrCnStride)
  double *p0s = reinterpret_cast<double *>(smem + sb);
  unsigned short *cslot = reinterpret_cast<unsigned short *>(smem + sb + (size_t)c.cc_len * 8);
  int *red = reinterpret_cast<int *>(smem + sb + (size_t)c.E * 2 + (size_t)c.cc_len * 8);
  unsigned char *cch = smem + sb + (size_t)c.E * 2 + (size_t)c.cc_len * 8 + kRedBytes;

  for (int e = tid; e < c.E; e += T) cslot[e] = (unsigned short)c.irr_col_slot[e];
  int vcol[3], crow[3];
#pragma unroll
  for (int r = 0; r < 3; ++r) {
    vcol[r] = c.irr_vn[r * T + tid];
    crow[r] = c.irr_cn[r * (T / 2) + (tid >> 1)];
  }

  const int B = a.B_dev ? (int)*a.B_dev : a.B;  // the exact kernel: the FAST kernel's defer count
  for (;;) {
    __syncthreads();
    if (tid == 0) {
      red[3] = (int)atomicAdd(queue, 1u);
      red[0] = 0;
      red[1] = 0;
    }
    __syncthreads();
    const int entry = red[3];
    if (entry >= B) break;
    const int cw = a.cw_idx ? a.cw_idx[entry] : entry;
    const double *p0 = a.p0 + (long long)cw * a.p0_stride;
    if (a.p0_sel) p0 += (long long)a.p0_sel[cw] * a.p0_sel_stride;

    bool ok = true;
    for (int i = tid; i < c.cc_len; i += T) {
      const double q = p0[i];
      p0s[i] = q;
      ok = ok && fast_prior_ok(q, plo);
    }
    for (int e = tid; e < c.irr_slots; e += T) slots[e].x = 0.5;  // InitMsg
    const bool fast = wg_all<T / 64>(ok ? 1 : 0, pflags) && (fast_allowed & 1);

    int iter = 0;
    bool conv = false;
    if constexpr (!EXACT) {
      bool defer = !fast;
      if (fast && decode_irr<T, SYN, true>(c, a, cw, slots, cslot, p0s, cch, odd, vcol, crow, iter, conv,
                                           (fast_allowed & 2) != 0)) {
        defer = true;  // an unproven quotient: the exact kernel redoes the codeword
        if (tid == 0 && a.counters) atomicAdd(&a.counters[CNT_REDONE], 1ull);
      }
      if (defer) {
        if (tid == 0) a.defer_idx[atomicAdd(a.defer_cnt, 1u)] = cw;
        continue;
      }
    } else {
      decode_irr<T, SYN, false>(c, a, cw, slots, cslot, p0s, cch, odd, vcol, crow, iter, conv);
    }

    if (a.iter_count > 0) {
      if (a.uu_hat) {
        uint8_t *u = a.uu_hat + (long long)cw * c.K;
        for (int i = tid; i < c.K; i += T) u[i] = cch[i + c.info_off];
      }
      if (a.cc_hat) {
        uint8_t *o = a.cc_hat + (long long)cw * c.N;
        for (int v = tid; v < c.N; v += T) o[v] = cch[v];
      }
      if (a.parity_cnt) {  // ParityCheck(cc_hat) (:281-300)
        int cnt = 0;
        for (int r = tid; r < c.M; r += T) {
          int p = 0;
          for (int e = c.row_ptr[r]; e < c.row_ptr[r + 1]; ++e) p ^= cch[c.row_col[e]];
          cnt += p;
        }
        if (cnt) atomicAdd(&red[0], cnt);
      }
      if (a.ref_bits) {
        const int errs =
            count_info_errors<T>(cch, nullptr, c.info_off, c.K, c.Kw, a.ref_bits + (long long)cw * c.Kw, tid);
        if (errs) atomicAdd(&red[1], errs);
      }
    }
    __syncthreads();
    if (tid == 0) {
      if (a.ret) a.ret[cw] = iter + (iter < a.max_iter);
      if (a.parity_cnt) a.parity_cnt[cw] = red[0];
      if (a.cw_err && a.ref_bits) a.cw_err[cw] = a.iter_count > 0 ? red[1] : 0;
      if (a.iters) a.iters[cw] = iter;
      if (a.counters) {
        const unsigned long long vn = conv ? (unsigned long long)iter + 1 : (unsigned long long)iter;
        atomicAdd(&a.counters[CNT_VN_PHASES], vn);
        atomicAdd(&a.counters[CNT_CN_PHASES], (unsigned long long)iter);
        if (conv) atomicAdd(&a.counters[CNT_CONVERGED], 1ull);
        if (a.ref_bits && a.iter_count > 0) {
          const int errs = red[1];
          atomicAdd(&a.counters[CNT_ERR_BIT], (unsigned long long)errs);
          atomicAdd(&a.counters[CNT_ERR_BLK], errs > 0 ? 1ull : 0ull);
          atomicAdd(&a.counters[CNT_TOT_BIT], (unsigned long long)c.K);
          atomicAdd(&a.counters[CNT_TOT_BLK], 1ull);
        }
      }
    }
  }
}

size_t irr_lds_bytes(const DevCode &c) {
  return (size_t)c.irr_slots * 16 + (size_t)c.E * 2 + (size_t)c.cc_len * 8 + kRedBytes + (size_t)c.N;
}

template <int T, bool SYN, bool EXACT>
hipError_t launch_irr_one(const DevCode &c, const BpLaunch &a, hipStream_t s, int fast_allowed) {
  auto kern = bp_irregular_kernel<T, SYN, EXACT>;
  const size_t lds = irr_lds_bytes(c);
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

// FAST kernel, then the exact kernel over its defer list (bp_regular.hip launch_reg_t)
template <int T, bool SYN>
hipError_t launch_irr_t(const DevCode &c, const BpLaunch &a, hipStream_t s, int fast_allowed) {
  if (!(fast_allowed & 1)) return launch_irr_one<T, SYN, true>(c, a, s, 0);
  if (!a.defer_idx || !a.defer_cnt) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(a.defer_cnt, 0, sizeof(unsigned), s);
  if (e != hipSuccess) return e;
  e = launch_irr_one<T, SYN, false>(c, a, s, fast_allowed);
  if (e != hipSuccess) return e;
  BpLaunch b = a;
  b.cw_idx = a.defer_idx;
  b.B_dev = a.defer_cnt;
  return launch_irr_one<T, SYN, true>(c, b, s, 0);
}

}  // namespace

hipError_t launch_bp_irregular(const DevCode &c, const BpLaunch &a, hipStream_t s) {
  constexpr int T = kIrrThreads;
  if (irr_lds_bytes(c) > 160 * 1024 || c.irr_slots > 16383) return hipErrorNotSupported;
  if (!c.irr_ok || !c.irr_vn) return hipErrorNotSupported;
  const int fast = bp_fast_mode(c);
  return a.syn ? launch_irr_t<T, true>(c, a, s, fast) : launch_irr_t<T, false>(c, a, s, fast);
}

}  // namespace kml

#if KML_STAMPS
extern "C" int kml_debug_irr_stamps(unsigned long long *out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(kml::kml_irr_stamps), sizeof(kml::kml_irr_stamps));
  if (reset) {
    unsigned long long zero[sizeof(kml::kml_irr_stamps) / 8] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(kml::kml_irr_stamps), zero, sizeof(zero));
  }
  return e == hipSuccess ? 0 : -3;
}
#endif

#if KML_DIV_STATS
KML_DIV_STATS_ACCESSOR(kml_debug_div_stats_irr)
#endif
