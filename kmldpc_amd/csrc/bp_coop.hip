// bp_coop.hip — BP decoder for regular (3, 6) codes whose message state does
// not fit one CU's LDS (PEG8064: 24,192 edges, 378 KiB of slots).
//
// Arithmetic: bit-exact restatement of lab::BinaryLDPCCodec::Decoder
// (lib/lab/src/binaryldpccodec.cc:165-278), like the other BP kernels.
//
// Mapping: a GROUP of kG workgroups on the same XCD decodes one codeword.
// Workgroup i runs on XCD i % 8, so groups are {i, i+8, i+16, i+24} + 32k and
// the group's 16-byte message slots (one per edge, in global memory) stay in
// that XCD's 4 MiB L2: 8 groups x 378 KiB = 3 MiB per XCD.  One workgroup per
// codeword (the generic kernel's global mode) puts 256 x 378 KiB in flight,
// which only the Infinity Cache holds, and the VN phase's gathers/scatters of
// 8- and 16-byte messages are then request-bound there.
//   * member m owns a quarter of the columns (in the planner's vn_order) and a
//     quarter of the rows; a thread owns RV columns and RC half-rows (the
//     lane-pair split of bp_regular.hip: even lane forward trellis, odd lane
//     backward, DPP swap of the chain states);
//   * the three phase boundaries of an iteration (VN done, parity flag known,
//     CN done) are group barriers: every wave waits for its stores
//     (vmcnt(0)), then one lane adds to a per-group arrival counter and polls
//     it with L1-bypassing loads.  Members share an XCD, so plain stores land
//     in the L2 every member reads: no L2 write-back is needed, and every
//     load of another member's data bypasses the (never refreshed) vector L1
//     (nontemporal loads).  Group members are checked to share an XCD
//     (HW_REG_XCC_ID) at start; a group that does not falls back to full
//     agent-scope fences (correct across XCDs, slower).  Every poll is
//     bounded: a stuck group raises an abort flag that ends every workgroup;
//   * the early-stop parity check ORs each member's failing-row flag into a
//     per-group word, alternating between two words per iteration;
//   * hard decisions live in a per-group byte array in global memory, indexed
//     by vn position so each wave stores 64 consecutive bytes.
// The launch is cooperative (every workgroup co-resident), which the group
// barriers require.
#include <cstdio>
#include <cstdlib>

#include <algorithm>

#include "bp_common.hpp"
#include "kernels.hpp"

namespace kml {

namespace {


struct GroupSync {
  unsigned bar;      // barrier arrivals (monotonic within a launch)
  unsigned flag[2];  // parity-failure flags, alternating per iteration
  unsigned cw;       // the group's current codeword (entry index)
  unsigned nofast;   // some member saw a prior outside the FAST division domain
  unsigned errs;     // error bits of the codeword, summed over members
  unsigned pcnt;     // unsatisfied checks of the final hard decisions, summed
  unsigned xcc;      // bit per XCD a member runs on
  // partitioned kernel: barrier counters by barrier parity, arrivals in the
  // low 32 bits, parity-failure reports in the high 32 bits (part_barrier)
  unsigned long long bar2[2];
};

constexpr int kPartG = 4;  // workgroups per codeword of the partitioned kernel

// LDS of the partitioned kernel: the member's row slots, its mirror slots, and
// every column's hard decision.
size_t part_lds_bytes(const DevCode &c) {
  return ((size_t)c.M / kPartG * 6 + (size_t)c.pt_mirror) * 16 + (size_t)c.N;
}

constexpr long long kSpinLimit = 20000000;  // ~1 s of s_sleep(1) polls

__device__ __forceinline__ unsigned ld_rlx(const unsigned *p) {  // L1-bypassing (sc1) load
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Group barrier.  Returns false when the launch is aborted (a poll timed out).
// same_xcd: members share an L2, plain stores + vmcnt(0) suffice; otherwise
// agent-scope release / acquire fences (L2 write-back / L1 invalidate).
template <int kG>
__device__ __forceinline__ bool group_barrier(GroupSync *gs, unsigned &gen, bool same_xcd, unsigned *abort) {
  if (same_xcd)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else
    __threadfence();
  __syncthreads();
  gen += kG;
  __shared__ int ok;
  if (threadIdx.x == 0) {
    if (!same_xcd) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __hip_atomic_fetch_add(&gs->bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int good = 1;
    for (long long spin = 0; ld_rlx(&gs->bar) < gen; ++spin) {
      if (spin > kSpinLimit || ld_rlx(abort)) {
        __hip_atomic_store(abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        good = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!same_xcd) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    ok = good;
  }
  __syncthreads();
  return ok != 0;
}

// loads of data other members wrote: bypass the vector L1
template <class T>
__device__ __forceinline__ T ld_nt(const T *p) {
  return __builtin_nontemporal_load(p);
}
typedef double nt_double2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ld_nt(const double2 *p) {
  const nt_double2 v = __builtin_nontemporal_load(reinterpret_cast<const nt_double2 *>(p));
  return make_double2(v.x, v.y);
}

__device__ __forceinline__ double swap_pair(double x) {
  const int lo = __double2loint(x), hi = __double2hiint(x);
  const int lo2 = __builtin_amdgcn_mov_dpp(lo, 0xB1, 0xF, 0xF, false);
  const int hi2 = __builtin_amdgcn_mov_dpp(hi, 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi2, lo2);
}
__device__ __forceinline__ int swap_pair_i(int x) { return __builtin_amdgcn_mov_dpp(x, 0xB1, 0xF, 0xF, false); }

// Per-launch control block shared by every workgroup.
struct CoopCtl {
  unsigned abort;  // a group barrier timed out: every workgroup exits
};

template <int kG, int RV, int RC, bool SYN, bool FAST>
__device__ __forceinline__ bool coop_iterations(const DevCode &c, const BpLaunch &a, int cw, GroupSync *gs,
                                                unsigned &gen, bool same_xcd, unsigned *abort, double2 *slots,
                                                uint8_t *gc, const int (&vpos)[RV], const int (&es)[RV][3],
                                                const bool (&vact)[RV], const double (&pv)[RV], const int (&crow)[RC],
                                                const int (&cbase)[RC], const int (&ccol)[RC][3],
                                                const bool (&cact)[RC], int odd, int member, int &iter_out,
                                                bool &conv_out) {
  constexpr int DV = 3, DC = 6, H = 3;
  int iter = 0;
  bool conv = false;
  for (; iter < a.iter_count; ++iter) {
    // ------------------------------------------------------------ VN phase
    // falling wave priorities within a phase (see bp_regular.hip)
    __builtin_amdgcn_s_setprio(3);
    {
      double c0s[RV][DV];
#pragma unroll
      for (int r = 0; r < RV; ++r)
#pragma unroll
        for (int k = 0; k < DV; ++k) c0s[r][k] = ld_nt(&slots[es[r][k]].x);
      double a0[RV], a1[RV], al0[RV][DV], al1[RV][DV];
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
          if (k + 1 < DV) {
            div2<FAST>(n0, n1, n0 + n1, a0[r], a1[r]);
          } else {
            const int hd = hard_decision<FAST>(n0, n1);
            if (vact[r]) gc[vpos[r]] = (unsigned char)hd;
          }
        }
      double b0[RV], b1[RV];
#pragma unroll
      for (int r = 0; r < RV; ++r) b0[r] = b1[r] = 1.0;
      __builtin_amdgcn_s_setprio(2);
#pragma unroll
      for (int k = DV - 1; k >= 0; --k) {
        if (k == DV - 2) __builtin_amdgcn_s_setprio(1);
        if (k == DV - 3) __builtin_amdgcn_s_setprio(0);
#pragma unroll
        for (int r = 0; r < RV; ++r) {
          const bool unit = FAST && k == DV - 1;
          const double t0 = unit ? al0[r][k] : al0[r][k] * b0[r];
          const double t1 = unit ? al1[r][k] : al1[r][k] * b1[r];
          double q0, q1;
          if (unit)  // beta = (1, 1): t is the normalised alpha, its sum within ulps of 1 (bp_common.hpp rcp_near1)
            div2<FAST, true>(t0, t1, t0 + t1, q0, q1);
          else
            div2<FAST>(t0, t1, t0 + t1, q0, q1);
          if (vact[r]) slots[es[r][k]] = make_double2(q0, q1);
          if (k > 0) {
            const double c0 = c0s[r][k];
            if (unit) {  // (c0, 1 - c0) / (c0 + (1 - c0)): the sum rounds to exactly 1 (bp_common.hpp)
              b0[r] = c0;
              b1[r] = 1.0 - c0;
            } else {
              div2<FAST>(b0[r] * c0, b1[r] * (1.0 - c0), b0[r] * c0 + b1[r] * (1.0 - c0), b0[r], b1[r]);
            }
          }
        }
      }
    }
    if (!group_barrier<kG>(gs, gen, same_xcd, abort)) return false;

    // -------------------- early-stop parity check, folded into the CN barrier
    // Every member ORs its failing-row flag now and runs the CN phase
    // speculatively; the flag is read after the CN barrier.  A converged
    // codeword's speculative CN results (slots) are never read again, and its
    // syndromes are only written when the phase counts.
    {
      int fail = 0;
#pragma unroll
      for (int r = 0; r < RC; ++r) {
        int p = 0;
#pragma unroll
        for (int k = 0; k < H; ++k) p ^= ld_nt(&gc[ccol[r][k]]);
        fail |= cact[r] ? (p ^ swap_pair_i(p)) : 0;
      }
      if (__ballot(fail) != 0 && (threadIdx.x & 63) == 0)
        __hip_atomic_fetch_or(&gs->flag[iter & 1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }

    // ------------------------------------------------------------ CN phase
    // Step st: loads first, the c2v of this step from the swapped states, the
    // chain update (which waits for the loads), and only then the c2v stores:
    // the partner lane's load of the slot stored here has completed by then.
    double syn0[RC];
    {
      double x0[RC][H], x1[RC][H];
      double s0[RC], s1[RC];
#pragma unroll
      for (int r = 0; r < RC; ++r) {
        s0[r] = 1.0;
        s1[r] = 0.0;
      }
      __builtin_amdgcn_s_setprio(2);
#pragma unroll
      for (int st = 0; st < DC; ++st) {
        if (st == 2) __builtin_amdgcn_s_setprio(1);
        if (st == 4) __builtin_amdgcn_s_setprio(0);
        const bool advance = SYN || st + 1 < DC;
        double m0[RC], m1[RC];
        if (advance) {
#pragma unroll
          for (int r = 0; r < RC; ++r) {
            const double2 m = ld_nt(&slots[cbase[r] + (odd ? DC - 1 - st : st)]);
            m0[r] = m.x;
            m1[r] = m.y;
          }
        }
        double q[RC];
#pragma unroll
        for (int r = 0; r < RC; ++r) {
          q[r] = 0.0;
          if (st < H) {
            x0[r][st] = s0[r];
            x1[r][st] = s1[r];
          } else {
            const double y0 = swap_pair(s0[r]);
            const double y1 = swap_pair(s1[r]);
            const double o0 = x0[r][DC - 1 - st], o1 = x1[r][DC - 1 - st];
            const bool unit = FAST && st == DC - 1;
            const double t0 = unit ? y0 : o0 * y0 + o1 * y1;
            const double t1 = unit ? y1 : o0 * y1 + o1 * y0;
            q[r] = clip_c2v<FAST>(div1<FAST, true>(t0, t0 + t1));
          }
        }
        if (advance) {
#pragma unroll
          for (int r = 0; r < RC; ++r) {
            const bool unit = FAST && st == 0;
            const double n0 = unit ? m0[r] : s0[r] * m0[r] + s1[r] * m1[r];
            const double n1 = unit ? m1[r] : s0[r] * m1[r] + s1[r] * m0[r];
            div2<FAST, true>(n0, n1, n0 + n1, s0[r], s1[r]);
          }
        }
        if (st >= H) {
#pragma unroll
          for (int r = 0; r < RC; ++r)
            if (cact[r]) slots[cbase[r] + (odd ? st : DC - 1 - st)].x = q[r];
        }
      }
#pragma unroll
      for (int r = 0; r < RC; ++r) syn0[r] = s0[r];
    }
    if (!group_barrier<kG>(gs, gen, same_xcd, abort)) return false;
    if (!ld_rlx(&gs->flag[iter & 1])) {  // every row satisfied: stop before this CN phase
      conv = true;
      break;
    }
    if (member == 0 && threadIdx.x == 0)  // cleared before anyone can OR into it (next VN barrier)
      __hip_atomic_store(&gs->flag[(iter + 1) & 1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if constexpr (SYN) {
#pragma unroll
      for (int r = 0; r < RC; ++r)
        if (cact[r] && !odd) a.syn[(long long)cw * c.M + crow[r]] = syn0[r];  // alpha past the last edge (:274)
    }
  }
  iter_out = iter;
  conv_out = conv;
  return true;
}

template <int kG, int T, int RV, int RC, bool SYN>
__global__ __launch_bounds__(T) void bp_coop_kernel(DevCode c, BpLaunch a, GroupSync *gsync, uint8_t *gcch,
                                                    unsigned *abort, unsigned int *queue, int fast_allowed) {
  const int tid = threadIdx.x;
  const int odd = tid & 1;
  const int member = (blockIdx.x >> 3) % kG;
  const int group = (blockIdx.x / (8 * kG)) * 8 + (blockIdx.x & 7);
  GroupSync *gs = gsync + group;
  double2 *slots = a.gslots + (size_t)group * c.E;
  uint8_t *gc = gcch + (size_t)group * c.N;

  // static assignment: member m owns vn positions [v_lo, v_hi) and rows [r_lo, r_hi);
  // every index the iterations use is register-resident
  const int v_lo = (int)((long long)c.N * member / kG), v_hi = (int)((long long)c.N * (member + 1) / kG);
  const int r_lo = (int)((long long)c.M * member / kG), r_hi = (int)((long long)c.M * (member + 1) / kG);
  int vpos[RV], vcol[RV], es[RV][3];
  bool vact[RV];
#pragma unroll
  for (int r = 0; r < RV; ++r) {
    const int p = v_lo + r * T + tid;
    vact[r] = p < v_hi;
    vpos[r] = vact[r] ? p : v_lo;
    vcol[r] = c.vn_order[vpos[r]];
    const int b = c.col_ptr[vcol[r]];
#pragma unroll
    for (int k = 0; k < 3; ++k) es[r][k] = c.col_slot[b + k];
  }
  int crow[RC], cbase[RC], ccol[RC][3];
  bool cact[RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int q = r_lo + ((r * T + tid) >> 1);  // lane pairs share a row
    cact[r] = q < r_hi;
    crow[r] = c.cn_order[cact[r] ? q : r_lo];
    cbase[r] = c.row_ptr[crow[r]];
#pragma unroll
    for (int k = 0; k < 3; ++k) ccol[r][k] = c.reg_pos[c.row_col[cbase[r] + (odd ? 3 + k : k)]];
  }

  // do the group's members share an XCD (one L2)?  HW_REG_XCC_ID, bits [3:0]
  unsigned gen = 0;
  if (tid == 0) {
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;
    __hip_atomic_fetch_or(&gs->xcc, 1u << xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!group_barrier<kG>(gs, gen, false, abort)) return;
  const bool same_xcd = __popc(ld_rlx(&gs->xcc)) == 1;

  for (;;) {
    if (member == 0 && tid == 0) {
      __hip_atomic_store(&gs->cw, atomicAdd(queue, 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&gs->nofast, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&gs->errs, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&gs->pcnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&gs->flag[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&gs->flag[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (!group_barrier<kG>(gs, gen, same_xcd, abort)) return;
    const int entry = (int)ld_rlx(&gs->cw);
    if (entry >= a.B) break;
    const int cw = a.cw_idx ? a.cw_idx[entry] : entry;
    const double *p0 = a.p0 + (long long)cw * a.p0_stride;
    if (a.p0_sel) p0 += (long long)a.p0_sel[cw] * a.p0_sel_stride;

    double pv[RV];
    bool ok = true;
#pragma unroll
    for (int r = 0; r < RV; ++r) {
      pv[r] = (vcol[r] >= c.punct) ? p0[vcol[r] - c.punct] : 0.5;
      ok = ok && fast_prior_ok(pv[r]);
    }
    // InitMsg on this member's share of the slots
    {
      const int e_lo = (int)((long long)c.E * member / kG), e_hi = (int)((long long)c.E * (member + 1) / kG);
      for (int e = e_lo + tid; e < e_hi; e += T) slots[e].x = 0.5;
    }
    if (__ballot(!ok) != 0 && (tid & 63) == 0)
      __hip_atomic_fetch_or(&gs->nofast, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!group_barrier<kG>(gs, gen, same_xcd, abort)) return;
    const bool fast = fast_allowed && !ld_rlx(&gs->nofast);

    int iter = 0;
    bool conv = false;
    bool alive;
    if (fast)
      alive = coop_iterations<kG, RV, RC, SYN, true>(c, a, cw, gs, gen, same_xcd, abort, slots, gc, vpos, es, vact,
                                                     pv, crow, cbase, ccol, cact, odd, member, iter, conv);
    else
      alive = coop_iterations<kG, RV, RC, SYN, false>(c, a, cw, gs, gen, same_xcd, abort, slots, gc, vpos, es, vact,
                                                      pv, crow, cbase, ccol, cact, odd, member, iter, conv);
    if (!alive) return;

    // ---- outputs: every member writes its share; member 0 the scalars
    if (a.iter_count > 0) {
      if (a.uu_hat) {
        uint8_t *u = a.uu_hat + (long long)cw * c.K;
        const int lo = (int)((long long)c.K * member / kG), hi = (int)((long long)c.K * (member + 1) / kG);
        for (int i = lo + tid; i < hi; i += T) u[i] = ld_nt(&gc[c.reg_pos[i + c.info_off]]);
      }
      if (a.cc_hat) {
        uint8_t *o = a.cc_hat + (long long)cw * c.N;
        for (int v = v_lo + tid; v < v_hi; v += T) o[c.vn_order[v]] = ld_nt(&gc[v]);
      }
      if (a.parity_cnt) {
        int cnt = 0;
#pragma unroll
        for (int r = 0; r < RC; ++r) {
          int p = 0;
#pragma unroll
          for (int k = 0; k < 3; ++k) p ^= ld_nt(&gc[ccol[r][k]]);
          const int full = p ^ swap_pair_i(p);
          if (!odd && cact[r]) cnt += full;
        }
        if (cnt) __hip_atomic_fetch_add(&gs->pcnt, (unsigned)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (a.ref_bits) {
        const uint64_t *ref = a.ref_bits + (long long)cw * c.Kw;
        const int lo = (int)((long long)c.Kw * member / kG), hi = (int)((long long)c.Kw * (member + 1) / kG);
        int errs = 0;
        for (int w = lo + tid; w < hi; w += T) {
          uint64_t word = 0;
          const int base = w * 64;
          const int nb = min(64, c.K - base);
          for (int j = 0; j < nb; ++j) word |= (uint64_t)ld_nt(&gc[c.reg_pos[c.info_off + base + j]]) << j;
          errs += __popcll(word ^ ref[w]);
        }
        if (errs) __hip_atomic_fetch_add(&gs->errs, (unsigned)errs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (!group_barrier<kG>(gs, gen, same_xcd, abort)) return;  // the members' sums are complete
    if (member == 0 && tid == 0) {
      const int errs = (int)ld_rlx(&gs->errs);
      const int pcnt = (int)ld_rlx(&gs->pcnt);
      if (a.ret) a.ret[cw] = iter + (iter < a.max_iter);
      if (a.iters) a.iters[cw] = iter;
      if (a.parity_cnt) a.parity_cnt[cw] = a.iter_count > 0 ? pcnt : 0;
      if (a.cw_err && a.ref_bits) a.cw_err[cw] = a.iter_count > 0 ? errs : 0;
      if (a.counters) {
        const unsigned long long vn = conv ? (unsigned long long)iter + 1 : (unsigned long long)iter;
        atomicAdd(&a.counters[CNT_VN_PHASES], vn);
        atomicAdd(&a.counters[CNT_CN_PHASES], (unsigned long long)iter);
        if (conv) atomicAdd(&a.counters[CNT_CONVERGED], 1ull);
        if (a.ref_bits && a.iter_count > 0) {
          atomicAdd(&a.counters[CNT_ERR_BIT], (unsigned long long)errs);
          atomicAdd(&a.counters[CNT_ERR_BLK], errs > 0 ? 1ull : 0ull);
          atomicAdd(&a.counters[CNT_TOT_BIT], (unsigned long long)c.K);
          atomicAdd(&a.counters[CNT_TOT_BLK], 1ull);
        }
      }
    }
  }
}

#ifdef KML_STAMPS
// Phase timing of the partitioned kernel (a KML_STAMPS=1 build only): wave 0
// of every workgroup adds s_memtime deltas per phase of its iterations.
constexpr int kStampSlots = 10;
__device__ unsigned long long kml_part_stamps[256 * kStampSlots];
#define KML_STAMP(i)                                                                   \
  do {                                                                                 \
    const unsigned long long _t = __builtin_amdgcn_s_memtime();                        \
    if (threadIdx.x == 0 && blockIdx.x < 256)                                          \
      atomicAdd(&kml_part_stamps[blockIdx.x * kStampSlots + (i)], _t - stamp_prev);    \
    stamp_prev = _t;                                                                   \
  } while (0)
#else
#define KML_STAMP(i) \
  do {               \
  } while (0)
#endif

// Group barrier of the partitioned kernel, which also ORs the members'
// early-stop flags: each member adds 1 + (its flag << 32) to the counter of
// this barrier's parity (no member can reach the next barrier of the same
// parity before every member has passed this one, so the value a poller sees
// holds exactly this barrier's arrivals).  st (LDS, thread 0 only): expected
// arrivals and flag totals seen, per parity.  Returns the number of members
// that reported a flag, or -1 when the launch aborts.  The abort word is read
// every 64 polls only, so a poll costs one L2 round trip.
__device__ __forceinline__ unsigned long long ld_rlx64(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <int kG>
__device__ __forceinline__ int part_barrier(GroupSync *gs, unsigned long long *st, unsigned &nb, bool same_xcd,
                                            unsigned *abort, int *flag) {
  if (same_xcd)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else
    __threadfence();
  __syncthreads();
  const int p = nb & 1;
  ++nb;
  __shared__ int res;
  if (threadIdx.x == 0) {
    if (!same_xcd) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    unsigned long long add = 1;
    if (flag) {
      if (*flag) add += 1ull << 32;
      *flag = 0;  // the next reports follow this barrier
    }
    st[p] += kG;
    __hip_atomic_fetch_add(&gs->bar2[p], add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int r = 0;
    unsigned long long v;
    for (long long spin = 0;; ++spin) {
      v = ld_rlx64(&gs->bar2[p]);
      if ((unsigned)v >= (unsigned)st[p]) break;
      if ((spin & 63) == 63 && (spin > kSpinLimit || ld_rlx(abort))) {
        __hip_atomic_store(abort, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        r = -1;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (r == 0) {
      const unsigned f = (unsigned)(v >> 32);
      r = (int)(f - (unsigned)st[2 + p]);
      st[2 + p] = f;
    }
    if (!same_xcd) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    res = r;
  }
  __syncthreads();
  return res;
}

// ===========================================================================
// Partitioned cooperative kernel (bp_part_kernel): the group mapping and the
// group barriers above, but every message access of the arithmetic is an LDS
// access.  Member m keeps the 16-byte slots of ITS rows in LDS, plus one
// MIRROR slot per cut edge of its columns (an edge whose row another member
// owns; layout.hpp PartitionPlan).  The planner's partition cuts ~27% of
// PEG8064's edges; those messages cross members through two mailboxes in the
// group's global scratch, copied by short coalesced loops around the group
// barriers:
//   VN compute (row slots + mirrors) -> send v2c (mirrors -> v2c mailbox)
//   -> barrier -> receive v2c (mailbox -> row slots) and the other members'
//   hard decisions -> parity check + CN compute (row slots) -> send c2v (row
//   slots -> c2v mailbox) -> barrier -> receive c2v (mailbox -> mirrors).
// The global-slot kernel above gathers and scatters every edge's message
// through the XCD's L2 at 8-16 bytes per lane, which bounds its iterations
// by the L2 request rate; here the exchange moves ~24 bytes per cut edge per
// iteration in mostly contiguous runs.

template <int kG, int RV, int RC, int RX, bool SYN, bool FAST>
__device__ __forceinline__ bool part_iterations(const BpLaunch &a, int M, int N, int NG, int cw, GroupSync *gs,
                                                unsigned long long *bst, unsigned &nb, int *sfail, bool same_xcd,
                                                unsigned *abort, unsigned char *smem,
                                                uint8_t *dec, double2 *mb_v2c, double *mb_c2v, uint8_t *gc,
                                                const int (&vaddr)[RV][3], const int (&vpos)[RV],
                                                const bool (&vact)[RV], const double (&pv)[RV], const int (&crow)[RC],
                                                const int (&cbase)[RC], const int (&ccol)[RC][3],
                                                const bool (&cact)[RC], const int (&xr)[RX], const int (&xc)[RX],
                                                int odd, int member, int &iter_out, bool &conv_out) {
  constexpr int DV = 3, DC = 6, H = 3;
  const int tid = threadIdx.x;
  double2 *slots = reinterpret_cast<double2 *>(smem);
  int iter = 0;
  bool conv = false;
#ifdef KML_STAMPS
  unsigned long long stamp_prev = __builtin_amdgcn_s_memtime();
#endif
  for (; iter < a.iter_count; ++iter) {
    KML_STAMP(0);  // iteration boundary
    // ---------------------------------- receive c2v of the cut edges (mirrors)
    if (iter > 0) {  // iteration 0 reads InitMsg's 0.5
#pragma unroll
      for (int q = 0; q < RX; ++q)
        if (xc[q] >= 0) *reinterpret_cast<double *>(smem + (xc[q] & 0xFFFF) * 16) = ld_nt(&mb_c2v[xc[q] >> 16]);
      __syncthreads();
    }
    KML_STAMP(1);  // receive c2v
    // ------------------------------------------------------------ VN phase
    __builtin_amdgcn_s_setprio(3);
    {
      double c0s[RV][DV];
#pragma unroll
      for (int r = 0; r < RV; ++r)
#pragma unroll
        for (int k = 0; k < DV; ++k) c0s[r][k] = *reinterpret_cast<const double *>(smem + vaddr[r][k]);
      double a0[RV], a1[RV], al0[RV][DV], al1[RV][DV];
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
          if (k + 1 < DV) {
            div2<FAST>(n0, n1, n0 + n1, a0[r], a1[r]);
          } else {
            const int hd = hard_decision<FAST>(n0, n1);
            if (vact[r]) {
              dec[vpos[r]] = (unsigned char)hd;
              gc[vpos[r]] = (unsigned char)hd;
            }
          }
        }
      double b0[RV], b1[RV];
#pragma unroll
      for (int r = 0; r < RV; ++r) b0[r] = b1[r] = 1.0;
      __builtin_amdgcn_s_setprio(2);
#pragma unroll
      for (int k = DV - 1; k >= 0; --k) {
        if (k == DV - 2) __builtin_amdgcn_s_setprio(1);
        if (k == DV - 3) __builtin_amdgcn_s_setprio(0);
#pragma unroll
        for (int r = 0; r < RV; ++r) {
          const bool unit = FAST && k == DV - 1;
          const double t0 = unit ? al0[r][k] : al0[r][k] * b0[r];
          const double t1 = unit ? al1[r][k] : al1[r][k] * b1[r];
          double q0, q1;
          if (unit)  // beta = (1, 1): t is the normalised alpha, its sum within ulps of 1 (bp_common.hpp rcp_near1)
            div2<FAST, true>(t0, t1, t0 + t1, q0, q1);
          else
            div2<FAST>(t0, t1, t0 + t1, q0, q1);
          if (vact[r]) *reinterpret_cast<double2 *>(smem + vaddr[r][k]) = make_double2(q0, q1);
          if (k > 0) {
            const double c0 = c0s[r][k];
            if (unit) {  // the sum rounds to exactly 1 (bp_common.hpp)
              b0[r] = c0;
              b1[r] = 1.0 - c0;
            } else {
              div2<FAST>(b0[r] * c0, b1[r] * (1.0 - c0), b0[r] * c0 + b1[r] * (1.0 - c0), b0[r], b1[r]);
            }
          }
        }
      }
    }
    KML_STAMP(2);  // VN compute (wave 0)
    // ---------------------------------------------- send v2c of the cut edges
    __syncthreads();
    KML_STAMP(3);  // VN drain (other waves)
#pragma unroll
    for (int q = 0; q < RX; ++q)
      if (xc[q] >= 0) mb_v2c[xc[q] >> 16] = slots[xc[q] & 0xFFFF];
    if (part_barrier<kG>(gs, bst, nb, same_xcd, abort, nullptr) < 0) return false;
    KML_STAMP(4);  // send v2c + group barrier

    // ------------------- receive v2c and the other members' hard decisions
#pragma unroll
    for (int q = 0; q < RX; ++q)
      if (xr[q] >= 0) slots[xr[q] & 0xFFFF] = ld_nt(&mb_v2c[xr[q] >> 16]);
    for (int i = tid; i < (kG - 1) * (NG / 16); i += blockDim.x) {
      int m = i / (NG / 16);
      const int off = (m + (m >= member)) * NG + (i - m * (NG / 16)) * 16;
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(gc + off));
      *reinterpret_cast<u32x4 *>(dec + off) = v;
    }
    __syncthreads();
    KML_STAMP(5);  // receive v2c + decisions

    // -------------------- early-stop parity check, folded into the CN barrier
    {
      int fail = 0;
#pragma unroll
      for (int r = 0; r < RC; ++r) {
        int p = 0;
#pragma unroll
        for (int k = 0; k < H; ++k) p ^= dec[ccol[r][k]];
        fail |= cact[r] ? (p ^ swap_pair_i(p)) : 0;
      }
      if (__ballot(fail) != 0 && (tid & 63) == 0) atomicOr(sfail, 1);  // reported at the CN barrier
    }

    // ------------------------------------------------------------ CN phase
    // (bp_regular.hip's step order: every load of a step before its stores)
    double syn0[RC];
    {
      double x0[RC][H], x1[RC][H];
      double s0[RC], s1[RC];
#pragma unroll
      for (int r = 0; r < RC; ++r) {
        s0[r] = 1.0;
        s1[r] = 0.0;
      }
      __builtin_amdgcn_s_setprio(2);
#pragma unroll
      for (int st = 0; st < DC; ++st) {
        if (st == 2) __builtin_amdgcn_s_setprio(1);
        if (st == 4) __builtin_amdgcn_s_setprio(0);
        const bool advance = SYN || st + 1 < DC;
        double m0[RC], m1[RC];
        if (advance) {
#pragma unroll
          for (int r = 0; r < RC; ++r) {
            const double2 m = *reinterpret_cast<const double2 *>(smem + cbase[r] + (odd ? DC - 1 - st : st) * 16);
            m0[r] = m.x;
            m1[r] = m.y;
          }
        }
#pragma unroll
        for (int r = 0; r < RC; ++r) {
          if (st < H) {
            x0[r][st] = s0[r];
            x1[r][st] = s1[r];
          } else {
            const double y0 = swap_pair(s0[r]);
            const double y1 = swap_pair(s1[r]);
            const double o0 = x0[r][DC - 1 - st], o1 = x1[r][DC - 1 - st];
            const bool unit = FAST && st == DC - 1;
            const double t0 = unit ? y0 : o0 * y0 + o1 * y1;
            const double t1 = unit ? y1 : o0 * y1 + o1 * y0;
            const double q = clip_c2v<FAST>(div1<FAST, true>(t0, t0 + t1));
            if (cact[r]) *reinterpret_cast<double *>(smem + cbase[r] + (odd ? st : DC - 1 - st) * 16) = q;
          }
        }
        if (advance) {
#pragma unroll
          for (int r = 0; r < RC; ++r) {
            const bool unit = FAST && st == 0;
            const double n0 = unit ? m0[r] : s0[r] * m0[r] + s1[r] * m1[r];
            const double n1 = unit ? m1[r] : s0[r] * m1[r] + s1[r] * m0[r];
            div2<FAST, true>(n0, n1, n0 + n1, s0[r], s1[r]);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < RC; ++r) syn0[r] = s0[r];
    }
    KML_STAMP(6);  // parity + CN compute (wave 0)
    // ---------------------------------------------- send c2v of the cut edges
    __syncthreads();
    KML_STAMP(7);  // CN drain (other waves)
#pragma unroll
    for (int q = 0; q < RX; ++q)
      if (xr[q] >= 0) mb_c2v[xr[q] >> 16] = slots[xr[q] & 0xFFFF].x;
    const int failing = part_barrier<kG>(gs, bst, nb, same_xcd, abort, sfail);
    KML_STAMP(8);  // send c2v + group barrier
    if (failing < 0) return false;
    if (failing == 0) {  // every row satisfied: stop before this CN phase
      conv = true;
      break;
    }
    if constexpr (SYN) {
#pragma unroll
      for (int r = 0; r < RC; ++r)
        if (cact[r] && !odd) a.syn[(long long)cw * M + crow[r]] = syn0[r];  // alpha past the last edge (:274)
    }
  }
  iter_out = iter;
  conv_out = conv;
  return true;
}

template <int kG, int T, int RV, int RC, int RX, bool SYN>
__global__ __launch_bounds__(T) void bp_part_kernel(DevCode c, BpLaunch a, GroupSync *gsync, uint8_t *gcch,
                                                    unsigned *abort, unsigned int *queue, int fast_allowed) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int DV = 3, DC = 6, H = 3;
  const int tid = threadIdx.x;
  const int odd = tid & 1;
  const int member = (blockIdx.x >> 3) % kG;
  const int group = (blockIdx.x / (8 * kG)) * 8 + (blockIdx.x & 7);
  GroupSync *gs = gsync + group;
  const int MG = c.M / kG, NG = c.N / kG, EG = MG * DC;
  double2 *mb_v2c = a.gslots + (size_t)group * c.E;       // [ncut] double2
  double *mb_c2v = reinterpret_cast<double *>(mb_v2c + c.pt_ncut);  // [ncut] double
  uint8_t *gc = gcch + (size_t)group * c.N;
  const int nslots = EG + c.pt_mirror;
  uint8_t *dec = smem + (size_t)nslots * 16;  // N hard decisions, plan order

  int vaddr[RV][DV], vpos[RV];
  bool vact[RV];
#pragma unroll
  for (int r = 0; r < RV; ++r) {
    const int i = r * T + tid;
    vact[r] = i < NG;
    vpos[r] = member * NG + (vact[r] ? i : 0);
#pragma unroll
    for (int k = 0; k < DV; ++k) vaddr[r][k] = c.pt_vaddr[vpos[r] * DV + k];
  }
  int crow[RC], cbase[RC], ccol[RC][H];
  bool cact[RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int i = (r * T + tid) >> 1;  // lane pairs share a row
    cact[r] = i < MG;
    const int li = cact[r] ? i : 0;
    const int row = c.pt_cn[member * MG + li];
    crow[r] = row;
    cbase[r] = li * DC * 16;
#pragma unroll
    for (int k = 0; k < H; ++k) ccol[r][k] = c.pt_pos[c.row_col[c.row_ptr[row] + (odd ? H + k : k)]];
  }
  int xr[RX], xc[RX];
  {
    const int r0 = c.pt_xr_ptr[member], r1 = c.pt_xr_ptr[member + 1];
    const int c0 = c.pt_xc_ptr[member], c1 = c.pt_xc_ptr[member + 1];
#pragma unroll
    for (int q = 0; q < RX; ++q) {
      const int i = q * T + tid;
      xr[q] = r0 + i < r1 ? c.pt_xr[r0 + i] : -1;
      xc[q] = c0 + i < c1 ? c.pt_xc[c0 + i] : -1;
    }
  }

  __shared__ unsigned long long bst[4];  // part_barrier state (thread 0)
  __shared__ int sfail;                  // this member's early-stop flag (parity failures)
  unsigned nb = 0;                       // barrier sequence number (uniform, same on every member)
  if (tid == 0) {
    bst[0] = bst[1] = bst[2] = bst[3] = 0;
    sfail = 0;
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;
    __hip_atomic_fetch_or(&gs->xcc, 1u << xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (part_barrier<kG>(gs, bst, nb, false, abort, nullptr) < 0) return;
  const bool same_xcd = __popc(ld_rlx(&gs->xcc)) == 1;

  for (;;) {
    if (member == 0 && tid == 0) {
      __hip_atomic_store(&gs->cw, atomicAdd(queue, 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&gs->nofast, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&gs->errs, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&gs->pcnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (part_barrier<kG>(gs, bst, nb, same_xcd, abort, nullptr) < 0) return;
    const int entry = (int)ld_rlx(&gs->cw);
    if (entry >= a.B) break;
    const int cw = a.cw_idx ? a.cw_idx[entry] : entry;
    const double *p0 = a.p0 + (long long)cw * a.p0_stride;
    if (a.p0_sel) p0 += (long long)a.p0_sel[cw] * a.p0_sel_stride;

    double pv[RV];
    bool ok = true;
#pragma unroll
    for (int r = 0; r < RV; ++r) {
      const int col = c.pt_vn[vpos[r]];
      pv[r] = (col >= c.punct) ? p0[col - c.punct] : 0.5;
      ok = ok && fast_prior_ok(pv[r]);
    }
    // InitMsg: row slots and mirror slots (c2v = 0.5)
    for (int e = tid; e < nslots; e += T) reinterpret_cast<double2 *>(smem)[e] = make_double2(0.5, 0.5);
    if (__ballot(!ok) != 0 && (tid & 63) == 0)
      __hip_atomic_fetch_or(&gs->nofast, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (part_barrier<kG>(gs, bst, nb, same_xcd, abort, nullptr) < 0) return;
    const bool fast = fast_allowed && !ld_rlx(&gs->nofast);

    int iter = 0;
    bool conv = false;
    bool alive;
    if (fast)
      alive = part_iterations<kG, RV, RC, RX, SYN, true>(a, c.M, c.N, NG, cw, gs, bst, nb, &sfail, same_xcd, abort, smem, dec,
                                                         mb_v2c, mb_c2v, gc, vaddr, vpos, vact, pv, crow, cbase, ccol,
                                                         cact, xr, xc, odd, member, iter, conv);
    else
      alive = part_iterations<kG, RV, RC, RX, SYN, false>(a, c.M, c.N, NG, cw, gs, bst, nb, &sfail, same_xcd, abort, smem, dec,
                                                          mb_v2c, mb_c2v, gc, vaddr, vpos, vact, pv, crow, cbase,
                                                          ccol, cact, xr, xc, odd, member, iter, conv);
    if (!alive) return;

    // ---- outputs: every member holds all hard decisions in LDS (dec) and
    // writes its share; member 0 the scalars
    if (a.iter_count > 0) {
      if (a.uu_hat) {
        uint8_t *u = a.uu_hat + (long long)cw * c.K;
        const int lo = (int)((long long)c.K * member / kG), hi = (int)((long long)c.K * (member + 1) / kG);
        for (int i = lo + tid; i < hi; i += T) u[i] = dec[c.pt_pos[i + c.info_off]];
      }
      if (a.cc_hat) {
        uint8_t *o = a.cc_hat + (long long)cw * c.N;
        for (int v = member * NG + tid; v < (member + 1) * NG; v += T) o[c.pt_vn[v]] = dec[v];
      }
      if (a.parity_cnt) {
        int cnt = 0;
#pragma unroll
        for (int r = 0; r < RC; ++r) {
          int p = 0;
#pragma unroll
          for (int k = 0; k < H; ++k) p ^= dec[ccol[r][k]];
          const int full = p ^ swap_pair_i(p);
          if (!odd && cact[r]) cnt += full;
        }
        if (cnt) __hip_atomic_fetch_add(&gs->pcnt, (unsigned)cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (a.ref_bits) {
        const uint64_t *ref = a.ref_bits + (long long)cw * c.Kw;
        const int lo = (int)((long long)c.Kw * member / kG), hi = (int)((long long)c.Kw * (member + 1) / kG);
        int errs = 0;
        for (int w = lo + tid; w < hi; w += T) {
          uint64_t word = 0;
          const int base = w * 64;
          const int nb = min(64, c.K - base);
          for (int j = 0; j < nb; ++j) word |= (uint64_t)dec[c.pt_pos[c.info_off + base + j]] << j;
          errs += __popcll(word ^ ref[w]);
        }
        if (errs) __hip_atomic_fetch_add(&gs->errs, (unsigned)errs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (part_barrier<kG>(gs, bst, nb, same_xcd, abort, nullptr) < 0) return;  // the members' sums are complete
    if (member == 0 && tid == 0) {
      const int errs = (int)ld_rlx(&gs->errs);
      const int pcnt = (int)ld_rlx(&gs->pcnt);
      if (a.ret) a.ret[cw] = iter + (iter < a.max_iter);
      if (a.iters) a.iters[cw] = iter;
      if (a.parity_cnt) a.parity_cnt[cw] = a.iter_count > 0 ? pcnt : 0;
      if (a.cw_err && a.ref_bits) a.cw_err[cw] = a.iter_count > 0 ? errs : 0;
      if (a.counters) {
        const unsigned long long vn = conv ? (unsigned long long)iter + 1 : (unsigned long long)iter;
        atomicAdd(&a.counters[CNT_VN_PHASES], vn);
        atomicAdd(&a.counters[CNT_CN_PHASES], (unsigned long long)iter);
        if (conv) atomicAdd(&a.counters[CNT_CONVERGED], 1ull);
        if (a.ref_bits && a.iter_count > 0) {
          atomicAdd(&a.counters[CNT_ERR_BIT], (unsigned long long)errs);
          atomicAdd(&a.counters[CNT_ERR_BLK], errs > 0 ? 1ull : 0ull);
          atomicAdd(&a.counters[CNT_TOT_BIT], (unsigned long long)c.K);
          atomicAdd(&a.counters[CNT_TOT_BLK], 1ull);
        }
      }
    }
  }
}

template <int kG, int T, int RV, int RC, int RX, bool SYN>
hipError_t launch_part_t(const DevCode &c, const BpLaunch &a, hipStream_t s, int fast, int groups) {
  auto kern = bp_part_kernel<kG, T, RV, RC, RX, SYN>;
  const size_t lds = part_lds_bytes(c);
  hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(a.queue, 0, sizeof(unsigned int), s);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(a.gsync, 0, sizeof(GroupSync) * (size_t)groups + sizeof(unsigned), s);
  if (e != hipSuccess) return e;
  DevCode cc = c;
  BpLaunch aa = a;
  GroupSync *gs = reinterpret_cast<GroupSync *>(a.gsync);
  uint8_t *gcch = a.gcch;
  unsigned *abort = reinterpret_cast<unsigned *>(gs + groups);
  unsigned int *q = a.queue;
  int f = fast;
  void *args[] = {&cc, &aa, &gs, &gcch, &abort, &q, &f};
  return hipLaunchCooperativeKernel((const void *)kern, dim3((unsigned)(groups * kG)), dim3(T), args, (unsigned)lds,
                                    s);
}

template <int kG, int T, int RV, int RC, bool SYN>
hipError_t launch_coop_t(const DevCode &c, const BpLaunch &a, hipStream_t s, int fast, int groups) {
  auto kern = bp_coop_kernel<kG, T, RV, RC, SYN>;
  hipError_t e = hipMemsetAsync(a.queue, 0, sizeof(unsigned int), s);
  if (e != hipSuccess) return e;
  // group blocks + the abort word
  e = hipMemsetAsync(a.gsync, 0, sizeof(GroupSync) * (size_t)groups + sizeof(unsigned), s);
  if (e != hipSuccess) return e;
  DevCode cc = c;
  BpLaunch aa = a;
  GroupSync *gs = reinterpret_cast<GroupSync *>(a.gsync);
  uint8_t *gcch = a.gcch;
  unsigned *abort = reinterpret_cast<unsigned *>(gs + groups);
  unsigned int *q = a.queue;
  int f = fast;
  void *args[] = {&cc, &aa, &gs, &gcch, &abort, &q, &f};
  return hipLaunchCooperativeKernel((const void *)kern, dim3((unsigned)(groups * kG)), dim3(T), args, 0, s);
}

// Kernel choice and tiling.  Default: the partitioned kernel (groups of 4,
// KML_PART = threads per workgroup: 512, 768 or 1024) when the context built a
// partition plan.  KML_COOP = "G,T" selects the global-slot kernel instead
// (workgroups per codeword, threads per workgroup), for A/B measurements.
struct CoopCfg {
  bool part;
  int G, T;
};
CoopCfg coop_cfg(const DevCode &c) {
  CoopCfg k{c.pt_G == kPartG && c.pt_vn != nullptr, 4, 512};
  if (k.part) k.T = 1024;
  if (const char *e = getenv("KML_COOP")) {
    int g = 0, t = 0;
    if (sscanf(e, "%d,%d", &g, &t) == 2 && (g == 4 || g == 8) && (t == 512 || t == 1024)) k = {false, g, t};
  }
  if (k.part)
    if (const char *e = getenv("KML_PART")) {
      const int t = atoi(e);
      if (t == 512 || t == 768 || t == 1024) k.T = t;
    }
  return k;
}

}  // namespace

size_t bp_coop_sync_bytes(int groups) { return sizeof(GroupSync) * (size_t)groups + 64; }

int bp_part_group_size(int N, int M, int E, int dv_max, int dc_max, int regular) {
  if (!regular || dv_max != 3 || dc_max != 6 || (long long)E * 16 + 16 + N <= 160 * 1024) return 0;
  if (N % kPartG || M % kPartG || (N / kPartG) % 16) return 0;
  const int NG = N / kPartG, MG = M / kPartG;
  // the largest tiling covers 2048 columns and half-rows per member; the LDS
  // check including the mirror slots is part_plan_fits (after planning)
  if ((long long)MG * 6 * 16 + N > 160 * 1024 || NG > 2048 || 2 * MG > 2048) return 0;
  return kPartG;
}

bool part_plan_fits(int N, int M, int E, int ncut, int mirror_max, int xmax) {
  const long long lds = ((long long)M / kPartG * 6 + mirror_max) * 16 + N;
  return lds <= 160 * 1024 && 3LL * ncut <= 2LL * E && xmax <= 2 * 1024;
}

int bp_coop_groups(const DevCode &c) {
  if (!c.regular || !c.reg_pos || c.dv_max != 3 || c.dc_max != 6 || bp_uses_lds(c)) return 0;
  const CoopCfg k = coop_cfg(c);
  if (!k.part) {
    const int R = 8192 / (k.G * k.T);  // columns (and half-rows) per thread of the instantiated tilings
    if ((c.N + k.G - 1) / k.G > R * k.T || (2 * c.M + k.G - 1) / k.G > R * k.T) return 0;
  }
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  return (ncu / (8 * k.G)) * 8;  // one workgroup per CU; 8 XCDs, groups of G per XCD
}

#ifdef KML_STAMPS
}  // namespace kml
extern "C" int kml_debug_part_stamps(unsigned long long *out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(kml::kml_part_stamps), sizeof(kml::kml_part_stamps));
  if (reset) {
    static unsigned long long zero[256 * kml::kStampSlots];
    hipMemcpyToSymbol(HIP_SYMBOL(kml::kml_part_stamps), zero, sizeof(zero));
  }
  return e == hipSuccess ? 0 : -1;
}
namespace kml {
#endif

const char *bp_coop_family(const DevCode &c) { return coop_cfg(c).part ? "bp_part_kernel" : "bp_coop_kernel"; }

hipError_t launch_bp_coop(const DevCode &c, const BpLaunch &a, hipStream_t s) {
  const int groups = bp_coop_groups(c);
  if (groups <= 0 || !a.gsync || !a.gcch || (long long)groups * c.E > a.gslots_cap) return hipErrorNotSupported;
  if (const char *k = getenv("KML_BP_KERNEL"))
    if (k[0] == 'g') return hipErrorNotSupported;
  const int fast = c.dv_max <= kFastMaxColumnDegree ? 1 : 0;
  const CoopCfg k = coop_cfg(c);
  if (k.part) {
    // exchange entries per thread: every member's lists must fit RX * T
    int xmax = 0;
    for (int m = 0; m < kPartG; m++) xmax = std::max(xmax, std::max(c.pt_xr_n[m], c.pt_xc_n[m]));
#define KML_PART_CASE(T_, R_, X_)                                                                  \
  if (k.T == T_ && xmax <= X_ * T_)                                                               \
    return a.syn ? launch_part_t<kPartG, T_, R_, R_, X_, true>(c, a, s, fast, groups)             \
                 : launch_part_t<kPartG, T_, R_, R_, X_, false>(c, a, s, fast, groups);
    KML_PART_CASE(512, 4, 4)
    KML_PART_CASE(768, 3, 3)
    KML_PART_CASE(1024, 2, 2)
#undef KML_PART_CASE
    return hipErrorNotSupported;
  }
#define KML_COOP_CASE(G_, T_, R_)                                                                               \
  if (k.G == G_ && k.T == T_)                                                                                  \
    return a.syn ? launch_coop_t<G_, T_, R_, R_, true>(c, a, s, fast, groups)                                  \
                 : launch_coop_t<G_, T_, R_, R_, false>(c, a, s, fast, groups);
  KML_COOP_CASE(4, 512, 4)
  KML_COOP_CASE(4, 1024, 2)
  KML_COOP_CASE(8, 512, 2)
  KML_COOP_CASE(8, 1024, 1)
#undef KML_COOP_CASE
  return hipErrorNotSupported;
}

// Did the last cooperative launch abort (a group barrier timed out)?
bool bp_coop_aborted(const BpLaunch &a, int groups, hipStream_t s) {
  unsigned v = 0;
  hipMemcpyAsync(&v, reinterpret_cast<GroupSync *>(a.gsync) + groups, sizeof(v), hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  return v != 0;
}

}  // namespace kml
