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
  unsigned flag[2];  // per iteration parity: bit 0 failing rows, bit 1 an unproven VN quotient
  unsigned cw;       // the group's current codeword (entry index)
  unsigned errs;     // error bits of the codeword, summed over members
  unsigned pcnt;     // unsatisfied checks of the final hard decisions, summed
  unsigned xcc;      // bit per XCD a member runs on
  // partitioned kernel: barrier counters by barrier parity, arrivals in the
  // low 32 bits, parity-failure reports in the high 32 bits (part_barrier)
  unsigned long long bar2[2];
  // tagged exchange: early-stop flags per iteration parity and member,
  // ((global iteration + 1) << 2) | (an unproven quotient in its VN phase) << 1
  // | (the member has failing rows)
  unsigned long long mflag[2][8];
};

// Workgroups per codeword of the partitioned kernel.  (Groups of 8 with two
// codewords in flight, and two 512-thread workgroups per CU, measured slower
// in round 4 and were removed: DESIGN.md, Round-4 changes.)
constexpr int kPartG = 4;

// c2v placement: a c2v message lives in the lower or upper 8 bytes of its
// 16-byte slot (the v2c pair fills the whole slot), by bit 2 of its row's
// member-local index for row slots and bit 2 of the slot index for mirror
// slots.  The CN phase's 16-lane ds_write_b64 groups (8 rows, 24 dwords
// apart) then hit distinct banks (rows q and q + 4 no longer collide), and the
// VN phase's scattered ds_read_b64 use all 64 banks instead of the 32 of
// slot-aligned addresses.  vaddr holds the half-slot index 2 slot + half.
#ifndef KML_PART_C2V_HALF
#define KML_PART_C2V_HALF 1
#endif
__host__ __device__ constexpr int part_c2v_half(int slot, int EG, int DC) {
  return KML_PART_C2V_HALF ? (slot < EG ? ((slot / DC) >> 2) & 1 : (slot >> 2) & 1) : 0;
}
__device__ __forceinline__ unsigned vaddr_c2v(int v) { return (unsigned)(v & 0x1FFFF) * 8u; }  // c2v word (bytes)
__device__ __forceinline__ unsigned vaddr_slot(int v) { return (unsigned)(v & 0x1FFFE) * 8u; }  // slot (bytes)

// LDS of the partitioned kernel: the member's row slots, its mirror slots, and
// every column's hard decision.
// kPartDummy slots past the mirrors: the target of the branch-free tagged
// stores of inactive lanes (a lane past the member's columns or rows), which
// compute throw-away messages.
constexpr int kPartDummy = 7;
size_t part_lds_bytes(const DevCode &c) {
  return ((size_t)c.M / c.pt_G * 6 + (size_t)c.pt_mirror + kPartDummy) * 16 + (size_t)c.N;
}

#ifndef KML_POLL_SLEEP  // (A/B) s_sleep between the tagged mailbox polls
#define KML_POLL_SLEEP 0  // measured: no sleep 8.52 -> 8.48 ms per 4096 PEG8064 codewords
#endif
constexpr long long kSpinLimit = 20000000;  // ~1 s of s_sleep(1) polls

// The tagged mailboxes (bp_part_kernel) follow the barrier-exchange ones in
// the group's E double2 of scratch: 3 ncut doubles, rounded to 16 bytes, then
// another 3 ncut.
// The branch-free tagged stores address a row slot's (absent) v2c entry as
// kMbOob (entry 0x7FFF, byte offset 0x7FFF0) and a row slot's c2v entry as
// kMbOobOff: both out of the mailbox buffer's range (24 ncut bytes), which the
// hardware's range check drops, so ncut <= 0x7FFF0 / 24.
constexpr int kMbOob = 0x7FFF;
constexpr unsigned kMbOobOff = 0x80000000u;
__host__ __device__ constexpr bool part_tagged_fits(int E, int ncut) {
  return 6LL * ncut + 2 <= 2LL * E && 24LL * ncut <= 16LL * kMbOob;
}
// The partitioned launches' scratch per group (double2): the barrier-exchange
// mailboxes (3 ncut doubles) and the tagged ones, in E double2; the tagged
// launch's defer list follows the groups' strides.
__host__ __device__ inline long long part_group_stride(const DevCode &c) { return ((long long)c.E + 7) & ~7LL; }
// byte offset of the deferred-codeword count in the sync block (past the abort word)
constexpr size_t part_defer_offset(int groups) { return sizeof(GroupSync) * (size_t)groups + 16; }

__device__ __forceinline__ unsigned ld_rlx(const unsigned *p) {  // L1-bypassing (sc1) load
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Leave a poll of the cooperative launch.  A poller whose own spin limit ran
// out (timed_out) aborts the launch: it records where it gave up in abort[1]
// (site << 24 | workgroup: 1 group barrier, 2 v2c mailbox poll, 3 c2v mailbox
// poll, 4 early-stop flag poll; the first such poller wins), then sets
// abort[0] = 1, which stops every poll.  A poller that only saw abort[0] set
// (by another poller, or by the host: kml_debug_inject_abort) records nothing,
// so abort[1] names the site that actually timed out, or stays 0 for a
// host-raised abort (bp_coop_aborted reports it).
enum { kAbortBarrier = 1, kAbortV2c = 2, kAbortC2v = 3, kAbortFlag = 4 };
__device__ __forceinline__ void coop_abort(unsigned *abort, unsigned site, bool timed_out) {
  if (!timed_out) return;
  atomicCAS(abort + 1, 0u, (site << 24) | (blockIdx.x & 0xFFFFFFu));
  __hip_atomic_store(abort, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
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
    if (flag) {  // bit 0: failing rows (counts 1), bit 1: an unproven quotient (counts 256)
      add += (unsigned long long)(((*flag & 1) ? 1u : 0u) + ((*flag & 2) ? 256u : 0u)) << 32;
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
        coop_abort(abort, kAbortBarrier, spin > kSpinLimit);
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

// -1: the launch aborts; 1: a FAST decode met an unproven quotient (redo with
// FAST = false, see coop_iterations); 0: done.
template <int kG, int RV, int RC, int RX, bool SYN, bool FAST>
__device__ __forceinline__ int part_iterations(const BpLaunch &a, int M, int N, int NG, int cw, GroupSync *gs,
                                                unsigned long long *bst, unsigned &nb, int *sfail, bool same_xcd,
                                                unsigned *abort, unsigned char *smem,
                                                uint8_t *dec, double2 *mb_v2c, double *mb_c2v, uint8_t *gc,
                                                const DevCode &c, const int (&vaddr)[RV][3], const int (&vpos)[RV],
                                                const bool (&vact)[RV], const double (&pv)[RV], const int (&crow)[RC],
                                                const int (&cbase)[RC],
                                                const bool (&cact)[RC], const int (&xr)[RX], const int (&xc)[RX],
                                                int odd, int member, int &iter_out, bool &conv_out,
                                                bool sus0 = false) {
  constexpr int DV = 3, DC = 6, H = 3;
  const int tid = threadIdx.x;
  int ccol[RC][H];  // parity-check columns (positions in dec): even lane edges [0, H), odd lane [H, DC)
#pragma unroll
  for (int r = 0; r < RC; ++r)
#pragma unroll
    for (int k = 0; k < H; ++k) ccol[r][k] = c.pt_pos[c.row_col[c.row_ptr[crow[r]] + (odd ? H + k : k)]];
  double2 *slots = reinterpret_cast<double2 *>(smem);
  int iter = 0;
  bool conv = false, sus = sus0;
#ifdef KML_STAMPS
  unsigned long long stamp_prev = __builtin_amdgcn_s_memtime();
#endif
  for (; iter < a.iter_count; ++iter) {
    KML_STAMP(0);  // iteration boundary
    // ---------------------------------- receive c2v of the cut edges (mirrors)
    if (iter > 0) {  // iteration 0 reads InitMsg's 0.5
#pragma unroll
      for (int q = 0; q < RX; ++q)
        if (xc[q] >= 0) {
          const int sl = xc[q] & 0xFFFF;
          *reinterpret_cast<double *>(smem + sl * 16 + (KML_PART_C2V_HALF ? ((sl >> 2) & 1) * 8 : 0)) =
              ld_nt(&mb_c2v[xc[q] >> 16]);
        }
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
        for (int k = 0; k < DV; ++k) c0s[r][k] = *reinterpret_cast<const double *>(smem + vaddr_c2v(vaddr[r][k]));
      // one column's chains at a time (column-major): the FAST divisions'
      // proofs keep a normalisation's operands live, and interleaving the RV
      // columns step by step doubled the live set (scratch spills in the loop)
#pragma unroll
      for (int r = 0; r < RV; ++r) {
        double a0 = pv[r], a1 = 1.0 - pv[r], al0[DV], al1[DV];
#pragma unroll
        for (int k = 0; k < DV; ++k) {
          al0[k] = a0;
          al1[k] = a1;
          const double c0 = c0s[r][k];
          const double n0 = a0 * c0;
          const double n1 = a1 * (1.0 - c0);
          if (k + 1 < DV) {
            div2<FAST>(n0, n1, n0 + n1, a0, a1, sus);
          } else {
            const int hd = hard_decision<FAST>(n0, n1, sus);
            if (vact[r]) {
              dec[vpos[r]] = (unsigned char)hd;
              gc[vpos[r]] = (unsigned char)hd;
            }
          }
        }
        if (r == RV / 2) __builtin_amdgcn_s_setprio(1);  // falling priorities within the phase
        double b0 = 1.0, b1 = 1.0;
#pragma unroll
        for (int k = DV - 1; k >= 0; --k) {
          const bool unit = FAST && k == DV - 1;
          const double t0 = unit ? al0[k] : al0[k] * b0;
          const double t1 = unit ? al1[k] : al1[k] * b1;
          double q0, q1;
          if (unit)  // beta = (1, 1): t is the normalised alpha, its sum within ulps of 1 (bp_common.hpp rcp_near1)
            div2<FAST, true>(t0, t1, t0 + t1, q0, q1, sus);
          else
            div2<FAST>(t0, t1, t0 + t1, q0, q1, sus);
          if (vact[r]) *reinterpret_cast<double2 *>(smem + vaddr_slot(vaddr[r][k])) = make_double2(q0, q1);
          if (k > 0) {
            const double c0 = c0s[r][k];
            if (unit) {  // the sum rounds to exactly 1 (bp_common.hpp)
              b0 = c0;
              b1 = 1.0 - c0;
            } else {
              div2<FAST>(b0 * c0, b1 * (1.0 - c0), b0 * c0 + b1 * (1.0 - c0), b0, b1, sus);
            }
          }
        }
      }
      __builtin_amdgcn_s_setprio(0);
    }
    KML_STAMP(2);  // VN compute (wave 0)
    // ---------------------------------------------- send v2c of the cut edges
    __syncthreads();
    KML_STAMP(3);  // VN drain (other waves)
#pragma unroll
    for (int q = 0; q < RX; ++q)
      if (xc[q] >= 0) mb_v2c[xc[q] >> 16] = slots[xc[q] & 0xFFFF];
    if (part_barrier<kG>(gs, bst, nb, same_xcd, abort, nullptr) < 0) return -1;
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
      const int bits = (__ballot(fail) != 0 ? 1 : 0) | (__ballot(sus) != 0 ? 2 : 0);
      if (bits && (tid & 63) == 0) atomicOr(sfail, bits);  // reported at the CN barrier
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
            if (cact[r])
              *reinterpret_cast<double *>(smem + cbase[r] + (odd ? st : DC - 1 - st) * 16 +
                                          part_c2v_half(cbase[r] / 16, 0x7FFFFFFF, DC) * 8) = q;
          }
        }
        if (advance) {
#pragma unroll
          for (int r = 0; r < RC; ++r) {
            const bool unit = FAST && st == 0;
            const double n0 = unit ? m0[r] : s0[r] * m0[r] + s1[r] * m1[r];
            const double n1 = unit ? m1[r] : s0[r] * m1[r] + s1[r] * m0[r];
            div2<FAST, true>(n0, n1, n0 + n1, s0[r], s1[r], sus);
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
      if (xr[q] >= 0) {  // the row slot's c2v half (part_c2v_half)
        const int sl = xr[q] & 0xFFFF;
        mb_c2v[xr[q] >> 16] = part_c2v_half(sl, 0x7FFFFFFF, DC) ? slots[sl].y : slots[sl].x;
      }
    const int failing = part_barrier<kG>(gs, bst, nb, same_xcd, abort, sfail);
    KML_STAMP(8);  // send c2v + group barrier
    if (failing < 0) return -1;
    if (FAST && (failing >> 8)) {  // a member met an unproven quotient in this VN phase
      iter_out = iter;
      conv_out = false;
      return 1;
    }
    if ((failing & 0xFF) == 0) {  // every row satisfied: stop before this CN phase
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
  return 0;
}

// ---------------------------------------------------------------------------
// Tagged exchange (FAST codewords of same-XCD groups): no group barrier inside
// the iterations.  Every cut edge has one mailbox entry per direction, and
// the entry's producer writes it directly from the arithmetic (plain store,
// landing in the XCD's L2) with a TAG in the sign bit of every word: the
// parity of the group's global iteration counter g (all members run the same
// iterations, so they agree on g).  A consumer polls its entries (L1-bypassing
// loads) until the tags read g & 1.  FAST messages lie in [0, 1], so bits 63
// and 62 of their words are zero; the v2c entry also carries the column's
// hard decision in bit 62 of its first word, which replaces the exchange of
// the decision array for the row owner's parity check.
// Why one tag bit is enough: each entry is written exactly once per global
// iteration (the CN phase runs speculatively in the converged iteration too),
// and its producer cannot write it again before the consumer has read it:
// v2c(e) of iteration g+1 follows the VN phase that polled c2v(e) of iteration
// g, which the row owner computes only after its CN lanes polled v2c(e) of
// iteration g (every lane polls all its entries before any arithmetic); the
// symmetric argument holds for c2v, and across codewords the early-stop flags
// of iteration g (posted after the member's loads of iteration g) gate the
// next codeword's first writes.
// Early stop, checked one phase late: after its CN phase of iteration g the
// member's LAST wave to finish (an LDS arrival count, no workgroup barrier)
// posts (g + 1, failing rows?) to its flag word of parity g & 1, and wave 0
// polls the members' flags (one per lane) after the NEXT VN phase, beside
// the v2c receive — by then the flags have long arrived.  A codeword whose
// checks all hold after iteration g therefore also runs VN g + 1 (its
// decisions go to the other half of a double-buffered decision array; the
// outputs take iteration g's half) and then stops, before CN g + 1.  VN
// g + 1's v2c messages were received; the c2v entries still hold iteration
// g - 1's tag parity, which the next codeword's first CN (iteration g + 2)
// would match, so the stopping members overwrite their c2v entries with tag
// g + 1 (a flush nobody reads) before the codeword's closing barrier.
// A flag word is rewritten (iteration g + 2) only after the poster received
// the v2c of iteration g + 2, which its partners send after their iteration
// g + 1 flag polls.  Measured against the CN-closing-barrier form (flags
// checked before the next VN): see DESIGN.md.
#ifndef KML_PART_CN_AGE_PRIO
#define KML_PART_CN_AGE_PRIO 5
#endif
#ifndef KML_PART_FLAG_LATE  // (A/B) 0: the last wave of the CN phase posts the flag (returned LDS atomics)
#define KML_PART_FLAG_LATE 1
#endif
#ifndef KML_PART_VN_AGE_PRIO
#define KML_PART_VN_AGE_PRIO 0
#endif
#ifndef KML_PART_QUEUE_EARLY  // the next entry taken under the outputs (bp_part_kernel's loop)
#define KML_PART_QUEUE_EARLY 1
#endif
constexpr unsigned kTagHi = 0x80000000u;  // bit 63 of a message word (hi dword bit 31)
constexpr unsigned kHdHi = 0x40000000u;   // bit 62: hard decision (v2c first word)


__device__ __forceinline__ double or_hi(double x, unsigned bits) {
  return __hiloint2double(__double2hiint(x) | (int)bits, __double2loint(x));
}
__device__ __forceinline__ double and_hi(double x, unsigned mask) {
  return __hiloint2double(__double2hiint(x) & (int)mask, __double2loint(x));
}
__device__ __forceinline__ unsigned hi_of(unsigned long long w) { return (unsigned)(w >> 32); }

// Mailbox accesses through a buffer resource (SGPRs) and 32-bit byte offsets:
// no 64-bit per-lane addresses to keep live across the phases.  Polls load
// with sc1 (L2-served, bypassing the never-refreshed vector L1).
// Hardware assumption (the tag protocol's only one): a naturally aligned 8-byte
// word written by one b64 / b128 store is read whole by one b64 / b128 load —
// no load returns a new high dword (the tag) with a stale low dword.  Each
// 8-byte word carries its own tag, so nothing wider than 8 bytes must be
// single-copy atomic.  This is the property the AMDGPU backend itself relies on
// when it lowers a relaxed 64-bit atomic load / store to a plain dwordx2
// access.  A 16-byte entry is 16-byte aligned, so it never straddles a
// 128-byte L2 line and reaches the L2 as one request.  All members of a
// group run on one XCD (same_xcd: the tagged launch defers every other group's
// codewords to the barrier-exchange launch), so producer and consumer share
// that L2 and no cross-XCD coherence is involved.
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
constexpr int kBufFlags = 0x00020000;  // gfx9 raw buffer resource, dword 3
constexpr int kAuxSc1 = 16;            // cache-policy operand: sc1
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mailbox_rsrc(void *p, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, bytes, kBufFlags);
}
__device__ __forceinline__ unsigned long long mb_ld64(__amdgpu_buffer_rsrc_t r, unsigned off) {
  const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, kAuxSc1);
  return ((unsigned long long)v.y << 32) | v.x;
}
__device__ __forceinline__ void mb_st64(__amdgpu_buffer_rsrc_t r, unsigned off, double x) {
  const u32x2 v = {(unsigned)__double2loint(x), (unsigned)__double2hiint(x)};
  __builtin_amdgcn_raw_buffer_store_b64(v, r, (int)off, 0, 0);
}
__device__ __forceinline__ void mb_st128(__amdgpu_buffer_rsrc_t r, unsigned off, double x, double y) {
  const u32x4 v = {(unsigned)__double2loint(x), (unsigned)__double2hiint(x), (unsigned)__double2loint(y),
                   (unsigned)__double2hiint(y)};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, (int)off, 0, 0);
}

// Poll n (<= R) mailbox entries of W words (8 B each) until every word's tag
// bit equals tag, then store them to LDS.  entry q = (x << 16) | LDS slot, or
// < 0 when absent.  Returns false on a timeout / aborted launch.
template <int R, int W>
__device__ __forceinline__ bool poll_entries(const int (&ent)[R], __amdgpu_buffer_rsrc_t mb, unsigned mb_off,
                                             unsigned char *smem, unsigned tag, unsigned *abort) {
  bool need[R];
#pragma unroll
  for (int q = 0; q < R; ++q) need[q] = ent[q] >= 0;
  for (long long spin = 0;; ++spin) {
    unsigned long long w[R][W];
#pragma unroll
    for (int q = 0; q < R; ++q)
      if (need[q]) {
        if constexpr (W == 2) {  // one 16-byte load (each word carries its own tag)
          const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(mb, (int)(mb_off + (unsigned)(ent[q] >> 16) * 16u), 0,
                                                                kAuxSc1);
          w[q][0] = ((unsigned long long)v.y << 32) | v.x;
          w[q][1] = ((unsigned long long)v.w << 32) | v.z;
        } else {
#pragma unroll
          for (int i = 0; i < W; ++i) w[q][i] = mb_ld64(mb, mb_off + (unsigned)(ent[q] >> 16) * (8 * W) + 8 * i);
        }
      }
    bool pend = false;
#pragma unroll
    for (int q = 0; q < R; ++q)
      if (need[q]) {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < W; ++i) ok = ok && (hi_of(w[q][i]) >> 31) == tag;
        if (ok) {
          // stored without the tags (a v2c message keeps its hard-decision bit)
          const int sl = ent[q] & 0xFFFF;
          unsigned long long *d = reinterpret_cast<unsigned long long *>(
              smem + sl * 16 + (W == 1 && KML_PART_C2V_HALF ? ((sl >> 2) & 1) * 8 : 0));
#pragma unroll
          for (int i = 0; i < W; ++i) d[i] = w[q][i] & ~(1ull << 63);
          need[q] = false;
        } else {
          pend = true;
        }
      }
    if (!pend) return true;
    if ((spin & 63) == 63 && (spin > kSpinLimit || ld_rlx(abort))) {
      coop_abort(abort, W == 2 ? kAbortV2c : kAbortC2v, spin > kSpinLimit);
      return false;
    }
    if (KML_POLL_SLEEP) __builtin_amdgcn_s_sleep(1);
  }
}

// -1: the launch aborts; 1: a member met a quotient dd_check could not prove
// (exact_div.hpp) — the decode stops like a converged one (the same mailbox
// flush) and the caller defers the codeword to the barrier-exchange launch on
// the exact path; 0: done.
template <int kG, int T, int RV, int RC, int RX, bool SYN>
__device__ __forceinline__ int part_iterations_tagged(
    const BpLaunch &a, int M, int cw, GroupSync *gs, unsigned &g, int *sfail, int *sdead, int member,
    unsigned *abort, unsigned char *smem, uint8_t *dec, int NG, __amdgpu_buffer_rsrc_t tb, unsigned tb_c2v,
    const int (&vaddr)[RV][3],
    const bool (&vact)[RV], const double (&pv)[RV], const int (&crow)[RC],
    const int (&cbase)[RC], const int (&crx)[RC], const int (&cwb)[RC], const bool (&cact)[RC], const int (&xr)[RX],
    const int (&xc)[RX],
    int odd, int &iter_out, bool &conv_out, int &pcnt_out, int &decbuf_out, bool sus0 = false) {
  constexpr int DV = 3, DC = 6, H = 3, NW = T / 64;
  const int tid = threadIdx.x;
#if !KML_PART_FLAG_LATE
  __shared__ int sarrive;  // waves done with the CN phase of this iteration
  if (tid == 0) sarrive = 0;
#endif
  __shared__ int sany;     // bit 0: some member had failing rows after the previous CN phase; bit 1: an unproven quotient
  int iter = 0, pcnt_prev = 0;
  bool sus = sus0;
  double syn_prev[RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) syn_prev[r] = 0.0;
  bool conv = false;
#ifdef KML_STAMPS
  unsigned long long stamp_prev = __builtin_amdgcn_s_memtime();
#endif
  for (;; ++iter, ++g) {
    const unsigned tag = g & 1u;
    const bool run = iter < a.iter_count;  // else only the last CN phase's early-stop check remains
    uint8_t *decb = dec + (iter & 1) * NG;
    KML_STAMP(0);
    // wave 0 issues the load of the members' early-stop flags of iteration
    // g - 1 now: it is used after this VN phase and the v2c receive, so its L2
    // round trip overlaps them (the flags were posted before the partners'
    // c2v messages this member received)
    unsigned long long vflag = 0;
    if (iter > 0 && tid < kG) vflag = ld_rlx64(&gs->mflag[(g - 1) & 1][tid]);
    // ------------------------------------------------------------ VN phase
    // (c2v of cut edges sit in the mirror slots, received at the end of the
    // previous iteration; iteration 0 reads InitMsg's 0.5)
    if (run) {
#if KML_PART_VN_AGE_PRIO  // (A/B) VN priorities by wave age for the whole phase (measured +5%: off)
      {
        const int grp = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) * 4 / NW;
        if (grp >= 3) __builtin_amdgcn_s_setprio(3);
        else if (grp == 2) __builtin_amdgcn_s_setprio(2);
        else if (grp == 1) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
#else
      __builtin_amdgcn_s_setprio(3);
#endif
      // one column's chains at a time (column-major): the FAST divisions'
      // proofs keep a normalisation's operands live, and interleaving the RV
      // columns step by step doubled the live set (scratch spills in the loop)
#pragma unroll
      for (int r = 0; r < RV; ++r) {
        double c0c[DV];  // the column's c2v, loaded per column (registers)
#pragma unroll
        for (int k = 0; k < DV; ++k) c0c[k] = *reinterpret_cast<const double *>(smem + vaddr_c2v(vaddr[r][k]));
        double a0 = pv[r], a1 = 1.0 - pv[r], al0[DV], al1[DV];
        unsigned hdb = 0;
#pragma unroll
        for (int k = 0; k < DV; ++k) {
          al0[k] = a0;
          al1[k] = a1;
          const double c0 = c0c[k];
          const double n0 = a0 * c0;
          const double n1 = a1 * (1.0 - c0);
          if (k + 1 < DV) {
            div2<true>(n0, n1, n0 + n1, a0, a1, sus);
          } else {
            const int hd = hard_decision<true>(n0, n1, sus);
            hdb = hd ? kHdHi : 0u;
            if (vact[r]) decb[r * T + tid] = (unsigned char)hd;
          }
        }
        if (r == RV / 2) __builtin_amdgcn_s_setprio(1);  // falling priorities within the phase
        double b0 = 1.0, b1 = 1.0;
#pragma unroll
        for (int k = DV - 1; k >= 0; --k) {
          const bool unit = k == DV - 1;
          const double t0 = unit ? al0[k] : al0[k] * b0;
          const double t1 = unit ? al1[k] : al1[k] * b1;
          double q0, q1;
          if (unit)
            div2<true, true>(t0, t1, t0 + t1, q0, q1, sus);
          else
            div2<true>(t0, t1, t0 + t1, q0, q1, sus);
          {  // branch-free (see vaddr): the mailbox entry (dropped for a row slot) and the LDS slot
            const unsigned va = (unsigned)vaddr[r][k];
            const unsigned tb_tag = tag ? kTagHi : 0u;
            mb_st128(tb, (va >> 17) << 4, or_hi(q0, tb_tag | hdb), or_hi(q1, tb_tag));
            *reinterpret_cast<double2 *>(smem + vaddr_slot(vaddr[r][k])) = make_double2(or_hi(q0, hdb), q1);
          }
          if (k > 0) {
            const double c0 = c0c[k];
            if (unit) {
              b0 = c0;
              b1 = 1.0 - c0;
            } else {
              div2<true>(b0 * c0, b1 * (1.0 - c0), b0 * c0 + b1 * (1.0 - c0), b0, b1, sus);
            }
          }
        }
      }
      __builtin_amdgcn_s_setprio(0);
    }
    KML_STAMP(2);
    // ------------------- receive v2c of the cut edges; the previous CN's flags
    if (run)
      if (!poll_entries<RX, 2>(xr, tb, 0u, smem, tag, abort)) *sdead = 1;
    KML_STAMP(4);
    if (iter > 0 && tid < 64) {  // wave 0: lane m polls member m's flag of iteration g - 1
      unsigned long long v = (unsigned long long)g << 2;
      if (tid < kG) {
        for (long long spin = 0;; ++spin) {
          v = spin == 0 ? vflag : ld_rlx64(&gs->mflag[(g - 1) & 1][tid]);  // first: the load issued before VN
          if ((v >> 2) == (unsigned long long)g) break;
          if ((spin & 63) == 63 && (spin > kSpinLimit || ld_rlx(abort))) {
            coop_abort(abort, kAbortFlag, spin > kSpinLimit);
            *sdead = 1;
            break;
          }
          __builtin_amdgcn_s_sleep(1);
        }
      }
      const int any = (__ballot((v & 1) != 0) != 0 ? 1 : 0) | (__ballot((v & 2) != 0) != 0 ? 2 : 0);
      if (tid == 0) sany = any;
    }
    __syncthreads();
    KML_STAMP(5);
    if (*sdead) return -1;
    // stop before the CN phase of iteration iter - 1's successor when every row
    // was satisfied after it, or when a member met an unproven quotient in VN
    // iter - 1 (then the codeword is redone exactly; the same mailbox flush)
    const bool suspect = iter > 0 && (sany & 2);
    if (iter > 0 && (!(sany & 1) || suspect)) {
      conv = !suspect;
      --iter;
      if (iter + 1 < a.iter_count) {  // VN iter + 1 ran: flush the c2v entries (see above)
        const double dummy = or_hi(0.5, tag ? kTagHi : 0u);
#pragma unroll
        for (int r = 0; r < RC; ++r)
          if (cact[r]) {
            const int mask = crx[r] & 0x3F;
#pragma unroll
            for (int k = 0; k < H; ++k) {
              const int e = odd ? H + k : k;
              if ((mask >> e) & 1) mb_st64(tb, tb_c2v + (unsigned)((crx[r] >> 8) + __popc(mask & ((1 << e) - 1))) * 8,
                                           dummy);
            }
          }
        ++g;
      }
      if (suspect) return 1;
      break;
    }
    if constexpr (SYN) {  // the previous CN phase counted: its syndromes stand (alpha past the last edge, :274)
      if (iter > 0) {
#pragma unroll
        for (int r = 0; r < RC; ++r)
          if (cact[r] && !odd) a.syn[(long long)cw * M + crow[r]] = syn_prev[r];
      }
    }
    if (!run) break;  // max iterations without convergence

    // ------------------------------------------ CN phase (+ the parity check)
    // bp_regular.hip's step order: every load of a step before its stores.
    // A message's first word carries the column's hard decision in bit 62
    // (the receive strips the mailbox tags).
    int par[RC];
    {
      double x0[RC][H], x1[RC][H];
      double s0[RC], s1[RC];
#pragma unroll
      for (int r = 0; r < RC; ++r) {
        s0[r] = 1.0;
        s1[r] = 0.0;
        par[r] = 0;
      }
// (the tagged CN phase's wave priorities by age, youngest quarter highest,
// until step KML_PART_CN_AGE_PRIO, then 0: 8.69 -> 8.54 ms per 4096 PEG8064
// codewords against falling-by-step priorities (0), as in bp_regular.hip)
#if KML_PART_CN_AGE_PRIO
      {
        const int grp = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)) * 4 / NW;  // 0 oldest .. 3 youngest
        if (grp >= 3) __builtin_amdgcn_s_setprio(3);
        else if (grp == 2) __builtin_amdgcn_s_setprio(2);
        else if (grp == 1) __builtin_amdgcn_s_setprio(1);
        else __builtin_amdgcn_s_setprio(0);
      }
#else
      __builtin_amdgcn_s_setprio(2);
#endif
#pragma unroll
      for (int st = 0; st < DC; ++st) {
#if KML_PART_CN_AGE_PRIO
        if (st == KML_PART_CN_AGE_PRIO) __builtin_amdgcn_s_setprio(0);
#else
        if (st == 2) __builtin_amdgcn_s_setprio(1);
        if (st == 4) __builtin_amdgcn_s_setprio(0);
#endif
        const bool advance = SYN || st + 1 < DC || st < H;
        double m0[RC], m1[RC];
        if (advance) {
#pragma unroll
          for (int r = 0; r < RC; ++r) {
            const double2 m = *reinterpret_cast<const double2 *>(smem + cbase[r] + (odd ? DC - 1 - st : st) * 16);
            if (st < H) par[r] ^= (__double2hiint(m.x) >> 30) & 1;
            m0[r] = and_hi(m.x, ~kHdHi);
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
            const bool unit = st == DC - 1;
            const double t0 = unit ? y0 : o0 * y0 + o1 * y1;
            const double t1 = unit ? y1 : o0 * y1 + o1 * y0;
            const double q = clip_c2v<true>(div1<true, true>(t0, t0 + t1));
            {
              // branch-free: the mailbox entry of a cut edge (a row slot's
              // offset is out of the buffer's range: dropped) and the row
              // slot's c2v half (a cut edge's is never read; an inactive lane
              // writes the dummy slots).  Offsets from crx at the store: kept
              // per lane across the loop they spilled at the 128-VGPR limit.
              const unsigned cr = (unsigned)crx[r];
              const unsigned e = odd ? st : DC - 1 - st;  // the edge this c2v belongs to
              const unsigned cut = __builtin_amdgcn_ubfe(cr, e, 1);
              const unsigned x = __popc(__builtin_amdgcn_ubfe(cr, 0, e)) + (cr >> 8);
              mb_st64(tb, cut ? tb_c2v + x * 8 : kMbOobOff, or_hi(q, tag ? kTagHi : 0u));
              *reinterpret_cast<double *>(smem + cwb[r] + e * 16) = q;
            }
          }
        }
        if (st + 1 < DC || SYN) {
#pragma unroll
          for (int r = 0; r < RC; ++r) {
            const bool unit = st == 0;
            const double n0 = unit ? m0[r] : s0[r] * m0[r] + s1[r] * m1[r];
            const double n1 = unit ? m1[r] : s0[r] * m1[r] + s1[r] * m0[r];
            div2<true, true>(n0, n1, n0 + n1, s0[r], s1[r], sus);
          }
        }
      }
#pragma unroll
      for (int r = 0; r < RC; ++r) syn_prev[r] = s0[r];
    }
    // the row's parity: the even lane XORed edges 0..2, the odd lane 5..3
    int fail = 0, nfail = 0;
#pragma unroll
    for (int r = 0; r < RC; ++r) {
      const int full = par[r] ^ swap_pair_i(par[r]);
      fail |= cact[r] ? full : 0;
      nfail += (cact[r] && !odd) ? full : 0;
    }
    pcnt_prev = nfail;  // unsatisfied checks of this iteration's hard decisions (final if the loop ends after it)
    const int wbits = (__ballot(fail) != 0 ? 1 : 0) | (__ballot(sus) != 0 ? 2 : 0);
    KML_STAMP(6);
#if KML_PART_FLAG_LATE
    // every wave ORs its bits in (no returned atomic on its path); thread 0
    // posts the member's flag after the closing barrier below — the partners
    // read it only after their next VN phase and v2c receive
    if ((tid & 63) == 0 && wbits) atomicOr(sfail, wbits);
#else
    if ((tid & 63) == 0) {  // the member's last wave to get here posts its flag
      if (wbits) atomicOr(sfail, wbits);
      if (atomicAdd(&sarrive, 1) == NW - 1) {
        const int f = atomicExch(sfail, 0);
        sarrive = 0;
        __hip_atomic_store(&gs->mflag[g & 1][member], ((unsigned long long)(g + 1) << 2) | (unsigned long long)(f & 3),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
#endif
    KML_STAMP(7);
    // --------------------------------------- receive c2v of the cut edges
    if (iter + 1 < a.iter_count)
      if (!poll_entries<RX, 1>(xc, tb, tb_c2v, smem, tag, abort)) *sdead = 1;
    __syncthreads();
#if KML_PART_FLAG_LATE
    if (tid == 0) {
      const int f = *sfail;
      *sfail = 0;
      __hip_atomic_store(&gs->mflag[g & 1][member], ((unsigned long long)(g + 1) << 2) | (unsigned long long)(f & 3),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#endif
    KML_STAMP(8);
    if (*sdead) return -1;
  }
  iter_out = iter;
  conv_out = conv;
  pcnt_out = conv ? 0 : pcnt_prev;
  decbuf_out = iter & 1;  // the decisions of the last counted VN phase (iteration iter, or iter - 1 at max)
  if (!conv) decbuf_out = (iter - 1) & 1;
  return 0;
}

// Three launches (launch_bp_coop): TAGGED (FAST codewords of same-XCD groups;
// defers the rest, marking the ones that need the exact path with bit 31),
// then the barrier-exchange FAST kernel over those (TAGGED = EXACT = false;
// defers non-FAST and suspect codewords), then the barrier-exchange EXACT
// kernel over what remains.  Each follow-up launch is usually empty.
template <int kG, int T, int RV, int RC, int RX, bool SYN, bool TAGGED, bool EXACT>
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(1))) void bp_part_kernel(DevCode c, BpLaunch a, GroupSync *gsync, uint8_t *gcch,
                                                    unsigned *abort, unsigned int *queue, int fast_allowed) {
  const double plo = fast_prior_lo(c.dv_max);  // FAST prior domain (bp_common.hpp)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int DV = 3, DC = 6;
  const int tid = threadIdx.x;
  const int odd = tid & 1;
  const int member = (blockIdx.x >> 3) % kG;
  const int group = (blockIdx.x / (8 * kG)) * 8 + (blockIdx.x & 7);
  GroupSync *gs = gsync + group;
  const int MG = c.M / kG, NG = c.N / kG, EG = MG * DC;
  double2 *mb_v2c = a.gslots + (size_t)group * c.E;       // [ncut] double2
  double *mb_c2v = reinterpret_cast<double *>(mb_v2c + c.pt_ncut);  // [ncut] double
  // tagged mailboxes, after the barrier-exchange ones (16-byte aligned; part_tagged_fits)
  double2 *tb_v2c = reinterpret_cast<double2 *>(reinterpret_cast<double *>(mb_v2c) + ((3 * c.pt_ncut + 1) & ~1));
  const __amdgpu_buffer_rsrc_t tb = mailbox_rsrc(tb_v2c, 24 * c.pt_ncut);  // v2c [ncut] x 16 B, then c2v [ncut] x 8 B
  const unsigned tb_c2v = 16u * (unsigned)c.pt_ncut;
  uint8_t *gc = gcch + (size_t)group * c.N;
  const int nslots = EG + c.pt_mirror;
  uint8_t *dec = smem + (size_t)(nslots + kPartDummy) * 16;  // N hard decisions, plan order

  // vaddr: (v2c mailbox index of a cut edge, kMbOob for a row slot) << 17 |
  // (2 LDS slot + c2v half).  The tagged kernel stores every v2c to both the
  // LDS slot and the mailbox entry, branch-free: a row slot's mailbox store
  // lands out of the buffer's range (dropped by the hardware's range check),
  // a cut edge's LDS store in its mirror slot (whose c2v the column has
  // already read).  An inactive lane (past the member's columns) reads and
  // writes the dummy slots.
  int vaddr[RV][DV], vpos[RV];
  bool vact[RV];
#pragma unroll
  for (int r = 0; r < RV; ++r) {
    const int i = r * T + tid;
    vact[r] = i < NG;
    vpos[r] = member * NG + (vact[r] ? i : 0);
#pragma unroll
    for (int k = 0; k < DV; ++k)
    {
      // (an inactive lane reads the upper half of its dummy slot: the q1 word
      // it wrote itself, a probability)
      const int sl = vact[r] ? c.pt_vaddr[vpos[r] * DV + k] >> 4 : nslots + k;
      const int vx = vact[r] ? c.pt_vx[vpos[r] * DV + k] : -1;
      vaddr[r][k] = ((vx >= 0 ? vx : kMbOob) << 17) | (2 * sl + (vact[r] ? part_c2v_half(sl, EG, DC) : 1));
    }
  }
  int crow[RC], cbase[RC], crx[RC], cwb[RC];
  bool cact[RC];
#pragma unroll
  for (int r = 0; r < RC; ++r) {
    const int i = (r * T + tid) >> 1;  // lane pairs share a row
    cact[r] = i < MG;
    const int li = cact[r] ? i : 0;
    const int row = c.pt_cn[member * MG + li];
    crow[r] = row;
    cbase[r] = li * DC * 16;
    crx[r] = cact[r] ? c.pt_rx[member * MG + li] | (part_c2v_half(li * DC, EG, DC) << 7) : 0;
    // c2v write base: the row's slots + its c2v half, or the dummy slots
    cwb[r] = cact[r] ? cbase[r] + part_c2v_half(li * DC, EG, DC) * 8 : nslots * 16;
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
  __shared__ int sdead;                  // a tagged-exchange poll timed out: every wave leaves
  __shared__ int spcnt;                  // unsatisfied checks of the member's rows (tagged path)
  __shared__ int snf;                    // this member saw a prior outside the FAST domain (barrier B's flag)
  unsigned nb = 0;                       // barrier sequence number (uniform, same on every member)
  unsigned g = 0;                        // global iteration counter of the tagged exchange (same on every member)
  if (a.B_dev && *a.B_dev == 0) return;  // nothing deferred: every workgroup leaves before the first barrier
  if (tid == 0) {
    bst[0] = bst[1] = bst[2] = bst[3] = 0;
    sfail = 0;
    sdead = 0;
    snf = 0;
    const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20) & 15u;
    __hip_atomic_fetch_or(&gs->xcc, 1u << xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (part_barrier<kG>(gs, bst, nb, false, abort, nullptr) < 0) return;
  const bool same_xcd = __popc(ld_rlx(&gs->xcc)) == 1;
  // TAGGED: this launch decodes the FAST codewords of same-XCD groups with the
  // tagged exchange and defers every other codeword to a barrier-exchange
  // launch that follows it (a.defer_*); that launch takes its entry count
  // from the device (a.B_dev).
  const int B = a.B_dev ? (int)*a.B_dev : a.B;  // (read again: every read sees the finished count)

  // KML_PART_QUEUE_EARLY: after a decoded codeword, member 0 has taken the
  // next entry during the outputs and published it before their closing
  // barrier, and clears the sums after reading them, so the next codeword
  // starts without a group barrier; after a deferred codeword (no outputs, a
  // group-uniform branch) and at the start, the entry is taken here.
  bool top_sync = true;
  for (;;) {
    if (top_sync) {
      if (member == 0 && tid == 0) {
        __hip_atomic_store(&gs->cw, atomicAdd(queue, 1u), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&gs->errs, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&gs->pcnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (tid == 0) spcnt = 0;
      if (part_barrier<kG>(gs, bst, nb, same_xcd, abort, nullptr) < 0) return;
    } else if (tid == 0) {
      spcnt = 0;  // (read by this thread before the outputs' closing barrier)
    }
    top_sync = !KML_PART_QUEUE_EARLY;
    const int entry = (int)ld_rlx(&gs->cw);
    if (entry >= B) break;
    // a deferred entry with bit 31 set: a codeword the tagged launch stopped on
    // an unproven quotient, decoded here on the exact path
    const int raw = a.cw_idx ? a.cw_idx[entry] : entry;
    const int cw = raw & 0x7FFFFFFF;
    const double *p0 = a.p0 + (long long)cw * a.p0_stride;
    if (a.p0_sel) p0 += (long long)a.p0_sel[cw] * a.p0_sel_stride;

    double pv[RV];
    bool ok = raw >= 0;
#pragma unroll
    for (int r = 0; r < RV; ++r) {
      const int col = c.pt_vn[vpos[r]];
      pv[r] = (col >= c.punct) ? p0[col - c.punct] : 0.5;
      ok = ok && fast_prior_ok(pv[r], plo);
    }
    // InitMsg: row slots and mirror slots (c2v = 0.5)
    for (int e = tid; e < nslots + kPartDummy; e += T) reinterpret_cast<double2 *>(smem)[e] = make_double2(0.5, 0.5);
    // "some member holds a prior outside the FAST domain" travels as this
    // barrier's flag count, which every thread of every member reads from the
    // same arrivals.  (It was a group word that member 0 cleared at the top of
    // the next codeword: after a deferred codeword, which has no closing
    // barrier, that clear could land before a slower member's waves read the
    // word, so members and waves disagreed on fast, took different paths and
    // a group barrier timed out — tools/stress_part.py)
    if (__ballot(!ok) != 0 && (tid & 63) == 0) atomicOr(&snf, 1);
    const int nf = part_barrier<kG>(gs, bst, nb, same_xcd, abort, &snf);
    if (nf < 0) return;
    const bool fast = !EXACT && (fast_allowed & 1) && (nf & 0xFF) == 0;
    constexpr bool tagged = TAGGED;

    int iter = 0, pcnt = 0, decbuf = 0;
    bool conv = false;
    if constexpr (TAGGED) {
      if (!fast || !same_xcd) {  // to the barrier-exchange launches (bit 31: the exact one)
        if (member == 0 && tid == 0) a.defer_idx[atomicAdd(a.defer_cnt, 1u)] = fast ? cw : (int)((unsigned)cw | 0x80000000u);
        top_sync = true;
        continue;
      }
      const int st = part_iterations_tagged<kG, T, RV, RC, RX, SYN>(a, c.M, cw, gs, g, &sfail, &sdead, member, abort,
                                                                   smem, dec, NG, tb, tb_c2v, vaddr, vact, pv, crow,
                                                                   cbase, crx, cwb, cact, xr, xc, odd, iter, conv, pcnt,
                                                                   decbuf, (fast_allowed & 2) != 0);
      if (st < 0) return;
      if (st == 1) {  // an unproven quotient: redone by the exact launch (every member took this branch)
        if (member == 0 && tid == 0) {
          a.defer_idx[atomicAdd(a.defer_cnt, 1u)] = (int)((unsigned)cw | 0x80000000u);
          if (a.counters) atomicAdd(&a.counters[CNT_REDONE], 1ull);
        }
        top_sync = true;
        continue;
      }
    } else if constexpr (!EXACT) {
      int st = 1;  // 1: to the exact launch
      if (fast)
        st = part_iterations<kG, RV, RC, RX, SYN, true>(a, c.M, c.N, NG, cw, gs, bst, nb, &sfail, same_xcd, abort, smem,
                                                        dec, mb_v2c, mb_c2v, gc, c, vaddr, vpos, vact, pv, crow, cbase,
                                                        cact, xr, xc, odd, member, iter, conv, (fast_allowed & 2) != 0);
      if (st < 0) return;
      if (st == 1) {  // group-wide: not FAST, or the suspect count every member read at the same barrier
        if (member == 0 && tid == 0) {
          a.defer_idx[atomicAdd(a.defer_cnt, 1u)] = cw;
          if (fast && a.counters) atomicAdd(&a.counters[CNT_REDONE], 1ull);
        }
        top_sync = true;
        continue;
      }
    } else {
      if (part_iterations<kG, RV, RC, RX, SYN, false>(a, c.M, c.N, NG, cw, gs, bst, nb, &sfail, same_xcd, abort, smem,
                                                      dec, mb_v2c, mb_c2v, gc, c, vaddr, vpos, vact, pv, crow, cbase,
                                                      cact, xr, xc, odd, member, iter, conv) < 0)
        return;
    }

    // ---- outputs
    unsigned nxt = 0;  // KML_PART_QUEUE_EARLY: the next entry, in flight through the outputs
    if (KML_PART_QUEUE_EARLY && member == 0 && tid == 0) nxt = atomicAdd(queue, 1u);
    if (a.iter_count > 0) {
      if constexpr (tagged) {
        // a member holds the decisions of its own columns (double-buffered by
        // iteration, dec[2][NG]): it writes theirs
        for (int p = member * NG + tid; p < (member + 1) * NG; p += T) {
          const int col = c.pt_vn[p];
          const int hd = dec[decbuf * NG + (p - member * NG)];
          if (a.cc_hat) a.cc_hat[(long long)cw * c.N + col] = (uint8_t)hd;
          const int i = col - c.info_off;
          if (i >= 0 && i < c.K) {
            if (a.uu_hat) a.uu_hat[(long long)cw * c.K + i] = (uint8_t)hd;
            if (a.ref_bits) {
              const int rb = (int)((a.ref_bits[(long long)cw * c.Kw + (i >> 6)] >> (i & 63)) & 1ull);
              if (rb != hd) atomicAdd(&spcnt, 1 << 16);  // error bits in the high half
            }
          }
        }
        if (a.parity_cnt && pcnt) atomicAdd(&spcnt, pcnt);
        __syncthreads();
        if (tid == 0) {
          const int v = spcnt;
          if (v >> 16) __hip_atomic_fetch_add(&gs->errs, (unsigned)(v >> 16), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (v & 0xFFFF)
            __hip_atomic_fetch_add(&gs->pcnt, (unsigned)(v & 0xFFFF), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      } else {
        // every member holds all hard decisions in LDS (dec) and writes its share
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
            for (int k = 0; k < 3; ++k) p ^= dec[c.pt_pos[c.row_col[c.row_ptr[crow[r]] + (odd ? 3 + k : k)]]];
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
            const int nbits = min(64, c.K - base);
            for (int j = 0; j < nbits; ++j) word |= (uint64_t)dec[c.pt_pos[c.info_off + base + j]] << j;
            errs += __popcll(word ^ ref[w]);
          }
          if (errs) __hip_atomic_fetch_add(&gs->errs, (unsigned)errs, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
    // (every member read gs->cw at this codeword's start, several barriers ago)
    if (KML_PART_QUEUE_EARLY && member == 0 && tid == 0)
      __hip_atomic_store(&gs->cw, nxt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (part_barrier<kG>(gs, bst, nb, same_xcd, abort, nullptr) < 0) return;  // the members' sums are complete
    if (member == 0 && tid == 0) {
      const int errs = (int)ld_rlx(&gs->errs);
      const int pc = (int)ld_rlx(&gs->pcnt);
      if (KML_PART_QUEUE_EARLY) {  // no member adds to the sums before the next codeword's flag barrier
        __hip_atomic_store(&gs->errs, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&gs->pcnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      if (a.ret) a.ret[cw] = iter + (iter < a.max_iter);
      if (a.iters) a.iters[cw] = iter;
      if (a.parity_cnt) a.parity_cnt[cw] = a.iter_count > 0 ? pc : 0;
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

// Launch of a grid whose workgroups must all be co-resident (the group
// barriers and tag polls wait on each other): a cooperative launch, which
// also keeps another process's kernels from taking CUs the grid needs (two
// ranks sharing one GPU).  KML_COOP_LAUNCH=0 launches plainly after the same
// occupancy check, for rocprofv3 --pmc runs only: a cooperative launch under
// counter collection crashed the profiled process at exit.  A group that is
// not co-resident times out its polls and aborts the launch (bp_coop_aborted).
hipError_t launch_resident(const void *kern, unsigned grid, unsigned block, void **args, unsigned lds, hipStream_t s) {
  if (const char *e = getenv("KML_COOP_LAUNCH"))
    if (e[0] == '0') {
      int per_cu = 0, dev = 0, ncu = 0;
      hipError_t r = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, (int)block, lds);
      if (r != hipSuccess) return r;
      hipGetDevice(&dev);
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
      if ((long long)per_cu * ncu < (long long)grid) return hipErrorCooperativeLaunchTooLarge;
      return hipLaunchKernel(kern, dim3(grid), dim3(block), args, lds, s);
    }
  return hipLaunchCooperativeKernel(kern, dim3(grid), dim3(block), args, lds, s);
}

template <int kG, int T, int RV, int RC, int RX, bool SYN, bool TAGGED, bool EXACT>
hipError_t launch_part_t(const DevCode &c, const BpLaunch &a, hipStream_t s, int fast, int groups, bool reset_abort) {
  auto kern = bp_part_kernel<kG, T, RV, RC, RX, SYN, TAGGED, EXACT>;
  const size_t lds = part_lds_bytes(c);
  hipError_t e = hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(a.queue, 0, sizeof(unsigned int), s);
  if (e != hipSuccess) return e;
  // the group blocks, and the abort word unless this launch follows one whose abort must persist
  e = hipMemsetAsync(a.gsync, 0, sizeof(GroupSync) * (size_t)groups + (reset_abort ? 2 * sizeof(unsigned) : 0), s);
  if (e != hipSuccess) return e;
  if (TAGGED) {  // every tagged mailbox word starts with tag 1 (the first iteration writes tag 0)
    e = hipMemsetAsync(a.gslots, 0xFF, sizeof(double2) * (size_t)groups * c.E, s);
    if (e != hipSuccess) return e;
  }
  DevCode cc = c;
  BpLaunch aa = a;
  GroupSync *gs = reinterpret_cast<GroupSync *>(a.gsync);
  uint8_t *gcch = a.gcch;
  unsigned *abort = reinterpret_cast<unsigned *>(gs + groups);
  unsigned int *q = a.queue;
  int f = fast;
  void *args[] = {&cc, &aa, &gs, &gcch, &abort, &q, &f};
  return launch_resident((const void *)kern, (unsigned)(groups * kG), (unsigned)T, args, (unsigned)lds, s);
}

// The partitioned kernel's launches for one batch.  a.defer_* (the caller's
// list) receives the codewords for the exact launch; d.defer_* (scratch past
// the groups' mailboxes) the tagged launch's deferrals.
template <int kG, int T_, int R_, int X_, bool SYN>
hipError_t launch_part_chain(const DevCode &c, const BpLaunch &a, const BpLaunch &d, hipStream_t s, int fast, int groups,
                             bool tagged) {
  if (!(fast & 1)) return launch_part_t<kG, T_, R_, R_, X_, SYN, false, true>(c, a, s, 0, groups, a.reset_abort);
  if (!a.defer_idx || !a.defer_cnt) return hipErrorInvalidValue;
  hipError_t e = hipMemsetAsync(a.defer_cnt, 0, sizeof(unsigned), s);
  if (e != hipSuccess) return e;
  BpLaunch bf = a;  // barrier-exchange FAST launch: the whole batch, or the tagged launch's deferrals
  bool reset = a.reset_abort;
  if (tagged) {
    e = launch_part_t<kG, T_, R_, R_, X_, SYN, true, false>(c, d, s, fast, groups, reset);
    if (e != hipSuccess) return e;
    bf.cw_idx = d.defer_idx;
    bf.B_dev = d.defer_cnt;
    reset = false;  // an abort of an earlier launch stays visible
  }
  e = launch_part_t<kG, T_, R_, R_, X_, SYN, false, false>(c, bf, s, fast, groups, reset);
  if (e != hipSuccess) return e;
  BpLaunch be = a;  // exact launch over what the FAST launches deferred
  be.cw_idx = a.defer_idx;
  be.B_dev = a.defer_cnt;
  return launch_part_t<kG, T_, R_, R_, X_, SYN, false, true>(c, be, s, 0, groups, false);
}

// Tiling of the partitioned kernel: KML_PART = threads per workgroup (512,
// 768 or 1024; default 1024).
int part_threads() {
  if (const char *e = getenv("KML_PART")) {
    const int t = atoi(e);
    if (t == 512 || t == 768 || t == 1024) return t;
  }
  return 1024;
}

}  // namespace

size_t bp_coop_sync_bytes(int groups) { return part_defer_offset(groups) + 16; }

int bp_part_group_size(int N, int M, int E, int dv_max, int dc_max, int regular) {
  if (!regular || dv_max != 3 || dc_max != 6 || (long long)E * 16 + 16 + N <= 160 * 1024) return 0;
  const int G = kPartG;
  if (N % G || M % G || (N / G) % 16) return 0;
  // tilings up to 2048 columns and half-rows per member; the LDS check
  // including the mirror slots is part_plan_fits (after planning)
  const int NG = N / G, MG = M / G;
  return ((long long)MG * 6 * 16 + N <= 160 * 1024 && NG <= 2048 && 2 * MG <= 2048) ? G : 0;
}

bool part_plan_fits(int G, int N, int M, int E, int ncut, int mirror_max, int xmax) {
  const long long lds = ((long long)M / G * 6 + mirror_max + kPartDummy) * 16 + N;
  return G == kPartG && lds <= 160 * 1024 && 3LL * ncut <= 2LL * E && xmax <= 2 * 1024;
}

// Codes without a partition plan (or whose plan did not fit) decode on the
// generic bp_kernel (launch_bp_coop returns hipErrorNotSupported).
int bp_coop_groups(const DevCode &c) {
  if (!c.regular || !c.reg_pos || c.dv_max != 3 || c.dc_max != 6 || bp_uses_lds(c)) return 0;
  if (c.pt_G != kPartG || c.pt_vn == nullptr) return 0;
  int dev = 0, ncu = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  return (ncu / (8 * kPartG)) * 8;  // 8 XCDs, groups of 4 per XCD
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

const char *bp_coop_family(const DevCode &) { return "bp_part_kernel"; }

hipError_t launch_bp_coop(const DevCode &c, const BpLaunch &a, hipStream_t s) {
  const int groups = bp_coop_groups(c);
  if (groups <= 0 || !a.gsync || !a.gcch || (long long)groups * c.E > a.gslots_cap) return hipErrorNotSupported;
  if (const char *k = getenv("KML_BP_KERNEL"))
    if (k[0] == 'g') return hipErrorNotSupported;
  const int fast = bp_fast_mode(c);
  const int T = part_threads();
  {
    // exchange entries per thread: every member's lists must fit RX * T
    int xmax = 0;
    for (int m = 0; m < c.pt_G; m++) xmax = std::max(xmax, std::max(c.pt_xr_n[m], c.pt_xc_n[m]));
    // Tagged exchange (default): one launch for the FAST codewords of same-XCD
    // groups, then a barrier-exchange launch over the codewords it deferred
    // (list and count in scratch past the groups' mailboxes / sync blocks).
    bool tagged = part_tagged_fits(c.E, c.pt_ncut) && fast;
    if (const char *t = getenv("KML_PART_TAGGED"))
      if (t[0] == '0') tagged = false;
    BpLaunch d = a;
    if (tagged) {
      // the tagged launch's defer list past the groups' mailboxes
      const long long mb = (long long)groups * part_group_stride(c);
      if ((a.gslots_cap - mb) * 16 < 5LL * a.B + 64) return hipErrorNotSupported;
      d.defer_idx = reinterpret_cast<int32_t *>(a.gslots + (size_t)mb);
      d.defer_cnt = reinterpret_cast<unsigned *>(reinterpret_cast<char *>(a.gsync) + part_defer_offset(groups));
      hipError_t e = hipMemsetAsync(d.defer_cnt, 0, sizeof(unsigned), s);
      if (e != hipSuccess) return e;
    }
#define KML_PART_CASE(G_, T_, R_, X_)                \
  if (T == T_ && xmax <= X_ * T_) \
    return a.syn ? launch_part_chain<G_, T_, R_, X_, true>(c, a, d, s, fast, groups, tagged) \
                 : launch_part_chain<G_, T_, R_, X_, false>(c, a, d, s, fast, groups, tagged);
    KML_PART_CASE(4, 512, 4, 4)
    KML_PART_CASE(4, 768, 3, 3)
    KML_PART_CASE(4, 1024, 2, 2)
#undef KML_PART_CASE
    return hipErrorNotSupported;
  }
}

hipError_t bp_coop_raise_abort(const BpLaunch &a, int groups, hipStream_t s) {
  return hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(reinterpret_cast<GroupSync *>(a.gsync) + groups), 1u, 1, s);
}

// Did the last cooperative launch abort (a poll timed out)?  why: the first
// aborter's site << 24 | workgroup (0: raised by the host, kml_debug_inject_abort).
bool bp_coop_aborted(const BpLaunch &a, int groups, hipStream_t s, unsigned *why) {
  unsigned v[2] = {0, 0};
  hipMemcpyAsync(v, reinterpret_cast<GroupSync *>(a.gsync) + groups, sizeof(v), hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  if (why) *why = v[1];
  return v[0] != 0;
}

}  // namespace kml

#if KML_DIV_STATS
KML_DIV_STATS_ACCESSOR(kml_debug_div_stats_coop)
#endif
