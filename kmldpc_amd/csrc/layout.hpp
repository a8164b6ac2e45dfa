// layout.hpp — LDS placement plan for the regular-code BP kernel (bp_regular.hip).
//
// The kernel keeps one 16-byte slot per edge in LDS, in the reference's row
// traversal order (rows contiguous, so a check-row lane pair reads its row as
// consecutive slots).  The variable-node phase gathers and scatters those slots
// by column, which on gfx950 serialises on LDS banks (MI355X_MICROARCH.md §LDS:
// ds_read_b64 banks by 32-lane halves mod 64 dwords, ds_write_b128 by 8-lane
// groups mod 32 dwords).  The plan changes nothing in the arithmetic; it picks
//   * which lane owns which column (`order`, any permutation is valid: the VN
//     phase is column-independent), by simulated annealing on the bank-conflict
//     count of the VN gathers/scatters, and
//   * which half of its slot a check-to-variable message is written to
//     (`c2v_addr`): rows whose position in the CN phase has bit 2 set store it
//     in the upper 8 bytes, which makes the CN phase's 16-lane ds_write_b64
//     groups conflict-free (8 rows x 2 edges on 16 distinct bank pairs).
#pragma once
#include <cstdint>
#include <vector>

#include "code.hpp"

namespace kml {

struct RegularLayout {
  std::vector<int32_t> order;     // position -> column (position = r*T + thread)
  std::vector<int32_t> pos;       // column -> position
  std::vector<int32_t> c2v_addr;  // aligned with col_slot: byte offset of the c2v message
  long long cost_initial = 0;     // modelled extra LDS cycles per VN phase (all waves)
  long long cost_final = 0;
};

// T = threads per workgroup of the kernel (positions are grouped by wave).
void plan_regular_layout(const LdpcCode &L, int T, RegularLayout &out);

}  // namespace kml

namespace kml {

// Partition plan for the partitioned cooperative BP kernel (bp_coop.hip,
// bp_part_kernel): a group of G workgroups decodes one codeword; member m owns
// the rows [m*MG, (m+1)*MG) and the columns [m*NG, (m+1)*NG) of the orders
// below.  Its LDS holds the 16-byte slots of its rows (slot (P - m*MG)*dc + k
// for the k-th edge of the row at plan index P) followed by one MIRROR slot per
// CUT edge of its columns (an edge whose row another member owns).  Cut edges
// are exchanged through two mailboxes in global memory, v2c (column owner ->
// row owner) and c2v (row owner -> column owner), indexed by the cut-edge
// index x, which is sorted by (row owner, row slot): each row owner's share
// is one contiguous run and the cut edges of one row are consecutive (the
// tagged exchange addresses a row's mailbox entries from its first index and
// a 6-bit mask); each column owner's share is a few runs.  The planner
// minimises the number of cut edges (balanced G-way partition of the Tanner
// graph: alternating majority assignment of columns given rows and rows given
// columns, capacity-bounded).  Any partition gives the same decoder output: it
// only moves work between lanes.
struct PartitionPlan {
  int G = 0, MG = 0, NG = 0;
  int ncut = 0;                 // cut edges (mailbox entries)
  int mirror_max = 0;           // most mirror slots of one member
  std::vector<int32_t> vn;      // N: columns in member order (member m: [m*NG, (m+1)*NG))
  std::vector<int32_t> cn;      // M: rows in member order
  std::vector<int32_t> pos;     // N: column -> index into vn
  std::vector<int32_t> vaddr;   // 3N (dv = 3): [p*dv + k] = LDS byte offset of the k-th edge of column vn[p]
                                // in its owner's LDS (a row slot or a mirror slot)
  // exchange lists, per member [ptr[m], ptr[m+1]); entry = (x << 16) | (LDS slot index)
  std::vector<int32_t> xr, xr_ptr;  // as row owner: cut edges of its rows
  std::vector<int32_t> xc, xc_ptr;  // as column owner: cut edges of its columns (-> mirror slots)
  // tagged exchange (bp_part_kernel's direct mailbox stores):
  std::vector<int32_t> vx;  // 3N: [p*dv + k] = mailbox index x of that edge when it is cut, else -1
  std::vector<int32_t> rx;  // M, plan order: (x of the row's first cut edge << 8) | mask of its cut
                            // edges by position in the row (0 when none are cut)
  long long anneal_initial = 0, anneal_final = 0;  // VN bank-conflict model cost before / after annealing
  int interior = 0;  // columns whose edges are all their member's (each member's last run of vn)
  // every member owns rows that receive cut-edge v2c messages from every other
  // member (the tagged exchanges' ordering arguments use it, bp_coop.hip)
  bool all_pairs = false;
};

// False when the code is not regular or M, N are not multiples of G.
bool plan_partition(const LdpcCode &L, int G, PartitionPlan &out);

}  // namespace kml

namespace kml {

// Round plan of the irregular-code BP kernel (bp_irregular.hip): T threads in
// W = T/64 waves, three rounds per phase.  In rounds 0 and 1 a lane owns TWO
// columns (two half-rows) of the same degree and runs their chains
// interleaved; round 2 holds single columns (half-rows).  Every wave of a
// round runs one degree (64 columns, or 32 rows as lane pairs), except at
// most a few waves that mix the leftovers of two degrees.  Pairs are formed
// from the highest degrees up to a limit (the longest dependent chains gain
// most from a second chain; the limits keep two chains within the registers), and the waves are placed so that the modelled VALU work of
// the 4 SIMDs (wave w runs on SIMD w % 4) is balanced.  Any placement gives
// the same decoder output: it only moves work between lanes.
constexpr int kIrrThreads = 768;  // threads per workgroup of bp_irregular.hip (its plan is made for this)
#ifndef KML_IRR_VN_PAIR_MAX  // overridable for experiment builds (Makefile "variant")
#define KML_IRR_VN_PAIR_MAX 4
#endif
#ifndef KML_IRR_CN_PAIR_MAX
#define KML_IRR_CN_PAIR_MAX 8
#endif
constexpr int kIrrVnPairMax = KML_IRR_VN_PAIR_MAX;  // highest column degree bp_irregular.hip pairs
constexpr int kIrrCnPairMax = KML_IRR_CN_PAIR_MAX;  // highest row degree it pairs (BG2, 50 iterations: 4/8 19.7 ms,
                                  // 5/8 20.5, 7/8 21.8, 9/8 23.0 with c2v reloads against spills)

// Slot layout of the irregular kernel: the rows of a wave's round (32 lane
// pairs, one degree) form a block in which edge e of the row at pair index pi
// sits at slot pi + e * kIrrCnStride, so at every CN step a wave reads two
// contiguous 512-byte runs (conflict-free b128 reads) instead of 32 rows
// strided by their degree.
constexpr int kIrrCnStride = 32;

struct IrregularPlan {
  std::vector<int32_t> vn;        // [3*T]: column of position r*T + t, -1 = idle
  std::vector<int32_t> cn;        // [3*T/2]: row of lane pair r*T/2 + (t >> 1), -1 = idle
  std::vector<int32_t> cn_base;   // [3*T/2]: slot of edge 0 of that row, -1 = idle
  std::vector<int32_t> col_slot;  // [E]: slot of each column-ordered edge (as LdpcCode::col_slot)
  int n_slots = 0;                // slots incl. the holes of partly filled blocks
};

// False when the code's degree groups do not fit three rounds of T lanes.
bool plan_irregular(const LdpcCode &L, int T, int vn_pair_max, int cn_pair_max, IrregularPlan &out);

}  // namespace kml

