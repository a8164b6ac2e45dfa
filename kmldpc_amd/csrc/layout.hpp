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
