// code.hpp — host-side LDPC code planner.
//
// Replaces the reference's Tanner-graph construction (orthogonal linked lists of
// 104-byte `Edge` nodes, lib/lab/include/utility.h:23-34) with flat arrays laid
// out for the gfx950 decoder:
//
//   * edge SLOT order = the reference's row traversal order: rows 0..M-1, and
//     inside a row the order of row_head->right (descending permuted column
//     after SystemMatrixH, lib/lab/src/binaryldpccodec.cc:465-481; reverse file
//     order when [ldpc] active = false, :107-123).  A CN thread therefore reads
//     its row's messages as one contiguous run of 16-byte slots.
//   * col_slot = for each column, its slot ids in column-list order
//     (col_head->down: descending row index).
//   * vn_order / cn_order = processing order of columns / rows inside a phase,
//     sorted by degree so a 64-lane wavefront walks equal-length chains.  The
//     phases are order-independent (every column / row owns disjoint slots), so
//     this changes no bit of the result.
//
// The GF(2) systematic elimination reproduces SystemMatrixH exactly (forward
// pivot search for PEG, binaryldpccodec.cc:386-431; backward for 5G,
// binary5gldpccodec.cc:281-325), on a bit-packed matrix.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace kml {

struct LdpcCode {
  // dimensions
  int M = 0;       // check rows
  int N = 0;       // internal columns (num_col_), incl. punctured ones for 5G
  int K = 0;       // info bits (code_dim_)
  int cc_len = 0;  // transmitted bits
  int Z = 0;       // 5G lifting factor (0 for PEG)
  int E = 0;       // edges
  int chk = 0;     // code_chk_ (GF(2) rank found by the elimination)
  int punct = 0;   // leading punctured columns with prior 0.5 (2Z for 5G)
  int info_off = 0;  // uu_hat[i] = cc_hat[i + info_off]
  bool is5g = false, active = true;
  int dv_max = 0, dc_max = 0;

  std::vector<int32_t> perm;      // tempP: new column j = file column perm[j]
  std::vector<int32_t> row_ptr;   // M+1
  std::vector<int32_t> row_col;   // E: column of each slot
  std::vector<int32_t> col_ptr;   // N+1
  std::vector<int32_t> col_slot;  // E
  std::vector<int32_t> vn_order;  // N
  std::vector<int32_t> cn_order;  // M

  // Encoder: parity bit t = <enc_info row t, uu> over GF(2); rows packed in Kw
  // 64-bit words over the K info bits.  Codeword assembly is described by
  // `layout`: PEG = [parity(chk) | info(K)], 5G = [info(K) | parity(chk)]
  // with the first 2Z bits dropped (binaryldpccodec.cc:148-155,
  // binary5gldpccodec.cc:92-102).
  int Kw = 0;
  std::vector<uint64_t> enc_info;  // chk x Kw

  bool load(const std::string &path, bool is5g, bool active, bool reversed_rows, std::string &err);
  // host encoder (used by the C++ driver's CPU-side checks and tests)
  void encode(const uint8_t *uu, uint8_t *cc) const;
};

}  // namespace kml
