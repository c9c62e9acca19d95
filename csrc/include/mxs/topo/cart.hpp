// Cartesian process grid (reference: MPI_Cart_create/MPI_Cart_coords/MPI_Cart_rank
// usage at stencil2d/mpi-2d-stencil-subarray.cpp:42-58, OffsetTaskId
// stencil2d/stencil2D.h:232-244, PrintCartesianGrid :513-530).
//
// Pure arithmetic so that the same topology drives the MPI backends, the RCCL
// backend (which has no notion of a Cartesian communicator) and the Python
// torch.distributed backends. Rank order is row-major, identical to
// MPI_Cart_create with reorder = 0: rank = row * cols + col, coords = {row, col}.
//
// New vs the reference: any process count (not just perfect squares)
// via a MPI_Dims_create-compatible factorisation; non-periodic dimensions; the
// neighbour of a rank is computed from its *own* Cartesian rank (the reference
// mixed the MPI_COMM_WORLD rank into that computation).
#pragma once

#include <array>
#include <ostream>
#include <stdexcept>
#include <string>
#include <vector>

#include "mxs/grid/regions.hpp"

namespace mxs {

constexpr int kProcNull = -1;  // same role as MPI_PROC_NULL (printed as -1 by MPICH)

struct CartTopology {
  int rows = 1;  // dims[0]
  int cols = 1;  // dims[1]
  bool periodic_rows = true;
  bool periodic_cols = true;

  CartTopology() = default;
  CartTopology(int r, int c, bool prow = true, bool pcol = true)
      : rows(r), cols(c), periodic_rows(prow), periodic_cols(pcol) {
    if (r < 1 || c < 1) throw std::invalid_argument("CartTopology: dims must be >= 1");
  }

  int size() const { return rows * cols; }
  std::array<int, 2> coords(int rank) const { return {rank / cols, rank % cols}; }
  int rank_of(int row, int col) const {
    if (row < 0 || row >= rows) {
      if (!periodic_rows) return kProcNull;
      row = ((row % rows) + rows) % rows;
    }
    if (col < 0 || col >= cols) {
      if (!periodic_cols) return kProcNull;
      col = ((col % cols) + cols) % cols;
    }
    return row * cols + col;
  }
  // Rank at offset (dx columns, dy rows) from `rank`; kProcNull off a
  // non-periodic edge.
  int shift(int rank, int dx, int dy) const {
    const auto c = coords(rank);
    return rank_of(c[0] + dy, c[1] + dx);
  }
  int neighbor(int rank, int dir) const {
    const DirOffset o = dir_offset(dir);
    return shift(rank, o.dx, o.dy);
  }
  // MPI_Cart_shift semantics along dimension `dim` (0 = rows, 1 = cols).
  std::array<int, 2> cart_shift(int rank, int dim, int disp) const {
    if (dim == 0) return {shift(rank, 0, -disp), shift(rank, 0, disp)};
    return {shift(rank, -disp, 0), shift(rank, disp, 0)};
  }
};

// Balanced 2D factorisation with the MPI_Dims_create contract (dims[0] >= dims[1],
// as close to square as possible): 8 -> 4x2, 9 -> 3x3, 6 -> 3x2, 7 -> 7x1.
inline std::array<int, 2> dims_create(int n) {
  if (n < 1) throw std::invalid_argument("dims_create: n must be >= 1");
  int best = 1;
  for (int d = 1; d * d <= n; ++d)
    if (n % d == 0) best = d;
  return {n / best, best};
}

// Parse "RxC" (e.g. "2x4"); returns {0, 0} on a malformed string.
inline std::array<int, 2> parse_dims(const std::string& s) {
  const auto p = s.find_first_of("xX");
  if (p == std::string::npos) return {0, 0};
  try {
    return {std::stoi(s.substr(0, p)), std::stoi(s.substr(p + 1))};
  } catch (...) {
    return {0, 0};
  }
}

// Reference text format: the rank grid, one row per line, each id followed by a
// space (stencil2d/stencil2D.h:513-530).
inline void print_cartesian_grid(std::ostream& os, const CartTopology& t) {
  for (int r = 0; r < t.rows; ++r) {
    for (int c = 0; c < t.cols; ++c) os << t.rank_of(r, c) << ' ';
    os << '\n';
  }
}

// Block decomposition of a global extent n over p parts; part i gets
// [start, start + len). Remainder cells go to the first parts.
struct Block1D {
  index_t start, len;
};
inline Block1D block_split(index_t n, int p, int i) {
  const index_t base = n / p, rem = n % p;
  const index_t len = base + (i < rem ? 1 : 0);
  const index_t start = i * base + (i < rem ? i : rem);
  return {start, len};
}

}  // namespace mxs
