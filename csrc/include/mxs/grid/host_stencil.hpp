// Host (CPU) stencil update — the CPU path of the stencil apps and the exact
// reference the HIP kernels are tested against. Same formula and evaluation
// order as kernels::stencil5_rows: fma(c1, (n + s) + (w + e), c0 * c).
#pragma once

#include <cmath>

#include "mxs/grid/layout.hpp"

namespace mxs {

template <typename T>
void jacobi5_host(const T* in, T* out, const TileGeom& g, index_t r0, index_t r1, T c0, T c1) {
  const index_t p = g.pitch;
  for (index_t y = r0; y < r1; ++y) {
    const T* row = in + g.core_offset() + y * p;
    T* o = out + g.core_offset() + y * p;
    for (index_t x = 0; x < g.width; ++x)
      o[x] = std::fma(c1, (row[x - p] + row[x + p]) + (row[x - 1] + row[x + 1]), c0 * row[x]);
  }
}

}  // namespace mxs
