// Host implementation of the deterministic random init used by
// kernels::fill_random (csrc/kernels/fill.hip): the value of a cell depends only
// on its global coordinates and the seed, so CPU and GPU runs of any
// decomposition start from identical data.
#pragma once

#include <cstdint>

#include "mxs/grid/layout.hpp"

namespace mxs {

inline std::uint64_t mix64(std::uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <typename T>
void fill_random_host(T* tile, const TileGeom& g, index_t gx0, index_t gy0, index_t gw, std::uint64_t seed) {
  const std::uint64_t hs = mix64(seed);
  for (index_t y = 0; y < g.height; ++y)
    for (index_t x = 0; x < g.width; ++x) {
      const std::uint64_t h = mix64(std::uint64_t((gy0 + y) * gw + (gx0 + x)) ^ hs);
      tile[g.core_offset() + y * g.pitch + x] = T(double(h >> 40) * (1.0 / 16777216.0));
    }
}

}  // namespace mxs
