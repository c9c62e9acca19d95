// Built with -DMXS_DEBUG_BOUNDS: in-window accesses work, an
// out-of-window access aborts with the coordinates (argv[1] == "oob").
#include <cstdio>
#include <cstring>
#include <vector>

#include "mxs/grid/layout.hpp"

int main(int argc, char** argv) {
  using namespace mxs;
  const TileGeom g = TileGeom::compact(6, 4, 1, 1);
  std::vector<double> buf(size_t(g.alloc_elems()), 0.0);
  Accessor2D<double> core(buf.data(), g.core());
  for (index_t y = 0; y < 4; ++y)
    for (index_t x = 0; x < 6; ++x) core(x, y) = double(y * 6 + x);
  double sum = 0;
  for (index_t y = 0; y < 4; ++y)
    for (index_t x = 0; x < 6; ++x) sum += core(x, y);
  std::printf("sum %g\n", sum);
  if (argc > 1 && std::strcmp(argv[1], "oob") == 0) core(6, 0) = 1.0;  // one past the core row
  return 0;
}
