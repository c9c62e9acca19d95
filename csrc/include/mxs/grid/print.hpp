// Text output compatible with the reference (Print, TestSubRegionExtraction:
// stencil2d/stencil2D.h:92-102, 441-510) and the per-rank dump file of the
// stencil apps (stencil2d/mpi-2d-stencil-subarray.cpp:60-98).
#pragma once

#include <ostream>
#include <string>
#include <vector>

#include "mxs/grid/regions.hpp"
#include "mxs/topo/cart.hpp"

namespace mxs {

// One line per row, every value followed by a space (std::ostream default
// formatting: -1, 0, 8, 0.25 ...).
template <typename T>
void print_region(std::ostream& os, const T* data, const Array2D& g) {
  for (index_t y = 0; y < g.height; ++y) {
    for (index_t x = 0; x < g.width; ++x) os << data[g.index(x, y)] << ' ';
    os << '\n';
  }
}

// The reference's region self-test, reproduced for its unit test: it pads only
// one side of the grid (w + s/2) and prints every region of the
// grid and of its core.
inline void test_subregion_extraction(std::ostream& os) {
  const int w = 32, h = 32, sw = 5, sh = 5;
  const int tw = w + sw / 2, th = h + sh / 2;
  const Array2D grid(tw, th, tw);
  static const char* labels[] = {"top left:      ", "top center:    ", "top right:     ",
                                 "center left:   ", "center:        ", "center right:  ",
                                 "bottom left:   ", "bottom center: ", "bottom right:  ",
                                 "top:           ", "left:          ", "bottom:        ",
                                 "right:         "};
  os << "\nGRID TEST\n";
  os << "Width: " << tw << ", " << "Height: " << th << '\n';
  os << "Stencil: " << sw << ", " << sh << '\n';
  for (int r = TOP_LEFT; r <= BOTTOM_RIGHT; ++r)
    os << labels[r] << sub_array_region(grid, sw, sh, RegionID(r)) << '\n';
  os << "\nSUBGRID TEST\n";
  const Array2D core = sub_array_region(grid, sw, sh, CENTER);
  os << "Width: " << core.width << ", " << "Height: " << core.height << '\n';
  os << "Stencil: " << sw << ", " << sh << '\n';
  for (int r = TOP_LEFT; r <= BOTTOM_RIGHT; ++r)
    os << labels[r] << sub_array_region(core, sw, sh, RegionID(r)) << '\n';
  // The reference printed the strips in the order top, right, bottom, left.
  for (RegionID r : {TOP, RIGHT, BOTTOM, LEFT}) os << labels[r] << sub_array_region(core, sw, sh, r) << '\n';
}

// Header of a per-rank dump file (everything up to the first "Array" line).
inline void write_dump_header(std::ostream& os, const CartTopology& topo, int rank, int device_id,
                              index_t local_w, index_t local_h, int sw, int sh, const char* device_label) {
  const auto c = topo.coords(rank);
  os << "Rank:  " << rank << '\n' << "Coord: " << c[0] << ", " << c[1] << '\n';
  if (device_id >= 0) os << '\n' << device_label << " device id: " << device_id << '\n';
  os << '\n' << "Compute grid" << '\n';
  print_cartesian_grid(os, topo);
  os << '\n';
  os << local_w << " x " << local_h << " grid size" << '\n';
  os << local_w + 2 * (sw / 2) << " x " << local_h + 2 * (sh / 2) << " total(with ghost/halo regions) grid size"
     << '\n';
  os << sw << " x " << sh << " stencil\n" << '\n';
}

inline std::string dump_file_name(const CartTopology& topo, int rank) {
  const auto c = topo.coords(rank);
  return std::to_string(c[0]) + "_" + std::to_string(c[1]);
}

}  // namespace mxs
