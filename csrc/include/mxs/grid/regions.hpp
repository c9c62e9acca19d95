// Region algebra of a tile (reference: RegionID + SubArrayRegion,
// stencil2d/stencil2D.h:79-201).
//
// A window g is cut by a stencil of size sw x sh (ghost width gw = sw/2,
// ghost height gh = sh/2) into a 3x3 partition (TOP_LEFT .. BOTTOM_RIGHT) plus
// four full-length strips (TOP, LEFT, BOTTOM, RIGHT). The numeric values of
// RegionID are observable: the reference uses them as MPI tags and so does the
// MPI backend here.
//
// Unlike the reference the regions are defined with *physical* semantics:
// x is the column (fastest-varying) axis and y the row axis. The reference
// handed {width, height} to MPI_Type_create_subarray in MPI_ORDER_C and so
// transposed every region; for square tiles the two
// transpositions cancelled, which is why its golden outputs still match ours.
#pragma once

#include <array>
#include <string>

#include "mxs/grid/layout.hpp"

namespace mxs {

enum RegionID : int {
  TOP_LEFT = 0,
  TOP_CENTER = 1,
  TOP_RIGHT = 2,
  CENTER_LEFT = 3,
  CENTER = 4,
  CENTER_RIGHT = 5,
  BOTTOM_LEFT = 6,
  BOTTOM_CENTER = 7,
  BOTTOM_RIGHT = 8,
  TOP = 9,
  LEFT = 10,
  BOTTOM = 11,
  RIGHT = 12,
};
constexpr int kNumRegions = 13;

inline const char* region_name(RegionID r) {
  static const char* names[kNumRegions] = {
      "top left", "top center", "top right", "center left", "center", "center right",
      "bottom left", "bottom center", "bottom right", "top", "left", "bottom", "right"};
  return (r >= 0 && r < kNumRegions) ? names[r] : "invalid";
}

// Window of region `rid` inside window `g` (same row stride as g).
inline Array2D sub_array_region(const Array2D& g, int stencil_width, int stencil_height,
                                RegionID rid) {
  const index_t gw = stencil_width / 2;
  const index_t gh = stencil_height / 2;
  const index_t x0 = g.x_offset, y0 = g.y_offset;
  const index_t xin = x0 + gw, yin = y0 + gh;                    // inner start
  const index_t xr = x0 + g.width - gw, yb = y0 + g.height - gh;  // right / bottom band start
  const index_t win = g.width - 2 * gw, hin = g.height - 2 * gh;  // inner extents
  const index_t s = g.row_stride;
  switch (rid) {
    case TOP_LEFT:      return Array2D(gw, gh, s, x0, y0);
    case TOP_CENTER:    return Array2D(win, gh, s, xin, y0);
    case TOP_RIGHT:     return Array2D(gw, gh, s, xr, y0);
    case CENTER_LEFT:   return Array2D(gw, hin, s, x0, yin);
    case CENTER:        return Array2D(win, hin, s, xin, yin);
    case CENTER_RIGHT:  return Array2D(gw, hin, s, xr, yin);
    case BOTTOM_LEFT:   return Array2D(gw, gh, s, x0, yb);
    case BOTTOM_CENTER: return Array2D(win, gh, s, xin, yb);
    case BOTTOM_RIGHT:  return Array2D(gw, gh, s, xr, yb);
    case TOP:           return Array2D(g.width, gh, s, x0, y0);
    case LEFT:          return Array2D(gw, g.height, s, x0, y0);
    case BOTTOM:        return Array2D(g.width, gh, s, x0, yb);
    case RIGHT:         return Array2D(gw, g.height, s, xr, y0);
  }
  return Array2D();
}

// The eight neighbour directions of a Cartesian rank, in the order the
// reference enumerates its transfers (stencil2d/stencil2D.h:389-391): row-major
// over (dy, dx) skipping the centre. This order is the canonical message order
// of every halo backend.
enum Dir : int { D_TOP_LEFT = 0, D_TOP, D_TOP_RIGHT, D_LEFT, D_RIGHT, D_BOTTOM_LEFT, D_BOTTOM, D_BOTTOM_RIGHT };
constexpr int kNumDirs = 8;

struct DirOffset {
  int dx, dy;
};
// dy = -1 is the row above (smaller row index), dx = -1 the column to the left.
MXS_HD DirOffset dir_offset(int d) {
  constexpr int dxs[kNumDirs] = {-1, 0, 1, -1, 1, -1, 0, 1};
  constexpr int dys[kNumDirs] = {-1, -1, -1, 0, 0, 1, 1, 1};
  return DirOffset{dxs[d], dys[d]};
}
MXS_HD int dir_opposite(int d) { return kNumDirs - 1 - d; }
MXS_HD bool dir_is_corner(int d) { return d == D_TOP_LEFT || d == D_TOP_RIGHT || d == D_BOTTOM_LEFT || d == D_BOTTOM_RIGHT; }

inline const char* dir_name(int d) {
  static const char* n[kNumDirs] = {"top-left", "top", "top-right", "left", "right", "bottom-left", "bottom", "bottom-right"};
  return (d >= 0 && d < kNumDirs) ? n[d] : "invalid";
}

// Core-edge region of a tile sent towards direction d (the band of core cells
// that the neighbour at d needs as its ghost cells).
inline Array2D send_region(const TileGeom& t, int d) {
  const Array2D c = t.core();
  const DirOffset o = dir_offset(d);
  const index_t w = o.dx == 0 ? c.width : t.halo_x;
  const index_t h = o.dy == 0 ? c.height : t.halo_y;
  const index_t x = o.dx < 0 ? c.x_offset : (o.dx > 0 ? c.x_offset + c.width - t.halo_x : c.x_offset);
  const index_t y = o.dy < 0 ? c.y_offset : (o.dy > 0 ? c.y_offset + c.height - t.halo_y : c.y_offset);
  return Array2D(w, h, t.pitch, x, y);
}

// Ghost region of a tile that receives data from the neighbour at direction d.
inline Array2D recv_region(const TileGeom& t, int d) {
  const Array2D c = t.core();
  const DirOffset o = dir_offset(d);
  const index_t w = o.dx == 0 ? c.width : t.halo_x;
  const index_t h = o.dy == 0 ? c.height : t.halo_y;
  const index_t x = o.dx < 0 ? c.x_offset - t.halo_x : (o.dx > 0 ? c.x_offset + c.width : c.x_offset);
  const index_t y = o.dy < 0 ? c.y_offset - t.halo_y : (o.dy > 0 ? c.y_offset + c.height : c.y_offset);
  return Array2D(w, h, t.pitch, x, y);
}

}  // namespace mxs
