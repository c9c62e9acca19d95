// 2D layouts and accessors (reference: Array2D / Array2DAccessor,
// stencil2d/stencil2D.h:30-75).
//
// Differences from the reference, all deliberate:
//  * 64-bit extents and offsets;
//  * `row_stride` is honoured by the accessor (the reference carried it but
//    documented it as unused);
//  * TileGeom describes a pitched, alignment-padded tile (core + ghost ring)
//    so that the first core column of every row starts on a 16-byte boundary:
//    the HIP stencil kernels issue 16-byte vector loads along x
//    (cdna_hip_programming.md Guideline 13) and need that alignment.
#pragma once

#include <ostream>
#ifdef MXS_DEBUG_BOUNDS
#include <cstdio>
#include <cstdlib>
#endif

#include "mxs/core/config.hpp"

namespace mxs {

// A rectangular window inside a row-major buffer whose rows are `row_stride`
// elements apart. (x_offset, y_offset) is the window origin in buffer
// coordinates.
struct Array2D {
  index_t width = 0;
  index_t height = 0;
  index_t x_offset = 0;
  index_t y_offset = 0;
  index_t row_stride = 0;

  MXS_HD Array2D() = default;
  MXS_HD Array2D(index_t w, index_t h, index_t stride, index_t xoff = 0, index_t yoff = 0)
      : width(w), height(h), x_offset(xoff), y_offset(yoff), row_stride(stride) {}

  MXS_HD index_t size() const { return width * height; }
  // Linear element index of window-relative (x, y).
  MXS_HD index_t index(index_t x, index_t y) const {
    return (y_offset + y) * row_stride + (x_offset + x);
  }
  MXS_HD bool empty() const { return width <= 0 || height <= 0; }
};

inline bool operator==(const Array2D& a, const Array2D& b) {
  return a.width == b.width && a.height == b.height && a.x_offset == b.x_offset &&
         a.y_offset == b.y_offset && a.row_stride == b.row_stride;
}

// Same text as the reference's operator<< (stencil2d/stencil2D.h:44-50): two
// spaces after "width:" are part of the observable format.
inline std::ostream& operator<<(std::ostream& os, const Array2D& a) {
  os << "width:  " << a.width << ", "
     << "height: " << a.height << ", "
     << "x offset: " << a.x_offset << ", "
     << "y offset: " << a.y_offset;
  return os;
}

#ifdef MXS_DEBUG_BOUNDS
[[noreturn]] inline void bounds_fail(index_t x, index_t y) {
  std::fprintf(stderr, "Accessor2D: (%lld, %lld) outside the window\n", static_cast<long long>(x),
               static_cast<long long>(y));
  std::abort();
}
#endif

// Random access into a window of a buffer.
template <typename T>
class Accessor2D {
 public:
  MXS_HD Accessor2D() = default;
  MXS_HD Accessor2D(T* data, const Array2D& layout) : data_(data), layout_(layout) {}
  // -DMXS_DEBUG_BOUNDS: every access is checked against the window (host: assert
  // with the offending coordinates; device: __builtin_trap, a visible fault
  // instead of a silent out-of-window read) — SURVEY §5.2.
  MXS_HD T& operator()(index_t x, index_t y) const {
#ifdef MXS_DEBUG_BOUNDS
    if (x < 0 || y < 0 || x >= layout_.width || y >= layout_.height) {
#if defined(__HIP_DEVICE_COMPILE__)
      __builtin_trap();
#else
      bounds_fail(x, y);
#endif
    }
#endif
    return data_[layout_.index(x, y)];
  }
  MXS_HD const Array2D& layout() const { return layout_; }
  MXS_HD T* data() const { return data_; }

 private:
  T* data_ = nullptr;
  Array2D layout_;
};

// A local tile: `width` x `height` core cells surrounded by a ghost ring of
// `halo_x` columns and `halo_y` rows, stored row-major with `pitch` elements
// per row. Logical tile coordinates (lx, ly) run over
// [0, width + 2*halo_x) x [0, height + 2*halo_y); the core starts at
// (halo_x, halo_y). Logical column lx lives at buffer column `x_origin + lx`,
// logical row ly at buffer row ly.
struct TileGeom {
  index_t width = 0;
  index_t height = 0;
  int halo_x = 0;
  int halo_y = 0;
  index_t pitch = 0;
  index_t x_origin = 0;

  MXS_HD index_t total_width() const { return width + 2 * halo_x; }
  MXS_HD index_t total_height() const { return height + 2 * halo_y; }
  // Elements to allocate for the tile.
  MXS_HD index_t alloc_elems() const { return pitch * total_height(); }
  // Full logical tile (core + ghosts) as an Array2D over the buffer.
  MXS_HD Array2D full() const { return Array2D(total_width(), total_height(), pitch, x_origin, 0); }
  // Core region.
  MXS_HD Array2D core() const { return Array2D(width, height, pitch, x_origin + halo_x, halo_y); }
  MXS_HD index_t core_offset() const { return halo_y * pitch + x_origin + halo_x; }

  // Compact layout identical to the reference's (total width = row stride, no
  // alignment padding): used for byte-compatible dumps and the CPU MPI path.
  static TileGeom compact(index_t w, index_t h, int hx, int hy) {
    TileGeom g;
    g.width = w;
    g.height = h;
    g.halo_x = hx;
    g.halo_y = hy;
    g.pitch = w + 2 * hx;
    g.x_origin = 0;
    return g;
  }

  // GPU layout: the first core column of each row is aligned to `align_bytes`
  // and the pitch is a multiple of `pitch_align_bytes` (a 256-byte pitch keeps
  // every row's wave-wide 1 KiB vector loads on whole cache lines).
  static TileGeom aligned(index_t w, index_t h, int hx, int hy, int elem_bytes,
                          int align_bytes = 16, int pitch_align_bytes = 256) {
    TileGeom g;
    g.width = w;
    g.height = h;
    g.halo_x = hx;
    g.halo_y = hy;
    const index_t a = align_bytes / elem_bytes;                // elements per alignment unit
    const index_t lead = ((hx + a - 1) / a) * a;               // core starts here
    g.x_origin = lead - hx;                                    // first ghost column
    // Room for the last (possibly partial) core vector, the right ghost columns
    // rounded up to whole vectors, plus one more vector: a 16-byte load that starts
    // at any column < width + roundup(halo_x) stays inside the row.
    const index_t min_pitch = lead + ((w + a - 1) / a) * a + ((hx + a - 1) / a) * a + a;
    const index_t pa = pitch_align_bytes / elem_bytes;
    g.pitch = ((min_pitch + pa - 1) / pa) * pa;
    return g;
  }
};

inline bool operator==(const TileGeom& a, const TileGeom& b) {
  return a.width == b.width && a.height == b.height && a.halo_x == b.halo_x &&
         a.halo_y == b.halo_y && a.pitch == b.pitch && a.x_origin == b.x_origin;
}

}  // namespace mxs
