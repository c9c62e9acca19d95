// Collective checkpoint / resume of a block-decomposed 2-D field.
//
// The reference persists nothing but its per-rank text dumps
// (stencil2d/mpi-2d-stencil-subarray-cuda.cu:114-118,161-176) and mentions
// MPI_File_* input "in the real world" (mpicuda2.cu:156-157). Here every rank
// writes its core block straight into ONE global row-major file with
// MPI_File_write_at_all through two subarray views — the memory view selects
// the core out of the padded tile (ghost ring and row padding skipped), the
// file view places the block at (gy0, gx0) of the global grid — so the file is
// independent of the decomposition: a run on a 2x4 grid resumes on 1x1 or 3x3.
//
// File layout: a 64-byte little-endian header, then gh rows of gw elements.
//   0  char[8]  magic "MXSGRID1"
//   8  u32      element bytes (4 or 8)
//  12  u32      reserved (0)
//  16  i64      global width
//  24  i64      global height
//  32  i64      iterations completed
//  40  u64      seed of the initial field
//  48  u8[16]   reserved
// The Python side (cuda_mpi_scratch_amd/utils/checkpoint.py) reads and writes
// the same format.
#pragma once

#include <mpi.h>

#include <cstdint>
#include <cstring>
#include <string>

#include "mxs/comm/mpi_env.hpp"
#include "mxs/comm/mpi_types.hpp"
#include "mxs/grid/layout.hpp"

namespace mxs {

struct GridFileHeader {
  char magic[8] = {'M', 'X', 'S', 'G', 'R', 'I', 'D', '1'};
  std::uint32_t elem_bytes = 0;
  std::uint32_t reserved0 = 0;
  std::int64_t width = 0;
  std::int64_t height = 0;
  std::int64_t iteration = 0;
  std::uint64_t seed = 0;
  std::uint8_t reserved1[16] = {};

  bool valid() const { return std::memcmp(magic, "MXSGRID1", 8) == 0; }
};
static_assert(sizeof(GridFileHeader) == 64, "grid file header must be 64 bytes");

// Where this rank's core block sits in the global grid.
struct GlobalBlock {
  index_t gx0 = 0, gy0 = 0;  // first global column / row of the core
  index_t gw = 0, gh = 0;    // global grid
};

namespace detail {

class MpiFile {
 public:
  MpiFile(MPI_Comm comm, const std::string& path, int amode) {
    const int rc = MPI_File_open(comm, path.c_str(), amode, MPI_INFO_NULL, &fh_);
    if (rc != MPI_SUCCESS) raise_error("cannot open '" + path + "': " + format_mpi_error(rc), rc);
  }
  ~MpiFile() {
    if (fh_ != MPI_FILE_NULL) MPI_File_close(&fh_);
  }
  MpiFile(const MpiFile&) = delete;
  MpiFile& operator=(const MpiFile&) = delete;
  MPI_File get() const { return fh_; }

 private:
  MPI_File fh_ = MPI_FILE_NULL;
};

template <typename T>
void set_block_view(MPI_File fh, const TileGeom& g, const GlobalBlock& b, MpiType& filetype) {
  filetype = make_subarray_type<T>(b.gh, Array2D(g.width, g.height, b.gw, b.gx0, b.gy0));
  char native[] = "native";
  MXS_MPI_CHECK(MPI_File_set_view(fh, MPI_Offset(sizeof(GridFileHeader)), mpi_element_type<T>(), filetype.get(),
                                  native, MPI_INFO_NULL));
}

}  // namespace detail

// Collective over `comm`. `tile` is a HOST buffer laid out by `g`.
template <typename T>
void write_grid_file(MPI_Comm comm, const std::string& path, const T* tile, const TileGeom& g, const GlobalBlock& b,
                     std::int64_t iteration, std::uint64_t seed) {
  int rank = 0;
  MXS_MPI_CHECK(MPI_Comm_rank(comm, &rank));
  detail::MpiFile f(comm, path, MPI_MODE_CREATE | MPI_MODE_WRONLY);
  MXS_MPI_CHECK(MPI_File_set_size(f.get(), MPI_Offset(sizeof(GridFileHeader)) +
                                               MPI_Offset(b.gw) * MPI_Offset(b.gh) * MPI_Offset(sizeof(T))));
  if (rank == 0) {
    GridFileHeader h;
    h.elem_bytes = sizeof(T);
    h.width = b.gw;
    h.height = b.gh;
    h.iteration = iteration;
    h.seed = seed;
    MXS_MPI_CHECK(MPI_File_write_at(f.get(), 0, &h, int(sizeof(h)), MPI_BYTE, MPI_STATUS_IGNORE));
  }
  MpiType filetype;
  detail::set_block_view<T>(f.get(), g, b, filetype);
  MpiType memtype = make_subarray_type<T>(g.total_height(), g.core());
  MXS_MPI_CHECK(MPI_File_write_at_all(f.get(), 0, tile, 1, memtype.get(), MPI_STATUS_IGNORE));
}

// Every rank reads and validates the header (collective).
inline GridFileHeader read_grid_header(MPI_Comm comm, const std::string& path) {
  detail::MpiFile f(comm, path, MPI_MODE_RDONLY);
  GridFileHeader h;
  MXS_MPI_CHECK(MPI_File_read_at_all(f.get(), 0, &h, int(sizeof(h)), MPI_BYTE, MPI_STATUS_IGNORE));
  MXS_CHECK(h.valid(), "'" << path << "' is not an mxs grid file");
  return h;
}

// Collective. Fills the core of `tile` (ghost ring untouched) and returns the
// header; the file's grid size and element type must match.
template <typename T>
GridFileHeader read_grid_file(MPI_Comm comm, const std::string& path, T* tile, const TileGeom& g,
                              const GlobalBlock& b) {
  const GridFileHeader h = read_grid_header(comm, path);
  MXS_CHECK(h.elem_bytes == sizeof(T), "'" << path << "' holds " << h.elem_bytes << "-byte elements, expected "
                                           << sizeof(T));
  MXS_CHECK(h.width == b.gw && h.height == b.gh,
            "'" << path << "' holds a " << h.width << "x" << h.height << " grid, expected " << b.gw << "x" << b.gh);
  detail::MpiFile f(comm, path, MPI_MODE_RDONLY);
  MpiType filetype;
  detail::set_block_view<T>(f.get(), g, b, filetype);
  MpiType memtype = make_subarray_type<T>(g.total_height(), g.core());
  MXS_MPI_CHECK(MPI_File_read_at_all(f.get(), 0, tile, 1, memtype.get(), MPI_STATUS_IGNORE));
  return h;
}

}  // namespace mxs
