// MPI datatype factory (reference: CreateArrayElementType<T> customisation point
// and CreateMPISubArrayType, stencil2d/stencil2D.h:203-228).
//
// Fixes vs the reference: the subarray is built with sizes {rows, cols} in
// MPI_ORDER_C, i.e. dimension 0 is y (the reference passed {width, height} and
// so transposed every region; only square tiles survived); types are
// owned by an RAII handle and freed (the reference leaked 16 per rank, Q5).
#pragma once

#include <mpi.h>

#include <cstdint>
#include <utility>

#include "mxs/comm/mpi_env.hpp"
#include "mxs/grid/layout.hpp"

namespace mxs {

// Customisation point: specialise for user element types.
template <typename T>
MPI_Datatype mpi_element_type();
template <>
inline MPI_Datatype mpi_element_type<double>() { return MPI_DOUBLE; }
template <>
inline MPI_Datatype mpi_element_type<float>() { return MPI_FLOAT; }
template <>
inline MPI_Datatype mpi_element_type<int>() { return MPI_INT; }
template <>
inline MPI_Datatype mpi_element_type<unsigned char>() { return MPI_UNSIGNED_CHAR; }
template <>
inline MPI_Datatype mpi_element_type<char>() { return MPI_CHAR; }

class MpiType {
 public:
  MpiType() = default;
  explicit MpiType(MPI_Datatype t) : t_(t) {}
  ~MpiType() { reset(); }
  MpiType(const MpiType&) = delete;
  MpiType& operator=(const MpiType&) = delete;
  MpiType(MpiType&& o) noexcept : t_(std::exchange(o.t_, MPI_DATATYPE_NULL)) {}
  MpiType& operator=(MpiType&& o) noexcept {
    if (this != &o) {
      reset();
      t_ = std::exchange(o.t_, MPI_DATATYPE_NULL);
    }
    return *this;
  }
  void reset() {
    int fin = 0;
    MPI_Finalized(&fin);
    if (t_ != MPI_DATATYPE_NULL && !fin) MPI_Type_free(&t_);
    t_ = MPI_DATATYPE_NULL;
  }
  MPI_Datatype get() const { return t_; }

 private:
  MPI_Datatype t_ = MPI_DATATYPE_NULL;
};

// Subarray `sub` of a buffer whose rows are `buf.row_stride` elements wide and
// `buf_rows` rows tall; messages are sent with count 1 from the buffer base.
template <typename T>
MpiType make_subarray_type(index_t buf_rows, const Array2D& sub) {
  int sizes[2] = {int(buf_rows), int(sub.row_stride)};
  int subsizes[2] = {int(sub.height), int(sub.width)};
  int starts[2] = {int(sub.y_offset), int(sub.x_offset)};
  MPI_Datatype t;
  MXS_MPI_CHECK(MPI_Type_create_subarray(2, sizes, subsizes, starts, MPI_ORDER_C, mpi_element_type<T>(), &t));
  MXS_MPI_CHECK(MPI_Type_commit(&t));
  return MpiType(t);
}

}  // namespace mxs
