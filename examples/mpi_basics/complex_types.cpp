// MPI tutorial 11: composed derived datatypes — a 1D subarray (3 of 8 ints)
// replicated over three separately allocated arrays with MPI_Type_create_hindexed
// and absolute byte displacements (reference: mpi-complex-types.cpp).
// Rank 0 sends elements [3,6) of B1, B2, B3; rank 1 receives them into [0,3).
#include <mpi.h>

#include <cstdio>
#include <memory>

#include "mxs/comm/mpi_env.hpp"
#include "mxs/comm/mpi_types.hpp"

namespace {
mxs::MpiType composed(int start, int* b1, int* b2, int* b3) {
  int sz = 8, ssz = 3;
  MPI_Datatype block;
  MXS_MPI_CHECK(MPI_Type_create_subarray(1, &sz, &ssz, &start, MPI_ORDER_C, MPI_INT, &block));
  MXS_MPI_CHECK(MPI_Type_commit(&block));
  mxs::MpiType blk(block);
  int lens[3] = {1, 1, 1};
  MPI_Aint disp[3] = {0, reinterpret_cast<char*>(b2) - reinterpret_cast<char*>(b1),
                      reinterpret_cast<char*>(b3) - reinterpret_cast<char*>(b1)};
  MPI_Datatype t;
  MXS_MPI_CHECK(MPI_Type_create_hindexed(3, lens, disp, blk.get(), &t));
  MXS_MPI_CHECK(MPI_Type_commit(&t));
  return mxs::MpiType(t);
}
}  // namespace

int main(int argc, char** argv) {
  mxs::MpiEnv env(&argc, &argv);
  if (env.size() < 2) {
    std::printf("Please run with 2 processes.\n");
    return 1;
  }
  auto b1 = std::make_unique<int[]>(1500), b2 = std::make_unique<int[]>(8), b3 = std::make_unique<int[]>(28);
  if (env.rank() == 0) {
    for (int i = 0; i < 8; ++i) {
      b1[i] = i;
      b2[i] = 2 * i;
      b3[i] = 2 * i + 1;
    }
    mxs::MpiType t = composed(3, b1.get(), b2.get(), b3.get());
    MXS_MPI_CHECK(MPI_Send(b1.get(), 1, t.get(), 1, 123, MPI_COMM_WORLD));
  } else if (env.rank() == 1) {
    for (int i = 0; i < 8; ++i) b1[i] = b2[i] = b3[i] = -1;
    mxs::MpiType t = composed(0, b1.get(), b2.get(), b3.get());
    MXS_MPI_CHECK(MPI_Recv(b1.get(), 1, t.get(), 0, 123, MPI_COMM_WORLD, MPI_STATUS_IGNORE));
    for (int i = 0; i < 8; ++i) std::printf("B1[%d] = %d\n", i, b1[i]);
    for (int i = 0; i < 8; ++i) std::printf("B2[%d] = %d\n", i, b2[i]);
    for (int i = 0; i < 8; ++i) std::printf("B3[%d] = %d\n", i, b3[i]);
    std::fflush(stdout);
  }
  return 0;
}
