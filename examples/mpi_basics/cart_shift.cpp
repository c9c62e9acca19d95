// MPI tutorial 10: non-periodic DIM x DIM Cartesian grid, MPI_Cart_shift in both
// dimensions and an exchange of rank ids with the 4 neighbours (MPI_PROC_NULL at
// the edges, printed as -1 by MPICH) (reference: mpi10.cpp). Non-square sizes use
// the MPI_Dims_create factorisation.
#include <mpi.h>

#include <cmath>
#include <iostream>
#include <sstream>
#include <vector>

#include "mxs/comm/mpi_env.hpp"

int main(int argc, char** argv) {
  mxs::MpiEnv env(&argc, &argv);
  int dims[2] = {0, 0}, periods[2] = {0, 0};
  MXS_MPI_CHECK(MPI_Dims_create(env.size(), 2, dims));
  MPI_Comm cart;
  MXS_MPI_CHECK(MPI_Cart_create(MPI_COMM_WORLD, 2, dims, periods, 0, &cart));
  int me = -1, coords[2] = {-1, -1};
  MXS_MPI_CHECK(MPI_Comm_rank(cart, &me));
  MXS_MPI_CHECK(MPI_Cart_coords(cart, me, 2, coords));
  enum { UP = 0, DOWN, LEFT, RIGHT };
  int nb[4];
  MXS_MPI_CHECK(MPI_Cart_shift(cart, 0, 1, &nb[UP], &nb[DOWN]));
  MXS_MPI_CHECK(MPI_Cart_shift(cart, 1, 1, &nb[LEFT], &nb[RIGHT]));
  int recv[4] = {MPI_PROC_NULL, MPI_PROC_NULL, MPI_PROC_NULL, MPI_PROC_NULL};
  MPI_Request req[8];
  for (int i = 0; i < 4; ++i) {
    MXS_MPI_CHECK(MPI_Isend(&me, 1, MPI_INT, nb[i], 1, cart, &req[i]));
    MXS_MPI_CHECK(MPI_Irecv(&recv[i], 1, MPI_INT, nb[i], 1, cart, &req[4 + i]));
  }
  MXS_MPI_CHECK(MPI_Waitall(8, req, MPI_STATUSES_IGNORE));
  std::ostringstream os;
  os << "rank= " << me << " coords= " << coords[0] << ',' << coords[1] << " neighbors= " << nb[UP] << ','
     << nb[DOWN] << ',' << nb[LEFT] << ',' << nb[RIGHT] << '\n';
  std::cout << os.str() << std::flush;
  MXS_MPI_CHECK(MPI_Comm_free(&cart));
  return 0;
}
