// MPI tutorial 5: non-blocking exchange with the left/right neighbour on a
// non-periodic 1D chain (reference: mpi5.cpp). Missing neighbours print -1.
#include <mpi.h>

#include <iostream>
#include <sstream>
#include <vector>

#include "mxs/comm/mpi_env.hpp"

int main(int argc, char** argv) {
  mxs::MpiEnv env(&argc, &argv);
  const int me = env.rank(), n = env.size();
  const int prev = me - 1, next = me + 1;
  const int right_tag = 0x01, left_tag = 0x10;
  int from_prev = -1, from_next = -1;
  std::vector<MPI_Request> req;
  auto post = [&](bool send, int* buf, int peer, int tag) {
    MPI_Request r;
    if (send) MXS_MPI_CHECK(MPI_Isend(buf, 1, MPI_INT, peer, tag, MPI_COMM_WORLD, &r));
    else MXS_MPI_CHECK(MPI_Irecv(buf, 1, MPI_INT, peer, tag, MPI_COMM_WORLD, &r));
    req.push_back(r);
  };
  int mine = me;
  if (prev >= 0) post(true, &mine, prev, left_tag);
  if (next < n) post(true, &mine, next, right_tag);
  if (prev >= 0) post(false, &from_prev, prev, right_tag);
  if (next < n) post(false, &from_next, next, left_tag);
  MXS_MPI_CHECK(MPI_Waitall(int(req.size()), req.data(), MPI_STATUSES_IGNORE));
  std::ostringstream os;
  os << me << '/' << n - 1 << ":\t(" << from_prev << ", " << me << ", " << from_next << ")\t- "
     << env.processor_name() << '\n';
  std::cout << os.str() << std::flush;
  return 0;
}
