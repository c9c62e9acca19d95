// MPI tutorial 6: neighbour exchange + MPI_Gather of 3 ints per rank to rank 0
// (reference: mpi6.cpp). A missing neighbour shows the rank's own id. Output on
// rank 0: "(prev<rank>next) " for every rank.
#include <mpi.h>

#include <iostream>
#include <vector>

#include "mxs/comm/mpi_env.hpp"

int main(int argc, char** argv) {
  mxs::MpiEnv env(&argc, &argv);
  const int me = env.rank(), n = env.size();
  const int right_tag = 0x01, left_tag = 0x10;
  std::vector<int> nb(3, me);  // {self, prev, next}
  std::vector<MPI_Request> req;
  auto post = [&](bool send, int* buf, int peer, int tag) {
    MPI_Request r;
    if (send) MXS_MPI_CHECK(MPI_Isend(buf, 1, MPI_INT, peer, tag, MPI_COMM_WORLD, &r));
    else MXS_MPI_CHECK(MPI_Irecv(buf, 1, MPI_INT, peer, tag, MPI_COMM_WORLD, &r));
    req.push_back(r);
  };
  int mine = me;
  if (me > 0) post(true, &mine, me - 1, left_tag);
  if (me + 1 < n) post(true, &mine, me + 1, right_tag);
  if (me > 0) post(false, &nb[1], me - 1, right_tag);
  if (me + 1 < n) post(false, &nb[2], me + 1, left_tag);
  MXS_MPI_CHECK(MPI_Waitall(int(req.size()), req.data(), MPI_STATUSES_IGNORE));
  std::vector<int> all(me == 0 ? size_t(3 * n) : 0, -2);
  MXS_MPI_CHECK(MPI_Gather(nb.data(), 3, MPI_INT, me == 0 ? all.data() : nullptr, 3, MPI_INT, 0, MPI_COMM_WORLD));
  if (me == 0) {
    for (int r = 0; r < n; ++r) std::cout << '(' << all[3 * r + 1] << '<' << all[3 * r] << '>' << all[3 * r + 2] << ") ";
    std::cout << std::endl;
  }
  return 0;
}
