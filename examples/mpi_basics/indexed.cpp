// MPI tutorial 7: MPI_Type_indexed — blocks {4 at 5, 2 at 12} of a 16-float array
// sent by rank 0 to every rank (itself included); everyone prints 5,6,7,8,12,13,
// (reference: mpi7.cpp, whose send requests were never completed).
#include <mpi.h>

#include <iostream>
#include <iterator>
#include <sstream>
#include <vector>

#include "mxs/comm/mpi_env.hpp"
#include "mxs/comm/mpi_types.hpp"

int main(int argc, char** argv) {
  mxs::MpiEnv env(&argc, &argv);
  float a[16];
  for (int i = 0; i < 16; ++i) a[i] = float(i);
  int lens[2] = {4, 2}, disps[2] = {5, 12};
  MPI_Datatype raw;
  MXS_MPI_CHECK(MPI_Type_indexed(2, lens, disps, MPI_FLOAT, &raw));
  MXS_MPI_CHECK(MPI_Type_commit(&raw));
  mxs::MpiType indexed(raw);
  const int tag = 1;
  std::vector<MPI_Request> sends;
  if (env.rank() == 0) {
    sends.resize(size_t(env.size()));
    for (int r = 0; r < env.size(); ++r)
      MXS_MPI_CHECK(MPI_Isend(a, 1, indexed.get(), r, tag, MPI_COMM_WORLD, &sends[size_t(r)]));
  }
  std::vector<float> b(6);
  MXS_MPI_CHECK(MPI_Recv(b.data(), 6, MPI_FLOAT, 0, tag, MPI_COMM_WORLD, MPI_STATUS_IGNORE));
  if (!sends.empty()) MXS_MPI_CHECK(MPI_Waitall(int(sends.size()), sends.data(), MPI_STATUSES_IGNORE));
  std::ostringstream os;
  os << env.processor_name() << " - rank " << env.rank() << ":\t";
  std::copy(b.begin(), b.end(), std::ostream_iterator<float>(os, ","));
  os << '\n';
  std::cout << os.str() << std::flush;
  return 0;
}
