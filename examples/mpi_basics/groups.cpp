// MPI tutorial 9: groups and communicators — split the world into two halves with
// MPI_Group_incl + MPI_Comm_create and MPI_Allreduce within each half and over the
// world (reference: mpi9.cpp). Odd sizes put the extra rank in the second half.
#include <mpi.h>

#include <iostream>
#include <numeric>
#include <sstream>
#include <vector>

#include "mxs/comm/mpi_env.hpp"

int main(int argc, char** argv) {
  mxs::MpiEnv env(&argc, &argv);
  const int me = env.rank(), n = env.size(), half = n / 2;
  MPI_Group world_group, my_group;
  MXS_MPI_CHECK(MPI_Comm_group(MPI_COMM_WORLD, &world_group));
  const bool first = me < half;
  std::vector<int> members(size_t(first ? half : n - half));
  std::iota(members.begin(), members.end(), first ? 0 : half);
  MXS_MPI_CHECK(MPI_Group_incl(world_group, int(members.size()), members.data(), &my_group));
  MPI_Comm comm;
  MXS_MPI_CHECK(MPI_Comm_create(MPI_COMM_WORLD, my_group, &comm));
  int new_rank = -1;
  MXS_MPI_CHECK(MPI_Group_rank(my_group, &new_rank));
  int group_sum = -1, total = -1;
  MXS_MPI_CHECK(MPI_Allreduce(&me, &group_sum, 1, MPI_INT, MPI_SUM, comm));
  MXS_MPI_CHECK(MPI_Allreduce(&me, &total, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD));
  std::ostringstream os;
  os << env.processor_name() << " - group: " << (first ? 0 : 1) << " - rank: " << me << "\tnew rank: " << new_rank
     << "\treceived: " << group_sum << '\n';
  std::cout << os.str() << std::flush;
  if (me == 0) {
    std::ostringstream t;
    t << "\nAllreduce total: " << total << '\n';
    std::cout << t.str() << std::flush;
  }
  MXS_MPI_CHECK(MPI_Comm_free(&comm));
  MXS_MPI_CHECK(MPI_Group_free(&my_group));
  MXS_MPI_CHECK(MPI_Group_free(&world_group));
  return 0;
}
