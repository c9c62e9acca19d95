// MPI tutorial 8: MPI_Type_create_struct for a Particle {4 float, 2 int}; rank 0
// sends particle i to rank i (reference: mpi8.cpp; MPI_Type_extent, removed in
// MPI-3, is replaced by MPI_Type_get_extent and the offsets by offsetof).
#include <mpi.h>

#include <cstddef>
#include <iostream>
#include <sstream>
#include <vector>

#include "mxs/comm/mpi_env.hpp"
#include "mxs/comm/mpi_types.hpp"

struct Particle {
  float x, y, z;
  float velocity;
  int id, type;
};

int main(int argc, char** argv) {
  mxs::MpiEnv env(&argc, &argv);
  MPI_Aint lb = 0, extent = 0;
  MXS_MPI_CHECK(MPI_Type_get_extent(MPI_FLOAT, &lb, &extent));
  if (env.rank() == 0) std::cout << "\nMPI_FLOAT extent: " << extent << std::endl;
  int counts[2] = {4, 2};
  MPI_Aint offsets[2] = {offsetof(Particle, x), offsetof(Particle, id)};
  MPI_Datatype types[2] = {MPI_FLOAT, MPI_INT}, raw;
  MXS_MPI_CHECK(MPI_Type_create_struct(2, counts, offsets, types, &raw));
  MXS_MPI_CHECK(MPI_Type_commit(&raw));
  mxs::MpiType ptype(raw);
  std::vector<Particle> ps(size_t(env.size()));
  std::vector<MPI_Request> sends;
  const int tag = 1;
  if (env.rank() == 0) {
    sends.resize(ps.size());
    for (int i = 0; i < env.size(); ++i) {
      ps[size_t(i)] = Particle{float(i), float(-i), float(i), 0.5f, i, i % 2};
      MXS_MPI_CHECK(MPI_Isend(&ps[size_t(i)], 1, ptype.get(), i, tag, MPI_COMM_WORLD, &sends[size_t(i)]));
    }
  }
  Particle p{};
  MXS_MPI_CHECK(MPI_Recv(&p, 1, ptype.get(), 0, tag, MPI_COMM_WORLD, MPI_STATUS_IGNORE));
  if (!sends.empty()) MXS_MPI_CHECK(MPI_Waitall(int(sends.size()), sends.data(), MPI_STATUSES_IGNORE));
  std::ostringstream os;
  os << env.processor_name() << " - rank " << env.rank() << ":\t" << "particle id: " << p.id << '\n';
  std::cout << os.str() << std::flush;
  return 0;
}
