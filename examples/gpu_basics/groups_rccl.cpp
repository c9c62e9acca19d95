// Device variant of MPI tutorial 9 (reference mpi9.cpp): the world is
// split into two halves — on the host with MPI_Comm_split and on the device with
// ncclCommSplit (same colour / key) — and every rank's id, held in HBM, is summed
// with ncclAllReduce per half and over the world. Prints the host and device sums
// side by side; they must agree.
#include <mpi.h>

#include <iostream>
#include <sstream>
#include <string>

#include "mxs/comm/mpi_env.hpp"
#include "mxs/comm/rccl_comm.hpp"
#include "mxs/core/device.hpp"
#include "mxs/runtime/hip_utils.hpp"

int main(int argc, char** argv) {
  using namespace mxs;
  MpiEnv env(&argc, &argv);
  const DeviceBinding dev = bind_device(env, "bunch");
  (void)dev;
  const int me = env.rank(), n = env.size(), half = n / 2;
  const int color = me < half ? 0 : 1;

  MPI_Comm host_half;
  MXS_MPI_CHECK(MPI_Comm_split(MPI_COMM_WORLD, color, me, &host_half));
  int host_group_sum = 0, host_total = 0;
  MXS_MPI_CHECK(MPI_Allreduce(&me, &host_group_sum, 1, MPI_INT, MPI_SUM, host_half));
  MXS_MPI_CHECK(MPI_Allreduce(&me, &host_total, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD));

  std::string uid = me == 0 ? RcclComm::make_unique_id() : std::string(sizeof(ncclUniqueId), '\0');
  MXS_MPI_CHECK(MPI_Bcast(&uid[0], int(uid.size()), MPI_BYTE, 0, MPI_COMM_WORLD));
  RcclComm world(uid, n, me);
  ncclComm_t half_comm = nullptr;
  MXS_RCCL_CHECK(ncclCommSplit(world.get(), color, me, &half_comm, nullptr));
  int half_rank = -1;
  MXS_RCCL_CHECK(ncclCommUserRank(half_comm, &half_rank));

  DeviceBuffer<int> d(3);  // [my id, half sum, world sum]
  MXS_HIP_CHECK(hipMemcpy(d.get(), &me, sizeof(int), hipMemcpyHostToDevice));
  Stream s;
  MXS_RCCL_CHECK(ncclAllReduce(d.get(), d.get() + 1, 1, ncclInt32, ncclSum, half_comm, s.get()));
  world.allreduce_sum<int>(d.get(), d.get() + 2, 1, s.get());
  world.wait(s.get(), "group all-reduce");
  int out[3];
  MXS_HIP_CHECK(hipMemcpy(out, d.get(), sizeof(out), hipMemcpyDeviceToHost));
  std::ostringstream os;
  os << env.processor_name() << " - group: " << color << " - rank: " << me << "\tnew rank: " << half_rank
     << "\treceived: " << out[1] << "\t(host " << host_group_sum << ")\n";
  std::cout << os.str() << std::flush;
  if (me == 0) {
    std::ostringstream t;
    t << "\nAllreduce total: " << out[2] << " (host " << host_total << ")\n";
    std::cout << t.str() << std::flush;
  }
  MXS_CHECK(out[1] == host_group_sum && out[2] == host_total, "device and host reductions disagree");
  (void)ncclCommDestroy(half_comm);
  MXS_MPI_CHECK(MPI_Comm_free(&host_half));
  return 0;
}
