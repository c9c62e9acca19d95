// Device-buffer variant of MPI tutorial 5 (reference mpi5.cpp): each
// rank's id lives in HBM and is exchanged with its left/right neighbour on a
// non-periodic chain by RCCL point-to-point (one ncclGroup of up to two sends and
// two receives) — the message never touches the host. MPI only bootstraps the
// communicator and prints. Output matches mpi_neighbors1d: "i/N-1:\t(prev, i, next)\t- host",
// missing neighbours print -1.
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
  const int me = env.rank(), n = env.size();
  std::string uid = me == 0 ? RcclComm::make_unique_id() : std::string(sizeof(ncclUniqueId), '\0');
  MXS_MPI_CHECK(MPI_Bcast(&uid[0], int(uid.size()), MPI_BYTE, 0, MPI_COMM_WORLD));
  RcclComm comm(uid, n, me);

  // d[0] = my id, d[1] = from prev, d[2] = from next (initialised to -1).
  DeviceBuffer<int> d(3);
  const int init[3] = {me, -1, -1};
  MXS_HIP_CHECK(hipMemcpy(d.get(), init, sizeof(init), hipMemcpyHostToDevice));
  Stream s;
  comm.group_start();
  if (me > 0) {
    comm.send<int>(d.get(), 1, me - 1, s.get());
    comm.recv<int>(d.get() + 1, 1, me - 1, s.get());
  }
  if (me + 1 < n) {
    comm.send<int>(d.get(), 1, me + 1, s.get());
    comm.recv<int>(d.get() + 2, 1, me + 1, s.get());
  }
  comm.group_end();
  comm.wait(s.get(), "neighbour exchange");
  int out[3];
  MXS_HIP_CHECK(hipMemcpy(out, d.get(), sizeof(out), hipMemcpyDeviceToHost));
  std::ostringstream os;
  os << me << '/' << n - 1 << ":\t(" << out[1] << ", " << out[0] << ", " << out[2] << ")\t- " << env.processor_name()
     << " (HIP device " << dev.device << ")\n";
  std::cout << os.str() << std::flush;
  return 0;
}
