#include "mxs/core/device.hpp"

#include <hip/hip_runtime_api.h>

#include <cstdlib>

#include "mxs/comm/mpi_env.hpp"
#include "mxs/core/error.hpp"

namespace mxs {

int local_rank_from_env() {
  for (const char* v : {"LOCAL_RANK", "OMPI_COMM_WORLD_LOCAL_RANK", "MV2_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID",
                        "SLURM_LOCALID"}) {
    if (const char* s = std::getenv(v)) return std::atoi(s);
  }
  return 0;
}

DeviceBinding bind_device(const MpiEnv& env, const std::string& mode) {
  DeviceBinding b;
  b.mode = mode;
  b.local_rank = env.local_rank();
  MXS_HIP_CHECK(hipGetDeviceCount(&b.devices_visible));
  MXS_CHECK(b.devices_visible > 0, "no HIP devices found");
  b.devices_used = b.devices_visible;
  if (const char* cap = std::getenv("NUM_GPU_DEVICES")) {
    const int c = std::atoi(cap);
    if (c > 0 && c < b.devices_used) b.devices_used = c;
  }
  if (mode == "rrobin")
    b.device = (env.rank() / (env.node_count() > 0 ? env.node_count() : 1)) % b.devices_used;
  else
    b.device = b.local_rank % b.devices_used;
  MXS_HIP_CHECK(hipSetDevice(b.device));
  hipUUID u{};
  MXS_HIP_CHECK(hipDeviceGetUuid(&u, b.device));
  const std::string mine(u.bytes, sizeof(u.bytes));
  int same = 0;
  for (const auto& other : mpi_allgather_bytes(MPI_COMM_WORLD, mine)) same += other == mine ? 1 : 0;
  b.sharing = same;
  b.shared = same > 1;
  return b;
}

}  // namespace mxs
