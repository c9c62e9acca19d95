// Rank -> GPU binding (reference: BindDevice, stencil2d/mpi-2d-stencil-subarray-cuda.cu:40-73;
// `rank % count` / `(rank / node_count) % count` in mpicuda4.cu:278-302).
//
// The node-local rank comes from MPI_Comm_split_type (MpiEnv) — the reference
// read OMPI_/MV2_ environment variables and used an uninitialised value when
// neither was set. NUM_GPU_DEVICES caps the device count, as in the
// reference; HIP_VISIBLE_DEVICES is honoured by the HIP runtime itself.
#pragma once

#include <string>

namespace mxs {

class MpiEnv;

struct DeviceBinding {
  int device = -1;
  int local_rank = 0;
  int devices_visible = 0;
  int devices_used = 0;
  std::string mode;  // "bunch" | "rrobin"
  // Some other rank of the job runs on this rank's GPU (device UUIDs compared
  // over all ranks, not counts: a launcher that gives each rank one visible
  // device makes every rank see "1 device" on distinct GPUs).
  bool shared = false;
  int sharing = 1;  // ranks on this GPU, this one included
};

// Selects and sets (hipSetDevice) this rank's GPU. mode "bunch": local_rank % n;
// "rrobin": (world_rank / node_count) % n (ranks dealt round-robin over nodes).
DeviceBinding bind_device(const MpiEnv& env, const std::string& mode = "bunch");

// Environment-only fallback used before MPI_Init (launchers that need the device
// selected before MPI starts): LOCAL_RANK, OMPI_COMM_WORLD_LOCAL_RANK,
// MV2_COMM_WORLD_LOCAL_RANK, MPI_LOCALRANKID, SLURM_LOCALID; default 0.
int local_rank_from_env();

}  // namespace mxs
