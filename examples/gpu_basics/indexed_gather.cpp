// Device counterpart of MPI tutorial 7 (reference mpi7.cpp): the
// MPI_Type_indexed({4, 2}, {5, 12}) view over 16 floats, i.e. elements 5..8 and
// 12..13, gathered into a contiguous buffer by a HIP kernel instead of by MPI's
// datatype engine — the same thing the halo pack kernel (copy2d_batch) does for
// subarrays. Every rank receives the 6 floats from rank 0 (MPI on the packed
// device buffer staged through the host: MPICH here is not GPU-aware) and prints
// "5,6,7,8,12,13," like mpi_indexed.
#include <mpi.h>

#include <iostream>
#include <sstream>
#include <vector>

#include <hip/hip_runtime.h>

#include "mxs/comm/mpi_env.hpp"
#include "mxs/core/device.hpp"
#include "mxs/runtime/hip_utils.hpp"

namespace {

// One thread per output element: find its block by a prefix scan of the lengths
// (a handful of blocks: a linear scan is fine).
__global__ void indexed_gather(const float* __restrict__ src, float* __restrict__ dst, const int* __restrict__ lens,
                               const int* __restrict__ displs, int nblocks, int total) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  int b = 0, start = 0;
  while (b < nblocks && i >= start + lens[b]) start += lens[b++];
  dst[i] = src[displs[b] + (i - start)];
}

}  // namespace

int main(int argc, char** argv) {
  using namespace mxs;
  MpiEnv env(&argc, &argv);
  const DeviceBinding dev = bind_device(env, "bunch");
  (void)dev;
  const std::vector<int> lens = {4, 2}, displs = {5, 12};
  const int total = 6;
  std::vector<float> packed(total, -1.f);
  if (env.rank() == 0) {
    std::vector<float> h(16);
    for (int i = 0; i < 16; ++i) h[size_t(i)] = float(i);
    DeviceBuffer<float> src(16), dst(total);
    DeviceBuffer<int> dl(2), dd(2);
    MXS_HIP_CHECK(hipMemcpy(src.get(), h.data(), 16 * sizeof(float), hipMemcpyHostToDevice));
    MXS_HIP_CHECK(hipMemcpy(dl.get(), lens.data(), 2 * sizeof(int), hipMemcpyHostToDevice));
    MXS_HIP_CHECK(hipMemcpy(dd.get(), displs.data(), 2 * sizeof(int), hipMemcpyHostToDevice));
    indexed_gather<<<1, 64>>>(src.get(), dst.get(), dl.get(), dd.get(), 2, total);
    MXS_HIP_CHECK_LAUNCH();
    MXS_HIP_CHECK(hipMemcpy(packed.data(), dst.get(), total * sizeof(float), hipMemcpyDeviceToHost));
  }
  MXS_MPI_CHECK(MPI_Bcast(packed.data(), total, MPI_FLOAT, 0, MPI_COMM_WORLD));
  std::ostringstream os;
  os << "rank " << env.rank() << ": ";
  for (float v : packed) os << v << ',';
  os << '\n';
  std::cout << os.str() << std::flush;
  return 0;
}
