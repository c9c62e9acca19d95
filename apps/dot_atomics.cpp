// dot_atomics — single-GPU dot product with one device atomic per workgroup.
// Reference: ref_parallel-dot-product-atomics.cu (1024 floats, 64 blocks x 16 threads,
// LDS tree + atomicAdd; -DNO_SYNC replaces the atomic with a racy `*out +=`).
//
//   dot_atomics [--n N] [--no-sync] [--blocks B]
// Output (reference format): the HIP error string, "GPU: <value>", "CPU: <value>".
#include <hip/hip_runtime.h>

#include <iostream>
#include <vector>

#include "mxs/core/cli.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/hip_utils.hpp"

using namespace mxs;

int main(int argc, char** argv) {
  Cli cli(argc, argv, {"no-sync"});
  const index_t n = index_t(cli.get_int("n", 1024));
  const bool racy = cli.flag("no-sync");
  // The reference used 64 blocks of 16 threads (a quarter of one wave64 each);
  // here 256-thread workgroups, and enough of them for the racy demo to race.
  const int blocks = int(cli.get_int("blocks", 64));
  DeviceBuffer<float> x(n), y(n);
  DeviceBuffer<float> out(1), partials(blocks);
  DeviceBuffer<unsigned> counter(4);
  kernels::fill<float>(x.get(), n, 1.0f, nullptr);
  kernels::fill<float>(y.get(), n, 1.0f, nullptr);
  kernels::dot<float, float>(x.get(), y.get(), n, out.get(), partials.get(), counter.get(),
                             racy ? kernels::DotReduce::Racy : kernels::DotReduce::Atomic, blocks, nullptr);
  std::cout << hipGetErrorString(hipGetLastError()) << std::endl;
  float g = 0.f;
  MXS_HIP_CHECK(hipMemcpy(&g, out.get(), sizeof(float), hipMemcpyDeviceToHost));
  std::vector<float> hx(static_cast<size_t>(n)), hy(static_cast<size_t>(n));
  MXS_HIP_CHECK(hipMemcpy(hx.data(), x.get(), x.bytes(), hipMemcpyDeviceToHost));
  MXS_HIP_CHECK(hipMemcpy(hy.data(), y.get(), y.bytes(), hipMemcpyDeviceToHost));
  float c = 0.f;
  for (index_t i = 0; i < n; ++i) c += hx[size_t(i)] * hy[size_t(i)];
  std::cout << "GPU: " << g << std::endl;
  std::cout << "CPU: " << c << std::endl;
  return 0;
}
