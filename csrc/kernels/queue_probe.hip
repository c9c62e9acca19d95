// Whether two HIP streams execute concurrently. HIP maps streams onto a pool of
// hardware queues (GPU_MAX_HW_QUEUES, 4 here); two streams on one queue run in
// submission order. The interior-first opening runs its inner chunks on one
// stream while the exchange and the outer chunks go to another: on a shared
// queue they serialise and the 8-GPU-tile opening takes ~0.5 ms instead of
// ~0.3 (seen in 2 of 14 bench-flow windows, profiles/r04_sg).
// Also: spin_delay, the one-GPU rehearsal's stand-in for xGMI wire time.
#include <hip/hip_runtime.h>

#include <chrono>

#include "mxs/core/error.hpp"
#include "mxs/kernels/kernels.hpp"

namespace mxs {
namespace kernels {
namespace {

// One wave sleeping `rounds` x 127 x 64 cycles (~0.8 ms for 200 rounds): bounded.
__global__ __launch_bounds__(64) void sleep_kernel(unsigned rounds) {
  for (unsigned i = 0; i < rounds; ++i) __builtin_amdgcn_s_sleep(127);
}

__global__ __launch_bounds__(64) void touch_kernel(unsigned* p) {
  if (threadIdx.x == 0 && p) *p = 1u;
}

// One wave holding its queue for `ticks` of the constant-rate wall clock
// (wall_clock64(), hipDeviceAttributeWallClockRate): bounded by the host's cap.
__global__ __launch_bounds__(64) void spin_delay_kernel(unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(2);
}

// kClockStampWgs one-wave workgroups (dealt over the CUs); lane 0 of each
// records (XCD and CU id, shader clock, wall clock) at out[3 b ..]. The shader
// clock counter (s_memtime: SCLK cycles, its rate follows DVFS) is not
// synchronised between counters, so two stamps are compared CU by CU; the
// wall clock (100 MHz) is global.
__global__ __launch_bounds__(64) void clock_stamp_kernel(unsigned long long* out) {
  if (threadIdx.x != 0) return;
  const unsigned xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);  // HW_REG_XCC_ID[3:0]
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);   // HW_REG_HW_ID: SE, SH, CU
  out[3 * blockIdx.x] = (xcc << 16) | ((hw >> 8) & 0x7Fu);                  // XCD, SE/SH/CU: one counter's id
  out[3 * blockIdx.x + 1] = clock64();
  out[3 * blockIdx.x + 2] = wall_clock64();
}

}  // namespace

void clock_stamp(unsigned long long* out, hipStream_t s) {
  clock_stamp_kernel<<<kClockStampWgs, 64, 0, s>>>(out);
  MXS_HIP_CHECK_LAUNCH();
}

void spin_delay(double us, hipStream_t s) {
  static const double ticks_per_us = [] {
    int dev = 0, khz = 0;
    MXS_HIP_CHECK(hipGetDevice(&dev));
    MXS_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
    return khz > 0 ? double(khz) / 1e3 : 100.0;
  }();
  const double capped = us < 0 ? 0 : (us > 10000.0 ? 10000.0 : us);  // at most 10 ms
  spin_delay_kernel<<<1, 64, 0, s>>>((unsigned long long)(capped * ticks_per_us));
  MXS_HIP_CHECK_LAUNCH();
}

bool streams_concurrent(hipStream_t a, hipStream_t b) {
  hipEvent_t done_b = nullptr;
  MXS_HIP_CHECK(hipEventCreateWithFlags(&done_b, hipEventDisableTiming));
  sleep_kernel<<<1, 64, 0, a>>>(200u);
  MXS_HIP_CHECK_LAUNCH();
  touch_kernel<<<1, 64, 0, b>>>(nullptr);
  MXS_HIP_CHECK_LAUNCH();
  MXS_HIP_CHECK(hipEventRecord(done_b, b));
  bool concurrent = false;
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const hipError_t q = hipEventQuery(done_b);
    if (q == hipSuccess) {
      const hipError_t qa = hipStreamQuery(a);
      concurrent = qa == hipErrorNotReady;
      (void)hipGetLastError();
      break;
    }
    if (q != hipErrorNotReady) MXS_HIP_CHECK(q);
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200)) break;
  }
  MXS_HIP_CHECK(hipStreamSynchronize(a));
  MXS_HIP_CHECK(hipStreamSynchronize(b));
  (void)hipEventDestroy(done_b);
  return concurrent;
}

}  // namespace kernels
}  // namespace mxs
