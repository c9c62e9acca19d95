// CPU pinning for host-compute ranks. Busy-polling MPI ranks that start on the
// same core crawl until the scheduler separates them (measured: the CPU stencil
// plumbing config ran 20x slower for its first ~100-300 iterations); pinning
// rank i to the i-th CPU of the inherited affinity mask removes that.
#pragma once

#include <sched.h>

namespace mxs {

// Pin the calling process to the (local_rank mod n)-th CPU it is allowed to run
// on. Returns the CPU id, or -1 when the mask could not be read or set.
inline int pin_to_cpu(int local_rank) {
  cpu_set_t mask;
  CPU_ZERO(&mask);
  if (sched_getaffinity(0, sizeof(mask), &mask) != 0) return -1;
  const int n = CPU_COUNT(&mask);
  if (n <= 0) return -1;
  int want = local_rank % n, seen = 0;
  for (int cpu = 0; cpu < CPU_SETSIZE; ++cpu) {
    if (!CPU_ISSET(cpu, &mask)) continue;
    if (seen++ == want) {
      cpu_set_t one;
      CPU_ZERO(&one);
      CPU_SET(cpu, &one);
      return sched_setaffinity(0, sizeof(one), &one) == 0 ? cpu : -1;
    }
  }
  return -1;
}

}  // namespace mxs
