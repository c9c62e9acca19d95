// Error handling for the HIP runtime and RCCL (reference: cuda_error_handler.h:47-86,
// CHECK_CUDA_ERROR at test-benchmark/mpi-pingpong-gpu.cpp:17-22). MPI errors live in
// comm/mpi_error.hpp so that translation units without MPI do not pull in <mpi.h>.
//
// Policy: by default every failure throws mxs::Error (callers that run under MPI
// install an abort hook that calls MPI_Abort so one failing rank tears the job down
// instead of leaving its peers blocked in a collective).
#pragma once

#include <cstdio>
#include <cstdlib>
#include <functional>
#include <sstream>
#include <stdexcept>
#include <string>

namespace mxs {

class Error : public std::runtime_error {
 public:
  explicit Error(const std::string& what) : std::runtime_error(what) {}
};

enum class ErrorPolicy { Throw, Abort };

struct ErrorConfig {
  ErrorPolicy policy = ErrorPolicy::Throw;
  // Called before std::abort() under ErrorPolicy::Abort (e.g. MPI_Abort).
  std::function<void(int)> abort_hook;
};

inline ErrorConfig& error_config() {
  static ErrorConfig cfg;
  return cfg;
}

[[noreturn]] inline void raise_error(const std::string& msg, int code = 1) {
  if (error_config().policy == ErrorPolicy::Abort) {
    std::fputs((msg + "\n").c_str(), stderr);
    std::fflush(stderr);
    if (error_config().abort_hook) error_config().abort_hook(code);
    std::abort();
  }
  throw Error(msg);
}

inline std::string where(const char* file, int line) {
  std::ostringstream os;
  os << file << ':' << line;
  return os.str();
}

#define MXS_CHECK(cond, msg)                                                   \
  do {                                                                         \
    if (!(cond)) {                                                             \
      std::ostringstream mxs_os_;                                              \
      mxs_os_ << ::mxs::where(__FILE__, __LINE__) << " - check failed: " #cond \
              << " - " << msg;                                                 \
      ::mxs::raise_error(mxs_os_.str());                                       \
    }                                                                          \
  } while (0)

}  // namespace mxs

#if defined(__HIP_PLATFORM_AMD__) || defined(__HIPCC__) || defined(MXS_WITH_HIP)
#include <hip/hip_runtime_api.h>

namespace mxs {
inline void hip_check(hipError_t err, const char* expr, const char* file, int line) {
  if (err != hipSuccess) {
    std::ostringstream os;
    os << where(file, line) << " - HIP error " << int(err) << " (" << hipGetErrorName(err)
       << "): " << hipGetErrorString(err) << " in `" << expr << "`";
    raise_error(os.str(), int(err));
  }
}
}  // namespace mxs

#define MXS_HIP_CHECK(expr) ::mxs::hip_check((expr), #expr, __FILE__, __LINE__)
// Kernel-launch check (reference DIE_ON_FAILED_KERNEL_LAUNCH, cuda_error_handler.h:80-86).
#define MXS_HIP_CHECK_LAUNCH() ::mxs::hip_check(hipGetLastError(), "kernel launch", __FILE__, __LINE__)
#endif

// RCCL checks (MXS_RCCL_CHECK) live in comm/rccl_comm.hpp.
