// RCCL communicator: the device data plane over xGMI.
//
// The reference pushed device pointers through a CUDA-aware MVAPICH2
// (stencil2d/stencil2D.h:369,373; test-benchmark/mpi-pingpong-gpu.cpp:52-53).
// Here every device-to-device byte goes through RCCL point-to-point or
// collectives on a HIP stream; the control plane (rank discovery, unique-id
// broadcast, host scalars) is MPI for the C++ apps and torch.distributed for the
// Python launcher. Bootstrap is therefore a plain byte string.
#pragma once

#include <atomic>

#include <rccl/rccl.h>

#include <memory>
#include <sstream>
#include <string>
#include <type_traits>

#include "mxs/core/error.hpp"

namespace mxs {

inline void rccl_check(ncclResult_t res, const char* expr, const char* file, int line) {
  if (res != ncclSuccess) {
    std::ostringstream os;
    os << where(file, line) << " - RCCL error " << int(res) << ": " << ncclGetErrorString(res) << " in `" << expr
       << "`";
    raise_error(os.str(), int(res));
  }
}
#define MXS_RCCL_CHECK(expr) ::mxs::rccl_check((expr), #expr, __FILE__, __LINE__)

template <typename T>
constexpr ncclDataType_t rccl_type() {
  if constexpr (std::is_same_v<T, float>) return ncclFloat32;
  else if constexpr (std::is_same_v<T, double>) return ncclFloat64;
  else if constexpr (std::is_same_v<T, int>) return ncclInt32;
  else if constexpr (std::is_same_v<T, unsigned char> || std::is_same_v<T, char>) return ncclUint8;
  else if constexpr (std::is_same_v<T, long long> || std::is_same_v<T, long>) return ncclInt64;
  else if constexpr (std::is_same_v<T, unsigned>) return ncclUint32;
  else if constexpr (std::is_same_v<T, unsigned long long> || std::is_same_v<T, unsigned long>) return ncclUint64;
  else static_assert(sizeof(T) == 0, "unsupported RCCL element type");
}

class RcclComm {
 public:
  // NCCL_UNIQUE_ID_BYTES raw bytes; call on one rank and broadcast.
  static std::string make_unique_id();

  // Collective over all `nranks` processes; the calling process must have
  // selected its HIP device already.
  RcclComm(const std::string& unique_id, int nranks, int rank);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  ncclComm_t get() const { return comm_.load(std::memory_order_acquire); }
  bool aborted() const { return get() == nullptr; }
  int rank() const { return rank_; }
  int size() const { return nranks_; }

  // Non-blocking health probe (ncclCommGetAsyncError): returns false and fills
  // `msg` when the communicator is in an error state (e.g. a peer died).
  bool healthy(std::string* msg = nullptr) const;
  // Tear the communicator down without waiting for peers (after a failure).
  // Later calls on it fail with "communicator aborted"; the destructor skips it.
  void abort() const;
  // Wait for `stream` under the communication watchdog (mxs/core/fault.hpp):
  // fails on an RCCL async error, or after comm_timeout() seconds (the
  // communicator is aborted first so the error path cannot block on it).
  void wait(hipStream_t stream, const char* what) const;
  // The same for several streams in one poll loop (each stream is queried until
  // it has drained; a window's end is noticed one poll after its last kernel).
  void wait_all(const hipStream_t* streams, int n, const char* what) const;

  // A communicator over the same ranks whose kernels use at most `max_ctas`
  // workgroups (ncclCommSplit with ncclConfig_t::maxCTAs; collective). The
  // halo exchange of the interior-first opening runs on the CUs the inner
  // chunk launch leaves free (32-48 of 256): a cap keeps RCCL's kernels from
  // queueing behind it. Throws when the RCCL in use rejects the config.
  std::unique_ptr<RcclComm> split_with_max_ctas(int max_ctas) const;
  int max_ctas() const { return max_ctas_; }

  // Ranks the communicator really spans (ncclCommCount) and the HIP device
  // this rank's end of it runs on (ncclCommCuDevice): the run records quote
  // these, not the launcher's view.
  int count() const;
  int device() const;

  // Sum-allreduce `count` elements in place or out of place on `stream`.
  template <typename T>
  void allreduce_sum(const T* send, T* recv, size_t count, hipStream_t stream) const {
    MXS_RCCL_CHECK(ncclAllReduce(send, recv, count, rccl_type<T>(), ncclSum, live(), stream));
  }
  // Element-wise max over ranks (the solver's collective schedule decisions).
  template <typename T>
  void allreduce_max(const T* send, T* recv, size_t count, hipStream_t stream) const {
    MXS_RCCL_CHECK(ncclAllReduce(send, recv, count, rccl_type<T>(), ncclMax, live(), stream));
  }
  template <typename T>
  void send(const T* buf, size_t count, int peer, hipStream_t stream) const {
    MXS_RCCL_CHECK(ncclSend(buf, count, rccl_type<T>(), peer, live(), stream));
  }
  template <typename T>
  void recv(T* buf, size_t count, int peer, hipStream_t stream) const {
    MXS_RCCL_CHECK(ncclRecv(buf, count, rccl_type<T>(), peer, live(), stream));
  }
  void group_start() const { MXS_RCCL_CHECK(ncclGroupStart()); }
  void group_end() const { MXS_RCCL_CHECK(ncclGroupEnd()); }

 private:
  ncclComm_t live() const {
    ncclComm_t c = get();
    MXS_CHECK(c != nullptr, "RCCL communicator aborted (an earlier wait timed out or failed)");
    return c;
  }
  RcclComm() = default;
  // Mutable: a watchdog timeout inside a const wait() aborts and clears it.
  // Atomic: abort() may come from a watchdog thread while this thread is
  // blocked in a device wait (parallel/watchdog.py); exactly one caller takes
  // the handle and aborts it.
  mutable std::atomic<ncclComm_t> comm_{nullptr};
  int rank_ = 0;
  int nranks_ = 1;
  int max_ctas_ = 0;  // 0: RCCL's default
};

}  // namespace mxs
