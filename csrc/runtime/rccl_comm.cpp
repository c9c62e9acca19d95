#include "mxs/comm/rccl_comm.hpp"

#include <chrono>
#include <cstring>

#include "mxs/core/fault.hpp"

namespace mxs {

std::string RcclComm::make_unique_id() {
  ncclUniqueId id;
  MXS_RCCL_CHECK(ncclGetUniqueId(&id));
  return std::string(reinterpret_cast<const char*>(&id), sizeof(id));
}

RcclComm::RcclComm(const std::string& unique_id, int nranks, int rank) : rank_(rank), nranks_(nranks) {
  MXS_CHECK(unique_id.size() == sizeof(ncclUniqueId),
            "RcclComm: unique id must be " << sizeof(ncclUniqueId) << " bytes, got " << unique_id.size());
  MXS_CHECK(rank >= 0 && rank < nranks, "RcclComm: bad rank " << rank << " of " << nranks);
  ncclUniqueId id;
  std::memcpy(&id, unique_id.data(), sizeof(id));
  ncclComm_t c = nullptr;
  MXS_RCCL_CHECK(ncclCommInitRank(&c, nranks, id, rank));
  comm_.store(c, std::memory_order_release);
}

RcclComm::~RcclComm() {
  if (ncclComm_t c = comm_.exchange(nullptr)) (void)ncclCommDestroy(c);
}

bool RcclComm::healthy(std::string* msg) const {
  ncclComm_t c = get();
  if (!c) return false;
  ncclResult_t async = ncclSuccess;
  if (ncclCommGetAsyncError(c, &async) != ncclSuccess || async != ncclSuccess) {
    if (msg) *msg = ncclGetErrorString(async);
    return false;
  }
  return true;
}

void RcclComm::wait(hipStream_t stream, const char* what) const { wait_all(&stream, 1, what); }

void RcclComm::wait_all(const hipStream_t* streams, int n, const char* what) const {
  // The stream is polled on every spin; the communicator's async error state
  // (a call into RCCL) only once per millisecond: querying it on every spin
  // delayed noticing the completion of a 20-step window by ~100 us.
  using clock = std::chrono::steady_clock;
  auto next_check = clock::now();
  int done = 0;  // streams [0, done) have drained
  wait_with_timeout(
      [&] {
        while (done < n) {
          const hipError_t q = hipStreamQuery(streams[done]);
          if (q == hipSuccess) {
            ++done;
            continue;
          }
          if (q != hipErrorNotReady) MXS_HIP_CHECK(q);
          break;
        }
        if (done == n) return true;
        const auto now = clock::now();
        if (now >= next_check) {
          next_check = now + std::chrono::milliseconds(1);
          std::string msg;
          if (!healthy(&msg)) raise_error(std::string(what) + ": RCCL communicator failed: " + msg);
        }
        return false;
      },
      what, [&] { abort(); });
}

std::unique_ptr<RcclComm> RcclComm::split_with_max_ctas(int max_ctas) const {
  MXS_CHECK(max_ctas > 0, "split_with_max_ctas: cap must be positive, got " << max_ctas);
  ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
  cfg.maxCTAs = max_ctas;
  cfg.minCTAs = 1;
  std::unique_ptr<RcclComm> c(new RcclComm());
  c->rank_ = rank_;
  c->nranks_ = nranks_;
  c->max_ctas_ = max_ctas;
  ncclComm_t sc = nullptr;
  MXS_RCCL_CHECK(ncclCommSplit(live(), 0, rank_, &sc, &cfg));
  MXS_CHECK(sc != nullptr, "ncclCommSplit returned no communicator");
  c->comm_.store(sc, std::memory_order_release);
  return c;
}

int RcclComm::count() const {
  int n = 0;
  MXS_RCCL_CHECK(ncclCommCount(live(), &n));
  return n;
}

int RcclComm::device() const {
  int d = -1;
  MXS_RCCL_CHECK(ncclCommCuDevice(live(), &d));
  return d;
}

void RcclComm::abort() const {
  if (ncclComm_t c = comm_.exchange(nullptr)) (void)ncclCommAbort(c);
}

}  // namespace mxs
