// MPI control plane for the C++ apps (reference: mpierr.h — the MPI_ macro that
// formats "Error <code>: error message / error class message" and either throws
// (-DMPI_ERR_USE_EXCEPTIONS) or prints and MPI_Aborts).
//
// MpiEnv is the RAII owner of MPI_Init/MPI_Finalize. It installs
// MPI_ERRORS_RETURN on MPI_COMM_WORLD with MPI_Comm_set_errhandler (the
// reference used MPI_Errhandler_set, removed in MPI-3, and called it before
// MPI_Init in mpicuda2.cpp — SURVEY Q6) and routes every mxs failure (HIP, RCCL,
// checks) to MPI_Abort so one failing rank never leaves its peers blocked.
#pragma once

#include <mpi.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "mxs/core/error.hpp"
#include "mxs/core/fault.hpp"

namespace mxs {

// "Error <code>:\n  error message: <string>\n  error class message: <class string>"
inline std::string format_mpi_error(int code) {
  char buf[MPI_MAX_ERROR_STRING];
  int len = 0;
  std::ostringstream os;
  MPI_Error_string(code, buf, &len);
  os << "Error " << code << ":\n  error message: " << std::string(buf, size_t(len));
  int cls = 0;
  MPI_Error_class(code, &cls);
  MPI_Error_string(cls, buf, &len);
  os << "\n  error class message: " << std::string(buf, size_t(len));
  return os.str();
}

inline void mpi_check(int code, const char* expr, const char* file, int line) {
  if (code == MPI_SUCCESS) return;
  std::ostringstream os;
  os << where(file, line) << " - " << expr << " failed\n" << format_mpi_error(code);
  raise_error(os.str(), code);
}

#define MXS_MPI_CHECK(expr) ::mxs::mpi_check((expr), #expr, __FILE__, __LINE__)

// MPI_Waitall under the communication watchdog (mxs/core/fault.hpp): with a
// comm_timeout() set, polls MPI_Testall and fails after the timeout instead of
// blocking forever on a dead or hung peer.
inline void mpi_wait_all(std::vector<MPI_Request>& req, const char* what) {
  if (req.empty()) return;
  if (comm_timeout() <= 0) {
    MXS_MPI_CHECK(MPI_Waitall(int(req.size()), req.data(), MPI_STATUSES_IGNORE));
    return;
  }
  wait_with_timeout(
      [&] {
        int flag = 0;
        MXS_MPI_CHECK(MPI_Testall(int(req.size()), req.data(), &flag, MPI_STATUSES_IGNORE));
        return flag != 0;
      },
      what, [] {});
}

// Variable-length allgather of byte strings (control-plane sized), rank order.
// Usable as the IPC halo backend's HostAllgather bootstrap.
inline std::vector<std::string> mpi_allgather_bytes(MPI_Comm comm, const std::string& blob) {
  int n = 0;
  MXS_MPI_CHECK(MPI_Comm_size(comm, &n));
  int len = int(blob.size());
  std::vector<int> lens(static_cast<size_t>(n)), displs(static_cast<size_t>(n), 0);
  MXS_MPI_CHECK(MPI_Allgather(&len, 1, MPI_INT, lens.data(), 1, MPI_INT, comm));
  for (int r = 1; r < n; ++r) displs[size_t(r)] = displs[size_t(r - 1)] + lens[size_t(r - 1)];
  std::string all(size_t(displs[size_t(n - 1)] + lens[size_t(n - 1)]), '\0');
  MXS_MPI_CHECK(MPI_Allgatherv(blob.data(), len, MPI_BYTE, &all[0], lens.data(), displs.data(), MPI_BYTE, comm));
  std::vector<std::string> out(static_cast<size_t>(n));
  for (int r = 0; r < n; ++r) out[size_t(r)] = all.substr(size_t(displs[size_t(r)]), size_t(lens[size_t(r)]));
  return out;
}

enum class MpiErrors { Abort, Throw };

class MpiEnv {
 public:
  MpiEnv(int* argc, char*** argv, MpiErrors mode = MpiErrors::Abort);
  ~MpiEnv();
  MpiEnv(const MpiEnv&) = delete;
  MpiEnv& operator=(const MpiEnv&) = delete;

  int rank() const { return rank_; }
  int size() const { return size_; }
  const std::string& processor_name() const { return name_; }
  // Ranks sharing this node (MPI_Comm_split_type(MPI_COMM_TYPE_SHARED)).
  int local_rank() const { return local_rank_; }
  int local_size() const { return local_size_; }
  int node_count() const { return node_count_; }
  int node_index() const { return node_index_; }

  void barrier() const { MXS_MPI_CHECK(MPI_Barrier(MPI_COMM_WORLD)); }
  double max_over_ranks(double v) const;
  double sum_over_ranks(double v) const;

 private:
  int rank_ = 0, size_ = 1, local_rank_ = 0, local_size_ = 1, node_count_ = 1, node_index_ = 0;
  std::string name_;
  bool finalize_ = false;
};

// ----------------------------------------------------------------- inline impl
inline MpiEnv::MpiEnv(int* argc, char*** argv, MpiErrors mode) {
  int inited = 0;
  MPI_Initialized(&inited);
  if (!inited) {
    MPI_Init(argc, argv);
    finalize_ = true;
  }
  MPI_Comm_set_errhandler(MPI_COMM_WORLD, MPI_ERRORS_RETURN);
  MXS_MPI_CHECK(MPI_Comm_rank(MPI_COMM_WORLD, &rank_));
  MXS_MPI_CHECK(MPI_Comm_size(MPI_COMM_WORLD, &size_));
  char name[MPI_MAX_PROCESSOR_NAME];
  int len = 0;
  MXS_MPI_CHECK(MPI_Get_processor_name(name, &len));
  name_.assign(name, size_t(len));

  if (mode == MpiErrors::Abort) {
    error_config().policy = ErrorPolicy::Abort;
    error_config().abort_hook = [](int code) {
      // Let the launcher's stdio forwarding drain the error message before the
      // abort tears every rank down (otherwise it is often lost).
      std::fflush(nullptr);
      std::this_thread::sleep_for(std::chrono::milliseconds(300));
      MPI_Abort(MPI_COMM_WORLD, code == 0 ? 1 : code);
    };
  } else {
    error_config().policy = ErrorPolicy::Throw;
  }

  // Node-local rank and node count: the reference counted nodes by sending
  // every processor name to rank 0 (mpicuda2.cu:118-155); the
  // shared-memory split gives both directly.
  MPI_Comm node;
  MXS_MPI_CHECK(MPI_Comm_split_type(MPI_COMM_WORLD, MPI_COMM_TYPE_SHARED, rank_, MPI_INFO_NULL, &node));
  MXS_MPI_CHECK(MPI_Comm_rank(node, &local_rank_));
  MXS_MPI_CHECK(MPI_Comm_size(node, &local_size_));
  int leader = local_rank_ == 0 ? 1 : 0;
  MXS_MPI_CHECK(MPI_Allreduce(&leader, &node_count_, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD));
  // Node index = number of node leaders with a smaller world rank than this
  // node's leader; computed by the leader, broadcast inside the node.
  int before = 0;
  MXS_MPI_CHECK(MPI_Exscan(&leader, &before, 1, MPI_INT, MPI_SUM, MPI_COMM_WORLD));
  if (rank_ == 0) before = 0;  // MPI_Exscan leaves rank 0's result undefined
  node_index_ = before;
  MXS_MPI_CHECK(MPI_Bcast(&node_index_, 1, MPI_INT, 0, node));
  MXS_MPI_CHECK(MPI_Comm_free(&node));
}

inline MpiEnv::~MpiEnv() {
  if (finalize_) {
    int fin = 0;
    MPI_Finalized(&fin);
    if (!fin) MPI_Finalize();
  }
}

inline double MpiEnv::max_over_ranks(double v) const {
  double r = v;
  MXS_MPI_CHECK(MPI_Allreduce(&v, &r, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD));
  return r;
}

inline double MpiEnv::sum_over_ranks(double v) const {
  double r = v;
  MXS_MPI_CHECK(MPI_Allreduce(&v, &r, 1, MPI_DOUBLE, MPI_SUM, MPI_COMM_WORLD));
  return r;
}

}  // namespace mxs
