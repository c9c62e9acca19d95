#include "mxs/comm/mpi_env.hpp"

#include <cstdlib>

namespace mxs {

MpiEnv::MpiEnv(int* argc, char*** argv, MpiErrors mode) {
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
    error_config().abort_hook = [](int code) { MPI_Abort(MPI_COMM_WORLD, code == 0 ? 1 : code); };
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

MpiEnv::~MpiEnv() {
  if (finalize_) {
    int fin = 0;
    MPI_Finalized(&fin);
    if (!fin) MPI_Finalize();
  }
}

double MpiEnv::max_over_ranks(double v) const {
  double r = v;
  MXS_MPI_CHECK(MPI_Allreduce(&v, &r, 1, MPI_DOUBLE, MPI_MAX, MPI_COMM_WORLD));
  return r;
}

double MpiEnv::sum_over_ranks(double v) const {
  double r = v;
  MXS_MPI_CHECK(MPI_Allreduce(&v, &r, 1, MPI_DOUBLE, MPI_SUM, MPI_COMM_WORLD));
  return r;
}

}  // namespace mxs
