// MPI tutorial 2: error handling (reference: mpi2.cpp + mpierr.h).
// MPI_ERRORS_RETURN is installed with MPI_Comm_set_errhandler (MPI_Errhandler_set was
// removed in MPI-3) and every call goes through MXS_MPI_CHECK, which formats
// "Error <code>: error message / error class message" and aborts (or throws with
// --throw). --demo-error sends to an invalid rank to show the formatted message.
#include <mpi.h>

#include <iostream>

#include "mxs/comm/mpi_env.hpp"

int main(int argc, char** argv) {
  bool demo = false, use_throw = false;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    demo |= a == "--demo-error";
    use_throw |= a == "--throw";
  }
  mxs::MpiEnv env(&argc, &argv, use_throw ? mxs::MpiErrors::Throw : mxs::MpiErrors::Abort);
  std::cout << "Hello world from process " << env.rank() << " of " << env.size() << " -- " << env.processor_name()
            << std::endl;
  if (demo) {
    int x = 0;
    const int rc = MPI_Send(&x, 1, MPI_INT, env.size() + 7, 0, MPI_COMM_WORLD);  // invalid rank
    if (rc != MPI_SUCCESS && env.rank() == 0) std::cout << mxs::format_mpi_error(rc) << std::endl;
    try {
      MXS_MPI_CHECK(rc);
    } catch (const mxs::Error& e) {
      if (env.rank() == 0) std::cout << "caught: " << e.what() << std::endl;
    }
  }
  return 0;
}
