// MPI tutorial 4: blocking ping-pong counter between ranks 0 and 1 (reference: mpi4.cpp).
// Ranks >= 2 take no part (in the reference they spun forever).
// --sleep-ms N sets the pause per step (reference: 1000 ms).
#include <mpi.h>

#include <chrono>
#include <cstdlib>
#include <iostream>
#include <string>
#include <thread>

#include "mxs/comm/mpi_env.hpp"

int main(int argc, char** argv) {
  int sleep_ms = 1000;
  for (int i = 1; i + 1 < argc; ++i)
    if (std::string(argv[i]) == "--sleep-ms") sleep_ms = std::atoi(argv[i + 1]);
  mxs::MpiEnv env(&argc, &argv);
  const int tag0to1 = 0x01, tag1to0 = 0x10, kmax = 10;
  int k = 0;
  if (env.rank() == 0) std::cout << "\nRank 0\tRank 1\n" << std::endl;
  if (env.rank() < 2 && env.size() >= 2) {
    while (k != kmax) {
      if (env.rank() == 0) {
        ++k;
        std::cout << '\r' << k << std::flush;
        std::this_thread::sleep_for(std::chrono::milliseconds(sleep_ms));
        MXS_MPI_CHECK(MPI_Send(&k, 1, MPI_INT, 1, tag0to1, MPI_COMM_WORLD));
        MXS_MPI_CHECK(MPI_Recv(&k, 1, MPI_INT, 1, tag1to0, MPI_COMM_WORLD, MPI_STATUS_IGNORE));
      } else {
        MXS_MPI_CHECK(MPI_Recv(&k, 1, MPI_INT, 0, tag0to1, MPI_COMM_WORLD, MPI_STATUS_IGNORE));
        ++k;
        std::cout << "\r\t" << k << std::flush;
        std::this_thread::sleep_for(std::chrono::milliseconds(sleep_ms));
        MXS_MPI_CHECK(MPI_Send(&k, 1, MPI_INT, 0, tag1to0, MPI_COMM_WORLD));
      }
    }
  }
  if (env.rank() == 0) std::cout << "\n\nTotal: " << k << std::endl;
  return 0;
}
