// MPI tutorial 3: send / probe / recv of a message of unknown size (reference: mpi3.cpp).
#include <mpi.h>

#include <iostream>
#include <string>
#include <vector>

#include "mxs/comm/mpi_env.hpp"

int main(int argc, char** argv) {
  mxs::MpiEnv env(&argc, &argv);
  const int tag0to1 = 0x01, tag1to0 = 0x10;
  auto receive = [](int src, int tag) {
    MPI_Status st;
    MXS_MPI_CHECK(MPI_Probe(src, tag, MPI_COMM_WORLD, &st));
    int count = 0;
    MXS_MPI_CHECK(MPI_Get_count(&st, MPI_CHAR, &count));
    std::vector<char> buf(size_t(count) + 1, '\0');
    MXS_MPI_CHECK(MPI_Recv(buf.data(), count, MPI_CHAR, src, tag, MPI_COMM_WORLD, &st));
    return std::string(buf.data());
  };
  auto send = [](const std::string& s, int dst, int tag) {
    MXS_MPI_CHECK(MPI_Send(s.c_str(), int(s.size() + 1), MPI_CHAR, dst, tag, MPI_COMM_WORLD));
  };
  if (env.rank() == 0) {
    send("Hello from rank 0", 1, tag0to1);
    // Receive first, then print the whole line in one write: the two ranks'
    // lines must not interleave on a shared stdout.
    const std::string msg = receive(1, tag1to0);
    std::cout << "Task 0:  received message \"" + msg + "\"\n" << std::flush;
  } else if (env.rank() == 1) {
    const std::string msg = receive(0, tag0to1);
    std::cout << "Task 1:  received message \"" + msg + "\"\n" << std::flush;
    send("Hello from rank 1", 0, tag1to0);
  }
  return 0;
}
