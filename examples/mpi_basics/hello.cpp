// MPI tutorial 1: init / finalize (reference: mpi1.cpp).
#include <mpi.h>

#include <cstdio>

int main(int argc, char** argv) {
  MPI_Init(&argc, &argv);
  int rank = 0, size = 0, len = 0;
  char node[MPI_MAX_PROCESSOR_NAME];
  MPI_Comm_rank(MPI_COMM_WORLD, &rank);
  MPI_Comm_size(MPI_COMM_WORLD, &size);
  MPI_Get_processor_name(node, &len);
  std::printf("Hello world from process %d of %d -- Node ID = %s\n", rank, size, node);
  MPI_Finalize();
  return 0;
}
