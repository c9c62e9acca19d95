// stencil2d_cpu — 2D domain-decomposed stencil on the CPU over MPI (host memory,
// subarray datatypes). Reference: stencil2d/mpi-2d-stencil-subarray.cpp.
//
//   mpiexec -n 9 stencil2d_cpu                 # reference run: 16x16 tiles, 5x5 stencil,
//                                              # fp64, one exchange, per-rank dump files
//   mpiexec -n 2 stencil2d_cpu --global 256x256 --dtype f32 --iters 200
//                                              # BASELINE plumbing config, Gcells/s
//
// Positional arguments keep the reference contract: [local width (= height) [stencil width]].
// Options: --local WxH | --global WxH, --dims RxC, --stencil-height H, --dtype f32|f64,
// --iters N (0 = one exchange, reference behaviour), --warmup N, --dump / --no-dump,
// --non-periodic, --strict-square (reproduce the reference's perfect-square check),
// --seed S, --json FILE, --checkpoint FILE (collective MPI-IO global grid file
// after the last iteration), --resume FILE (start from such a file, any
// decomposition), --comm-timeout SECONDS (halo watchdog), --fault-inject
// RANK:ITER[:exit|hang|error] (failure-path testing), --no-bind-cpu
// (keep the launcher's CPU placement instead of one core per rank).
#include <mpi.h>

#include <chrono>
#include <cmath>
#include <fstream>
#include <iostream>
#include <sstream>
#include <vector>

#include "app_common.hpp"
#include "mxs/comm/mpi_checkpoint.hpp"
#include "mxs/comm/mpi_env.hpp"
#include "mxs/comm/mpi_host_halo.hpp"
#include "mxs/core/affinity.hpp"
#include "mxs/core/cli.hpp"
#include "mxs/grid/host_stencil.hpp"
#include "mxs/grid/init.hpp"
#include "mxs/grid/print.hpp"

using namespace mxs;

template <typename T>
int run(MpiEnv& env, const Cli& cli, const CartTopology& topo, index_t lw, index_t lh, index_t gx0, index_t gy0,
        index_t gw, index_t gh, int sw, int sh) {
  const int rank = env.rank();
  const TileGeom g = TileGeom::compact(lw, lh, sw / 2, sh / 2);
  MPI_Comm cart = make_cart_comm(topo);
  const long long iters = cli.get_int("iters", 0);
  const bool dump = cli.has("dump") ? cli.flag("dump") : (iters == 0 && lw <= 64 && lh <= 64 && !cli.flag("no-dump"));
  std::vector<T> a(size_t(g.alloc_elems()), T(-1)), b(size_t(g.alloc_elems()), T(-1));
  MpiHostHalo<T> halo(topo, rank, g, cart, /*corners=*/true);

  if (iters == 0) {
    // Reference run: core = rank id, ghosts = -1, one exchange, dump before/after.
    const Array2D core = g.core();
    for (index_t y = 0; y < core.height; ++y)
      for (index_t x = 0; x < core.width; ++x) a[size_t(core.index(x, y))] = T(rank);
    std::ostringstream os;
    if (dump) {
      write_dump_header(os, topo, rank, -1, lw, lh, sw, sh, "");
      os << "Array" << '\n';
      app::dump_tile(os, a.data(), g);
      os << '\n';
    }
    halo.exchange(a.data());
    if (dump) {
      os << "Array after exchange" << '\n';
      app::dump_tile(os, a.data(), g);
      std::ofstream f(dump_file_name(topo, rank));
      f << os.str();
    }
  } else {
    MXS_CHECK(sw >= 3 && sh >= 3, "--iters needs a stencil of width >= 3 (ghost ring >= 1)");
    const std::uint64_t seed = std::uint64_t(cli.get_int("seed", 1234));
    const GlobalBlock blk{gx0, gy0, gw, gh};
    std::int64_t start_iter = 0;
    if (cli.has("resume")) {
      const GridFileHeader hdr = read_grid_file<T>(MPI_COMM_WORLD, cli.get("resume"), a.data(), g, blk);
      start_iter = hdr.iteration;
      if (rank == 0) std::cout << "resumed from " << cli.get("resume") << " at iteration " << start_iter << '\n';
    } else {
      fill_random_host<T>(a.data(), g, gx0, gy0, gw, seed);
    }
    const T c0 = T(cli.get_double("c-center", 0.2)), c1 = T(cli.get_double("c-neighbor", 0.2));
    T* cur = a.data();
    T* nxt = b.data();
    const FaultSpec fault = parse_fault_spec(cli.get("fault-inject", ""));
    long long it = 0;
    auto step = [&]() {
      maybe_inject_fault(fault, rank, it++);
      halo.exchange(cur);
      jacobi5_host<T>(cur, nxt, g, 0, lh, c0, c1);
      std::swap(cur, nxt);
    };
    // MPICH reaches its fast polling regime only after ~100 round trips: time the
    // steady state (warm-up iterations count towards --iters).
    const long long warmup = cli.get_int("warmup", std::min<long long>(100, iters / 2));
    for (long long i = 0; i < warmup; ++i) step();
    env.barrier();
    const double t0 = MPI_Wtime();
    for (long long i = warmup; i < iters; ++i) step();
    env.barrier();
    const double dt = env.max_over_ranks(MPI_Wtime() - t0);
    double local = 0;
    for (index_t y = 0; y < lh; ++y)
      for (index_t x = 0; x < lw; ++x) local += double(cur[size_t(g.core_offset() + y * g.pitch + x)]);
    const double checksum = env.sum_over_ranks(local);
    const long long timed = iters - warmup;
    const double gcells = double(gw) * double(gh) * double(timed) / dt / 1e9;
    if (rank == 0) {
      std::ostringstream js;
      js << "{\"app\": \"stencil2d_cpu\", \"metric\": \"gcells_per_s\", \"value\": " << app::fmt(gcells)
         << ", \"ranks\": " << env.size() << ", \"dims\": \"" << topo.rows << "x" << topo.cols << "\", \"global\": \""
         << gw << "x" << gh << "\", \"dtype\": \"" << (sizeof(T) == 4 ? "f32" : "f64") << "\", \"iters\": " << timed
         << ", \"seconds\": " << app::fmt(dt) << ", \"checksum\": " << app::fmt(checksum)
         << app::meta_json("cpu") << "}";
      std::cout << "Gcells/s: " << app::fmt(gcells) << "\nchecksum: " << app::fmt(checksum) << "\n" << js.str()
                << std::endl;
      app::append_json(cli.get("json"), js.str());
    }
    if (cli.has("checkpoint")) write_grid_file<T>(MPI_COMM_WORLD, cli.get("checkpoint"), cur, g, blk, start_iter + iters, seed);
    if (dump) {
      std::ofstream f(dump_file_name(topo, rank));
      write_dump_header(f, topo, rank, -1, lw, lh, sw, sh, "");
      f << "Array after " << iters << " iterations" << '\n';
      app::dump_tile(f, cur, g);
    }
  }
  MPI_Comm_free(&cart);
  return 0;
}

int main(int argc, char** argv) {
  MpiEnv env(&argc, &argv);
  Cli cli(argc, argv, {"dump", "no-dump", "non-periodic", "strict-square", "no-bind-cpu"});
  // One core per rank (node-local order) unless the launcher already bound us.
  if (!cli.flag("no-bind-cpu")) pin_to_cpu(env.local_rank());
  comm_timeout() = cli.get_double("comm-timeout", 0.0);
  const int n = env.size();
  // Process grid: the reference's sqrt(N) x sqrt(N) when N is a perfect square,
  // otherwise MPI_Dims_create (the reference refused).
  int rows, cols;
  const int dim = int(std::lround(std::sqrt(double(n))));
  if (cli.has("dims")) {
    auto d = parse_dims(cli.get("dims"));
    rows = d[0];
    cols = d[1];
  } else if (dim * dim == n) {
    rows = cols = dim;
  } else {
    if (cli.flag("strict-square")) {
      if (env.rank() == 0) std::cerr << "Numer of MPI tasks must be a perfect square" << std::endl;
      return 1;
    }
    auto d = dims_create(n);
    rows = d[0];
    cols = d[1];
  }
  if (rows * cols != n) {
    if (env.rank() == 0) std::cerr << "process grid " << rows << "x" << cols << " != " << n << " ranks" << std::endl;
    return 1;
  }
  const bool periodic = !cli.flag("non-periodic");
  const CartTopology topo(rows, cols, periodic, periodic);
  const auto c = topo.coords(env.rank());

  // Tile size: positional argv[1] (square, reference), --local, or --global split.
  const auto& pos = cli.positional();
  index_t gw = 0, gh = 0, lw = 16, lh = 16;
  int sw = 5;
  if (!pos.empty()) lw = lh = std::atoll(pos[0].c_str());
  if (pos.size() >= 2) sw = std::atoi(pos[1].c_str());
  if (cli.has("stencil")) sw = int(cli.get_int("stencil", sw));
  int sh = int(cli.get_int("stencil-height", sw));  // the reference ignored argv for the height (Q3)
  index_t gx0, gy0;
  if (cli.has("global")) {
    auto wh = parse_wxh(cli.get("global"));
    gw = wh.first;
    gh = wh.second;
    const Block1D bx = block_split(gw, cols, c[1]), by = block_split(gh, rows, c[0]);
    lw = bx.len;
    lh = by.len;
    gx0 = bx.start;
    gy0 = by.start;
  } else {
    if (cli.has("local")) {
      auto wh = parse_wxh(cli.get("local"));
      lw = wh.first;
      lh = wh.second;
    }
    gw = lw * cols;
    gh = lh * rows;
    gx0 = lw * c[1];
    gy0 = lh * c[0];
  }
  if (lw < sw || lh < sh) {
    if (env.rank() == 0) std::cerr << "Error: grid size < stencil size" << std::endl;
    return 1;
  }
  if (cli.get("dtype", "f64") == "f32") return run<float>(env, cli, topo, lw, lh, gx0, gy0, gw, gh, sw, sh);
  return run<double>(env, cli, topo, lw, lh, gx0, gy0, gw, gh, sw, sh);
}
