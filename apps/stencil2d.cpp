// stencil2d — 2D domain-decomposed stencil on MI355X GPUs.
// Reference: stencil2d/mpi-2d-stencil-subarray-cuda.cu (+ stencil2d/stencil2D.h).
//
// MPI is the control plane (ranks, Cartesian grid, RCCL bootstrap, timing);
// device data moves by one of:
//   --backend rccl        per-peer ncclSend/ncclRecv over xGMI (default when every
//                         rank has its own GPU): each pass, then the exchange of its
//                         output (post-exchange); a call's opening super-step runs
//                         its priming exchange under the core chunks when prepare()
//                         measured that faster on every rank (--opening);
//   --backend ipc         HIP IPC: direct writes into the peers' receive buffers,
//                         device-side ready/free counters, overlap + hipGraph
//                         (default when ranks share a GPU, where RCCL refuses);
//   --backend mpi-staged  HIP pack -> pinned host staging -> MPI -> HIP unpack
//                         (--pageable for the non-PAGE_LOCKED variant);
//   --backend local       1x1 periodic grid: a single HIP self-copy launch.
//
//   mpiexec -n 9 stencil2d            # reference run: 16x16 tiles, 5x5 stencil, fp64,
//                                     # one exchange, per-rank dump files "row_col"
//   mpiexec -n 8 stencil2d --global 32768x32768 --dims 2x4 --dtype f32 --iters 200
//
// Positional arguments keep the reference contract: [local width (= height) [stencil width]].
// More options: --local WxH | --global WxH, --dims RxC, --stencil-height H, --dtype f32|f64,
// --iters N, --warmup N, --time-block S (default: measured per tile size and dtype), --no-overlap, --no-graph,
// --opening auto|serial|interior-first (--halo-last = interior-first; default auto: prepare() times the
// serial and interior-first openings, agrees the per-round maxima over all ranks and keeps the faster),
// --steady auto|serial|interior-first (the super-steps after an interior-first opening; auto: prepare() of a
// run with two or more super-steps times both the same way),
// --no-direct-halo (IPC backend: pack -> put -> unpack instead of the device-initiated push),
// --halo-max-ctas N (RCCL: the halo exchange on a communicator split off with at most N workgroups per kernel),
// --direct-halo on|off|validate (validate: prepare() compares the push with the backend's exchange bitwise on
// every rank, times both, and uses it only if equal everywhere and faster),
// --c-center C --c-neighbor C (default 0.2 / 0.2), --no-sum-form (keep the per-step evaluation in the
// time-blocked kernels: bitwise equal to the CPU app; default: sum form when the coefficients are equal,
// scaled form when they differ),
// --loopback, --bind bunch|rrobin,
// --dump / --no-dump, --checksum, --non-periodic, --seed S, --json FILE,
// --checkpoint FILE / --resume FILE (collective MPI-IO global grid file, any
// decomposition; same format as stencil2d_cpu and the Python package),
// --comm-timeout SECONDS (halo watchdog, default 300), --fault-inject
// RANK:ITER[:exit|hang|error] (failure-path testing).
#include <mpi.h>

#include <algorithm>
#include <cmath>
#include <fstream>
#include <iostream>
#include <memory>
#include <sstream>
#include <vector>

#include "app_common.hpp"
#include "mxs/comm/mpi_checkpoint.hpp"
#include "mxs/comm/mpi_env.hpp"
#include "mxs/comm/mpi_halo.hpp"
#include "mxs/comm/rccl_comm.hpp"
#include "mxs/core/cli.hpp"
#include "mxs/core/device.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/stencil_solver.hpp"

using namespace mxs;

namespace {

std::unique_ptr<RcclComm> make_comm(const MpiEnv& env) {
  std::string uid = env.rank() == 0 ? RcclComm::make_unique_id() : std::string(sizeof(ncclUniqueId), '\0');
  MXS_MPI_CHECK(MPI_Bcast(&uid[0], int(uid.size()), MPI_BYTE, 0, MPI_COMM_WORLD));
  return std::make_unique<RcclComm>(uid, env.size(), env.rank());
}

template <typename T>
void copy_tile_to_host(std::vector<T>& h, const T* d, const TileGeom& g) {
  h.resize(size_t(g.alloc_elems()));
  MXS_HIP_CHECK(hipMemcpy(h.data(), d, h.size() * sizeof(T), hipMemcpyDeviceToHost));
}

template <typename T>
int run(MpiEnv& env, const Cli& cli, const CartTopology& topo, const DeviceBinding& dev, index_t lw, index_t lh,
        index_t gx0, index_t gy0, index_t gw, index_t gh, int sw, int sh) {
  const int rank = env.rank();
  const long long iters = cli.get_int("iters", 0);
  const bool dump = cli.has("dump") ? cli.flag("dump") : (iters == 0 && lw <= 64 && lh <= 64 && !cli.flag("no-dump"));

  // Backend selection.
  std::string backend = cli.get("backend", "auto");
  const bool loopback = cli.flag("loopback");
  if (backend == "auto") {
    if (env.size() == 1) backend = loopback ? "rccl" : "local";
    else if (dev.shared) backend = "ipc";  // GPUs shared: RCCL refuses
    else backend = "rccl";
  }
  // Temporal blocking (timed runs on the solver backends): S Jacobi steps per
  // launch on an S-deep ghost ring exchanged once per S steps.
  // A non-periodic grid has fixed boundary values that the S-step kernels
  // would advance as cells: one exchange per iteration there (as the solver does).
  const bool all_periodic = topo.periodic_rows && topo.periodic_cols;
  const double c_center = cli.get_double("c-center", 0.2), c_neighbor = cli.get_double("c-neighbor", 0.2);
  // --no-sum-form: per-step evaluation everywhere (bitwise equal to the CPU app).
  const bool sum_form = !cli.flag("no-sum-form") && c_center == c_neighbor;
  int time_block =
      (backend == "mpi-staged" || !all_periodic)
          ? 1
          : int(cli.get_int("time-block", iters > 0 && lw >= 64 && lh >= 64
                                              ? kernels::auto_time_block(lw, lh, int(sizeof(T)), sum_form)
                                              : 1));
  // The time block sets the ghost depth and the exchanges per call: the same on
  // every rank (an uneven decomposition gives ranks different tile sizes).
  time_block = -int(env.max_over_ranks(-double(time_block)));
  const TileGeom g = TileGeom::aligned(lw, lh, std::max(sw / 2, time_block), std::max(sh / 2, time_block),
                                       int(sizeof(T)));
  std::unique_ptr<RcclComm> comm;
  if (backend == "rccl") comm = make_comm(env);

  DeviceBuffer<T> a(g.alloc_elems()), b(g.alloc_elems());
  Stream init_stream;
  MPI_Comm cart = make_cart_comm(topo);

  SolverConfig cfg;
  cfg.backend = backend == "rccl" ? HaloBackend::Rccl : backend == "ipc" ? HaloBackend::Ipc : HaloBackend::Local;
  // Host allgather: the IPC backend's set-up and the solver's collective
  // agreements (time block, opening, sum-form range) without RCCL.
  cfg.bootstrap = [](const std::string& b) { return mpi_allgather_bytes(MPI_COMM_WORLD, b); };
  // IPC: device-initiated halo (each pass pushes its edge bands into the
  // neighbours' tiles) unless --no-direct-halo asks for pack -> put -> unpack.
  // --direct-halo validate (RCCL or IPC, ranks on any GPUs): prepare() checks
  // the device-initiated push bitwise against the backend and times it.
  const std::string direct = cli.get("direct-halo", backend == "ipc" && !cli.flag("no-direct-halo") ? "on" : "off");
  MXS_CHECK(direct == "on" || direct == "off" || direct == "validate",
            "--direct-halo must be on, off or validate, got " << direct);
  cfg.direct = direct == "on" ? DirectHalo::On : direct == "validate" ? DirectHalo::Validate : DirectHalo::Off;
  // Overlap (interior on a forked stream while the halo moves) defaults on only
  // for one-exchange-per-iteration runs: with temporal blocking the exchange is
  // ~5-8% of a super-step and the concurrent thin boundary strips cost more than
  // they hide (docs/PERF.md). Ranks sharing a GPU never overlap by default: their
  // cross-process waits plus the forked branch oversubscribe the GPU's queues and
  // get time-sliced (measured: 3-28 vs ~3000 Gcells/s).
  const bool shared_gpu = dev.shared;
  // Ranks sharing a GPU: each persistent stencil kernel takes its share of the chip.
  kernels::set_gpu_share(dev.sharing);
  cfg.overlap = cli.flag("overlap") || (!cli.flag("no-overlap") && !shared_gpu && time_block == 1);
  cfg.use_graph = !cli.flag("no-graph");
  const std::string opening = cli.flag("halo-last") ? "interior-first" : cli.get("opening", "auto");
  MXS_CHECK(opening == "auto" || opening == "serial" || opening == "interior-first",
            "--opening must be auto, serial or interior-first, got " << opening);
  cfg.opening = opening == "serial" ? Opening::Serial : opening == "interior-first" ? Opening::InteriorFirst : Opening::Auto;
  const std::string steady = cli.get("steady", "auto");
  MXS_CHECK(steady == "auto" || steady == "serial" || steady == "interior-first",
            "--steady must be auto, serial or interior-first, got " << steady);
  cfg.steady = steady == "serial" ? Opening::Serial : steady == "interior-first" ? Opening::InteriorFirst : Opening::Auto;
  cfg.halo_max_ctas = int(cli.get_int("halo-max-ctas", 0));  // RCCL: the halo on a CTA-capped communicator
  cfg.loopback_self = loopback;
  cfg.coeffs = {c_center, c_neighbor, sum_form};
  cfg.time_block = time_block;
  std::unique_ptr<StencilSolver<T>> solver;
  std::unique_ptr<MpiStagedHalo<T>> staged;
  const HaloPlan plan = make_halo_plan(topo, rank, g, true, loopback);
  if (backend == "mpi-staged") {
    staged = std::make_unique<MpiStagedHalo<T>>(plan, cart, !cli.flag("pageable"));
  } else {
    MXS_CHECK(backend == "rccl" || backend == "local" || backend == "ipc", "unknown backend " << backend);
    solver = std::make_unique<StencilSolver<T>>(topo, rank, g, a.get(), b.get(), comm.get(), cfg);
  }

  if (iters == 0) {
    // Reference run: ghosts -1, core = rank id, one exchange, dump before/after.
    kernels::fill<T>(a.get(), g.alloc_elems(), T(-1), init_stream.get());
    kernels::fill_region<T>(a.get(), g.core(), T(rank), init_stream.get());
    init_stream.sync();
    std::ostringstream os;
    std::vector<T> h;
    if (dump) {
      copy_tile_to_host(h, a.get(), g);
      write_dump_header(os, topo, rank, dev.device, lw, lh, sw, sh, "HIP");
      os << "Array" << '\n';
      app::dump_tile(os, h.data(), g);
      os << '\n';
    }
    if (staged) {
      staged->exchange(a.get(), init_stream.get());
      init_stream.sync();
    } else {
      solver->exchange_only();
      solver->synchronize();
    }
    if (dump) {
      copy_tile_to_host(h, a.get(), g);
      os << "Array after exchange" << '\n';
      app::dump_tile(os, h.data(), g);
      std::ofstream f(dump_file_name(topo, rank));
      f << os.str();
    }
  } else {
    kernels::fill<T>(a.get(), g.alloc_elems(), T(0), init_stream.get());
    kernels::fill<T>(b.get(), g.alloc_elems(), T(0), init_stream.get());
    const std::uint64_t seed = std::uint64_t(cli.get_int("seed", 1234));
    const GlobalBlock blk{gx0, gy0, gw, gh};
    std::int64_t start_iter = 0;
    if (cli.has("resume")) {
      std::vector<T> h(size_t(g.alloc_elems()), T(0));
      start_iter = read_grid_file<T>(MPI_COMM_WORLD, cli.get("resume"), h.data(), g, blk).iteration;
      // The zero fills above run on the non-blocking init stream, which the
      // null-stream hipMemcpy does not wait for: order the copy after them.
      MXS_HIP_CHECK(hipMemcpyAsync(a.get(), h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice, init_stream.get()));
      init_stream.sync();
      if (rank == 0) std::cout << "resumed from " << cli.get("resume") << " at iteration " << start_iter << '\n';
    } else {
      kernels::fill_random<T>(a.get(), g, gx0, gy0, gw, seed, T(0), T(1), init_stream.get());
    }
    init_stream.sync();
    T* cur = a.get();
    T* nxt = b.get();
    const FaultSpec fault = parse_fault_spec(cli.get("fault-inject", ""));
    long long it = 0;
    auto steps = [&](long long n) {
      if (solver && !fault.armed()) {
        solver->run(int(n));
        return;
      }
      for (long long i = 0; i < n; ++i) {
        maybe_inject_fault(fault, rank, it++);
        if (solver) {
          solver->run(1);
          continue;
        }
        staged->exchange(cur, init_stream.get());
        kernels::stencil5_rows<T>(cur, nxt, g, 0, lh, cfg.coeffs, init_stream.get());
        std::swap(cur, nxt);
      }
    };
    auto sync = [&]() {
      if (solver) solver->synchronize();
      init_stream.sync();
    };
    const long long warmup = cli.get_int("warmup", 10);
    steps(warmup);
    if (solver && !fault.armed()) solver->prepare(int(iters));  // graphs + first launches, untimed
    sync();
    env.barrier();
    const double t0 = MPI_Wtime();
    steps(iters);
    sync();
    env.barrier();
    const double dt = env.max_over_ranks(MPI_Wtime() - t0);
    if (solver) cur = solver->current();
    if (cli.has("checkpoint")) {
      std::vector<T> h;
      copy_tile_to_host(h, cur, g);
      write_grid_file<T>(MPI_COMM_WORLD, cli.get("checkpoint"), h.data(), g, blk, start_iter + warmup + iters, seed);
    }
    const double gcells = double(gw) * double(gh) * double(iters) / dt / 1e9;
    double checksum = std::nan("");
    const bool want_sum = cli.has("checksum") ? cli.flag("checksum") : (lw * lh <= (index_t(1) << 24));
    if (want_sum) {
      std::vector<T> h;
      copy_tile_to_host(h, cur, g);
      double local = 0;
      for (index_t y = 0; y < lh; ++y)
        for (index_t x = 0; x < lw; ++x) local += double(h[size_t(g.core_offset() + y * g.pitch + x)]);
      checksum = env.sum_over_ranks(local);
    }
    if (rank == 0) {
      std::ostringstream js;
      js << "{\"app\": \"stencil2d\", \"metric\": \"gcells_per_s\", \"value\": " << app::fmt(gcells)
         << ", \"ms_per_iter\": " << app::fmt(dt / double(iters) * 1e3) << ", \"ranks\": " << env.size()
         << ", \"dims\": \"" << topo.rows << "x" << topo.cols << "\", \"global\": \"" << gw << "x" << gh
         << "\", \"dtype\": \"" << (sizeof(T) == 4 ? "f32" : "f64") << "\", \"backend\": \"" << backend
         << "\", \"graph\": \"" << (solver ? solver->graph_status() : std::string("n/a"))
         << "\", \"time_block\": " << time_block << ", \"iters\": " << iters;
      if (solver) {
        js << ", \"interior_first_opening\": " << (solver->halo_last(solver->time_block()) ? "true" : "false");
        if (!solver->opening_choice().empty()) js << ", \"opening_choice\": \"" << solver->opening_choice() << "\"";
        js << ", \"last_opening\": \"" << solver->last_run_opening() << "\"";
        if (!solver->steady_choice().empty()) js << ", \"steady_choice\": \"" << solver->steady_choice() << "\"";
        if (!solver->direct_state().empty()) js << ", \"direct_halo\": \"" << solver->direct_state() << "\"";
      }
      if (want_sum) js << ", \"checksum\": " << app::fmt(checksum);
      js << app::meta_json(device_description(dev.device)) << "}";
      std::cout << "Gcells/s: " << app::fmt(gcells) << '\n';
      if (want_sum) std::cout << "checksum: " << app::fmt(checksum) << '\n';
      std::cout << js.str() << std::endl;
      app::append_json(cli.get("json"), js.str());
    }
  }
  solver.reset();
  staged.reset();
  MPI_Comm_free(&cart);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  MpiEnv env(&argc, &argv);
  Cli cli(argc, argv, {"dump", "no-dump", "non-periodic", "strict-square", "no-overlap", "overlap", "no-graph",
                       "loopback", "pageable", "checksum", "halo-last", "no-sum-form",
                       "no-direct-halo"});
  comm_timeout() = cli.get_double("comm-timeout", 300.0);
  const DeviceBinding dev = bind_device(env, cli.get("bind", "bunch"));
  const int n = env.size();
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
  const auto& pos = cli.positional();
  index_t gw = 0, gh = 0, lw = 16, lh = 16, gx0 = 0, gy0 = 0;
  int sw = 5;
  if (!pos.empty()) lw = lh = std::atoll(pos[0].c_str());
  if (pos.size() >= 2) sw = std::atoi(pos[1].c_str());
  if (cli.has("stencil")) sw = int(cli.get_int("stencil", sw));
  const int sh = int(cli.get_int("stencil-height", sw));
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
  if (cli.get("dtype", "f64") == "f32") return run<float>(env, cli, topo, dev, lw, lh, gx0, gy0, gw, gh, sw, sh);
  return run<double>(env, cli, topo, dev, lw, lh, gx0, gy0, gw, gh, sw, sh);
}
