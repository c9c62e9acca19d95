// dot — parallel dot product over MPI ranks, one GPU per rank.
// Reference: mpicuda2.cu / mpicuda3.cu / mpicuda4.cu (2^28 floats, per-rank GPU partial,
// MPI_Reduce to rank 0, clock() timing) and mpicuda2.cpp (2^30 doubles).
//
//   mpiexec -n 8 dot --n 1073741824 --dtype f64 --reduce single-pass   # BASELINE config
//   mpiexec -n 4 dot                                                   # mpicuda defaults (2^28 f32)
//
// --reduce   atomic (mpicuda2/3 default kernel) | two-pass | single-pass (mpicuda4 -DREDUCE_GPU)
//            | host (-DREDUCE_CPU: per-block partials summed on the host) | racy (-DNO_SYNC demo)
// --acc      f64 (default) | f32 (reproduces the reference's float accumulation)
// --allreduce rccl (device ncclAllReduce) | mpi (host MPI_Reduce, the reference) | auto
// --device   gpu | cpu,  --bind bunch | rrobin (-DMPI_RROBIN_),  --quiet (-DNO_LOG),
// --include-alloc-time (time allocation + H2D too, the reference's default), --reps N,
// --grid G (workgroups of the reduction kernel; default from the device CU count)
#include <mpi.h>

#include <algorithm>
#include <iostream>
#include <memory>
#include <sstream>
#include <vector>

#include "app_common.hpp"
#include "mxs/comm/mpi_env.hpp"
#include "mxs/comm/rccl_comm.hpp"
#include "mxs/core/cli.hpp"
#include "mxs/core/device.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/hip_utils.hpp"

using namespace mxs;

namespace {

kernels::DotReduce parse_reduce(const std::string& r) {
  if (r == "atomic") return kernels::DotReduce::Atomic;
  if (r == "two-pass") return kernels::DotReduce::TwoPass;
  if (r == "host" || r == "cpu") return kernels::DotReduce::HostPartials;
  if (r == "racy" || r == "no-sync") return kernels::DotReduce::Racy;
  return kernels::DotReduce::SinglePass;
}

template <typename T, typename Acc>
int run(MpiEnv& env, const Cli& cli, index_t n_global) {
  const int rank = env.rank(), size = env.size();
  const index_t n = block_split(n_global, size, rank).len;
  const bool quiet = cli.flag("quiet");
  const bool gpu = cli.get("device", "gpu") == "gpu";
  const int reps = std::max(1, int(cli.get_int("reps", 5)));
  const auto mode = parse_reduce(cli.get("reduce", "single-pass"));
  std::vector<T> hx(size_t(n), T(1)), hy(size_t(n), T(1));  // reference: v1 = v2 = 1
  double best = 1e300, result = 0, partial = 0;
  int device_used = -1;
  int grid_used = 0;
  if (!gpu) {
    for (int r = 0; r < reps; ++r) {
      env.barrier();
      const double t0 = MPI_Wtime();
      Acc p = Acc(0);
      for (index_t i = 0; i < n; ++i) p += Acc(hx[size_t(i)]) * Acc(hy[size_t(i)]);
      partial = double(p);
      MXS_MPI_CHECK(MPI_Reduce(&partial, &result, 1, MPI_DOUBLE, MPI_SUM, 0, MPI_COMM_WORLD));
      best = std::min(best, env.max_over_ranks(MPI_Wtime() - t0));
    }
  } else {
    const DeviceBinding dev = bind_device(env, cli.get("bind", "bunch"));
    device_used = dev.device;
    if (!quiet) {
      std::ostringstream os;
      os << env.processor_name() << " - rank: " << rank << "\tGPU: " << dev.device << '\n';
      std::cout << os.str() << std::flush;
    }
    std::string ar = cli.get("allreduce", "auto");
    if (ar == "auto") ar = (size > 1 && !dev.shared) ? "rccl" : "mpi";
    std::unique_ptr<RcclComm> comm;
    if (ar == "rccl" && mode != kernels::DotReduce::HostPartials) {
      std::string uid = rank == 0 ? RcclComm::make_unique_id() : std::string(sizeof(ncclUniqueId), '\0');
      MXS_MPI_CHECK(MPI_Bcast(&uid[0], int(uid.size()), MPI_BYTE, 0, MPI_COMM_WORLD));
      comm = std::make_unique<RcclComm>(uid, size, rank);
    }
    const bool include_alloc = cli.flag("include-alloc-time");
    const int grid = cli.has("grid") ? int(cli.get_int("grid", 0)) : kernels::dot_grid_size(n, kernels::kDotBlock);
    MXS_CHECK(grid > 0, "--grid must be positive");
    grid_used = grid;
    Stream s;
    DeviceBuffer<T> x, y;
    // Reduction workspaces: allocated once, outside every timed region.
    DeviceBuffer<Acc> partials(grid), out(1), total(1);
    DeviceBuffer<unsigned> counter(4);
    for (int r = 0; r < reps; ++r) {
      env.barrier();
      double t0 = MPI_Wtime();
      if (include_alloc || r == 0) {
        x.reset(n);
        y.reset(n);
        MXS_HIP_CHECK(hipMemcpyAsync(x.get(), hx.data(), x.bytes(), hipMemcpyHostToDevice, s.get()));
        MXS_HIP_CHECK(hipMemcpyAsync(y.get(), hy.data(), y.bytes(), hipMemcpyHostToDevice, s.get()));
        s.sync();
      }
      if (!include_alloc) {  // -DNO_GPU_MALLOC_TIME: time the resident-data reduction only
        env.barrier();
        t0 = MPI_Wtime();
      }
      kernels::dot<T, Acc>(x.get(), y.get(), n, out.get(), partials.get(), counter.get(), mode, grid, s.get());
      if (mode == kernels::DotReduce::HostPartials) {
        std::vector<Acc> hp(static_cast<size_t>(grid));
        MXS_HIP_CHECK(hipMemcpyAsync(hp.data(), partials.get(), hp.size() * sizeof(Acc), hipMemcpyDeviceToHost,
                                     s.get()));
        s.sync();
        double acc = 0;  // f64 host sum (the reference used std::accumulate(..., 0.f), Q10)
        for (Acc v : hp) acc += double(v);
        partial = acc;
      } else {
        Acc p = Acc(0), t = Acc(0);
        if (comm) comm->allreduce_sum<Acc>(out.get(), total.get(), 1, s.get());
        MXS_HIP_CHECK(hipMemcpyAsync(&p, out.get(), sizeof(Acc), hipMemcpyDeviceToHost, s.get()));
        if (comm) MXS_HIP_CHECK(hipMemcpyAsync(&t, total.get(), sizeof(Acc), hipMemcpyDeviceToHost, s.get()));
        s.sync();
        partial = double(p);
        result = double(t);
      }
      if (!comm) MXS_MPI_CHECK(MPI_Reduce(&partial, &result, 1, MPI_DOUBLE, MPI_SUM, 0, MPI_COMM_WORLD));
      best = std::min(best, env.max_over_ranks(MPI_Wtime() - t0));
    }
  }
  if (!quiet) {
    std::ostringstream os;
    os << env.processor_name() << " - rank: " << rank << " partial dot: " << partial << '\n';
    std::cout << os.str() << std::flush;
  }
  env.barrier();  // the partial lines go out before the result (mpiexec still may interleave them)
  if (rank == 0) {
    std::ostringstream res;  // one write: the result line cannot be split by another rank's output
    res << "dot product result: " << result << '\n' << "time: " << best << "s\n";
    std::cout << res.str() << std::flush;
    std::ostringstream js;
    js << "{\"app\": \"dot\", \"n\": " << n_global << ", \"dtype\": \"" << (sizeof(T) == 4 ? "f32" : "f64")
       << "\", \"reduce\": \"" << cli.get("reduce", "single-pass") << "\", \"ranks\": " << size
       << ", \"device\": \"" << (gpu ? "gpu" : "cpu") << "\", \"result\": " << app::fmt(result)
       << ", \"seconds\": " << app::fmt(best) << ", \"grid\": " << grid_used
       << ", \"gbytes_per_s\": " << app::fmt(2.0 * double(n_global) * sizeof(T) / best / 1e9)
       << app::meta_json(gpu ? device_description(device_used) : std::string("cpu")) << "}";
    if (!quiet) std::cout << js.str() << std::endl;
    app::append_json(cli.get("json"), js.str());
  }
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  MpiEnv env(&argc, &argv);
  Cli cli(argc, argv, {"quiet", "include-alloc-time"});
  const index_t n = index_t(cli.get_int("n", index_t(1) << 28));
  const std::string dt = cli.get("dtype", "f32"), acc = cli.get("acc", "f64");
  if (dt == "f64") return run<double, double>(env, cli, n);
  if (acc == "f32") return run<float, float>(env, cli, n);
  return run<float, double>(env, cli, n);
}
