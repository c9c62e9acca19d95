// _mxs_hip: bindings of the HIP kernels and the native runtime (RCCL
// communicator, halo exchanger, stencil solver, ping-pong).
//
// Buffers cross the boundary as raw device addresses (Python ints, e.g.
// torch.Tensor.data_ptr()) and streams as hipStream_t handles
// (torch.cuda.current_stream().cuda_stream), so the Python side keeps using the
// PyTorch caching allocator while all device work is launched from C++.
// Import torch BEFORE this module: then libamdhip64.so.7 / librccl.so.1 resolve
// to the copies torch already loaded (one HIP runtime per process).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <memory>
#include <stdexcept>
#include <string>

#include "mxs/comm/rccl_comm.hpp"
#include "mxs/core/fault.hpp"
#include "mxs/halo/exchange.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/ipc.hpp"
#include "mxs/runtime/pingpong.hpp"
#include "mxs/runtime/stencil_solver.hpp"

namespace py = pybind11;
using namespace mxs;

namespace {

template <typename T>
T* ptr(std::uintptr_t p) {
  return reinterpret_cast<T*>(p);
}
hipStream_t strm(std::uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

enum class DType { F32, F64 };
DType parse_dtype(const std::string& d) {
  if (d == "f32" || d == "float32" || d == "float") return DType::F32;
  if (d == "f64" || d == "float64" || d == "double") return DType::F64;
  throw std::invalid_argument("unsupported dtype '" + d + "' (use f32 or f64)");
}

// Python callable (bytes -> list[bytes], collective) as the IPC backend's host
// allgather. Only called during construction, with the GIL held.
HostAllgather wrap_allgather(py::object fn) {
  if (fn.is_none()) return {};
  return [fn](const std::string& blob) {
    py::gil_scoped_acquire gil;
    py::list parts = fn(py::bytes(blob));
    std::vector<std::string> out;
    for (auto item : parts) out.push_back(std::string(py::bytes(py::reinterpret_borrow<py::object>(item))));
    return out;
  };
}

kernels::StencilVariant parse_variant(const std::string& v) {
  if (v == "auto") return kernels::StencilVariant::Auto;
  if (v == "roll") return kernels::StencilVariant::RegisterRoll;
  if (v == "lds") return kernels::StencilVariant::LdsTile;
  throw std::invalid_argument("unknown stencil variant '" + v + "' (auto|roll|lds)");
}

kernels::DotReduce parse_reduce(const std::string& r) {
  if (r == "atomic") return kernels::DotReduce::Atomic;
  if (r == "two-pass" || r == "two_pass") return kernels::DotReduce::TwoPass;
  if (r == "single-pass" || r == "single_pass" || r == "gpu") return kernels::DotReduce::SinglePass;
  if (r == "host" || r == "cpu") return kernels::DotReduce::HostPartials;
  if (r == "racy" || r == "no-sync") return kernels::DotReduce::Racy;
  throw std::invalid_argument("unknown reduction '" + r + "'");
}

kernels::BoxWeights make_box(int radius, const std::vector<float>& w) {
  kernels::BoxWeights b;
  b.radius = radius;
  const size_t k = size_t(2 * radius + 1) * size_t(2 * radius + 1);
  if (radius < 1 || radius > kernels::kMaxBoxRadius) throw std::invalid_argument("box radius must be 1 or 2");
  if (w.size() != k) throw std::invalid_argument("box weights must have (2r+1)^2 entries");
  for (size_t i = 0; i < k; ++i) b.w[i] = w[i];
  return b;
}

// Type-erased solver handle so Python sees one class.
struct SolverHandle {
  DType dt;
  std::unique_ptr<StencilSolver<float>> f;
  std::unique_ptr<StencilSolver<double>> d;
  template <typename F>
  auto visit(F&& fn) {
    return dt == DType::F32 ? fn(*f) : fn(*d);
  }
};

struct ExchangerHandle {
  DType dt;
  std::unique_ptr<HaloExchanger<float>> f;
  std::unique_ptr<HaloExchanger<double>> d;
};

}  // namespace

PYBIND11_MODULE(_mxs_hip, m) {
  m.doc() = "mxs HIP kernels (gfx950) and native runtime";

  m.def("device_count", []() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
      (void)hipGetLastError();
      return 0;
    }
    return n;
  });
  m.def("set_device", [](int d) { MXS_HIP_CHECK(hipSetDevice(d)); });
  m.def("device_sync", []() { MXS_HIP_CHECK(hipDeviceSynchronize()); });
  m.def("stream_sync", [](std::uintptr_t s) { MXS_HIP_CHECK(hipStreamSynchronize(strm(s))); });
  m.def("device_arch", [](int d) {
    hipDeviceProp_t p;
    MXS_HIP_CHECK(hipGetDeviceProperties(&p, d));
    return std::string(p.gcnArchName);
  });

  // ------------------------------------------------------------------ kernels
  m.def(
      "fill",
      [](std::uintptr_t p, index_t n, double v, const std::string& dt, std::uintptr_t s) {
        if (parse_dtype(dt) == DType::F32) kernels::fill<float>(ptr<float>(p), n, float(v), strm(s));
        else kernels::fill<double>(ptr<double>(p), n, v, strm(s));
      },
      py::arg("ptr"), py::arg("n"), py::arg("value"), py::arg("dtype"), py::arg("stream") = 0);
  m.def(
      "fill_region",
      [](std::uintptr_t p, const Array2D& r, double v, const std::string& dt, std::uintptr_t s) {
        if (parse_dtype(dt) == DType::F32) kernels::fill_region<float>(ptr<float>(p), r, float(v), strm(s));
        else kernels::fill_region<double>(ptr<double>(p), r, v, strm(s));
      },
      py::arg("ptr"), py::arg("region"), py::arg("value"), py::arg("dtype"), py::arg("stream") = 0);
  m.def(
      "fill_random",
      [](std::uintptr_t p, const TileGeom& g, index_t gx0, index_t gy0, index_t gw, std::uint64_t seed, double lo,
         double hi, const std::string& dt, std::uintptr_t s) {
        if (parse_dtype(dt) == DType::F32)
          kernels::fill_random<float>(ptr<float>(p), g, gx0, gy0, gw, seed, float(lo), float(hi), strm(s));
        else
          kernels::fill_random<double>(ptr<double>(p), g, gx0, gy0, gw, seed, lo, hi, strm(s));
      },
      py::arg("ptr"), py::arg("geom"), py::arg("global_x0"), py::arg("global_y0"), py::arg("global_width"),
      py::arg("seed"), py::arg("lo") = 0.0, py::arg("hi") = 1.0, py::arg("dtype") = "f32", py::arg("stream") = 0);
  m.def(
      "stencil5_rows",
      [](std::uintptr_t in, std::uintptr_t out, const TileGeom& g, index_t r0, index_t r1, double c0, double c1,
         const std::string& dt, std::uintptr_t s, const std::string& variant) {
        kernels::Stencil5Coeffs c{c0, c1};
        const auto v = parse_variant(variant);
        if (parse_dtype(dt) == DType::F32)
          kernels::stencil5_rows<float>(ptr<float>(in), ptr<float>(out), g, r0, r1, c, strm(s), v);
        else
          kernels::stencil5_rows<double>(ptr<double>(in), ptr<double>(out), g, r0, r1, c, strm(s), v);
      },
      py::arg("src"), py::arg("dst"), py::arg("geom"), py::arg("row_begin"), py::arg("row_end"),
      py::arg("c_center") = 0.2, py::arg("c_neighbor") = 0.2, py::arg("dtype") = "f32", py::arg("stream") = 0,
      py::arg("variant") = "auto");
  m.def(
      "auto_time_block",
      [](index_t w, index_t h, const std::string& dt, bool sum_form) {
        return kernels::auto_time_block(w, h, parse_dtype(dt) == DType::F32 ? 4 : 8, sum_form);
      },
      py::arg("width"), py::arg("height"), py::arg("dtype") = "f32", py::arg("sum_form") = true,
      "measured default Jacobi steps per pass / halo exchange for a tile");
  m.attr("MAX_TIME_BLOCK") = kernels::kMaxTimeBlock;
  m.attr("MAX_TIME_BLOCK_DEEP") = kernels::kMaxTimeBlockDeep;
  m.def(
      "last_stencil_dispatch", [] { return std::string(kernels::last_stencil_dispatch()); },
      "kernel form chosen by the most recent stencil launcher (e.g. 'stream_balanced_rot')");
  m.def("device_cu_count", &device_cu_count, "compute units of the current HIP device");
  m.def("set_gpu_share", &kernels::set_gpu_share, py::arg("processes"),
        "processes sharing this GPU: persistent stencil kernels take 1/processes of the chip");
  m.def("gpu_share", &kernels::gpu_share);
  m.def("set_pipe_joint", &kernels::set_pipe_joint, py::arg("on"),
        "joint stage-1 windows in the fp32 two-stage pipeline (default on; bitwise equal output)");
  m.def("pipe_joint", &kernels::pipe_joint);
  m.def("set_pipe_lag1", &kernels::set_pipe_lag1, py::arg("on"),
        "ascending level order in the joint fp32 pipeline where it pays (default on; bitwise equal output)");
  m.def("pipe_lag1", &kernels::pipe_lag1);
  m.def("set_pipe_balanced", &kernels::set_pipe_balanced, py::arg("on"),
        "fill-aware workgroup shares in the pipeline passes (default on; bitwise equal output)");
  m.def("pipe_balanced", &kernels::pipe_balanced_on);
  m.def(
      "absmax",
      [](std::uintptr_t x, index_t n, const std::string& dt) {
        double r = 0;
        if (parse_dtype(dt) == DType::F32) {
          DeviceBuffer<float> o(1);
          kernels::absmax<float>(ptr<float>(x), n, o.get(), nullptr);
          float h = 0;
          MXS_HIP_CHECK(hipMemcpy(&h, o.get(), sizeof(float), hipMemcpyDeviceToHost));
          r = h;
        } else {
          DeviceBuffer<double> o(1);
          kernels::absmax<double>(ptr<double>(x), n, o.get(), nullptr);
          MXS_HIP_CHECK(hipMemcpy(&r, o.get(), sizeof(double), hipMemcpyDeviceToHost));
        }
        return r;
      },
      py::arg("x"), py::arg("n"), py::arg("dtype") = "f32", "max |x[i]| (device reduction; NaN if any is NaN)");
  m.def(
      "stencil5_chunk_pass",
      [](std::uintptr_t in, std::uintptr_t out, const TileGeom& g, int steps, double c0, double c1,
         const std::string& dt, int outer_wgs, std::uintptr_t s, bool sum_form, double range, double lead_frac,
         const std::string& part) -> py::object {
        // One interior-first pass (tests / tuning): the inner and the outer
        // chunk lists of kernels::make_halo_last_schedule as two launches of the
        // chunk-list kernel on one stream. The tables live for the call, so the
        // launches are synchronised before return. part: "both", or "inner" /
        // "outer" alone (timing one set against the one-launch pass).
        MXS_CHECK(part == "both" || part == "inner" || part == "outer", "stencil5_chunk_pass: part both|inner|outer");
        kernels::Stencil5Coeffs c{c0, c1, sum_form, range};
        auto run = [&](auto tag) -> py::object {
          using T = decltype(tag);
          kernels::ChunkPassShape sh;
          if (!kernels::chunk_pass_shape<T>(g, steps, c, &sh) || sh.blocks < 2) return py::none();
          std::vector<std::uint8_t> ghost(size_t(sh.groups), 0);
          for (index_t k = 0; k < sh.groups; ++k) {
            const index_t x0 = k * sh.owg - sh.read_lead;
            ghost[size_t(k)] = (x0 < 0 || x0 + sh.read_span > g.width) ? 1 : 0;
          }
          const auto hl = kernels::make_halo_last_schedule(sh.groups, g.height, sh.blocks, sh.fill, steps, ghost,
                                                           outer_wgs, lead_frac, 0, sh.blocks % kNumXCDs == 0 ? kNumXCDs : 1,
                                                           32);
          DeviceBuffer<kernels::PassChunk> ti(index_t(hl.inner.table.size())), to(index_t(hl.outer.table.size()));
          MXS_HIP_CHECK(hipMemcpy(ti.get(), hl.inner.table.data(), ti.bytes(), hipMemcpyHostToDevice));
          MXS_HIP_CHECK(hipMemcpy(to.get(), hl.outer.table.data(), to.bytes(), hipMemcpyHostToDevice));
          kernels::ChunkPassShape si = sh, so = sh;
          si.blocks = hl.inner.blocks;
          so.blocks = hl.outer.blocks;
          Event e0(true), e1(true);
          e0.record(strm(s));
          if (part != "outer")
            kernels::stencil5_chunk_pass<T>(ptr<T>(in), ptr<T>(out), g, c, si, ti.get(), hl.inner.entries, strm(s));
          if (part != "inner")
            kernels::stencil5_chunk_pass<T>(ptr<T>(in), ptr<T>(out), g, c, so, to.get(), hl.outer.entries, strm(s));
          e1.record(strm(s));
          MXS_HIP_CHECK(hipStreamSynchronize(strm(s)));
          py::dict d;
          d["inner_blocks"] = hl.inner.blocks;
          d["outer_blocks"] = hl.outer.blocks;
          d["check"] = kernels::check_halo_last_schedule(hl, sh.groups, g.height, steps, ghost);
          d["js0"] = sh.js0;
          d["lag1"] = sh.lag1;
          d["fill"] = sh.fill;
          d["band"] = hl.band;
          d["inner_cost"] = hl.inner_cost;
          d["outer_cost"] = hl.outer_cost;
          d["serial_cost"] = hl.serial_cost;
          d["kernel_us"] = double(e1.since(e0)) * 1000.0;
          return d;
        };
        return parse_dtype(dt) == DType::F32 ? run(float{}) : run(double{});
      },
      py::arg("src"), py::arg("dst"), py::arg("geom"), py::arg("steps"), py::arg("c_center") = 0.2,
      py::arg("c_neighbor") = 0.2, py::arg("dtype") = "f32", py::arg("outer_wgs") = 0, py::arg("stream") = 0,
      py::arg("sum_form") = true, py::arg("range") = -1.0, py::arg("lead_frac") = 0.12, py::arg("part") = "both",
      "one interior-first pass (inner + outer chunk lists) over the core of a ghost-ring tile (None: no "
      "chunk-list form for this depth); sum_form / range as for stencil5_tb; lead_frac: the exchange's share "
      "of the pass the schedule assumes; part: both, inner or outer alone");
  m.def("last_pipe_lag1", &kernels::last_pipe_lag1,
        "whether the most recent stencil launch was a pipeline pass in ascending level order");
  m.def(
      "stencil5_tb",
      [](std::uintptr_t in, std::uintptr_t out, const TileGeom& g, int steps, index_t x0, index_t x1, index_t y0,
         index_t y1, double c0, double c1, bool wrap, const std::string& dt, std::uintptr_t s,
         const std::string& variant, bool sum_form, double range) {
        kernels::Stencil5Coeffs c{c0, c1, sum_form, range};
        const kernels::StencilVariant v = parse_variant(variant);
        if (parse_dtype(dt) == DType::F32)
          kernels::stencil5_tb<float>(ptr<float>(in), ptr<float>(out), g, steps, x0, x1, y0, y1, c, wrap, strm(s), v);
        else
          kernels::stencil5_tb<double>(ptr<double>(in), ptr<double>(out), g, steps, x0, x1, y0, y1, c, wrap, strm(s),
                                       v);
      },
      py::arg("src"), py::arg("dst"), py::arg("geom"), py::arg("steps"), py::arg("x0"), py::arg("x1"), py::arg("y0"),
      py::arg("y1"), py::arg("c_center") = 0.2, py::arg("c_neighbor") = 0.2, py::arg("wrap") = false,
      py::arg("dtype") = "f32", py::arg("stream") = 0, py::arg("variant") = "auto", py::arg("sum_form") = true,
      py::arg("range") = -1.0,
      "S Jacobi steps over [x0, x1) x [y0, y1). sum_form: allow the fast forms — the sum form (c_center == "
      "c_neighbor) or the scaled form (unequal, c_neighbor != 0) — within their bounds (kernels::fast_form_safe: "
      "|c_center| + 4 |c_neighbor| <= 1, c_neighbor^S normal, range (4 + |c_center / c_neighbor|)^S < max / 4). "
      "range: a bound on max|u| of the input (< 0: unknown; then only forms growing no faster than the sum form "
      "run fast, under its contract max|u| 5^S < max / 4); otherwise the per-step form");
  m.def(
      "streams_concurrent",
      [](std::uintptr_t a, std::uintptr_t b) { return kernels::streams_concurrent(strm(a), strm(b)); },
      py::arg("a"), py::arg("b"), py::call_guard<py::gil_scoped_release>(),
      "whether work on stream b runs while a kernel on stream a still runs (different hardware queues)");
  m.def(
      "clock_stamp",
      [](std::uintptr_t out, std::uintptr_t s) { kernels::clock_stamp(ptr<unsigned long long>(out), strm(s)); },
      py::arg("out"), py::arg("stream") = 0,
      "kClockStampWgs workgroups write (XCC id, shader clock cycles, wall clock ticks) to out[3b..3b+2] "
      "(int64 device buffer of 3 * clock_stamp_slots())");
  m.def("clock_stamp_slots", [] { return kernels::kClockStampWgs; });
  m.def(
      "wall_clock_rate_khz",
      [] {
        int dev = 0, khz = 0;
        MXS_HIP_CHECK(hipGetDevice(&dev));
        MXS_HIP_CHECK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev));
        return khz;
      },
      "rate of wall_clock64() on the current device (kHz)");
  m.def(
      "spin_delay", [](double us, std::uintptr_t s) { kernels::spin_delay(us, strm(s)); }, py::arg("us"),
      py::arg("stream") = 0, "a single-wave kernel holding `stream` for `us` microseconds (wire-time rehearsal)");
  m.def(
      "stencil5_rect",
      [](std::uintptr_t in, std::uintptr_t out, const TileGeom& g, index_t x0, index_t x1, index_t y0, index_t y1,
         double c0, double c1, const std::string& dt, std::uintptr_t s) {
        kernels::Stencil5Coeffs c{c0, c1};
        if (parse_dtype(dt) == DType::F32)
          kernels::stencil5_rect<float>(ptr<float>(in), ptr<float>(out), g, x0, x1, y0, y1, c, strm(s));
        else
          kernels::stencil5_rect<double>(ptr<double>(in), ptr<double>(out), g, x0, x1, y0, y1, c, strm(s));
      },
      py::arg("src"), py::arg("dst"), py::arg("geom"), py::arg("x0"), py::arg("x1"), py::arg("y0"), py::arg("y1"),
      py::arg("c_center") = 0.2, py::arg("c_neighbor") = 0.2, py::arg("dtype") = "f32", py::arg("stream") = 0);
  m.def(
      "stencil_box",
      [](std::uintptr_t in, std::uintptr_t out, const TileGeom& g, index_t x0, index_t x1, index_t y0, index_t y1,
         int radius, const std::vector<float>& w, const std::string& dt, std::uintptr_t s) {
        const auto b = make_box(radius, w);
        if (parse_dtype(dt) == DType::F32)
          kernels::stencil_box<float>(ptr<float>(in), ptr<float>(out), g, x0, x1, y0, y1, b, strm(s));
        else
          kernels::stencil_box<double>(ptr<double>(in), ptr<double>(out), g, x0, x1, y0, y1, b, strm(s));
      },
      py::arg("src"), py::arg("dst"), py::arg("geom"), py::arg("x0"), py::arg("x1"), py::arg("y0"), py::arg("y1"),
      py::arg("radius"), py::arg("weights"), py::arg("dtype") = "f32", py::arg("stream") = 0);
  m.def("dot_grid_size", [](index_t n) { return kernels::dot_grid_size(n, kernels::kDotBlock); });
  m.def(
      "dot",
      [](std::uintptr_t x, std::uintptr_t y, index_t n, std::uintptr_t out, std::uintptr_t partials,
         std::uintptr_t counter, const std::string& reduce, const std::string& dt, const std::string& acc, int grid,
         std::uintptr_t s) {
        const auto mode = parse_reduce(reduce);
        const DType d = parse_dtype(dt), a = parse_dtype(acc);
        if (d == DType::F32 && a == DType::F32)
          kernels::dot<float, float>(ptr<float>(x), ptr<float>(y), n, ptr<float>(out), ptr<float>(partials),
                                     ptr<unsigned>(counter), mode, grid, strm(s));
        else if (d == DType::F32)
          kernels::dot<float, double>(ptr<float>(x), ptr<float>(y), n, ptr<double>(out), ptr<double>(partials),
                                      ptr<unsigned>(counter), mode, grid, strm(s));
        else if (a == DType::F64)
          kernels::dot<double, double>(ptr<double>(x), ptr<double>(y), n, ptr<double>(out), ptr<double>(partials),
                                       ptr<unsigned>(counter), mode, grid, strm(s));
        else
          throw std::invalid_argument("f64 inputs need an f64 accumulator");
      },
      py::arg("x"), py::arg("y"), py::arg("n"), py::arg("out"), py::arg("partials"), py::arg("counter"),
      py::arg("reduce") = "single-pass", py::arg("dtype") = "f64", py::arg("acc") = "f64", py::arg("grid") = 0,
      py::arg("stream") = 0);

  // ------------------------------------------------------------------ RCCL
  m.def(
      "set_comm_timeout", [](double s) { comm_timeout() = s; }, py::arg("seconds"),
      "communication watchdog: waits on RCCL streams / IPC peers fail after this many seconds (0 = forever)");
  m.def("comm_timeout", [] { return comm_timeout(); });
  m.def("experiments_build", [] { return kExperimentsBuild; },
        "whether this build honours the MXS_* tuning environment knobs (-DMXS_EXPERIMENTS=ON)");
  py::class_<RcclComm>(m, "RcclComm")
      .def(py::init([](py::bytes uid, int nranks, int rank) {
             return std::make_unique<RcclComm>(std::string(uid), nranks, rank);
           }),
           py::arg("unique_id"), py::arg("nranks"), py::arg("rank"), py::call_guard<py::gil_scoped_release>())
      .def_static("make_unique_id", []() { return py::bytes(RcclComm::make_unique_id()); })
      .def_property_readonly("rank", &RcclComm::rank)
      .def_property_readonly("size", &RcclComm::size)
      .def("count", &RcclComm::count, "ranks the communicator spans (ncclCommCount)")
      .def("device", &RcclComm::device, "HIP device of this rank's end (ncclCommCuDevice)")
      .def("healthy",
           [](const RcclComm& c) {
             std::string msg;
             const bool ok = c.healthy(&msg);
             return py::make_tuple(ok, msg);
           })
      .def("abort", &RcclComm::abort, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("aborted", &RcclComm::aborted)
      .def(
          "wait",
          [](const RcclComm& c, std::uintptr_t s, const std::string& what) { c.wait(strm(s), what.c_str()); },
          py::arg("stream") = 0, py::arg("what") = "RCCL stream", py::call_guard<py::gil_scoped_release>(),
          "wait for `stream` under the communication watchdog (set_comm_timeout)")
      .def(
          "allreduce_sum",
          [](const RcclComm& c, std::uintptr_t send, std::uintptr_t recv, size_t count, const std::string& dt,
             std::uintptr_t s) {
            if (parse_dtype(dt) == DType::F32) c.allreduce_sum<float>(ptr<float>(send), ptr<float>(recv), count, strm(s));
            else c.allreduce_sum<double>(ptr<double>(send), ptr<double>(recv), count, strm(s));
          },
          py::arg("send"), py::arg("recv"), py::arg("count"), py::arg("dtype"), py::arg("stream") = 0)
      .def(
          "send_bytes",
          [](const RcclComm& c, std::uintptr_t buf, size_t n, int peer, std::uintptr_t s) {
            c.send<unsigned char>(ptr<unsigned char>(buf), n, peer, strm(s));
          },
          py::arg("buf"), py::arg("nbytes"), py::arg("peer"), py::arg("stream") = 0)
      .def(
          "recv_bytes",
          [](const RcclComm& c, std::uintptr_t buf, size_t n, int peer, std::uintptr_t s) {
            c.recv<unsigned char>(ptr<unsigned char>(buf), n, peer, strm(s));
          },
          py::arg("buf"), py::arg("nbytes"), py::arg("peer"), py::arg("stream") = 0)
      .def("group_start", &RcclComm::group_start)
      .def("group_end", &RcclComm::group_end);

  // ------------------------------------------------------------------ halo
  py::enum_<HaloBackend>(m, "HaloBackend")
      .value("LOCAL", HaloBackend::Local)
      .value("RCCL", HaloBackend::Rccl)
      .value("IPC", HaloBackend::Ipc);
  py::class_<ExchangerHandle>(m, "HaloExchanger")
      .def(py::init([](const HaloPlan& plan, HaloBackend b, const RcclComm* comm, const std::string& dt,
                       py::object bootstrap, int world_size) {
             auto h = std::make_unique<ExchangerHandle>();
             h->dt = parse_dtype(dt);
             HaloBootstrap boot;
             boot.rank = plan.rank;
             boot.world_size = world_size;
             boot.allgather = wrap_allgather(bootstrap);
             if (h->dt == DType::F32) h->f = std::make_unique<HaloExchanger<float>>(plan, b, comm, &boot);
             else h->d = std::make_unique<HaloExchanger<double>>(plan, b, comm, &boot);
             return h;
           }),
           py::arg("plan"), py::arg("backend"), py::arg("comm") = nullptr, py::arg("dtype") = "f32",
           py::arg("bootstrap") = py::none(), py::arg("world_size") = 1, py::keep_alive<1, 4>())
      .def("check", [](const ExchangerHandle& h) { h.dt == DType::F32 ? h.f->check() : h.d->check(); })
      .def(
          "exchange",
          [](ExchangerHandle& h, std::uintptr_t tile, std::uintptr_t s) {
            if (h.dt == DType::F32) h.f->exchange(ptr<float>(tile), strm(s));
            else h.d->exchange(ptr<double>(tile), strm(s));
          },
          py::arg("tile"), py::arg("stream") = 0)
      .def("wire_bytes", [](const ExchangerHandle& h) { return h.dt == DType::F32 ? h.f->wire_bytes() : h.d->wire_bytes(); });

  // ------------------------------------------------------------------ solver
  py::enum_<StencilKind>(m, "StencilKind").value("JACOBI5", StencilKind::Jacobi5).value("BOX", StencilKind::Box);
  py::class_<SolverHandle>(m, "StencilSolver")
      .def(py::init([](const CartTopology& topo, int rank, const TileGeom& tile, std::uintptr_t a, std::uintptr_t b,
                       const RcclComm* comm, const std::string& dt, HaloBackend backend, bool overlap,
                       bool use_graph, bool loopback_self, StencilKind kind, double c0, double c1, int box_radius,
                       const std::vector<float>& box_w, const std::string& variant, bool fuse_periodic, int time_block,
                       py::object bootstrap, int graph_supersteps, bool sum_form, const std::string& direct_halo,
                       double graph_max_superstep_us, const std::string& opening, bool rehearse_peers,
                       double min_gain, int halo_max_ctas, int main_priority, int side_priority,
                       double wire_delay_us, const std::string& direct_engine, const std::string& steady) {
             SolverConfig cfg;
             if (steady == "auto") cfg.steady = Opening::Auto;
             else if (steady == "serial") cfg.steady = Opening::Serial;
             else if (steady == "interior-first") cfg.steady = Opening::InteriorFirst;
             else throw std::invalid_argument("steady must be auto, serial or interior-first, got '" + steady + "'");
             if (direct_engine == "kernel") cfg.direct_engine = PushEngine::Kernel;
             else if (direct_engine == "copy-engine") cfg.direct_engine = PushEngine::CopyEngine;
             else throw std::invalid_argument("direct_engine must be kernel or copy-engine, got '" + direct_engine + "'");
             cfg.main_priority = main_priority;
             cfg.side_priority = side_priority;
             cfg.halo_max_ctas = halo_max_ctas;
             cfg.wire_delay_us = wire_delay_us;
             if (opening == "auto") cfg.opening = Opening::Auto;
             else if (opening == "serial") cfg.opening = Opening::Serial;
             else if (opening == "interior-first") cfg.opening = Opening::InteriorFirst;
             else throw std::invalid_argument("opening must be auto, serial or interior-first, got '" + opening + "'");
             cfg.rehearse_peers = rehearse_peers;
             cfg.min_gain = min_gain;
             cfg.graph_max_superstep_us = graph_max_superstep_us;
             cfg.bootstrap = wrap_allgather(bootstrap);
             cfg.graph_supersteps = graph_supersteps;
             if (direct_halo == "off") cfg.direct = DirectHalo::Off;
             else if (direct_halo == "on") cfg.direct = DirectHalo::On;
             else if (direct_halo == "validate") cfg.direct = DirectHalo::Validate;
             else throw std::invalid_argument("direct_halo must be off, on or validate, got '" + direct_halo + "'");
             cfg.backend = backend;
             cfg.overlap = overlap;
             cfg.use_graph = use_graph;
             cfg.loopback_self = loopback_self;
             cfg.fuse_periodic_self = fuse_periodic;
             cfg.time_block = time_block;
             cfg.kind = kind;
             cfg.coeffs = {c0, c1, sum_form};
             cfg.variant = parse_variant(variant);
             if (kind == StencilKind::Box) cfg.box = make_box(box_radius, box_w);
             auto h = std::make_unique<SolverHandle>();
             h->dt = parse_dtype(dt);
             if (h->dt == DType::F32)
               h->f = std::make_unique<StencilSolver<float>>(topo, rank, tile, ptr<float>(a), ptr<float>(b), comm, cfg);
             else
               h->d = std::make_unique<StencilSolver<double>>(topo, rank, tile, ptr<double>(a), ptr<double>(b), comm,
                                                              cfg);
             return h;
           }),
           py::arg("topo"), py::arg("rank"), py::arg("tile"), py::arg("buf_a"), py::arg("buf_b"),
           py::arg("comm") = nullptr, py::arg("dtype") = "f32", py::arg("backend") = HaloBackend::Local,
           py::arg("overlap") = true, py::arg("use_graph") = true, py::arg("loopback_self") = false,
           py::arg("kind") = StencilKind::Jacobi5, py::arg("c_center") = 0.2, py::arg("c_neighbor") = 0.2,
           py::arg("box_radius") = 1, py::arg("box_weights") = std::vector<float>{}, py::arg("variant") = "auto",
           py::arg("fuse_periodic") = true, py::arg("time_block") = 1, py::arg("bootstrap") = py::none(),
           py::arg("graph_supersteps") = 0, py::arg("sum_form") = true, py::arg("direct_halo") = "off",
           py::arg("graph_max_superstep_us") = 150.0, py::arg("opening") = "auto", py::arg("rehearse_peers") = false,
           py::arg("min_gain") = 0.0, py::arg("halo_max_ctas") = 0, py::arg("main_priority") = -1,
           py::arg("side_priority") = 0, py::arg("wire_delay_us") = 0.0, py::arg("direct_engine") = "kernel",
           py::arg("steady") = "auto",
           py::keep_alive<1, 7>())
      .def("field_changed", [](SolverHandle& h) { h.visit([](auto& s) { s.field_changed(); }); },
           "the caller wrote the field: re-exchange the ghost ring and re-check the sum form's range next run")
      .def(
          "halo_last", [](SolverHandle& h, int S) { return h.visit([S](auto& s) { return s.halo_last(S); }); },
          py::arg("S"), "whether a call's opening super-step of depth S runs interior-first on this rank")
      .def(
          "force_opening",
          [](SolverHandle& h, const std::string& o) {
            const Opening op = o == "serial" ? Opening::Serial
                               : o == "interior-first" ? Opening::InteriorFirst
                               : o == "auto" ? Opening::Auto
                                             : throw std::invalid_argument("opening: auto|serial|interior-first");
            h.visit([op](auto& s) { s.force_opening(op); });
          },
          py::arg("opening"),
          "paired measurements: the opening of the following calls (serial, interior-first, or auto = the one "
          "construction / prepare() chose); collective")
      .def(
          "force_steady",
          [](SolverHandle& h, const std::string& o) {
            const Opening op = o == "serial" ? Opening::Serial
                               : o == "interior-first" ? Opening::InteriorFirst
                               : o == "auto" ? Opening::Auto
                                             : throw std::invalid_argument("steady: auto|serial|interior-first");
            h.visit([op](auto& s) { s.force_steady(op); });
          },
          py::arg("steady"), "paired measurements: the later super-steps' schedule of the following calls")
      .def("multi_rank", [](SolverHandle& h) { return h.visit([](auto& s) { return s.multi_rank(); }); },
           "whether the solver follows the peers' schedule (remote peers or a loopback rehearsal)")
      .def("schedule_times",
           [](SolverHandle& h) {
             return h.visit([](auto& s) {
               py::dict d;
               d["opening"] = s.opening_choice();
               d["reason"] = s.opening_reason();
               d["rule"] = s.opening_rule();
               d["serial_ms"] = s.opening_serial_ms();
               d["interior_first_ms"] = s.opening_halo_last_ms();
               d["serial_iqr_ms"] = s.opening_serial_spread_ms();
               d["ratio"] = s.opening_ratio();
               d["ratio_iqr"] = s.opening_ratio_iqr();
               d["samples"] = s.opening_samples();
               d["outer_wgs"] = s.halo_last_outer_wgs(s.time_block());
               // Paired ratios of the per-round maxima over ranks per candidate
               // outer set, and this rank's own ratios (diagnostics).
               py::list rs, ls;
               for (const auto& c : s.opening_ratio_samples()) rs.append(py::make_tuple(c.first, c.second));
               for (const auto& c : s.opening_local_ratio_samples()) ls.append(py::make_tuple(c.first, c.second));
               d["candidate_ratios"] = rs;
               d["local_candidate_ratios"] = ls;
               d["agreement"] = s.agreement_path();
               d["steady"] = s.steady_choice();
               d["steady_reason"] = s.steady_reason();
               d["lead_us"] = s.opening_lead_us();
               d["lead_pass_us"] = s.opening_pass_us();
               d["lead_phases_us"] = s.opening_lead_phases();  // (exchange end, inner end, outer end)
               return d;
             });
           },
           "prepare()'s opening decision: the median paired ratio of the per-round maxima over ranks, "
           "interior-first / serial, its IQR, and the medians of the maxima (ms; 0 = not measured)")
      .def("direct_state", [](SolverHandle& h) { return h.visit([](auto& s) { return s.direct_state(); }); },
           "direct halo: '' (not configured), on, pending validation, validated: ..., rejected: ...")
      .def("direct_times",
           [](SolverHandle& h) {
             return h.visit([](auto& s) { return py::make_tuple(s.direct_backend_ms(), s.direct_ms()); });
           },
           "validation timings (ms, worst-rank medians): (backend opening, direct opening); 0 = not measured")
      .def(
          "inject_direct_mismatch",
          [](SolverHandle& h, bool on) { h.visit([on](auto& s) { s.inject_direct_mismatch(on); }); },
          py::arg("on") = true, "fault injection: corrupt one received cell of the direct push before validation")
      .def(
          "inject_direct_skip_wait",
          [](SolverHandle& h, bool on) { h.visit([on](auto& s) { s.inject_direct_skip_wait(on); }); },
          py::arg("on") = true, "fault injection: the validation's direct schedule skips its first wait on this rank")
      .def("agreement_path", [](SolverHandle& h) { return h.visit([](auto& s) { return s.agreement_path(); }); },
           "how collective agreements travel: host allgather, rccl all-reduce or none (one rank)")
      .def("barrier_path", [](SolverHandle& h) { return h.visit([](auto& s) { return s.barrier_path(); }); },
           "the device barrier's path ('' before the first barrier): rccl all-reduce, host allgather (...), "
           "or the host allgather as the agreed fallback after an RCCL barrier failed on some rank")
      .def(
          "set_barrier_comm",
          [](SolverHandle& h, const RcclComm* c) { h.visit([c](auto& s) { s.set_barrier_comm(c); }); },
          py::arg("comm"), py::keep_alive<1, 2>(),
          "tests: the device barrier's own RCCL communicator (default: the halo's)")
      .def(
          "inject_barrier_failure",
          [](SolverHandle& h, bool on) { h.visit([on](auto& s) { s.inject_barrier_failure(on); }); },
          py::arg("on") = true, "fault injection: this rank's RCCL barrier probe fails (tests of the fallback)")
      .def("wire_delay_us", [](SolverHandle& h) { return h.visit([](auto& s) { return s.wire_delay_us(); }); },
           "rehearsal wire time added after each RCCL transfer (us)")
      .def("halo_max_ctas", [](SolverHandle& h) { return h.visit([](auto& s) { return s.halo_max_ctas(); }); },
           "CTA cap of the halo's RCCL communicator (0: RCCL's default)")
      .def("halo_comm_note", [](SolverHandle& h) { return h.visit([](auto& s) { return s.halo_comm_note(); }); })
      .def("abort_halo_comm", [](SolverHandle& h) { h.visit([](auto& s) { s.abort_halo_comm(); }); },
           py::call_guard<py::gil_scoped_release>(),
           "abort the halo's own RCCL communicator (halo_max_ctas), e.g. from a watchdog thread")
      .def("stream_note", [](SolverHandle& h) { return h.visit([](auto& s) { return s.stream_note(); }); },
           "the side stream's hardware-queue check (two-stream schedules)")
      .def("last_run_forks", [](SolverHandle& h) { return h.visit([](auto& s) { return s.last_run_forks(); }); })
      .def("last_run_opening", [](SolverHandle& h) { return h.visit([](auto& s) { return s.last_run_opening(); }); },
           "opening of the last run(): interior-first, serial, fresh, fused, direct, overlap or ''")
      .def(
          "inject_stall",
          [](SolverHandle& h, const std::string& phase, double seconds) {
            h.visit([&](auto& s) { s.inject_stall(phase, seconds); });
          },
          py::arg("phase"), py::arg("seconds"),
          "fault injection: sleep `seconds` on entering `phase` (prepare, warm, run, profile_window)")
      .def(
          "profile_window",
          [](SolverHandle& h, int iters) {
            WindowPhases w;
            {
              py::gil_scoped_release nogil;
              w = h.visit([iters](auto& s) { return s.profile_window(iters); });
            }
            py::dict d;
            d["opening"] = w.opening;
            d["exchanges"] = w.exchanges;
            d["host_enqueue_us"] = w.host_enqueue_us;
            d["gpu_span_us"] = w.gpu_span_us;
            d["wall_us"] = w.wall_us;
            d["plain_wall_us"] = w.plain_wall_us;
            py::list ph;
            for (const auto& [name, t0, t1] : w.phases) ph.append(py::make_tuple(name, t0, t1));
            d["phases"] = ph;
            return d;
          },
          py::arg("iters"),
          "collective, state-preserving: one event-timed replica of run(iters)'s opening super-step "
          "(phases: (stream:phase, start us, end us))")
      .def("sum_form_active", [](SolverHandle& h) { return h.visit([](auto& s) { return s.sum_form_active(); }); })
      .def("scaled_form_active",
           [](SolverHandle& h) { return h.visit([](auto& s) { return s.scaled_form_active(); }); })
      .def("sum_form_note", [](SolverHandle& h) { return h.visit([](auto& s) { return s.sum_form_note(); }); })
      .def("last_run_blocks", [](SolverHandle& h) { return h.visit([](auto& s) { return s.last_run_blocks(); }); },
           "(S, count) super-steps the last run() enqueued")
      .def("last_run_exchanges", [](SolverHandle& h) { return h.visit([](auto& s) { return s.last_run_exchanges(); }); },
           "halo exchanges the last run() enqueued (priming included)")
      .def("step", [](SolverHandle& h) { h.visit([](auto& s) { s.step(); }); })
      .def("direct_halo", [](SolverHandle& h) { return h.visit([](auto& s) { return s.direct_halo(); }); },
           "whether halos are pushed tile-to-tile by the device (IPC backend, direct mode)")
      .def("graph_supersteps", [](SolverHandle& h) { return h.visit([](auto& s) { return s.graph_supersteps(); }); })
      .def(
          "run", [](SolverHandle& h, int n) { h.visit([n](auto& s) { s.run(n); }); }, py::arg("iters"),
          py::call_guard<py::gil_scoped_release>())
      .def(
          "prepare", [](SolverHandle& h, int n) { h.visit([n](auto& s) { s.prepare(n); }); }, py::arg("iters"),
          py::call_guard<py::gil_scoped_release>(),
          "capture graphs and launch every kernel shape run(iters) uses, without advancing the state")
      .def(
          "warm", [](SolverHandle& h, int n, int passes) { h.visit([n, passes](auto& s) { s.warm(n, passes); }); },
          py::arg("iters"), py::arg("passes"), py::call_guard<py::gil_scoped_release>(),
          "untimed state-preserving passes of run(iters)'s shapes (sustained clocks before a short window)")
      .def("exchange_only", [](SolverHandle& h) { h.visit([](auto& s) { s.exchange_only(); }); })
      .def("synchronize", [](SolverHandle& h) { h.visit([](auto& s) { s.synchronize(); }); },
           py::call_guard<py::gil_scoped_release>())
      .def("current",
           [](SolverHandle& h) {
             return h.visit([](auto& s) { return reinterpret_cast<std::uintptr_t>(s.current()); });
           })
      .def("main_stream",
           [](SolverHandle& h) {
             return h.visit([](auto& s) { return reinterpret_cast<std::uintptr_t>(s.main_stream()); });
           })
      .def("side_stream",
           [](SolverHandle& h) {
             return h.visit([](auto& s) { return reinterpret_cast<std::uintptr_t>(s.side_stream()); });
           })
      .def("graph_active", [](SolverHandle& h) { return h.visit([](auto& s) { return s.graph_active(); }); })
      .def("graph_status", [](SolverHandle& h) { return h.visit([](auto& s) { return s.graph_status(); }); })
      .def("fused_periodic", [](SolverHandle& h) { return h.visit([](auto& s) { return s.fused_periodic(); }); })
      .def("overlapped", [](SolverHandle& h) { return h.visit([](auto& s) { return s.overlapped(); }); })
      .def("time_block", [](SolverHandle& h) { return h.visit([](auto& s) { return s.time_block(); }); });

  // ------------------------------------------------------------------ ping-pong
  py::enum_<PingPongMode>(m, "PingPongMode")
      .value("BLOCKING", PingPongMode::Blocking)
      .value("ASYNC", PingPongMode::Async)
      .value("OVERLAP", PingPongMode::Overlap)
      .value("BIDIRECTIONAL", PingPongMode::Bidirectional);
  py::enum_<LocalPath>(m, "LocalPath")
      .value("DEVICE_COPY", LocalPath::DeviceCopy)
      .value("PINNED_STAGING", LocalPath::PinnedStaging)
      .value("PAGEABLE_STAGING", LocalPath::PageableStaging);
  py::class_<PingPongStats>(m, "PingPongStats")
      .def_readonly("bytes", &PingPongStats::bytes)
      .def_readonly("reps", &PingPongStats::reps)
      .def_readonly("min_rtt_us", &PingPongStats::min_rtt_us)
      .def_readonly("median_rtt_us", &PingPongStats::median_rtt_us)
      .def_readonly("max_rtt_us", &PingPongStats::max_rtt_us)
      .def_readonly("compute_alone_us", &PingPongStats::compute_alone_us)
      .def_readonly("comm_alone_us", &PingPongStats::comm_alone_us)
      .def_readonly("overlapped_us", &PingPongStats::overlapped_us)
      .def_readonly("verified", &PingPongStats::verified)
      .def("latency_us", &PingPongStats::latency_us)
      .def("bandwidth_gbps", &PingPongStats::bandwidth_gbps)
      .def("bidir_gbps", &PingPongStats::bidir_gbps);
  m.def(
      "pingpong_rccl",
      [](const RcclComm& c, int peer, std::uintptr_t sb, std::uintptr_t rb, size_t bytes, int warmup, int reps,
         PingPongMode mode, std::uintptr_t s) {
        return pingpong_rccl(c, peer, ptr<void>(sb), ptr<void>(rb), bytes, warmup, reps, mode, strm(s));
      },
      py::arg("comm"), py::arg("peer"), py::arg("sendbuf"), py::arg("recvbuf"), py::arg("nbytes"),
      py::arg("warmup") = 5, py::arg("reps") = 20, py::arg("mode") = PingPongMode::Blocking, py::arg("stream") = 0,
      py::call_guard<py::gil_scoped_release>());
  m.def(
      "pingpong_local",
      [](LocalPath p, std::uintptr_t a, std::uintptr_t b, size_t bytes, int warmup, int reps, std::uintptr_t s) {
        return pingpong_local(p, ptr<void>(a), ptr<void>(b), bytes, warmup, reps, strm(s));
      },
      py::arg("path"), py::arg("buf_a"), py::arg("buf_b"), py::arg("nbytes"), py::arg("warmup") = 5,
      py::arg("reps") = 20, py::arg("stream") = 0, py::call_guard<py::gil_scoped_release>());

  // Device-initiated ping-pong over HIP IPC mappings (runtime/ipc.hpp).
  py::class_<IpcMailbox>(m, "IpcMailbox")
      .def(py::init<size_t>(), py::arg("capacity"))
      .def("handle", [](const IpcMailbox& b) { return py::bytes(b.handle()); })
      .def("base", [](const IpcMailbox& b) { return reinterpret_cast<std::uintptr_t>(b.base()); })
      .def("data", [](const IpcMailbox& b) { return reinterpret_cast<std::uintptr_t>(b.data()); })
      .def_property_readonly("capacity", &IpcMailbox::capacity);
  py::class_<IpcPeerMailbox>(m, "IpcPeerMailbox")
      .def(py::init([](py::bytes h) { return new IpcPeerMailbox(std::string(h)); }), py::arg("handle"))
      .def("base", [](const IpcPeerMailbox& b) { return reinterpret_cast<std::uintptr_t>(b.base()); });
  m.def(
      "pingpong_ipc",
      [](const IpcMailbox& mine, std::uintptr_t peer_base, std::uintptr_t src, bool ping, size_t bytes, int warmup,
         int reps, int workgroups, double timeout_s, std::uintptr_t s) {
        IpcPingPongConfig cfg;
        cfg.bytes = bytes;
        cfg.warmup = warmup;
        cfg.reps = reps;
        cfg.workgroups = workgroups;
        cfg.timeout_s = timeout_s;
        return pingpong_ipc(mine, ptr<unsigned char>(peer_base), ptr<void>(src), ping, cfg, strm(s));
      },
      py::arg("mailbox"), py::arg("peer_base"), py::arg("src"), py::arg("ping"), py::arg("nbytes"),
      py::arg("warmup") = 5, py::arg("reps") = 50, py::arg("workgroups") = 0, py::arg("timeout_s") = 20.0,
      py::arg("stream") = 0, py::call_guard<py::gil_scoped_release>());
  m.def("pingpong_ipc_loopback", &pingpong_ipc_loopback, py::arg("nbytes"), py::arg("warmup") = 5,
        py::arg("reps") = 50, py::arg("workgroups") = 0, py::call_guard<py::gil_scoped_release>());
  // Copy-engine ping-pong (SDMA copies into the peer's IPC-mapped mailbox).
  m.def(
      "pingpong_peer_copy",
      [](const IpcMailbox& mine, std::uintptr_t peer_base, std::uintptr_t src, bool ping, size_t bytes, int warmup,
         int reps, PingPongMode mode, double timeout_s, std::uintptr_t s) {
        PeerCopyConfig cfg;
        cfg.bytes = bytes;
        cfg.warmup = warmup;
        cfg.reps = reps;
        cfg.mode = mode;
        cfg.timeout_s = timeout_s;
        return pingpong_peer_copy(mine, ptr<unsigned char>(peer_base), ptr<void>(src), ping, cfg, strm(s));
      },
      py::arg("mailbox"), py::arg("peer_base"), py::arg("src"), py::arg("ping"), py::arg("nbytes"),
      py::arg("warmup") = 3, py::arg("reps") = 20, py::arg("mode") = PingPongMode::Async, py::arg("timeout_s") = 20.0,
      py::arg("stream") = 0, py::call_guard<py::gil_scoped_release>());
  m.def("pingpong_peer_copy_local", &pingpong_peer_copy_local, py::arg("nbytes"), py::arg("warmup") = 3,
        py::arg("reps") = 20, py::arg("dev_a") = 0, py::arg("dev_b") = 0, py::call_guard<py::gil_scoped_release>(),
        "one process: the copy-engine protocol between two local mailboxes (dev_a != dev_b: hipMemcpyPeerAsync)");
}
