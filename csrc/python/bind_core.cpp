// _mxs_core: host-only bindings of the layout / region / topology / halo-plan
// library (no HIP, no MPI), so CPU-only tests and the gloo halo backend share
// exactly the plan the GPU and MPI backends execute.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <sstream>

#include "mxs/core/error.hpp"
#include "mxs/grid/layout.hpp"
#include "mxs/grid/regions.hpp"
#include "mxs/halo/plan.hpp"
#include "mxs/kernels/chunk_schedule.hpp"
#include "mxs/runtime/decision.hpp"
#include "mxs/topo/cart.hpp"

namespace py = pybind11;
using namespace mxs;

PYBIND11_MODULE(_mxs_core, m) {
  m.doc() = "mxs host-side core: layouts, regions, Cartesian topology, halo plans";

  py::class_<Array2D>(m, "Array2D")
      .def(py::init<index_t, index_t, index_t, index_t, index_t>(), py::arg("width"), py::arg("height"),
           py::arg("row_stride"), py::arg("x_offset") = 0, py::arg("y_offset") = 0)
      .def_readwrite("width", &Array2D::width)
      .def_readwrite("height", &Array2D::height)
      .def_readwrite("x_offset", &Array2D::x_offset)
      .def_readwrite("y_offset", &Array2D::y_offset)
      .def_readwrite("row_stride", &Array2D::row_stride)
      .def("size", &Array2D::size)
      .def("index", &Array2D::index)
      .def("__eq__", [](const Array2D& a, const Array2D& b) { return a == b; })
      .def("__str__", [](const Array2D& a) {
        std::ostringstream os;
        os << a;
        return os.str();
      })
      .def("__repr__", [](const Array2D& a) {
        std::ostringstream os;
        os << "Array2D(" << a << ", stride: " << a.row_stride << ")";
        return os.str();
      });

  py::class_<TileGeom>(m, "TileGeom")
      .def(py::init<>())
      .def_readwrite("width", &TileGeom::width)
      .def_readwrite("height", &TileGeom::height)
      .def_readwrite("halo_x", &TileGeom::halo_x)
      .def_readwrite("halo_y", &TileGeom::halo_y)
      .def_readwrite("pitch", &TileGeom::pitch)
      .def_readwrite("x_origin", &TileGeom::x_origin)
      .def("total_width", &TileGeom::total_width)
      .def("total_height", &TileGeom::total_height)
      .def("alloc_elems", &TileGeom::alloc_elems)
      .def("full", &TileGeom::full)
      .def("core", &TileGeom::core)
      .def("core_offset", &TileGeom::core_offset)
      .def_static("compact", &TileGeom::compact, py::arg("width"), py::arg("height"), py::arg("halo_x"),
                  py::arg("halo_y"))
      .def_static("aligned", &TileGeom::aligned, py::arg("width"), py::arg("height"), py::arg("halo_x"),
                  py::arg("halo_y"), py::arg("elem_bytes"), py::arg("align_bytes") = 16,
                  py::arg("pitch_align_bytes") = 256)
      .def("__eq__", [](const TileGeom& a, const TileGeom& b) { return a == b; })
      .def("__repr__", [](const TileGeom& g) {
        std::ostringstream os;
        os << "TileGeom(width=" << g.width << ", height=" << g.height << ", halo=(" << g.halo_x << ", "
           << g.halo_y << "), pitch=" << g.pitch << ", x_origin=" << g.x_origin << ")";
        return os.str();
      });

  py::enum_<RegionID>(m, "RegionID")
      .value("TOP_LEFT", TOP_LEFT)
      .value("TOP_CENTER", TOP_CENTER)
      .value("TOP_RIGHT", TOP_RIGHT)
      .value("CENTER_LEFT", CENTER_LEFT)
      .value("CENTER", CENTER)
      .value("CENTER_RIGHT", CENTER_RIGHT)
      .value("BOTTOM_LEFT", BOTTOM_LEFT)
      .value("BOTTOM_CENTER", BOTTOM_CENTER)
      .value("BOTTOM_RIGHT", BOTTOM_RIGHT)
      .value("TOP", TOP)
      .value("LEFT", LEFT)
      .value("BOTTOM", BOTTOM)
      .value("RIGHT", RIGHT);
  m.def("region_name", [](RegionID r) { return std::string(region_name(r)); });
  m.def("sub_array_region", &sub_array_region, py::arg("grid"), py::arg("stencil_width"),
        py::arg("stencil_height"), py::arg("region"));
  m.def("send_region", &send_region);
  m.def("recv_region", &recv_region);
  m.attr("NUM_DIRS") = kNumDirs;
  m.def("dir_offset", [](int d) {
    auto o = dir_offset(d);
    return py::make_tuple(o.dx, o.dy);
  });
  m.def("dir_opposite", &dir_opposite);
  m.def("dir_name", [](int d) { return std::string(dir_name(d)); });
  m.def("dir_is_corner", &dir_is_corner);
  m.def("reference_tag", &reference_tag);

  m.attr("PROC_NULL") = kProcNull;
  py::class_<CartTopology>(m, "CartTopology")
      .def(py::init<int, int, bool, bool>(), py::arg("rows"), py::arg("cols"), py::arg("periodic_rows") = true,
           py::arg("periodic_cols") = true)
      .def_readonly("rows", &CartTopology::rows)
      .def_readonly("cols", &CartTopology::cols)
      .def_readonly("periodic_rows", &CartTopology::periodic_rows)
      .def_readonly("periodic_cols", &CartTopology::periodic_cols)
      .def("size", &CartTopology::size)
      .def("coords", [](const CartTopology& t, int r) {
        auto c = t.coords(r);
        return py::make_tuple(c[0], c[1]);
      })
      .def("rank_of", &CartTopology::rank_of)
      .def("shift", &CartTopology::shift, py::arg("rank"), py::arg("dx"), py::arg("dy"))
      .def("neighbor", &CartTopology::neighbor)
      .def("cart_shift", [](const CartTopology& t, int rank, int dim, int disp) {
        auto s = t.cart_shift(rank, dim, disp);
        return py::make_tuple(s[0], s[1]);
      })
      .def("grid_text", [](const CartTopology& t) {
        std::ostringstream os;
        print_cartesian_grid(os, t);
        return os.str();
      });
  m.def("dims_create", [](int n) {
    auto d = dims_create(n);
    return py::make_tuple(d[0], d[1]);
  });
  m.def("block_split", [](index_t n, int p, int i) {
    auto b = block_split(n, p, i);
    return py::make_tuple(b.start, b.len);
  });

  py::class_<HaloSegment>(m, "HaloSegment")
      .def_readonly("dir", &HaloSegment::dir)
      .def_readonly("region", &HaloSegment::region)
      .def_readonly("offset", &HaloSegment::offset);
  py::class_<HaloMessage>(m, "HaloMessage")
      .def_readonly("peer", &HaloMessage::peer)
      .def_readonly("offset", &HaloMessage::offset)
      .def_readonly("count", &HaloMessage::count)
      .def_readonly("segments", &HaloMessage::segments);
  py::class_<HaloCopy>(m, "HaloCopy")
      .def_readonly("dir", &HaloCopy::dir)
      .def_readonly("src", &HaloCopy::src)
      .def_readonly("dst", &HaloCopy::dst);
  py::class_<HaloPlan>(m, "HaloPlan")
      .def_readonly("tile", &HaloPlan::tile)
      .def_readonly("rank", &HaloPlan::rank)
      .def_readonly("corners", &HaloPlan::corners)
      .def_readonly("sends", &HaloPlan::sends)
      .def_readonly("recvs", &HaloPlan::recvs)
      .def_readonly("self_copies", &HaloPlan::self_copies)
      .def_readonly("send_elems", &HaloPlan::send_elems)
      .def_readonly("recv_elems", &HaloPlan::recv_elems);
  m.def("make_halo_plan", &make_halo_plan, py::arg("topo"), py::arg("rank"), py::arg("tile"),
        py::arg("corners") = true, py::arg("loopback_self") = false);
  m.def(
      "paired_decision",
      [](std::vector<double> ratios, double min_gain) {
        const int n = int(ratios.size());
        const auto [med, iqr] = median_iqr(ratios);
        py::dict d;
        d["median"] = med;
        d["iqr"] = iqr;
        d["notch"] = median_notch(med, iqr, n);
        d["win"] = paired_win(med, iqr, n, min_gain);
        return d;
      },
      py::arg("ratios"), py::arg("min_gain") = 0.0,
      "the solver's opening / direct-halo rule on per-round ratios candidate / baseline (runtime/decision.hpp)");
  m.def(
      "opening_rule",
      [](double lead_frac) { return opening_rule(lead_frac) == WinRule::Median ? "median" : "notch"; },
      py::arg("lead_frac"),
      "the opening decision's rule for a measured exchange lead / pass: median (a tie goes to interior-first) "
      "or notch");
  m.def(
      "opening_decision",
      [](const std::vector<std::vector<double>>& serial, const std::vector<std::vector<std::vector<double>>>& cands,
         double min_gain, const std::string& rule) {
        // serial[rank][round], cands[rank][candidate][round]: what every rank timed.
        // The solver agrees the element-wise max (one vector per rank), then decides.
        MXS_CHECK(!serial.empty() && serial.size() == cands.size(), "one serial and one candidate set per rank");
        const size_t nr = serial[0].size(), nc = cands[0].size();
        std::vector<std::vector<double>> flat(serial.size());
        for (size_t r = 0; r < serial.size(); ++r) {
          MXS_CHECK(serial[r].size() == nr && cands[r].size() == nc, "ranks must time the same rounds and slots");
          flat[r] = serial[r];
          for (const auto& c : cands[r]) {
            MXS_CHECK(c.size() == nr, "ranks must time the same rounds");
            flat[r].insert(flat[r].end(), c.begin(), c.end());
          }
        }
        const std::vector<double> v = elementwise_max(flat);
        std::vector<std::vector<double>> cm(nc);
        for (size_t c = 0; c < nc; ++c) cm[c].assign(v.begin() + (1 + c) * nr, v.begin() + (2 + c) * nr);
        MXS_CHECK(rule == "median" || rule == "notch", "rule: median (the opening) or notch");
        const RoundDecision d = decide_on_maxima(std::vector<double>(v.begin(), v.begin() + nr), cm, min_gain,
                                                 rule == "median" ? WinRule::Median : WinRule::Notch);
        py::dict out;
        out["best"] = d.best;
        out["win"] = d.win;
        out["ratio"] = d.ratio;
        out["ratio_iqr"] = d.ratio_iqr;
        out["notch"] = d.notch;
        out["serial_ms"] = d.baseline_ms;
        out["candidate_ms"] = d.candidate_ms;
        out["ratios"] = d.ratios;
        return out;
      },
      py::arg("serial"), py::arg("candidates"), py::arg("min_gain") = 0.0, py::arg("rule") = "median",
      "StencilSolver::choose_opening's collective rule: per-round maxima over ranks, paired ratios of the maxima, "
      "the lowest notch among candidates, which wins when its median ratio is <= 1 - min_gain (rule 'median', the "
      "opening) or its notch is below it (rule 'notch', the steady and direct-halo decisions) "
      "(runtime/decision.hpp); missing slots: kMissingSample");
  m.attr("MISSING_SAMPLE") = kMissingSample;
  m.def("balanced_starts", &kernels::balanced_starts, py::arg("groups"), py::arg("rows"), py::arg("blocks"),
        py::arg("fill"), "fill-aware linear starts of the pipeline workgroups' shares (blocks + 1 entries)");
  // Interior-first (halo-last) schedule of the multi-GPU opening super-step.
  m.def(
      "halo_last_schedule",
      [](std::int64_t groups, std::int64_t rows, int blocks, std::int64_t fill, std::int64_t depth,
         std::vector<std::uint8_t> ghost, int outer_wgs, double lead_frac, std::int64_t band_rows, int granule, int min_outer) {
        const auto h = kernels::make_halo_last_schedule(groups, rows, blocks, fill, depth, ghost, outer_wgs, lead_frac,
                                                        band_rows, granule, min_outer);
        auto lists = [](const kernels::ChunkSchedule& s) {
          py::list table;
          for (int w = 0; w < s.blocks; ++w) {
            py::list l;
            for (int e = 0; e < s.entries; ++e) {
              const auto& c = s.at(w, e);
              if (c.r1 > c.r0) l.append(py::make_tuple(c.group, c.r0, c.r1));
            }
            table.append(l);
          }
          return table;
        };
        py::dict d;
        d["inner"] = lists(h.inner);
        d["outer"] = lists(h.outer);
        d["hf"] = h.hf;
        d["inner_cost"] = h.inner_cost;
        d["outer_cost"] = h.outer_cost;
        d["serial_cost"] = h.serial_cost;
        d["moved_rows"] = h.moved_rows;
        d["band"] = h.band;
        d["check"] = kernels::check_halo_last_schedule(h, groups, rows, depth, ghost);
        return d;
      },
      py::arg("groups"), py::arg("rows"), py::arg("blocks"), py::arg("fill"), py::arg("depth"), py::arg("ghost"),
      py::arg("outer_wgs") = 0, py::arg("lead_frac") = 0.12, py::arg("band_rows") = 0, py::arg("granule") = 1,
      py::arg("min_outer") = 1,
      "inner / outer chunk lists (group, r0, r1) of the interior-first pass + the check ('' = ok)");
}
