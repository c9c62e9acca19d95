// Halo pack / unpack timing on one tile (the S-deep exchange of the
// time-blocked solver): the whole batch and its parts (row bands, column
// bands, corners) at several grid sizes, so the cost of a launch can be split
// into its segments.
//   halo_pack_bench [W H S reps]      (default: the 8-GPU tile, 16384 8192 20 400)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "mxs/core/error.hpp"
#include "mxs/halo/exchange.hpp"
#include "mxs/halo/plan.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/hip_utils.hpp"

using namespace mxs;

namespace {

kernels::Copy2DBatch subset(const kernels::Copy2DBatch& b, int S, const std::string& which) {
  kernels::Copy2DBatch o;
  for (int i = 0; i < b.n; ++i) {
    const auto& op = b.op[i];
    const bool rows = op.height == S && op.width > S, cols = op.width == S && op.height > S;
    const bool corner = op.width == S && op.height == S;
    if (which == "all" || (which == "rows" && rows) || (which == "cols" && cols) || (which == "corners" && corner))
      o.op[o.n++] = op;
  }
  return o;
}

double bytes_of(const kernels::Copy2DBatch& b) {
  double n = 0;
  for (int i = 0; i < b.n; ++i) n += double(b.op[i].width) * double(b.op[i].height);
  return n * sizeof(float) * 2;  // read + write
}

}  // namespace

int main(int argc, char** argv) {
  const index_t W = argc > 1 ? std::atoll(argv[1]) : 16384, H = argc > 2 ? std::atoll(argv[2]) : 8192;
  const int S = argc > 3 ? std::atoi(argv[3]) : 20, reps = argc > 4 ? std::atoi(argv[4]) : 400;
  const TileGeom g = TileGeom::aligned(W, H, S, S, int(sizeof(float)));
  // 1x1 periodic grid with every neighbour routed as a message to itself: the
  // pack and unpack programs of an 8-neighbour rank.
  const HaloPlan plan = make_halo_plan(CartTopology(1, 1), 0, g, true, true);
  const HaloCopyPrograms progs = build_halo_copy_programs(plan);
  DeviceBuffer<float> tile(g.alloc_elems()), send(plan.send_elems), recv(plan.recv_elems);
  MXS_HIP_CHECK(hipMemset(tile.get(), 0, g.alloc_elems() * sizeof(float)));
  MXS_HIP_CHECK(hipMemset(send.get(), 0, plan.send_elems * sizeof(float)));
  MXS_HIP_CHECK(hipMemset(recv.get(), 0, plan.recv_elems * sizeof(float)));
  Stream st;
  Event e0(true), e1(true);
  std::printf("{\"tile\": \"%lldx%lld\", \"S\": %d, \"pack_ops\": %d, \"unpack_ops\": %d}\n", (long long)W, (long long)H,
              S, progs.pack.n, progs.unpack.n);
  for (const char* side : {"pack", "unpack"}) {
    const kernels::Copy2DBatch& full = std::string(side) == "pack" ? progs.pack : progs.unpack;
    for (const char* which : {"all", "rows", "cols", "corners"}) {
      const kernels::Copy2DBatch b = subset(full, S, which);
      if (b.n == 0) continue;
      for (int gx : {0, 16, 32, 64, 128, 256, 512}) {
        for (int w = 0; w < 20; ++w) kernels::copy2d_batch<float>(tile.get(), send.get(), recv.get(), b, st.get(), gx);
        e0.record(st.get());
        for (int r = 0; r < reps; ++r)
          kernels::copy2d_batch<float>(tile.get(), send.get(), recv.get(), b, st.get(), gx);
        e1.record(st.get());
        st.sync();
        const double us = double(e1.since(e0)) * 1e3 / reps;
        std::printf("{\"side\": \"%s\", \"segments\": \"%s\", \"ops\": %d, \"grid_x\": %d, \"us\": %.2f, "
                    "\"tb_s\": %.2f}\n",
                    side, which, b.n, gx, us, bytes_of(b) / (us * 1e-6) / 1e12);
      }
    }
  }
  return 0;
}
