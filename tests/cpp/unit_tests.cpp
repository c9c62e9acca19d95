// Host-only unit tests of the C++ core ("Unit tests"): region
// algebra, accessor indexing, Cartesian neighbour tables, halo-plan
// aggregation/ordering, the collective decision statistics and the
// interior-first chunk schedule. Run by ctest and by tests/test_cpp_unit.py
// (and under host ASan/UBSan by scripts/cpu_sanitize.sh).
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <set>
#include <sstream>
#include <string>

#include "mxs/grid/layout.hpp"
#include "mxs/grid/print.hpp"
#include "mxs/grid/regions.hpp"
#include "mxs/halo/plan.hpp"
#include "mxs/kernels/chunk_schedule.hpp"
#include "mxs/runtime/decision.hpp"
#include "mxs/topo/cart.hpp"

using namespace mxs;

static int g_failures = 0;
#define EXPECT(cond)                                                    \
  do {                                                                  \
    if (!(cond)) {                                                      \
      std::fprintf(stderr, "%s:%d: EXPECT failed: %s\n", __FILE__, __LINE__, #cond); \
      ++g_failures;                                                     \
    }                                                                   \
  } while (0)

static std::string str(const Array2D& a) {
  std::ostringstream os;
  os << a;
  return os.str();
}

static void test_regions() {
  // 20x20 tile of the reference default (16x16 core, 5x5 stencil).
  const Array2D g(20, 20, 20);
  EXPECT(str(sub_array_region(g, 5, 5, CENTER)) == "width:  16, height: 16, x offset: 2, y offset: 2");
  EXPECT(str(sub_array_region(g, 5, 5, TOP_LEFT)) == "width:  2, height: 2, x offset: 0, y offset: 0");
  EXPECT(str(sub_array_region(g, 5, 5, BOTTOM_CENTER)) == "width:  16, height: 2, x offset: 2, y offset: 18");
  EXPECT(str(sub_array_region(g, 5, 5, RIGHT)) == "width:  2, height: 20, x offset: 18, y offset: 0");
  // TestSubRegionExtraction values quoted in SURVEY §4.
  std::ostringstream os;
  test_subregion_extraction(os);
  const std::string t = os.str();
  EXPECT(t.find("Width: 34, Height: 34") != std::string::npos);
  EXPECT(t.find("top center:    width:  30, height: 2, x offset: 2, y offset: 0") != std::string::npos);
  EXPECT(t.find("top:           width:  30, height: 2, x offset: 2, y offset: 2") != std::string::npos);
}

static void test_layout() {
  const TileGeom g = TileGeom::aligned(8192, 8192, 1, 1, 4);
  EXPECT((g.x_origin + g.halo_x) % 4 == 0);
  EXPECT(g.pitch % 64 == 0);
  EXPECT(g.pitch >= g.x_origin + g.halo_x + 8192 + 4);
  const TileGeom c = TileGeom::compact(16, 16, 2, 2);
  EXPECT(c.pitch == 20 && c.core_offset() == 2 * 20 + 2);
  double buf[400];
  for (int i = 0; i < 400; ++i) buf[i] = i;
  Accessor2D<double> a(buf, c.core());
  EXPECT(a(0, 0) == 42 && a(3, 1) == 42 + 20 + 3);
  // send/recv regions of an aligned tile
  const Array2D top_send = send_region(g, D_TOP);
  EXPECT(top_send.width == 8192 && top_send.height == 1 && top_send.y_offset == 1);
  const Array2D left_recv = recv_region(g, D_LEFT);
  EXPECT(left_recv.width == 1 && left_recv.x_offset == g.x_origin && left_recv.y_offset == 1);
}

static void test_cart() {
  auto d = dims_create(8);
  EXPECT(d[0] == 4 && d[1] == 2);
  d = dims_create(9);
  EXPECT(d[0] == 3 && d[1] == 3);
  d = dims_create(7);
  EXPECT(d[0] == 7 && d[1] == 1);
  const CartTopology t(3, 3);
  // rank 4 = centre of a 3x3 periodic grid; its 8 neighbours are all others.
  std::set<int> n;
  for (int dd = 0; dd < kNumDirs; ++dd) n.insert(t.neighbor(4, dd));
  EXPECT(n.size() == 8 && !n.count(4));
  EXPECT(t.neighbor(0, D_TOP_LEFT) == 8);  // periodic wrap
  const CartTopology np(3, 3, false, false);
  EXPECT(np.neighbor(0, D_TOP) == kProcNull);
  auto s = np.cart_shift(4, 0, 1);
  EXPECT(s[0] == 1 && s[1] == 7);  // mpi10.cpp: rank 4 neighbours 1,7,3,5
  s = np.cart_shift(4, 1, 1);
  EXPECT(s[0] == 3 && s[1] == 5);
  std::ostringstream os;
  print_cartesian_grid(os, t);
  EXPECT(os.str() == "0 1 2 \n3 4 5 \n6 7 8 \n");
  auto b = block_split(10, 3, 0);
  EXPECT(b.start == 0 && b.len == 4);
  b = block_split(10, 3, 2);
  EXPECT(b.start == 7 && b.len == 3);
}

static void test_plan() {
  const TileGeom g = TileGeom::compact(16, 16, 2, 2);
  // 3x3: 8 distinct peers, one segment each, no self copies.
  HaloPlan p = make_halo_plan(CartTopology(3, 3), 4, g);
  EXPECT(p.sends.size() == 8 && p.self_copies.empty());
  for (const auto& m : p.sends) EXPECT(m.segments.size() == 1);
  EXPECT(p.send_elems == 4 * 4 + 4 * 32 && p.recv_elems == p.send_elems);
  // 1x1: everything is a self copy.
  p = make_halo_plan(CartTopology(1, 1), 0, g);
  EXPECT(p.sends.empty() && p.self_copies.size() == 8);
  // 2x4 periodic (the 8-GPU config): 5 distinct peers; up == down.
  const CartTopology t24(2, 4);
  p = make_halo_plan(t24, 1, g);
  EXPECT(p.sends.size() == 5);
  for (const auto& m : p.sends) {
    // Symmetry: what I send to m.peer equals, segment by segment, what m.peer
    // expects from me.
    const HaloPlan q = make_halo_plan(t24, m.peer, g);
    bool found = false;
    for (const auto& r : q.recvs) {
      if (r.peer != 1) continue;
      found = true;
      EXPECT(r.count == m.count && r.segments.size() == m.segments.size());
      for (size_t i = 0; i < r.segments.size() && i < m.segments.size(); ++i) {
        EXPECT(r.segments[i].dir == m.segments[i].dir);
        EXPECT(r.segments[i].region.size() == m.segments[i].region.size());
      }
    }
    EXPECT(found);
  }
  // Star (no corners): 4 directions.
  p = make_halo_plan(CartTopology(3, 3), 4, g, /*corners=*/false);
  EXPECT(p.sends.size() == 4);
  // Loopback routes self through the wire.
  p = make_halo_plan(CartTopology(1, 1), 0, g, true, /*loopback_self=*/true);
  EXPECT(p.sends.size() == 1 && p.sends[0].peer == 0 && p.sends[0].segments.size() == 8 && p.self_copies.empty());
  EXPECT(reference_tag(D_TOP) == TOP && reference_tag(D_BOTTOM_RIGHT) == BOTTOM_RIGHT);
}

static void test_decision() {
  // 20 rounds; the baseline drifts between rounds, the candidate stays 5% faster in each.
  std::vector<double> base, fast, slow, missing;
  for (int r = 0; r < 20; ++r) {
    const double clock = 1.0 + 0.1 * ((r * 7) % 5);
    base.push_back(0.30 * clock);
    fast.push_back(0.285 * clock);
    slow.push_back(0.33 * clock);
    missing.push_back(r == 3 ? kMissingSample : 0.2 * clock);
  }
  RoundDecision d = decide_on_maxima(base, {slow, fast, missing}, 0.0);
  EXPECT(d.best == 1 && d.win && std::fabs(d.ratio - 0.95) < 1e-9 && d.ratio_iqr < 1e-9);
  EXPECT(d.ratios[2].empty() && d.ratios[0].size() == 20);  // a missing sample drops the candidate
  EXPECT(!decide_on_maxima(base, {slow}, 0.0).win);
  EXPECT(!decide_on_maxima(base, {fast}, 0.06).win);  // a 5% gain does not meet a 6% margin
  // Element-wise max over ranks: one rank in a fast-serial state does not veto.
  const std::vector<double> r0{0.30, 0.30}, r1{0.25, 0.28};
  const std::vector<double> m = elementwise_max({r0, r1});
  EXPECT(m.size() == 2 && m[0] == 0.30 && m[1] == 0.30);
  std::vector<double> v{3, 1, 2, 4};
  const auto mi = median_iqr(v);
  EXPECT(mi.first == 3 && mi.second == 4 - 2);
  EXPECT(std::fabs(median_notch(1.0, 0.1, 25) - 1.0316) < 1e-9);
}

static void test_halo_last_schedule() {
  // 8 column groups x 600 rows, the edge groups reading the ghost columns, 256
  // workgroups, depth 20: both sets cover every row once, inner chunks stay in the core.
  const std::vector<std::uint8_t> ghost{1, 0, 0, 0, 0, 0, 0, 1};
  const auto h = kernels::make_halo_last_schedule(8, 600, 256, 60, 20, ghost, 0, 0.12, 0, 8, 32);
  EXPECT(kernels::check_halo_last_schedule(h, 8, 600, 20, ghost).empty());
  EXPECT(h.outer.blocks % 8 == 0 && h.outer.blocks >= 32 && h.inner.blocks + h.outer.blocks == 256);
  EXPECT(h.band >= 20);
  // A fixed outer set.
  const auto f = kernels::make_halo_last_schedule(8, 600, 256, 60, 20, ghost, 48);
  EXPECT(f.outer.blocks == 48 && kernels::check_halo_last_schedule(f, 8, 600, 20, ghost).empty());
  // Balanced starts: monotone, cover the whole range.
  const auto st = kernels::balanced_starts(9, 8192, 256, 47);
  EXPECT(st.size() == 257 && st.front() == 0 && st.back() == 9 * 8192);
  bool mono = true;
  for (size_t i = 1; i < st.size(); ++i) mono = mono && st[i] >= st[i - 1];
  EXPECT(mono);
}

int main() {
  test_regions();
  test_layout();
  test_cart();
  test_plan();
  test_decision();
  test_halo_last_schedule();
  if (g_failures) {
    std::fprintf(stderr, "%d failure(s)\n", g_failures);
    return 1;
  }
  std::printf("mxs_unit_tests: all passed\n");
  return 0;
}
