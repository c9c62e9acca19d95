// fp64 stencil tuning harness: the natural-layout wave-streaming kernel (one
// 16-byte vector = 2 cells per lane, the round-1 fp64 path) against the
// wide-lane body (4 cells per lane, BodyWideF64) in the single-wave balanced
// launch and in the two-stage pipeline, on a W x H tile, wrap (1x1 periodic)
// and ghost-ring forms. Every variant is first checked bitwise against the
// natural kernel of the same depth (itself validated against the CPU
// reference by tests/test_gpu_headline.py); timed launches ping-pong in/out
// like the solver. One JSON line per variant.
//
//   stencil_tune64 [W] [H] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "mxs/core/error.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/hip_utils.hpp"
#include "tune_kernels.hpp"

using namespace mxs;
using namespace mxs::kernels::detail;

namespace {

struct Variant {
  std::string name;
  int steps = 1;
  std::function<void(const double*, double*, hipStream_t)> launch;
  std::function<void(const double*, double*, hipStream_t)> ref;  // same result, validated kernel(s)
  std::vector<float> ms;
  double tol = 0;  // 0: bitwise against ref; > 0: max |difference| (sum form)
};

int resident(const void* fn, int threads) {
  int occ = 0, cus = 0;
  MXS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, threads, 0));
  MXS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  return std::max(1, occ) * cus;
}

// Single-wave balanced launch; FAST = wide-lane body.
template <int S, bool WRAP, bool FAST, int PF = 3>
std::function<void(const double*, double*, hipStream_t)> balanced_fn(const TileGeom& g, int* blocks_out = nullptr) {
  const int blocks = resident(reinterpret_cast<const void*>(stencil5_stream_balanced_kernel<double, S, PF, WRAP, true, FAST>), 256);
  if (blocks_out) *blocks_out = blocks / 256;
  return [=](const double* I, double* O, hipStream_t s) {
    constexpr int OW = StripShape<double, S, FAST>::OW;
    const index_t groups = ((g.width + OW - 1) / OW + 3) / 4;
    const index_t share = (groups * g.height + blocks - 1) / blocks;
    stencil5_stream_balanced_kernel<double, S, PF, WRAP, true, FAST><<<blocks, 256, 0, s>>>(
        I, O, g.pitch, g.core_offset(), g.width, g.height, 0, g.width, 0, g.height, share, 0.2, 0.2);
  };
}

template <int S0, int S1, int PF, bool WRAP, bool SUM = false, bool JOINT = false, int LAG1 = 0, int XB = 0>
std::function<void(const double*, double*, hipStream_t)> pipe_fn(const TileGeom& g, int* per_cu = nullptr) {
  const int blocks = resident(
      reinterpret_cast<const void*>(stencil5_stream_pipe_kernel<S0, S1, PF, WRAP, 0, double, SUM, 4, false, JOINT, LAG1, XB>),
      512);
  if (per_cu) *per_cu = blocks / 256;
  const double c0 = SUM ? std::pow(0.2, S0 + S1) : 0.2;  // sum form: c0 carries c^S
  return [=](const double* I, double* O, hipStream_t s) {
    constexpr int OW = StripShape<double, S0 + S1, true>::OW;
    constexpr int OWG = JointShape<S0, S1, 4>::OWG;
    const index_t groups = JOINT ? (g.width + OWG - 1) / OWG : ((g.width + OW - 1) / OW + 3) / 4;
    const index_t share = (groups * g.height + blocks - 1) / blocks;
    PipeShares shares = PipeShares::equal(share);
    if (pipe_balanced() && blocks <= kMaxShareBlocks)
      pipe_starts(groups, g.height, blocks, pipe_fill_rows<S0, S1, PF, LAG1>(), &shares);
    stencil5_stream_pipe_kernel<S0, S1, PF, WRAP, 0, double, SUM, 4, false, JOINT, LAG1, XB><<<blocks, 512, 0, s>>>(
        I, O, g.pitch, g.core_offset(), g.width, g.height, 0, g.width, 0, g.height, shares, c0, 0.2);
  };
}

// Reference for S levels: the natural kernel, in two halves through tmp past 16.
template <int S, bool WRAP>
std::function<void(const double*, double*, hipStream_t)> ref_fn(const TileGeom& g, double* tmp) {
  if constexpr (S <= 16) {
    return balanced_fn<S, WRAP, false>(g);
  } else {
    static_assert(S % 2 == 0, "reference halves");
    auto h = balanced_fn<S / 2, WRAP, false>(g);
    return [=](const double* I, double* O, hipStream_t s) {
      h(I, tmp, s);
      h(tmp, O, s);
    };
  }
}

template <int S, bool WRAP, bool FAST, int PF = 3>
Variant balanced(const TileGeom& g, double* tmp) {
  int per_cu = 0;
  Variant v;
  v.launch = balanced_fn<S, WRAP, FAST, PF>(g, &per_cu);
  char buf[128];
  std::snprintf(buf, sizeof(buf), "%s_s%d_pf%d_b%d%s", FAST ? "wide" : "natural", S, PF, per_cu, WRAP ? "_wrap" : "");
  v.name = buf;
  v.steps = S;
  if (FAST) v.ref = ref_fn<S, WRAP>(g, tmp);
  return v;
}

template <int S0, int S1, int PF, bool WRAP, bool SUM = false, bool JOINT = false, int LAG1 = 0, int XB = 0>
Variant pipe(const TileGeom& g, double* tmp) {
  int per_cu = 0;
  Variant v;
  v.launch = pipe_fn<S0, S1, PF, WRAP, SUM, JOINT, LAG1, XB>(g, &per_cu);
  char buf[128];
  std::snprintf(buf, sizeof(buf), "pipe_s%d+%d_pf%d_b%d%s%s%s%s%s", S0, S1, PF, per_cu, WRAP ? "_wrap" : "",
                SUM ? "_sum" : "", JOINT ? "_joint" : "", LAG1 == 3 ? "_lag1" : (LAG1 == 2 ? "_lag1s1" : (LAG1 == 1 ? "_lag1s0" : "")),
                XB == 1 ? "_perm" : "");
  v.name = buf;
  v.steps = S0 + S1;
  v.ref = ref_fn<S0 + S1, WRAP>(g, tmp);
  if (SUM) v.tol = 1e-14;
  return v;
}

// Three-stage pipeline (768-thread workgroups, 3 waves per SIMD), sum form.
template <int S0, int S1, int S2, int PF, bool WRAP>
Variant pipe3(const TileGeom& g, double* tmp) {
  constexpr int S = S0 + S1 + S2;
  const int blocks =
      resident(reinterpret_cast<const void*>(stencil5_stream_pipe3_kernel<S0, S1, S2, PF, WRAP, double, true>), 768);
  const double c0 = std::pow(0.2, S);
  Variant v;
  v.launch = [=](const double* I, double* O, hipStream_t s) {
    constexpr int OW = StripShape<double, S, true>::OW;
    const index_t groups = ((g.width + OW - 1) / OW + 3) / 4;
    const index_t share = (groups * g.height + blocks - 1) / blocks;
    stencil5_stream_pipe3_kernel<S0, S1, S2, PF, WRAP, double, true><<<blocks, 768, 0, s>>>(
        I, O, g.pitch, g.core_offset(), g.width, g.height, 0, g.width, 0, g.height, share, c0, 0.2);
  };
  char buf[128];
  std::snprintf(buf, sizeof(buf), "pipe3_s%d+%d+%d_pf%d_b%d%s_sum", S0, S1, S2, PF, blocks / 256, WRAP ? "_wrap" : "");
  v.name = buf;
  v.steps = S;
  v.ref = ref_fn<S, WRAP>(g, tmp);
  v.tol = 1e-14;
  return v;
}

}  // namespace

int main(int argc, char** argv) {
  const index_t W = argc > 1 ? atol(argv[1]) : 8192;
  const index_t H = argc > 2 ? atol(argv[2]) : 8192;
  const int rounds = argc > 3 ? atoi(argv[3]) : 5;
  const TileGeom g = TileGeom::aligned(W, H, 24, 24, 8);  // ghost-ring variants up to S = 24
  DeviceBuffer<double> a(g.alloc_elems()), b(g.alloc_elems()), c(g.alloc_elems()), d(g.alloc_elems());
  for (double* p : {a.get(), b.get(), c.get(), d.get()}) kernels::fill<double>(p, g.alloc_elems(), 0.0, nullptr);
  kernels::fill_random<double>(a.get(), g, 0, 0, W, 7, 0.0, 1.0, nullptr);
  kernels::fill_random<double>(b.get(), g, 0, 0, W, 8, 0.0, 1.0, nullptr);
  // Ghost ring of the non-wrap runs: random too (frozen boundary values).
  MXS_HIP_CHECK(hipDeviceSynchronize());
  double* tmp = d.get();
  std::vector<Variant> vs;
  const char* focus = std::getenv("TUNE_FOCUS");
  const std::string f = focus ? focus : "";
  if (f == "" || f == "wrap") {
    vs.push_back(balanced<12, true, false>(g, tmp));
    vs.push_back(balanced<16, true, false>(g, tmp));
    vs.push_back(balanced<8, true, true>(g, tmp));
    vs.push_back(balanced<8, true, true, 6>(g, tmp));
    vs.push_back(pipe<6, 6, 3, true>(g, tmp));
    vs.push_back(pipe<6, 6, 6, true>(g, tmp));
    vs.push_back(pipe<7, 5, 3, true>(g, tmp));
    vs.push_back(pipe<7, 7, 3, true>(g, tmp));
    vs.push_back(pipe<7, 7, 6, true>(g, tmp));
    vs.push_back(pipe<8, 6, 3, true>(g, tmp));
    vs.push_back(pipe<8, 8, 3, true>(g, tmp));
  }
  if (f == "lag1") {  // ascending level order on the joint sum-form default (8 + 8), bitwise vs descending
    Variant a = pipe<8, 8, 3, true, true, true>(g, tmp);
    Variant b = pipe<8, 8, 3, true, true, true, 3>(g, tmp);
    b.ref = a.launch;
    b.tol = 0.0;
    Variant c = pipe<6, 6, 3, true, false, false>(g, tmp);
    Variant d = pipe<6, 6, 3, true, false, false, 3>(g, tmp);
    d.ref = c.launch;
    d.tol = 0.0;
    vs.push_back(a);
    vs.push_back(b);
    vs.push_back(c);
    vs.push_back(d);
  }
  if (f == "spill") {  // the 8192^2 default (8 + 8 joint, ascending, sum form) vs its register-pressure variants
    Variant a = pipe<8, 8, 3, true, true, true, 3>(g, tmp);
    Variant b = pipe<8, 8, 3, true, true, true, 3, 5>(g, tmp);
    Variant c = pipe<8, 8, 3, true, true, true, 3, 6>(g, tmp);
    b.ref = c.ref = a.launch;
    b.tol = c.tol = 0.0;
    b.name += "_nocopy";
    c.name += "_fence";
    Variant d = pipe<8, 8, 3, true, true, true>(g, tmp);  // descending (no spill)
    vs.push_back(a);
    vs.push_back(b);
    vs.push_back(c);
    vs.push_back(d);
  }
  if (f == "perm") {  // lane-crossing neighbours via ds_bpermute (LDS pipe) vs DPP moves, bitwise twins
    Variant a = pipe<8, 8, 3, true, true, true, 3>(g, tmp);
    Variant b = pipe<8, 8, 3, true, true, true, 3, 1>(g, tmp);
    b.ref = a.launch;
    b.tol = 0.0;
    Variant c = pipe<8, 8, 3, true, true, true>(g, tmp);
    Variant d = pipe<8, 8, 3, true, true, true, 0, 1>(g, tmp);
    d.ref = c.launch;
    d.tol = 0.0;
    vs.push_back(a);
    vs.push_back(b);
    vs.push_back(c);
    vs.push_back(d);
  }
  if (f == "split") {  // around the 6 + 6 winner of the first pass (profiles/r02_f64)
    vs.push_back(balanced<12, true, false>(g, tmp));
    vs.push_back(pipe<5, 5, 3, true>(g, tmp));
    vs.push_back(pipe<5, 5, 6, true>(g, tmp));
    vs.push_back(pipe<6, 5, 3, true>(g, tmp));
    vs.push_back(pipe<6, 6, 3, true>(g, tmp));
    vs.push_back(pipe<6, 7, 3, true>(g, tmp));
    vs.push_back(pipe<7, 6, 3, true>(g, tmp));
    vs.push_back(pipe<7, 6, 6, true>(g, tmp));
    vs.push_back(pipe<5, 7, 3, true>(g, tmp));
    vs.push_back(pipe<4, 4, 3, true>(g, tmp));
    vs.push_back(balanced<12, false, false>(g, tmp));
    vs.push_back(pipe<6, 6, 3, false>(g, tmp));
    vs.push_back(pipe<5, 5, 3, false>(g, tmp));
  }
  if (f == "pipe3") {  // three-stage pipeline vs the two-stage 8 + 8 sum form
    vs.push_back(pipe<8, 8, 3, true, true>(g, tmp));
    vs.push_back(pipe3<5, 5, 5, 3, true>(g, tmp));
    vs.push_back(pipe3<5, 5, 6, 3, true>(g, tmp));
    vs.push_back(pipe3<6, 5, 5, 3, true>(g, tmp));
    vs.push_back(pipe3<6, 6, 6, 3, true>(g, tmp));
    vs.push_back(pipe3<6, 6, 4, 3, true>(g, tmp));
  }
  if (f == "sum") {  // sum form (c_center == c_neighbor) vs the general wide-lane body
    vs.push_back(pipe<6, 6, 3, true>(g, tmp));
    vs.push_back(pipe<6, 6, 3, true, true>(g, tmp));
    vs.push_back(pipe<8, 8, 3, true, true>(g, tmp));
    vs.push_back(pipe<6, 6, 6, true, true>(g, tmp));
    vs.push_back(pipe<6, 6, 3, false>(g, tmp));
    vs.push_back(pipe<6, 6, 3, false, true>(g, tmp));
  }
  if (f == "" || f == "ghost") {
    vs.push_back(balanced<12, false, false>(g, tmp));
    vs.push_back(balanced<16, false, false>(g, tmp));
    vs.push_back(balanced<8, false, true>(g, tmp));
    vs.push_back(pipe<7, 7, 3, false>(g, tmp));
    vs.push_back(pipe<8, 8, 3, false>(g, tmp));
  }

  Stream st;
  Event e0(true), e1(true);
  const double* in = a.get();
  double* out = b.get();
  double* out2 = c.get();
  std::vector<Variant> ok;
  for (auto& v : vs) {
    (void)hipGetLastError();
    v.launch(in, out, st.get());
    const hipError_t e = hipGetLastError();
    st.sync();
    if (e != hipSuccess) {
      std::printf("{\"variant\": \"%s\", \"error\": \"%s\"}\n", v.name.c_str(), hipGetErrorString(e));
      continue;
    }
    if (v.ref) {
      v.ref(in, out2, st.get());
      st.sync();
      std::vector<double> got(size_t(g.alloc_elems())), want(size_t(g.alloc_elems()));
      MXS_HIP_CHECK(hipMemcpy(got.data(), out, got.size() * 8, hipMemcpyDeviceToHost));
      MXS_HIP_CHECK(hipMemcpy(want.data(), out2, want.size() * 8, hipMemcpyDeviceToHost));
      long long bad = 0;
      double maxdiff = 0;
      for (index_t y = 0; y < H; ++y)
        for (index_t x = 0; x < W; ++x) {
          const size_t i = size_t(g.core_offset() + y * g.pitch + x);
          const double d = std::fabs(got[i] - want[i]);
          maxdiff = std::max(maxdiff, d);
          bad += v.tol > 0 ? !(d <= v.tol) : got[i] != want[i];
        }
      std::printf("{\"variant\": \"%s\", \"mismatches\": %lld, \"max_abs_diff\": %.3g}\n", v.name.c_str(), bad,
                  maxdiff);
      std::fflush(stdout);
      if (bad) continue;
    }
    ok.push_back(std::move(v));
  }
  vs = std::move(ok);
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) {
      e0.record(st.get());
      for (int k = 0; k < 4; ++k) {
        if (k & 1) v.launch(out, const_cast<double*>(in), st.get());
        else v.launch(in, out, st.get());
      }
      e1.record(st.get());
      e1.sync();
      v.ms.push_back(e1.since(e0) / 4);
    }
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
    std::printf("{\"variant\": \"%s\", \"median_ms\": %.4f, \"best_ms\": %.4f, \"gcells_s\": %.1f}\n", v.name.c_str(),
                med, best, double(W) * double(H) * v.steps / (med * 1e-3) / 1e9);
  }
  return 0;
}
