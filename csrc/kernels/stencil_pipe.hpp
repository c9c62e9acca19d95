// Two-stage pipeline launchers (stencil_device.hpp: stencil5_stream_pipe_kernel),
// compiled in their own translation units (stencil_pipe_f32.hip,
// stencil_pipe_f64.hip: ~100 kernel instantiations) and called by the shape
// dispatch in stencil.hip.
#pragma once

#include <algorithm>

#include "mxs/core/error.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/hip_utils.hpp"
#include "stencil_device.hpp"

namespace mxs {
namespace kernels {
namespace detail {

void note_dispatch(const char* kernel);  // stencil.hip: last_stencil_dispatch() record
void note_pipe_lag1(bool lag1);          // stencil.hip: last_pipe_lag1() record

// fp64 depths the wide-lane pipeline takes (S0 = S/2, S1 = S - S0 <= 8 levels
// per stage: the windows fit 2 waves/SIMD without spilling).
constexpr int kPipeMinF64 = 9;

// Two-stage pipeline. fp32 (S = 17..32), per-step form: the fetching stage
// takes one level more than half, S0 = S/2 + 1 (at most 16) — measured 2-3%
// ahead of the even split on 4 of 5 tile shapes (profiles/r02_deep/pipe2_*,
// pipe20_*); sum form: the even split (S = 20: 10 + 10 beats 11 + 9 by 4-5% on
// 32768^2, 16384 x 8192 and 8192^2, profiles/r02_sum). 6 input rows in flight
// up to S = 28 (the fetch ring fits beside the windows at 2 waves/SIMD), 3
// above. fp64 (S = 12 and 16, wide-lane body): even split, 3 rows in flight —
// 6 + 6 is the fastest per-step fp64 form on every measured tile (8192^2 3.0
// vs 2.2 T cells/s for the single-wave natural kernel, 16384^2 3.35 vs 2.5;
// odd depths lose to the apron rounding: profiles/r02_f64), 8 + 8 the fastest
// sum form (3.5 / 4.05). One 512-thread workgroup per CU: the occupancy API
// decides, as for the single-wave balanced kernel.
template <typename T, int S, bool SUM>
constexpr int pipe_s0() {
  if constexpr (sizeof(T) == 8 || SUM) return S / 2;
  return S / 2 + 1 < 16 ? S / 2 + 1 : 16;
}
template <typename T, int S>
constexpr int pipe_pf() {
  return (sizeof(T) == 4 && S <= 28) ? 6 : 3;
}
// Joint stage-1 windows (JointShape): fp32 time blocks that split into two
// multiples of 4 levels, so the joint read reach A0 + A1 equals the per-strip
// apron SA(S) and the ghost-ring / padding requirements do not change. Splits
// (tuner, sum form, profiles/r02_joint): 20 = 12 + 8 from 24576 columns
// (32768^2 10.9 vs 10.7 T cells/s for 8 + 12 and 10.0 per-strip 10 + 10), else
// 8 + 12 (2-3% ahead on the 16384- and 8192-wide tiles), 24 = 12 + 12 (11.1 vs
// 10.2 per-strip),
// 28 = 12 + 16 (11.5), 32 = 16 + 16 (11.8; PF = 3).
// fp64 (wide-lane body, 4 doubles per lane: the same 256-column strips): the
// sum form's S = 16 as 8 + 8, 944 vs 896 columns per group.
template <typename T, int S>
constexpr bool pipe_joint_ok() {
  return sizeof(T) == 4 ? (S % 4 == 0 && S >= 20) : S == 16;
}
template <typename T, int S>
constexpr int joint_s0() {
  return sizeof(T) == 8 ? S / 2 : (S >= 32 ? 16 : 12);
}
// Level order (LAG1, stencil_device.hpp pipe_chunk): ascending levels lag one
// row per level instead of three, so a chunk fills its pipeline S - 1 rows
// sooner per stage, at the cost of a dependent chain of levels per row. Round 2
// (wall-clock tuner, profiles/r02_lag1) found it paying on short chunks only
// and kept the descending order past 768-row shares. Round 6 measured it in
// shader cycles per workgroup (tuner focus fillfit, profiles/r06_fill): the two
// orders cost the same per row (796 cycles per group-row at S = 20, 12 + 8) and
// the ascending one less per share (38 k vs 51 k cycles of fill), so fp32 S = 20
// ascends at every share length: 32768^2 -0.65%, 16384^2 -1.8%, the 8-GPU tile
// -2.3% workgroup cycles. S = 24 (12 + 12) took LAG1 everywhere already.
constexpr index_t kLag1MaxChunk = index_t(1) << 62;  // fp32 S = 20: every share length
constexpr int kLagBoth = 3;  // LAG1 stage mask: both stages ascend
// fp64 (S = 16 as 8 + 8, wide lanes): 8192^2 (288-row chunks) 3.88 -> 4.00 T
// cells/s (profiles/r02_lag1/*64*); on 2240-row shares (32768 x 16384) the two
// orders tie (4,354 vs 4,346 G cells/s, profiles/r06_fp64), so fp64 ascends at
// every share length too.
constexpr index_t kLag1MaxChunkF64 = index_t(1) << 62;
// With LAG1 (short chunks) S = 20 runs 8 + 12 below 12288 columns (8192^2:
// 9.49 vs 9.36 for 12 + 8), else 12 + 8.
constexpr index_t kJointWide = 12288;

// JS0: 0 = per-strip layout (pipe_s0 split), else joint windows with S0 = JS0.
// XB = kScaledBody (with SUM): the scaled form's body (stencil_device.hpp).
template <typename T, int S, bool WRAP, bool SUM, int JS0 = 0, int LAG1 = 0, int XB = 0>
constexpr auto pipe_kernel() {
  if constexpr (JS0 > 0)
    return stencil5_stream_pipe_kernel<JS0, S - JS0, pipe_pf<T, S>(), WRAP, 0, T, SUM, kWavesPerBlock, false, true,
                                       LAG1, XB>;
  else
    return stencil5_stream_pipe_kernel<pipe_s0<T, S, SUM>(), S - pipe_s0<T, S, SUM>(), pipe_pf<T, S>(), WRAP, 0, T,
                                       SUM>;
}

template <typename T, int S, bool WRAP, bool SUM, int JS0 = 0>
int pipe_blocks() {
  static int blocks = 0;
  if (blocks == 0) {
    int occ = 0;
    MXS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &occ, reinterpret_cast<const void*>(pipe_kernel<T, S, WRAP, SUM, JS0>()), 2 * kBlock, 0));
    blocks = std::max(occ, 1) * device_cu_count();
  }
  return std::max(1, blocks / gpu_share());
}

template <typename T, int S, bool WRAP, bool SUM, int JS0 = 0>
index_t pipe_share(index_t x0, index_t x1, index_t y0, index_t y1) {
  constexpr int OW = StripShape<T, S, true>::OW;
  constexpr int OWG = JointShape<(JS0 > 0 ? JS0 : S / 2), S - (JS0 > 0 ? JS0 : S / 2), kWavesPerBlock>::OWG;
  const index_t groups =
      JS0 > 0 ? (x1 - x0 + OWG - 1) / OWG : ((x1 - x0 + OW - 1) / OW + kWavesPerBlock - 1) / kWavesPerBlock;
  const int blocks = pipe_blocks<T, S, WRAP, SUM, JS0>();
  return (groups * (y1 - y0) + blocks - 1) / blocks;
}

// Row iterations a chunk of R rows costs beyond R (pipe_chunk: the longer of
// the two stages' block counts, rounded up to a block).
template <int S0, int S1, int PF, int LAG1>
constexpr index_t pipe_fill_rows() {
  constexpr bool A0 = (LAG1 & 1) != 0, A1 = (LAG1 & 2) != 0;
  constexpr int E0 = A0 ? 2 * S0 : 3 * S0 - 1, E1 = A1 ? 2 * S1 : 3 * S1 - 1;
  constexpr int D = (PF - E0 % PF) % PF;
  constexpr int T1 = (E0 + D) / PF + 1;
  constexpr int a = 2 * S1 + E0 + D, b = T1 * PF + E1;
  return (a > b ? a : b) + PF - 1;
}

// Fill-aware shares (balanced_starts), memoised per shape: the binary search
// costs ~10 us of host time, a launch must not.
void pipe_starts(index_t groups, index_t rows, int blocks, index_t fill, PipeShares* out);

// MXS_PIPE_BALANCED=0: equal row shares (the round-2 rule), for comparison.
bool pipe_balanced();

template <typename T, int S, bool WRAP, bool SUM, int JS0, int LAG1 = 0, int XB = 0>
void launch_pipe_form(const T* in, T* out, const TileGeom& g, index_t x0, index_t x1, index_t y0, index_t y1, T c0,
                      T c1, T sc, hipStream_t s) {
  static_assert(XB == 0 || (SUM && XB == kScaledBody && JS0 > 0), "the scaled form runs the joint pipeline");
  const index_t share = pipe_share<T, S, WRAP, SUM, JS0>(x0, x1, y0, y1);
  const int blocks = pipe_blocks<T, S, WRAP, SUM, JS0>();
  PipeShares shares = PipeShares::equal(share);
  if (pipe_balanced() && blocks <= kMaxShareBlocks) {
    constexpr int S0 = JS0 > 0 ? JS0 : pipe_s0<T, S, SUM>();
    constexpr int OW = StripShape<T, S, true>::OW;
    constexpr int OWG = JointShape<(JS0 > 0 ? JS0 : S / 2), S - (JS0 > 0 ? JS0 : S / 2), kWavesPerBlock>::OWG;
    const index_t groups =
        JS0 > 0 ? (x1 - x0 + OWG - 1) / OWG : ((x1 - x0 + OW - 1) / OW + kWavesPerBlock - 1) / kWavesPerBlock;
    pipe_starts(groups, y1 - y0, blocks, pipe_fill_rows<S0, S - S0, pipe_pf<T, S>(), LAG1>(), &shares);
  }
  // Shares longer than kMaxChunkBytes are walked in pieces inside the kernel;
  // a piece must still hold a useful number of rows.
  MXS_CHECK(g.pitch * index_t(sizeof(T)) * kMinChunkRows <= kMaxChunkBytes,
            "stencil5_tb: rows of " << g.pitch * index_t(sizeof(T)) << " bytes leave fewer than " << kMinChunkRows
                                    << " rows per pipeline chunk (buffer-descriptor stores)");
  // Sum form: (c^S, c); scaled form: (c1^S, c0 / c1); per step: (c0, c1).
  const T kc = XB == kScaledBody ? T(double(c0) / double(c1)) : c1;
  pipe_kernel<T, S, WRAP, SUM, JS0, LAG1, XB>()<<<blocks, 2 * kBlock, 0, s>>>(
      in, out, g.pitch, g.core_offset(), g.width, g.height, x0, x1, y0, y1, shares, SUM ? sc : c0, kc);
  note_dispatch(XB == kScaledBody ? "stream_pipe_scaled" : SUM ? "stream_pipe_sum" : "stream_pipe");
  note_pipe_lag1(LAG1 != 0);
}

template <typename T, int S, bool WRAP, bool SUM, int XB = 0>
void launch_pipe_impl(const T* in, T* out, const TileGeom& g, index_t x0, index_t x1, index_t y0, index_t y1, T c0, T c1,
                 T sc, hipStream_t s) {
  if constexpr (pipe_joint_ok<T, S>()) {
    if (pipe_joint()) {
      if constexpr (sizeof(T) == 4 && S == 20) {
        if (pipe_lag1() && pipe_share<T, S, WRAP, SUM, 12>(x0, x1, y0, y1) <= kLag1MaxChunk) {
          if (x1 - x0 < kJointWide)
            return launch_pipe_form<T, S, WRAP, SUM, 8, kLagBoth, XB>(in, out, g, x0, x1, y0, y1, c0, c1, sc, s);
          return launch_pipe_form<T, S, WRAP, SUM, 12, kLagBoth, XB>(in, out, g, x0, x1, y0, y1, c0, c1, sc, s);
        }
      } else if constexpr (sizeof(T) == 4 && S == 24) {
        if (pipe_lag1())
          return launch_pipe_form<T, S, WRAP, SUM, 12, kLagBoth, XB>(in, out, g, x0, x1, y0, y1, c0, c1, sc, s);
      } else if constexpr (sizeof(T) == 8 && S == 16) {
        if (pipe_lag1() && pipe_share<T, S, WRAP, SUM, 8>(x0, x1, y0, y1) <= kLag1MaxChunkF64)
          return launch_pipe_form<T, S, WRAP, SUM, 8, kLagBoth, XB>(in, out, g, x0, x1, y0, y1, c0, c1, sc, s);
      }
      return launch_pipe_form<T, S, WRAP, SUM, joint_s0<T, S>(), 0, XB>(in, out, g, x0, x1, y0, y1, c0, c1, sc, s);
    }
  }
  if constexpr (XB == 0) {
    launch_pipe_form<T, S, WRAP, SUM, 0>(in, out, g, x0, x1, y0, y1, c0, c1, sc, s);
  } else {
    // The scaled body runs in the joint windows only: with them off (the
    // experiments knob MXS_PIPE_JOINT=0) the pass runs per step, exact.
    launch_pipe_form<T, S, WRAP, false, 0>(in, out, g, x0, x1, y0, y1, c0, c1, sc, s);
  }
}

// Whether the fp64 wide-lane pipeline can take [x0, x1) x [y0, y1) at depth S:
// whole 4-cell lane vectors (x0, x1 and, wrapping, the width multiples of 4),
// the apron inside the row padding, and rows narrow enough for kMinChunkRows
// per descriptor-sized piece.
template <typename T, int S, bool WRAP>
bool wide_pipe_ok_impl(const TileGeom& g, index_t x0, index_t x1, index_t y0, index_t y1) {
  constexpr int SA = StripShape<T, S, true>::SA;
  if (x0 % 4 != 0 || x1 % 4 != 0) return false;
  if (WRAP && g.width % 4 != 0) return false;
  const index_t lead = g.x_origin + g.halo_x;
  if (!WRAP && (lead < SA || g.pitch < lead + (g.width + 3) / 4 * 4 + SA)) return false;
  (void)y0;
  (void)y1;
  return g.pitch * index_t(sizeof(T)) * kMinChunkRows <= kMaxChunkBytes;  // longer chunks go in pieces
}


// Explicitly instantiated in the pipeline TUs (XB = kScaledBody: the scaled
// form, instantiated at the solver's depths only: fp32 20 / 24, fp64 16).
template <typename T, int S, bool WRAP, bool SUM, int XB = 0>
void launch_pipe(const T* in, T* out, const TileGeom& g, index_t x0, index_t x1, index_t y0, index_t y1, T c0, T c1,
                 T sc, hipStream_t s);
template <typename T, int S, bool WRAP>
bool wide_pipe_ok(const TileGeom& g, index_t x0, index_t x1, index_t y0, index_t y1);

}  // namespace detail
}  // namespace kernels
}  // namespace mxs
