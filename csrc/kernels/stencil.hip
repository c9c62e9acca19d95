// 2D stencil update kernels (K10; not present in the reference, whose Compute()
// is empty: stencil2d/mpi-2d-stencil-subarray-cuda.cu:32-33).
//
// Regime: a 5-point Jacobi sweep moves 2 x sizeof(T) bytes of compulsory HBM
// traffic per cell (read u, write u') for ~6 flops: HBM-bound by two orders of
// magnitude. One sweep per iteration therefore tops out at the copy roofline
// (~0.7 T cells/s fp32); the framework's default path is temporal blocking
// (stencil5_tb below: the wave-streaming kernels of stencil_device.hpp advance
// S iterations per pass over HBM, ~6 T cells/s at S = 12). The single-sweep
// kernels remain for S = 1, remainders and box stencils:
//
// Variant RegisterRoll (single sweep, default):
//   * a wave owns a 64 x VEC column segment (VEC = 16 B / sizeof(T): 256 fp32
//     or 128 fp64 columns) and a strip of ROWS rows;
//   * each lane issues one 16-byte load per row (global_load_dwordx4, a whole
//     1 KiB wave-instruction on aligned rows: TileGeom::aligned) and keeps a
//     rolling 3-row window (up / mid / down) in registers, so vertical reuse
//     inside a strip costs nothing;
//   * horizontal neighbours come from the adjacent lane by a wave shuffle
//     (x-1 of the first element, x+1 of the last); only lanes 0 and 63 load the
//     single column just outside the segment;
//   * rows are processed in chunks of CH: the CH row loads of a chunk are issued
//     back to back before any arithmetic. Measured (bench/stencil_tune.hip,
//     profiles/stencil_tuning): the winner is a SHORT strip (3-4 rows) loaded in
//     one chunk — ROWS+2 independent 1 KiB loads in flight per wave from its
//     first instruction — with 4 waves side by side covering 4 KiB of a row. The
//     two rows a strip re-reads at its ends come from L2 / Infinity Cache
//     (vertically adjacent strips run concurrently on one XCD), while long
//     rolling strips (32 rows) lose ~30 % to exposed HBM latency;
//   * non-temporal (streaming) stores: the output is not re-read before the
//     next sweep, so it should not displace the input rows in L2.
// Variant LdsTile: the textbook LDS-staged tile (a (TH+2) x (TW+2) input tile
//   staged once per workgroup with 16-byte loads, five LDS reads per output).
//   Kept as the measured alternative (see profiles/ and docs/PERF.md).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <limits>
#include <cstdlib>
#include <string>
#include <vector>

#include "mxs/core/error.hpp"
#include "mxs/kernels/kernels.hpp"
#include "mxs/runtime/hip_utils.hpp"

#include "stencil_device.hpp"
#include "stencil_pipe.hpp"

namespace mxs {
namespace kernels {
namespace {
using namespace detail;
constexpr int kLdsRows = 16;

// Host-side record of the kernel form the last stencil launcher picked (the
// tests assert that their shapes reach the kernel the benchmarks time).
std::atomic<const char*> g_last_dispatch{"none"};
std::atomic<bool> g_last_lag1{false};  // the pipeline launcher sets it after note()
inline void note(const char* k) {
  g_last_dispatch.store(k, std::memory_order_relaxed);
  g_last_lag1.store(false, std::memory_order_relaxed);
}

// Tuned on MI355X with bench/stencil_tune.hip (profiles/stencil_tuning/*.log):
// short strips whose ROWS+2 row loads are all issued up front beat long rolling
// strips — the extra rows a short strip re-reads are L2/Infinity-Cache hits
// (vertically adjacent strips run concurrently on the same XCD), while
// per-wave bytes in flight are what the HBM stream needs. 4 waves side by side
// cover 4 KiB of a row per workgroup. 3-row strips are best up to ~16K-wide
// tiles, 4-row strips on wider ones (32768^2: 738 vs 731 Gcells/s).
template <typename T, int ROWS>
void launch_roll(const T* in, T* out, const TileGeom& g, index_t row_begin, index_t row_end, T c0, T c1,
                 hipStream_t s) {
  constexpr int N = Vec16<T>::N;
  constexpr int WX = 4, NW = 4;
  const index_t rows = row_end - row_begin;
  const index_t gx = (g.width + index_t(kWaveSize) * N * WX - 1) / (index_t(kWaveSize) * N * WX);
  const index_t gy = (rows + ROWS - 1) / ROWS;
  stencil5_roll_kernel<T, ROWS, ROWS, true, WX, false, NW><<<dim3(unsigned(gx), unsigned(gy)), NW * kWaveSize, 0, s>>>(
      in, out, g.pitch, g.core_offset(), g.width, row_begin, row_end, c0, c1);
}

}  // namespace

template <typename T>
void stencil5_rows(const T* in, T* out, const TileGeom& g, index_t row_begin, index_t row_end,
                   Stencil5Coeffs c, hipStream_t s, StencilVariant v) {
  if (row_end <= row_begin || g.width <= 0) return;
  MXS_CHECK(g.halo_x >= 1 && g.halo_y >= 1, "stencil5 needs a ghost ring of at least 1");
  MXS_CHECK(row_begin >= 0 && row_end <= g.height, "row range out of the core");
  constexpr int N = Vec16<T>::N;
  MXS_CHECK((g.pitch % N) == 0 && ((g.x_origin + g.halo_x) % N) == 0,
            "stencil5_rows needs a TileGeom::aligned layout (16-byte aligned core rows)");
  MXS_CHECK(g.pitch >= g.x_origin + g.halo_x + ((g.width + N - 1) / N) * N + N,
            "pitch too small for vector loads");
  const T c0 = T(c.center), c1 = T(c.neighbor);
  const index_t rows = row_end - row_begin;
  const index_t gx = (g.width + kWaveSize * N - 1) / (kWaveSize * N);
  if (v == StencilVariant::LdsTile) {
    const index_t gy = (rows + kLdsRows - 1) / kLdsRows;
    const size_t lds = size_t(kLdsRows + 2) * (kWaveSize * N + 2 * N) * sizeof(T);
    stencil5_lds_kernel<T, kLdsRows><<<dim3(unsigned(gx), unsigned(gy)), kBlock, lds, s>>>(
        in, out, g.pitch, g.core_offset(), g.width, row_begin, row_end, c0, c1);
    note("lds");
  } else {
    note("roll");
    if (g.width * int(sizeof(T)) >= 32768 * 4) launch_roll<T, 4>(in, out, g, row_begin, row_end, c0, c1, s);
    else launch_roll<T, 3>(in, out, g, row_begin, row_end, c0, c1, s);
  }
  MXS_HIP_CHECK_LAUNCH();
}

template <typename T>
bool stencil5_periodic_supported(const TileGeom& g) {
  constexpr int N = Vec16<T>::N;
  return g.width % N == 0 && g.width >= N && g.height >= 1 && (g.pitch % N) == 0 &&
         ((g.x_origin + g.halo_x) % N) == 0;
}

template <typename T>
void stencil5_periodic(const T* in, T* out, const TileGeom& g, Stencil5Coeffs c, hipStream_t s) {
  MXS_CHECK(stencil5_periodic_supported<T>(g), "stencil5_periodic: width must be a multiple of the vector width");
  constexpr int N = Vec16<T>::N;
  constexpr int WX = 4, NW = 4;
  const T c0 = T(c.center), c1 = T(c.neighbor);
  const index_t gx = (g.width + index_t(kWaveSize) * N * WX - 1) / (index_t(kWaveSize) * N * WX);
  auto go = [&](auto rows_tag) {
    constexpr int R = decltype(rows_tag)::value;
    const index_t gy = (g.height + R - 1) / R;
    stencil5_roll_kernel<T, R, R, true, WX, false, NW, true><<<dim3(unsigned(gx), unsigned(gy)), NW * kWaveSize, 0, s>>>(
        in, out, g.pitch, g.core_offset(), g.width, 0, g.height, c0, c1, g.height);
  };
  if (g.width * int(sizeof(T)) >= 32768 * 4) go(std::integral_constant<int, 4>{});
  else go(std::integral_constant<int, 3>{});
  note("roll_wrap");
  MXS_HIP_CHECK_LAUNCH();
}

namespace {
template <typename T, int S, int TW, int TH, bool WRAP>
void launch_tb_tile(const T* in, T* out, const TileGeom& g, index_t x0, index_t x1, index_t y0, index_t y1, T c0, T c1,
                    hipStream_t s) {
  const size_t lds = tb1_lds_bytes<T, S, TW, TH>();
  const dim3 grid(unsigned((x1 - x0 + TW - 1) / TW), unsigned((y1 - y0 + TH - 1) / TH));
  stencil5_tb1_kernel<T, S, TW, TH, WRAP><<<grid, 256, lds, s>>>(in, out, g.pitch, g.core_offset(), g.width,
                                                                 g.height, x0, x1, y0, y1, c0, c1);
  note("tb_tile");
}

// Workgroups of the balanced stream kernel resident at once on this device:
// occupancy x CUs, at least 2 per CU (at S = 16, 1 fits; two rounds of
// half-size shares still beat one round: profiles/stencil_tuning/tune16).
// Rows in flight per wave (the fetch ring) of the fp32 rotated kernel: 6 up to
// S = 12, where a 3-row lookahead (~1 us of work) no longer covers HBM latency
// under load (8192^2, S = 12: +5%); 3 above, where 6 pushes S = 16 to 253
// VGPRs and measured no better (profiles/stencil_tuning/tunePF_*).
template <typename T, int S>
constexpr int stream_pf() {
  return (sizeof(T) == 4 && S <= 12) ? 6 : 3;
}

template <typename T, int S, bool WRAP, bool SUM>
int balanced_blocks() {
  static int blocks = 0;
  if (blocks == 0) {
    int occ = 0, cus = 0, dev = 0;
    MXS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &occ,
        reinterpret_cast<const void*>(
            stencil5_stream_balanced_kernel<T, S, stream_pf<T, S>(), WRAP, true, sizeof(T) == 4, SUM>),
        kBlock, 0));
    MXS_HIP_CHECK(hipGetDevice(&dev));
    MXS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    blocks = std::max(occ, 2) * std::max(cus, 1);
  }
  return std::max(1, blocks / gpu_share());
}

// Wave-streaming kernels (stencil_device.hpp). Bulk rectangles: the balanced
// persistent launch — as many workgroups as are resident, each streaming an
// equal share of (4-strip group) x rows (profiles/stencil_tuning/tune16: +12-17%
// over the grid form on 8192^2 and on the 8-GPU tile 8192 x 16384, equal on
// 32768^2). Rectangles too small to give every workgroup >= 64 rows use the
// grid form, whose row chunk CH is the largest of 512..64 that still yields
// >= 4096 waves.
// The fp32 rotated-pair form (stream_chunk_rot: 11 VALU per level-row instead
// of ~15, DPP shifts folded into the adds) stores through a buffer descriptor
// over one chunk's rows: it needs whole output vectors and a chunk of at most
// kMaxChunkBytes (the balanced kernel walks longer shares in pieces, so there
// only kMinChunkRows rows have to fit).
template <typename T>
bool rot_ok(const TileGeom& g, index_t x1, index_t chunk_rows) {
  return sizeof(T) == 4 && x1 % 4 == 0 && chunk_rows * g.pitch * index_t(sizeof(T)) <= kMaxChunkBytes;
}

// SUM: the balanced rotated kernel runs the sum form (sc = c^S, see
// stencil_device.hpp), with XB = kScaledBody the scaled form (sc = c1^S,
// k = c0 / c1); every other form keeps the per-step coefficients.
template <typename T, int S, bool WRAP, bool SUM = false, int XB = 0>
void launch_stream(const T* in, T* out, const TileGeom& g, index_t x0, index_t x1, index_t y0, index_t y1, T c0, T c1,
                   T sc, hipStream_t s) {
  constexpr int OW = StreamShape<T, S>::OW;
  constexpr bool kF32 = sizeof(T) == 4;
  const index_t strips = (x1 - x0 + OW - 1) / OW;
  const index_t rows = y1 - y0;
  const index_t groups = (strips + kWavesPerBlock - 1) / kWavesPerBlock;
  const int blocks = balanced_blocks<T, S, WRAP, SUM>();
  if (groups * rows >= index_t(blocks) * 64) {
    const index_t share = (groups * rows + blocks - 1) / blocks;
    if (kF32 && rot_ok<T>(g, x1, std::min<index_t>(kMinChunkRows, std::min(share, rows)))) {
      const T kc = XB == kScaledBody ? T(double(c0) / double(c1)) : c1;
      stencil5_stream_balanced_kernel<T, S, stream_pf<T, S>(), WRAP, true, kF32, SUM, XB><<<blocks, kBlock, 0, s>>>(
          in, out, g.pitch, g.core_offset(), g.width, g.height, x0, x1, y0, y1, share, SUM ? sc : c0, kc);
      note(XB == kScaledBody ? "stream_balanced_rot_scaled" : SUM ? "stream_balanced_rot_sum" : "stream_balanced_rot");
    } else {
      stencil5_stream_balanced_kernel<T, S, 3, WRAP><<<blocks, kBlock, 0, s>>>(
          in, out, g.pitch, g.core_offset(), g.width, g.height, x0, x1, y0, y1, share, c0, c1);
      note("stream_balanced");
    }
    return;
  }
  index_t ch = 512;
  while (ch > 64 && strips * ((rows + ch - 1) / ch) < 4096) ch /= 2;
  const dim3 grid(unsigned(groups), unsigned((rows + ch - 1) / ch));
  if (kF32 && rot_ok<T>(g, x1, std::min(ch, rows))) {
    stencil5_stream_kernel<T, S, stream_pf<T, S>(), WRAP, true, kF32><<<grid, kBlock, 0, s>>>(
        in, out, g.pitch, g.core_offset(), g.width, g.height, x0, x1, y0, y1, ch, c0, c1);
    note("stream_grid_rot");
  } else {
    stencil5_stream_kernel<T, S, 3, WRAP><<<grid, kBlock, 0, s>>>(in, out, g.pitch, g.core_offset(), g.width,
                                                                  g.height, x0, x1, y0, y1, ch, c0, c1);
    note("stream_grid");
  }
}

// Dispatch by shape. Bulk rectangles take the wave-streaming kernel (Auto) or
// the LDS tile (LdsTile, S <= 8): 128 fp32 columns (64 fp64: same bytes) x 32
// rows per 256-thread workgroup, single LDS buffer. The overlap schedule's
// boundary strips are only S rows or S columns thin; a bulk tile or a 256-column
// wave strip would recompute 8-32x the strip, so thin strips get a matching thin
// LDS tile (32 x 128 for column strips, 128 x 16 for row strips).
// XB = kScaledBody (with SUM): the scaled form, on the fp64 wide pipeline at
// S = 16 and the fp32 balanced stream kernel; the thin-strip tiles, the grid
// form and the fp64 stream kernels run per step.
template <typename T, int S, bool WRAP, bool SUM, int XB = 0>
void launch_tb(const T* in, T* out, const TileGeom& g, index_t x0, index_t x1, index_t y0, index_t y1, T c0, T c1,
               T sc, StencilVariant v, hipStream_t s) {
  constexpr int TW = sizeof(T) == 4 ? 128 : 64;
  constexpr int NW = sizeof(T) == 4 ? 32 : 16;
  constexpr int NH = (sizeof(T) == 8 && S > 8) ? 64 : 128;  // keeps the fp64 thin tile under 64 KB of LDS
  if constexpr (!WRAP) {
    if (x1 - x0 <= NW) return launch_tb_tile<T, S, NW, NH, false>(in, out, g, x0, x1, y0, y1, c0, c1, s);
    if (y1 - y0 <= 16) return launch_tb_tile<T, S, TW, 16, false>(in, out, g, x0, x1, y0, y1, c0, c1, s);
  }
  if constexpr (S <= 8) {
    if (v == StencilVariant::LdsTile)
      return launch_tb_tile<T, S, TW, 32, WRAP>(in, out, g, x0, x1, y0, y1, c0, c1, s);
  }
  if constexpr (sizeof(T) == 8 && S >= kPipeMinF64 && (XB == 0 || S == 16)) {
    if (wide_pipe_ok<T, S, WRAP>(g, x0, x1, y0, y1))
      return launch_pipe<T, S, WRAP, SUM, XB>(in, out, g, x0, x1, y0, y1, c0, c1, sc, s);
  }
  // fp32: the balanced rotated kernel takes the sum or the scaled form; fp64's
  // stream kernels run per step.
  launch_stream<T, S, WRAP, SUM && sizeof(T) == 4, sizeof(T) == 4 ? XB : 0>(in, out, g, x0, x1, y0, y1, c0, c1, sc, s);
}

// form: 1 = sum form (c_center == c_neighbor, allowed by the caller: the fast
// bodies take sc = c^S), 2 = scaled form (c_center != c_neighbor: sc = c1^S and
// k = c0 / c1; fp32 depths 2-16 and 20 / 24, fp64 16; elsewhere per step),
// 0 = per step. S = 1 always keeps the per-step form.
template <typename T, bool WRAP, int S = 1>
void dispatch_tb(int steps, int form, const T* in, T* out, const TileGeom& g, index_t x0, index_t x1, index_t y0,
                 index_t y1, T c0, T c1, StencilVariant v, hipStream_t s) {
  const T sc = T(std::pow(double(c1), double(S)));
  if constexpr (S <= kMaxTimeBlock) {
    if (steps == S) {
      if constexpr (S > 1) {
        if (form == 1) return launch_tb<T, S, WRAP, true>(in, out, g, x0, x1, y0, y1, c0, c1, sc, v, s);
      }
      if constexpr ((sizeof(T) == 8 && S == 16) || (sizeof(T) == 4 && S > 1)) {
        if (form == 2)
          return launch_tb<T, S, WRAP, true, kScaledBody>(in, out, g, x0, x1, y0, y1, c0, c1, sc, v, s);
      }
      return launch_tb<T, S, WRAP, false>(in, out, g, x0, x1, y0, y1, c0, c1, sc, v, s);
    }
    return dispatch_tb<T, WRAP, S + 1>(steps, form, in, out, g, x0, x1, y0, y1, c0, c1, v, s);
  } else if constexpr (S <= kMaxTimeBlockDeep && sizeof(T) == 4) {
    if (steps == S) {
      if (form == 1) return launch_pipe<T, S, WRAP, true>(in, out, g, x0, x1, y0, y1, c0, c1, sc, s);
      if constexpr (S == 20 || S == 24) {
        if (form == 2) return launch_pipe<T, S, WRAP, true, kScaledBody>(in, out, g, x0, x1, y0, y1, c0, c1, sc, s);
      }
      return launch_pipe<T, S, WRAP, false>(in, out, g, x0, x1, y0, y1, c0, c1, sc, s);
    }
    return dispatch_tb<T, WRAP, S + 1>(steps, form, in, out, g, x0, x1, y0, y1, c0, c1, v, s);
  } else {
    MXS_CHECK(false, "stencil5_tb: steps must be in [1, " << (sizeof(T) == 4 ? kMaxTimeBlockDeep : kMaxTimeBlock)
                                                          << "], got " << steps);
  }
}
}  // namespace

template <typename T>
void stencil5_tb(const T* in, T* out, const TileGeom& g, int steps, index_t x0, index_t x1, index_t y0, index_t y1,
                 Stencil5Coeffs c, bool wrap, hipStream_t s, StencilVariant v) {
  if (x1 <= x0 || y1 <= y0) return;
  constexpr int N = Vec16<T>::N;
  MXS_CHECK(x0 >= 0 && y0 >= 0 && x1 <= g.width && y1 <= g.height, "stencil5_tb: rect out of the core");
  MXS_CHECK(stencil5_deep_supported<T>(steps, x0, x1),
            "stencil5_tb: " << steps << "-step blocks need fp32 and a column range of whole vectors (got "
                            << sizeof(T) * 8 << "-bit, [" << x0 << ", " << x1 << "))");
  MXS_CHECK(x0 % N == 0, "stencil5_tb: x0 must be a multiple of the vector width");
  MXS_CHECK((g.pitch % N) == 0 && ((g.x_origin + g.halo_x) % N) == 0, "stencil5_tb needs a TileGeom::aligned layout");
  const int sa = ((steps + N - 1) / N) * N;
  if (wrap) {
    MXS_CHECK(g.width % N == 0, "stencil5_tb wrap: width must be a multiple of the vector width");
    MXS_CHECK(g.height >= steps, "stencil5_tb wrap: tile height " << g.height << " < time block " << steps);
  } else {
    MXS_CHECK(g.halo_x >= steps && g.halo_y >= steps,
              "stencil5_tb: ghost ring (" << g.halo_x << ") shallower than the time block (" << steps << ")");
    MXS_CHECK(g.x_origin + g.halo_x >= sa && g.pitch >= g.x_origin + g.halo_x + ((g.width + N - 1) / N) * N + sa,
              "stencil5_tb: row padding too small for the x apron");
  }
  const T c0 = T(c.center), c1 = T(c.neighbor);
  // Fast forms only inside their bounds (fast_form_safe: coefficients, c1^S
  // normal, growth x the caller's range); else the per-step form.
  const bool fast = v != StencilVariant::LdsTile && fast_form_safe<T>(c, steps);
  const int form = !fast ? 0 : uses_sum_form(c) ? 1 : uses_scaled_form(c) ? 2 : 0;
  if (wrap) dispatch_tb<T, true>(steps, form, in, out, g, x0, x1, y0, y1, c0, c1, v, s);
  else dispatch_tb<T, false>(steps, form, in, out, g, x0, x1, y0, y1, c0, c1, v, s);
  MXS_HIP_CHECK_LAUNCH();
}

template <typename T>
void stencil5_rect(const T* in, T* out, const TileGeom& g, index_t x0, index_t x1, index_t y0, index_t y1,
                   Stencil5Coeffs c, hipStream_t s) {
  if (x1 <= x0 || y1 <= y0) return;
  MXS_CHECK(g.halo_x >= 1 && g.halo_y >= 1, "stencil5 needs a ghost ring of at least 1");
  MXS_CHECK(x0 >= 0 && y0 >= 0 && x1 <= g.width && y1 <= g.height, "rect out of the core");
  const index_t n = (x1 - x0) * (y1 - y0);
  const index_t blocks = std::min<index_t>((n + kBlock - 1) / kBlock, index_t(device_cu_count()) * 8);
  stencil5_rect_kernel<T><<<unsigned(blocks), kBlock, 0, s>>>(in, out, g.pitch, g.core_offset(), x0, x1 - x0, y0,
                                                              y1 - y0, T(c.center), T(c.neighbor));
  note("rect");
  MXS_HIP_CHECK_LAUNCH();
}

template <typename T>
void stencil_box(const T* in, T* out, const TileGeom& g, index_t x0, index_t x1, index_t y0, index_t y1,
                 const BoxWeights& w, hipStream_t s) {
  if (x1 <= x0 || y1 <= y0) return;
  MXS_CHECK(w.radius == 1 || w.radius == 2, "box radius must be 1 or 2");
  MXS_CHECK(g.halo_x >= w.radius && g.halo_y >= w.radius, "ghost ring narrower than the box radius");
  const dim3 grid(unsigned((x1 - x0 + 63) / 64), unsigned((y1 - y0 + 15) / 16));
  if (w.radius == 1)
    stencil_box_kernel<T, 1><<<grid, kBlock, 0, s>>>(in, out, g.pitch, g.core_offset(), x0, x1 - x0, y0, y1 - y0, w);
  else
    stencil_box_kernel<T, 2><<<grid, kBlock, 0, s>>>(in, out, g.pitch, g.core_offset(), x0, x1 - x0, y0, y1 - y0, w);
  note("box");
  MXS_HIP_CHECK_LAUNCH();
}

const char* last_stencil_dispatch() { return g_last_dispatch.load(std::memory_order_relaxed); }

namespace {
std::atomic<int> g_gpu_share{1};
std::atomic<bool> g_pipe_joint{[] {
  const char* e = experiment_env("MXS_PIPE_JOINT");  // experiments build only
  return !(e && std::string(e) == "0");
}()};
std::atomic<bool> g_pipe_lag1{[] {
  const char* e = experiment_env("MXS_PIPE_LAG1");  // experiments build only
  return !(e && std::string(e) == "0");
}()};
std::atomic<bool> g_pipe_balanced{[] {
  const char* e = experiment_env("MXS_PIPE_BALANCED");  // experiments build only
  return !(e && std::string(e) == "0");
}()};
}  // namespace
void set_gpu_share(int processes) { g_gpu_share.store(std::max(1, processes), std::memory_order_relaxed); }
int gpu_share() { return g_gpu_share.load(std::memory_order_relaxed); }
void set_pipe_joint(bool on) { g_pipe_joint.store(on, std::memory_order_relaxed); }
bool pipe_joint() { return g_pipe_joint.load(std::memory_order_relaxed); }
void set_pipe_lag1(bool on) { g_pipe_lag1.store(on, std::memory_order_relaxed); }
bool pipe_lag1() { return g_pipe_lag1.load(std::memory_order_relaxed); }
bool last_pipe_lag1() { return g_last_lag1.load(std::memory_order_relaxed); }
void set_pipe_balanced(bool on) { g_pipe_balanced.store(on, std::memory_order_relaxed); }
bool pipe_balanced_on() { return g_pipe_balanced.load(std::memory_order_relaxed); }
namespace detail {
bool pipe_balanced() { return g_pipe_balanced.load(std::memory_order_relaxed); }
void pipe_starts(index_t groups, index_t rows, int blocks, index_t fill, PipeShares* out) {
  struct Entry {
    index_t groups, rows, fill;
    int blocks;
    std::vector<std::int64_t> start;
  };
  thread_local std::vector<Entry> cache;
  const Entry* hit = nullptr;
  for (const auto& e : cache)
    if (e.groups == groups && e.rows == rows && e.fill == fill && e.blocks == blocks) hit = &e;
  if (!hit) {
    if (cache.size() >= 16) cache.erase(cache.begin());
    cache.push_back(Entry{groups, rows, fill, blocks, balanced_starts(groups, rows, blocks, fill)});
    hit = &cache.back();
  }
  out->n = blocks;
  for (int w = 0; w <= blocks; ++w) out->start[w] = int(hit->start[size_t(w)]);
}
void note_dispatch(const char* k) { note(k); }
void note_pipe_lag1(bool lag1) { g_last_lag1.store(lag1, std::memory_order_relaxed); }
}  // namespace detail

#define MXS_INST_STENCIL(T)                                                                                    \
  template void stencil5_rows<T>(const T*, T*, const TileGeom&, index_t, index_t, Stencil5Coeffs, hipStream_t, \
                                 StencilVariant);                                                              \
  template void stencil5_rect<T>(const T*, T*, const TileGeom&, index_t, index_t, index_t, index_t,             \
                                 Stencil5Coeffs, hipStream_t);                                                 \
  template void stencil5_periodic<T>(const T*, T*, const TileGeom&, Stencil5Coeffs, hipStream_t);              \
  template void stencil5_tb<T>(const T*, T*, const TileGeom&, int, index_t, index_t, index_t, index_t,          \
                               Stencil5Coeffs, bool, hipStream_t, StencilVariant);                             \
  template bool stencil5_periodic_supported<T>(const TileGeom&);                                               \
  template void stencil_box<T>(const T*, T*, const TileGeom&, index_t, index_t, index_t, index_t,               \
                               const BoxWeights&, hipStream_t);
MXS_INST_STENCIL(float)
MXS_INST_STENCIL(double)

}  // namespace kernels
}  // namespace mxs
