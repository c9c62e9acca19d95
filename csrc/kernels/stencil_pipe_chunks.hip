// Chunk-list pipeline pass of the interior-first multi-GPU super-step
// (kernels.hpp: chunk_pass_shape / stencil5_chunk_pass; device body
// stencil5_pipe_chunks_kernel in stencil_device.hpp; chunk lists
// kernels/chunk_schedule.hpp). The forms mirror launch_pipe_impl's choice for a
// ghost-ring tile, so the split pass runs exactly the kernel body the one-launch
// pass runs: fp32 S = 20 (8 + 12 or 12 + 8, ascending levels on short chunks)
// and S = 24 (12 + 12), fp64 S = 16 (8 + 8), each in the sum and the per-step
// form. Other depths keep the one-launch pass.
#include <cmath>
#include <limits>

#include "stencil_pipe.hpp"

namespace mxs {
namespace kernels {
namespace detail {
namespace {

template <typename T, int S, bool SUM, int JS0, int LAG1, int XB = 0>
constexpr auto chunks_kernel() {
  return stencil5_pipe_chunks_kernel<JS0, S - JS0, pipe_pf<T, S>(), T, SUM, LAG1, XB>;
}

template <typename T, int S, bool SUM, int JS0, int LAG1>
void fill_shape(const TileGeom& g, ChunkPassShape* out) {
  constexpr int OWG = JointShape<JS0, S - JS0, kWavesPerBlock>::OWG;
  static int blocks = 0;
  if (blocks == 0) {
    int occ = 0;
    MXS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &occ, reinterpret_cast<const void*>(chunks_kernel<T, S, SUM, JS0, LAG1>()), 2 * kBlock, 0));
    blocks = std::max(occ, 1) * device_cu_count();
  }
  out->steps = S;
  out->sum = SUM;
  out->js0 = JS0;
  out->lag1 = LAG1;
  out->blocks = std::max(1, blocks / gpu_share());
  out->owg = OWG;
  out->groups = (g.width + OWG - 1) / OWG;
  out->fill = pipe_fill_rows<JS0, S - JS0, pipe_pf<T, S>(), LAG1>();
  using J = JointShape<JS0, S - JS0, kWavesPerBlock>;
  out->read_lead = J::LEAD;
  out->read_span = (kWavesPerBlock - 1) * J::OW0 + 256;
}

template <typename T, int S, bool SUM>
bool shape_for(const TileGeom& g, ChunkPassShape* out) {
  if (!pipe_joint()) return false;  // the per-strip layout has no chunk-list form
  const index_t W = g.width, H = g.height;
  if constexpr (sizeof(T) == 4 && S == 20) {
    if (pipe_lag1() && pipe_share<T, S, false, SUM, 12>(0, W, 0, H) <= kLag1MaxChunk) {
      if (W < kJointWide) fill_shape<T, S, SUM, 8, kLagBoth>(g, out);
      else fill_shape<T, S, SUM, 12, kLagBoth>(g, out);
    } else {
      fill_shape<T, S, SUM, joint_s0<T, S>(), 0>(g, out);
    }
    return true;
  } else if constexpr (sizeof(T) == 4 && S == 24) {
    if (pipe_lag1()) fill_shape<T, S, SUM, 12, kLagBoth>(g, out);
    else fill_shape<T, S, SUM, joint_s0<T, S>(), 0>(g, out);
    return true;
  } else if constexpr (sizeof(T) == 8 && S == 16) {
    if (!wide_pipe_ok_impl<T, S, false>(g, 0, W, 0, H)) return false;
    if (pipe_lag1() && pipe_share<T, S, false, SUM, 8>(0, W, 0, H) <= kLag1MaxChunkF64)
      fill_shape<T, S, SUM, 8, kLagBoth>(g, out);
    else
      fill_shape<T, S, SUM, 8, 0>(g, out);
    return true;
  }
  return false;
}

template <typename T, int S, bool SUM, int JS0, int LAG1, int XB>
void launch_chunks(const T* in, T* out, const TileGeom& g, T c0, T c1, const ChunkPassShape& sh,
                   const PassChunk* table, int entries, hipStream_t s) {
  chunks_kernel<T, S, SUM, JS0, LAG1, XB>()<<<sh.blocks, 2 * kBlock, 0, s>>>(
      in, out, g.pitch, g.core_offset(), g.width, g.height, 0, g.width, 0, table, entries, c0, c1);
  note_dispatch(XB == kScaledBody ? "stream_pipe_scaled_chunks" : SUM ? "stream_pipe_sum_chunks" : "stream_pipe_chunks");
  note_pipe_lag1(LAG1 != 0);
}

template <typename T, int S, bool SUM, int XB = 0>
void launch_for(const T* in, T* out, const TileGeom& g, T c0, T c1, const ChunkPassShape& sh, const PassChunk* table,
                int entries, hipStream_t s) {
  const bool lag = sh.lag1 != 0;
  if constexpr (sizeof(T) == 4 && S == 20) {
    if (sh.js0 == 8 && lag) return launch_chunks<T, S, SUM, 8, kLagBoth, XB>(in, out, g, c0, c1, sh, table, entries, s);
    if (sh.js0 == 12 && lag) return launch_chunks<T, S, SUM, 12, kLagBoth, XB>(in, out, g, c0, c1, sh, table, entries, s);
    if (sh.js0 == 12) return launch_chunks<T, S, SUM, 12, 0, XB>(in, out, g, c0, c1, sh, table, entries, s);
  } else if constexpr (sizeof(T) == 4 && S == 24) {
    if (sh.js0 == 12 && lag) return launch_chunks<T, S, SUM, 12, kLagBoth, XB>(in, out, g, c0, c1, sh, table, entries, s);
    if (sh.js0 == 12) return launch_chunks<T, S, SUM, 12, 0, XB>(in, out, g, c0, c1, sh, table, entries, s);
  } else if constexpr (sizeof(T) == 8 && S == 16) {
    if (sh.js0 == 8 && lag) return launch_chunks<T, S, SUM, 8, kLagBoth, XB>(in, out, g, c0, c1, sh, table, entries, s);
    if (sh.js0 == 8) return launch_chunks<T, S, SUM, 8, 0, XB>(in, out, g, c0, c1, sh, table, entries, s);
  }
  MXS_CHECK(false, "stencil5_chunk_pass: no kernel for S = " << S << ", js0 = " << sh.js0 << ", lag1 = " << sh.lag1);
}

}  // namespace
}  // namespace detail

template <typename T>
bool chunk_pass_shape(const TileGeom& g, int steps, const Stencil5Coeffs& c, ChunkPassShape* out) {
  using namespace detail;
  constexpr index_t N = 16 / index_t(sizeof(T));
  if (g.width % 4 != 0 || g.width < 4 * kWaveSize || g.height < 2 * steps) return false;
  if (g.halo_x < steps || g.halo_y < steps) return false;
  if ((g.pitch % N) != 0 || ((g.x_origin + g.halo_x) % N) != 0) return false;
  const index_t sa = (steps + 3) / 4 * 4;  // the joint read reach A0 + A1
  if (g.x_origin + g.halo_x < sa || g.pitch < g.x_origin + g.halo_x + (g.width + 3) / 4 * 4 + sa) return false;
  // Entries longer than kMaxChunkBytes run in pieces (stencil5_pipe_chunks_kernel).
  if (g.pitch * index_t(sizeof(T)) * kMinChunkRows > kMaxChunkBytes) return false;
  // Fast forms only inside their bounds (kernels.hpp: fast_form_safe).
  const bool fast = fast_form_safe<T>(c, steps);
  const bool scaled = fast && uses_scaled_form(c);
  const bool sum = fast;  // both fast forms share the sum-form shape
  ChunkPassShape sh;
  bool ok = false;
  if constexpr (sizeof(T) == 4) {
    if (steps == 20) ok = sum ? shape_for<T, 20, true>(g, &sh) : shape_for<T, 20, false>(g, &sh);
    if (steps == 24) ok = sum ? shape_for<T, 24, true>(g, &sh) : shape_for<T, 24, false>(g, &sh);
  } else {
    if (steps == 16) ok = sum ? shape_for<T, 16, true>(g, &sh) : shape_for<T, 16, false>(g, &sh);
  }
  sh.scaled = scaled;
  if (ok && out) *out = sh;
  return ok;
}

template <typename T>
void stencil5_chunk_pass(const T* in, T* out, const TileGeom& g, const Stencil5Coeffs& c, const ChunkPassShape& sh,
                         const PassChunk* table, int entries, hipStream_t s) {
  using namespace detail;
  MXS_CHECK(table != nullptr && entries > 0 && sh.blocks > 0, "stencil5_chunk_pass: no schedule");
  ChunkPassShape now;
  MXS_CHECK(chunk_pass_shape<T>(g, sh.steps, c, &now) && now.sum == sh.sum && now.scaled == sh.scaled,
            "stencil5_chunk_pass: shape built for the other evaluation form");
  const T c0 = T(c.center), c1 = T(c.neighbor);
  const T sc = T(std::pow(double(c1), double(sh.steps)));
  // Kernel coefficients: sum form (c^S, c), scaled form (c1^S, c0 / c1), per step (c0, c1).
  const T k0 = sh.sum ? sc : c0;
  // k from the element-type coefficients, exactly as launch_pipe_form forms it:
  // the one-launch and the chunk-list passes must run the same k to stay bitwise equal.
  const T k1 = sh.scaled ? T(double(c0) / double(c1)) : c1;
  if constexpr (sizeof(T) == 4) {
    if (sh.steps == 20) {
      if (sh.scaled) launch_for<T, 20, true, kScaledBody>(in, out, g, k0, k1, sh, table, entries, s);
      else if (sh.sum) launch_for<T, 20, true>(in, out, g, k0, k1, sh, table, entries, s);
      else launch_for<T, 20, false>(in, out, g, k0, k1, sh, table, entries, s);
    } else if (sh.steps == 24) {
      if (sh.scaled) launch_for<T, 24, true, kScaledBody>(in, out, g, k0, k1, sh, table, entries, s);
      else if (sh.sum) launch_for<T, 24, true>(in, out, g, k0, k1, sh, table, entries, s);
      else launch_for<T, 24, false>(in, out, g, k0, k1, sh, table, entries, s);
    } else {
      MXS_CHECK(false, "stencil5_chunk_pass: fp32 depth " << sh.steps);
    }
  } else {
    MXS_CHECK(sh.steps == 16, "stencil5_chunk_pass: fp64 depth " << sh.steps);
    if (sh.scaled) launch_for<T, 16, true, kScaledBody>(in, out, g, k0, k1, sh, table, entries, s);
    else if (sh.sum) launch_for<T, 16, true>(in, out, g, k0, k1, sh, table, entries, s);
    else launch_for<T, 16, false>(in, out, g, k0, k1, sh, table, entries, s);
  }
  MXS_HIP_CHECK_LAUNCH();
}

template bool chunk_pass_shape<float>(const TileGeom&, int, const Stencil5Coeffs&, ChunkPassShape*);
template bool chunk_pass_shape<double>(const TileGeom&, int, const Stencil5Coeffs&, ChunkPassShape*);
template void stencil5_chunk_pass<float>(const float*, float*, const TileGeom&, const Stencil5Coeffs&,
                                         const ChunkPassShape&, const PassChunk*, int, hipStream_t);
template void stencil5_chunk_pass<double>(const double*, double*, const TileGeom&, const Stencil5Coeffs&,
                                          const ChunkPassShape&, const PassChunk*, int, hipStream_t);

}  // namespace kernels
}  // namespace mxs
