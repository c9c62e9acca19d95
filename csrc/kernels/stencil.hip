// 2D stencil update kernels (K10; not present in the reference, whose Compute()
// is empty: stencil2d/mpi-2d-stencil-subarray-cuda.cu:32-33).
//
// Regime: a 5-point Jacobi sweep moves 2 x sizeof(T) bytes of compulsory HBM
// traffic per cell (read u, write u') for ~6 flops: HBM-bound by two orders of
// magnitude. The design goal is therefore "every input byte crosses HBM once,
// with enough bytes in flight per CU", not arithmetic.
//
// Variant RegisterRoll (default):
//   * a wave owns a 64 x VEC column segment (VEC = 16 B / sizeof(T): 256 fp32
//     or 128 fp64 columns) and walks a strip of ROWS rows top to bottom;
//   * each lane issues one 16-byte load per row (global_load_dwordx4, a whole
//     1 KiB wave-instruction on aligned rows: TileGeom::aligned) and keeps a
//     rolling 3-row window (up / mid / down) in registers, so vertical reuse
//     costs nothing and every input element is fetched from HBM once per strip;
//   * horizontal neighbours come from the adjacent lane by a wave shuffle
//     (x-1 of the first element, x+1 of the last); only lanes 0 and 63 load the
//     single column just outside the segment;
//   * rows are processed in chunks of CH: the CH row loads of a chunk are issued
//     back to back before any arithmetic, so each wave keeps CH KiB in flight
//     (Little's law: ~50 KiB per CU covers HBM latency at 6+ TB/s);
//   * 4 waves per workgroup take 4 vertically adjacent strips of the same
//     columns, so the two rows a strip re-reads at its ends are L2 hits.
// Variant LdsTile: the textbook LDS-staged tile (a (TH+2) x (TW+2) input tile
//   staged once per workgroup with 16-byte loads, five LDS reads per output).
//   Kept as the measured alternative (see profiles/ and docs/PERF.md).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "mxs/core/error.hpp"
#include "mxs/kernels/kernels.hpp"

namespace mxs {
namespace kernels {
namespace {

template <typename T>
struct Vec16 {
  static constexpr int N = 16 / sizeof(T);
  using type = T __attribute__((ext_vector_type(N)));
};

template <typename T>
__device__ __forceinline__ T fma_t(T a, T b, T c);
template <>
__device__ __forceinline__ float fma_t<float>(float a, float b, float c) { return __builtin_fmaf(a, b, c); }
template <>
__device__ __forceinline__ double fma_t<double>(double a, double b, double c) { return __builtin_fma(a, b, c); }

// One output cell, fixed evaluation order (see kernels.hpp).
template <typename T>
__device__ __forceinline__ T jac(T c, T n, T s, T w, T e, T c0, T c1) {
  return fma_t<T>(c1, (n + s) + (w + e), c0 * c);
}

constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWavesPerBlock * kWaveSize;

// ------------------------------------------------------------- RegisterRoll
template <typename T, int ROWS, int CH, bool NT>
__global__ __launch_bounds__(kBlock) void stencil5_roll_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                               index_t pitch, index_t core_off, index_t W,
                                                               index_t row_begin, index_t row_end, T c0, T c1) {
  static_assert(ROWS % CH == 0, "ROWS must be a multiple of CH");
  constexpr int N = Vec16<T>::N;
  constexpr int SEG = kWaveSize * N;
  using V = typename Vec16<T>::type;

  const int lane = threadIdx.x & (kWaveSize - 1);
  const int wave = threadIdx.x / kWaveSize;
  const index_t seg_base = index_t(blockIdx.x) * SEG;
  const index_t x = seg_base + index_t(lane) * N;
  const index_t y0 = row_begin + (index_t(blockIdx.y) * kWavesPerBlock + wave) * ROWS;
  if (y0 >= row_end) return;  // wave-uniform exit
  const index_t y1 = y0 + ROWS < row_end ? y0 + ROWS : row_end;

  const bool load_ok = x < W + N;  // covers the lane right after the last core vector
  const bool active = x < W;
  const bool right_edge = (lane == kWaveSize - 1) && (seg_base + SEG <= W);
  const T* __restrict__ pin = in + core_off + x;
  T* __restrict__ pout = out + core_off + x;

  auto ldv = [&](index_t y) -> V {
    V v = V(T(0));
    if (load_ok) v = *reinterpret_cast<const V*>(pin + y * pitch);
    return v;
  };
  auto lde = [&](index_t y) -> T {
    T e = T(0);
    if (lane == 0) e = pin[y * pitch - 1];
    else if (right_edge) e = pin[y * pitch + N];
    return e;
  };
  auto emit = [&](index_t y, const V& up, const V& mid, const V& dn, T emid) {
    T left = __shfl_up(mid[N - 1], 1);
    T right = __shfl_down(mid[0], 1);
    if (lane == 0) left = emid;
    if (lane == kWaveSize - 1) right = emid;
    V o;
    o[0] = jac<T>(mid[0], up[0], dn[0], left, mid[1 % N], c0, c1);
    if constexpr (N == 2) {
      o[1] = jac<T>(mid[1], up[1], dn[1], mid[0], right, c0, c1);
    } else {
#pragma unroll
      for (int i = 1; i < N - 1; ++i) o[i] = jac<T>(mid[i], up[i], dn[i], mid[i - 1], mid[i + 1], c0, c1);
      o[N - 1] = jac<T>(mid[N - 1], up[N - 1], dn[N - 1], mid[N - 2], right, c0, c1);
    }
    if (active) {
      T* p = pout + y * pitch;
      if (x + N <= W) {
        if constexpr (NT) __builtin_nontemporal_store(o, reinterpret_cast<V*>(p));
        else *reinterpret_cast<V*>(p) = o;
      } else {
#pragma unroll
        for (int i = 0; i < N; ++i)
          if (x + i < W) p[i] = o[i];
      }
    }
  };

  V up = ldv(y0 - 1);
  V mid = ldv(y0);
  T emid = lde(y0);

  if (y1 - y0 == ROWS) {
    // Full strip: chunks of CH rows, loads of a chunk issued before its math.
#pragma unroll 1
    for (int c = 0; c < ROWS; c += CH) {
      V dn[CH];
      T edn[CH];
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        dn[k] = ldv(y0 + c + k + 1);
        edn[k] = lde(y0 + c + k + 1);
      }
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        emit(y0 + c + k, up, mid, dn[k], emid);
        up = mid;
        mid = dn[k];
        emid = edn[k];
      }
    }
  } else {
#pragma unroll 1
    for (index_t y = y0; y < y1; ++y) {
      const V dn = ldv(y + 1);
      const T edn = lde(y + 1);
      emit(y, up, mid, dn, emid);
      up = mid;
      mid = dn;
      emid = edn;
    }
  }
}

// ----------------------------------------------------------------- LdsTile
// Workgroup tile: TW = 64*N columns x TH rows of outputs, 256 threads.
template <typename T, int TH>
__global__ __launch_bounds__(kBlock) void stencil5_lds_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                              index_t pitch, index_t core_off, index_t W,
                                                              index_t row_begin, index_t row_end, T c0, T c1) {
  constexpr int N = Vec16<T>::N;
  constexpr int TW = kWaveSize * N;
  constexpr int LW = TW + 2 * N;  // staged row: one extra vector on each side (keeps 16 B alignment)
  using V = typename Vec16<T>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  T* tile = reinterpret_cast<T*>(smem_raw);  // (TH + 2) x LW

  const index_t x0 = index_t(blockIdx.x) * TW;
  const index_t y0 = row_begin + index_t(blockIdx.y) * TH;
  const index_t rows = (y0 + TH <= row_end) ? TH : (row_end - y0);
  const int nvec = LW / N;  // vectors per staged row
  // Stage rows y0-1 .. y0+rows (inclusive), columns x0-N .. x0+TW+N-1.
  for (int i = threadIdx.x; i < (rows + 2) * nvec; i += kBlock) {
    const int r = i / nvec, v = i - r * nvec;
    const index_t gx = x0 - N + index_t(v) * N;
    V val = V(T(0));
    if (gx < W + N) val = *reinterpret_cast<const V*>(in + core_off + (y0 - 1 + r) * pitch + gx);
    *reinterpret_cast<V*>(tile + r * LW + v * N) = val;
  }
  __syncthreads();
  // Each thread: one column group of N, rows strided by 4 (one wave per row).
  const int lane = threadIdx.x & (kWaveSize - 1);
  const int wave = threadIdx.x / kWaveSize;
  const index_t x = x0 + index_t(lane) * N;
  if (x >= W) return;
  for (int r = wave; r < rows; r += kWavesPerBlock) {
    const T* up = tile + r * LW + N + lane * N;
    const T* mid = up + LW;
    const T* dn = mid + LW;
    V o;
#pragma unroll
    for (int i = 0; i < N; ++i) o[i] = jac<T>(mid[i], up[i], dn[i], mid[i - 1], mid[i + 1], c0, c1);
    T* p = out + core_off + (y0 + r) * pitch + x;
    if (x + N <= W) {
      *reinterpret_cast<V*>(p) = o;
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i)
        if (x + i < W) p[i] = o[i];
    }
  }
}

// ------------------------------------------------------------------ rect
template <typename T>
__global__ __launch_bounds__(kBlock) void stencil5_rect_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                               index_t pitch, index_t core_off, index_t x0,
                                                               index_t w, index_t y0, index_t h, T c0, T c1) {
  const index_t n = w * h;
  const index_t stride = index_t(gridDim.x) * blockDim.x;
  for (index_t i = index_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    const index_t yy = i / w, xx = i - yy * w;
    const index_t o = core_off + (y0 + yy) * pitch + (x0 + xx);
    out[o] = jac<T>(in[o], in[o - pitch], in[o + pitch], in[o - 1], in[o + 1], c0, c1);
  }
}

// -------------------------------------------------------------- box (LDS)
// Output tile 64 x 16 per 256-thread workgroup: thread (tx, ty) computes column
// tx, rows 4*ty .. 4*ty+3. The (16+2R) x (64+2R) input tile is staged in LDS once;
// every output then reads its (2R+1)^2 taps from LDS, rolling down the 4 rows.
template <typename T, int R>
__global__ __launch_bounds__(kBlock) void stencil_box_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                             index_t pitch, index_t core_off, index_t x0,
                                                             index_t w, index_t y0, index_t h, BoxWeights bw) {
  constexpr int TW = 64, TH = 16, LW = TW + 2 * R + 1;  // +1 breaks the power-of-two row stride
  constexpr int LH = TH + 2 * R, K = 2 * R + 1;
  __shared__ T tile[LH * LW];
  const index_t bx = x0 + index_t(blockIdx.x) * TW;
  const index_t by = y0 + index_t(blockIdx.y) * TH;
  for (int i = threadIdx.x; i < LH * (TW + 2 * R); i += kBlock) {
    const int r = i / (TW + 2 * R), c = i - r * (TW + 2 * R);
    const index_t gx = bx - R + c, gy = by - R + r;
    // Cells past the rectangle are never written; clamp reads to the tile + ghost ring.
    T v = T(0);
    if (gx < x0 + w + R && gy < y0 + h + R) v = in[core_off + gy * pitch + gx];
    tile[r * LW + c] = v;
  }
  __syncthreads();
  float wk[K * K];
#pragma unroll
  for (int i = 0; i < K * K; ++i) wk[i] = bw.w[i];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const index_t gx = bx + tx;
  if (gx >= x0 + w) return;
#pragma unroll
  for (int rr = 0; rr < 4; ++rr) {
    const int r = ty * 4 + rr;
    const index_t gy = by + r;
    if (gy >= y0 + h) break;
    T acc = T(0);
#pragma unroll
    for (int ky = 0; ky < K; ++ky)
#pragma unroll
      for (int kx = 0; kx < K; ++kx) acc = fma_t<T>(T(wk[ky * K + kx]), tile[(r + ky) * LW + tx + kx], acc);
    out[core_off + gy * pitch + gx] = acc;
  }
}

// Tuned defaults (see docs/PERF.md for the sweep behind them).
constexpr int kRollRows = 32;
constexpr int kRollChunk = 8;
constexpr int kLdsRows = 16;

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
  } else {
    const index_t gy = (rows + index_t(kWavesPerBlock) * kRollRows - 1) / (index_t(kWavesPerBlock) * kRollRows);
    stencil5_roll_kernel<T, kRollRows, kRollChunk, true><<<dim3(unsigned(gx), unsigned(gy)), kBlock, 0, s>>>(
        in, out, g.pitch, g.core_offset(), g.width, row_begin, row_end, c0, c1);
  }
  MXS_HIP_CHECK_LAUNCH();
}

template <typename T>
void stencil5_rect(const T* in, T* out, const TileGeom& g, index_t x0, index_t x1, index_t y0, index_t y1,
                   Stencil5Coeffs c, hipStream_t s) {
  if (x1 <= x0 || y1 <= y0) return;
  MXS_CHECK(g.halo_x >= 1 && g.halo_y >= 1, "stencil5 needs a ghost ring of at least 1");
  MXS_CHECK(x0 >= 0 && y0 >= 0 && x1 <= g.width && y1 <= g.height, "rect out of the core");
  const index_t n = (x1 - x0) * (y1 - y0);
  const index_t blocks = std::min<index_t>((n + kBlock - 1) / kBlock, index_t(kNumCUs) * 8);
  stencil5_rect_kernel<T><<<unsigned(blocks), kBlock, 0, s>>>(in, out, g.pitch, g.core_offset(), x0, x1 - x0, y0,
                                                              y1 - y0, T(c.center), T(c.neighbor));
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
  MXS_HIP_CHECK_LAUNCH();
}

#define MXS_INST_STENCIL(T)                                                                                    \
  template void stencil5_rows<T>(const T*, T*, const TileGeom&, index_t, index_t, Stencil5Coeffs, hipStream_t, \
                                 StencilVariant);                                                              \
  template void stencil5_rect<T>(const T*, T*, const TileGeom&, index_t, index_t, index_t, index_t,             \
                                 Stencil5Coeffs, hipStream_t);                                                 \
  template void stencil_box<T>(const T*, T*, const TileGeom&, index_t, index_t, index_t, index_t,               \
                               const BoxWeights&, hipStream_t);
MXS_INST_STENCIL(float)
MXS_INST_STENCIL(double)

}  // namespace kernels
}  // namespace mxs
