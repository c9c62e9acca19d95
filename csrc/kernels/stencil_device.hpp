// Device-side templates of the stencil kernels (included by stencil.hip and by
// the tuning harness bench/stencil_tune.hip so both compile the same code).
// See stencil.hip for the design notes.
#pragma once

#include <hip/hip_runtime.h>

#include "mxs/kernels/kernels.hpp"

namespace mxs {
namespace kernels {
namespace detail {

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
constexpr int kNumXcds = 8;  // MI355X: workgroups are dealt round-robin over 8 XCDs
constexpr int kBlock = kWavesPerBlock * kWaveSize;

// ------------------------------------------------------------- RegisterRoll
// WX waves side by side along x (4/WX stacked along y) per 256-thread workgroup;
// NT = non-temporal (streaming) stores, NTL = non-temporal loads.
// WRAP: periodic wrap-around addressing inside the tile (rows -1 / H map to H-1 / 0,
// columns -1 / W to W-1 / 0) — the fused self-exchange of a 1x1 periodic grid, so
// no ghost cell is read or written. Requires W % VEC == 0.
template <typename T, int ROWS, int CH, bool NT, int WX = 1, bool NTL = false, int NW = kWavesPerBlock,
          bool WRAP = false>
__global__ __launch_bounds__(NW * kWaveSize) void stencil5_roll_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                               index_t pitch, index_t core_off, index_t W,
                                                               index_t row_begin, index_t row_end, T c0, T c1,
                                                               index_t H = 0) {
  static_assert(ROWS % CH == 0, "ROWS must be a multiple of CH");
  constexpr int N = Vec16<T>::N;
  constexpr int SEG = kWaveSize * N;
  using V = typename Vec16<T>::type;

  const int lane = threadIdx.x & (kWaveSize - 1);
  const int wave = threadIdx.x / kWaveSize;
  constexpr int WY = NW / WX;
  static_assert(NW % WX == 0, "WX must divide the waves per workgroup");
  const int wx = wave % WX, wy = wave / WX;
  const index_t seg_base = (index_t(blockIdx.x) * WX + wx) * SEG;
  const index_t x = seg_base + index_t(lane) * N;
  const index_t y0 = row_begin + (index_t(blockIdx.y) * WY + wy) * ROWS;
  if (y0 >= row_end) return;  // wave-uniform exit
  const index_t y1 = y0 + ROWS < row_end ? y0 + ROWS : row_end;

  const bool load_ok = x < W + N;  // covers the lane right after the last core vector
  const bool active = x < W;
  // Lane whose x+1 neighbour of its last element is not in the next lane's vector:
  // lane 63 (next segment), or under WRAP the lane holding column W-1.
  const bool right_lane = (lane == kWaveSize - 1) || (WRAP && x + N == W);
  const bool right_load = WRAP ? right_lane && active : (lane == kWaveSize - 1) && (seg_base + SEG <= W);
  // Column offsets (relative to x) of the two edge values.
  const index_t left_col = (WRAP && x == 0) ? W - 1 : -1;
  const index_t right_col = (WRAP && x + N == W) ? -x : N;
  const T* __restrict__ pin = in + core_off + x;
  T* __restrict__ pout = out + core_off + x;

  auto row = [&](index_t y) -> index_t {
    if constexpr (WRAP) return y < 0 ? y + H : (y >= H ? y - H : y);
    else return y;
  };
  auto ldv = [&](index_t y) -> V {
    V v = V(T(0));
    const index_t r = row(y);
    if (load_ok) {
      if constexpr (NTL) v = __builtin_nontemporal_load(reinterpret_cast<const V*>(pin + r * pitch));
      else v = *reinterpret_cast<const V*>(pin + r * pitch);
    }
    return v;
  };
  struct Edge {
    T l, r;
  };
  auto lde = [&](index_t y) -> Edge {
    Edge e{T(0), T(0)};
    const index_t r = row(y);
    if (lane == 0) e.l = pin[r * pitch + left_col];
    if (right_load) e.r = pin[r * pitch + right_col];
    return e;
  };
  auto emit = [&](index_t y, const V& up, const V& mid, const V& dn, Edge emid) {
    T left = __shfl_up(mid[N - 1], 1);
    T right = __shfl_down(mid[0], 1);
    if (lane == 0) left = emid.l;
    if (right_lane) right = emid.r;
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
  Edge emid = lde(y0);

  if (y1 - y0 == ROWS) {
    // Full strip: chunks of CH rows, loads of a chunk issued before its math.
#pragma unroll 1
    for (int c = 0; c < ROWS; c += CH) {
      V dn[CH];
      Edge edn[CH];
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
      const Edge edn = lde(y + 1);
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

}  // namespace detail
}  // namespace kernels
}  // namespace mxs

namespace mxs {
namespace kernels {
namespace detail {

// LDS bytes of the ping-pong LDS tile (bench/tune_kernels.hpp: stencil5_tb_kernel,
// the tuner's alternative); the single-buffer tile below takes half.
template <typename T, int S, int TW, int TH>
constexpr size_t tb_lds_bytes() {
  constexpr int N = Vec16<T>::N;
  constexpr int SA = ((S + N - 1) / N) * N;
  return size_t(2) * (TH + 2 * S) * (TW + 2 * SA + 2 * N) * sizeof(T);
}

}  // namespace detail
}  // namespace kernels
}  // namespace mxs

namespace mxs {
namespace kernels {
namespace detail {

// Single-LDS-buffer variant of stencil5_tb_kernel: each step reads its cells into
// registers (a compile-time number of vectors per thread, statically indexed so
// they stay in VGPRs), barrier, writes them back in place, barrier. Half the LDS
// of the ping-pong form, so more workgroups per CU keep HBM busy while others
// compute.
template <typename T, int S, int TW, int TH, bool WRAP>
__global__ __launch_bounds__(256) void stencil5_tb1_kernel(const T* __restrict__ in, T* __restrict__ out, index_t pitch,
                                                          index_t core_off, index_t W, index_t H, index_t x_begin,
                                                          index_t x_end, index_t y_begin, index_t y_end, T c0, T c1) {
  constexpr int N = Vec16<T>::N;
  constexpr int SA = ((S + N - 1) / N) * N;
  constexpr int LW = TW + 2 * SA;
  constexpr int LP = LW + 2 * N;
  constexpr int LH = TH + 2 * S;
  constexpr int NV = LW / N;
  constexpr int CELLS = (LH - 2) * NV;            // vectors updated per step
  constexpr int PER = (CELLS + 255) / 256;        // per thread
  static_assert(TW % N == 0, "tile width must be a multiple of the vector width");
  using V = typename Vec16<T>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_tb1[];
  T* buf = reinterpret_cast<T*>(smem_tb1);

  const index_t tx0 = x_begin + index_t(blockIdx.x) * TW;
  const index_t ty0 = y_begin + index_t(blockIdx.y) * TH;
  const int tid = threadIdx.x;
  // Staged coordinates stay within one period of the tile unless the tile is
  // smaller than the workgroup's footprint: then fall back to a full modulo.
  const bool one_period = W >= TW + 2 * SA && H >= TH + 2 * S;

  for (int i = tid; i < LH * NV; i += 256) {
    const int r = i / NV, v = i - r * NV;
    index_t gy = ty0 - S + r;
    index_t gx = tx0 - SA + index_t(v) * N;
    V val = V(T(0));
    bool ok;
    if constexpr (WRAP) {
      if (one_period) {
        gy = gy < 0 ? gy + H : (gy >= H ? gy - H : gy);
        gx = gx < 0 ? gx + W : (gx >= W ? gx - W : gx);
      } else {
        gy = ((gy % H) + H) % H;
        gx = ((gx % W) + W) % W;
      }
      ok = true;
    } else {
      ok = gy < H + S && gx < W + SA;
    }
    if (ok) val = *reinterpret_cast<const V*>(in + core_off + gy * pitch + gx);
    *reinterpret_cast<V*>(buf + r * LP + N + v * N) = val;
  }
  __syncthreads();

#pragma unroll 1
  for (int s = 0; s < S; ++s) {
    V res[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = tid + k * 256;
      if (i < CELLS) {
        const int r = 1 + i / NV, v = i - (r - 1) * NV;
        const int base = r * LP + N + v * N;
        const V mid = *reinterpret_cast<const V*>(buf + base);
        const V up = *reinterpret_cast<const V*>(buf + base - LP);
        const V dn = *reinterpret_cast<const V*>(buf + base + LP);
        const T left = buf[base - 1];
        const T right = buf[base + N];
        V o;
        o[0] = jac<T>(mid[0], up[0], dn[0], left, mid[1 % N], c0, c1);
        if constexpr (N == 2) {
          o[1] = jac<T>(mid[1], up[1], dn[1], mid[0], right, c0, c1);
        } else {
#pragma unroll
          for (int q = 1; q < N - 1; ++q) o[q] = jac<T>(mid[q], up[q], dn[q], mid[q - 1], mid[q + 1], c0, c1);
          o[N - 1] = jac<T>(mid[N - 1], up[N - 1], dn[N - 1], mid[N - 2], right, c0, c1);
        }
        res[k] = o;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int i = tid + k * 256;
      if (i < CELLS) {
        const int r = 1 + i / NV, v = i - (r - 1) * NV;
        *reinterpret_cast<V*>(buf + r * LP + N + v * N) = res[k];
      }
    }
    __syncthreads();
  }

  constexpr int OV = TW / N;
  for (int i = tid; i < TH * OV; i += 256) {
    const int r = i / OV, v = i - r * OV;
    const index_t gy = ty0 + r, gx = tx0 + index_t(v) * N;
    if (gy >= y_end || gx >= x_end) continue;
    const V o = *reinterpret_cast<const V*>(buf + (r + S) * LP + N + SA + v * N);
    T* p = out + core_off + gy * pitch + gx;
    if (gx + N <= x_end) {
      __builtin_nontemporal_store(o, reinterpret_cast<V*>(p));
    } else {
#pragma unroll
      for (int k = 0; k < N; ++k)
        if (gx + k < x_end) p[k] = o[k];
    }
  }
}

template <typename T, int S, int TW, int TH>
constexpr size_t tb1_lds_bytes() {
  return tb_lds_bytes<T, S, TW, TH>() / 2;
}

// One vector of outputs from its three rows and the two scalars beside `mid`.
template <typename T, typename V, int N>
__device__ __forceinline__ V jac_vec(const V& up, const V& mid, const V& dn, T left, T right, T c0, T c1) {
  V o;
  o[0] = jac<T>(mid[0], up[0], dn[0], left, mid[1 % N], c0, c1);
  if constexpr (N == 2) {
    o[1] = jac<T>(mid[1], up[1], dn[1], mid[0], right, c0, c1);
  } else {
#pragma unroll
    for (int q = 1; q < N - 1; ++q) o[q] = jac<T>(mid[q], up[q], dn[q], mid[q - 1], mid[q + 1], c0, c1);
    o[N - 1] = jac<T>(mid[N - 1], up[N - 1], dn[N - 1], mid[N - 2], right, c0, c1);
  }
  return o;
}

// fp32 x4 form written on aligned register pairs, so the backend emits packed
// v_pk_{add,mul,fma}_f32 without pair-building moves; the horizontal sums are
// scalar adds written straight into pairs. Same per-element operations and
// order as jac() (IEEE add is commutative), so results are bitwise identical.
using f32x2 = float __attribute__((ext_vector_type(2)));
using f32x4 = float __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f32x4 jac_vec4f(const f32x4& up, const f32x4& mid, const f32x4& dn, float left,
                                           float right, float c0, float c1) {
  const f32x2 ns_lo = up.xy + dn.xy, ns_hi = up.zw + dn.zw;
  f32x2 we_lo, we_hi;
  we_lo.x = left + mid.y;
  we_lo.y = mid.x + mid.z;
  we_hi.x = mid.y + mid.w;
  we_hi.y = mid.z + right;
  const f32x2 c0v = f32x2(c0), c1v = f32x2(c1);
  const f32x2 lo = __builtin_elementwise_fma(c1v, ns_lo + we_lo, c0v * mid.xy);
  const f32x2 hi = __builtin_elementwise_fma(c1v, ns_hi + we_hi, c0v * mid.zw);
  f32x4 o;
  o.xy = lo;
  o.zw = hi;
  return o;
}

template <typename T, typename V>
__device__ __forceinline__ V jac_row(const V& up, const V& mid, const V& dn, T left, T right, T c0, T c1) {
  if constexpr (sizeof(T) == 4) return jac_vec4f(up, mid, dn, left, right, c0, c1);
  else return jac_vec<T, V, Vec16<T>::N>(up, mid, dn, left, right, c0, c1);
}

// ------------------------------------------------------- wave-streaming blocks
// Temporal blocking without LDS and without vertical recompute. Each wave owns a
// column strip (64 lanes x one 16-byte vector = 256 fp32 / 128 fp64 columns, of
// which the outer SA columns per side are apron) and streams down a chunk of CH
// rows. It keeps a three-row window per time level in registers: when input row
// y arrives, level 1 row y-1 is computed from level-0 rows y-2..y, level 2 row
// y-2 from level-1 rows y-3..y-1, ..., level S row y-S is stored. Row neighbours
// come from the same lane's window; column neighbours from the adjacent lanes
// through ds_bpermute. Every level advances once per input row, so HBM sees one
// read and one write per cell per S steps (plus 2S/CH rows and 2SA/256 columns
// of redundant apron). The window is three register slots per level used
// round-robin (the loop is unrolled by a multiple of 3), so no row is ever
// copied between registers: VALU work is just the stencil arithmetic.
template <typename T>
__device__ __forceinline__ T lane_fetch(T v, int byte_addr);
template <>
__device__ __forceinline__ float lane_fetch<float>(float v, int a) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(a, __float_as_int(v)));
}
template <>
__device__ __forceinline__ double lane_fetch<double>(double v, int a) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(a, int(b & 0xffffffff));
  const int hi = __builtin_amdgcn_ds_bpermute(a, int(b >> 32));
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

// Whole-wavefront DPP shifts (CDNA keeps the GFX9 wave_shr / wave_shl controls):
// lane i reads lane i-1 (kDppWaveShr1) or lane i+1 (kDppWaveShl1); the shifted-in
// lane gets 0. As a DPP source modifier the shift folds into the consuming
// v_add_f32, so a column neighbour costs no instruction and no LDS round trip.
constexpr int kDppWaveShl1 = 0x130;
constexpr int kDppWaveShr1 = 0x138;
template <typename T, int CTRL>
__device__ __forceinline__ T lane_shift(T v);
template <>
__device__ __forceinline__ float lane_shift<float, kDppWaveShr1>(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), kDppWaveShr1, 0xf, 0xf, true));
}
template <>
__device__ __forceinline__ float lane_shift<float, kDppWaveShl1>(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), kDppWaveShl1, 0xf, 0xf, true));
}
// 64-bit DPP takes no wave shifts: two dword moves. bound_ctrl zero-fills the
// shifted-in lane (0.0), so no zeroed `old` register (one v_mov each) is needed.
template <>
__device__ __forceinline__ double lane_shift<double, kDppWaveShr1>(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp(int(b & 0xffffffff), kDppWaveShr1, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(int(b >> 32), kDppWaveShr1, 0xf, 0xf, true);
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}
template <>
__device__ __forceinline__ double lane_shift<double, kDppWaveShl1>(double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp(int(b & 0xffffffff), kDppWaveShl1, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp(int(b >> 32), kDppWaveShl1, 0xf, 0xf, true);
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

// ------------------------------------------------ rotated-pair fp32 layout
// Measured on the S = 16 stream kernel (scripts/isa_mix.py): with the natural
// register layout (c0 c1 | c2 c3) the horizontal sums (c[i-1] + c[i+1]) straddle
// the 64-bit pairs the packed VALU works on, so the backend builds pairs with 4
// v_mov_b32 and keeps 2 v_mov_b32_dpp: 18 VALU issue slots per level-row, ~75
// cycles at one wave per SIMD. Holding every intermediate row ROTATED as
// A = (c1, c2), B = (c3, c0) makes the in-lane pair (c0 + c2, c3 + c1) one
// v_pk_add_f32 with swapped halves (op_sel), and the two lane-crossing sums
// c2 + c0[lane+1], c1 + c3[lane-1] two v_add_f32 with a DPP wave shift folded
// into the source, written straight into the pair (we3, we0) that lines up with
// B. Per level-row: 9 packed + 2 DPP adds, no moves. Same operations, same
// operand order per cell as jac() (IEEE add is commutative): bitwise identical.
// Only the input rows (natural order from HBM) and the stored top level are
// rotated, once per row each.
__device__ __forceinline__ f32x4 rot_in(const f32x4& n) { return __builtin_shufflevector(n, n, 1, 2, 3, 0); }
__device__ __forceinline__ f32x4 rot_out(const f32x4& r) { return __builtin_shufflevector(r, r, 3, 0, 1, 2); }
// rot_in as two v_pk_mov_b32 into fresh registers. From the shufflevector the
// backend often keeps the rotated row as halves of the loaded registers (the
// op_sel of later adds reads them in place), so the next load into that
// prefetch slot needs other registers and the loop back edge copies them back:
// ~21 v_mov per 6 rows of the fetching stage, plus 4 v_mov instead of 2
// v_pk_mov for some rotations (ISA of the S = 20 pipeline). Copying here ends
// the loaded registers' lifetime at the rotation.
__device__ __forceinline__ f32x4 rot_in_copy(const f32x4& n) {
  const f32x2 lo = n.xy, hi = n.zw;
  f32x2 a, b;
  asm("v_pk_mov_b32 %0, %1, %2 op_sel:[1,0]" : "=v"(a) : "v"(lo), "v"(hi));  // (c1, c2)
  asm("v_pk_mov_b32 %0, %1, %2 op_sel:[1,0]" : "=v"(b) : "v"(hi), "v"(lo));  // (c3, c0)
  return __builtin_shufflevector(a, b, 0, 1, 2, 3);
}

__device__ __forceinline__ f32x4 jac_rot4f(const f32x4& up, const f32x4& mid, const f32x4& dn, float c0, float c1) {
  const f32x2 am = mid.xy, bm = mid.zw;  // (c1, c2), (c3, c0)
  const f32x2 ns_a = up.xy + dn.xy, ns_b = up.zw + dn.zw;
  const f32x2 we_a = bm.yx + am.yx;  // (c0 + c2, c3 + c1)
  f32x2 we_b;
  we_b.x = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(bm.y), kDppWaveShl1, 0xf, 0xf, true)) + am.y;
  we_b.y = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(bm.x), kDppWaveShr1, 0xf, 0xf, true)) + am.x;
  const f32x2 c0v = f32x2(c0), c1v = f32x2(c1);
  const f32x2 oa = __builtin_elementwise_fma(c1v, ns_a + we_a, c0v * am);
  const f32x2 ob = __builtin_elementwise_fma(c1v, ns_b + we_b, c0v * bm);
  f32x4 o;
  o.xy = oa;
  o.zw = ob;
  return o;
}

template <typename T, int S>
struct StreamShape {
  static constexpr int N = Vec16<T>::N;
  static constexpr int SA = ((S + N - 1) / N) * N;      // apron columns per side
  static constexpr int OW = kWaveSize * N - 2 * SA;     // output columns per wave
};

// ------------------------------------------------ wide-lane fp64 layout
// fp64 has no packed VALU and 64-bit DPP cannot take the wave shifts, so the
// natural fp64 form (one 16-byte vector = 2 cells per lane, 128-column strips)
// pays 2 neighbour moves (4 v_mov_b32_dpp) per 2 cells and an apron of 2S of
// 128 columns. Four cells per lane (two 16-byte loads, 256-column strips as
// fp32) halve both: 20 fp64 ops + 4 dword moves per 4 cells, apron 2S of 256.
// Same per-cell operations and order as jac(): bitwise identical.
using f64x2 = double __attribute__((ext_vector_type(2)));
using f64x4 = double __attribute__((ext_vector_type(4)));
// The loaded row into fresh registers (4 v_mov_b64): as rot_in_copy for fp32,
// this ends the prefetch registers' lifetime at entry, so the next load can
// reuse them instead of the loop back edge copying rows around.
__device__ __forceinline__ f64x4 copy_w4d(const f64x4& v) {
  f64x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    double x;
    asm("v_mov_b64 %0, %1" : "=v"(x) : "v"(v[i]));
    r[i] = x;
  }
  return r;
}
__device__ __forceinline__ f64x4 jac_w4d(const f64x4& up, const f64x4& mid, const f64x4& dn, double c0, double c1) {
  const double left = lane_shift<double, kDppWaveShr1>(mid.w);   // lane - 1's last cell
  const double right = lane_shift<double, kDppWaveShl1>(mid.x);  // lane + 1's first cell
  f64x4 o;
  o.x = jac<double>(mid.x, up.x, dn.x, left, mid.y, c0, c1);
  o.y = jac<double>(mid.y, up.y, dn.y, mid.x, mid.z, c0, c1);
  o.z = jac<double>(mid.z, up.z, dn.z, mid.y, mid.w, c0, c1);
  o.w = jac<double>(mid.w, up.w, dn.w, mid.z, right, c0, c1);
  return o;
}

// Per-lane bodies of the branch-free streaming kernels (stream_chunk_fast,
// pipe_chunk): 4 cells per lane in both, so a strip is 256 columns and the
// apron S rounded up to 4. `enter` maps a row loaded from HBM into the
// register layout the levels work on; `store` maps it back and writes one
// lane's 4 cells through the chunk's buffer descriptor (an offset past the
// range is dropped by the hardware range check: no branch, no exec mask).
using u32x4 = unsigned __attribute__((ext_vector_type(4)));
struct BodyRotF32 {  // rotated-pair fp32 (jac_rot4f)
  using T = float;
  using V = f32x4;
  static constexpr int N = 4;
  // A scheduling fence after each row iteration of the pipeline's fetching
  // stage (pipe_chunk): keeps the scheduler from overlapping consecutive rows'
  // level chains, which holds more rows live (see BodySumF64).
  static constexpr bool kStage0Fence = false;
  static __device__ __forceinline__ V zero() { return f32x4(0.f); }
  static __device__ __forceinline__ V load(const float* p) { return *reinterpret_cast<const f32x4*>(p); }
  static __device__ __forceinline__ V enter(const V& v) { return rot_in_copy(v); }
  static __device__ __forceinline__ V jac(const V& u, const V& m, const V& d, float c0, float c1) {
    return jac_rot4f(u, m, d, c0, c1);
  }
  static __device__ __forceinline__ void store(const V& top, __amdgpu_buffer_rsrc_t r, unsigned off, float) {
    const f32x4 nat = rot_out(top);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, nat), r, int(off), 0, 2 /* nt */);
  }
};
struct BodyWideF64 {  // 4 consecutive fp64 cells per lane (jac_w4d)
  using T = double;
  using V = f64x4;
  static constexpr int N = 4;
  static constexpr bool kStage0Fence = false;  // see BodyRotF32
  static __device__ __forceinline__ V zero() { return f64x4(0.0); }
  static __device__ __forceinline__ V load(const double* p) {
    const f64x2 a = *reinterpret_cast<const f64x2*>(p), b = *reinterpret_cast<const f64x2*>(p + 2);
    return __builtin_shufflevector(a, b, 0, 1, 2, 3);
  }
  static __device__ __forceinline__ V enter(const V& v) { return copy_w4d(v); }
  static __device__ __forceinline__ V jac(const V& u, const V& m, const V& d, double c0, double c1) {
    return jac_w4d(u, m, d, c0, c1);
  }
  static __device__ __forceinline__ void store(const V& top, __amdgpu_buffer_rsrc_t r, unsigned off, double) {
    const f64x2 lo = top.xy, hi = top.zw;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, lo), r, int(off), 0, 2 /* nt */);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, hi), r, int(off + 16u), 0, 2 /* nt */);
  }
};

// Sum form (c_center == c_neighbor == c, the default 5-point average). The
// S-level recurrence u' = c * (5-point sum of u) is linear with one uniform
// scale, so a pass carries v_l = u_l / c^l — plain 5-point sums, no multiply —
// and applies c^S once when it stores (the kernels' c0 argument holds c^S).
// The horizontal 3-sums come from pair sums: with p = u[2k] + u[2k+1],
// h3(x) = p(x) + u[x even ? x - 1 : x + 1]. Rotated fp32: 8 VALU issue slots
// per 4 cells and level instead of 11 (2 ns + 1 pair + 1 + 2 DPP h3 + 2 sum);
// wide fp64: 14 fp64 ops + 4 moves instead of 20 + 4. The result equals the
// step-by-step evaluation up to rounding (not bit for bit: different
// association, one scale per pass instead of one per step); magnitudes grow
// as 5^S inside a pass (|u| up to 3e38 / 5^S stays finite).
// (a.x + b.y, a.y + b.x): one v_pk_add_f32 with the halves of src1 swapped by
// op_sel. Written as asm so the swap is never materialised as a register pair
// of its own (from a shufflevector the backend copies swapped pairs with
// v_mov_b32: ~1 per level-row of the sum body, measured in the ISA). Plain
// VALU, no hazard the compiler would have to know about.
__device__ __forceinline__ f32x2 pk_add_swap(const f32x2& a, const f32x2& b) {
  f32x2 r;
  asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0]" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ f32x4 sum_rot4f(const f32x4& up, const f32x4& mid, const f32x4& dn) {
  const f32x2 am = mid.xy, bm = mid.zw;  // (c1, c2), (c3, c0)
  const f32x2 ns_a = up.xy + dn.xy, ns_b = up.zw + dn.zw;
  const f32x2 p = pk_add_swap(am, bm);   // (c1 + c0, c2 + c3)
  const f32x2 h_a = pk_add_swap(p, am);  // (p01 + c2, p23 + c1) = h3(c1), h3(c2)
  f32x2 h_b;                             // h3(c3) = c4 + p23, h3(c0) = c[-1] + p01
  h_b.x = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(bm.y), kDppWaveShl1, 0xf, 0xf, true)) + p.y;
  h_b.y = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(bm.x), kDppWaveShr1, 0xf, 0xf, true)) + p.x;
  f32x4 o;
  o.xy = ns_a + h_a;
  o.zw = ns_b + h_b;
#ifdef MXS_TEST_VALU_PAD
  // Test builds only (tests/test_gpu_cycles.py, profiles/r06_cycles): one more
  // VALU slot per level-row (9 instead of 8, +12.5%), results unchanged (x * 1).
  float pad = o.x;
  asm volatile("v_mul_f32 %0, 1.0, %0" : "+v"(pad));
  o.x = pad;
#endif
  return o;
}
__device__ __forceinline__ f64x4 sum_w4d(const f64x4& up, const f64x4& mid, const f64x4& dn) {
  const double left = lane_shift<double, kDppWaveShr1>(mid.w);
  const double right = lane_shift<double, kDppWaveShl1>(mid.x);
  const double p01 = mid.x + mid.y, p23 = mid.z + mid.w;
  f64x4 o;
  o.x = (up.x + dn.x) + (p01 + left);
  o.y = (up.y + dn.y) + (p01 + mid.z);
  o.z = (up.z + dn.z) + (p23 + mid.y);
  o.w = (up.w + dn.w) + (p23 + right);
  return o;
}
struct BodySumF32 : BodyRotF32 {
  static __device__ __forceinline__ V jac(const V& u, const V& m, const V& d, float, float) { return sum_rot4f(u, m, d); }
  static __device__ __forceinline__ void store(const V& top, __amdgpu_buffer_rsrc_t r, unsigned off, float scale) {
    BodyRotF32::store(top * scale, r, off, scale);
  }
};
struct BodySumF64 : BodyWideF64 {
  // Without the fence the ascending 8 + 8 pass (fp64 8192^2) needs more than
  // the 256 VGPRs two waves per SIMD allow and spills 44 B per lane to
  // scratch; fenced: 231 VGPRs, no scratch, 1.5% faster (profiles/r06_fp64).
  static constexpr bool kStage0Fence = true;
  static __device__ __forceinline__ V jac(const V& u, const V& m, const V& d, double, double) { return sum_w4d(u, m, d); }
  static __device__ __forceinline__ void store(const V& top, __amdgpu_buffer_rsrc_t r, unsigned off, double scale) {
    BodyWideF64::store(top * scale, r, off, scale);
  }
};

// Scaled form (any c_center, c_neighbor != 0; the fp32 pipeline and balanced
// stream kernels, the fp64 wide pipeline at depth 16). The update is this framework's (the reference's
// Compute() is empty: stencil2d/mpi-2d-stencil-subarray-cuda.cu:32-37; SURVEY
// K10). u' = c1 (N + S + W + E + k u) with k = c0 / c1, so a pass
// carries v_l = u_l / c1^l, v' = (N + S + W + E) + k v — one packed FMA per
// cell pair in place of the per-step form's multiply and FMA — and applies c1^S
// once when it stores (the kernels' c0 argument holds c1^S, their c1 argument
// k). Rotated fp32: 9 VALU issue slots per 4 cells and level instead of 11;
// wide fp64: 16 fp64 ops + 4 moves instead of 20 + 4. The sum form is the
// k = 1 case with the centre folded into the horizontal pair sums (8 slots).
// Equal to the per-step evaluation up to rounding; magnitudes grow as
// (4 + |k|)^S inside a pass (the solver's range guard).
__device__ __forceinline__ f32x4 scaled_rot4f(const f32x4& up, const f32x4& mid, const f32x4& dn, float k) {
  const f32x2 am = mid.xy, bm = mid.zw;  // (c1, c2), (c3, c0)
  const f32x2 ns_a = up.xy + dn.xy, ns_b = up.zw + dn.zw;
  const f32x2 we = am + bm;                 // (c1 + c3, c2 + c0): the in-lane neighbour pairs, swapped
  const f32x2 t_a = pk_add_swap(ns_a, we);  // (ns(c1) + c0 + c2, ns(c2) + c1 + c3)
  f32x2 we_b;                               // c3: c2 + c0[lane + 1], c0: c1 + c3[lane - 1]
  we_b.x = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(bm.y), kDppWaveShl1, 0xf, 0xf, true)) + am.y;
  we_b.y = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(bm.x), kDppWaveShr1, 0xf, 0xf, true)) + am.x;
  const f32x2 kv = f32x2(k);
  f32x4 o;
  o.xy = __builtin_elementwise_fma(kv, am, t_a);
  o.zw = __builtin_elementwise_fma(kv, bm, ns_b + we_b);
  return o;
}
__device__ __forceinline__ f64x4 scaled_w4d(const f64x4& up, const f64x4& mid, const f64x4& dn, double k) {
  const double left = lane_shift<double, kDppWaveShr1>(mid.w);
  const double right = lane_shift<double, kDppWaveShl1>(mid.x);
  f64x4 o;
  o.x = __builtin_fma(k, mid.x, (up.x + dn.x) + (left + mid.y));
  o.y = __builtin_fma(k, mid.y, (up.y + dn.y) + (mid.x + mid.z));
  o.z = __builtin_fma(k, mid.z, (up.z + dn.z) + (mid.y + mid.w));
  o.w = __builtin_fma(k, mid.w, (up.w + dn.w) + (mid.z + right));
  return o;
}
struct BodyScaledF32 : BodyRotF32 {
  static __device__ __forceinline__ V jac(const V& u, const V& m, const V& d, float, float k) {
    return scaled_rot4f(u, m, d, k);
  }
  static __device__ __forceinline__ void store(const V& top, __amdgpu_buffer_rsrc_t r, unsigned off, float scale) {
    BodyRotF32::store(top * scale, r, off, scale);
  }
};
struct BodyScaledF64 : BodyWideF64 {
  static __device__ __forceinline__ V jac(const V& u, const V& m, const V& d, double, double k) {
    return scaled_w4d(u, m, d, k);
  }
  static __device__ __forceinline__ void store(const V& top, __amdgpu_buffer_rsrc_t r, unsigned off, double scale) {
    BodyWideF64::store(top * scale, r, off, scale);
  }
};

// XB: alternative bodies. The tuner specialises FastBody<T, SUM, 1>
// (bench/tune_kernels.hpp); the library uses XB = 0 and, with SUM, the scaled
// form as XB = kScaledBody.
constexpr int kScaledBody = 2;
template <typename T, bool SUM = false, int XB = 0>
struct FastBody;
template <>
struct FastBody<float, true, kScaledBody> {
  using type = BodyScaledF32;
};
template <>
struct FastBody<double, true, kScaledBody> {
  using type = BodyScaledF64;
};
template <>
struct FastBody<float, false, 0> {
  using type = BodyRotF32;
};
template <>
struct FastBody<double, false, 0> {
  using type = BodyWideF64;
};
template <>
struct FastBody<float, true, 0> {
  using type = BodySumF32;
};
template <>
struct FastBody<double, true, 0> {
  using type = BodySumF64;
};

// Strip geometry of the kernels: FAST = the 4-cells-per-lane bodies above,
// else one 16-byte vector per lane (StreamShape). Identical for fp32.
template <typename T, int S, bool FAST>
struct StripShape {
  static constexpr int N = FAST ? 4 : Vec16<T>::N;
  static constexpr int SA = ((S + N - 1) / N) * N;
  static constexpr int OW = kWaveSize * N - 2 * SA;
};

// One wave streams output rows [ys, ye) of the column strip whose first output
// column is xw. PF = input rows in flight (a register ring, statically indexed;
// a multiple of 3, the window's slot period).
//
// Skewed schedule: in iteration j level l works on the row level l-1 made in
// iteration j-1, so the S levels of one iteration are independent (S-way ILP
// instead of an S-long dependent chain of cross-lane move -> VALU). Slots per
// level rotate with the phase p = j % 3: up = win[p], mid = win[p+1],
// dn = win[p+2]; level l writes its output into win[p][l+1], the slot that is
// level l+1's dn next iteration, after level l+1 has read it as up (so levels
// run top-down). Level S-1 outputs row y_first + j - 2S + 1.
template <typename T, int S, int PF, bool WRAP, bool DPP>
__device__ __forceinline__ void stream_chunk(const T* __restrict__ in, T* __restrict__ out, index_t pitch,
                                             index_t core_off, index_t W, index_t H, index_t xw, index_t x_end,
                                             index_t ys, index_t ye, T c0, T c1) {
  static_assert(PF % 3 == 0, "the window rotates through 3 slots: PF must be a multiple of 3");
  using Sh = StreamShape<T, S>;
  constexpr int N = Sh::N, SA = Sh::SA, AL = SA / N;
  using V = typename Vec16<T>::type;
  const int lane = threadIdx.x & (kWaveSize - 1);
  const index_t gx = xw - SA + index_t(lane) * N;

  index_t lx = gx;
  bool load_ok = true;
  if constexpr (WRAP) {
    if (W >= kWaveSize * N) lx = gx < 0 ? gx + W : (gx >= W ? gx - W : gx);
    else lx = ((gx % W) + W) % W;
  } else {
    load_ok = gx < W + SA;  // inside the row padding of TileGeom::aligned
  }
  const T* __restrict__ pin = in + core_off + lx;
  const bool store_lane = lane >= AL && lane < kWaveSize - AL && gx < x_end;
  const bool full_vec = gx + N <= x_end;
  const int addr_l = ((lane + kWaveSize - 1) & (kWaveSize - 1)) << 2;
  const int addr_r = ((lane + 1) & (kWaveSize - 1)) << 2;

  // Next input row to fetch, as a (wrapped) row index.
  const index_t y_first = ys - S;
  index_t next = y_first;
  if constexpr (WRAP) next = next < 0 ? next + H : next;
  auto fetch = [&]() -> V {
    V v = V(T(0));
    if (load_ok) v = *reinterpret_cast<const V*>(pin + next * pitch);
    ++next;
    if constexpr (WRAP) next = next == H ? 0 : next;
    return v;
  };
  T* __restrict__ pout = out + core_off + gx + ys * pitch;  // first output row

  V win[3][S];
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int l = 0; l < S; ++l) win[q][l] = V(T(0));

  const index_t n_in = (ye - ys) + 2 * S;
  const index_t n_it = (ye - ys) + 3 * S - 1;
  V pf[PF];
#pragma unroll
  for (int k = 0; k < PF; ++k) pf[k] = k < n_in ? fetch() : V(T(0));
#pragma unroll 1
  for (index_t i = 0; i < n_it; i += PF) {
#pragma unroll
    for (int k = 0; k < PF; ++k) {
      const index_t j = i + k;
      if (j < n_it) {
        const int p0 = k % 3, p1 = (k + 1) % 3, p2 = (k + 2) % 3;  // static after the unroll
        win[p2][0] = pf[k];
        if (j + PF < n_in) pf[k] = fetch();
        V top = V(T(0));
#pragma unroll
        for (int l = S - 1; l >= 0; --l) {
          const V m = win[p1][l];
          const T left = DPP ? lane_shift<T, kDppWaveShr1>(m[N - 1]) : lane_fetch<T>(m[N - 1], addr_l);
          const T right = DPP ? lane_shift<T, kDppWaveShl1>(m[0]) : lane_fetch<T>(m[0], addr_r);
          const V o = jac_row<T, V>(win[p0][l], m, win[p2][l], left, right, c0, c1);
          if (l == S - 1) top = o;
          else win[p0][l + 1] = o;
        }
        if (j >= 3 * S - 1 && store_lane) {  // row ys + (j - 3S + 1)
          T* p = pout + (j - (3 * S - 1)) * pitch;
          if (full_vec) {
            __builtin_nontemporal_store(top, reinterpret_cast<V*>(p));
          } else {
#pragma unroll
            for (int q = 0; q < N; ++q)
              if (gx + q < x_end) p[q] = top[q];
          }
        }
      }
    }
  }
}

// fp32 form of stream_chunk on the rotated-pair layout (jac_rot4f) with a
// branch-free row loop, so the whole unrolled PF-row body is ONE basic block:
// any branch inside it (a guarded fetch, an exec-masked store) lets the backend
// hoist the DPP shifts of the next row above it, and a v_mov_b32_dpp that is
// not in its consumer's block cannot fold into the add (measured: 96 separate
// v_mov_b32_dpp per 48 level-rows otherwise). Hence:
//   * fetches always load: the row index saturates at the last input row (or
//     wraps, WRAP) and lanes past the row padding read its last vector —
//     values that cannot reach a stored cell within S levels (a stored cell at
//     x < x_end <= W depends on inputs in [x - S, x + S] only, SA >= S);
//   * stores go through a buffer descriptor over this chunk's output rows, and
//     a lane/row that must not store gets an out-of-range offset, which the
//     buffer range check drops (no exec mask, no branch);
//   * the row count is rounded up to PF; the extra iterations store nothing.
// Needs x_end % 4 == 0 (whole vectors) and (ye - ys) * pitch * 4 < 2^31 bytes
// (checked by the launcher, which falls back to stream_chunk otherwise).
// Progress-based wave priority (balanced launch). Two waves share each SIMD and
// the VALU arbiter prefers the older one, so with equal work the first-launched
// workgroup of a CU finished at ~62% of the kernel and its partner ran the last
// ~38% alone at ~70% of the paired issue rate (per-wave s_memrealtime stamps on
// 32768^2, TUNE_FOCUS=stamp of bench/stencil_tune). Each wave instead sets its
// priority from the fraction of its share still ahead of it (4 levels), so
// the laggard gets the issue slots and both finish together.
struct WavePrio {
  index_t done = 0;       // rows of the share finished before this chunk
  float quarters = 0.f;   // 4 / share rows (0: priority left alone)
  int level = -1;         // current level (s_setprio value)
};
__device__ __forceinline__ void wave_prio_update(WavePrio& wp, index_t done) {
  if (wp.quarters == 0.f) return;
  const float q = float(done) * wp.quarters;
  const int level = q >= 3.f ? 0 : (q >= 2.f ? 1 : (q >= 1.f ? 2 : 3));
  if (level == wp.level) return;
  wp.level = level;
  switch (level) {  // s_setprio takes an immediate
    case 3: __builtin_amdgcn_s_setprio(3); break;
    case 2: __builtin_amdgcn_s_setprio(2); break;
    case 1: __builtin_amdgcn_s_setprio(1); break;
    default: __builtin_amdgcn_s_setprio(0); break;
  }
}

// Generic over the per-lane body B (BodyRotF32: the rotated fp32 layout,
// BodyWideF64: 4 fp64 cells per lane); stream_chunk_rot is the fp32 form.
// Non-WRAP reads need x_origin + halo_x >= SA (the launcher checks it).
template <typename B, int S, int PF, bool WRAP>
__device__ __forceinline__ void stream_chunk_fast(const typename B::T* __restrict__ in, typename B::T* __restrict__ out,
                                                  index_t pitch, index_t core_off, index_t W, index_t H, index_t xw,
                                                  index_t x_end, index_t ys, index_t ye, typename B::T c0,
                                                  typename B::T c1, WavePrio* wp = nullptr) {
  static_assert(PF % 3 == 0, "the window rotates through 3 slots: PF must be a multiple of 3");
  using T = typename B::T;
  using V = typename B::V;
  using Sh = StripShape<T, S, true>;
  constexpr int N = Sh::N, SA = Sh::SA, AL = SA / N;
  const int lane = threadIdx.x & (kWaveSize - 1);
  const index_t gx = xw - SA + index_t(lane) * N;

  index_t lx;
  if constexpr (WRAP) {
    if (W >= kWaveSize * N) lx = gx < 0 ? gx + W : (gx >= W ? gx - W : gx);
    else lx = ((gx % W) + W) % W;
  } else {
    const index_t last_col = (W + N - 1) / N * N + SA - N;  // last vector of the row padding
    lx = gx < last_col ? gx : last_col;
  }
  const T* __restrict__ pin = in + core_off + lx;

  // Output descriptor: rows [ys, ye) from column xw - SA (wave-uniform base).
  const index_t rows = ye - ys;
  const T* obase = out + core_off + (xw - SA) + ys * pitch;
  const unsigned long long ob = reinterpret_cast<unsigned long long>(obase);
  const unsigned ob_lo = __builtin_amdgcn_readfirstlane(unsigned(ob)), ob_hi = __builtin_amdgcn_readfirstlane(unsigned(ob >> 32));
  T* obase_u = reinterpret_cast<T*>((static_cast<unsigned long long>(ob_hi) << 32) | ob_lo);
  const int nbytes = __builtin_amdgcn_readfirstlane(int(rows * pitch * index_t(sizeof(T))));
  const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(obase_u, 0, nbytes, 0x00020000);
  const bool store_lane = lane >= AL && lane < kWaveSize - AL && gx < x_end;
  const unsigned lane_off = unsigned(lane) * unsigned(N * sizeof(T));
  const unsigned row_bytes = unsigned(pitch) * unsigned(sizeof(T));
  constexpr unsigned kDrop = 0x80000000u;  // >= nbytes: dropped by the range check

  const index_t y_first = ys - S;
  const index_t last_row = ye + S - 1;
  index_t next = y_first;
  if constexpr (WRAP) next = next < 0 ? next + H : next;
  index_t roff = next * pitch;  // element offset of row `next`, stepped (see pipe_chunk)
  auto fetch = [&]() -> V {
    const V v = B::load(pin + roff);
    if constexpr (WRAP) {
      ++next;
      const bool wrap = next == H;
      next = wrap ? 0 : next;
      roff = wrap ? 0 : roff + pitch;
    } else {
      const bool adv = next < last_row;
      next = adv ? next + 1 : next;
      roff = adv ? roff + pitch : roff;
    }
    return v;
  };

  V win[3][S];
#pragma unroll
  for (int q = 0; q < 3; ++q)
#pragma unroll
    for (int l = 0; l < S; ++l) win[q][l] = B::zero();

  const index_t n_it = rows + 3 * S - 1;
  V pf[PF];
#pragma unroll
  for (int k = 0; k < PF; ++k) pf[k] = fetch();
  // Warm-up: level l first produces a row any stored cell depends on at
  // iteration 3l + 2, so iteration block b (iterations 3b .. 3b+2) only runs
  // levels 0..b; the skipped levels would compute rows outside every stored
  // cell's dependency cone. The warm-up covers the whole PF-steps below
  // 3(S-1) (the first store is at 3S-1); it halves the warm-up work of the
  // (3S-1) extra iterations every chunk pays, 14% of a 292-row share of the
  // 8-GPU tile.
  constexpr int kWarm = (3 * (S - 1)) / PF * PF;
  if (wp) wave_prio_update(*wp, wp->done);
#pragma unroll 1
  for (int ib = 0; ib < kWarm; ib += PF) {
#pragma unroll
    for (int k = 0; k < PF; ++k) {
      const int p0 = k % 3, p1 = (k + 1) % 3, p2 = (k + 2) % 3;
      const int b = (ib + k) / 3;  // wave-uniform
      win[p2][0] = B::enter(pf[k]);
      pf[k] = fetch();
#pragma unroll
      for (int l = S - 2; l >= 0; --l) {
        if (l <= b) win[p0][l + 1] = B::jac(win[p0][l], win[p1][l], win[p2][l], c0, c1);
      }
    }
  }
#pragma unroll 1
  for (index_t i = kWarm; i < n_it; i += PF) {
    if (wp && (i & 63) == 0) wave_prio_update(*wp, wp->done + i);
#pragma unroll
    for (int k = 0; k < PF; ++k) {
      const index_t j = i + k;
      const int p0 = k % 3, p1 = (k + 1) % 3, p2 = (k + 2) % 3;  // static after the unroll
      if (j >= n_it) break;  // wave-uniform (scalar branch); without it the allocator spills to AGPRs
      win[p2][0] = B::enter(pf[k]);
      pf[k] = fetch();
      V top;
#pragma unroll
      for (int l = S - 1; l >= 0; --l) {
        const V o = B::jac(win[p0][l], win[p1][l], win[p2][l], c0, c1);
        if (l == S - 1) top = o;
        else win[p0][l + 1] = o;
      }
      const index_t r = j - (3 * S - 1);  // output row (relative to ys) of this iteration
      const bool ok = store_lane && r >= 0 && r < rows;
      const unsigned off = ok ? lane_off + unsigned(r) * row_bytes : kDrop;
      B::store(top, orsrc, off, c0);
    }
  }
}

template <int S, int PF, bool WRAP>
__device__ __forceinline__ void stream_chunk_rot(const float* __restrict__ in, float* __restrict__ out, index_t pitch,
                                                 index_t core_off, index_t W, index_t H, index_t xw, index_t x_end,
                                                 index_t ys, index_t ye, float c0, float c1, WavePrio* wp = nullptr) {
  stream_chunk_fast<BodyRotF32, S, PF, WRAP>(in, out, pitch, core_off, W, H, xw, x_end, ys, ye, c0, c1, wp);
}

// Grid form: workgroup = 4 waves on 4 adjacent strips of the same CH-row chunk.
// ROT: the branch-free 4-cells-per-lane body (stream_chunk_fast: rotated-pair
// fp32 or wide-lane fp64; the launcher checks its preconditions).
template <typename T, int S, int PF, bool WRAP, bool DPP = true, bool ROT = false>
__global__ __launch_bounds__(kBlock) void stencil5_stream_kernel(const T* __restrict__ in, T* __restrict__ out,
                                                                 index_t pitch, index_t core_off, index_t W, index_t H,
                                                                 index_t x_begin, index_t x_end, index_t y_begin,
                                                                 index_t y_end, index_t CH, T c0, T c1) {
  constexpr int OW = StripShape<T, S, ROT>::OW;
  const index_t xw = x_begin + (index_t(blockIdx.x) * kWavesPerBlock + threadIdx.x / kWaveSize) * OW;
  if (xw >= x_end) return;  // wave-uniform
  const index_t ys = y_begin + index_t(blockIdx.y) * CH;
  const index_t ye = ys + CH < y_end ? ys + CH : y_end;
  if constexpr (ROT)
    stream_chunk_fast<typename FastBody<T>::type, S, PF, WRAP>(in, out, pitch, core_off, W, H, xw, x_end, ys, ye, c0, c1);
  else stream_chunk<T, S, PF, WRAP, DPP>(in, out, pitch, core_off, W, H, xw, x_end, ys, ye, c0, c1);
}

// Balanced persistent form: exactly as many workgroups as fit on the chip at
// once. The work is (group of 4 adjacent strips) x rows, split into equal
// shares of rows per workgroup (group-major); a workgroup's 4 waves stream the
// 4 strips of its group over the same rows side by side — as in the grid form,
// so the apron columns two neighbouring waves both read are L2 hits — and a
// share that crosses a group boundary restarts there. No tail round, and
// (3S-1)/share redundant rows instead of (3S-1)/CH per chunk.
template <typename T, int S, int PF, bool WRAP, bool DPP = true, bool ROT = false, bool SUM = false, int XB = 0>
__global__ __launch_bounds__(kBlock) void stencil5_stream_balanced_kernel(
    const T* __restrict__ in, T* __restrict__ out, index_t pitch, index_t core_off, index_t W, index_t H,
    index_t x_begin, index_t x_end, index_t y_begin, index_t y_end, index_t share, T c0, T c1) {
  constexpr int OW = StripShape<T, S, ROT>::OW;
  const index_t rows = y_end - y_begin;
  const index_t strips = (x_end - x_begin + OW - 1) / OW;
  const index_t groups = (strips + kWavesPerBlock - 1) / kWavesPerBlock;
  const index_t total = groups * rows;
  const int wave = threadIdx.x / kWaveSize;
  index_t a = index_t(blockIdx.x) * share;
  const index_t a0 = a;
  const index_t b = a + share < total ? a + share : total;
  WavePrio wp;
  if (b > a) wp.quarters = 4.f / float(b - a);
  // ROT stores go through one buffer descriptor per call: longer shares are
  // walked in pieces of at most kMaxChunkBytes (see stencil5_stream_pipe_kernel).
  const index_t max_rows = ROT ? kMaxChunkBytes / (pitch * index_t(sizeof(T))) : rows;
  if (max_rows < 1) return;  // workgroup-uniform (rot_ok keeps such rows on the plain body)
#pragma unroll 1
  while (a < b) {  // workgroup-uniform
    const index_t grp = a / rows, r0 = a - grp * rows;
    index_t r1 = rows < r0 + (b - a) ? rows : r0 + (b - a);
    r1 = r1 - r0 > max_rows ? r0 + max_rows : r1;
    const index_t xw = x_begin + (grp * kWavesPerBlock + wave) * OW;
    if (xw < x_end) {
      wp.done = a - a0;
      if constexpr (ROT)
        stream_chunk_fast<typename FastBody<T, SUM, XB>::type, S, PF, WRAP>(in, out, pitch, core_off, W, H, xw, x_end,
                                                                        y_begin + r0, y_begin + r1, c0, c1, &wp);
      else
        stream_chunk<T, S, PF, WRAP, DPP>(in, out, pitch, core_off, W, H, xw, x_end, y_begin + r0, y_begin + r1, c0,
                                          c1);
    }
    a += r1 - r0;
  }
}

// ------------------------------------------------- two-stage wave pipeline
// Deeper time blocks without more registers per wave. A single wave holds a
// three-slot window per level (12 VGPRs per level at fp32), so S = 16 already
// needs ~237 VGPRs; S = 20 in one wave drops to 1 wave per SIMD and spills to
// AGPRs, measured 35-45% slower per iteration (profiles/r02_deep). Here a
// column strip is streamed by TWO waves of the workgroup: stage 0 runs levels
// 1..S0 on rows fetched from HBM and hands each level-S0 row to stage 1
// through an LDS ring (one ds_write_b128 / ds_read_b128 per lane and row);
// stage 1 runs levels S0+1..S0+S1 and stores. Each wave keeps only its own
// levels' windows, so S = S0 + S1 reaches 20-32 at 2 waves per SIMD, and HBM
// sees one read + one write per cell per S iterations.
//
// Lock-step: all 8 waves of the workgroup (4 strips x 2 stages) advance in
// blocks of PF iterations with one barrier per block. Stage 0 emits its k-th
// output row at its iteration 3*S0 - 1 + k; stage 1 starts T1 blocks later and
// consumes row k at its iteration k, so every row it reads was written at
// least one barrier earlier; a ring of 3*PF rows per strip is never
// overwritten before it is read (see the derivation in docs/PERF.md). Both
// stages run the same number of blocks (their extra iterations read / write
// rows outside every stored cell's dependency cone). The apron is that of a
// single S-level wave (the strip's edge contamination spreads one column per
// level through both stages): OW = 256 - 2 * SA(S) output columns per strip.
template <int S0, int S1, int PF>
struct PipeShape {
  static constexpr int S = S0 + S1;
  static constexpr int RING = 3 * PF;                      // rows per strip in the LDS ring
  static constexpr int T1 = (3 * S0 + PF - 1 + PF - 1) / PF;  // stage-1 start block: ceil((3*S0 + PF - 1) / PF)
};

// Joint stage-1 windows (JOINT). In the layout above every strip pays the
// apron of all S levels: 256 - 2 SA(S) output columns per strip (208 of 256 at
// S = 24). Stage 1 does not need its own strip's stage-0 edges, though: the
// level-S0 columns a stage-0 wave gets right (all but A0 = S0 rounded up to 4
// per side) are laid side by side, for the G strips of the workgroup, in ONE
// LDS row of G * OW0 valid columns, and stage 1's G windows (256 columns each,
// stride OW1 = 256 - 2 A1) are cut from that row. Stage 0's apron is still
// paid per strip, stage 1's once per group: OWG = G (256 - 2 A0) - 2 A1 output
// columns per group, capped at G * OW1 (S = 24 as 12 + 12: 904 vs 4 x 208 =
// 832, +8.7% per pass at the same VALU work; S = 20 as 8 + 12: 928 vs 864;
// S = 28 as 12 + 16: 896 vs 800). The stage-0 lanes that hold no valid
// column write into the row's tail (G * 2 A0 / 4 slots, exactly the lanes that
// need one), which stage 1 only reads into columns it never stores. Same
// operations per cell as the per-strip layout: bitwise identical output.
template <int S0, int S1, int G>
struct JointShape {
  static constexpr int A0 = (S0 + 3) / 4 * 4, A1 = (S1 + 3) / 4 * 4;  // per-stage aprons (4-column lanes)
  static constexpr int OW0 = 256 - 2 * A0;    // valid level-S0 columns per stage-0 wave
  static constexpr int OW1 = 256 - 2 * A1;    // stride of stage 1's windows
  static constexpr int SPAN = G * OW0;        // valid columns of the joint row
  // Output columns per group: the joint row's valid span less stage 1's apron,
  // or what the G windows can store (G * OW1) when that is less (A0 < A1).
  static constexpr int OWG = SPAN - 2 * A1 < G * OW1 ? SPAN - 2 * A1 : G * OW1;
  static constexpr int ROW = G * kWaveSize;   // joint row length in lane vectors (SPAN / 4 + the tail)
  static constexpr int LEAD = A0 + A1;        // input columns left of the group's first output column
  static_assert((G - 1) * OW1 + 256 <= 4 * ROW, "stage-1 windows must stay inside the joint row");
  static_assert(OWG > 0, "time block too deep for a joint group");
};

template <typename B, int S0, int S1, int PF, bool WRAP, bool JOINT = false, int G = kWavesPerBlock, int LAG1 = 0>
__device__ __forceinline__ void pipe_chunk(const typename B::T* __restrict__ in, typename B::T* __restrict__ out,
                                           index_t pitch, index_t core_off, index_t W, index_t H, index_t xw,
                                           index_t x_end, index_t ys, index_t ye, typename B::T c0, typename B::T c1,
                                           typename B::V* __restrict__ ring, int stage, int strip = 0) {
  static_assert(PF % 3 == 0, "the window rotates through 3 slots: PF must be a multiple of 3");
  using P = PipeShape<S0, S1, PF>;
  constexpr int S = P::S, RING = P::RING;
  using T = typename B::T;
  using V = typename B::V;
  using Sh = StripShape<T, S, true>;
  using J = JointShape<S0, S1, G>;
  // Level order within a row iteration. Default: levels descend, so every
  // level reads only rows of earlier iterations (S independent evaluations per
  // row, level l lags 3 rows per level: a stage emits its first valid row at
  // iteration 3 * levels - 1). LAG1: levels ascend and each reads the row its
  // lower level made in the same iteration (a dependent chain per row), so a
  // level lags one row and a stage emits its first row at iteration 2 * levels:
  // S - 1 fewer fill iterations per chunk and stage. Same arithmetic per cell.
  // LAG1 is a stage mask: bit 0 = stage 0 ascends, bit 1 = stage 1 ascends.
  constexpr bool ASC0 = (LAG1 & 1) != 0, ASC1 = (LAG1 & 2) != 0;
  constexpr int E0 = ASC0 ? 2 * S0 : 3 * S0 - 1, E1 = ASC1 ? 2 * S1 : 3 * S1 - 1;
  constexpr int N = Sh::N, SA = Sh::SA, AL = SA / N;
  static_assert(!JOINT || N == 4, "joint windows assume 4-cell lanes");
  const int lane = threadIdx.x & (kWaveSize - 1);
  // Per-strip layout: xw = the strip's first output column, both stages cover
  // [xw - SA, xw - SA + 256). Joint: xw = the GROUP's first output column;
  // stage-0 wave `strip` covers [xw - LEAD + strip OW0, + 256), stage-1 wave
  // `strip` the window [xw - A1 + strip OW1, + 256).
  const index_t gx = JOINT ? (stage == 0 ? xw - J::LEAD + index_t(strip) * J::OW0 : xw - J::A1 + index_t(strip) * J::OW1) +
                                 index_t(lane) * N
                           : xw - SA + index_t(lane) * N;
  const index_t rows = ye - ys;
  // Stage 0 starts D rows early so that its ring writes start block-aligned
  // (row k is emitted at iteration 3*S0 - 1 + D + k, a multiple of PF for k = 0):
  // no per-row slot wrap. The lead rows only feed level-S0 rows before ys - S1.
  constexpr int D = (PF - E0 % PF) % PF;
  constexpr int T1 = (E0 + D) / PF + 1;  // stage-1 start block (P::T1 for the default order)
  static_assert(ASC0 || T1 == P::T1, "stage-1 start block");
  const index_t n_it0 = rows + 2 * S1 + E0 + D;  // stage 0: level-S0 rows [ys - S1, ye + S1)
  const index_t n_it1 = rows + E1;               // stage 1: output rows [ys, ye)
  const index_t blocks0 = (n_it0 + PF - 1) / PF, blocks1 = T1 + (n_it1 + PF - 1) / PF;
  const index_t blocks = blocks0 > blocks1 ? blocks0 : blocks1;
  // This lane's slot in a ring row, and the ring's row stride (lane vectors).
  constexpr int RSTRIDE = JOINT ? J::ROW : kWaveSize;
  int slot = lane;
  if constexpr (JOINT) {
    constexpr int AL0 = J::A0 / 4;  // stage-0 lanes per side without a valid level-S0 column
    if (stage == 0) {
      const bool valid = lane >= AL0 && lane < kWaveSize - AL0;
      const int tail = J::SPAN / 4 + strip * 2 * AL0 + (lane < AL0 ? lane : lane - (kWaveSize - 2 * AL0));
      slot = valid ? strip * (J::OW0 / 4) + lane - AL0 : tail;
    } else {
      slot = strip * (J::OW1 / 4) + lane;
    }
  }
  V* __restrict__ my = ring + slot;

  if (stage == 0) {  // wave-uniform
    index_t lx;
    if (!JOINT && xw >= x_end) {
      lx = 0;  // idle strip past the rectangle: any valid address, nothing it makes is stored
    } else if constexpr (WRAP) {
      // Joint groups read up to G * 256 columns past their first output column.
      if (W >= (JOINT ? G : 1) * kWaveSize * N) lx = gx < 0 ? gx + W : (gx >= W ? gx - W : gx);
      else lx = ((gx % W) + W) % W;
    } else {
      const index_t last_col = (W + N - 1) / N * N + SA - N;
      lx = gx < last_col ? gx : last_col;
    }
    const T* __restrict__ pin = in + core_off + lx;
    const index_t last_row = ye + S - 1;
    // The first PF rows (the D lead rows clamped to the first needed row when
    // there is no wrap: they may lie above the ghost ring).
    V pf[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) {
      index_t r = ys - S - D + k;
      if constexpr (WRAP) r = r < 0 ? r + H : r;
      else r = r < ys - S ? ys - S : r;
      pf[k] = B::load(pin + r * pitch);
    }
    index_t next = ys - S - D + PF;
    if constexpr (WRAP) next = next < 0 ? next + H : next;
    index_t roff = next * pitch;  // element offset of row `next`, stepped (no multiply per row)
    auto fetch = [&]() -> V {
      const V v = B::load(pin + roff);
      if constexpr (WRAP) {
        ++next;
        const bool wrap = next == H;
        next = wrap ? 0 : next;
        roff = wrap ? 0 : roff + pitch;
      } else {
        const bool adv = next < last_row;
        next = adv ? next + 1 : next;
        roff = adv ? roff + pitch : roff;
      }
      return v;
    };
    V win[3][S0];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int l = 0; l < S0; ++l) win[q][l] = B::zero();
    // See stream_chunk_rot: level l matters from iteration 3l + 2 (LAG1: 2l).
    constexpr int kWarm = ASC0 ? (2 * S0) / PF * PF : (3 * (S0 - 1)) / PF * PF;
#pragma unroll 1
    for (int ib = 0; ib < kWarm; ib += PF) {
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        if constexpr (ASC0) {
          const int n = k % 3, o = (k + 1) % 3, m = (k + 2) % 3;  // rows of iterations j, j-2, j-1
          const int b = (ib + k) / 2;
          win[n][0] = B::enter(pf[k]);
          pf[k] = fetch();
#pragma unroll
          for (int l = 0; l < S0 - 1; ++l)
            if (l < b) win[n][l + 1] = B::jac(win[o][l], win[m][l], win[n][l], c0, c1);
        } else {
          const int p0 = k % 3, p1 = (k + 1) % 3, p2 = (k + 2) % 3;
          const int b = (ib + k) / 3;
          win[p2][0] = B::enter(pf[k]);
          pf[k] = fetch();
#pragma unroll
          for (int l = S0 - 2; l >= 0; --l)
            if (l <= b) win[p0][l + 1] = B::jac(win[p0][l], win[p1][l], win[p2][l], c0, c1);
        }
      }
      __syncthreads();
    }
    // Ring slot of each block's first row k = i - (3*S0 - 1): a wave-uniform
    // counter stepping by PF modulo RING (a 64-bit modulo per block cost ~40
    // scalar instructions).
    int base = ((kWarm - (E0 + D)) % RING + RING) % RING;  // 0, PF or 2 PF
#pragma unroll 1
    for (index_t i = kWarm; i < blocks * PF; i += PF) {
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        V top;
        if constexpr (ASC0) {
          const int n = k % 3, o = (k + 1) % 3, m = (k + 2) % 3;
          win[n][0] = B::enter(pf[k]);
          pf[k] = fetch();
#pragma unroll
          for (int l = 0; l < S0; ++l) {
            const V v = B::jac(win[o][l], win[m][l], win[n][l], c0, c1);
            if (l == S0 - 1) top = v;
            else win[n][l + 1] = v;
          }
        } else {
          const int p0 = k % 3, p1 = (k + 1) % 3, p2 = (k + 2) % 3;
          win[p2][0] = B::enter(pf[k]);
          pf[k] = fetch();
#pragma unroll
          for (int l = S0 - 1; l >= 0; --l) {
            const V o = B::jac(win[p0][l], win[p1][l], win[p2][l], c0, c1);
            if (l == S0 - 1) top = o;
            else win[p0][l + 1] = o;
          }
        }
        // Row k = j - (3*S0 - 1 + D) of stage 1's input (rotated layout);
        // writes for k < 0 land in slots no reader touches before they are
        // rewritten. base + k < RING: blocks are ring-aligned.
        my[(base + k) * RSTRIDE] = top;
        if constexpr (B::kStage0Fence) __builtin_amdgcn_sched_barrier(0);
      }
      base = base + PF < RING ? base + PF : 0;
      __syncthreads();
    }
  } else {
    // Output descriptor over rows [ys, ye) (see stream_chunk_rot).
    const index_t x0w = gx - index_t(lane) * N;  // the window's first column
    const T* obase = out + core_off + x0w + ys * pitch;
    const unsigned long long ob = reinterpret_cast<unsigned long long>(obase);
    const unsigned ob_lo = __builtin_amdgcn_readfirstlane(unsigned(ob)),
                   ob_hi = __builtin_amdgcn_readfirstlane(unsigned(ob >> 32));
    T* obase_u = reinterpret_cast<T*>((static_cast<unsigned long long>(ob_hi) << 32) | ob_lo);
    const int nbytes = __builtin_amdgcn_readfirstlane(int(rows * pitch * index_t(sizeof(T))));
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(obase_u, 0, nbytes, 0x00020000);
    bool store_lane;
    if constexpr (JOINT) {
      // Inside this window's own apron and inside the group's output span
      // [A1, A1 + OWG) (the last window may run past it); windows tile the group.
      constexpr int AL1 = J::A1 / 4;
      const int q = strip * J::OW1 + lane * N;  // joint-row column of this lane's first cell
      store_lane = lane >= AL1 && lane < kWaveSize - AL1 && q + N <= J::A1 + J::OWG && gx < x_end;
    } else {
      store_lane = lane >= AL && lane < kWaveSize - AL && gx < x_end && xw < x_end;
    }
    // Store offset = lane term + row term, both past the range when dropped: a
    // dropped lane adds 2^31, a dropped row 0x7F000000 (chunks are at most
    // kMaxChunkBytes = 0x7F000000 bytes, so no sum wraps past 2^32 and every
    // sum with a dropped term is >= the range). The row term is wave-uniform
    // (scalar select), so a row costs one v_add_u32 (a 64-bit v_cmp and a
    // v_cndmask per row before).
    const unsigned lane_term = store_lane ? unsigned(lane) * unsigned(N * sizeof(T)) : 0x80000000u;
    const unsigned row_bytes = unsigned(pitch) * unsigned(sizeof(T));
    const int rows_i = int(rows);
    V win[3][S1];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int l = 0; l < S1; ++l) win[q][l] = B::zero();
#pragma unroll 1
    for (int t = 0; t < T1; ++t) __syncthreads();  // stage 0 fills the ring
    constexpr int kWarm = ASC1 ? (2 * S1) / PF * PF : (3 * (S1 - 1)) / PF * PF;
#pragma unroll 1
    for (int ib = 0; ib < kWarm; ib += PF) {
      V inrow[PF];
      const int base = (ib / PF) % 3 * PF;  // RING = 3 * PF and ib is a multiple of PF
#pragma unroll
      for (int k = 0; k < PF; ++k) inrow[k] = my[(base + k) * RSTRIDE];
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        if constexpr (ASC1) {
          const int n = k % 3, o = (k + 1) % 3, m = (k + 2) % 3;
          const int b = (ib + k) / 2;
          win[n][0] = inrow[k];
#pragma unroll
          for (int l = 0; l < S1 - 1; ++l)
            if (l < b) win[n][l + 1] = B::jac(win[o][l], win[m][l], win[n][l], c0, c1);
        } else {
          const int p0 = k % 3, p1 = (k + 1) % 3, p2 = (k + 2) % 3;
          const int b = (ib + k) / 3;
          win[p2][0] = inrow[k];
#pragma unroll
          for (int l = S1 - 2; l >= 0; --l)
            if (l <= b) win[p0][l + 1] = B::jac(win[p0][l], win[p1][l], win[p2][l], c0, c1);
        }
      }
      __syncthreads();
    }
    int base = (kWarm / PF) % 3 * PF;  // ring slot of the block's first row (counter, see stage 0)
#pragma unroll 1
    for (index_t i = kWarm; i < (blocks - T1) * PF; i += PF) {
      V inrow[PF];
#pragma unroll
      for (int k = 0; k < PF; ++k) inrow[k] = my[(base + k) * RSTRIDE];
      base = base + PF < RING ? base + PF : 0;
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        const index_t j = i + k;
        V top;
        if constexpr (ASC1) {
          const int n = k % 3, o = (k + 1) % 3, m = (k + 2) % 3;
          win[n][0] = inrow[k];
#pragma unroll
          for (int l = 0; l < S1; ++l) {
            const V v = B::jac(win[o][l], win[m][l], win[n][l], c0, c1);
            if (l == S1 - 1) top = v;
            else win[n][l + 1] = v;
          }
        } else {
          const int p0 = k % 3, p1 = (k + 1) % 3, p2 = (k + 2) % 3;
          win[p2][0] = inrow[k];
#pragma unroll
          for (int l = S1 - 1; l >= 0; --l) {
            const V o = B::jac(win[p0][l], win[p1][l], win[p2][l], c0, c1);
            if (l == S1 - 1) top = o;
            else win[p0][l + 1] = o;
          }
        }
        const int r = int(j - E1);
        const unsigned row_term = r >= 0 && r < rows_i ? unsigned(r) * row_bytes : unsigned(kMaxChunkBytes);
        B::store(top, orsrc, lane_term + row_term, c0);
      }
      __syncthreads();
    }
  }
}

// Balanced persistent launch of the two-stage pipeline: 512-thread workgroups
// (4 strips x 2 stages), equal shares of (4-strip group) x rows as in
// stencil5_stream_balanced_kernel. T = float: rotated-pair layout; T = double:
// wide-lane body (FastBody<T>). Needs x_end % 4 == 0 and a chunk of at most
// kMaxChunkBytes (the output buffer descriptor and its drop offsets).
// PRIO (tuning): 1 raises the fetching stage's wave priority, 2 the storing stage's.
// G: strips per workgroup (2G waves; the barriers of one block of rows span the
// workgroup, so smaller groups decouple the strips of a CU).
// XM (tuning): XCD-major share order — the workgroups one XCD runs (blockIdx
// congruent mod 8) take consecutive shares, so vertically adjacent chunks, which
// read the same 2S apron rows, share that XCD's L2.
// JOINT: joint stage-1 windows (JointShape), OWG output columns per group.
// Workgroup ranges of the linear (group x rows) space: equal shares of `share`
// rows (n == 0), or explicit fill-aware starts (kernels/chunk_schedule.hpp:
// balanced_starts), start[w] .. start[w + 1] for workgroup w — passed by value
// in the kernel arguments (2 KB), so a launch needs no device table and stays
// graph-capturable.
constexpr int kMaxShareBlocks = 512;
struct PipeShares {
  index_t share = 0;
  int n = 0;
  int start[kMaxShareBlocks + 1];
  static PipeShares equal(index_t share) {
    PipeShares p;
    p.share = share;
    return p;
  }
};

template <int S0, int S1, int PF, bool WRAP, int PRIO = 0, typename T = float, bool SUM = false,
          int G = kWavesPerBlock, bool XM = false, bool JOINT = false, int LAG1 = 0, int XB = 0>
__global__ __launch_bounds__(2 * G * kWaveSize) void stencil5_stream_pipe_kernel(
    const T* __restrict__ in, T* __restrict__ out, index_t pitch, index_t core_off, index_t W, index_t H,
    index_t x_begin, index_t x_end, index_t y_begin, index_t y_end, const PipeShares shares, T c0, T c1) {
  using P = PipeShape<S0, S1, PF>;
  using B = typename FastBody<T, SUM, XB>::type;
  constexpr int OW = StripShape<T, P::S, true>::OW;
  constexpr int OWG = JointShape<S0, S1, G>::OWG;
  __shared__ typename B::V ring[G * P::RING * kWaveSize];
  const index_t rows = y_end - y_begin;
  const index_t strips = (x_end - x_begin + OW - 1) / OW;
  const index_t groups = JOINT ? (x_end - x_begin + OWG - 1) / OWG : (strips + G - 1) / G;
  const index_t total = groups * rows;
  const int wave = threadIdx.x / kWaveSize;
  const int strip = wave % G, stage = wave / G;
  if constexpr (PRIO == 1) {
    if (stage == 0) __builtin_amdgcn_s_setprio(1);
  } else if constexpr (PRIO == 2) {
    if (stage == 1) __builtin_amdgcn_s_setprio(1);
  }
  index_t slot = blockIdx.x;
  if constexpr (XM) {
    if (gridDim.x % kNumXcds == 0) slot = (blockIdx.x % kNumXcds) * (gridDim.x / kNumXcds) + blockIdx.x / kNumXcds;
  }
  index_t a, b;
  if (shares.n > 0) {
    a = shares.start[slot];
    b = shares.start[slot + 1];
  } else {
    a = slot * shares.share;
    b = a + shares.share < total ? a + shares.share : total;
  }
  // Rows per pipe_chunk call: its output buffer descriptor spans at most
  // kMaxChunkBytes (32-bit offsets), so on very wide tiles (rows of MiBs: a
  // 65536^2 fp32 tile, 16 GiB per buffer) a share is walked in pieces, each
  // paying its own pipeline fill (the launcher checks >= 64 rows fit).
  const index_t max_rows = kMaxChunkBytes / (pitch * index_t(sizeof(T)));
  if (max_rows < 1) return;  // workgroup-uniform, before any barrier (never launched so: the host checks)
#pragma unroll 1
  while (a < b) {  // workgroup-uniform: all 8 waves take every chunk (barriers inside)
    const index_t grp = a / rows, r0 = a - grp * rows;
    index_t r1 = rows < r0 + (b - a) ? rows : r0 + (b - a);
    r1 = r1 - r0 > max_rows ? r0 + max_rows : r1;
    if constexpr (JOINT) {
      pipe_chunk<B, S0, S1, PF, WRAP, true, G, LAG1>(in, out, pitch, core_off, W, H, x_begin + grp * OWG, x_end,
                                               y_begin + r0, y_begin + r1, c0, c1, ring, stage, strip);
    } else {
      const index_t xw = x_begin + (grp * G + strip) * OW;
      pipe_chunk<B, S0, S1, PF, WRAP, false, G, LAG1>(in, out, pitch, core_off, W, H, xw, x_end, y_begin + r0, y_begin + r1, c0, c1,
                                      ring + strip * P::RING * kWaveSize, stage);
    }
    a += r1 - r0;
  }
}

// Chunk-list pass (kernels/chunk_schedule.hpp): the joint-window pipeline of
// stencil5_stream_pipe_kernel (ghost-ring tile, no wrap) over an explicit chunk
// list per workgroup instead of one contiguous share. The interior-first
// multi-GPU super-step runs two launches of it on disjoint CUs (core chunks
// beside the halo exchange, then the ghost-ring chunks). The halo copy kernel
// (copy2d_batch_kernel, 32 VGPRs) runs beside it: two pass waves per SIMD leave
// it 32 of the 512 VGPRs in the sum forms (fp32 12 + 8 / 12 + 12: 238, 8 + 12:
// 225, 8-VGPR granules); the per-step 8 + 12 and fp64 8 + 8 forms (244) leave
// 16, and their copies take the CUs the inner launch leaves free.
template <int S0, int S1, int PF, typename T, bool SUM, int LAG1, int XB = 0>
__global__ __launch_bounds__(2 * kWavesPerBlock * kWaveSize) void stencil5_pipe_chunks_kernel(
    const T* __restrict__ in, T* __restrict__ out, index_t pitch, index_t core_off, index_t W, index_t H,
    index_t x_begin, index_t x_end, index_t y_begin, const PassChunk* __restrict__ table, int entries, T c0, T c1) {
  constexpr int G = kWavesPerBlock;
  using P = PipeShape<S0, S1, PF>;
  using B = typename FastBody<T, SUM, XB>::type;
  constexpr int OWG = JointShape<S0, S1, G>::OWG;
  __shared__ typename B::V ring[G * P::RING * kWaveSize];
  const int wave = threadIdx.x / kWaveSize;
  const int strip = wave % G, stage = wave / G;
  const PassChunk* __restrict__ mine = table + index_t(blockIdx.x) * entries;
  const index_t max_rows = kMaxChunkBytes / (pitch * index_t(sizeof(T)));  // pieces, as in stencil5_stream_pipe_kernel
  if (max_rows < 1) return;  // workgroup-uniform, before any barrier (chunk_pass_shape refuses such rows)
#pragma unroll 1
  for (int e = 0; e < entries; ++e) {  // workgroup-uniform
    const PassChunk c = mine[e];
    if (c.r1 <= c.r0) break;  // lists are packed from slot 0
#pragma unroll 1
    for (index_t r0 = c.r0; r0 < c.r1; r0 += max_rows) {
      const index_t r1 = c.r1 - r0 > max_rows ? r0 + max_rows : c.r1;
      pipe_chunk<B, S0, S1, PF, false, true, G, LAG1>(in, out, pitch, core_off, W, H, x_begin + index_t(c.group) * OWG,
                                                     x_end, y_begin + r0, y_begin + r1, c0, c1, ring, stage, strip);
    }
  }
}

}  // namespace detail
}  // namespace kernels
}  // namespace mxs
