// Kernels only the tuners time (bench/stencil_tune.hip, bench/stencil_tune64.hip),
// kept out of csrc/kernels/stencil_device.hpp so the production library does
// not compile them: the LDS ping-pong temporal-block tile (stencil5_tb_kernel;
// production runs the single-buffer tile stencil5_tb1_kernel) and the
// three-stage wave pipeline (stencil5_stream_pipe3_kernel: measured 3-5% behind
// the two-stage pipeline, docs/PERF.md), and the LDS-crossbar bodies (XB = 1).
#pragma once

#include "../csrc/kernels/stencil_pipe.hpp"

namespace mxs {
namespace kernels {
namespace detail {

// --------------------------------------------------------- temporal blocking
// S Jacobi iterations per launch, LDS-tiled (the "LDS tiling" of the stencil):
// a workgroup stages its TW x TH output tile plus an S-deep apron once from HBM
// into LDS (16-byte vector loads, all issued up front), runs S 5-point steps
// LDS -> LDS (ping-pong buffers; the valid region shrinks by one cell per step,
// so no intermediate halo is ever exchanged), then writes the TW x TH result
// once (non-temporal 16-byte stores). HBM traffic per iteration drops by ~S x
// (plus the apron re-read, (TW+2SA)(TH+2S)/(TW*TH)). The tile's source region
// needs a ghost ring of depth >= S (exchanged S-deep every S iterations), or
// WRAP for the 1x1 periodic grid (global reads wrap around the tile).
//
// The x apron SA = S rounded up to the vector width keeps every staged row and
// every LDS access 16-byte aligned; LDS rows are padded by one vector on each
// side (the x-1 / x+N reads of the edge chunks land in the padding: those cells
// are outside the valid region and never reach the output).
template <typename T, int S, int TW, int TH, bool WRAP>
__global__ __launch_bounds__(256) void stencil5_tb_kernel(const T* __restrict__ in, T* __restrict__ out, index_t pitch,
                                                         index_t core_off, index_t W, index_t H, index_t x_begin,
                                                         index_t x_end, index_t y_begin, index_t y_end, T c0, T c1) {
  constexpr int N = Vec16<T>::N;
  constexpr int SA = ((S + N - 1) / N) * N;  // x apron, vector aligned
  constexpr int LW = TW + 2 * SA;            // staged columns
  constexpr int LP = LW + 2 * N;             // LDS row pitch (elements)
  constexpr int LH = TH + 2 * S;             // staged rows
  constexpr int NV = LW / N;                 // vectors per staged row
  static_assert(TW % N == 0, "tile width must be a multiple of the vector width");
  using V = typename Vec16<T>::type;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_tb[];
  T* buf0 = reinterpret_cast<T*>(smem_tb);
  T* buf1 = buf0 + LH * LP;

  const index_t tx0 = x_begin + index_t(blockIdx.x) * TW;
  const index_t ty0 = y_begin + index_t(blockIdx.y) * TH;
  const int tid = threadIdx.x;

  // ---- stage (rows ty0-S .. ty0+TH+S-1, cols tx0-SA .. tx0+TW+SA-1)
  for (int i = tid; i < LH * NV; i += 256) {
    const int r = i / NV, v = i - r * NV;
    index_t gy = ty0 - S + r;
    index_t gx = tx0 - SA + index_t(v) * N;
    V val = V(T(0));
    bool ok;
    if constexpr (WRAP) {
      gy = ((gy % H) + H) % H;
      gx = ((gx % W) + W) % W;  // W % N == 0: a wrapped vector never straddles the seam
      ok = true;
    } else {
      ok = gy < H + S && gx < W + SA;  // inside the tile's ghost ring + padding
    }
    if (ok) val = *reinterpret_cast<const V*>(in + core_off + gy * pitch + gx);
    *reinterpret_cast<V*>(buf0 + r * LP + N + v * N) = val;
  }
  __syncthreads();

  // ---- S steps in LDS
  T* src = buf0;
  T* dst = buf1;
#pragma unroll 1
  for (int s = 0; s < S; ++s) {
    for (int i = tid; i < (LH - 2) * NV; i += 256) {
      const int r = 1 + i / NV, v = i - (r - 1) * NV;
      const int base = r * LP + N + v * N;
      const V mid = *reinterpret_cast<const V*>(src + base);
      const V up = *reinterpret_cast<const V*>(src + base - LP);
      const V dn = *reinterpret_cast<const V*>(src + base + LP);
      const T left = src[base - 1];
      const T right = src[base + N];
      V o;
      o[0] = jac<T>(mid[0], up[0], dn[0], left, mid[1 % N], c0, c1);
      if constexpr (N == 2) {
        o[1] = jac<T>(mid[1], up[1], dn[1], mid[0], right, c0, c1);
      } else {
#pragma unroll
        for (int k = 1; k < N - 1; ++k) o[k] = jac<T>(mid[k], up[k], dn[k], mid[k - 1], mid[k + 1], c0, c1);
        o[N - 1] = jac<T>(mid[N - 1], up[N - 1], dn[N - 1], mid[N - 2], right, c0, c1);
      }
      *reinterpret_cast<V*>(dst + base) = o;
    }
    __syncthreads();
    T* t = src;
    src = dst;
    dst = t;
  }

  // ---- write the TW x TH result
  constexpr int OV = TW / N;
  for (int i = tid; i < TH * OV; i += 256) {
    const int r = i / OV, v = i - r * OV;
    const index_t gy = ty0 + r, gx = tx0 + index_t(v) * N;
    if (gy >= y_end || gx >= x_end) continue;
    const V o = *reinterpret_cast<const V*>(src + (r + S) * LP + N + SA + v * N);
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


}  // namespace detail
}  // namespace kernels
}  // namespace mxs

namespace mxs {
namespace kernels {
namespace detail {

// Three-stage pipeline (tuning): levels 1..S0 on the fetching wave, S0+1..S0+S1
// on a middle wave (LDS ring in, LDS ring out), the last S2 on the storing wave;
// 12-wave workgroups (4 strips x 3 stages), 3 waves per SIMD, one wave of each
// stage per SIMD. Same lock-step rule as pipe_chunk, applied per ring: the
// middle stage starts T1 blocks after the fetching one, the storing stage T2
// blocks after the middle one.
template <int S0, int S1, int S2, int PF>
struct Pipe3Shape {
  static constexpr int S = S0 + S1 + S2;
  static constexpr int RING = 3 * PF;
  static constexpr int T1 = (3 * S0 + PF - 1 + PF - 1) / PF;
  static constexpr int T2 = (3 * S1 + PF - 1 + PF - 1) / PF;
};

template <typename B, int S0, int S1, int S2, int PF, bool WRAP>
__device__ __forceinline__ void pipe3_chunk(const typename B::T* __restrict__ in, typename B::T* __restrict__ out,
                                            index_t pitch, index_t core_off, index_t W, index_t H, index_t xw,
                                            index_t x_end, index_t ys, index_t ye, typename B::T c0,
                                            typename B::T c1, typename B::V* __restrict__ ring_a,
                                            typename B::V* __restrict__ ring_b, int stage) {
  static_assert(PF % 3 == 0, "the window rotates through 3 slots: PF must be a multiple of 3");
  using P = Pipe3Shape<S0, S1, S2, PF>;
  constexpr int S = P::S, RING = P::RING, T1 = P::T1, T2 = P::T2;
  using T = typename B::T;
  using V = typename B::V;
  using Sh = StripShape<T, S, true>;
  constexpr int N = Sh::N, SA = Sh::SA, AL = SA / N;
  const int lane = threadIdx.x & (kWaveSize - 1);
  const index_t gx = xw - SA + index_t(lane) * N;
  const index_t rows = ye - ys;
  const index_t n_it0 = rows + 2 * (S1 + S2) + 3 * S0 - 1;  // level-S0 rows [ys - S1 - S2, ye + S1 + S2)
  const index_t n_it1 = rows + 2 * S2 + 3 * S1 - 1;         // level-(S0+S1) rows [ys - S2, ye + S2)
  const index_t n_it2 = rows + 3 * S2 - 1;                  // output rows [ys, ye)
  const index_t b0 = (n_it0 + PF - 1) / PF, b1 = T1 + (n_it1 + PF - 1) / PF, b2 = T1 + T2 + (n_it2 + PF - 1) / PF;
  const index_t blocks = b0 > b1 ? (b0 > b2 ? b0 : b2) : (b1 > b2 ? b1 : b2);

  if (stage == 0) {  // wave-uniform
    V* __restrict__ my = ring_a + lane;
    index_t lx;
    if (xw >= x_end) {
      lx = 0;
    } else if constexpr (WRAP) {
      if (W >= kWaveSize * N) lx = gx < 0 ? gx + W : (gx >= W ? gx - W : gx);
      else lx = ((gx % W) + W) % W;
    } else {
      const index_t last_col = (W + N - 1) / N * N + SA - N;
      lx = gx < last_col ? gx : last_col;
    }
    const T* __restrict__ pin = in + core_off + lx;
    const index_t last_row = ye + S - 1;
    index_t next = ys - S;
    if constexpr (WRAP) next = next < 0 ? next + H : next;
    auto fetch = [&]() -> V {
      const V v = B::load(pin + next * pitch);
      if constexpr (WRAP) {
        ++next;
        next = next == H ? 0 : next;
      } else {
        next = next < last_row ? next + 1 : next;
      }
      return v;
    };
    V win[3][S0];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int l = 0; l < S0; ++l) win[q][l] = B::zero();
    V pf[PF];
#pragma unroll
    for (int k = 0; k < PF; ++k) pf[k] = fetch();
    constexpr int kWarm = (3 * (S0 - 1)) / PF * PF;
#pragma unroll 1
    for (int ib = 0; ib < kWarm; ib += PF) {
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        const int p0 = k % 3, p1 = (k + 1) % 3, p2 = (k + 2) % 3;
        const int b = (ib + k) / 3;
        win[p2][0] = B::enter(pf[k]);
        pf[k] = fetch();
#pragma unroll
        for (int l = S0 - 2; l >= 0; --l)
          if (l <= b) win[p0][l + 1] = B::jac(win[p0][l], win[p1][l], win[p2][l], c0, c1);
      }
      __syncthreads();
    }
#pragma unroll 1
    for (index_t i = kWarm; i < blocks * PF; i += PF) {
      const int base = int((i - (3 * S0 - 1) + index_t(RING) * (3 * S0)) % RING);
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        const int p0 = k % 3, p1 = (k + 1) % 3, p2 = (k + 2) % 3;
        win[p2][0] = B::enter(pf[k]);
        pf[k] = fetch();
        V top;
#pragma unroll
        for (int l = S0 - 1; l >= 0; --l) {
          const V o = B::jac(win[p0][l], win[p1][l], win[p2][l], c0, c1);
          if (l == S0 - 1) top = o;
          else win[p0][l + 1] = o;
        }
        const int slot = base + k < RING ? base + k : base + k - RING;
        my[slot * kWaveSize] = top;
      }
      __syncthreads();
    }
  } else if (stage == 1) {
    const V* __restrict__ src = ring_a + lane;
    V* __restrict__ dst = ring_b + lane;
    V win[3][S1];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int l = 0; l < S1; ++l) win[q][l] = B::zero();
#pragma unroll 1
    for (int t = 0; t < T1; ++t) __syncthreads();
    constexpr int kWarm = (3 * (S1 - 1)) / PF * PF;
#pragma unroll 1
    for (int ib = 0; ib < kWarm; ib += PF) {
      V inrow[PF];
      const int rbase = (ib / PF) % 3 * PF;
#pragma unroll
      for (int k = 0; k < PF; ++k) inrow[k] = src[(rbase + k) * kWaveSize];
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        const int p0 = k % 3, p1 = (k + 1) % 3, p2 = (k + 2) % 3;
        const int b = (ib + k) / 3;
        win[p2][0] = inrow[k];
#pragma unroll
        for (int l = S1 - 2; l >= 0; --l)
          if (l <= b) win[p0][l + 1] = B::jac(win[p0][l], win[p1][l], win[p2][l], c0, c1);
      }
      __syncthreads();
    }
#pragma unroll 1
    for (index_t i = kWarm; i < (blocks - T1) * PF; i += PF) {
      V inrow[PF];
      const int rbase = int((i / PF) % 3) * PF;
      const int wbase = int((i - (3 * S1 - 1) + index_t(RING) * (3 * S1)) % RING);
#pragma unroll
      for (int k = 0; k < PF; ++k) inrow[k] = src[(rbase + k) * kWaveSize];
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        const int p0 = k % 3, p1 = (k + 1) % 3, p2 = (k + 2) % 3;
        win[p2][0] = inrow[k];
        V top;
#pragma unroll
        for (int l = S1 - 1; l >= 0; --l) {
          const V o = B::jac(win[p0][l], win[p1][l], win[p2][l], c0, c1);
          if (l == S1 - 1) top = o;
          else win[p0][l + 1] = o;
        }
        const int slot = wbase + k < RING ? wbase + k : wbase + k - RING;
        dst[slot * kWaveSize] = top;
      }
      __syncthreads();
    }
  } else {
    const V* __restrict__ src = ring_b + lane;
    const T* obase = out + core_off + (xw - SA) + ys * pitch;
    const unsigned long long ob = reinterpret_cast<unsigned long long>(obase);
    const unsigned ob_lo = __builtin_amdgcn_readfirstlane(unsigned(ob)),
                   ob_hi = __builtin_amdgcn_readfirstlane(unsigned(ob >> 32));
    T* obase_u = reinterpret_cast<T*>((static_cast<unsigned long long>(ob_hi) << 32) | ob_lo);
    const int nbytes = __builtin_amdgcn_readfirstlane(int(rows * pitch * index_t(sizeof(T))));
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(obase_u, 0, nbytes, 0x00020000);
    const bool store_lane = lane >= AL && lane < kWaveSize - AL && gx < x_end && xw < x_end;
    const unsigned lane_off = unsigned(lane) * unsigned(N * sizeof(T));
    const unsigned row_bytes = unsigned(pitch) * unsigned(sizeof(T));
    constexpr unsigned kDrop = 0x80000000u;
    V win[3][S2];
#pragma unroll
    for (int q = 0; q < 3; ++q)
#pragma unroll
      for (int l = 0; l < S2; ++l) win[q][l] = B::zero();
#pragma unroll 1
    for (int t = 0; t < T1 + T2; ++t) __syncthreads();
    constexpr int kWarm = (3 * (S2 - 1)) / PF * PF;
#pragma unroll 1
    for (int ib = 0; ib < kWarm; ib += PF) {
      V inrow[PF];
      const int rbase = (ib / PF) % 3 * PF;
#pragma unroll
      for (int k = 0; k < PF; ++k) inrow[k] = src[(rbase + k) * kWaveSize];
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        const int p0 = k % 3, p1 = (k + 1) % 3, p2 = (k + 2) % 3;
        const int b = (ib + k) / 3;
        win[p2][0] = inrow[k];
#pragma unroll
        for (int l = S2 - 2; l >= 0; --l)
          if (l <= b) win[p0][l + 1] = B::jac(win[p0][l], win[p1][l], win[p2][l], c0, c1);
      }
      __syncthreads();
    }
#pragma unroll 1
    for (index_t i = kWarm; i < (blocks - T1 - T2) * PF; i += PF) {
      V inrow[PF];
      const int rbase = int((i / PF) % 3) * PF;
#pragma unroll
      for (int k = 0; k < PF; ++k) inrow[k] = src[(rbase + k) * kWaveSize];
#pragma unroll
      for (int k = 0; k < PF; ++k) {
        const index_t j = i + k;
        const int p0 = k % 3, p1 = (k + 1) % 3, p2 = (k + 2) % 3;
        win[p2][0] = inrow[k];
        V top;
#pragma unroll
        for (int l = S2 - 1; l >= 0; --l) {
          const V o = B::jac(win[p0][l], win[p1][l], win[p2][l], c0, c1);
          if (l == S2 - 1) top = o;
          else win[p0][l + 1] = o;
        }
        const index_t r = j - (3 * S2 - 1);
        const bool ok = store_lane && r >= 0 && r < rows;
        const unsigned off = ok ? lane_off + unsigned(r) * row_bytes : kDrop;
        B::store(top, orsrc, off, c0);
      }
      __syncthreads();
    }
  }
}

template <int S0, int S1, int S2, int PF, bool WRAP, typename T = float, bool SUM = false>
__global__ __launch_bounds__(3 * kBlock) void stencil5_stream_pipe3_kernel(
    const T* __restrict__ in, T* __restrict__ out, index_t pitch, index_t core_off, index_t W, index_t H,
    index_t x_begin, index_t x_end, index_t y_begin, index_t y_end, index_t share, T c0, T c1) {
  using P = Pipe3Shape<S0, S1, S2, PF>;
  using B = typename FastBody<T, SUM>::type;
  constexpr int OW = StripShape<T, P::S, true>::OW;
  __shared__ typename B::V ring[2 * kWavesPerBlock * P::RING * kWaveSize];
  const index_t rows = y_end - y_begin;
  const index_t strips = (x_end - x_begin + OW - 1) / OW;
  const index_t groups = (strips + kWavesPerBlock - 1) / kWavesPerBlock;
  const index_t total = groups * rows;
  const int wave = threadIdx.x / kWaveSize;
  const int strip = wave % kWavesPerBlock, stage = wave / kWavesPerBlock;
  index_t a = index_t(blockIdx.x) * share;
  const index_t b = a + share < total ? a + share : total;
  typename B::V* ra = ring + strip * P::RING * kWaveSize;
  typename B::V* rb = ring + (kWavesPerBlock + strip) * P::RING * kWaveSize;
#pragma unroll 1
  while (a < b) {  // workgroup-uniform: all 12 waves take every chunk (barriers inside)
    const index_t grp = a / rows, r0 = a - grp * rows;
    const index_t r1 = rows < r0 + (b - a) ? rows : r0 + (b - a);
    const index_t xw = x_begin + (grp * kWavesPerBlock + strip) * OW;
    pipe3_chunk<B, S0, S1, S2, PF, WRAP>(in, out, pitch, core_off, W, H, xw, x_end, y_begin + r0, y_begin + r1, c0,
                                         c1, ra, rb, stage);
    a += r1 - r0;
  }
}

// ------------------------------------------------ LDS-crossbar neighbours
// Lane-crossing operands through the LDS crossbar (XB = 1; measured 35-40%
// SLOWER than the DPP forms, profiles/r03_perm). The DPP
// forms spend VALU issue slots on every lane-crossing value: fp32 sum form 2
// scalar v_add_f32_dpp of its 8 slots per level-row (the packed add cannot take
// a DPP source), fp64 4 v_mov_b32_dpp of 18. ds_bpermute_b32 moves the same
// values on the LDS pipe, so the fp32 sum body becomes 7 packed adds (the two
// neighbours land in one pair) and the fp64 sum body 14 adds. Lanes 0 / 63 read
// the other end of the wave instead of DPP's zero fill: apron lanes, never
// stored. Same operands per stored cell: bitwise identical.
__device__ __forceinline__ int lane_addr(int d) { return ((int(__lane_id()) + d) & (kWaveSize - 1)) << 2; }
__device__ __forceinline__ float perm_f(int addr, float v) {
  return __int_as_float(__builtin_amdgcn_ds_bpermute(addr, __float_as_int(v)));
}
__device__ __forceinline__ double perm_d(int addr, double v) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_ds_bpermute(addr, int(b & 0xffffffff));
  const int hi = __builtin_amdgcn_ds_bpermute(addr, int(b >> 32));
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}
__device__ __forceinline__ f32x4 sum_rot4f_perm(const f32x4& up, const f32x4& mid, const f32x4& dn) {
  const f32x2 am = mid.xy, bm = mid.zw;  // (c1, c2), (c3, c0)
  const f32x2 ns_a = up.xy + dn.xy, ns_b = up.zw + dn.zw;
  const f32x2 p = pk_add_swap(am, bm);   // (c1 + c0, c2 + c3)
  const f32x2 h_a = pk_add_swap(p, am);  // h3(c1), h3(c2)
  f32x2 nb;
  nb.x = perm_f(lane_addr(1), bm.y);      // c4 = lane + 1's c0
  nb.y = perm_f(lane_addr(-1), bm.x);     // c[-1] = lane - 1's c3
  const f32x2 h_b = pk_add_swap(nb, p);  // (c4 + p23, c[-1] + p01) = h3(c3), h3(c0)
  f32x4 o;
  o.xy = ns_a + h_a;
  o.zw = ns_b + h_b;
  return o;
}
__device__ __forceinline__ f64x4 sum_w4d_perm(const f64x4& up, const f64x4& mid, const f64x4& dn) {
  const double left = perm_d(lane_addr(-1), mid.w);
  const double right = perm_d(lane_addr(1), mid.x);
  const double p01 = mid.x + mid.y, p23 = mid.z + mid.w;
  f64x4 o;
  o.x = (up.x + dn.x) + (p01 + left);
  o.y = (up.y + dn.y) + (p01 + mid.z);
  o.z = (up.z + dn.z) + (p23 + mid.y);
  o.w = (up.w + dn.w) + (p23 + right);
  return o;
}
struct BodySumF32Perm : BodySumF32 {
  static __device__ __forceinline__ V jac(const V& u, const V& m, const V& d, float, float) {
    return sum_rot4f_perm(u, m, d);
  }
};
struct BodySumF64Perm : BodySumF64 {
  static __device__ __forceinline__ V jac(const V& u, const V& m, const V& d, double, double) {
    return sum_w4d_perm(u, m, d);
  }
};


// fp64 register-pressure variants of the sum body (TUNE_FOCUS=spill in
// stencil_tune64): XB = 5 enters loaded rows without the copy into fresh
// registers, XB = 6 fences the fetching stage's row iterations.
struct BodySumF64NoCopy : BodySumF64 {
  static __device__ __forceinline__ V enter(const V& v) { return v; }
};
struct BodySumF64Fence : BodySumF64 {
  static constexpr bool kStage0Fence = true;
};
template <>
struct FastBody<double, true, 5> {
  using type = BodySumF64NoCopy;
};
template <>
struct FastBody<double, true, 6> {
  using type = BodySumF64Fence;
};

template <>
struct FastBody<float, true, 1> {
  using type = BodySumF32Perm;
};
// Non-temporal 16-byte loads of the fetching stage (TUNE_FOCUS=ntload): the
// input rows are read once per pass.
struct BodySumF32NT : BodySumF32 {
  static __device__ __forceinline__ V load(const float* p) {
    return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(p));
  }
};
template <>
struct FastBody<float, true, 7> {
  using type = BodySumF32NT;
};
template <>
struct FastBody<double, true, 1> {
  using type = BodySumF64Perm;
};

}  // namespace detail
}  // namespace kernels
}  // namespace mxs
