// Stencil kernel tuning harness (one process, interleaved rounds: rule 24 of
// cdna_hip_programming.md §5.4). Times every RegisterRoll instantiation, the
// LDS-tile variant and a float4 copy of the same bytes (the achievable
// read+write roofline) on a W x H fp32 tile; prints one JSON line per variant.
//
//   stencil_tune [W] [H] [rounds]
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

__global__ __launch_bounds__(256) void copy4(const float4* __restrict__ a, float4* __restrict__ b, index_t n) {
  const index_t stride = index_t(gridDim.x) * blockDim.x;
  for (index_t i = index_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) b[i] = a[i];
}

// Balanced rotated kernel with per-wave timestamps (s_memrealtime, 100 MHz, and
// s_memtime, shader clock) at start and end: measures the wave lifetime against
// the dispatch, i.e. tail / imbalance vs clock (TUNE_FOCUS=stamp).
template <int S, bool WRAP, bool PRIO>
__global__ __launch_bounds__(256) void balanced_stamped(const float* __restrict__ in, float* __restrict__ out,
                                                        index_t pitch, index_t core_off, index_t W, index_t H,
                                                        index_t x_begin, index_t x_end, index_t y_begin,
                                                        index_t y_end, index_t share, float c0, float c1,
                                                        unsigned long long* stamps) {
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), t0 = __builtin_amdgcn_s_memtime();
  constexpr int OW = StreamShape<float, S>::OW;
  const index_t rows = y_end - y_begin;
  const index_t strips = (x_end - x_begin + OW - 1) / OW;
  const index_t groups = (strips + kWavesPerBlock - 1) / kWavesPerBlock;
  const index_t total = groups * rows;
  const int wave = threadIdx.x / kWaveSize;
  index_t a = index_t(blockIdx.x) * share;
  const index_t a0 = a;
  const index_t b = a + share < total ? a + share : total;
  WavePrio wp;
  if (PRIO && b > a) wp.quarters = 4.f / float(b - a);
  while (a < b) {
    const index_t grp = a / rows, q0 = a - grp * rows;
    const index_t q1 = rows < q0 + (b - a) ? rows : q0 + (b - a);
    const index_t xw = x_begin + (grp * kWavesPerBlock + wave) * OW;
    wp.done = a - a0;
    if (xw < x_end)
      stream_chunk_rot<S, 3, WRAP>(in, out, pitch, core_off, W, H, xw, x_end, y_begin + q0, y_begin + q1, c0, c1, &wp);
    a += q1 - q0;
  }
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime(), t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) {
    unsigned long long* p = stamps + (size_t(blockIdx.x) * 4 + wave) * 6;
    p[0] = r0; p[1] = r1; p[2] = t0; p[3] = t1;
    p[4] = __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_REG_HW_ID
    p[5] = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // HW_REG_XCC_ID
  }
}


// The production pipeline pass (joint windows, sum form) with per-workgroup
// clock stamps at entry and exit (TUNE_FOCUS=fillfit): the shader cycles each
// workgroup spends on its share, against the share's rows, fitted to
// cycles = fixed + per_row x rows over several tile heights (the fill per
// share is the fixed part). stamps[6 b ..]: realtime in / out, s_memtime in /
// out, share rows, chunks.
template <int S0, int S1, int PF, bool WRAP, int LAG1>
__global__ __launch_bounds__(2 * kWavesPerBlock * kWaveSize) void pipe_stamped(
    const float* __restrict__ in, float* __restrict__ out, index_t pitch, index_t core_off, index_t W, index_t H,
    index_t x_begin, index_t x_end, index_t y_begin, index_t y_end, const PipeShares shares, float c0, float c1,
    unsigned long long* stamps) {
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), t0 = __builtin_amdgcn_s_memtime();
  constexpr int G = kWavesPerBlock;
  using P = PipeShape<S0, S1, PF>;
  using B = BodySumF32;
  constexpr int OWG = JointShape<S0, S1, G>::OWG;
  __shared__ B::V ring[G * P::RING * kWaveSize];
  const index_t rows = y_end - y_begin;
  const int wave = threadIdx.x / kWaveSize;
  const int strip = wave % G, stage = wave / G;
  index_t a = shares.start[blockIdx.x], b = shares.start[blockIdx.x + 1];
  const index_t share_rows = b - a;
  int chunks = 0;
#pragma unroll 1
  while (a < b) {
    const index_t grp = a / rows, q0 = a - grp * rows;
    const index_t q1 = rows < q0 + (b - a) ? rows : q0 + (b - a);
    pipe_chunk<B, S0, S1, PF, WRAP, true, G, LAG1>(in, out, pitch, core_off, W, H, x_begin + grp * OWG, x_end,
                                                   y_begin + q0, y_begin + q1, c0, c1, ring, stage, strip);
    a += q1 - q0;
    ++chunks;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long* p = stamps + size_t(blockIdx.x) * 6;
    p[0] = r0;
    p[1] = __builtin_amdgcn_s_memrealtime();
    p[2] = t0;
    p[3] = __builtin_amdgcn_s_memtime();
    p[4] = (unsigned long long)share_rows;
    p[5] = (unsigned long long)chunks | ((unsigned long long)__builtin_amdgcn_s_getreg(20 | (31 << 11)) << 16) |
           ((unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11)) << 32);  // XCC_ID, HW_ID
  }
}

// TUNE_FOCUS=fillfit: one pipeline form over rows [0, h) of the ghost-ring
// tile for several h, `reps` stamped passes each; per h the median over passes
// of the median / max workgroup cycles and of the pass's span.
template <int S0, int S1, int PF, int LAG1>
void fillfit(const char* name, const float* in, float* out, const TileGeom& g, const std::vector<index_t>& heights,
             int reps) {
  constexpr int OWG = JointShape<S0, S1, kWavesPerBlock>::OWG;
  int cus = 0;
  MXS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = cus;  // one 512-thread workgroup per CU (VGPR-bound)
  DeviceBuffer<unsigned long long> st(index_t(blocks) * 6);
  std::vector<unsigned long long> h(size_t(blocks) * 6);
  const float c0 = float(std::pow(0.2, S0 + S1));
  const index_t groups = (g.width + OWG - 1) / OWG;
  for (index_t hh : heights) {
    PipeShares shares = PipeShares::equal((groups * hh + blocks - 1) / blocks);
    pipe_starts(groups, hh, blocks, pipe_fill_rows<S0, S1, PF, LAG1>(), &shares);
    auto launch = [&](const float* I, float* O) {
      pipe_stamped<S0, S1, PF, false, LAG1><<<blocks, 2 * kBlock>>>(I, O, g.pitch, g.core_offset(), g.width, g.height,
                                                                     0, g.width, 0, hh, shares, c0, 0.2f, st.get());
    };
    std::vector<double> med_c, max_c, span, mhz, rows_mean, start_p50, start_max, end_min, end_p50, end_max;
    std::vector<std::vector<double>> xcd_c(8), xcd_start(8), xcd_clk(8);
    for (int r = 0; r < reps + 3; ++r) {
      if (r & 1) launch(out, const_cast<float*>(in));
      else launch(in, out);
      MXS_HIP_CHECK(hipDeviceSynchronize());
      if (r < 3) continue;
      MXS_HIP_CHECK(hipMemcpy(h.data(), st.get(), h.size() * 8, hipMemcpyDeviceToHost));
      std::vector<double> c, clk;
      unsigned long long rmin = ~0ull, rmax = 0;
      double rows = 0;
      for (int b = 0; b < blocks; ++b) {
        const unsigned long long* p = &h[size_t(b) * 6];
        c.push_back(double(p[3] - p[2]));
        clk.push_back(double(p[3] - p[2]) / double(std::max<unsigned long long>(p[1] - p[0], 1)) * 100.0);  // MHz
        rmin = std::min(rmin, p[0]);
        rmax = std::max(rmax, p[1]);
        rows += double(p[4]);
      }
      std::vector<double> st0, en0;  // us after the first workgroup's start
      for (int b = 0; b < blocks; ++b) {
        const unsigned long long* p = &h[size_t(b) * 6];
        st0.push_back(double(p[0] - rmin) / 100.0);
        en0.push_back(double(p[1] - rmin) / 100.0);
        const int x = int((p[5] >> 16) & 0xf) & 7;
        xcd_c[size_t(x)].push_back(double(p[3] - p[2]));
        xcd_start[size_t(x)].push_back(double(p[0] - rmin) / 100.0);
        xcd_clk[size_t(x)].push_back(double(p[3] - p[2]) / double(std::max<unsigned long long>(p[1] - p[0], 1)) * 100.0);
      }
      std::sort(st0.begin(), st0.end());
      std::sort(en0.begin(), en0.end());
      start_p50.push_back(st0[st0.size() / 2]);
      start_max.push_back(st0.back());
      end_min.push_back(en0.front());
      end_p50.push_back(en0[en0.size() / 2]);
      end_max.push_back(en0.back());
      std::sort(c.begin(), c.end());
      std::sort(clk.begin(), clk.end());
      med_c.push_back(c[c.size() / 2]);
      max_c.push_back(c.back());
      span.push_back(double(rmax - rmin) / 100.0);
      mhz.push_back(clk[clk.size() / 2]);
      rows_mean.push_back(rows / blocks);
    }
    auto med = [](std::vector<double> v) {
      std::sort(v.begin(), v.end());
      return v[v.size() / 2];
    };
    std::printf("{\"fillfit\": \"%s\", \"W\": %ld, \"h\": %ld, \"groups\": %ld, \"rows_per_wg\": %.1f, "
                "\"model_fill_rows\": %ld, \"wg_kcycles_median\": %.2f, \"wg_kcycles_max\": %.2f, \"span_us\": %.2f, "
                "\"mhz\": %.0f, \"pass_kcycles\": %.1f}\n",
                name, long(g.width), long(hh), long(groups), med(rows_mean), long(pipe_fill_rows<S0, S1, PF, LAG1>()),
                med(med_c) / 1e3, med(max_c) / 1e3, med(span), med(mhz), med(span) * med(mhz) / 1e3);
    std::printf("{\"fillfit_skew\": \"%s\", \"h\": %ld, \"start_us_p50\": %.2f, \"start_us_max\": %.2f, "
                "\"end_us_min\": %.2f, \"end_us_p50\": %.2f, \"end_us_max\": %.2f, \"xcd\": [",
                name, long(hh), med(start_p50), med(start_max), med(end_min), med(end_p50), med(end_max));
    for (int x = 0; x < 8; ++x)
      std::printf("%s[%zu, %.1f, %.2f, %.0f]", x ? ", " : "", xcd_c[size_t(x)].size() / size_t(reps),
                  xcd_c[size_t(x)].empty() ? 0.0 : med(xcd_c[size_t(x)]) / 1e3,
                  xcd_start[size_t(x)].empty() ? 0.0 : med(xcd_start[size_t(x)]),
                  xcd_clk[size_t(x)].empty() ? 0.0 : med(xcd_clk[size_t(x)]));
    std::printf("]}\n");
    for (auto& v : xcd_c) v.clear();
    for (auto& v : xcd_start) v.clear();
    for (auto& v : xcd_clk) v.clear();
    std::fflush(stdout);
  }
}

struct Variant {
  std::string name;
  std::function<void(hipStream_t)> launch;
  std::vector<float> ms;
  int steps = 1;  // Jacobi iterations per launch
  std::function<void(hipStream_t)> ref;  // validated kernel computing the same thing
  // The same kernel with input and output swapped: timed launches alternate
  // launch / launch2 like the solver's ping-pong. Re-reading one never-written
  // input would let a 256 MiB tile (8192^2) stay in the 256 MB Infinity Cache
  // and read ~30% faster than any real time step (measured: 129 vs 171 us).
  std::function<void(hipStream_t)> launch2;
  float tol = 0.f;  // 0: bitwise against ref; > 0: max |difference| (sum-form kernels)
};

template <int ROWS, int CH, bool NT, int WX, bool NTL, int NW = 4>
Variant roll(const float* in, float* out, const TileGeom& g) {
  char buf[128];
  std::snprintf(buf, sizeof(buf), "roll_r%d_c%d_nt%d_wx%d_ntl%d_nw%d", ROWS, CH, int(NT), WX, int(NTL), NW);
  return {buf, [=](hipStream_t s) {
            constexpr int WY = NW / WX;
            const index_t gx = (g.width + 256 * WX - 1) / (256 * WX);
            const index_t gy = (g.height + ROWS * WY - 1) / (ROWS * WY);
            stencil5_roll_kernel<float, ROWS, CH, NT, WX, NTL, NW><<<dim3(gx, gy), NW * 64, 0, s>>>(
                in, out, g.pitch, g.core_offset(), g.width, 0, g.height, 0.2f, 0.2f);
          }};
}

template <int S, int TW, int TH>
Variant tb(const float* in, float* out, const TileGeom& g) {
  char buf[128];
  std::snprintf(buf, sizeof(buf), "tb_s%d_tw%d_th%d", S, TW, TH);
  Variant v{buf, [=](hipStream_t s) {
              const size_t lds = tb_lds_bytes<float, S, TW, TH>();
              const dim3 grid(unsigned((g.width + TW - 1) / TW), unsigned((g.height + TH - 1) / TH));
              stencil5_tb_kernel<float, S, TW, TH, true><<<grid, 256, lds, s>>>(
                  in, out, g.pitch, g.core_offset(), g.width, g.height, 0, g.width, 0, g.height, 0.2f, 0.2f);
            }};
  v.steps = S;
  return v;
}

template <int S, int TW, int TH, bool WRAP = true>
Variant tb1(const float* in, float* out, const TileGeom& g) {
  char buf[128];
  std::snprintf(buf, sizeof(buf), "tb1_s%d_tw%d_th%d%s", S, TW, TH, WRAP ? "_wrap" : "");
  Variant v{buf, [=](hipStream_t s) {
              const size_t lds = tb1_lds_bytes<float, S, TW, TH>();
              const dim3 grid(unsigned((g.width + TW - 1) / TW), unsigned((g.height + TH - 1) / TH));
              stencil5_tb1_kernel<float, S, TW, TH, WRAP><<<grid, 256, lds, s>>>(
                  in, out, g.pitch, g.core_offset(), g.width, g.height, 0, g.width, 0, g.height, 0.2f, 0.2f);
            }};
  v.steps = S;
  return v;
}

// Reference launcher for S-step variants: the validated LDS kernel (S <= 8), or
// two periodic half-blocks through `tmp` (wrap only; without wrap the frozen
// ghost ring differs).
template <int S, bool WRAP>
std::function<void(hipStream_t)> ref_for(const float* in, float* out, const TileGeom& g, float* tmp) {
  if constexpr (S <= 8) {
    return tb1<S, 128, 32, WRAP>(in, out, g).launch;
  } else if constexpr (WRAP && S % 2 == 0) {
    if (!tmp) return {};
    auto first = tb1<S / 2, 128, 32, true>(in, tmp, g).launch;
    auto second = tb1<S / 2, 128, 32, true>(tmp, out, g).launch;
    return [=](hipStream_t s) {
      first(s);
      second(s);
    };
  } else {
    return {};
  }
}

template <int S, int PF, bool WRAP = false, bool DPP = true, bool ROT = false>
Variant stream(const float* in, float* out, const TileGeom& g, int ch, float* tmp = nullptr) {
  char buf[128];
  std::snprintf(buf, sizeof(buf), "stream_s%d_pf%d_ch%d%s%s%s", S, PF, ch, WRAP ? "_wrap" : "", DPP ? "" : "_bperm",
                ROT ? "_rot" : "");
  auto mk = [=](const float* I, float* O) {
    return [=](hipStream_t s) {
      constexpr int OW = StreamShape<float, S>::OW;
      const index_t strips = (g.width + OW - 1) / OW;
      const dim3 grid(unsigned((strips + 3) / 4), unsigned((g.height + ch - 1) / ch));
      stencil5_stream_kernel<float, S, PF, WRAP, DPP, ROT><<<grid, 256, 0, s>>>(
          I, O, g.pitch, g.core_offset(), g.width, g.height, 0, g.width, 0, g.height, index_t(ch), 0.2f, 0.2f);
    };
  };
  Variant v{buf, mk(in, out)};
  v.launch2 = mk(out, const_cast<float*>(in));
  v.steps = S;
  v.ref = ref_for<S, WRAP>(in, out, g, tmp);
  return v;
}

// Balanced persistent launch: `per_cu` resident workgroups per CU (0 = occupancy API).
template <int S, int PF, bool WRAP = false, bool ROT = false, bool SUM = false>
Variant balanced(const float* in, float* out, const TileGeom& g, int per_cu, float* tmp = nullptr) {
  int blocks_per_cu = per_cu;
  if (blocks_per_cu <= 0)
    MXS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &blocks_per_cu,
        reinterpret_cast<const void*>(stencil5_stream_balanced_kernel<float, S, PF, WRAP, true, ROT, SUM>), 256, 0));
  int cus = 0;
  MXS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = std::max(1, blocks_per_cu * cus);
  char buf[128];
  std::snprintf(buf, sizeof(buf), "balanced_s%d_pf%d_b%d%s%s%s", S, PF, blocks_per_cu, WRAP ? "_wrap" : "",
                ROT ? "_rot" : "", SUM ? "_sum" : "");
  const float c0 = SUM ? float(std::pow(0.2, S)) : 0.2f;  // sum form: c0 carries c^S
  auto mk = [=](const float* I, float* O) {
    return [=](hipStream_t s) {
      constexpr int OW = StreamShape<float, S>::OW;
      const index_t groups = ((g.width + OW - 1) / OW + 3) / 4;
      const index_t share = (groups * g.height + blocks - 1) / blocks;
      stencil5_stream_balanced_kernel<float, S, PF, WRAP, true, ROT, SUM><<<blocks, 256, 0, s>>>(
          I, O, g.pitch, g.core_offset(), g.width, g.height, 0, g.width, 0, g.height, share, c0, 0.2f);
    };
  };
  Variant v{buf, mk(in, out)};
  v.launch2 = mk(out, const_cast<float*>(in));
  v.steps = S;
  v.ref = ref_for<S, WRAP>(in, out, g, tmp);
  if (SUM) v.tol = 2e-6f;
  return v;
}

// Two-stage wave pipeline (S = S0 + S1 levels; 512-thread workgroups).
template <int S0, int S1, int PF, bool WRAP = true, int PRIO = 0, bool SUM = false, int G = 4, bool XM = false,
          bool JOINT = false, int LAG1 = 0, int XB = 0>
Variant pipe(const float* in, float* out, const TileGeom& g, float* tmp = nullptr) {
  int per_cu = 0, cus = 0;
  constexpr int threads = 2 * G * kWaveSize;
  MXS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &per_cu, reinterpret_cast<const void*>(stencil5_stream_pipe_kernel<S0, S1, PF, WRAP, PRIO, float, SUM, G, XM, JOINT, LAG1, XB>),
      threads, 0));
  MXS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = std::max(1, per_cu * cus);
  char buf[128];
  std::snprintf(buf, sizeof(buf), "pipe_s%d+%d_pf%d_b%d%s%s%s%s%s%s%s%s", S0, S1, PF, per_cu, WRAP ? "_wrap" : "",
                PRIO == 1 ? "_prio0" : (PRIO == 2 ? "_prio1" : ""), SUM ? "_sum" : "",
                G == 4 ? "" : (G == 2 ? "_g2" : "_g1"), XM ? "_xcd" : "", JOINT ? "_joint" : "", LAG1 == 3 ? "_lag1" : (LAG1 == 2 ? "_lag1s1" : (LAG1 == 1 ? "_lag1s0" : "")),
                XB == 1 ? "_perm" : (XB == 7 ? "_ntload" : ""));
  const float c0 = SUM ? float(std::pow(0.2, S0 + S1)) : 0.2f;  // sum form: c0 carries c^S
  auto mk = [=](const float* I, float* O) {
    return [=](hipStream_t s) {
      constexpr int OW = StreamShape<float, S0 + S1>::OW;
      constexpr int OWG = JointShape<S0, S1, G>::OWG;
      const index_t groups = JOINT ? (g.width + OWG - 1) / OWG : ((g.width + OW - 1) / OW + G - 1) / G;
      const index_t share = (groups * g.height + blocks - 1) / blocks;
      // The production shares (fill-aware starts unless MXS_PIPE_BALANCED=0; XM
      // permutes workgroups, so it keeps equal shares).
      PipeShares shares = PipeShares::equal(share);
      if (!XM && G == kWavesPerBlock && pipe_balanced() && blocks <= kMaxShareBlocks)
        pipe_starts(groups, g.height, blocks, pipe_fill_rows<S0, S1, PF, LAG1>(), &shares);
      stencil5_stream_pipe_kernel<S0, S1, PF, WRAP, PRIO, float, SUM, G, XM, JOINT, LAG1, XB><<<blocks, threads, 0, s>>>(
          I, O, g.pitch, g.core_offset(), g.width, g.height, 0, g.width, 0, g.height, shares, c0, 0.2f);
    };
  };
  Variant v{buf, mk(in, out)};
  v.launch2 = mk(out, const_cast<float*>(in));
  v.steps = S0 + S1;
  v.ref = ref_for<S0 + S1, WRAP>(in, out, g, tmp);
  if (SUM) v.tol = 2e-6f;
  return v;
}

// Row-band shares (TUNE_FOCUS=bands): every column group split into `per_group`
// equal row bands, one per workgroup (groups x per_group workgroups, so some CUs
// idle), so the workgroups of neighbouring groups stream the same rows at the
// same time and the columns their joint windows both read (20 on each side)
// can hit the memory-side cache for the second reader.
template <int S0, int S1, int PF, int LAG1>
Variant pipe_bands(const float* in, float* out, const TileGeom& g, int per_group, float* tmp = nullptr) {
  constexpr int G = kWavesPerBlock, threads = 2 * G * kWaveSize;
  constexpr int OWG = JointShape<S0, S1, G>::OWG;
  const index_t groups = (g.width + OWG - 1) / OWG;
  const int blocks = int(groups) * per_group;
  MXS_CHECK(blocks <= kMaxShareBlocks, "pipe_bands: too many workgroups");
  char buf[128];
  std::snprintf(buf, sizeof(buf), "pipe_s%d+%d_pf%d_wrap_sum_joint_lag1_bands%d_b%d", S0, S1, PF, per_group, blocks);
  const float c0 = float(std::pow(0.2, S0 + S1));
  auto mk = [=](const float* I, float* O) {
    return [=](hipStream_t s) {
      PipeShares shares = PipeShares::equal(0);
      shares.n = blocks;
      for (int w = 0; w < blocks; ++w)
        shares.start[w] = int(index_t(w / per_group) * g.height + (index_t(w % per_group) * g.height) / per_group);
      shares.start[blocks] = int(groups * g.height);
      stencil5_stream_pipe_kernel<S0, S1, PF, true, 0, float, true, G, false, true, LAG1, 0><<<blocks, threads, 0, s>>>(
          I, O, g.pitch, g.core_offset(), g.width, g.height, 0, g.width, 0, g.height, shares, c0, 0.2f);
    };
  };
  Variant v{buf, mk(in, out)};
  v.launch2 = mk(out, const_cast<float*>(in));
  v.steps = S0 + S1;
  v.ref = ref_for<S0 + S1, true>(in, out, g, tmp);
  v.tol = 2e-6f;
  return v;
}

// Three-stage wave pipeline (S = S0 + S1 + S2 levels; 768-thread workgroups).
template <int S0, int S1, int S2, int PF, bool WRAP = true, bool SUM = true>
Variant pipe3(const float* in, float* out, const TileGeom& g, float* tmp = nullptr) {
  int per_cu = 0, cus = 0;
  constexpr int threads = 3 * 4 * kWaveSize;
  MXS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &per_cu, reinterpret_cast<const void*>(stencil5_stream_pipe3_kernel<S0, S1, S2, PF, WRAP, float, SUM>),
      threads, 0));
  MXS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = std::max(1, per_cu * cus);
  char buf[128];
  std::snprintf(buf, sizeof(buf), "pipe3_s%d+%d+%d_pf%d_b%d%s%s", S0, S1, S2, PF, per_cu, WRAP ? "_wrap" : "",
                SUM ? "_sum" : "");
  constexpr int S = S0 + S1 + S2;
  const float c0 = SUM ? float(std::pow(0.2, S)) : 0.2f;
  auto mk = [=](const float* I, float* O) {
    return [=](hipStream_t s) {
      constexpr int OW = StreamShape<float, S>::OW;
      const index_t groups = ((g.width + OW - 1) / OW + 3) / 4;
      const index_t share = (groups * g.height + blocks - 1) / blocks;
      stencil5_stream_pipe3_kernel<S0, S1, S2, PF, WRAP, float, SUM><<<blocks, threads, 0, s>>>(
          I, O, g.pitch, g.core_offset(), g.width, g.height, 0, g.width, 0, g.height, share, c0, 0.2f);
    };
  };
  Variant v{buf, mk(in, out)};
  v.launch2 = mk(out, const_cast<float*>(in));
  v.steps = S;
  v.ref = ref_for<S, WRAP>(in, out, g, tmp);
  if (SUM) v.tol = 2e-6f;
  return v;
}

int main(int argc, char** argv) {
  const index_t W = argc > 1 ? atol(argv[1]) : 32768;
  const index_t H = argc > 2 ? atol(argv[2]) : 32768;
  const int rounds = argc > 3 ? atoi(argv[3]) : 5;
  const TileGeom g = TileGeom::aligned(W, H, 32, 32, 4);  // 32-deep ghost ring: non-wrap variants up to S = 32
  DeviceBuffer<float> a(g.alloc_elems()), b(g.alloc_elems()), c(g.alloc_elems());
  // Random data: zero-filled operands raise the clock under load and inflate
  // the numbers (cdna_hip_programming.md §5.4 rule 25).
  kernels::fill<float>(a.get(), g.alloc_elems(), 0.f, nullptr);
  kernels::fill<float>(b.get(), g.alloc_elems(), 0.f, nullptr);
  kernels::fill_random<float>(a.get(), g, 0, 0, W, 7, 0.f, 1.f, nullptr);
  kernels::fill_random<float>(b.get(), g, 0, 0, W, 8, 0.f, 1.f, nullptr);
  MXS_HIP_CHECK(hipDeviceSynchronize());
  const float* in = a.get();
  float* out = b.get();
  std::vector<Variant> vs;
  const index_t n4 = g.alloc_elems() / 4;
  vs.push_back({"copy_float4", [=](hipStream_t s) {
                  copy4<<<kNumCUs * 8, 256, 0, s>>>(reinterpret_cast<const float4*>(in), reinterpret_cast<float4*>(out), n4);
                }});
  vs.back().launch2 = [=](hipStream_t s) {
    copy4<<<kNumCUs * 8, 256, 0, s>>>(reinterpret_cast<const float4*>(out), reinterpret_cast<float4*>(const_cast<float*>(in)), n4);
  };
  vs.push_back({"lds_th16", [=](hipStream_t s) {
                  const index_t gx = (W + 255) / 256, gy = (H + 15) / 16;
                  stencil5_lds_kernel<float, 16><<<dim3(gx, gy), 256, (16 + 2) * (256 + 8) * 4, s>>>(
                      in, out, g.pitch, g.core_offset(), W, 0, H, 0.2f, 0.2f);
                }});
  vs.push_back(roll<3, 3, true, 4, false>(in, out, g));
  vs.push_back(roll<4, 4, true, 4, false>(in, out, g));
  vs.push_back(tb1<4, 128, 32, false>(in, out, g));
  vs.push_back(tb1<4, 128, 32, true>(in, out, g));
  vs.push_back(tb1<4, 192, 24, false>(in, out, g));
  vs.push_back(tb1<6, 128, 32, false>(in, out, g));
  float* tmp = c.get();
  const char* focus = std::getenv("TUNE_FOCUS");
  if (focus && std::string(focus) == "fillfit") {  // fill per share: workgroup cycles vs share rows (ghost tile)
    const int reps = rounds;
    std::vector<index_t> hs;
    for (index_t hh = H; hh >= 1024 && hs.size() < 5; hh /= 2) hs.push_back(hh);
    const char* set = std::getenv("TUNE_FILL_SET");
    if (set && std::string(set) == "split") {  // stage splits of S = 20, ascending (10 + 10, 11 + 9 need a 24-deep ring)
      fillfit<12, 8, 6, 3>("12+8_pf6_asc", in, out, g, hs, reps);
      fillfit<10, 10, 6, 3>("10+10_pf6_asc", in, out, g, hs, reps);
      fillfit<11, 9, 6, 3>("11+9_pf6_asc", in, out, g, hs, reps);
      fillfit<13, 7, 6, 3>("13+7_pf6_asc", in, out, g, hs, reps);
      return 0;
    }
    if (set && std::string(set) == "deep0") {  // deeper stage 0: 16 + 4 (888-column groups) against 12 + 8
      fillfit<12, 8, 6, 3>("12+8_pf6_asc", in, out, g, hs, reps);
      fillfit<16, 4, 6, 3>("16+4_pf6_asc", in, out, g, hs, reps);
      fillfit<12, 8, 6, 3>("12+8_pf6_asc_b", in, out, g, hs, reps);
      fillfit<16, 4, 6, 3>("16+4_pf6_asc_b", in, out, g, hs, reps);
      return 0;
    }
    if (set && std::string(set) == "prod") {  // the forms the launcher picks: ascending <= 768-row shares, else descending
      fillfit<12, 8, 6, 3>("12+8_pf6_asc", in, out, g, hs, reps);
      fillfit<12, 8, 6, 0>("12+8_pf6_desc", in, out, g, hs, reps);
      return 0;
    }
    fillfit<12, 8, 6, 3>("12+8_pf6_asc", in, out, g, hs, reps);
    fillfit<12, 8, 3, 3>("12+8_pf3_asc", in, out, g, hs, reps);
    fillfit<12, 8, 6, 0>("12+8_pf6_desc", in, out, g, hs, reps);
    fillfit<8, 12, 6, 3>("8+12_pf6_asc", in, out, g, hs, reps);
    fillfit<16, 4, 6, 3>("16+4_pf6_asc", in, out, g, hs, reps);
    fillfit<12, 8, 9, 3>("12+8_pf9_asc", in, out, g, hs, reps);
    return 0;
  }
  if (focus && std::string(focus) == "stamp") {  // per-wave lifetimes of the default S = 16 rotated kernel
    int occ = 0, cus = 0;
    MXS_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &occ, reinterpret_cast<const void*>(balanced_stamped<16, true, true>), 256, 0));
    MXS_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int blocks = std::max(occ, 1) * cus;
    constexpr int OW = StreamShape<float, 16>::OW;
    const index_t groups = ((W + OW - 1) / OW + 3) / 4;
    const index_t share = (groups * H + blocks - 1) / blocks;
    DeviceBuffer<unsigned long long> st(size_t(blocks) * 24);
    Stream ss;
    for (int rep = 0; rep < 4; ++rep) {
      if (std::getenv("STAMP_NOPRIO"))
        balanced_stamped<16, true, false><<<blocks, 256, 0, ss.get()>>>(in, out, g.pitch, g.core_offset(), W, H, 0, W,
                                                                        0, H, share, 0.2f, 0.2f, st.get());
      else
        balanced_stamped<16, true, true><<<blocks, 256, 0, ss.get()>>>(in, out, g.pitch, g.core_offset(), W, H, 0, W,
                                                                       0, H, share, 0.2f, 0.2f, st.get());
      MXS_HIP_CHECK(hipGetLastError());
      ss.sync();
    }
    std::vector<unsigned long long> h(size_t(blocks) * 24);
    MXS_HIP_CHECK(hipMemcpy(h.data(), st.get(), h.size() * 8, hipMemcpyDeviceToHost));
    unsigned long long rmin = ~0ull, rmax = 0;
    for (int w = 0; w < blocks * 4; ++w) {
      rmin = std::min(rmin, h[size_t(w) * 6]);
      rmax = std::max(rmax, h[size_t(w) * 6 + 1]);
    }
    // One line per wave: block wave xcc se cu simd start_us end_us clock_ghz
    for (int w = 0; w < blocks * 4; ++w) {
      const unsigned long long* p = &h[size_t(w) * 6];
      const unsigned hw = unsigned(p[4]);
      const double clk = double(p[3] - p[2]) / double(std::max<unsigned long long>(p[1] - p[0], 1)) * 100e6 / 1e9;
      std::printf("W %d %d %u %u %u %u %.1f %.1f %.3f\n", w / 4, w % 4, unsigned(p[5]) & 0xf, (hw >> 13) & 0x7,
                  (hw >> 8) & 0xf, (hw >> 4) & 0x3, (p[0] - rmin) / 100.0, (p[1] - rmin) / 100.0, clk);
    }
    std::printf("{\"stamp_blocks\": %d, \"span_us\": %.1f}\n", blocks, (rmax - rmin) / 100.0);
    return 0;
  } else if (focus && std::string(focus) == "one") {  // counter runs: the default S = 16 kernel, both layouts
    vs.push_back(balanced<16, 3, true>(in, out, g, 0));
    vs.push_back(balanced<16, 3, true, true>(in, out, g, 0));
  } else if (focus && std::string(focus) == "rot") {  // rotated-pair fp32 layout vs natural, per S
    vs.push_back(balanced<16, 3, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<16, 3, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<16, 3, false>(in, out, g, 0));
    vs.push_back(balanced<16, 3, false, true>(in, out, g, 0));
    vs.push_back(balanced<12, 3, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<12, 3, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<8, 3, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<14, 3, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<16, 6, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<16, 6, false, true>(in, out, g, 0));
    vs.push_back(balanced<12, 6, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<14, 6, true, true>(in, out, g, 0, tmp));
  } else if (focus && std::string(focus) == "pipe") {  // two-stage wave pipeline vs the single-wave kernel
    vs.push_back(balanced<16, 3, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<10, 6, true, true>(in, out, g, 0, tmp));
    vs.push_back(pipe<8, 8, 3>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 3>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 6>(in, out, g, tmp));
    vs.push_back(pipe<12, 12, 3>(in, out, g, tmp));
    vs.push_back(pipe<12, 12, 6>(in, out, g, tmp));
    vs.push_back(pipe<16, 16, 3>(in, out, g, tmp));
  } else if (focus && std::string(focus) == "pipe2") {  // pipeline splits, depth, priority; wrap and ghost-ring forms
    vs.push_back(balanced<16, 3, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<16, 3, false, true>(in, out, g, 0));
    vs.push_back(pipe<12, 12, 6>(in, out, g, tmp));
    vs.push_back(pipe<11, 13, 6>(in, out, g, tmp));
    vs.push_back(pipe<13, 11, 6>(in, out, g, tmp));
    vs.push_back(pipe<10, 14, 6>(in, out, g, tmp));
    vs.push_back(pipe<13, 13, 6>(in, out, g, tmp));
    vs.push_back(pipe<14, 14, 6>(in, out, g, tmp));
    vs.push_back(pipe<12, 12, 6, true, 1>(in, out, g, tmp));
    vs.push_back(pipe<12, 12, 6, true, 2>(in, out, g, tmp));
    vs.push_back(pipe<12, 12, 6, false>(in, out, g));
    vs.push_back(pipe<14, 14, 6, false>(in, out, g));
    vs.push_back(pipe<10, 10, 6>(in, out, g, tmp));
    vs.push_back(pipe<9, 11, 6>(in, out, g, tmp));
  } else if (focus && std::string(focus) == "pipe20") {  // S = 20 forms
    vs.push_back(balanced<16, 3, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<16, 3, false, true>(in, out, g, 0));
    vs.push_back(pipe<10, 10, 6>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 6, true, 1>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 6, true, 2>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 3>(in, out, g, tmp));
    vs.push_back(pipe<11, 9, 6>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 6, false>(in, out, g));
    vs.push_back(pipe<10, 10, 6, false, 1>(in, out, g));
    vs.push_back(pipe<10, 10, 6, false, 2>(in, out, g));
    vs.push_back(pipe<9, 9, 6>(in, out, g, tmp));
    vs.push_back(pipe<11, 11, 6>(in, out, g, tmp));
  } else if (focus && std::string(focus) == "sum") {  // sum form (c_center == c_neighbor) vs the general body
    vs.push_back(pipe<11, 9, 6>(in, out, g, tmp));
    vs.push_back(pipe<11, 9, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<12, 12, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<13, 11, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<14, 14, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<11, 9, 6, false>(in, out, g));
    vs.push_back(pipe<11, 9, 6, false, 0, true>(in, out, g));
    vs.push_back(balanced<16, 3, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<16, 3, true, true, true>(in, out, g, 0, tmp));
  } else if (focus && std::string(focus) == "sum2") {  // sum-form splits, fetch depth, priority
    vs.push_back(pipe<10, 10, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 9, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 3, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<9, 11, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 6, true, 1, true>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 6, true, 2, true>(in, out, g, tmp));
    vs.push_back(pipe<12, 12, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<12, 12, 9, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<11, 13, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 6, false, 0, true>(in, out, g));
    vs.push_back(pipe<10, 10, 9, false, 0, true>(in, out, g));
    vs.push_back(pipe<12, 12, 6, false, 0, true>(in, out, g));
  } else if (focus && std::string(focus) == "group") {  // strips per workgroup (barrier scope)
    vs.push_back(pipe<10, 10, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 6, true, 0, true, 2>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 6, true, 0, true, 1>(in, out, g, tmp));
    vs.push_back(pipe<12, 12, 6, true, 0, true, 2>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 6, false, 0, true>(in, out, g));
    vs.push_back(pipe<10, 10, 6, false, 0, true, 2>(in, out, g));
    vs.push_back(pipe<10, 10, 6, false, 0, true, 1>(in, out, g));
    vs.push_back(pipe<12, 12, 6, false, 0, true, 2>(in, out, g));
  } else if (focus && std::string(focus) == "pipe3") {  // three-stage pipeline (3 waves / SIMD)
    vs.push_back(pipe<10, 10, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe3<7, 7, 6, 6>(in, out, g, tmp));
    vs.push_back(pipe3<6, 7, 7, 6>(in, out, g, tmp));
    vs.push_back(pipe3<7, 6, 7, 6>(in, out, g, tmp));
    vs.push_back(pipe3<8, 8, 8, 6>(in, out, g, tmp));
    vs.push_back(pipe3<7, 7, 6, 3>(in, out, g, tmp));
    vs.push_back(pipe<12, 12, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe3<7, 7, 6, 6, false>(in, out, g));
  } else if (focus && std::string(focus) == "joint") {  // joint stage-1 windows vs per-strip aprons
    // Every joint variant is checked BITWISE against the per-strip pipeline of
    // the same S (the split does not change the arithmetic).
    auto joint_vs = [&](Variant j, const Variant& plain) {
      j.ref = plain.launch;
      j.tol = 0.f;
      return j;
    };
    const Variant p20 = pipe<10, 10, 6, true, 0, true>(in, out, g, tmp);
    const Variant p24 = pipe<12, 12, 6, true, 0, true>(in, out, g, tmp);
    const Variant p28 = pipe<14, 14, 6, true, 0, true>(in, out, g, tmp);
    const Variant n20 = pipe<10, 10, 6, false, 0, true>(in, out, g);
    const Variant n24 = pipe<12, 12, 6, false, 0, true>(in, out, g);
    vs.push_back(p20);
    vs.push_back(p24);
    vs.push_back(joint_vs(pipe<10, 10, 6, true, 0, true, 4, false, true>(in, out, g), p20));
    vs.push_back(joint_vs(pipe<8, 12, 6, true, 0, true, 4, false, true>(in, out, g), p20));
    vs.push_back(joint_vs(pipe<12, 8, 6, true, 0, true, 4, false, true>(in, out, g), p20));
    vs.push_back(joint_vs(pipe<12, 12, 6, true, 0, true, 4, false, true>(in, out, g), p24));
    vs.push_back(joint_vs(pipe<8, 16, 6, true, 0, true, 4, false, true>(in, out, g), p24));
    vs.push_back(p28);
    vs.push_back(joint_vs(pipe<16, 16, 3, true, 0, true, 4, false, true>(in, out, g),
                          pipe<16, 16, 3, true, 0, true>(in, out, g, tmp)));
    vs.push_back(joint_vs(pipe<12, 16, 6, true, 0, true, 4, false, true>(in, out, g), p28));
    vs.push_back(joint_vs(pipe<12, 12, 6, true, 0, false, 4, false, true>(in, out, g),
                          pipe<12, 12, 6, true, 0, false>(in, out, g, tmp)));
    vs.push_back(n20);
    vs.push_back(joint_vs(pipe<8, 12, 6, false, 0, true, 4, false, true>(in, out, g), n20));
    vs.push_back(joint_vs(pipe<12, 12, 6, false, 0, true, 4, false, true>(in, out, g), n24));
  } else if (focus && std::string(focus) == "perm") {  // lane-crossing sums via ds_bpermute (LDS pipe) vs DPP
    // The production joint forms (32768^2: 12 + 8 top-down; 8192^2: 8 + 12
    // bottom-up; S = 24), each bpermute variant checked BITWISE against its DPP twin.
    auto twin = [&](Variant j, const Variant& plain) {
      j.ref = plain.launch;
      j.tol = 0.f;
      return j;
    };
    const Variant a = pipe<12, 8, 6, true, 0, true, 4, false, true>(in, out, g, tmp);
    const Variant b = pipe<8, 12, 6, true, 0, true, 4, false, true, 3>(in, out, g, tmp);
    const Variant c = pipe<12, 12, 6, true, 0, true, 4, false, true>(in, out, g, tmp);
    vs.push_back(a);
    vs.push_back(twin(pipe<12, 8, 6, true, 0, true, 4, false, true, 0, 1>(in, out, g), a));
    vs.push_back(b);
    vs.push_back(twin(pipe<8, 12, 6, true, 0, true, 4, false, true, 3, 1>(in, out, g), b));
    vs.push_back(c);
    vs.push_back(twin(pipe<12, 12, 6, true, 0, true, 4, false, true, 0, 1>(in, out, g), c));
  } else if (focus && std::string(focus) == "joint2") {  // joint windows: fetch depth, XCD-major order, priority
    vs.push_back(pipe<12, 8, 6, true, 0, true, 4, false, true>(in, out, g));
    vs.push_back(pipe<12, 8, 3, true, 0, true, 4, false, true>(in, out, g));
    vs.push_back(pipe<12, 8, 9, true, 0, true, 4, false, true>(in, out, g));
    vs.push_back(pipe<12, 8, 6, true, 0, true, 4, true, true>(in, out, g));
    vs.push_back(pipe<12, 8, 6, true, 1, true, 4, false, true>(in, out, g));
    vs.push_back(pipe<12, 8, 6, true, 2, true, 4, false, true>(in, out, g));
    vs.push_back(pipe<8, 12, 6, true, 0, true, 4, false, true>(in, out, g));
    vs.push_back(pipe<8, 12, 9, true, 0, true, 4, false, true>(in, out, g));
    vs.push_back(pipe<8, 12, 6, true, 0, true, 4, true, true>(in, out, g));
  } else if (focus && std::string(focus) == "lag1") {  // ascending level order (1-row lag per level) vs descending
    // Same arithmetic per cell: every LAG1 variant is checked BITWISE against the
    // default-order kernel of the same shape.
    auto vs_plain = [&](Variant v, const Variant& plain) {
      v.ref = plain.launch;
      v.tol = 0.f;
      return v;
    };
    const Variant a = pipe<12, 8, 6, true, 0, true, 4, false, true>(in, out, g);
    const Variant b = pipe<8, 12, 6, true, 0, true, 4, false, true>(in, out, g);
    const Variant c = pipe<12, 12, 6, true, 0, true, 4, false, true>(in, out, g);
    const Variant n = pipe<8, 12, 6, false, 0, true, 4, false, true>(in, out, g);
    vs.push_back(a);
    vs.push_back(vs_plain(pipe<12, 8, 6, true, 0, true, 4, false, true, 3>(in, out, g), a));
    vs.push_back(b);
    vs.push_back(vs_plain(pipe<8, 12, 6, true, 0, true, 4, false, true, 3>(in, out, g), b));
    vs.push_back(c);
    vs.push_back(vs_plain(pipe<12, 12, 6, true, 0, true, 4, false, true, 3>(in, out, g), c));
    vs.push_back(n);
    vs.push_back(vs_plain(pipe<8, 12, 6, false, 0, true, 4, false, true, 3>(in, out, g), n));
    vs.push_back(vs_plain(pipe<8, 12, 6, true, 0, false, 4, false, true, 3>(in, out, g),
                          pipe<8, 12, 6, true, 0, false, 4, false, true>(in, out, g)));
  } else if (focus && std::string(focus) == "lag2") {  // per-stage level order (LAG1 mask), bitwise vs descending
    auto vs_plain = [&](Variant v, const Variant& plain) {
      v.ref = plain.launch;
      v.tol = 0.f;
      return v;
    };
    const Variant a = pipe<12, 8, 6, true, 0, true, 4, false, true>(in, out, g);
    const Variant b = pipe<8, 12, 6, true, 0, true, 4, false, true>(in, out, g);
    const Variant c = pipe<12, 12, 6, true, 0, true, 4, false, true>(in, out, g);
    vs.push_back(a);
    vs.push_back(vs_plain(pipe<12, 8, 6, true, 0, true, 4, false, true, 1>(in, out, g), a));
    vs.push_back(vs_plain(pipe<12, 8, 6, true, 0, true, 4, false, true, 2>(in, out, g), a));
    vs.push_back(vs_plain(pipe<12, 8, 6, true, 0, true, 4, false, true, 3>(in, out, g), a));
    vs.push_back(b);
    vs.push_back(vs_plain(pipe<8, 12, 6, true, 0, true, 4, false, true, 2>(in, out, g), b));
    vs.push_back(vs_plain(pipe<8, 12, 6, true, 0, true, 4, false, true, 3>(in, out, g), b));
    vs.push_back(c);
    vs.push_back(vs_plain(pipe<12, 12, 6, true, 0, true, 4, false, true, 2>(in, out, g), c));
    vs.push_back(vs_plain(pipe<12, 12, 6, true, 0, true, 4, false, true, 3>(in, out, g), c));
  } else if (focus && std::string(focus) == "head20") {  // the headline pass: S = 20 12 + 8 descending vs ascending (r06)
    const Variant a = pipe<12, 8, 6, true, 0, true, 4, false, true>(in, out, g);
    Variant b = pipe<12, 8, 6, true, 0, true, 4, false, true, 3>(in, out, g);
    b.ref = a.launch;  // same arithmetic per cell: bitwise
    b.tol = 0.f;
    vs.push_back(a);
    vs.push_back(b);
    // Balanced stage splits (wrap only: their joint read reach A0 + A1 = 24 exceeds
    // SA(20), so a ghost-ring tile would need a 24-deep ring).
    for (auto v : {pipe<10, 10, 6, true, 0, true, 4, false, true, 3>(in, out, g),
                   pipe<11, 9, 6, true, 0, true, 4, false, true, 3>(in, out, g)}) {
      v.ref = a.launch;
      v.tol = 0.f;
      vs.push_back(v);
    }
  } else if (focus && std::string(focus) == "bands") {  // row-band shares (memory-side cache reuse), r06
    const Variant a = pipe<12, 8, 6, true, 0, true, 4, false, true, 3>(in, out, g);
    vs.push_back(a);
    for (int pg : {7}) {
      Variant b = pipe_bands<12, 8, 6, 3>(in, out, g, pg);
      b.ref = a.launch;
      b.tol = 0.f;
      vs.push_back(b);
    }
  } else if (focus && std::string(focus) == "ntload") {  // the headline pass with non-temporal input loads (r06)
    const Variant a = pipe<12, 8, 6, true, 0, true, 4, false, true, 3>(in, out, g);
    Variant b = pipe<12, 8, 6, true, 0, true, 4, false, true, 3, 7>(in, out, g);
    b.ref = a.launch;
    b.tol = 0.f;
    vs.push_back(a);
    vs.push_back(b);
  } else if (focus && std::string(focus) == "lag2head") {  // long-chunk tiles: the S = 20 / 24 candidates
    const Variant a = pipe<12, 8, 6, true, 0, true, 4, false, true>(in, out, g);
    Variant b = pipe<8, 12, 6, true, 0, true, 4, false, true, 2>(in, out, g);
    b.ref = a.launch;  // same arithmetic per cell whatever the split and order: bitwise
    b.tol = 0.f;
    Variant c = pipe<12, 12, 6, true, 0, true, 4, false, true, 2>(in, out, g);
    vs.push_back(a);
    vs.push_back(b);
    vs.push_back(pipe<8, 12, 6, true, 0, true, 4, false, true>(in, out, g));
    vs.push_back(c);
    vs.push_back(pipe<12, 12, 6, true, 0, true, 4, false, true, 3>(in, out, g));
  } else if (focus && std::string(focus) == "jointpmc") {  // counters: the S = 20 default, per-strip vs joint
    vs.push_back(pipe<10, 10, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<12, 8, 6, true, 0, true, 4, false, true>(in, out, g));
  } else if (focus && std::string(focus) == "s24") {  // S = 20 vs 24 (sum form) on large tiles
    vs.push_back(pipe<10, 10, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<12, 12, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<11, 13, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 6, false, 0, true>(in, out, g));
    vs.push_back(pipe<12, 12, 6, false, 0, true>(in, out, g));
    vs.push_back(pipe<11, 13, 6, false, 0, true>(in, out, g));
  } else if (focus && std::string(focus) == "xcd") {  // XCD-major share order
    vs.push_back(pipe<10, 10, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 6, true, 0, true, 4, true>(in, out, g, tmp));
    vs.push_back(pipe<12, 12, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<12, 12, 6, true, 0, true, 4, true>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 6, false, 0, true>(in, out, g));
    vs.push_back(pipe<10, 10, 6, false, 0, true, 4, true>(in, out, g));
  } else if (focus && std::string(focus) == "sum3") {  // shallower sum-form pipelines (narrower apron)
    vs.push_back(pipe<10, 10, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<8, 8, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<8, 8, 9, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<9, 9, 6, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<9, 9, 9, true, 0, true>(in, out, g, tmp));
    vs.push_back(pipe<10, 10, 6, false, 0, true>(in, out, g));
    vs.push_back(pipe<8, 8, 6, false, 0, true>(in, out, g));
    vs.push_back(pipe<9, 9, 6, false, 0, true>(in, out, g));
  } else if (focus && std::string(focus) == "deep") {  // time blocks past 16 (AGPR-backed window, 1 wave/SIMD)
    vs.push_back(balanced<16, 3, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<10, 6, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<18, 3, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<20, 3, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<20, 6, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<24, 3, true, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<20, 3, true, true>(in, out, g, 2, tmp));
  } else if (focus && std::string(focus) == "s") {  // S choice for the balanced launch
    vs.push_back(balanced<12, 3>(in, out, g, 0));
    vs.push_back(balanced<12, 3, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<16, 3>(in, out, g, 2));
    vs.push_back(balanced<16, 3, true>(in, out, g, 2, tmp));
    vs.push_back(balanced<14, 3, true>(in, out, g, 2, tmp));
    vs.push_back(balanced<10, 3, true>(in, out, g, 0, tmp));
  } else {
    for (int ch : {128, 256, 512}) {
      vs.push_back(stream<12, 3>(in, out, g, ch));
      vs.push_back(stream<12, 3, true>(in, out, g, ch, tmp));
    }
    for (int per_cu : {0, 1, 3}) {
      vs.push_back(balanced<12, 3>(in, out, g, per_cu));
      vs.push_back(balanced<12, 3, true>(in, out, g, per_cu, tmp));
    }
    vs.push_back(balanced<8, 3, true>(in, out, g, 0));
    vs.push_back(balanced<16, 3, true>(in, out, g, 0, tmp));
    vs.push_back(balanced<16, 3, true>(in, out, g, 2, tmp));
  }

  Stream st;
  Event e0(true), e1(true);
  // Warm-up / first-touch; drop variants whose launch is rejected (e.g. LDS over the limit).
  std::vector<Variant> ok;
  for (auto& v : vs) {
    (void)hipGetLastError();
    v.launch(st.get());
    const hipError_t e = hipGetLastError();
    st.sync();
    if (e != hipSuccess) {
      std::printf("{\"variant\": \"%s\", \"error\": \"%s\"}\n", v.name.c_str(), hipGetErrorString(e));
      continue;
    }
    if (v.ref) {
      // Bitwise check against the validated LDS kernel (same evaluation order).
      std::vector<float> got(size_t(g.alloc_elems())), want(size_t(g.alloc_elems()));
      MXS_HIP_CHECK(hipMemcpy(got.data(), out, got.size() * 4, hipMemcpyDeviceToHost));
      v.ref(st.get());
      st.sync();
      MXS_HIP_CHECK(hipMemcpy(want.data(), out, want.size() * 4, hipMemcpyDeviceToHost));
      long long bad = 0;
      float maxdiff = 0.f;
      for (index_t y = 0; y < H; ++y)
        for (index_t x = 0; x < W; ++x) {
          const size_t i = size_t(g.core_offset() + y * g.pitch + x);
          const float d = std::fabs(got[i] - want[i]);
          maxdiff = std::max(maxdiff, d);
          bad += v.tol > 0.f ? !(d <= v.tol) : got[i] != want[i];
        }
      std::printf("{\"variant\": \"%s\", \"mismatches\": %lld, \"max_abs_diff\": %.3g}\n", v.name.c_str(), bad,
                  double(maxdiff));
      if (bad) continue;
    }
    ok.push_back(std::move(v));
  }
  vs = std::move(ok);
  for (int r = 0; r < rounds; ++r)
    for (auto& v : vs) {
      e0.record(st.get());
      for (int k = 0; k < 3; ++k) {
        if ((k & 1) && v.launch2) v.launch2(st.get());
        else v.launch(st.get());
      }
      e1.record(st.get());
      e1.sync();
      v.ms.push_back(e1.since(e0) / 3);
    }
  const double bytes = 2.0 * double(W) * double(H) * 4.0;
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2], best = v.ms[0];
    const double cbytes = v.name == "copy_float4" ? 2.0 * double(g.alloc_elems()) * 4.0 : bytes;
    std::printf("{\"variant\": \"%s\", \"median_ms\": %.4f, \"best_ms\": %.4f, \"tb_s\": %.3f, \"gcells_s\": %.1f}\n",
                v.name.c_str(), med, best, cbytes / (med * 1e-3) / 1e12,
                double(W) * double(H) * v.steps / (med * 1e-3) / 1e9);
  }
  return 0;
}
