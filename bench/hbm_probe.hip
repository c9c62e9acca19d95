// HBM roofline probe: read+write copy, read-only and write-only streams with
// different unroll depths / cache policies, to calibrate the achievable
// bandwidth the stencil kernels are measured against (docs/PERF.md).
//   hbm_probe [GiB per buffer]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "mxs/core/error.hpp"
#include "mxs/runtime/hip_utils.hpp"

using namespace mxs;
typedef float v4f __attribute__((ext_vector_type(4)));

template <int U, bool NTS, bool NTL>
__global__ __launch_bounds__(256) void copy_u(const v4f* __restrict__ a, v4f* __restrict__ b, index_t n) {
  // Each block handles a contiguous chunk of U * 256 v4f per iteration.
  const index_t stride = index_t(gridDim.x) * 256 * U;
  for (index_t base = index_t(blockIdx.x) * 256 * U + threadIdx.x; base < n; base += stride) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const index_t i = base + u * 256;
      if (i < n) v[u] = NTL ? __builtin_nontemporal_load(a + i) : a[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const index_t i = base + u * 256;
      if (i < n) {
        if (NTS) __builtin_nontemporal_store(v[u], b + i);
        else b[i] = v[u];
      }
    }
  }
}

template <int U>
__global__ __launch_bounds__(256) void read_u(const v4f* __restrict__ a, float* __restrict__ out, index_t n) {
  const index_t stride = index_t(gridDim.x) * 256 * U;
  float acc = 0.f;
  for (index_t base = index_t(blockIdx.x) * 256 * U + threadIdx.x; base < n; base += stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const index_t i = base + u * 256;
      if (i < n) {
        const v4f v = a[i];
        acc += v.x + v.y + v.z + v.w;
      }
    }
  }
  if (acc == 12345.678f) out[0] = acc;  // keep the loads alive
}

// The dot kernel's pattern (kernels/dot.hip): one workgroup per CU, every lane
// issues U non-temporal 16-byte loads before any use (U x 1 KiB per wave
// instruction group in flight), grid-stride over whole chunks. dot.hip reads at
// 7.1 TB/s this way (profiles/r02_dot); the plain-load read_u above at 8-32
// workgroups per CU topped out at 6.3-6.4 TB/s.
template <int U>
__global__ __launch_bounds__(256) void read_nt(const v4f* __restrict__ a, float* __restrict__ out, index_t n) {
  const index_t stride = index_t(gridDim.x) * 256 * U;
  v4f acc = {0.f, 0.f, 0.f, 0.f};
  index_t base = index_t(blockIdx.x) * 256 * U + threadIdx.x;
  for (; base + (U - 1) * 256 < n; base += stride) {
    v4f v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(a + base + u * 256);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  for (; base < n; base += 256) acc += a[base];
  if (acc.x + acc.y + acc.z + acc.w == 12345.678f) out[0] = acc.x;  // keep the loads alive
}

template <bool NTS>
__global__ __launch_bounds__(256) void write_only(v4f* __restrict__ b, index_t n) {
  const index_t stride = index_t(gridDim.x) * 256;
  const v4f v = {1.f, 2.f, 3.f, 4.f};
  for (index_t i = index_t(blockIdx.x) * 256 + threadIdx.x; i < n; i += stride) {
    if (NTS) __builtin_nontemporal_store(v, b + i);
    else b[i] = v;
  }
}

int main(int argc, char** argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 4.0;
  const index_t n = index_t(gib * (1 << 30)) / 16;
  DeviceBuffer<v4f> a(n), b(n);
  DeviceBuffer<float> sink(1);
  MXS_HIP_CHECK(hipMemset(a.get(), 0, a.bytes()));
  MXS_HIP_CHECK(hipMemset(b.get(), 0, b.bytes()));
  v4f* pa = a.get();
  v4f* pb = b.get();
  float* ps = sink.get();
  const size_t abytes = a.bytes();
  struct V { std::string name; double bytes; std::function<void(hipStream_t)> f; std::vector<float> ms; };
  std::vector<V> vs;
  const double cb = 2.0 * n * 16, rb = 1.0 * n * 16;
  auto add_copy = [&](const char* nm, int grid, auto kern) {
    vs.push_back({std::string(nm) + "_g" + std::to_string(grid), cb, [=](hipStream_t s) { kern<<<grid, 256, 0, s>>>(pa, pb, n); }});
  };
  for (int grid : {2048, 4096, 16384}) {
    add_copy("copy_u1", grid, copy_u<1, false, false>);
    add_copy("copy_u4", grid, copy_u<4, false, false>);
    add_copy("copy_u4_nts", grid, copy_u<4, true, false>);
    add_copy("copy_u8_nts", grid, copy_u<8, true, false>);
    add_copy("copy_u4_nts_ntl", grid, copy_u<4, true, true>);
  }
  for (int grid : {2048, 8192}) {
    vs.push_back({"read_u4_g" + std::to_string(grid), rb, [=](hipStream_t s) { read_u<4><<<grid, 256, 0, s>>>(pa, ps, n); }});
    vs.push_back({"read_u8_g" + std::to_string(grid), rb, [=](hipStream_t s) { read_u<8><<<grid, 256, 0, s>>>(pa, ps, n); }});
    vs.push_back({"write_g" + std::to_string(grid), rb, [=](hipStream_t s) { write_only<false><<<grid, 256, 0, s>>>(pb, n); }});
    vs.push_back({"write_nts_g" + std::to_string(grid), rb, [=](hipStream_t s) { write_only<true><<<grid, 256, 0, s>>>(pb, n); }});
  }
  const int cus = device_cu_count();
  for (int per_cu : {1, 2, 4}) {
    const int grid = per_cu * cus;
    vs.push_back({"read_nt_u8_g" + std::to_string(grid), rb, [=](hipStream_t s) { read_nt<8><<<grid, 256, 0, s>>>(pa, ps, n); }});
    vs.push_back({"read_nt_u16_g" + std::to_string(grid), rb, [=](hipStream_t s) { read_nt<16><<<grid, 256, 0, s>>>(pa, ps, n); }});
    add_copy("copy_u8_nts_ntl", grid, copy_u<8, true, true>);
    add_copy("copy_u8_nts", grid, copy_u<8, true, false>);
  }
  vs.push_back({"hipMemcpyDtoD", cb, [=](hipStream_t s) { MXS_HIP_CHECK(hipMemcpyAsync(pb, pa, abytes, hipMemcpyDeviceToDevice, s)); }});
  Stream st;
  Event e0(true), e1(true);
  for (auto& v : vs) v.f(st.get());
  st.sync();
  for (int r = 0; r < 5; ++r)
    for (auto& v : vs) {
      e0.record(st.get());
      for (int k = 0; k < 3; ++k) v.f(st.get());
      e1.record(st.get());
      e1.sync();
      v.ms.push_back(e1.since(e0) / 3);
    }
  for (auto& v : vs) {
    std::sort(v.ms.begin(), v.ms.end());
    const double med = v.ms[v.ms.size() / 2];
    std::printf("{\"probe\": \"%s\", \"median_ms\": %.4f, \"tb_s\": %.3f}\n", v.name.c_str(), med, v.bytes / (med * 1e-3) / 1e12);
  }
  return 0;
}
