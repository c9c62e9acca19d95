// Standard-library allocator over page-locked host memory (reference:
// host_allocator.h:58-93, `std::vector<double, host_allocator<double>>` under
// -DPAGE_LOCKED in test-benchmark/mpi-pingpong-gpu-async.cpp:43-49).
//
// hipHostMalloc memory is pinned and mapped for DMA, so hipMemcpyAsync from/to it
// runs at PCIe rate without the driver's staging bounce. Differences from the
// reference: no non-inline specialisations in a header (ODR hazard);
// C++17 allocator requirements (rebind constructor, equality); optional
// hipHostMalloc flags (e.g. hipHostMallocNumaUser, hipHostMallocPortable).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstddef>
#include <limits>
#include <new>

namespace mxs {

template <typename T>
class PinnedAllocator {
 public:
  using value_type = T;
  using size_type = std::size_t;
  using difference_type = std::ptrdiff_t;
  template <typename U>
  struct rebind {
    using other = PinnedAllocator<U>;
  };

  PinnedAllocator() noexcept = default;
  explicit PinnedAllocator(unsigned flags) noexcept : flags_(flags) {}
  template <typename U>
  PinnedAllocator(const PinnedAllocator<U>& o) noexcept : flags_(o.flags()) {}

  T* allocate(size_type n) {
    if (n > max_size()) throw std::bad_array_new_length();
    void* p = nullptr;
    if (hipHostMalloc(&p, n * sizeof(T), flags_) != hipSuccess || p == nullptr) throw std::bad_alloc();
    return static_cast<T*>(p);
  }
  void deallocate(T* p, size_type) noexcept { (void)hipHostFree(p); }
  size_type max_size() const noexcept { return std::numeric_limits<size_type>::max() / sizeof(T); }
  unsigned flags() const noexcept { return flags_; }

 private:
  unsigned flags_ = hipHostMallocDefault;
};

template <typename T, typename U>
bool operator==(const PinnedAllocator<T>& a, const PinnedAllocator<U>& b) noexcept {
  return a.flags() == b.flags();
}
template <typename T, typename U>
bool operator!=(const PinnedAllocator<T>& a, const PinnedAllocator<U>& b) noexcept {
  return !(a == b);
}

}  // namespace mxs
