// Microbenchmark (not product code), after ring_copy.hip (4 KiB pieces per wave copy 5-10 %
// faster than 8-9 KiB pieces): is it the bytes per wave or the address span of the pieces in
// flight? Register copies, one wave per workgroup: (a) one 4 KiB piece per wave, (b) one 8 KiB
// piece, (c) two 4 KiB pieces per wave half the buffer apart (each wave 8 KiB, the pieces in
// flight at any time as close together as in (a)), (d) two 4 KiB pieces per wave, adjacent.
// Build + run:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/rc5 scripts/microbench/ring_copy5.hip && /tmp/rc5
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void copy4k(const u32x4* __restrict__ s, u32x4* __restrict__ d,
                                       int lane) {
  u32x4 v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) v[u] = __builtin_nontemporal_load(s + u * 64 + lane);
#pragma unroll
  for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(v[u], d + u * 64 + lane);
}

// kMode 0: piece w (4 KiB); 1: 8 KiB piece w; 2: 4 KiB pieces w and w + n/2; 3: 4 KiB pieces
// 2w and 2w + 1 (one after the other)
template <int kMode>
__global__ __launch_bounds__(64) void copy_k(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                             uint32_t n4k) {
  const int lane = threadIdx.x;
  const uint32_t w = blockIdx.x;
  if constexpr (kMode == 0) {
    copy4k(src + uint64_t(w) * 256, dst + uint64_t(w) * 256, lane);
  } else if constexpr (kMode == 1) {
    copy4k(src + uint64_t(2 * w) * 256, dst + uint64_t(2 * w) * 256, lane);
    copy4k(src + uint64_t(2 * w + 1) * 256, dst + uint64_t(2 * w + 1) * 256, lane);
  } else if constexpr (kMode == 2) {
    copy4k(src + uint64_t(w) * 256, dst + uint64_t(w) * 256, lane);
    copy4k(src + uint64_t(w + n4k / 2) * 256, dst + uint64_t(w + n4k / 2) * 256, lane);
  } else {
    u32x4 v[8];
    const u32x4* s = src + uint64_t(2 * w) * 256;
    u32x4* d = dst + uint64_t(2 * w) * 256;
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(s + u * 64 + lane);
#pragma unroll
    for (int u = 0; u < 8; ++u) __builtin_nontemporal_store(v[u], d + u * 64 + lane);
  }
}

int main() {
  const uint64_t bytes = 4ull << 30;
  const uint32_t n4k = uint32_t(bytes / 4096);
  u32x4 *src, *dst;
  CHECK(hipMalloc(&src, bytes));
  CHECK(hipMalloc(&dst, bytes));
  std::vector<uint8_t> h(1 << 20);
  for (size_t i = 0; i < h.size(); ++i) h[i] = uint8_t((i * 131 + 7) ^ (i >> 9));
  for (uint64_t o = 0; o < bytes; o += h.size())
    CHECK(hipMemcpy(reinterpret_cast<uint8_t*>(src) + o, h.data(), h.size(), hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const char* names[] = {"one_4k", "one_8k_contiguous_loop", "two_4k_half_apart", "one_8k_all_in_flight"};
  for (int rnd = 0; rnd < 3; ++rnd) {
    for (int m = 0; m < 4; ++m) {
      const unsigned grid = m == 0 ? n4k : n4k / 2;
      auto launch = [&]() {
        if (m == 0) hipLaunchKernelGGL(copy_k<0>, dim3(grid), dim3(64), 0, 0, src, dst, n4k);
        else if (m == 1) hipLaunchKernelGGL(copy_k<1>, dim3(grid), dim3(64), 0, 0, src, dst, n4k);
        else if (m == 2) hipLaunchKernelGGL(copy_k<2>, dim3(grid), dim3(64), 0, 0, src, dst, n4k);
        else hipLaunchKernelGGL(copy_k<3>, dim3(grid), dim3(64), 0, 0, src, dst, n4k);
      };
      launch();
      CHECK(hipEventRecord(a));
      const int iters = 8;
      for (int i = 0; i < iters; ++i) launch();
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      CHECK(hipGetLastError());
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      std::vector<uint8_t> got(1 << 20), want(1 << 20);
      bool ok = true;
      for (uint64_t o : {uint64_t(0), bytes / 2 + 8192, bytes - (1 << 20)}) {
        CHECK(hipMemcpy(got.data(), reinterpret_cast<uint8_t*>(dst) + o, got.size(), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(want.data(), reinterpret_cast<uint8_t*>(src) + o, want.size(), hipMemcpyDeviceToHost));
        ok = ok && std::memcmp(got.data(), want.data(), got.size()) == 0;
      }
      CHECK(hipMemset(dst, 0, bytes));
      std::printf("{\"round\": %d, \"variant\": \"%s\", \"GBps\": %.1f, \"ok\": %s}\n", rnd, names[m],
                  2.0 * bytes / (ms / iters) / 1e6, ok ? "true" : "false");
      std::fflush(stdout);
    }
  }
  return 0;
}
