// Microbenchmark (not product code): do 16-byte global loads from addresses that are NOT 16-byte
// aligned work on MI355X, and at what rate against aligned ones? The copy reads src + off (off =
// 0..15) and writes dst (aligned), 4 KiB per wave (4 x 16 B per lane), non-temporal, the shape of
// the copy-ceiling probe. Build + run:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/uc scripts/microbench/unaligned_copy.hip && /tmp/uc
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

// kAsm: inline-asm global_load_dwordx4 at the exact (unaligned) address; else a 16-byte memcpy
// (what the compiler makes of it).
template <bool kAsm>
__global__ __launch_bounds__(256) void copy_off(const uint8_t* __restrict__ src,
                                                u32x4* __restrict__ dst, uint64_t nq) {
  const uint64_t wave = (uint64_t(blockIdx.x) * 256 + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const uint64_t q0 = wave * 256;  // 4 KiB per wave
  if (q0 >= nq) return;
  u32x4 v[4];
  if constexpr (kAsm) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint8_t* p = src + 16 * (q0 + 64 * u + lane);
      asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v[u]) : "v"(p) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u) __builtin_memcpy(&v[u], src + 16 * (q0 + 64 * u + lane), 16);
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) __builtin_nontemporal_store(v[u], dst + q0 + 64 * u + lane);
}

int main() {
  const uint64_t bytes = 4ull << 30;
  const uint64_t nq = bytes / 16;
  uint8_t* src;
  u32x4* dst;
  CHECK(hipMalloc(&src, bytes + 256));
  CHECK(hipMalloc(&dst, bytes));
  std::vector<uint8_t> h(1 << 20);
  for (size_t i = 0; i < h.size(); ++i) h[i] = uint8_t((i * 131 + 7) ^ (i >> 9));
  for (uint64_t o = 0; o < bytes + 256; o += h.size())
    CHECK(hipMemcpy(src + o, h.data(), std::min<uint64_t>(h.size(), bytes + 256 - o),
                    hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const unsigned grid = unsigned((nq / 256 + 3) / 4);  // 4 waves per block, one 4 KiB piece each
  const int offs[] = {0, 1, 4, 7, 8, 13, 15};
  for (int variant = 0; variant < 2; ++variant) {
    for (int off : offs) {
      auto launch = [&]() {
        if (variant == 0)
          hipLaunchKernelGGL(copy_off<true>, dim3(grid), dim3(256), 0, 0, src + off, dst, nq);
        else
          hipLaunchKernelGGL(copy_off<false>, dim3(grid), dim3(256), 0, 0, src + off, dst, nq);
      };
      for (int w = 0; w < 3; ++w) launch();
      CHECK(hipEventRecord(a));
      const int iters = 10;
      for (int i = 0; i < iters; ++i) launch();
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms = 0;
      CHECK(hipEventElapsedTime(&ms, a, b));
      // check the first and last MiB against the source shifted by off
      std::vector<uint8_t> got(1 << 20), want(1 << 20);
      bool ok = true;
      for (uint64_t o : {uint64_t(0), bytes - (1 << 20)}) {
        CHECK(hipMemcpy(got.data(), reinterpret_cast<uint8_t*>(dst) + o, got.size(),
                        hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(want.data(), src + o + off, want.size(), hipMemcpyDeviceToHost));
        ok = ok && std::memcmp(got.data(), want.data(), got.size()) == 0;
      }
      std::printf("{\"variant\": \"%s\", \"off\": %d, \"GBps\": %.1f, \"ok\": %s}\n",
                  variant == 0 ? "asm_dwordx4" : "memcpy16", off, 2.0 * bytes / (ms / iters) / 1e6,
                  ok ? "true" : "false");
    }
  }
  return 0;
}
