// Microbenchmark (not product code), after ring_copy.hip (where a 16-slot ring copying 4 KiB
// pieces beat every other shape): is it the ring or the occupancy? The register copy and the
// 4-slot ring copy of 4 KiB pieces per wave, two waves per workgroup, with the workgroups per CU
// set by padding each workgroup's dynamic LDS (160 KiB / k).
// Build + run:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/rc3 scripts/microbench/ring_copy3.hip && /tmp/rc3
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
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

__device__ __forceinline__ void glds16(const void* g, uint32_t lds) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(lds);
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(g), "s"(l)
      : "memory");
}

__device__ __forceinline__ void wait_vm(uint32_t n) {  // vmcnt(m), m <= n from a coarse ladder
  if (n >= 16) {
    if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// Ring copy: S slots of 1 KiB per wave; the wave waits for kGroup slots, copies them, refills.
template <int S, int kGroup>
__global__ __launch_bounds__(128) void ring_copy(const u32x4* __restrict__ src,
                                                 u32x4* __restrict__ dst, uint32_t piece_kib,
                                                 uint32_t npieces) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t piece = blockIdx.x * 2 + uint32_t(wave);
  if (piece >= npieces) return;
  uint8_t* ring = smem + wave * S * 1024;
  const uint32_t ring_lds = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) uint8_t*)ring)));
  const u32x4* s = src + uint64_t(piece) * piece_kib * 64;
  u32x4* d = dst + uint64_t(piece) * piece_kib * 64;
  const uint32_t n = piece_kib;
  uint32_t issued = 0, ops = 0, op_at = 0;
  auto pump = [&](uint32_t low) {
    while (issued < n && issued < low + S) {
      glds16(s + issued * 64 + lane, ring_lds + (issued % S) * 1024u);
      if (lane == int(issued % S)) op_at = ops;
      ++ops;
      ++issued;
    }
  };
  pump(0);
  for (uint32_t g = 0; g < n; g += kGroup) {
    const uint32_t last = min(g + kGroup, n) - 1;
    const uint32_t at = uint32_t(__builtin_amdgcn_readlane(int(op_at), int(last % S)));
    wait_vm(ops - at - 1);
    for (uint32_t i = g; i <= last; ++i) {
      const u32x4 v = *(const __attribute__((address_space(3))) u32x4*)(
          (const __attribute__((address_space(3))) uint8_t*)ring + (i % S) * 1024 + 16 * lane);
      __builtin_nontemporal_store(v, d + i * 64 + lane);
      ++ops;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slots' reads done before refill
    pump(last + 1);
  }
}

// Register copy of the same pieces: 4 x 16 B per lane in flight, then stored.
__global__ __launch_bounds__(128) void reg_copy(const u32x4* __restrict__ src,
                                                u32x4* __restrict__ dst, uint32_t piece_kib,
                                                uint32_t npieces) {
  const int lane = threadIdx.x & 63;
  const uint32_t piece = blockIdx.x * 2 + (threadIdx.x >> 6);
  if (piece >= npieces) return;
  const u32x4* s = src + uint64_t(piece) * piece_kib * 64;
  u32x4* d = dst + uint64_t(piece) * piece_kib * 64;
  for (uint32_t g = 0; g < piece_kib; g += 4) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (g + u < piece_kib) v[u] = __builtin_nontemporal_load(s + (g + u) * 64 + lane);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (g + u < piece_kib) __builtin_nontemporal_store(v[u], d + (g + u) * 64 + lane);
  }
}

int main() {
  const uint64_t bytes = 4ull << 30;
  u32x4 *src, *dst;
  CHECK(hipMalloc(&src, bytes));
  CHECK(hipMalloc(&dst, bytes));
  std::vector<uint8_t> h(1 << 20);
  for (size_t i = 0; i < h.size(); ++i) h[i] = uint8_t((i * 131 + 7) ^ (i >> 9));
  for (uint64_t o = 0; o < bytes; o += h.size())
    CHECK(hipMemcpy(reinterpret_cast<uint8_t*>(src) + o, h.data(), h.size(), hipMemcpyHostToDevice));
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(reg_copy),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(ring_copy<4, 1>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int ks[] = {2, 3, 4, 5, 6, 8, 10, 12, 16};
  const uint32_t pk = 4;
  const uint32_t np = uint32_t(bytes / (pk * 1024ull));
  const unsigned grid = (np + 1) / 2;
  for (int rnd = 0; rnd < 2; ++rnd) {
    for (int kind = 0; kind < 2; ++kind) {
      for (int k : ks) {
        const size_t lds = std::max<size_t>((160 * 1024) / k - 512, 2 * 4 * 1024) & ~size_t(1023);
        auto launch = [&]() {
          if (kind == 0)
            hipLaunchKernelGGL(reg_copy, dim3(grid), dim3(128), lds, 0, src, dst, pk, np);
          else
            hipLaunchKernelGGL((ring_copy<4, 1>), dim3(grid), dim3(128), lds, 0, src, dst, pk, np);
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
        for (uint64_t o : {uint64_t(0), bytes - (1 << 20)}) {
          CHECK(hipMemcpy(got.data(), reinterpret_cast<uint8_t*>(dst) + o, got.size(), hipMemcpyDeviceToHost));
          CHECK(hipMemcpy(want.data(), reinterpret_cast<uint8_t*>(src) + o, want.size(), hipMemcpyDeviceToHost));
          ok = ok && std::memcmp(got.data(), want.data(), got.size()) == 0;
        }
        CHECK(hipMemset(dst, 0, bytes));
        std::printf("{\"round\": %d, \"variant\": \"%s\", \"wg_per_cu\": %d, \"lds\": %zu, \"GBps\": %.1f, \"ok\": %s}\n",
                    rnd, kind ? "ring4" : "reg", k, lds, 2.0 * bytes / (ms / iters) / 1e6, ok ? "true" : "false");
        std::fflush(stdout);
      }
    }
  }
  return 0;
}
