// HBM copy-ceiling microbenchmark (not product code): what a pure 16-byte-per-lane stream of
// N bytes read + N bytes written reaches on this MI355X, over kernel shapes. Build+run:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/cc scripts/microbench/copy_ceiling.hip && /tmp/cc
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_gs(const u32x4* __restrict__ s, u32x4* __restrict__ d,
                                               uint64_t n) {
  const uint64_t stride = uint64_t(gridDim.x) * 256;
  uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = NT ? __builtin_nontemporal_load(s + i + u * stride) : s[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], d + i + u * stride);
      else d[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) d[i] = s[i];
}

// each block copies a contiguous chunk (per-block contiguous), U x 1 KiB per wave per step
template <int U, bool NT>
__global__ __launch_bounds__(256) void copy_blk(const u32x4* __restrict__ s, u32x4* __restrict__ d,
                                                uint64_t n, uint64_t per_block) {
  const uint64_t b0 = uint64_t(blockIdx.x) * per_block;
  const uint64_t b1 = b0 + per_block < n ? b0 + per_block : n;
  for (uint64_t base = b0; base < b1; base += 256 * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + u * 256 + threadIdx.x;
      if (i < b1) v[u] = NT ? __builtin_nontemporal_load(s + i) : s[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + u * 256 + threadIdx.x;
      if (i < b1) {
        if (NT) __builtin_nontemporal_store(v[u], d + i);
        else d[i] = v[u];
      }
    }
  }
}

// read-only stream (xor-folded so the loads stay live) and write-only stream
template <int U>
__global__ __launch_bounds__(256) void read_blk(const u32x4* __restrict__ s, u32x4* __restrict__ sink,
                                                uint64_t n, uint64_t per_block) {
  const uint64_t b0 = uint64_t(blockIdx.x) * per_block;
  const uint64_t b1 = b0 + per_block < n ? b0 + per_block : n;
  u32x4 acc = {0, 0, 0, 0};
  for (uint64_t base = b0; base < b1; base += 256 * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + u * 256 + threadIdx.x;
      v[u] = i < b1 ? __builtin_nontemporal_load(s + i) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u];
  }
  if (acc.x == 0x9e3779b9u && acc.y == 0x7f4a7c15u) sink[threadIdx.x] = acc;
}

template <int U>
__global__ __launch_bounds__(256) void write_blk(u32x4* __restrict__ d, uint64_t n,
                                                 uint64_t per_block) {
  const uint64_t b0 = uint64_t(blockIdx.x) * per_block;
  const uint64_t b1 = b0 + per_block < n ? b0 + per_block : n;
  const u32x4 v = {1u, 2u, 3u, unsigned(blockIdx.x)};
  for (uint64_t base = b0; base < b1; base += 256 * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + u * 256 + threadIdx.x;
      if (i < b1) __builtin_nontemporal_store(v, d + i);
    }
  }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

template <class F>
float timeit(F f, int iters) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  f(); hipDeviceSynchronize();
  hipEventRecord(a);
  for (int k = 0; k < iters; ++k) f();
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / iters;
}

int main() {
  const uint64_t bytes = 4104012958ull & ~uint64_t(15);
  const uint64_t n = bytes / 16;
  u32x4 *s, *d;
  CK(hipMalloc(&s, bytes)); CK(hipMalloc(&d, bytes));
  CK(hipMemset(s, 1, bytes)); CK(hipMemset(d, 0, bytes));
  auto rep = [&](const char* name, float ms) {
    printf("%-34s %8.3f ms  %7.0f GB/s (read+write)\n", name, ms, 2.0 * bytes / ms / 1e6);
  };
  for (int grid : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, 64, "gs U4 nt grid=%d", grid);
    rep(nm, timeit([&] { copy_gs<4, true><<<grid, 256>>>(s, d, n); }, 10));
    snprintf(nm, 64, "gs U4 plain grid=%d", grid);
    rep(nm, timeit([&] { copy_gs<4, false><<<grid, 256>>>(s, d, n); }, 10));
    snprintf(nm, 64, "gs U8 nt grid=%d", grid);
    rep(nm, timeit([&] { copy_gs<8, true><<<grid, 256>>>(s, d, n); }, 10));
  }
  for (uint64_t per : {16384ull, 65536ull, 262144ull}) {  // 16-byte units per block
    const unsigned grid = unsigned((n + per - 1) / per);
    char nm[64];
    snprintf(nm, 64, "blk U4 nt %lluKiB/blk", (unsigned long long)(per * 16 / 1024));
    rep(nm, timeit([&] { copy_blk<4, true><<<grid, 256>>>(s, d, n, per); }, 10));
    snprintf(nm, 64, "blk U8 nt %lluKiB/blk", (unsigned long long)(per * 16 / 1024));
    rep(nm, timeit([&] { copy_blk<8, true><<<grid, 256>>>(s, d, n, per); }, 10));
    snprintf(nm, 64, "blk U8 plain %lluKiB/blk", (unsigned long long)(per * 16 / 1024));
    rep(nm, timeit([&] { copy_blk<8, false><<<grid, 256>>>(s, d, n, per); }, 10));
  }
  for (uint64_t per : {4096ull, 8192ull}) {
    const unsigned grid = unsigned((n + per - 1) / per);
    char nm[64];
    snprintf(nm, 64, "blk U8 nt %lluKiB/blk", (unsigned long long)(per * 16 / 1024));
    rep(nm, timeit([&] { copy_blk<8, true><<<grid, 256>>>(s, d, n, per); }, 10));
  }
  for (int grid : {16384, 32768}) {
    char nm[64];
    snprintf(nm, 64, "gs U4 nt grid=%d", grid);
    rep(nm, timeit([&] { copy_gs<4, true><<<grid, 256>>>(s, d, n); }, 10));
  }
  {
    const uint64_t per = 16384;
    const unsigned grid = unsigned((n + per - 1) / per);
    float ms = timeit([&] { read_blk<8><<<grid, 256>>>(s, d, n, per); }, 10);
    printf("%-34s %8.3f ms  %7.0f GB/s (read only)\n", "read blk U8 nt 256KiB/blk", ms, bytes / ms / 1e6);
    ms = timeit([&] { write_blk<8><<<grid, 256>>>(d, n, per); }, 10);
    printf("%-34s %8.3f ms  %7.0f GB/s (write only)\n", "write blk U8 nt 256KiB/blk", ms, bytes / ms / 1e6);
  }
  for (uint64_t sz : {256ull << 20, 1ull << 30, 2ull << 30}) {  // smaller copies
    const uint64_t m = sz / 16, per = 16384;
    const unsigned grid = unsigned((m + per - 1) / per);
    float ms = timeit([&] { copy_blk<8, true><<<grid, 256>>>(s, d, m, per); }, 20);
    char nm[64];
    snprintf(nm, 64, "blk U8 nt 256KiB/blk %lluMiB", (unsigned long long)(sz >> 20));
    printf("%-34s %8.3f ms  %7.0f GB/s (read+write)\n", nm, ms, 2.0 * sz / ms / 1e6);
  }
  rep("hipMemcpyDtoD", timeit([&] { hipMemcpyAsync(d, s, bytes, hipMemcpyDeviceToDevice, 0); }, 10));
  return 0;
}
