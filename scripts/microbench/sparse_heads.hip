// Microbenchmark (not product code): the scan pass reads 8 bytes (a sample's size heads) per
// sample from a shard of samples a few hundred bytes long -- one 8-byte load per lane at a stride
// of `stride` bytes. How fast is that with each load cache policy, and which request sizes does
// the L2 send to memory for it (run under rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum ...)?
// Build + run:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/sh scripts/microbench/sparse_heads.hip && /tmp/sh
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// kPol: 0 plain, 1 nt, 2 sc0 sc1 (system scope: no L2 allocation on this part?), 3 sc1,
// 4 nt sc1, 5 sc0. One 8-byte load per lane at base + i * stride (+ i % 8 * 4: the heads are
// 4-byte aligned, not 8), the sum per block written out.
template <int kPol>
__global__ __launch_bounds__(256) void heads(const uint8_t* __restrict__ base, uint64_t n,
                                            uint32_t stride, uint32_t* __restrict__ out) {
  const uint64_t i = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  uint32_t s = 0;
  if (i < n) {
    const uint8_t* p = base + i * stride + (i & 1) * 4;
    u32x2 v;
    if constexpr (kPol == 0)
      asm volatile("global_load_dwordx2 %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    else if constexpr (kPol == 1)
      asm volatile("global_load_dwordx2 %0, %1, off nt\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    else if constexpr (kPol == 2)
      asm volatile("global_load_dwordx2 %0, %1, off sc0 sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    else if constexpr (kPol == 3)
      asm volatile("global_load_dwordx2 %0, %1, off sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    else if constexpr (kPol == 4)
      asm volatile("global_load_dwordx2 %0, %1, off nt sc1\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    else
      asm volatile("global_load_dwordx2 %0, %1, off sc0\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
    s = v.x + v.y;
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) out[i >> 6] = s;
}

template <int P>
float run(const uint8_t* buf, uint64_t n, uint32_t stride, uint32_t* out, int iters) {
  const unsigned grid = unsigned((n + 255) / 256);
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  hipLaunchKernelGGL(heads<P>, dim3(grid), dim3(256), 0, 0, buf, n, stride, out);
  CHECK(hipEventRecord(a));
  for (int k = 0; k < iters; ++k)
    hipLaunchKernelGGL(heads<P>, dim3(grid), dim3(256), 0, 0, buf, n, stride, out);
  CHECK(hipEventRecord(b));
  CHECK(hipEventSynchronize(b));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, a, b));
  return ms / iters;
}

int main(int argc, char** argv) {
  const uint64_t bytes = 1ull << 30;
  uint8_t* buf;
  uint32_t* out;
  CHECK(hipMalloc(&buf, bytes + 4096));
  CHECK(hipMemset(buf, 1, bytes + 4096));
  CHECK(hipMalloc(&out, (bytes / 64 / 64 + 64) * 4));
  // a 1 GiB flush buffer read between timed launches would add its own traffic; the 1 GiB shard
  // is far larger than L2 + MALL, so each launch reads from HBM anyway
  const uint32_t strides[] = {254, 512, 4300};
  const char* names[] = {"plain", "nt", "sc0sc1", "sc1", "ntsc1", "sc0"};
  for (uint32_t stride : strides) {
    const uint64_t n = bytes / stride;
    float t[6];
    t[0] = run<0>(buf, n, stride, out, 5);
    t[1] = run<1>(buf, n, stride, out, 5);
    t[2] = run<2>(buf, n, stride, out, 5);
    t[3] = run<3>(buf, n, stride, out, 5);
    t[4] = run<4>(buf, n, stride, out, 5);
    t[5] = run<5>(buf, n, stride, out, 5);
    for (int k = 0; k < 6; ++k)
      std::printf("{\"stride\": %u, \"samples\": %llu, \"policy\": \"%s\", \"us\": %.1f, "
                  "\"ns_per_sample\": %.4f}\n",
                  stride, (unsigned long long)n, names[k], t[k] * 1e3, t[k] * 1e6 / double(n));
  }
  return 0;
}
