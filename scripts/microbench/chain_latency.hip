// Latency of one link of the XXH3 long-loop chain, acc = ((x ^ x >> 47) ^ key) * PRIME32_1 with
// x = acc + sum, on gfx950: one wave, N dependent links, timed with s_memtime (wall clock of the
// whole chain via hipEvents). Variants: plain C (compiler's choice), inline asm with the
// high-half product beside the low one (mul_lo || mad), and a three-multiply split.
//   hipcc --offload-arch=gfx950 -O3 -o chain_latency chain_latency.hip && ./chain_latency
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr uint32_t P = 0x9E3779B1u;
constexpr int N = 1 << 16;

__global__ void plain(const uint64_t* s, uint64_t key, uint64_t* out) {
  uint64_t acc = threadIdx.x;
  const uint64_t t = s[threadIdx.x];
#pragma unroll 16
  for (int i = 0; i < N; ++i) {
    uint64_t x = acc + (t ^ uint64_t(i));
    x ^= x >> 47;
    x ^= key;
    acc = x * P;
  }
  out[threadIdx.x] = acc;
}

// x_next = mad(xl', P, {S_lo, S_hi + xh' * P}): the high-half product feeds the addend.
__global__ void asm_mad(const uint64_t* s, uint64_t key, uint64_t* out) {
  uint64_t acc = threadIdx.x;
  const uint64_t t = s[threadIdx.x];
  const uint32_t klo = uint32_t(key), khi = uint32_t(key >> 32);
  uint64_t x = acc + t;
#pragma unroll 16
  for (int i = 0; i < N; ++i) {
    const uint64_t sn = t ^ uint64_t(i + 1);
    uint32_t xl = uint32_t(x), xh = uint32_t(x >> 32);
    uint32_t tt, hp;
    uint64_t nx;
    asm volatile(
        "v_lshrrev_b32 %[tt], 15, %[xh]\n\t"
        "v_xor_b32 %[xh], %[xh], %[khi]\n\t"
        "v_bitop3_b32 %[xl], %[xl], %[tt], %[klo] bitop3:0x96\n\t"
        "v_mul_lo_u32 %[hp], %[xh], %[P]\n\t"
        "v_add_u32 %[hp], %[hp], %[snh]\n\t"
        "v_mov_b32 %[tt], %[snl]\n\t"
        : [tt] "=&v"(tt), [hp] "=&v"(hp), [xh] "+v"(xh), [xl] "+v"(xl)
        : [khi] "v"(khi), [klo] "v"(klo), [P] "s"(P), [snh] "v"(uint32_t(sn >> 32)),
          [snl] "v"(uint32_t(sn)));
    asm volatile("v_mad_u64_u32 %[nx], s[100:101], %[xl], %[P], %[ad]\n\t"
                 : [nx] "=&v"(nx)
                 : [xl] "v"(xl), [P] "s"(P), [ad] "v"((uint64_t(hp) << 32) | tt)
                 : "s100", "s101");
    x = nx;
  }
  out[threadIdx.x] = x - (t ^ uint64_t(N));
}

// Three independent multiplies (mul_lo, mul_hi of the low half; mul_lo of the high half).
__global__ void three_mul(const uint64_t* s, uint64_t key, uint64_t* out) {
  uint64_t acc = threadIdx.x;
  const uint64_t t = s[threadIdx.x];
  const uint32_t klo = uint32_t(key), khi = uint32_t(key >> 32);
#pragma unroll 16
  for (int i = 0; i < N; ++i) {
    const uint64_t x = acc + (t ^ uint64_t(i));
    const uint32_t xh = uint32_t(x >> 32);
    const uint32_t xl = uint32_t(x) ^ (xh >> 15) ^ klo;
    const uint32_t kh = xh ^ khi;
    const uint32_t lo = xl * P;
    const uint32_t hi = __umulhi(xl, P) + kh * P;
    acc = (uint64_t(hi) << 32) | lo;
  }
  out[threadIdx.x] = acc;
}

template <typename K>
float run(K kern, const uint64_t* s, uint64_t* o) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, s, 0x1234567890abcdefull, o);
  hipEventRecord(a);
  hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, s, 0x1234567890abcdefull, o);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main_loaded();
int main() {
  if (main_loaded()) return 1;
  uint64_t *s, *o;
  hipMalloc(&s, 64 * 8);
  hipMalloc(&o, 64 * 8 * 3);
  hipMemset(s, 7, 64 * 8);
  const float a = run(plain, s, o), b = run(asm_mad, s, o + 64), c = run(three_mul, s, o + 128);
  uint64_t h[192];
  hipMemcpy(h, o, sizeof(h), hipMemcpyDeviceToHost);
  printf("{\"links\": %d, \"plain_ns_per_link\": %.2f, \"asm_mad_ns\": %.2f, \"three_mul_ns\": %.2f,"
         " \"agree\": %s}\n",
         N, a * 1e6 / N, b * 1e6 / N, c * 1e6 / N,
         (h[5] == h[64 + 5] && h[5] == h[128 + 5]) ? "true" : "false");
  return 0;
}

// The chain as the finish kernel runs it: lane k of segment g reads the block sums S[b][k] of
// its segment (8 x u64 per block, segment-major) with kAhead loads in flight.
template <int kAhead>
__global__ void loaded(const uint64_t* sums, uint64_t nb, uint64_t key, uint64_t* out) {
  const int g = threadIdx.x >> 3, k = threadIdx.x & 7;
  const uint64_t* S = sums + (uint64_t(blockIdx.x) * 8 + g) * nb * 8 + k;
  uint64_t acc = k;
  uint64_t t0[kAhead], t1[kAhead];
  for (int i = 0; i < kAhead; ++i) t0[i] = S[i * 8];
  __builtin_amdgcn_sched_barrier(0);
  for (uint64_t b = 0; b + 2 * kAhead <= nb; b += 2 * kAhead) {
#pragma unroll
    for (int i = 0; i < kAhead; ++i) t1[i] = S[(b + kAhead + i) * 8];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < kAhead; ++i) {
      uint64_t x = acc + t0[i];
      x ^= x >> 47;
      x ^= key;
      acc = x * P;
    }
#pragma unroll
    for (int i = 0; i < kAhead; ++i) t0[i] = S[(b + 2 * kAhead + i) * 8];
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int i = 0; i < kAhead; ++i) {
      uint64_t x = acc + t1[i];
      x ^= x >> 47;
      x ^= key;
      acc = x * P;
    }
  }
  out[blockIdx.x * 64 + threadIdx.x] = acc;
}

template <int kAhead>
float run_loaded(const uint64_t* sums, uint64_t nb, int waves, uint64_t* o) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(loaded<kAhead>, dim3(waves), dim3(64), 0, 0, sums, nb, 0x1234ull, o);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(loaded<kAhead>, dim3(waves), dim3(64), 0, 0, sums, nb, 0x1234ull, o);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms;
}

int main_loaded() {
  const uint64_t nb = 65536;  // blocks per segment (64 MiB shard)
  for (int waves : {8, 32}) {
    uint64_t* sums;
    uint64_t* o;
    const uint64_t bytes = uint64_t(waves) * 8 * (nb + 256) * 64;
    if (hipMalloc(&sums, bytes) != hipSuccess || hipMalloc(&o, waves * 64 * 8) != hipSuccess)
      return 1;
    (void)hipMemset(sums, 1, bytes);
    printf("{\"segments\": %d, \"ahead16_ns\": %.2f, \"ahead32_ns\": %.2f, \"ahead64_ns\": %.2f}\n",
           waves * 8, run_loaded<16>(sums, nb, waves, o) * 1e6 / nb,
           run_loaded<32>(sums, nb, waves, o) * 1e6 / nb,
           run_loaded<64>(sums, nb, waves, o) * 1e6 / nb);
    (void)hipFree(sums);
    (void)hipFree(o);
  }
  return 0;
}
