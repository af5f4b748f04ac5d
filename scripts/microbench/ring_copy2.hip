// Microbenchmark (not product code), after ring_copy.hip: the streaming decode's shape more
// closely -- each wave's piece (8 KiB = one run of two ~4 KiB samples) located by a table load,
// waits per sample (4 slots) -- one piece per wave (the decode today) against PERSISTENT waves
// that walk pieces w, w + G, w + 2G, ... (G waves in the grid) through one continuous ring, the
// next pieces' slots issued while the current one is copied, their table entries read 64 at a
// time (lane l: piece j + l). Also the grid size (workgroups per CU) of the persistent form.
// Build + run:
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/rc2 scripts/microbench/ring_copy2.hip && /tmp/rc2
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
#define LDS __attribute__((address_space(3)))

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

__device__ __forceinline__ void wait_vm(uint32_t n) {
  if (n >= 16) {
    if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

constexpr uint32_t kPieceSlots = 8;  // 8 KiB pieces
constexpr uint32_t kGroup = 4;       // waits per 4 KiB "sample"

// kPers: persistent waves over pieces w + j * G; else one piece per wave (G = pieces).
template <int S, bool kPers>
__global__ __launch_bounds__(128) void ring_copy(const u32x4* __restrict__ src,
                                                 u32x4* __restrict__ dst,
                                                 const uint32_t* __restrict__ table,
                                                 uint32_t npieces) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t w = blockIdx.x * 2 + uint32_t(wave);
  const uint32_t G = kPers ? gridDim.x * 2 : npieces;
  if (w >= npieces) return;
  const uint32_t mine = kPers ? (npieces - w + G - 1) / G : 1u;  // pieces of this wave
  const uint32_t nslots = mine * kPieceSlots;
  uint8_t* ring = smem + wave * S * 1024;
  const uint32_t ring_lds = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const LDS uint8_t*)ring)));
  // lane l: the table entry of this wave's piece j0 + l (refreshed every 64 pieces)
  uint32_t tab = lane < int(mine) ? table[w + uint32_t(lane) * G] : 0u;
  uint32_t tab_j0 = 0;
  uint32_t issued = 0, ops = 1, op_at = 0;  // (the table load counted)
  uint32_t slot_pb = 0;  // lane r: the piece of the slot at ring position r
  auto piece_base = [&](uint32_t j) -> uint32_t {  // wave-uniform
    if (j >= tab_j0 + 64) {  // (persistent waves with more than 64 pieces)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      tab_j0 += 64;
      tab = tab_j0 + lane < mine ? table[w + (tab_j0 + uint32_t(lane)) * G] : 0u;
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    return uint32_t(__builtin_amdgcn_readlane(int(tab), int(j - tab_j0)));
  };
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  auto pump = [&](uint32_t low) {
    while (issued < nslots && issued < low + S) {
      const uint32_t j = issued / kPieceSlots, ls = issued % kPieceSlots;
      const uint32_t pb = piece_base(j);
      glds16(src + (uint64_t(pb) * kPieceSlots + ls) * 64 + lane, ring_lds + (issued % S) * 1024u);
      if (lane == int(issued % S)) op_at = ops, slot_pb = pb;
      ++ops;
      ++issued;
    }
  };
  pump(0);
  for (uint32_t g = 0; g < nslots; g += kGroup) {
    const uint32_t last = g + kGroup - 1;
    wait_vm(ops - uint32_t(__builtin_amdgcn_readlane(int(op_at), int(last % S))) - 1);
    const uint32_t pb = uint32_t(__builtin_amdgcn_readlane(int(slot_pb), int(g % S)));
    for (uint32_t i = g; i <= last; ++i) {
      const u32x4 v = *(const LDS u32x4*)((const LDS uint8_t*)ring + (i % S) * 1024 + 16 * lane);
      __builtin_nontemporal_store(v, dst + (uint64_t(pb) * kPieceSlots + i % kPieceSlots) * 64 + lane);
      ++ops;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    pump(last + 1);
  }
}

int main() {
  const uint64_t bytes = 4ull << 30;
  const uint32_t np = uint32_t(bytes / (kPieceSlots * 1024));
  u32x4 *src, *dst;
  uint32_t* table;
  CHECK(hipMalloc(&src, bytes));
  CHECK(hipMalloc(&dst, bytes));
  CHECK(hipMalloc(&table, np * 4ull));
  std::vector<uint32_t> ht(np);
  for (uint32_t i = 0; i < np; ++i) ht[i] = i;
  CHECK(hipMemcpy(table, ht.data(), np * 4ull, hipMemcpyHostToDevice));
  std::vector<uint8_t> h(1 << 20);
  for (size_t i = 0; i < h.size(); ++i) h[i] = uint8_t((i * 131 + 7) ^ (i >> 9));
  for (uint64_t o = 0; o < bytes; o += h.size())
    CHECK(hipMemcpy(reinterpret_cast<uint8_t*>(src) + o, h.data(), h.size(), hipMemcpyHostToDevice));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  struct V {
    const char* name;
    int s;
    bool pers;
    int wg_per_cu;
  };
  const V vs[] = {{"one_S7", 7, false, 0},     {"one_S16", 16, false, 0},
                  {"pers_S7_k8", 7, true, 8},  {"pers_S7_k4", 7, true, 4},
                  {"pers_S16_k4", 16, true, 4}, {"pers_S16_k2", 16, true, 2},
                  {"pers_S16_k3", 16, true, 3}, {"pers_S7_k6", 7, true, 6}};
  for (int rnd = 0; rnd < 3; ++rnd) {
    for (const V& v : vs) {
      const unsigned grid = v.pers ? unsigned(cus * v.wg_per_cu) : (np + 1) / 2;
      const size_t lds = size_t(2) * v.s * 1024;
      auto launch = [&]() {
        if (v.s == 7 && !v.pers)
          hipLaunchKernelGGL((ring_copy<7, false>), dim3(grid), dim3(128), lds, 0, src, dst, table, np);
        else if (v.s == 16 && !v.pers)
          hipLaunchKernelGGL((ring_copy<16, false>), dim3(grid), dim3(128), lds, 0, src, dst, table, np);
        else if (v.s == 7)
          hipLaunchKernelGGL((ring_copy<7, true>), dim3(grid), dim3(128), lds, 0, src, dst, table, np);
        else
          hipLaunchKernelGGL((ring_copy<16, true>), dim3(grid), dim3(128), lds, 0, src, dst, table, np);
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
      for (uint64_t o : {uint64_t(0), bytes / 2 + 4096, bytes - (1 << 20)}) {
        CHECK(hipMemcpy(got.data(), reinterpret_cast<uint8_t*>(dst) + o, got.size(), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(want.data(), reinterpret_cast<uint8_t*>(src) + o, want.size(), hipMemcpyDeviceToHost));
        ok = ok && std::memcmp(got.data(), want.data(), got.size()) == 0;
      }
      CHECK(hipMemset(dst, 0, bytes));
      std::printf("{\"round\": %d, \"variant\": \"%s\", \"grid\": %u, \"GBps\": %.1f, \"ok\": %s}\n",
                  rnd, v.name, grid, 2.0 * bytes / (ms / iters) / 1e6, ok ? "true" : "false");
      std::fflush(stdout);
    }
  }
  return 0;
}
