// The per-wave LDS-DMA stream ring shared by the streaming decodes (mdsx_run.hip: the general
// and lean paths; mdsx_win.hip: the windowed decode of short samples), and small wave helpers.
//
// A wave streams a contiguous byte range of the batch (a run of consecutive samples of one
// shard) through a private ring of S 1 KiB slots in LDS (S any size; a power of two makes the
// modulo a mask): stream byte p lives at ring byte p % (S KiB), and a 64-byte mirror of the ring's first bytes sits behind it so that a 16-byte
// read crossing the ring's end is one contiguous read. Slots are loaded with
// global_load_lds_dwordx4 (1 KiB per wave-instruction, no VGPR destination) issued from inline
// asm, so the compiler neither counts nor waits for them: the wave waits with an explicit
// `s_waitcnt vmcnt(n)`, n = the vector-memory operations it issued after the slot's load (its
// loads, and the stores certain to have issued; counting fewer only waits longer).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mdsx_device.h"

namespace mdsx_kernels {

constexpr uint32_t kMirror = 64;

// Ring byte of stream byte p. p may have wrapped below 0 by less than a ring (a value's first
// chunk read from before the stream start, bytes then replaced by the carried ones): the ring
// size is added first, so the modulo of a ring that does not divide 2^32 stays consistent.
template <int S>
__device__ __forceinline__ uint32_t ring_pos(uint32_t p) {
  return (p + S * 1024u) % (S * 1024u);
}

// 16 stream bytes at stream byte p: one ds_read_b128 at any byte address (gfx950 reads LDS
// unaligned; the 16-byte realignment costs no instructions).
template <int S>
__device__ __forceinline__ uint4 ring16(const lds_u8* ring, uint32_t p) {
  const u32x4 v = *(const MDSX_L u32x4*)(ring + ring_pos<S>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// u32 at stream byte p (any alignment).
template <int S>
__device__ __forceinline__ uint32_t ring_u32(const lds_u8* ring, uint32_t p) {
  return *(const MDSX_L uint32_t*)(ring + ring_pos<S>(p));
}

// s_waitcnt vmcnt(m), m the largest of 0, 1, 2, 4, 8, 16, 32 not above n (three compares).
__device__ __forceinline__ void wait_vm_coarse(uint32_t n) {
  if (n >= 16) {
    if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  } else if (n >= 4) {
    if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else if (n >= 2) {
    asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  } else if (n == 1) {
    asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

// s_waitcnt vmcnt(n) for n <= 16 exactly (larger n: 16).
__device__ __forceinline__ void wait_vm_exact16(uint32_t n) {
  switch (n) {
#define MDSX_VMW(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
    MDSX_VMW(0) MDSX_VMW(1) MDSX_VMW(2) MDSX_VMW(3) MDSX_VMW(4) MDSX_VMW(5) MDSX_VMW(6)
    MDSX_VMW(7) MDSX_VMW(8) MDSX_VMW(9) MDSX_VMW(10) MDSX_VMW(11) MDSX_VMW(12) MDSX_VMW(13)
    MDSX_VMW(14) MDSX_VMW(15)
#undef MDSX_VMW
    default: asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  }
}

// The wave's stream: chunks [0, nq) from base, in slots of 64 chunks.
struct Stream {
  const uint4* base;
  uint32_t nq, nslots;
  uint32_t issued;  // slots issued
  uint32_t ops;     // vector-memory operations issued by this wave (loads; stores certain to issue)
  uint32_t op_at;   // lane r: `ops` when the slot now in ring position r was issued
  uint32_t mirrored;  // the last slot at ring position 0 copied to the mirror
  uint32_t landed;    // slots [0, landed) have landed (waited for)
};

// Issue slots while they fit in the ring above slot `low`: the stream bytes still to be read
// all lie in slots >= low (callers pass a non-decreasing low). kEdge: the stream's first and
// last slots -- the lines it shares with the neighbouring streams -- load with the default
// cache policy (the others with kNT), so that the neighbour's read of a shared line can hit L2.
template <int S, bool kNT, bool kEdge = false>
__device__ __forceinline__ void pump(Stream& st, uint32_t ring_lds, uint32_t low, int lane) {
  while (st.issued < st.nslots && st.issued < low + S) {
    const uint32_t k = st.issued * 64u + uint32_t(lane);
    const uint32_t slot = st.issued % uint32_t(S);
    if (kEdge && (st.issued == 0 || st.issued + 1 == st.nslots))
      glds16<false>(st.base + min(k, st.nq - 1), ring_lds + (slot << 10));
    else
      glds16<kNT>(st.base + min(k, st.nq - 1), ring_lds + (slot << 10));
    if (lane == int(slot)) st.op_at = st.ops;
    ++st.ops;
    ++st.issued;
  }
}

// pump, then wait until stream bytes [lo, hi] (hi - lo < (S - 1) KiB) have landed; a slot at ring
// position 0 that has landed is mirrored behind the ring for the reads that wrap.
template <int S, bool kNT, bool kEdge = false>
__device__ __forceinline__ void ensure(Stream& st, const lds_u8* ring, uint32_t ring_lds,
                                       uint32_t lo, uint32_t hi, int lane) {
  pump<S, kNT, kEdge>(st, ring_lds, lo >> 10, lane);
  const uint32_t upto = min(hi >> 10, st.nslots - 1);
  if (upto < st.landed) return;  // waited for already
  st.landed = upto + 1;
  wait_vm_coarse(st.ops - uint32_t(__builtin_amdgcn_readlane(int(st.op_at), int(upto % S))) - 1u);
  const uint32_t j0 = upto - upto % uint32_t(S);  // the slot at ring position 0
  if (j0 != st.mirrored) {
    st.mirrored = j0;
    if (lane < int(kMirror / 4))
      *(MDSX_L uint32_t*)(ring + S * 1024 + 4 * lane) = *(const MDSX_L uint32_t*)(ring + 4 * lane);
  }
}

__device__ __forceinline__ uint4 readlane4(const uint4 v, int l) {
  return make_uint4(__builtin_amdgcn_readlane(v.x, l), __builtin_amdgcn_readlane(v.y, l),
                    __builtin_amdgcn_readlane(v.z, l), __builtin_amdgcn_readlane(v.w, l));
}

__device__ __forceinline__ uint64_t readlane64(uint64_t v, int l) {
  return uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v)), l))) |
         (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(v >> 32)), l))) << 32);
}

// u32 inclusive prefix sum over lanes [0, n) (n <= 64 wave-uniform; other lanes: garbage)
__device__ __forceinline__ uint32_t wave_incl_u32(uint32_t x, int lane, int n) {
  for (int o = 1; o < n; o <<= 1) {
    const uint32_t y = uint32_t(__shfl_up(int(x), o));
    if (lane >= o) x += y;
  }
  return x;
}

// bytes [0, h) of `lo` and [h, 16) of `hi` (h wave-uniform, 0..16)
__device__ __forceinline__ uint4 splice_lo(const uint4 lo, const uint4 hi, uint32_t h) {
  const uint64_t m0 = h >= 8 ? ~0ull : (1ull << (8 * h)) - 1ull;
  const uint64_t m1 = h <= 8 ? 0ull : h >= 16 ? ~0ull : (1ull << (8 * (h - 8))) - 1ull;
  const uint32_t w0 = uint32_t(m0), w1 = uint32_t(m0 >> 32), w2 = uint32_t(m1),
                 w3 = uint32_t(m1 >> 32);
  return make_uint4((lo.x & w0) | (hi.x & ~w0), (lo.y & w1) | (hi.y & ~w1),
                    (lo.z & w2) | (hi.z & ~w2), (lo.w & w3) | (hi.w & ~w3));
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// n (1..16) bytes of `v` to LDS at p (p aligned to the largest power of two dividing n)
__device__ __forceinline__ void lds_put(MDSX_L uint8_t* p, const uint4 v, uint32_t n) {
  if (n == 8) {
    *(MDSX_L u32x2*)p = u32x2{v.x, v.y};
  } else if (n == 4) {
    *(MDSX_L uint32_t*)p = v.x;
  } else if (n == 16) {
    *(MDSX_L u32x4*)p = u32x4{v.x, v.y, v.z, v.w};
  } else {
    for (uint32_t k = 0; k < n; ++k) p[k] = uint8_t(byte_of(v, int(k)));
  }
}

// n (1..16) bytes from LDS at p to global memory at q (both aligned as in lds_put)
__device__ __forceinline__ void lds_out(const MDSX_L uint8_t* p, uint8_t* q, uint32_t n) {
  if (n == 8) {
    *(MDSX_G u32x2*)gp((u32x2*)q) = *(const MDSX_L u32x2*)p;
  } else if (n == 4) {
    *gp((uint32_t*)q) = *(const MDSX_L uint32_t*)p;
  } else if (n == 16) {
    const u32x4 v = *(const MDSX_L u32x4*)p;
    *(MDSX_G u32x4*)gp((u32x4*)q) = v;
  } else {
    for (uint32_t k = 0; k < n; ++k) *gp(q + k) = p[k];
  }
}

}  // namespace mdsx_kernels
