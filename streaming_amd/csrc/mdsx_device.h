// Device helpers shared by the decode, gather and encode kernels of libmdsx.so (gfx950, wave64):
// 16-byte (non-temporal) loads/stores, byte realignment (v_alignbyte funnels over neighbour-lane
// chunks), the strict UTF-8 SWAR check, and the wave-wide realigning row copy.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mdsx_internal.h"

namespace mdsx_kernels {

int hip_check(hipError_t e, const char* what);

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Every byte these kernels touch outside LDS is device (global) memory. Accesses go through
// address-space-1 pointers so they compile to global_* instructions: a flat_* access also counts
// in lgkmcnt (every LDS wait then waits for the outstanding stores as well) and retires out of
// order, which explicit vmcnt bookkeeping (the LDS-DMA ring) cannot tolerate.
#define MDSX_G __attribute__((address_space(1)))
template <class T>
__device__ __forceinline__ MDSX_G T* gp(T* p) {
  return (MDSX_G T*)p;
}
template <class T>
__device__ __forceinline__ const MDSX_G T* gp(const T* p) {
  return (const MDSX_G T*)p;
}
template <class T>
__device__ __forceinline__ MDSX_G T* gp_at(uint64_t a) {
  return (MDSX_G T*)a;
}

// LDS pointers carry their address space, so every stage access compiles to ds_read (a generic
// pointer compiles to flat_load, which counts in vmcnt too: every wait for it would also wait for
// the consumers' stores in flight). The host pass only parses these device functions: it gets no
// address space (its vector types do not bind LDS references).
#ifdef __HIP_DEVICE_COMPILE__
#define MDSX_L __attribute__((address_space(3)))
#else
#define MDSX_L
#endif
typedef MDSX_L uint8_t lds_u8;

// 16-byte global load / store, optionally non-temporal (streamed once: no reuse in L2/MALL).
template <bool kNT>
__device__ __forceinline__ uint4 ld16(const uint4* p) {
  if constexpr (kNT) {
    const u32x4 v = __builtin_nontemporal_load((const MDSX_G u32x4*)p);
    return make_uint4(v.x, v.y, v.z, v.w);
  } else {
    const u32x4 v = *(const MDSX_G u32x4*)p;
    return make_uint4(v.x, v.y, v.z, v.w);
  }
}

template <bool kNT>
__device__ __forceinline__ void st16(uint64_t addr, const uint4 v) {
  if constexpr (kNT) {
    const u32x4 w = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(w, gp_at<u32x4>(addr));
  } else {
    const u32x4 w = {v.x, v.y, v.z, v.w};
    *gp_at<u32x4>(addr) = w;
  }
}

// One global_load_lds_dwordx4: 16 bytes per lane from gsrc (per-lane address) into LDS at
// lds + 16 * lane (lds wave-uniform). Issued from inline asm, so the compiler neither counts nor
// waits for it: the issuing wave waits with an explicit s_waitcnt vmcnt (and a barrier orders
// other waves' reads behind that wait).
template <bool kNT>
__device__ __forceinline__ void glds16(const void* gsrc, uint32_t lds) {
  const uint32_t lds_dst = __builtin_amdgcn_readfirstlane(lds);  // wave-uniform by construction
  uint32_t keep;
  if constexpr (kNT)
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_dst)
        : "memory");
  else
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_dst)
        : "memory");
}

// One global_load_lds_dword: 4 bytes per lane from gsrc into LDS at lds + 4 * lane.
__device__ __forceinline__ void glds4(const void* gsrc, uint32_t lds) {
  const uint32_t lds_dst = __builtin_amdgcn_readfirstlane(lds);
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\t"
      "global_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_dst)
      : "memory");
}

// s_waitcnt vmcnt(m) for the largest listed m <= n (a smaller count only waits longer).
__device__ __forceinline__ void wait_vm_at_most(uint32_t n) {
  if (n >= 48) asm volatile("s_waitcnt vmcnt(48)" ::: "memory");
  else if (n >= 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if (n >= 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  else if (n >= 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t r) {
  return __builtin_amdgcn_alignbyte(hi, lo, r);
}

__device__ __forceinline__ void report(mdsx_status* st, int code, int shard, int row, int col) {
  if (atomicCAS(&st->code, 0, code) == 0) {
    st->shard = shard;
    st->row = row;
    st->column = col;
  }
}

// u32 at any byte address (reads the two aligned dwords that cover it).
__device__ __forceinline__ uint32_t load_u32_any(const uint8_t* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const MDSX_G uint32_t* q = gp_at<const uint32_t>(a & ~uint64_t(3));
  return alignbyte(q[1], q[0], uint32_t(a & 3));
}

// The u32 size heads of a sample (MDSReader.decode_sample, mds/reader.py:111-116) at p, any byte
// alignment, up to kHeadRegs of them held in registers: one or two dword-aligned 16-byte loads
// per row instead of two dword loads per head (per-row memory requests bound the scan pass).
// Reads up to 31 bytes past the heads: inside the sample or the batch's 256-byte slack.
constexpr int kHeadRegs = 7;
typedef unsigned int u32x4a4 __attribute__((ext_vector_type(4), aligned(4)));
struct Heads {
  uint32_t w[8];
  uint32_t sh;
  template <bool kNT = false>
  __device__ __forceinline__ void load(const uint8_t* p, int n) {
    const uint64_t a = reinterpret_cast<uint64_t>(p);
    const MDSX_G u32x4a4* q = gp_at<const u32x4a4>(a & ~uint64_t(3));
    sh = uint32_t(a & 3);
    const u32x4a4 x = kNT ? __builtin_nontemporal_load(q) : q[0];
    w[0] = x.x, w[1] = x.y, w[2] = x.z, w[3] = x.w;
    if (4 * n + int(sh) > 16) {
      const u32x4a4 y = kNT ? __builtin_nontemporal_load(q + 1) : q[1];
      w[4] = y.x, w[5] = y.y, w[6] = y.z, w[7] = y.w;
    } else {
      w[4] = w[5] = w[6] = w[7] = 0;
    }
  }
  // Head k (< kHeadRegs; k may differ per lane only through the select chain, no indexing).
  __device__ __forceinline__ uint32_t get(int k) const {
    uint32_t r = 0;
#pragma unroll
    for (int j = 0; j < kHeadRegs; ++j) r = k == j ? alignbyte(w[j + 1], w[j], sh) : r;
    return r;
  }
};

// ---------------------------------------------------------------------------------------------
// Realignment: bytes [sh, sh + 16) of the 32-byte pair (lo, hi). sh is wave-uniform.
__device__ __forceinline__ uint4 funnel16(const uint4 lo, const uint4 hi, uint32_t sh) {
  const uint32_t r = sh & 3;
  switch (sh >> 2) {
    case 0:
      return make_uint4(alignbyte(lo.y, lo.x, r), alignbyte(lo.z, lo.y, r),
                        alignbyte(lo.w, lo.z, r), alignbyte(hi.x, lo.w, r));
    case 1:
      return make_uint4(alignbyte(lo.z, lo.y, r), alignbyte(lo.w, lo.z, r),
                        alignbyte(hi.x, lo.w, r), alignbyte(hi.y, hi.x, r));
    case 2:
      return make_uint4(alignbyte(lo.w, lo.z, r), alignbyte(hi.x, lo.w, r),
                        alignbyte(hi.y, hi.x, r), alignbyte(hi.z, hi.y, r));
    default:
      return make_uint4(alignbyte(hi.x, lo.w, r), alignbyte(hi.y, hi.x, r),
                        alignbyte(hi.z, hi.y, r), alignbyte(hi.w, hi.z, r));
  }
}

// The same with a per-lane shift (selects instead of a uniform branch).
__device__ __forceinline__ uint4 funnel16_lane(const uint4 lo, const uint4 hi, uint32_t sh) {
  const uint32_t q = sh >> 2, r = sh & 3;
  const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  uint32_t s[5];
#pragma unroll
  for (int k = 0; k < 5; ++k)
    s[k] = q == 0 ? w[k] : q == 1 ? w[k + 1] : q == 2 ? w[k + 2] : w[k + 3];
  return make_uint4(alignbyte(s[1], s[0], r), alignbyte(s[2], s[1], r), alignbyte(s[3], s[2], r),
                    alignbyte(s[4], s[3], r));
}

__device__ __forceinline__ uint32_t byte_of(const uint4& v, int j) {
  const uint32_t w = (j < 4) ? v.x : (j < 8) ? v.y : (j < 12) ? v.z : v.w;
  return (w >> (8 * (j & 3))) & 0xffu;
}

// Cross-lane moves by DPP (a VALU modifier: no LDS round trip, unlike ds_bpermute). Lanes with
// no source read 0.
template <int kCtrl>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
  return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), kCtrl, 0xF, 0xF, true));
}
template <int kCtrl>
__device__ __forceinline__ uint4 dpp_mov4(const uint4 v) {
  return make_uint4(dpp_mov<kCtrl>(v.x), dpp_mov<kCtrl>(v.y), dpp_mov<kCtrl>(v.z),
                    dpp_mov<kCtrl>(v.w));
}
constexpr int kDppWaveShl1 = 0x130;  // lane i <- lane i + 1 across the wave (lane 63: 0)
constexpr int kDppRowShl1 = 0x101;   // lane i <- lane i + 1 inside its row of 16 (lane 15: 0)
constexpr int kDppRowRor15 = 0x12F;  // lane i <- lane (i + 1) mod 16 of its row

// Lane i gets lane i + 1's chunk (lane 63: zeros; every caller replaces it).
__device__ __forceinline__ uint4 shfl_down1(const uint4 v) { return dpp_mov4<kDppWaveShl1>(v); }

// Inclusive prefix sum over the 64 lanes of a wave by DPP (no LDS round trips): row_shr 1, 2, 4,
// 8 within each row of 16 lanes, then row_bcast:15 (lane 15 of rows 0 and 2 into rows 1 and 3)
// and row_bcast:31 (lane 31 into rows 2 and 3). Lanes reading outside their row get 0.
__device__ __forceinline__ uint32_t wave_incl_dpp(uint32_t x) {
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x111, 0xF, 0xF, true));  // row_shr:1
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x112, 0xF, 0xF, true));  // row_shr:2
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x114, 0xF, 0xF, true));  // row_shr:4
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x118, 0xF, 0xF, true));  // row_shr:8
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x142, 0xA, 0xF, false));  // row_bcast:15
  x += uint32_t(__builtin_amdgcn_update_dpp(0, int(x), 0x143, 0xC, 0xF, false));  // row_bcast:31
  return x;
}

__device__ __forceinline__ uint4 readlane0(const uint4 v) {
  return make_uint4(__builtin_amdgcn_readlane(v.x, 0), __builtin_amdgcn_readlane(v.y, 0),
                    __builtin_amdgcn_readlane(v.z, 0), __builtin_amdgcn_readlane(v.w, 0));
}

// 0xFF in byte i of the result where bit i of the nibble x is set (the four shifted copies of x
// that the multiply adds never overlap, so no carries).
__device__ __forceinline__ uint32_t nibble_bytes(uint32_t x) {
  return ((x * 0x00204081u) & 0x01010101u) * 0xFFu;
}

// Byte mask of bytes [a, b) of a 16-byte chunk (0 <= a <= b <= 16).
__device__ __forceinline__ uint4 byte_mask(uint32_t a, uint32_t b) {
  const uint32_t bits = ((1u << b) - 1u) & ~((1u << a) - 1u);
  return make_uint4(nibble_bytes(bits & 15u), nibble_bytes((bits >> 4) & 15u),
                    nibble_bytes((bits >> 8) & 15u), nibble_bytes(bits >> 12));
}

// Bytes [a, b) (0 <= a <= b <= 16) of `val` merged into `acc`.
__device__ __forceinline__ uint4 merge_bytes(uint4 acc, const uint4 val, uint32_t a, uint32_t b) {
  const uint4 m = byte_mask(a, b);
  return make_uint4((acc.x & ~m.x) | (val.x & m.x), (acc.y & ~m.y) | (val.y & m.y),
                    (acc.z & ~m.z) | (val.z & m.z), (acc.w & ~m.w) | (val.w & m.w));
}

// ---- strict UTF-8 well-formedness, 4 bytes per dword op (SWAR) ------------------------------
// What bytes.decode('utf-8') accepts (encodings.py:80-81; Unicode Table 3-7): every byte is
// checked against its 3 predecessors. Per-byte predicates are bit 7 of each byte lane.
__device__ __forceinline__ uint32_t hi_c0(uint32_t y) { return y & (y << 1) & 0x80808080u; }
__device__ __forceinline__ uint32_t hi_e0(uint32_t y) {
  return y & (y << 1) & (y << 2) & 0x80808080u;
}
__device__ __forceinline__ uint32_t hi_f0(uint32_t y) {
  return y & (y << 1) & (y << 2) & (y << 3) & 0x80808080u;
}
__device__ __forceinline__ uint32_t zero_bytes(uint32_t v) {  // bit 7 set where the byte is 0
  return ~(((v & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | v) & 0x80808080u;
}

// Error bits of dword x given the dword before it (p): lone / missing continuation bytes,
// C0, C1, F5..FF, overlong E0/F0 forms, surrogates (ED A0..BF), code points > U+10FFFF.
__device__ __forceinline__ uint32_t utf8_dword_err(uint32_t x, uint32_t p) {
  const uint32_t p1 = alignbyte(x, p, 3), p2 = alignbyte(x, p, 2), p3 = alignbyte(x, p, 1);
  const uint32_t cont = x & ~(x << 1) & 0x80808080u;
  const uint32_t need = hi_c0(p1) | hi_e0(p2) | hi_f0(p3);
  uint32_t err = need ^ cont;
  err |= zero_bytes((x & 0xFEFEFEFEu) ^ 0xC0C0C0C0u);              // C0, C1
  err |= ((x & 0x7F7F7F7Fu) + 0x0B0B0B0Bu) & x & 0x80808080u;      // F5..FF
  const uint32_t b5 = (x << 2) & 0x80808080u, b45 = ((x << 2) | (x << 3)) & 0x80808080u;
  err |= zero_bytes(p1 ^ 0xE0E0E0E0u) & ~b5 & 0x80808080u;         // E0 followed by < A0
  err |= zero_bytes(p1 ^ 0xEDEDEDEDu) & b5;                        // ED followed by > 9F
  err |= zero_bytes(p1 ^ 0xF0F0F0F0u) & ~b45 & 0x80808080u;        // F0 followed by < 90
  err |= zero_bytes(p1 ^ 0xF4F4F4F4u) & b45;                       // F4 followed by > 8F
  return err;
}

// 16 segment bytes `v` (bytes outside the segment already zeroed) and the dword before them
// (zero before the segment start). `last`: v holds the segment's last byte, so a sequence still
// open at the end of v is truncated. Zero bytes never err except after an unfinished lead byte,
// which is exactly the truncated-sequence case.
__device__ __forceinline__ bool utf8_chunk_bad(const uint4 v, uint32_t pw, bool last) {
  const bool ascii = ((v.x | v.y | v.z | v.w) & 0x80808080u) == 0;
  if (ascii && hi_c0(pw) == 0) return false;  // no open sequence enters, none starts
  uint32_t err = utf8_dword_err(v.x, pw) | utf8_dword_err(v.y, v.x) | utf8_dword_err(v.z, v.y) |
                 utf8_dword_err(v.w, v.z);
  if (last) err |= utf8_dword_err(0u, v.w);  // positions 16..18 after the segment end
  return err != 0;
}

// ---- The same check by nibble tables (the Keiser-Lemire classification), about half the
// operations of utf8_dword_err: the error bits of a byte are the AND of three 16-entry byte-table
// lookups -- the previous byte's high nibble, its low nibble, this byte's high nibble -- each
// done with v_perm_b32 (an 8-entry byte select) and a blend; a byte that two / three bytes back
// has a lead >= E0 / F0 must be a continuation, which flips bit 7 (two continuations in a row)
// via must23. Error bits: 0 too short, 1 too long, 2 overlong 3-byte, 3 too large, 4 surrogate,
// 5 overlong 2-byte, 6 too large / overlong 4-byte, 7 two continuations. p1: the previous byte of
// each byte (v_alignbyte of this dword and the one before). Nonzero bytes of the result err.
__device__ __forceinline__ uint32_t utf8_lookup_err(uint32_t x, uint32_t p1, uint32_t must23) {
  const uint32_t sign1 = ((p1 >> 7) & 0x01010101u) * 0xFFu;  // previous byte >= 0x80
  // previous byte, high nibble: 0..7 -> 02 (ASCII), 8..B -> 80, C 21, D 01, E 15, F 49
  const uint32_t b1h = (__builtin_amdgcn_perm(0x49150121u, 0x80808080u, (p1 >> 4) & 0x07070707u) &
                        sign1) | (0x02020202u & ~sign1);
  // previous byte, low nibble: E7 A3 83 83 8B CB CB CB | CB CB CB CB CB DB CB CB
  const uint32_t lo3 = p1 & 0x07070707u;
  const uint32_t m8 = ((p1 >> 3) & 0x01010101u) * 0xFFu;
  const uint32_t b1l = (__builtin_amdgcn_perm(0xCBCBDBCBu, 0xCBCBCBCBu, lo3) & m8) |
                       (__builtin_amdgcn_perm(0xCBCBCB8Bu, 0x8383A3E7u, lo3) & ~m8);
  // this byte, high nibble: 8 E6, 9 AE, A..B BA (continuations), else 01
  const uint32_t cont = (((x & ~(x << 1)) >> 7) & 0x01010101u) * 0xFFu;
  const uint32_t b2h = (__builtin_amdgcn_perm(0u, 0xBABAAEE6u, (x >> 4) & 0x03030303u) & cont) |
                       (0x01010101u & ~cont);
  return (b1h & b1l & b2h) ^ must23;
}

// Bytes [a, b) of v (0 <= a <= b <= 16), others zero.
__device__ __forceinline__ uint4 keep_bytes(const uint4 v, uint32_t a, uint32_t b) {
  const uint4 m = byte_mask(a, b);
  return make_uint4(v.x & m.x, v.y & m.y, v.z & m.z, v.w & m.w);
}

// A sequence still open after the byte before chunk byte s (1..16) of the stream pw | X: one of
// the bytes s-1 / s-2 / s-3 is a lead >= C0 / E0 / F0 (a lead that saw too few continuations; if
// its sequence was already broken the check errs there anyway).
__device__ __forceinline__ bool utf8_open_at(const uint4 X, uint32_t pw, uint32_t s) {
  const uint32_t q = s >> 2;
  const uint32_t lo = q == 0 ? pw : q == 1 ? X.x : q == 2 ? X.y : q == 3 ? X.z : X.w;
  const uint32_t hi = q == 0 ? X.x : q == 1 ? X.y : q == 2 ? X.z : X.w;
  const uint32_t w = alignbyte(hi, lo, s & 3);  // bytes s-4 .. s-1
  const uint32_t t = w & (w << 1);
  return ((t & 0x80000000u) | (t & (w << 2) & 0x00800000u) |
          (t & (w << 2) & (w << 3) & 0x00008000u)) != 0;
}

// The 16 chunk bytes X (bytes outside the chunk's pieces zero) of two consecutive values: A,
// bytes < sB, whose bytes before the chunk end in pw (bytes before A's start zero), and B, bytes
// >= sB (1 <= sB <= 16; 16: A only), starting at sB. Every byte takes its context from its own
// value. Returns bit 0: A errs inside the chunk, bit 1: B does (a value that ends in the chunk
// is followed by zeros, which err after an open sequence; A's end at sB and a value ending at
// the chunk's end are the caller's, utf8_open_at).
__device__ __forceinline__ uint32_t utf8_chunk_err2(const uint4 X, uint32_t pw, uint32_t sB) {
  const uint4 MB = byte_mask(sB, 16);
  const uint32_t xs[4] = {X.x, X.y, X.z, X.w};
  const uint32_t ms[4] = {MB.x, MB.y, MB.z, MB.w};
  uint32_t errA = 0, errB = 0;
  uint32_t prev = pw, prevB = 0;
  uint32_t Ep = hi_e0(pw), Fp = hi_f0(pw), EBp = 0, FBp = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t x = xs[j], mb = ms[j];
    const uint32_t xB = x & mb;
    const uint32_t E = hi_e0(x), F = hi_f0(x), EB = E & mb, FB = F & mb;
    const uint32_t p1 = (alignbyte(xB, prevB, 3) & mb) | (alignbyte(x, prev, 3) & ~mb);
    const uint32_t m23 = ((alignbyte(EB, EBp, 2) | alignbyte(FB, FBp, 1)) & mb) |
                         ((alignbyte(E, Ep, 2) | alignbyte(F, Fp, 1)) & ~mb);
    const uint32_t err = utf8_lookup_err(x, p1, m23);
    errA |= err & ~mb;
    errB |= err & mb;
    prev = x, prevB = xB, Ep = E, Fp = F, EBp = EB, FBp = FB;
  }
  return (errA != 0 ? 1u : 0u) | (errB != 0 ? 2u : 0u);
}

// Bytes of a 16-byte chunk at address D that lie in [lo, hi), others zeroed.
__device__ __forceinline__ uint4 keep_range(const uint4 v, uint64_t D, uint64_t lo, uint64_t hi) {
  const int64_t a = max(int64_t(lo) - int64_t(D), int64_t(0));
  const int64_t b = min(int64_t(hi) - int64_t(D), int64_t(16));
  if (a == 0 && b == 16) return v;
  if (b <= a) return make_uint4(0, 0, 0, 0);
  const uint4 m = byte_mask(uint32_t(a), uint32_t(b));
  return make_uint4(v.x & m.x, v.y & m.y, v.z & m.z, v.w & m.w);
}

// Store the bytes of `chunk` (held by lane `le`, 16-byte aligned destination D) that fall in
// [d0, dend): one byte per lane, lanes 0..15, in a single wave instruction.
__device__ __forceinline__ void wave_edge_store(const uint4 chunk, int le, uint64_t D,
                                                uint64_t d0, uint64_t dend, int lane) {
  const uint32_t w0 = __builtin_amdgcn_readlane(chunk.x, le);
  const uint32_t w1 = __builtin_amdgcn_readlane(chunk.y, le);
  const uint32_t w2 = __builtin_amdgcn_readlane(chunk.z, le);
  const uint32_t w3 = __builtin_amdgcn_readlane(chunk.w, le);
  const uint64_t A = D + uint64_t(lane);
  if (lane < 16 && A >= d0 && A < dend) {
    const uint32_t w = lane < 4 ? w0 : lane < 8 ? w1 : lane < 12 ? w2 : w3;
    *gp_at<uint8_t>(A) = uint8_t(w >> (8 * (lane & 3)));
  }
}

__device__ __forceinline__ bool chunk_touches(const uint4* c, const uint8_t* src, uint64_t len) {
  const uint64_t a = reinterpret_cast<uint64_t>(c), s0 = reinterpret_cast<uint64_t>(src);
  return a + 16 > s0 && a < s0 + len;
}

// One wave copies `len` bytes from src to dst (any alignment of either). Destination chunks are
// 16-byte aligned; lane k of a step owns chunk k. Its source bytes straddle two aligned 16-byte
// source chunks: it loads the first and takes the second from lane k+1 (lane 63 from lane 0 of
// the next step, or one extra load at the end of a batch). The (at most two) partial chunks at
// the ends are written one byte per lane. With kUtf8, returns whether the segment is not
// well-formed UTF-8 (wave-uniform).
//
// kClamp: the source is not padded (a caller's tensor): aligned chunks that do not touch
// [src, src + len) are not loaded (they could lie on an unmapped page), only zero-filled.
template <bool kUtf8, int kUnroll, bool kNT, bool kEdges = true, bool kClamp = false>
__device__ __forceinline__ bool wave_copy(const uint8_t* src, uint8_t* dst, uint64_t len,
                                          int lane) {
  if (len == 0) return false;
  const uint64_t d0 = reinterpret_cast<uint64_t>(dst);
  const uint64_t dend = d0 + len;
  const uint64_t dbeg = d0 & ~uint64_t(15);
  const uint64_t nchunks = (((dend + 15) & ~uint64_t(15)) - dbeg) >> 4;
  const uint64_t sfirst = reinterpret_cast<uint64_t>(src) - (d0 - dbeg);
  const uint32_t sh = uint32_t(sfirst & 15);
  const uint4* sal = reinterpret_cast<const uint4*>(sfirst & ~uint64_t(15));
  const uint64_t nload = nchunks + (sh ? 1 : 0);
  const bool head_partial = dbeg < d0 || dbeg + 16 > dend;
  const bool tail_partial = nchunks > 1 && (dend & 15) != 0;
  bool bad = false;
  uint32_t carry = 0;  // last dword of the previous chunk (UTF-8 look-back)
  for (uint64_t base = 0; base < nchunks; base += 64 * kUnroll) {
    uint4 lo[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint64_t k = base + uint64_t(u) * 64 + lane;
      bool live = k < nload;
      if (kClamp) live = live && chunk_touches(sal + k, src, len);
      lo[u] = live ? ld16<kNT>(sal + k) : make_uint4(0, 0, 0, 0);
    }
    uint4 tail = make_uint4(0, 0, 0, 0);
    if (sh != 0 && lane == 63) {
      const uint64_t k = base + 64 * kUnroll;
      if (k < nload && (!kClamp || chunk_touches(sal + k, src, len))) tail = ld16<kNT>(sal + k);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint64_t k0 = base + uint64_t(u) * 64;
      if (k0 >= nchunks) break;  // wave-uniform
      const uint64_t k = k0 + lane;
      uint4 out = lo[u];
      if (sh != 0) {
        uint4 hi = shfl_down1(lo[u]);
        const uint4 nxt = (u + 1 < kUnroll) ? readlane0(lo[u + 1 < kUnroll ? u + 1 : u]) : tail;
        if (lane == 63) hi = nxt;
        out = funnel16(lo[u], hi, sh);
      }
      const uint64_t D = dbeg + 16 * k;
      if (kUtf8) {
        const uint4 vout = keep_range(out, D, d0, dend);
        uint32_t pw = __shfl_up(vout.w, 1);
        if (lane == 0) pw = carry;
        carry = __shfl(vout.w, 63);
        if (k < nchunks) bad |= utf8_chunk_bad(vout, pw, k == nchunks - 1);
      }
      if (k < nchunks && D >= d0 && D + 16 <= dend) st16<kNT>(D, out);
      if (kEdges) {  // kEdges == false: the caller guarantees 16-byte aligned dst and length
        if (k0 == 0 && head_partial) wave_edge_store(out, 0, dbeg, d0, dend, lane);
        if (tail_partial && nchunks - 1 >= k0 && nchunks - 1 < k0 + 64)
          wave_edge_store(out, int(nchunks - 1 - k0), dbeg + 16 * (nchunks - 1), d0, dend, lane);
      }
    }
  }
  if (kUtf8) return __any(bad);
  return false;
}

// Four rows per wave, one per 16-lane group (g = lane / 16, gl = lane % 16): the same copy as
// wave_copy -- aligned 16-byte destination chunks, the source realigned from the chunk a lane
// loads and its group neighbour's (gl + 1; gl 15 takes the next step's gl 0 or one extra load)
// -- for medium rows (a few hundred bytes) that would leave most of a wave's 64 lanes idle. Each group has its own
// src / dst / len (len 0: the group idles); the loop runs to the longest row of the wave.
// Partial chunks at a row's ends are stored one byte per lane of the group. (str rows are
// validated afterwards by group_utf8_bad: fused here the check costs the decode kernel a wave per
// SIMD, 118 vs 89 VGPRs.)
// kClamp: the source is a caller's tensor (not a padded batch): only aligned chunks touching
// [src, src + len) are loaded.
template <int kUnroll, bool kNT, bool kClamp = false>
__device__ __forceinline__ void group_copy(const uint8_t* src, uint8_t* dst, uint64_t len,
                                           int lane) {
  const int gl = lane & 15;
  const uint64_t d0 = reinterpret_cast<uint64_t>(dst);
  const uint64_t dend = d0 + len;
  const uint64_t dbeg = d0 & ~uint64_t(15);
  const uint64_t nchunks = len ? (((dend + 15) & ~uint64_t(15)) - dbeg) >> 4 : 0;
  const uint64_t sfirst = reinterpret_cast<uint64_t>(src) - (d0 - dbeg);
  const uint32_t sh = uint32_t(sfirst & 15);
  const uint4* sal = reinterpret_cast<const uint4*>(sfirst & ~uint64_t(15));
  const uint64_t nload = nchunks ? nchunks + (sh ? 1 : 0) : 0;  // an empty row loads nothing
  const bool head_partial = nchunks > 0 && (dbeg < d0 || dbeg + 16 > dend);
  const bool tail_partial = nchunks > 1 && (dend & 15) != 0;
  uint64_t maxc = nchunks;  // wave-uniform trip count
  maxc = max(maxc, uint64_t(__shfl_xor(static_cast<unsigned long long>(maxc), 16)));
  maxc = max(maxc, uint64_t(__shfl_xor(static_cast<unsigned long long>(maxc), 32)));
  for (uint64_t base = 0; base < maxc; base += 16 * kUnroll) {
    uint4 lo[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint64_t k = base + uint64_t(u) * 16 + gl;
      const bool live = k < nload && (!kClamp || chunk_touches(sal + k, src, len));
      lo[u] = live ? ld16<kNT>(sal + k) : make_uint4(0, 0, 0, 0);
    }
    uint4 tail = make_uint4(0, 0, 0, 0);
    {
      const uint64_t k = base + 16 * kUnroll;
      if (sh != 0 && gl == 15 && k < nload && (!kClamp || chunk_touches(sal + k, src, len)))
        tail = ld16<kNT>(sal + k);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint64_t k0 = base + uint64_t(u) * 16;
      if (k0 >= maxc) break;  // wave-uniform
      const uint64_t k = k0 + gl;
      // the group neighbour's chunk (gl 15: the group's next step's gl 0, or the extra load)
      uint4 hi = dpp_mov4<kDppRowShl1>(lo[u]);
      const uint4 nxt = u + 1 < kUnroll ? dpp_mov4<kDppRowRor15>(lo[u + 1 < kUnroll ? u + 1 : u])
                                        : tail;
      if (gl == 15) hi = nxt;
      const uint4 out = sh ? funnel16_lane(lo[u], hi, sh) : lo[u];
      const uint64_t D = dbeg + 16 * k;
      if (k < nchunks && D >= d0 && D + 16 <= dend) st16<kNT>(D, out);
      // partial chunks at the row ends: the group's 16 lanes store one byte each
      const bool head = head_partial && k0 == 0;
      const bool tl = tail_partial && nchunks - 1 >= k0 && nchunks - 1 < k0 + 16;
      if (__any(head || tl)) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const bool on = e == 0 ? head : tl;
          const int le = e == 0 ? 0 : int((nchunks - 1 - k0) & 15);
          const uint32_t w0 = __shfl(out.x, le, 16), w1 = __shfl(out.y, le, 16);
          const uint32_t w2 = __shfl(out.z, le, 16), w3 = __shfl(out.w, le, 16);
          const uint64_t E = e == 0 ? dbeg : dbeg + 16 * (nchunks - 1);
          const uint64_t A = E + uint64_t(gl);
          if (on && A >= d0 && A < dend) {
            const uint32_t w = gl < 4 ? w0 : gl < 8 ? w1 : gl < 12 ? w2 : w3;
            *gp_at<uint8_t>(A) = uint8_t(w >> (8 * (gl & 3)));
          }
        }
      }
    }
  }
}

// Strict UTF-8 check of four rows per wave already packed in `values` (one row per 16-lane
// group): each lane reads aligned 16-byte chunks of its group's row [off, off + len), bytes
// outside the row zeroed, the look-back dword passed along the group (zero before the row
// start). Returns, per lane, whether its group's row is not well-formed UTF-8.
template <int kUnroll>
__device__ __forceinline__ bool group_utf8_bad(const uint8_t* values, uint64_t off, uint64_t len,
                                               int lane) {
  const int gl = lane & 15;
  const uint64_t d0 = reinterpret_cast<uint64_t>(values) + off;
  const uint64_t dend = d0 + len;
  const uint64_t dbeg = d0 & ~uint64_t(15);
  const uint64_t nchunks = len ? (((dend + 15) & ~uint64_t(15)) - dbeg) >> 4 : 0;
  uint64_t maxc = nchunks;
  maxc = max(maxc, uint64_t(__shfl_xor(static_cast<unsigned long long>(maxc), 16)));
  maxc = max(maxc, uint64_t(__shfl_xor(static_cast<unsigned long long>(maxc), 32)));
  bool bad = false;
  uint32_t carry = 0;
  for (uint64_t base = 0; base < maxc; base += 16 * kUnroll) {
    uint4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint64_t k = base + uint64_t(u) * 16 + gl;
      v[u] = k < nchunks ? ld16<false>(reinterpret_cast<const uint4*>(dbeg + 16 * k))
                         : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) {
      const uint64_t k0 = base + uint64_t(u) * 16;
      if (k0 >= maxc) break;  // wave-uniform
      const uint64_t k = k0 + gl;
      const uint4 vout = keep_range(v[u], dbeg + 16 * k, d0, dend);
      uint32_t pw = __shfl_up(vout.w, 1, 16);
      if (gl == 0) pw = carry;
      carry = __shfl(vout.w, 15, 16);
      if (k < nchunks) bad |= utf8_chunk_bad(vout, pw, k == nchunks - 1);
    }
  }
  const uint64_t m = __ballot(bad);
  return ((m >> (lane & 48)) & 0xffffull) != 0;
}

// Fixed column of 1..16 bytes: one row per lane. dst is aligned to the largest power of two
// dividing the row size (outputs are 256-byte aligned tensors). small_load: the row's bytes
// (from any alignment) into the low bytes of a chunk; small_store: them to dst.
__device__ __forceinline__ uint4 small_load(const uint8_t* p, uint32_t size) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const MDSX_G uint32_t* q = gp_at<const uint32_t>(a & ~uint64_t(3));
  const uint32_t r = uint32_t(a & 3);
  const uint32_t nd = (size + 6) >> 2;  // dwords covering r + size bytes for any r <= 3
  const uint32_t w0 = q[0];
  const uint32_t w1 = nd > 1 ? q[1] : 0u;
  const uint32_t w2 = nd > 2 ? q[2] : 0u;
  const uint32_t w3 = nd > 3 ? q[3] : 0u;
  const uint32_t w4 = nd > 4 ? q[4] : 0u;
  return make_uint4(alignbyte(w1, w0, r), alignbyte(w2, w1, r), alignbyte(w3, w2, r),
                    alignbyte(w4, w3, r));
}

__device__ __forceinline__ void small_store(uint8_t* dst_, const uint4 o, uint32_t size) {
  MDSX_G uint8_t* dst = gp(dst_);
  switch (size) {
    case 1: *dst = uint8_t(o.x); break;
    case 2: *(MDSX_G uint16_t*)dst = uint16_t(o.x); break;
    case 4: *(MDSX_G uint32_t*)dst = o.x; break;
    case 8:
      ((MDSX_G uint32_t*)dst)[0] = o.x;
      ((MDSX_G uint32_t*)dst)[1] = o.y;
      break;
    case 12:
      ((MDSX_G uint32_t*)dst)[0] = o.x;
      ((MDSX_G uint32_t*)dst)[1] = o.y;
      ((MDSX_G uint32_t*)dst)[2] = o.z;
      break;
    case 16: *(MDSX_G u32x4*)dst = u32x4{o.x, o.y, o.z, o.w}; break;
    default:
      for (uint32_t j = 0; j < size; ++j) dst[j] = uint8_t(byte_of(o, int(j)));
  }
}

__device__ __forceinline__ void gather_small(const uint8_t* p, uint8_t* dst, uint32_t size) {
  small_store(dst, small_load(p, size), size);
}

}  // namespace mdsx_kernels
