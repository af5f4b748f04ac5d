// MI355X kernels of shard-file hashing on the device: the xxHash digests the
// reference records per shard file in index.json (Writer._write_file, base/writer.py:197-200,
// through get_hash, hashing.py:55-68) and recomputes to validate a downloaded or decompressed
// shard (Stream._decompress_shard_part / _prepare_shard_part, stream.py:333-340,403-411),
// computed over shard files already resident in HBM instead of re-reading them on the host.
//
// Algorithms: xxh32, xxh64, xxh3_64, xxh3_128 (= xxh128), python-xxhash 3.x / xxHash 0.8.2
// semantics (seeded), as restated in oracle/xxh_oracle.py.
//
// XXH3 on inputs > 240 bytes (every shard) is split so that the HBM stream runs on the whole
// chip. Its long loop is, per 1 KiB block b (16 stripes of 64 B with the 192-byte secret):
//     acc = scramble(acc + S_b),   S_b[k] = sum over the block's stripes of the stripe terms,
// because the accumulate step only ADDS terms that depend on the data and the secret, never on
// acc. So
//   xxh3_sums_kernel   reads every full block once (coalesced 16-byte loads, 128 contiguous
//                      bytes per 8 lanes) and writes S_b (64 B per KiB: 1/16 of the input);
//                      grid-stride over 128-block chunks of all segments;
//   chain role         8 lanes per segment (one per accumulator) run the short dependent chain
//                      acc = scramble(acc + S_b) over the block sums (loads issued 16 blocks
//                      ahead), then one lane per segment hashes the tail (partial block, last
//                      stripe), merges the accumulators and writes the digest. Inputs <= 240
//                      bytes take the short paths in the same lane.
//   xxh3_fused_kernel  both roles in one launch: the first workgroups run the chains and wait on
//                      per-chunk flags (agent-scope acquire) that the streaming workgroups
//                      publish (release) as they finish each chunk, in segment-interleaved
//                      order -- the ~1 ms dependent chain of a 64 MiB shard then overlaps the
//                      HBM stream instead of following it. xxh3_sums_kernel + xxh3_finish_kernel
//                      are the two-launch form of the same work (MDSX_HASH_FUSED=0).
// XXH64 / XXH32 are one dependent chain per accumulator (4 lanes per segment, loads issued 8
// stripes ahead): xxh_seq_kernel. They are latency-bound per segment and only pay off over many
// resident shards at once; DESIGN.md reports both.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <cstring>

#include "mdsx_device.h"
#include "mdsx_internal.h"

// The default XXH3 secret (kSecret of xxHash 0.8.2), for the device and the host.
#define MDSX_XXH3_SECRET \
  0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c, \
  0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f, \
  0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21, \
  0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c, \
  0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3, \
  0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8, \
  0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d, \
  0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64, \
  0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb, \
  0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e, \
  0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce, \
  0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e

namespace mdsx_kernels {
namespace {

constexpr uint32_t P32_1 = 0x9E3779B1u, P32_2 = 0x85EBCA77u, P32_3 = 0xC2B2AE3Du,
                   P32_4 = 0x27D4EB2Fu, P32_5 = 0x165667B1u;
constexpr uint64_t P64_1 = 0x9E3779B185EBCA87ull, P64_2 = 0xC2B2AE3D27D4EB4Full,
                   P64_3 = 0x165667B19E3779F9ull, P64_4 = 0x85EBCA77C2B2AE63ull,
                   P64_5 = 0x27D4EB2F165667C5ull;
constexpr uint64_t PMX1 = 0x165667919E3779F9ull, PMX2 = 0x9FB21C651E98DF25ull;

constexpr int kSecretBytes = 192;
constexpr int kStripe = 64;
constexpr int kBlockBytes = 1024;     // (192 - 64) / 8 = 16 stripes per block
constexpr int kChunkBlocks = 512;     // blocks per sums-kernel chunk (4 waves x 16 x 8 blocks)
constexpr int kSumsBlock = 256;
constexpr int kChainAhead = 16;        // chain links whose block sums are loaded ahead (16 is
                                       // fastest: 17-23 ns per link, microbench/chain_latency)
constexpr int kChainSegs = 8;          // segments per chain workgroup: ONE wave (8 lanes each)
constexpr int kFusedMaxChain = 32;     // fused launch only up to 32 chain workgroups (256 segments)
constexpr int kSumsGridMax = 256 * 8;  // persistent grid: 8 workgroups per CU
constexpr int kSeqPerWave = 4;         // xxh_seq_kernel: segments per wave (4 lanes each)

__constant__ uint8_t kSecret[kSecretBytes] = {MDSX_XXH3_SECRET};
const uint8_t kSecretHost[kSecretBytes] = {MDSX_XXH3_SECRET};

typedef __attribute__((address_space(1))) uint32_t gu32;  // global (never flat) words
typedef __attribute__((address_space(1))) uint64_t gu64;

struct HashArgs {
  const uint8_t* data;
  uint64_t data_bytes;
  const mdsx_segment* segs;
  uint64_t* digests;     // 2 x u64 per segment: low 64 bits, high 64 bits (xxh3_128)
  mdsx_status* status;
  uint64_t* sums;        // 8 x u64 per full block of every long XXH3 segment
  uint64_t* block0;      // nseg + 1: prefix of block counts
  uint64_t* chunk0;      // nseg + 2: prefix of 128-block chunk counts, then the largest count
  uint32_t* ctrl;        // fused kernel: [0] chunk tickets, [1 + i] CU of chain workgroup i
  uint32_t* flags;       // per chunk: its sums are published (fused kernel)
  uint64_t sums_capacity;  // blocks the sums area holds
  uint64_t flags_capacity; // chunks the flag area holds
  uint64_t seed;
  int32_t nseg;
  int32_t algo;
  uint64_t secret[kSecretBytes / 8];  // secret of long XXH3 inputs (derived from the seed)
};

// ---- unaligned little-endian loads (tails and short inputs only) -----------------------------
// Reads only the aligned dwords that cover [p, p + 4): never past the dword of the last byte.
__device__ __forceinline__ uint32_t ld32u(const uint8_t* p) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~uint64_t(3));
  const uint32_t r = uint32_t(a & 3);
  const uint32_t lo = q[0];
  if (r == 0) return lo;
  return alignbyte(q[1], lo, r);
}
__device__ __forceinline__ uint64_t ld64u(const uint8_t* p) {
  return uint64_t(ld32u(p)) | (uint64_t(ld32u(p + 4)) << 32);
}
// Secret bytes (constant or LDS) at any offset.
__device__ __forceinline__ uint32_t sec32(const uint8_t* s, int off) {
  return uint32_t(s[off]) | (uint32_t(s[off + 1]) << 8) | (uint32_t(s[off + 2]) << 16) |
         (uint32_t(s[off + 3]) << 24);
}
__device__ __forceinline__ uint64_t sec64(const uint8_t* s, int off) {
  return uint64_t(sec32(s, off)) | (uint64_t(sec32(s, off + 4)) << 32);
}

__device__ __forceinline__ uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t fold64(uint64_t a, uint64_t b) {
  return (a * b) ^ __umul64hi(a, b);
}
__device__ __forceinline__ uint64_t swap64(uint64_t x) { return __builtin_bswap64(x); }
__device__ __forceinline__ uint32_t swap32(uint32_t x) { return __builtin_bswap32(x); }

// ---- XXH32 / XXH64 pieces --------------------------------------------------------------------
__device__ __forceinline__ uint32_t round32(uint32_t acc, uint32_t lane) {
  return rotl32(acc + lane * P32_2, 13) * P32_1;
}
__device__ __forceinline__ uint64_t round64(uint64_t acc, uint64_t lane) {
  return rotl64(acc + lane * P64_2, 31) * P64_1;
}
__device__ __forceinline__ uint64_t avalanche64(uint64_t h) {
  h ^= h >> 33;
  h *= P64_2;
  h ^= h >> 29;
  h *= P64_3;
  return h ^ (h >> 32);
}

// Tail + avalanche of XXH32 from byte i (h already holds the lane merge + length).
__device__ uint32_t xxh32_tail(const uint8_t* p, uint64_t i, uint64_t n, uint32_t h) {
  for (; i + 4 <= n; i += 4) h = rotl32(h + ld32u(p + i) * P32_3, 17) * P32_4;
  for (; i < n; ++i) h = rotl32(h + uint32_t(p[i]) * P32_5, 11) * P32_1;
  h ^= h >> 15;
  h *= P32_2;
  h ^= h >> 13;
  h *= P32_3;
  return h ^ (h >> 16);
}

__device__ uint64_t xxh64_tail(const uint8_t* p, uint64_t i, uint64_t n, uint64_t h) {
  for (; i + 8 <= n; i += 8) {
    h ^= round64(0, ld64u(p + i));
    h = rotl64(h, 27) * P64_1 + P64_4;
  }
  if (i + 4 <= n) {
    h ^= uint64_t(ld32u(p + i)) * P64_1;
    h = rotl64(h, 23) * P64_2 + P64_3;
    i += 4;
  }
  for (; i < n; ++i) {
    h ^= uint64_t(p[i]) * P64_5;
    h = rotl64(h, 11) * P64_1;
  }
  return avalanche64(h);
}

// ---- XXH3 pieces -----------------------------------------------------------------------------
__device__ __forceinline__ uint64_t avalanche3(uint64_t h) {
  h ^= h >> 37;
  h *= PMX1;
  return h ^ (h >> 32);
}
__device__ __forceinline__ uint64_t rrmxmx(uint64_t h, uint64_t n) {
  h ^= rotl64(h, 49) ^ rotl64(h, 24);
  h *= PMX2;
  h ^= (h >> 35) + n;
  h *= PMX2;
  return h ^ (h >> 28);
}
__device__ __forceinline__ uint64_t mix16(const uint8_t* p, const uint8_t* s, int off,
                                          uint64_t seed) {
  return fold64(ld64u(p) ^ (sec64(s, off) + seed), ld64u(p + 8) ^ (sec64(s, off + 8) - seed));
}

// XXH3 64-bit, inputs of at most 240 bytes (default secret, seed applied inline).
__device__ uint64_t xxh3_64_short(const uint8_t* p, uint64_t n, uint64_t seed) {
  const uint8_t* k = kSecret;
  if (n <= 16) {
    if (n > 8) {
      const uint64_t lo = ld64u(p) ^ ((sec64(k, 24) ^ sec64(k, 32)) + seed);
      const uint64_t hi = ld64u(p + n - 8) ^ ((sec64(k, 40) ^ sec64(k, 48)) - seed);
      return avalanche3(n + swap64(lo) + hi + fold64(lo, hi));
    }
    if (n >= 4) {
      const uint64_t s = seed ^ (uint64_t(swap32(uint32_t(seed))) << 32);
      const uint64_t x = (uint64_t(ld32u(p + n - 4)) + (uint64_t(ld32u(p)) << 32)) ^
                         ((sec64(k, 8) ^ sec64(k, 16)) - s);
      return rrmxmx(x, n);
    }
    if (n > 0) {
      const uint32_t c = (uint32_t(p[0]) << 16) | (uint32_t(p[n >> 1]) << 24) |
                         uint32_t(p[n - 1]) | (uint32_t(n) << 8);
      return avalanche64(uint64_t(c) ^ (uint64_t(sec32(k, 0) ^ sec32(k, 4)) + seed));
    }
    return avalanche64(seed ^ sec64(k, 56) ^ sec64(k, 64));
  }
  uint64_t acc = n * P64_1;
  if (n <= 128) {
    if (n > 32) {
      if (n > 64) {
        if (n > 96) acc += mix16(p + 48, k, 96, seed) + mix16(p + n - 64, k, 112, seed);
        acc += mix16(p + 32, k, 64, seed) + mix16(p + n - 48, k, 80, seed);
      }
      acc += mix16(p + 16, k, 32, seed) + mix16(p + n - 32, k, 48, seed);
    }
    acc += mix16(p, k, 0, seed) + mix16(p + n - 16, k, 16, seed);
    return avalanche3(acc);
  }
  for (int i = 0; i < 8; ++i) acc += mix16(p + 16 * i, k, 16 * i, seed);
  acc = avalanche3(acc);
  const int rounds = int(n / 16);
  for (int i = 8; i < rounds; ++i) acc += mix16(p + 16 * i, k, 16 * (i - 8) + 3, seed);
  acc += mix16(p + n - 16, k, 136 - 17, seed);
  return avalanche3(acc);
}

struct U128 {
  uint64_t lo, hi;
};

__device__ __forceinline__ void mix32(U128& a, const uint8_t* p1, const uint8_t* p2,
                                      const uint8_t* s, int off, uint64_t seed) {
  a.lo += mix16(p1, s, off, seed);
  a.lo ^= ld64u(p2) + ld64u(p2 + 8);
  a.hi += mix16(p2, s, off + 16, seed);
  a.hi ^= ld64u(p1) + ld64u(p1 + 8);
}

// XXH3 128-bit, inputs of at most 240 bytes.
__device__ U128 xxh3_128_short(const uint8_t* p, uint64_t n, uint64_t seed) {
  const uint8_t* k = kSecret;
  if (n <= 16) {
    if (n > 8) {
      const uint64_t bfl = (sec64(k, 32) ^ sec64(k, 40)) - seed;
      const uint64_t bfh = (sec64(k, 48) ^ sec64(k, 56)) + seed;
      const uint64_t ilo = ld64u(p);
      uint64_t ihi = ld64u(p + n - 8);
      const uint64_t m = ilo ^ ihi ^ bfl;
      uint64_t mlo = m * P64_1, mhi = __umul64hi(m, P64_1);
      mlo += uint64_t(n - 1) << 54;
      ihi ^= bfh;
      mhi += ihi + uint64_t(uint32_t(ihi)) * uint64_t(P32_2 - 1);
      mlo ^= swap64(mhi);
      const uint64_t hlo = mlo * P64_2;
      const uint64_t hhi = __umul64hi(mlo, P64_2) + mhi * P64_2;
      return {avalanche3(hlo), avalanche3(hhi)};
    }
    if (n >= 4) {
      const uint64_t s = seed ^ (uint64_t(swap32(uint32_t(seed))) << 32);
      const uint64_t x = (uint64_t(ld32u(p)) + (uint64_t(ld32u(p + n - 4)) << 32)) ^
                         ((sec64(k, 16) ^ sec64(k, 24)) + s);
      const uint64_t mul = P64_1 + (n << 2);
      uint64_t mlo = x * mul, mhi = __umul64hi(x, mul);
      mhi += mlo << 1;
      mlo ^= mhi >> 3;
      mlo ^= mlo >> 35;
      mlo *= PMX2;
      mlo ^= mlo >> 28;
      return {mlo, avalanche3(mhi)};
    }
    if (n > 0) {
      const uint32_t cl = (uint32_t(p[0]) << 16) | (uint32_t(p[n >> 1]) << 24) |
                          uint32_t(p[n - 1]) | (uint32_t(n) << 8);
      const uint32_t ch = rotl32(swap32(cl), 13);
      const uint64_t lo = uint64_t(cl) ^ (uint64_t(sec32(k, 0) ^ sec32(k, 4)) + seed);
      const uint64_t hi = uint64_t(ch) ^ (uint64_t(sec32(k, 8) ^ sec32(k, 12)) - seed);
      return {avalanche64(lo), avalanche64(hi)};
    }
    return {avalanche64(seed ^ sec64(k, 64) ^ sec64(k, 72)),
            avalanche64(seed ^ sec64(k, 80) ^ sec64(k, 88))};
  }
  U128 a = {n * P64_1, 0};
  if (n <= 128) {
    if (n > 32) {
      if (n > 64) {
        if (n > 96) mix32(a, p + 48, p + n - 64, k, 96, seed);
        mix32(a, p + 32, p + n - 48, k, 64, seed);
      }
      mix32(a, p + 16, p + n - 32, k, 32, seed);
    }
    mix32(a, p, p + n - 16, k, 0, seed);
  } else {
    for (int i = 0; i < 4; ++i) mix32(a, p + 32 * i, p + 32 * i + 16, k, 32 * i, seed);
    a.lo = avalanche3(a.lo);
    a.hi = avalanche3(a.hi);
    const int rounds = int(n / 32);
    for (int i = 4; i < rounds; ++i)
      mix32(a, p + 32 * i, p + 32 * i + 16, k, 3 + 32 * (i - 4), seed);
    mix32(a, p + n - 16, p + n - 32, k, 136 - 17 - 16, uint64_t(0) - seed);
  }
  const uint64_t rlo = a.lo + a.hi;
  const uint64_t rhi = a.lo * P64_1 + a.hi * P64_4 + (n - seed) * P64_2;
  return {avalanche3(rlo), uint64_t(0) - avalanche3(rhi)};
}

__device__ __forceinline__ uint64_t long_blocks(uint64_t n) { return (n - 1) / kBlockBytes; }

__device__ __forceinline__ bool xxh3_algo(int algo) {
  return algo == MDSX_HASH_XXH3_64 || algo == MDSX_HASH_XXH3_128;
}

// ---- kernels ---------------------------------------------------------------------------------
// Per-segment block / chunk prefixes, range checks and the largest chunk count (one workgroup).
__global__ __launch_bounds__(kSumsBlock) void hash_prep_kernel(const HashArgs a) {
  __shared__ uint64_t s_blk[kSumsBlock], s_chk[kSumsBlock];
  __shared__ uint64_t s_base[3];
  if (threadIdx.x == 0) s_base[0] = s_base[1] = s_base[2] = 0;
  __syncthreads();
  for (int base = 0; base < a.nseg; base += kSumsBlock) {
    const int s = base + int(threadIdx.x);
    uint64_t nb = 0;
    if (s < a.nseg) {
      const mdsx_segment g = a.segs[s];
      if (g.offset > a.data_bytes || g.bytes > a.data_bytes - g.offset || (g.offset & 15)) {
        report(a.status, MDSX_E_BOUNDS, s, -1, -1);
      } else if (xxh3_algo(a.algo) && g.bytes > 240) {
        nb = long_blocks(g.bytes);
      }
    }
    const uint64_t nc = (nb + kChunkBlocks - 1) / kChunkBlocks;
    if (nc) atomicMax(reinterpret_cast<unsigned long long*>(&s_base[2]),
                      static_cast<unsigned long long>(nc));
    s_blk[threadIdx.x] = nb;
    s_chk[threadIdx.x] = nc;
    __syncthreads();
    // Hillis-Steele inclusive scan of both (256 entries).
    for (int d = 1; d < kSumsBlock; d <<= 1) {
      const uint64_t b = threadIdx.x >= unsigned(d) ? s_blk[threadIdx.x - d] : 0;
      const uint64_t c = threadIdx.x >= unsigned(d) ? s_chk[threadIdx.x - d] : 0;
      __syncthreads();
      s_blk[threadIdx.x] += b;
      s_chk[threadIdx.x] += c;
      __syncthreads();
    }
    if (s < a.nseg) {
      a.block0[s] = s_base[0] + s_blk[threadIdx.x] - nb;
      a.chunk0[s] = s_base[1] + s_chk[threadIdx.x] - nc;
    }
    __syncthreads();
    if (threadIdx.x == kSumsBlock - 1) {
      s_base[0] += s_blk[threadIdx.x];
      s_base[1] += s_chk[threadIdx.x];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    a.block0[a.nseg] = s_base[0];
    a.chunk0[a.nseg] = s_base[1];
    a.chunk0[a.nseg + 1] = s_base[2];  // largest per-segment chunk count
    if (s_base[0] > a.sums_capacity || s_base[1] > a.flags_capacity)
      report(a.status, MDSX_E_CAPACITY, -1, -1, -1);
  }
}

// Block sums of one 128-block chunk (see the file comment). Lane l of a wave owns block l/8 of an
// 8-block group, stripes 2j + h (h = bit 2 of l) and accumulators 2q, 2q+1 (q = l & 3):
// instruction j reads 128 contiguous bytes per 8 lanes. k0/k1: the lane's secret words.
template <bool kPublish>
__device__ __forceinline__ void sums_chunk(const HashArgs& a, int seg, uint64_t c, int wave,
                                           int lane, const uint64_t* k0, const uint64_t* k1) {
  const int h = (lane >> 2) & 1, q = lane & 3;
  const uint64_t nb = a.block0[seg + 1] - a.block0[seg];
  const uint64_t cb = c * kChunkBlocks;  // first block of the chunk
  const uint8_t* base = a.data + a.segs[seg].offset;
  uint64_t* out = a.sums + a.block0[seg] * 8;
#pragma unroll 1
  for (int it = 0; it < kChunkBlocks / 32; ++it) {
    const uint64_t blk = cb + uint64_t(it * 32 + wave * 8 + (lane >> 3));
    const bool live = blk < nb;
    const uint4* src = reinterpret_cast<const uint4*>(base + blk * kBlockBytes + 16 * (lane & 7));
    uint4 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = live ? ld16<true>(src + 8 * j) : make_uint4(0, 0, 0, 0);
    uint64_t a0 = 0, a1 = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint64_t w0 = uint64_t(v[j].x) | (uint64_t(v[j].y) << 32);
      const uint64_t w1 = uint64_t(v[j].z) | (uint64_t(v[j].w) << 32);
      const uint64_t d0 = w0 ^ k0[j], d1 = w1 ^ k1[j];
      a0 += w1 + uint64_t(uint32_t(d0)) * (d0 >> 32);
      a1 += w0 + uint64_t(uint32_t(d1)) * (d1 >> 32);
    }
    a0 += __shfl_xor(a0, 4);
    a1 += __shfl_xor(a1, 4);
    if (live && h == 0) {
      gu64* dst = (gu64*)(out + blk * 8 + 2 * q);
      if constexpr (kPublish) {  // write-through (sc1): visible to every XCD once drained
        __hip_atomic_store(dst, a0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(dst + 1, a1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        ulonglong2 r;
        r.x = a0;
        r.y = a1;
        *reinterpret_cast<ulonglong2*>(out + blk * 8 + 2 * q) = r;
      }
    }
  }
}

// Which CU this workgroup runs on (XCC, SE, SH, CU fields of HW_REG_XCC_ID / HW_REG_HW_ID), + 1.
__device__ __forceinline__ uint32_t cu_key() {
  const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));    // HW_REG_HW_ID, 32 bits
  const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (3 << 11));   // HW_REG_XCC_ID, 4 bits
  return ((xcc << 16) | (hw & 0xFF00u)) + 1u;
}

// The sums role: chunks in segment-interleaved order (chunk c of every segment before chunk
// c + 1 of any), so that every segment's chain can advance while the stream runs. Two-launch
// form: grid-stride. Fused form: a ticket counter hands out the chunks, and a workgroup that
// finds a chain workgroup on its CU leaves at once (the chain's dependent multiplies then own
// their SIMDs; placement is observed, never relied on for correctness).
template <bool kPublish>
__device__ void sums_role(const HashArgs& a, uint64_t first, uint64_t stride, int nchain) {
  __shared__ uint64_t s_sec[kSecretBytes / 8];
  __shared__ uint64_t s_ticket;
  __shared__ int s_leave;
  if (threadIdx.x < kSecretBytes / 8) s_sec[threadIdx.x] = a.secret[threadIdx.x];
  if constexpr (kPublish) {
    if (threadIdx.x == 0) {
      const uint32_t me = cu_key();
      int leave = 0;
      for (int i = 0; i < nchain; ++i)
        leave |= __hip_atomic_load((gu32*)(a.ctrl + 1 + i), __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT) == me;
      s_leave = leave;
      s_ticket = leave ? ~uint64_t(0)
                       : __hip_atomic_fetch_add((gu32*)a.ctrl, 1u, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  __syncthreads();
  if (a.status->code != 0) return;
  const int lane = int(threadIdx.x & 63), wave = int(threadIdx.x >> 6);
  const int h = (lane >> 2) & 1, q = lane & 3;
  uint64_t k0[8], k1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    k0[j] = s_sec[2 * j + h + 2 * q];  // stripe s = 2j + h reads secret words s + 2q, s + 2q + 1
    k1[j] = s_sec[2 * j + h + 2 * q + 1];
  }
  const uint64_t virt = a.chunk0[a.nseg + 1] * uint64_t(a.nseg);
  uint64_t v = kPublish ? s_ticket : first;
  while (v < virt) {
    uint64_t next = v + stride;
    if constexpr (kPublish) {
      __syncthreads();  // everyone has read s_ticket
      if (threadIdx.x == 0) {
        s_ticket = s_leave ? ~uint64_t(0)
                           : __hip_atomic_fetch_add((gu32*)a.ctrl, 1u, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    const int seg = int(v % uint64_t(a.nseg));
    const uint64_t c = v / uint64_t(a.nseg);
    if (c < a.chunk0[seg + 1] - a.chunk0[seg]) {
      sums_chunk<kPublish>(a, seg, c, wave, lane, k0, k1);
      if constexpr (kPublish) {
        // MI355X_MICROARCH.md visibility recipe R1: every storing wave drains its sc1 stores,
        // then ONE lane stores the chunk's flag (agent-scope relaxed = sc1).
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0)
          __hip_atomic_store((gu32*)(a.flags + a.chunk0[seg] + c), 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if constexpr (kPublish) {
      __syncthreads();
      next = s_ticket;
    }
    v = next;
  }
}

__global__ __launch_bounds__(kSumsBlock) void xxh3_sums_kernel(const HashArgs a) {
  sums_role<false>(a, blockIdx.x, gridDim.x, 0);
}

// One link of the chain: scramble(acc + sum) = ((x ^ (x >> 47)) ^ key) * PRIME32_1, x = acc + sum.
// (The compiler folds the next link's sum into the 32x32+64 multiply-add: two v_mad_u64_u32 per
// link, ~21-24 ns per link measured by scripts/microbench/chain_latency.hip.)
__device__ __forceinline__ uint64_t scramble_step(uint64_t acc, uint64_t sum, uint64_t key) {
  uint64_t x = acc + sum;
  x ^= x >> 47;
  x ^= key;
  return x * P32_1;
}

// acc = scramble(acc + S_b) over blocks [0, nb) of one accumulator lane. Loads of the block sums
// run 16 blocks ahead of the dependent chain (double buffer). kWait: wait for each chunk's
// published flag (fused kernel) before reading its sums.
template <bool kWait>
__device__ __forceinline__ uint64_t xxh3_chain(const HashArgs& a, int seg, int k) {
  constexpr uint64_t kInit[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
  constexpr int kAhead = kChainAhead;
  uint64_t acc = kInit[k];
  const uint64_t key = a.secret[16 + k];  // secret + 192 - 64: the scramble key
  const uint64_t nb = a.block0[seg + 1] - a.block0[seg];
  const uint64_t* S = a.sums + a.block0[seg] * 8 + k;
  gu32* flag = (gu32*)(a.flags + (kWait ? a.chunk0[seg] : 0));
  // Fused: the sums were stored write-through (sc1) and drained before their chunk's flag, so a
  // relaxed sc1 poll followed by sc1 loads of every sum needs no acquire fence (recipe R1).
  auto wait = [&](uint64_t b) {
    if constexpr (kWait) {
      if (b % kChunkBlocks == 0) {
        while (__hip_atomic_load(flag + b / kChunkBlocks, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT) == 0)
          __builtin_amdgcn_s_sleep(2);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      }
    }
  };
  auto ld = [&](uint64_t b) -> uint64_t {
    if constexpr (kWait)
      return __hip_atomic_load((const gu64*)(S + b * 8), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    else
      return S[b * 8];
  };
  auto steps = [&](const uint64_t* t) {
#pragma unroll
    for (int i = 0; i < kAhead; ++i) {
      acc = scramble_step(acc, t[i], key);
    }
  };
  // Batches of kAhead links; the loads of batch i + 1 are issued before the links of batch i.
  // Every load is unconditional (the sums area has 2 * kAhead blocks of slack at its end, so a
  // batch past this segment's last block reads harmless junk it never uses): the compiler then
  // waits for exactly the older batch, vmcnt(kAhead), instead of draining.
  auto loadb = [&](uint64_t* t, uint64_t b) {
#pragma unroll
    for (int i = 0; i < kAhead; ++i) t[i] = ld(b + i);
    __builtin_amdgcn_sched_barrier(0);  // issue the whole batch before the links that follow
  };
  const uint64_t nfull = nb / kAhead;
  uint64_t t0[kAhead], t1[kAhead];
  if (nfull) {
    wait(0);
    loadb(t0, 0);
  }
  uint64_t i = 0;
  for (; i + 2 <= nfull; i += 2) {
    const uint64_t b = i * kAhead;
    wait(b + kAhead);
    loadb(t1, b + kAhead);
    steps(t0);
    if (i + 2 < nfull) wait(b + 2 * kAhead);
    loadb(t0, b + 2 * kAhead);  // unused junk when i + 2 == nfull
    steps(t1);
  }
  if (i < nfull) steps(t0);
  uint64_t b = nfull * kAhead;
  for (; b < nb; ++b) {
    wait(b);
    acc = scramble_step(acc, ld(b), key);
  }
  return acc;
}

// Secret word at any byte offset from the LDS copy (u64 words).
__device__ __forceinline__ uint64_t sec_at(const uint64_t* s64, int off) {
  const int w = off >> 3, r = (off & 7) * 8;
  return r ? (s64[w] >> r) | (s64[w + 1] << (64 - r)) : s64[w];
}

// Tail of a long XXH3 input, 8 lanes per segment (lane k = accumulator k, all lanes of the wave
// take part in the shuffles): the stripes of the partial last block and the last stripe are
// accumulated (acc[k] += v[k ^ 1] + lo(v[k] ^ key[k]) * hi(...)), then the accumulators are
// merged (mix2Accs over lane pairs, summed over the 4 pairs). Returns the 64-bit digest in every
// lane of the group; hi128 gets the high half for XXH3-128.
__device__ __forceinline__ uint64_t xxh3_long_tail(uint64_t acc, int k, bool live,
                                                   const uint8_t* p, uint64_t n,
                                                   const uint64_t* s64, bool want128,
                                                   uint64_t& hi128) {
  if (live) {
    const uint64_t nb = long_blocks(n);
    const int stripes = int(((n - 1) - kBlockBytes * nb) / kStripe);
    const uint64_t* tail = reinterpret_cast<const uint64_t*>(p + nb * kBlockBytes);
    uint64_t v[16], vx[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j < stripes) {
        v[j] = tail[8 * j + k];
        vx[j] = tail[8 * j + (k ^ 1)];
      }
    }
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (j < stripes) {
        const uint64_t dk = v[j] ^ s64[j + k];  // secret + 8j, word k
        acc += vx[j] + uint64_t(uint32_t(dk)) * (dk >> 32);
      }
    }
    const uint8_t* last = p + n - kStripe;
    const uint64_t lv = ld64u(last + 8 * k), lx = ld64u(last + 8 * (k ^ 1));
    const uint64_t dk = lv ^ sec_at(s64, kSecretBytes - kStripe - 7 + 8 * k);
    acc += lx + uint64_t(uint32_t(dk)) * (dk >> 32);
  }
  auto merge = [&](int off, uint64_t start) {
    const uint64_t m = acc ^ sec_at(s64, off + 8 * k);
    const uint64_t other = __shfl_xor(m, 1);
    uint64_t r = (k & 1) ? 0 : fold64(m, other);
    r += __shfl_xor(r, 2);
    r += __shfl_xor(r, 4);
    return avalanche3(start + r);
  };
  const uint64_t lo = merge(11, n * P64_1);
  if (want128) hi128 = merge(kSecretBytes - 64 - 11, ~(n * P64_2));
  return lo;
}

// The chain role: 8 lanes (accumulators) per segment, 8 segments per workgroup, run by its first
// wave alone (one chain wave per CU: measured 1.5x faster than four on one CU).
template <bool kWait>
__device__ void chain_role(const HashArgs& a, int group) {
  __shared__ uint64_t s_sec64[kSecretBytes / 8 + 1];
  const int t = int(threadIdx.x);
  if constexpr (kWait) {
    if (t == 0)
      __hip_atomic_store((gu32*)(a.ctrl + 1 + group), cu_key(), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  if (t < kSecretBytes / 8) s_sec64[t] = a.secret[t];
  if (t == kSecretBytes / 8) s_sec64[t] = 0;
  __syncthreads();
  if (t >= 64) return;
  __builtin_amdgcn_s_setprio(3);  // the dependent chain first when it shares a SIMD with streams
  const int ls = t >> 3, k = t & 7;
  const int seg = group * kChainSegs + ls;
  const bool ok = a.status->code == 0 && seg < a.nseg;
  const uint64_t n = ok ? a.segs[seg].bytes : 0;
  const uint8_t* p = ok ? a.data + a.segs[seg].offset : a.data;
  const bool lng = ok && n > 240;
  uint64_t acc = 0;
  if (lng) acc = xxh3_chain<kWait>(a, seg, k);
  uint64_t hi = 0;
  const uint64_t lo = xxh3_long_tail(acc, k, lng, p, n, s_sec64,
                                     a.algo == MDSX_HASH_XXH3_128, hi);
  if (!ok || k != 0) return;
  if (lng) {
    a.digests[2 * seg] = lo;
    a.digests[2 * seg + 1] = hi;
  } else if (a.algo == MDSX_HASH_XXH3_128) {
    const U128 r = xxh3_128_short(p, n, a.seed);
    a.digests[2 * seg] = r.lo;
    a.digests[2 * seg + 1] = r.hi;
  } else {
    a.digests[2 * seg] = xxh3_64_short(p, n, a.seed);
    a.digests[2 * seg + 1] = 0;
  }
}

__global__ __launch_bounds__(kSumsBlock) void xxh3_finish_kernel(const HashArgs a) {
  chain_role<false>(a, int(blockIdx.x));
}

// Sums and chains in one launch: workgroups [0, nchain) run the chains of 32 segments each and
// wait on per-chunk flags; the rest stream the block sums and publish each finished chunk.
__global__ __launch_bounds__(kSumsBlock) void xxh3_fused_kernel(const HashArgs a, int nchain) {
  if (int(blockIdx.x) < nchain)
    chain_role<true>(a, int(blockIdx.x));
  else
    sums_role<true>(a, 0, 0, nchain);
}

// XXH32 / XXH64: 4 lanes per segment run the 4 accumulator chains out of LDS windows that the
// whole wave streams in (double-buffered, 4 KiB per segment per window: the next window's loads
// are in flight for the ~128 dependent steps of the current one); lane 0 merges + tail.
template <bool k64>
__global__ __launch_bounds__(64) void xxh_seq_kernel(const HashArgs a) {
  constexpr int kWin = 4096;  // bytes per segment per window
  constexpr int kChunks = kSeqPerWave * kWin / 16 / 64;  // 16-byte loads per lane per window
  constexpr uint64_t kStripeBytes = k64 ? 32 : 16;
  __shared__ uint4 s_win[2][kSeqPerWave][kWin / 16];
  __shared__ uint64_t s_v[kSeqPerWave][4];
  const int lane = int(threadIdx.x);
  const int ls = lane >> 2, k = lane & 3;  // compute lanes: ls < kSeqPerWave
  const int seg0 = int(blockIdx.x) * kSeqPerWave;
  if (a.status->code != 0) return;
  // per-segment body (whole stripes) of the wave's segments
  uint64_t body[kSeqPerWave];
  const uint8_t* base[kSeqPerWave];
  uint64_t nwin = 0;
#pragma unroll
  for (int i = 0; i < kSeqPerWave; ++i) {
    const int s = seg0 + i;
    body[i] = 0;
    base[i] = a.data;
    if (s < a.nseg) {
      body[i] = a.segs[s].bytes / kStripeBytes * kStripeBytes;
      base[i] = a.data + a.segs[s].offset;
    }
    nwin = max(nwin, (body[i] + kWin - 1) / kWin);
  }
  auto fetch = [&](uint4* r, uint64_t w) {
#pragma unroll
    for (int c = 0; c < kChunks; ++c) {
      const int L = c * 64 + lane;
      const int i = L / (kWin / 16);
      const uint64_t off = w * kWin + uint64_t(L % (kWin / 16)) * 16;
      r[c] = off < body[i] ? ld16<true>(reinterpret_cast<const uint4*>(base[i] + off))
                           : make_uint4(0, 0, 0, 0);
    }
  };
  auto stash = [&](const uint4* r, int buf) {
#pragma unroll
    for (int c = 0; c < kChunks; ++c) {
      const int L = c * 64 + lane;
      s_win[buf][L / (kWin / 16)][L % (kWin / 16)] = r[c];
    }
  };
  const uint64_t seed = a.seed;
  uint64_t v64 = k == 0 ? seed + P64_1 + P64_2 : k == 1 ? seed + P64_2 : k == 2 ? seed
                                                                               : seed - P64_1;
  const uint32_t s32 = uint32_t(seed);
  uint32_t v32 = k == 0 ? s32 + P32_1 + P32_2 : k == 1 ? s32 + P32_2 : k == 2 ? s32
                                                                            : s32 - P32_1;
  const uint64_t mybody = ls < kSeqPerWave ? body[ls] : 0;
  uint4 r[kChunks];
  if (nwin) {
    fetch(r, 0);
    stash(r, 0);
  }
  __syncthreads();
  for (uint64_t w = 0; w < nwin; ++w) {
    if (w + 1 < nwin) fetch(r, w + 1);
    const uint64_t lo = w * kWin;
    if (lo < mybody) {
      const int steps = int(min(uint64_t(kWin), mybody - lo) / kStripeBytes);
      const uint8_t* win = reinterpret_cast<const uint8_t*>(s_win[w & 1][ls]);
      // The chain's inputs are read from LDS 16 at a time ahead of the dependent rounds (and
      // their lane * PRIME products formed off the chain).
      constexpr int kBatch = 16;
      int i = 0;
      if constexpr (k64) {
        const uint64_t* src = reinterpret_cast<const uint64_t*>(win) + k;
        for (; i + kBatch <= steps; i += kBatch) {
          uint64_t t[kBatch];
#pragma unroll
          for (int j = 0; j < kBatch; ++j) t[j] = src[4 * (i + j)] * P64_2;
#pragma unroll
          for (int j = 0; j < kBatch; ++j) v64 = rotl64(v64 + t[j], 31) * P64_1;
        }
        for (; i < steps; ++i) v64 = round64(v64, src[4 * i]);
      } else {
        const uint32_t* src = reinterpret_cast<const uint32_t*>(win) + k;
        for (; i + kBatch <= steps; i += kBatch) {
          uint32_t t[kBatch];
#pragma unroll
          for (int j = 0; j < kBatch; ++j) t[j] = src[4 * (i + j)] * P32_2;
#pragma unroll
          for (int j = 0; j < kBatch; ++j) v32 = rotl32(v32 + t[j], 13) * P32_1;
        }
        for (; i < steps; ++i) v32 = round32(v32, src[4 * i]);
      }
    }
    __syncthreads();  // every lane is done with buffer (w + 1) & 1's previous window
    if (w + 1 < nwin) stash(r, int((w + 1) & 1));
    __syncthreads();
  }
  if (ls < kSeqPerWave) s_v[ls][k] = k64 ? v64 : uint64_t(v32);
  __syncthreads();
  const int seg = seg0 + ls;
  if (ls >= kSeqPerWave || k != 0 || seg >= a.nseg) return;
  const uint64_t n = a.segs[seg].bytes;
  const uint8_t* p = a.data + a.segs[seg].offset;
  const uint64_t stripes = n / kStripeBytes;
  uint64_t out;
  if constexpr (k64) {
    uint64_t h;
    if (stripes > 0) {
      const uint64_t v0 = s_v[ls][0], v1 = s_v[ls][1], v2 = s_v[ls][2], v3 = s_v[ls][3];
      h = rotl64(v0, 1) + rotl64(v1, 7) + rotl64(v2, 12) + rotl64(v3, 18);
      const uint64_t vs[4] = {v0, v1, v2, v3};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        h ^= round64(0, vs[i]);
        h = h * P64_1 + P64_4;
      }
    } else {
      h = a.seed + P64_5;
    }
    out = xxh64_tail(p, stripes * kStripeBytes, n, h + n);
  } else {
    uint32_t h;
    if (stripes > 0) {
      h = rotl32(uint32_t(s_v[ls][0]), 1) + rotl32(uint32_t(s_v[ls][1]), 7) +
          rotl32(uint32_t(s_v[ls][2]), 12) + rotl32(uint32_t(s_v[ls][3]), 18);
    } else {
      h = uint32_t(a.seed) + P32_5;
    }
    out = xxh32_tail(p, stripes * kStripeBytes, n, h + uint32_t(n));
  }
  a.digests[2 * seg] = out;
  a.digests[2 * seg + 1] = 0;
}

uint64_t align256(uint64_t x) { return (x + 255) & ~uint64_t(255); }

struct HashLayout {
  uint64_t block0, chunk0, ctrl, flags, sums, total;
};

// status | block0[nseg + 1] | chunk0[nseg + 2] | ctrl[1 + chain workgroups] | flags[chunks] |
// sums[blocks][8]
HashLayout hash_layout(int nseg, uint64_t total_bytes) {
  const uint64_t blocks = total_bytes / kBlockBytes;
  const uint64_t chunks = blocks / kChunkBlocks + uint64_t(nseg);
  HashLayout l;
  l.block0 = align256(sizeof(mdsx_status));
  l.chunk0 = l.block0 + align256(uint64_t(nseg + 1) * 8);
  l.ctrl = l.chunk0 + align256(uint64_t(nseg + 2) * 8);
  l.flags = l.ctrl + align256(4 * (1 + uint64_t(nseg + kChainSegs - 1) / kChainSegs));
  l.sums = l.flags + align256(chunks * 4);
  l.total = l.sums + align256((blocks + 2 * kChainAhead) * 64);  // + slack for the chain's loads
  return l;
}

// MDSX_HASH_FUSED=0|1 (measurement knob): XXH3 sums and chains in one launch (default) or two.
bool hash_fused() {
  const char* env = std::getenv("MDSX_HASH_FUSED");
  return env ? std::atoi(env) != 0 : true;
}

}  // namespace
}  // namespace mdsx_kernels

using namespace mdsx_kernels;

extern "C" {

uint64_t mdsx_hash_workspace_bytes(int nseg, uint64_t total_segment_bytes) {
  if (nseg < 0) return 0;
  return hash_layout(nseg, total_segment_bytes).total;
}

int mdsx_hash_segments(int algo, uint64_t seed, const uint8_t* data, uint64_t data_bytes,
                       const mdsx_segment* d_segs, int nseg, uint64_t* d_digests,
                       void* d_workspace, uint64_t workspace_bytes, void* stream) {
  if (algo < MDSX_HASH_XXH32 || algo > MDSX_HASH_XXH3_128)
    return mdsx::fail(MDSX_E_ARG, "mdsx_hash_segments: unknown algorithm id");
  if (nseg < 0 || (nseg > 0 && (!data || !d_segs || !d_digests || !d_workspace)))
    return mdsx::fail(MDSX_E_ARG, "mdsx_hash_segments: null argument");
  if (reinterpret_cast<uint64_t>(data) & 15)
    return mdsx::fail(MDSX_E_ARG, "mdsx_hash_segments: data must be 16-byte aligned");
  // the flag area is sized for the segments' total length, recovered from the workspace size
  HashLayout l0 = hash_layout(nseg, 0);
  if (workspace_bytes < l0.total)
    return mdsx::fail(MDSX_E_ARG, "mdsx_hash_segments: workspace smaller than "
                                  "mdsx_hash_workspace_bytes(nseg, 0)");
  hipStream_t s = static_cast<hipStream_t>(stream);
  int rc = hip_check(hipMemsetAsync(d_workspace, 0, sizeof(mdsx_status), s), "hipMemsetAsync");
  if (rc || nseg == 0) return rc;
  uint8_t* ws = static_cast<uint8_t*>(d_workspace);
  HashArgs a;
  std::memset(&a, 0, sizeof(a));
  a.data = data;
  a.data_bytes = data_bytes;
  a.segs = d_segs;
  a.digests = d_digests;
  a.status = reinterpret_cast<mdsx_status*>(ws);
  a.block0 = reinterpret_cast<uint64_t*>(ws + l0.block0);
  a.chunk0 = reinterpret_cast<uint64_t*>(ws + l0.chunk0);
  // Largest total length this workspace was sized for: flags and sums grow together.
  uint64_t lo_b = 0, hi_b = (workspace_bytes / 64 + 2) * kBlockBytes;
  while (lo_b < hi_b) {
    const uint64_t mid = (lo_b + hi_b + 1) / 2;
    if (hash_layout(nseg, mid).total <= workspace_bytes) lo_b = mid; else hi_b = mid - 1;
  }
  l0 = hash_layout(nseg, lo_b);
  a.ctrl = reinterpret_cast<uint32_t*>(ws + l0.ctrl);
  a.flags = reinterpret_cast<uint32_t*>(ws + l0.flags);
  a.sums = reinterpret_cast<uint64_t*>(ws + l0.sums);
  a.flags_capacity = (l0.sums - l0.flags) / 4;
  a.sums_capacity = (workspace_bytes - l0.sums) / 64 - 2 * kChainAhead;
  a.seed = seed;
  a.nseg = nseg;
  a.algo = algo;
  // Secret of long XXH3 inputs: XXH3_initCustomSecret (the default secret when seed == 0).
  const uint8_t* k = kSecretHost;
  for (int i = 0; i < kSecretBytes / 16; ++i) {
    uint64_t lo, hi;
    std::memcpy(&lo, k + 16 * i, 8);
    std::memcpy(&hi, k + 16 * i + 8, 8);
    a.secret[2 * i] = lo + seed;
    a.secret[2 * i + 1] = hi - seed;
  }
  hipLaunchKernelGGL(hash_prep_kernel, dim3(1), dim3(kSumsBlock), 0, s, a);
  rc = hip_check(hipGetLastError(), "hash_prep_kernel launch");
  if (rc) return rc;
  if (algo == MDSX_HASH_XXH3_64 || algo == MDSX_HASH_XXH3_128) {
    const int nchain = (nseg + kChainSegs - 1) / kChainSegs;
    // Fused only while the waiting chain workgroups are few: they spin on flags, and the streams
    // that set them must always find room on the chip (at most kFusedMaxChain of its >= 2048
    // workgroup slots and CUs are ever held by chains). Above that, two launches.
    if (hash_fused() && nchain <= kFusedMaxChain) {
      rc = hip_check(hipMemsetAsync(a.ctrl, 0, l0.sums - l0.ctrl, s), "hipMemsetAsync");
      if (rc) return rc;
      hipLaunchKernelGGL(xxh3_fused_kernel, dim3(nchain + kSumsGridMax), dim3(kSumsBlock), 0, s,
                         a, nchain);
      return hip_check(hipGetLastError(), "xxh3_fused_kernel launch");
    }
    hipLaunchKernelGGL(xxh3_sums_kernel, dim3(kSumsGridMax), dim3(kSumsBlock), 0, s, a);
    rc = hip_check(hipGetLastError(), "xxh3_sums_kernel launch");
    if (rc) return rc;
    hipLaunchKernelGGL(xxh3_finish_kernel, dim3(nchain), dim3(kSumsBlock), 0, s, a);
    return hip_check(hipGetLastError(), "xxh3_finish_kernel launch");
  }
  const dim3 grid((nseg + kSeqPerWave - 1) / kSeqPerWave);
  if (algo == MDSX_HASH_XXH64)
    hipLaunchKernelGGL(xxh_seq_kernel<true>, grid, dim3(64), 0, s, a);
  else
    hipLaunchKernelGGL(xxh_seq_kernel<false>, grid, dim3(64), 0, s, a);
  return hip_check(hipGetLastError(), "xxh_seq_kernel launch");
}

}  // extern "C"
