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
//   xxh_finish_kernel  8 lanes per segment (one per accumulator) run the short dependent chain
//                      acc = scramble(acc + S_b) over the block sums (loads issued 16 blocks
//                      ahead), then one lane per segment hashes the tail (partial block, last
//                      stripe), merges the accumulators and writes the digest. Inputs <= 240
//                      bytes take the short paths in the same lane.
// XXH64 / XXH32 are one dependent chain per accumulator (4 lanes per segment, loads issued 8
// stripes ahead): xxh_seq_kernel. They are latency-bound per segment and only pay off over many
// resident shards at once; DESIGN.md reports both.
#include <hip/hip_runtime.h>

#include <cstdint>
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
constexpr int kChunkBlocks = 128;     // blocks per sums-kernel chunk (4 waves x 4 x 8 blocks)
constexpr int kSumsBlock = 256;
constexpr int kSumsGridMax = 256 * 8;  // persistent grid: 8 workgroups per CU
constexpr int kSegPerWave = 8;         // xxh_finish_kernel: 8 lanes (accumulators) per segment
constexpr int kSeqPerWave = 16;        // xxh_seq_kernel: 4 lanes per segment

__constant__ uint8_t kSecret[kSecretBytes] = {MDSX_XXH3_SECRET};
const uint8_t kSecretHost[kSecretBytes] = {MDSX_XXH3_SECRET};

struct HashArgs {
  const uint8_t* data;
  uint64_t data_bytes;
  const mdsx_segment* segs;
  uint64_t* digests;     // 2 x u64 per segment: low 64 bits, high 64 bits (xxh3_128)
  mdsx_status* status;
  uint64_t* sums;        // 8 x u64 per full block of every long XXH3 segment
  uint64_t* block0;      // nseg + 1: prefix of block counts
  uint64_t* chunk0;      // nseg + 1: prefix of 128-block chunk counts
  uint64_t sums_capacity;  // blocks the sums area holds
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

// One stripe of the long loop (any alignment of data and secret offset).
__device__ __forceinline__ void accumulate_stripe(uint64_t* acc, const uint8_t* p,
                                                  const uint8_t* s, int off) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint64_t v = ld64u(p + 8 * k);
    const uint64_t dk = v ^ sec64(s, off + 8 * k);
    acc[k ^ 1] += v;
    acc[k] += uint64_t(uint32_t(dk)) * (dk >> 32);
  }
}

__device__ __forceinline__ uint64_t merge_accs(const uint64_t* acc, const uint8_t* s, int off,
                                               uint64_t start) {
  uint64_t r = start;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    r += fold64(acc[2 * k] ^ sec64(s, off + 16 * k), acc[2 * k + 1] ^ sec64(s, off + 16 * k + 8));
  return avalanche3(r);
}

__device__ __forceinline__ uint64_t long_blocks(uint64_t n) { return (n - 1) / kBlockBytes; }

__device__ __forceinline__ bool xxh3_algo(int algo) {
  return algo == MDSX_HASH_XXH3_64 || algo == MDSX_HASH_XXH3_128;
}

// ---- kernels ---------------------------------------------------------------------------------
// Per-segment block / chunk prefixes and range checks (one workgroup).
__global__ __launch_bounds__(kSumsBlock) void hash_prep_kernel(const HashArgs a) {
  __shared__ uint64_t s_blk[kSumsBlock], s_chk[kSumsBlock];
  __shared__ uint64_t s_base[2];
  if (threadIdx.x == 0) s_base[0] = s_base[1] = 0;
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
    s_blk[threadIdx.x] = nb;
    s_chk[threadIdx.x] = (nb + kChunkBlocks - 1) / kChunkBlocks;
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
    const uint64_t eb = s_base[0] + s_blk[threadIdx.x] - nb;
    const uint64_t ec = s_base[1] + s_chk[threadIdx.x] - (nb + kChunkBlocks - 1) / kChunkBlocks;
    if (s < a.nseg) {
      a.block0[s] = eb;
      a.chunk0[s] = ec;
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
    if (s_base[0] > a.sums_capacity) report(a.status, MDSX_E_CAPACITY, -1, -1, -1);
  }
}

// Block sums of every full block of every long XXH3 segment (see the file comment). Lane l of a
// wave owns block l/8 of an 8-block group, stripes 2j + h (h = bit 2 of l) and accumulators
// 2q, 2q+1 (q = l & 3): instruction j reads 128 contiguous bytes per 8 lanes.
__global__ __launch_bounds__(kSumsBlock) void xxh3_sums_kernel(const HashArgs a) {
  __shared__ uint64_t s_sec[kSecretBytes / 8];
  if (threadIdx.x < kSecretBytes / 8) s_sec[threadIdx.x] = a.secret[threadIdx.x];
  __syncthreads();
  if (a.status->code != 0) return;
  const uint64_t nchunks = a.chunk0[a.nseg];
  const int lane = int(threadIdx.x & 63), wave = int(threadIdx.x >> 6);
  const int h = (lane >> 2) & 1, q = lane & 3;
  // Per-lane keys: stripe s = 2j + h reads secret words s + 2q and s + 2q + 1.
  uint64_t k0[8], k1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    k0[j] = s_sec[2 * j + h + 2 * q];
    k1[j] = s_sec[2 * j + h + 2 * q + 1];
  }
  for (uint64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    // segment owning chunk c: last s with chunk0[s] <= c
    int lo = 0, hi = a.nseg - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.chunk0[mid] <= c) lo = mid; else hi = mid - 1;
    }
    const int seg = lo;
    const uint64_t nb = a.block0[seg + 1] - a.block0[seg];
    const uint64_t cb = (c - a.chunk0[seg]) * kChunkBlocks;  // first block of the chunk
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
        ulonglong2 r;
        r.x = a0;
        r.y = a1;
        *reinterpret_cast<ulonglong2*>(out + blk * 8 + 2 * q) = r;
      }
    }
  }
}

// Long-loop chain + tail + merge for XXH3, short inputs for XXH3: 8 lanes per segment.
__global__ __launch_bounds__(64) void xxh3_finish_kernel(const HashArgs a) {
  __shared__ uint64_t s_sec64[kSecretBytes / 8];
  __shared__ uint64_t s_acc[kSegPerWave][8];
  const int lane = int(threadIdx.x);
  if (lane < kSecretBytes / 8) s_sec64[lane] = a.secret[lane];
  __syncthreads();
  const uint8_t* sec = reinterpret_cast<const uint8_t*>(s_sec64);
  const int ls = lane >> 3, k = lane & 7;
  const int seg = int(blockIdx.x) * kSegPerWave + ls;
  const bool ok = a.status->code == 0 && seg < a.nseg;
  uint64_t n = 0;
  const uint8_t* p = nullptr;
  if (ok) {
    n = a.segs[seg].bytes;
    p = a.data + a.segs[seg].offset;
  }
  if (ok && n > 240) {
    constexpr uint64_t kInit[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
    uint64_t acc = kInit[k];
    const uint64_t key = s_sec64[16 + k];  // secret + 192 - 64 (scramble key)
    const uint64_t nb = a.block0[seg + 1] - a.block0[seg];
    const uint64_t* S = a.sums + a.block0[seg] * 8 + k;
    uint64_t b = 0;
    constexpr int kAhead = 16;
    for (; b + kAhead <= nb; b += kAhead) {
      uint64_t t[kAhead];
#pragma unroll
      for (int i = 0; i < kAhead; ++i) t[i] = __builtin_nontemporal_load(S + (b + i) * 8);
#pragma unroll
      for (int i = 0; i < kAhead; ++i) {
        uint64_t x = acc + t[i];
        x ^= x >> 47;
        x ^= key;
        acc = x * P32_1;
      }
    }
    for (; b < nb; ++b) {
      uint64_t x = acc + S[b * 8];
      x ^= x >> 47;
      x ^= key;
      acc = x * P32_1;
    }
    s_acc[ls][k] = acc;
  }
  __syncthreads();
  if (!ok || k != 0) return;
  uint64_t lo, hi = 0;
  if (n > 240) {
    uint64_t acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = s_acc[ls][i];
    const uint64_t nb = long_blocks(n);
    const uint64_t stripes = ((n - 1) - kBlockBytes * nb) / kStripe;
    for (uint64_t j = 0; j < stripes; ++j)
      accumulate_stripe(acc, p + nb * kBlockBytes + j * kStripe, sec, int(8 * j));
    accumulate_stripe(acc, p + n - kStripe, sec, kSecretBytes - kStripe - 7);
    lo = merge_accs(acc, sec, 11, n * P64_1);
    if (a.algo == MDSX_HASH_XXH3_128)
      hi = merge_accs(acc, sec, kSecretBytes - 64 - 11, ~(n * P64_2));
  } else if (a.algo == MDSX_HASH_XXH3_128) {
    const U128 r = xxh3_128_short(p, n, a.seed);
    lo = r.lo;
    hi = r.hi;
  } else {
    lo = xxh3_64_short(p, n, a.seed);
  }
  a.digests[2 * seg] = lo;
  a.digests[2 * seg + 1] = hi;
}

// XXH32 / XXH64: 4 lanes per segment run the 4 accumulator chains; lane 0 merges + tail.
template <bool k64>
__global__ __launch_bounds__(64) void xxh_seq_kernel(const HashArgs a) {
  __shared__ uint64_t s_v[kSeqPerWave][4];
  const int lane = int(threadIdx.x);
  const int ls = lane >> 2, k = lane & 3;
  const int seg = int(blockIdx.x) * kSeqPerWave + ls;
  const bool ok = a.status->code == 0 && seg < a.nseg;
  uint64_t n = 0;
  const uint8_t* p = nullptr;
  if (ok) {
    n = a.segs[seg].bytes;
    p = a.data + a.segs[seg].offset;
  }
  constexpr uint64_t kStripeBytes = k64 ? 32 : 16;
  const uint64_t stripes = n / kStripeBytes;
  if (ok && stripes > 0) {
    constexpr int kAhead = 8;
    if constexpr (k64) {
      const uint64_t seed = a.seed;
      uint64_t v = k == 0 ? seed + P64_1 + P64_2 : k == 1 ? seed + P64_2 : k == 2 ? seed
                                                                                  : seed - P64_1;
      const uint64_t* src = reinterpret_cast<const uint64_t*>(p) + k;
      uint64_t i = 0;
      for (; i + kAhead <= stripes; i += kAhead) {
        uint64_t t[kAhead];
#pragma unroll
        for (int j = 0; j < kAhead; ++j) t[j] = __builtin_nontemporal_load(src + (i + j) * 4);
#pragma unroll
        for (int j = 0; j < kAhead; ++j) v = round64(v, t[j]);
      }
      for (; i < stripes; ++i) v = round64(v, src[i * 4]);
      s_v[ls][k] = v;
    } else {
      const uint32_t seed = uint32_t(a.seed);
      uint32_t v = k == 0 ? seed + P32_1 + P32_2 : k == 1 ? seed + P32_2 : k == 2 ? seed
                                                                                  : seed - P32_1;
      const uint32_t* src = reinterpret_cast<const uint32_t*>(p) + k;
      uint64_t i = 0;
      for (; i + kAhead <= stripes; i += kAhead) {
        uint32_t t[kAhead];
#pragma unroll
        for (int j = 0; j < kAhead; ++j) t[j] = __builtin_nontemporal_load(src + (i + j) * 4);
#pragma unroll
        for (int j = 0; j < kAhead; ++j) v = round32(v, t[j]);
      }
      for (; i < stripes; ++i) v = round32(v, src[i * 4]);
      s_v[ls][k] = v;
    }
  }
  __syncthreads();
  if (!ok || k != 0) return;
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
  uint64_t block0, chunk0, sums, total;
};

HashLayout hash_layout(int nseg, uint64_t total_bytes) {
  HashLayout l;
  l.block0 = align256(sizeof(mdsx_status));
  l.chunk0 = l.block0 + align256(uint64_t(nseg + 1) * 8);
  l.sums = l.chunk0 + align256(uint64_t(nseg + 1) * 8);
  l.total = l.sums + align256((total_bytes / kBlockBytes) * 64);
  return l;
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
  const HashLayout l0 = hash_layout(nseg, 0);
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
  a.sums = reinterpret_cast<uint64_t*>(ws + l0.sums);
  a.sums_capacity = (workspace_bytes - l0.sums) / 64;
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
    hipLaunchKernelGGL(xxh3_sums_kernel, dim3(kSumsGridMax), dim3(kSumsBlock), 0, s, a);
    rc = hip_check(hipGetLastError(), "xxh3_sums_kernel launch");
    if (rc) return rc;
    hipLaunchKernelGGL(xxh3_finish_kernel, dim3((nseg + kSegPerWave - 1) / kSegPerWave), dim3(64),
                       0, s, a);
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
