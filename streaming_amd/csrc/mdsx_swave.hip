// Ragged plans of long samples, one sample per one-wave workgroup, the sample in registers
// (gfx950): swave_decode_kernel.
//
// The reference decodes one sample per call: MDSReader.get_sample_data reads the sample's byte
// range (streaming/base/format/mds/reader.py:128-149), decode_sample splits it at the u32 size
// heads of the variable columns (mds/reader.py:103-126) and each column's decoder returns its
// value (encodings.py:62-81: bytes / str; 84-94: int; 270-397: ndarray and scalars).
//
// Here a wave takes one sample -- the same unit -- with nothing staged ahead of it:
//   * pass 1 is the register decode's scan (scan_tiles_kernel<true> + the chunk scans): each
//     row's ragged bytes, scanned into scan-block-local offsets (left in the offsets outputs) and
//     scan-block bases (tile_prefix); it also checks each row's offsets pair against the file
//     (mds/reader.py:137-142) and leaves one 16-byte record per sample slot: the sample's first
//     byte in the batch, its size (or idle / bad), its shard and output row. So every wave knows
//     where its sample is and where its ragged values go before it has read a byte of the sample;
//   * the wave requests, together: its record (one load), then the output positions of its ragged
//     columns, its size heads (lane v: head v) and the whole sample as aligned 16-byte chunks held
//     in registers (lane k: chunk k of every 1 KiB step; up to U KiB);
//   * lane-parallel geometry: lane c takes column c's length (its head, or the fixed size), a
//     wave prefix sum places it in the sample, one ballot checks the boundaries
//     (mds/reader.py:111-125);
//   * each wide column (ragged, or fixed > 16 B) is written destination-major: lane k owns 16-byte
//     output chunk k. The first wide column sits right behind the heads (and any fixed columns
//     before it), so its chunks are the loaded chunks shifted by at most one lane (DPP
//     wave_shl / wave_shr) and realigned with the neighbour lane's chunk (v_alignbyte funnel): no
//     LDS. Columns further in (config C's `n` and `s`), and fixed columns of <= 16 B, are read
//     from a copy of just their chunks in the wave's LDS (one unaligned ds_read_b128 per output
//     chunk);
//   * str values are checked for strict UTF-8 (bytes.decode('utf-8'), encodings.py:80-81) on the
//     same registers; the partial 16-byte chunks at a value's two ends are stored one byte per
//     lane (their other bytes are the neighbouring samples' values).
// Samples larger than U KiB are listed for stage_huge_kernel (mdsx_stage.hip), which copies each
// column straight from HBM in a second launch. A sample failing the
// file checks is reported (MDSX_E_BOUNDS / MDSX_E_EMPTY) and leaves zero-length ragged values and
// its fixed rows unwritten, the register decode's rule (the scan pass counted it zero).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "mdsx_decode.h"
#include "mdsx_device.h"
#include "mdsx_internal.h"
#include "mdsx_ring.h"

namespace mdsx_kernels {
namespace {

constexpr uint32_t kSwPad = 16;  // LDS bytes before the wave's chunk copy (reads from S >= -15)
constexpr int kDppWaveShr1 = 0x138;  // lane i <- lane i - 1 across the wave (lane 0: 0)

__device__ __forceinline__ uint4 lds16(const lds_u8* p) {
  const u32x4 v = *(const MDSX_L u32x4*)p;  // any byte address (gfx950 reads LDS unaligned)
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Lane k: loaded chunk q + 64 G + k (q in {-1, 0, 1}, wave-uniform; chunks outside: zeros). G
// is a constant once the caller's loop is unrolled.
template <int U>
__device__ __forceinline__ uint4 near_chunk(const uint4 (&L)[U], int G, int q, int lane) {
  if (q == 0) return L[G];
  const uint4 z = make_uint4(0, 0, 0, 0);
  if (q > 0) {
    uint4 x = dpp_mov4<kDppWaveShl1>(L[G]);
    const uint4 n = G + 1 < U ? readlane0(L[G + 1 < U ? G + 1 : G]) : z;
    if (lane == 63) x = n;
    return x;
  }
  uint4 x = dpp_mov4<kDppWaveShr1>(L[G]);
  const uint4 p = G > 0 ? readlane4(L[G > 0 ? G - 1 : 0], 63) : z;
  if (lane == 0) x = p;
  return x;
}

// One wide column of the sample: output bytes [d0, d0 + len) from stream byte S + h of the
// loaded chunks (S = the stream byte of output chunk 0's byte 0, h = d0 & 15; S >= -15). kNear:
// S in [-16, 32) -- chunks from the registers; else from the wave's LDS copy (buf: where stream
// byte 0 would be).
// Returns (utf8) whether the value is not well-formed UTF-8 (wave-uniform).
template <bool kNT, int U, bool kNear, int kX = 0>
__device__ __forceinline__ bool sw_copy(const uint4 (&L)[U], const lds_u8* buf, uint64_t d0,
                                        uint32_t len, int32_t S, bool utf8, int lane) {
  const uint64_t dend = d0 + len;
  const uint64_t dbeg = d0 & ~uint64_t(15);
  const uint32_t nch = uint32_t((((dend + 15) & ~uint64_t(15)) - dbeg) >> 4);
  const int q = S >> 4;  // arithmetic: -1 for S in [-16, 0)
  const uint32_t sh = uint32_t(S) & 15u;
  const uint4 z = make_uint4(0, 0, 0, 0);
  bool bad = false;
  uint32_t prev_w = 0;
#pragma unroll
  for (int g = 0; g < U; ++g) {
    if (64u * uint32_t(g) >= nch) break;  // wave-uniform
    const uint32_t k = 64u * uint32_t(g) + uint32_t(lane);
    uint4 out;
    if constexpr (kNear) {
      const uint4 lo = near_chunk<U>(L, g, q, lane);
      out = lo;
      if (sh != 0) {
        // the neighbour chunk: lane k + 1's, lane 63 the next step's lane 0
        uint4 hi = dpp_mov4<kDppWaveShl1>(lo);
        const uint4 n63 = q < 0 ? readlane4(L[g], 63)
                                : (g + 1 < U ? readlane4(L[g + 1 < U ? g + 1 : g], q) : z);
        if (lane == 63) hi = n63;
        out = funnel16(lo, hi, sh);
      }
    } else {
      out = k < nch ? lds16(buf + (S + int32_t(16u * k))) : z;
    }
    const uint64_t D = dbeg + 16ull * k;
    if (k < nch && D >= d0 && D + 16 <= dend) st16<kNT>(D, out);
    if ((kX & 2) == 0 && g == 0 && (dbeg < d0 || dbeg + 16 > dend))
      wave_edge_store(out, 0, dbeg, d0, dend, lane);
    if ((kX & 2) == 0 && nch > 1 && (dend & 15) != 0 && nch - 1 >= 64u * uint32_t(g) &&
        nch - 1 < 64u * uint32_t(g) + 64u)
      wave_edge_store(out, int(nch - 1 - 64u * uint32_t(g)), dbeg + 16ull * (nch - 1), d0, dend,
                      lane);
    if ((kX & 1) == 0 && utf8) {
      const uint4 vout = keep_range(out, D, d0, dend);  // this value's bytes only
      const uint32_t any8 = (vout.x | vout.y | vout.z | vout.w) & 0x80808080u;
      if (__any(any8 != 0) || hi_c0(prev_w)) {  // a byte >= 0x80 (or a sequence open before)
        uint32_t pw = dpp_mov<kDppWaveShr1>(vout.w);  // lane k - 1's last dword
        if (lane == 0) pw = prev_w;
        if (k < nch) bad |= utf8_chunk_bad(vout, pw, k == nch - 1);
      }
      prev_w = uint32_t(__builtin_amdgcn_readlane(int(vout.w), 63));
    }
  }
  return utf8 ? __any(bad) != 0 : false;
}

__device__ __forceinline__ uint64_t sw_clock() {
  uint64_t c;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c)::"memory");
  return c;
}

// kOcc: registers bounded for that many waves per SIMD (0: the compiler's choice).
// kX (measurement only, MDSX_TUNE swx; bits 1-4, 16, 32 leave outputs incomplete): 1 no UTF-8
// check, 2 no partial edge chunk stored, 4 only the register-path columns written (none through
// LDS), 16 no small fixed column stored, 32 no LDS-path column copied (the LDS copy made), 64 the
// LDS-path columns stored with the default cache policy, 8 shader-clock stamps per sample into
// src_abs (u32 x 4 per row, cycles from the wave's start: its record in, its loads landed -- an
// added vmcnt(0) wait --, its stores issued, its end).
template <bool kNT, int U, int kOcc, int kX = 0>
__global__ __launch_bounds__(64, kOcc > 0 ? kOcc : 1) void swave_decode_kernel(const DevArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const uint64_t t_start = (kX & 8) ? sw_clock() : 0;
  uint32_t t_pair = 0, t_loads = 0;
  const lds_u8* const buf = (const lds_u8*)smem + kSwPad;
  const int lane = threadIdx.x;
  // XCD-contiguous samples: the records' lines and the partial output chunks two neighbouring
  // samples share meet in one L2
  const uint32_t blk = (a.xcd_order & kXcdSeg) ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint32_t tile = blk >> uint32_t(__builtin_ctz(uint32_t(a.tile_rows)));
  if (tile >= a.ntiles) return;  // wave-uniform; no barrier in this kernel
  // ---- requested first: the sample's record (its scan pass: the sample's first byte, size,
  // shard and output row -- the offsets pair of mds/reader.py:137-142 checked there) and the
  // ragged outputs' positions (lane c: column c; the scan pass left the scan-block-local offset in
  // offsets[row])
  const uint4 rec = a.sw_rec[blk];
  // (readfirstlane returns an int: every field goes through uint32_t before it widens, or a byte
  // offset past 2 GiB would sign-extend)
  const uint32_t z = uint32_t(__builtin_amdgcn_readfirstlane(rec.z));
  if (z == kSwIdle) return;
  const uint32_t ry = uint32_t(__builtin_amdgcn_readfirstlane(rec.y));
  const uint64_t row = uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(rec.w)));
  const uint64_t src = uint64_t(uint32_t(__builtin_amdgcn_readfirstlane(rec.x))) |
                       (uint64_t(ry & 0xffu) << 32);
  const uint32_t shard = ry >> 8;
  const int ncols = a.ncols, nvar = a.nvar;
  const uint32_t hv = 4u * uint32_t(nvar);
  int vi = -1;
  uint32_t rb = 0;
  bool str = false;
  uint64_t data = 0, cap = 0;
  int64_t* offp = nullptr;
  uint8_t* flp = nullptr;
  for (int c = 0; c < ncols; ++c) {  // uniform
    const DevCol& col = a.cols[c];
    const int cv = col.var_index;
    const uint32_t crb = col.row_bytes;
    const bool cs = col.kind == MDSX_KIND_STR && col.flags != nullptr;
    const uint64_t cdata = reinterpret_cast<uint64_t>(col.data);
    int64_t* const coffs = col.offsets;
    uint8_t* const cflags = col.flags;
    const uint64_t ccap = col.capacity;
    if (lane == c)
      vi = cv, rb = crb, str = cs, data = cdata, offp = coffs, flp = cflags, cap = ccap;
  }
  int64_t off = 0;
  if (vi >= 0) off = a.tile_prefix[uint64_t(vi) * a.nscan + tile / a.scan_per] + offp[row];
  // the row inside its shard, for an error report (rare: one more load)
  auto row_in_shard = [&]() { return int(row - a.shards[shard].row0); };
  // ---- the sample (mds/reader.py:137-148): lane c's size head, then all of its bytes
  int rc = z == kSwBad ? MDSX_E_BOUNDS : z < hv ? MDSX_E_BOUNDS : MDSX_OK;
  const bool reported = z == kSwBad;  // (by the scan pass)
  const uint32_t size = rc == MDSX_OK ? z : 0u;
  if constexpr ((kX & 8) != 0) t_pair = uint32_t(sw_clock() - t_start);
  const uint64_t s0 = reinterpret_cast<uint64_t>(a.batch) + src;
  const uint32_t sa = uint32_t(s0 & 15);
  const uint4* const sal = reinterpret_cast<const uint4*>(s0 - sa);
  const uint32_t nload = (sa + size + 15u) >> 4;
  const bool inreg = rc == MDSX_OK && nload <= 64u * U;  // wave-uniform
  uint32_t hl = 0;
  if (rc == MDSX_OK && lane < ncols && vi >= 0)
    hl = load_u32_any(reinterpret_cast<const uint8_t*>(s0) + 4u * uint32_t(vi));
  uint4 L[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const uint32_t k = 64u * uint32_t(u) + uint32_t(lane);
    L[u] = inreg && k < nload ? ld16<kNT>(sal + k) : make_uint4(0, 0, 0, 0);
  }
  if constexpr ((kX & 8) != 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    t_loads = uint32_t(sw_clock() - t_start);
  }
  // ---- geometry (mds/reader.py:111-125): lane c's length, its place by a wave prefix sum (DPP;
  // 32-bit sums of at most 64 columns of a sample under 64 MiB cannot wrap)
  const uint32_t len = lane < ncols ? (vi >= 0 ? hl : rb) : 0u;
  const bool over = lane < ncols && len > size;
  const uint32_t lc = over ? 0u : len;
  const uint32_t incl = size < (1u << 26) ? wave_incl_dpp(lc) : wave_incl_u32(lc, lane, ncols);
  const uint32_t total = uint32_t(__builtin_amdgcn_readlane(int(incl), ncols - 1));
  if (rc == MDSX_OK && (__any(over) || total > size - hv)) rc = MDSX_E_BOUNDS;
  if (rc != MDSX_OK && !reported && lane == 0)
    report_decode(a, rc, int(shard), row_in_shard(), -1);
  const bool ok = rc == MDSX_OK;  // wave-uniform
  const uint32_t rel = hv + incl - lc;  // the column's first byte inside the sample
  bool skip = false;
  if (ok && vi >= 0 && uint64_t(off) + len > cap) {
    report_decode(a, MDSX_E_CAPACITY, int(shard), row_in_shard(), lane);
    skip = true;  // the sample writes nothing of the column
  }
  // the row's ragged offsets, now (their registers are then free for the copies)
  if (vi >= 0) *gp(offp + row) = off;
  const bool is_small = lane < ncols && vi < 0 && rb <= uint32_t(kSmallMax);
  const uint64_t D = vi >= 0 ? data + uint64_t(off) : data + row * rb;
  const bool small = ok && is_small;
  const bool wide = ok && lane < ncols && !is_small && !skip && len > 0;
  const uint64_t wide_mask = __ballot(wide);
  uint64_t badm = 0;  // bit c: column c's str value is not well-formed UTF-8
  // output chunk 0 of the column starts at stream byte S (relative to the aligned sample start)
  const int32_t S = int32_t(sa + rel) - int32_t(D & 15);
  // (str values are checked for UTF-8 from LDS: the check beside the whole sample in registers
  // would cost the kernel a wave per SIMD)
  const bool near = S >= -16 && S < 32 && !str;
  const bool via_lds = (kX & 4) ? false : small || (wide && !near);
  const uint64_t lds_mask = __ballot(via_lds);
  // the chunks the LDS columns' bytes lie in (columns lie in the sample in column order: from the
  // first such column's first chunk to the last one's end); a wider span than the wave's LDS
  // copy takes the huge-row kernel
  uint32_t jlo = 0, jhi = 0;
  if (lds_mask) {
    const uint32_t lo = (sa + rel) >> 4;
    const uint32_t hi = (sa + rel + (is_small ? rb : len) + 15u) >> 4;
    jlo = uint32_t(__builtin_amdgcn_readlane(int(lo), __builtin_ctzll(lds_mask)));
    jhi = uint32_t(__builtin_amdgcn_readlane(int(hi), 63 - __builtin_clzll(lds_mask)));
  }
  const bool fits = inreg && 16u * (jhi - jlo) <= a.sw_lds;  // wave-uniform
  if (ok && fits) {
    const uint64_t str_mask = __ballot(str), near_mask = __ballot(near);
    // the columns from the registers, then (the registers free) the ones from LDS
    for (uint64_t m = wide_mask & near_mask; m; m &= m - 1) {
      const int c = __builtin_ctzll(m);  // wave-uniform
      sw_copy<kNT, U, true, kX>(L, buf, readlane64(D, c),
                                uint32_t(__builtin_amdgcn_readlane(int(len), c)),
                                __builtin_amdgcn_readlane(S, c), false, lane);
    }
    // the LDS copy: stream chunk k at LDS byte kSwPad + 16 (k - jlo)
    const lds_u8* const base = buf - 16 * int32_t(jlo);
    if (lds_mask) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (64u * uint32_t(u) >= jhi || 64u * uint32_t(u) + 64u <= jlo) continue;  // uniform
        const uint32_t k = 64u * uint32_t(u) + uint32_t(lane);
        if (k >= jlo && k < jhi)
          *(MDSX_L u32x4*)(smem + kSwPad + 16u * (k - jlo)) =
              u32x4{L[u].x, L[u].y, L[u].z, L[u].w};
      }
      if ((kX & 16) == 0 && small)
        small_store(reinterpret_cast<uint8_t*>(D), lds16(base + (sa + rel)), rb);
    }
    // (measurement, kX bit 64: these columns stored with the default cache policy)
    for (uint64_t m = (kX & 36) ? 0ull : wide_mask & ~near_mask; m; m &= m - 1) {
      const int c = __builtin_ctzll(m);  // wave-uniform
      if (sw_copy<kNT && (kX & 64) == 0, U, false, kX>(L, base, readlane64(D, c),
                                     uint32_t(__builtin_amdgcn_readlane(int(len), c)),
                                     __builtin_amdgcn_readlane(S, c), (str_mask >> c) & 1ull, lane))
        badm |= 1ull << c;
    }
  } else if (ok && lane == 0) {
    // a sample past the register window (or its LDS copy): listed for stage_huge_kernel (every
    // column straight from HBM, after this launch; it reads the final offsets written above)
    uint32_t* count = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(a.status) +
                                                  kHugeCountOffset);
    a.src_abs[atomicAdd(count, 1u)] = (uint64_t(tile) << 32) | (blk & uint32_t(a.tile_rows - 1));
  }
  const uint32_t t_copied = (kX & 8) ? uint32_t(sw_clock() - t_start) : 0u;
  // ---- the row's str flags
  if (vi >= 0 && flp) *gp(flp + row) = uint8_t((badm >> lane) & 1ull);
  if constexpr ((kX & 8) != 0) {
    if (lane < 4) {
      const uint32_t st = lane == 0 ? t_pair : lane == 1 ? t_loads : lane == 2 ? t_copied
                                                                          : uint32_t(sw_clock() - t_start);
      *gp(reinterpret_cast<uint32_t*>(a.src_abs) + 4ull * row + lane) = st;
    }
  }
}

}  // namespace

int launch_swave_decode(const mdsx_plan* plan, const DevArgs& a, hipStream_t s) {
  const uint64_t waves = uint64_t(a.ntiles) * uint64_t(a.tile_rows);
  if (waves == 0) return MDSX_OK;
  if (waves > 0xffffffffull) return mdsx::fail(MDSX_E_ARG, "mdsx: swave: too many samples");
  // the list of samples past the register window starts empty
  const int zc = hip_check(hipMemsetAsync(reinterpret_cast<uint8_t*>(a.status) + kHugeCountOffset,
                                          0, 4, s),
                           "hipMemsetAsync");
  if (zc != MDSX_OK) return zc;
  const int U = plan->swave_kb, occ = plan->swave_occ;
  const bool nt = plan->run_nt != 0;
  DevArgs b = a;
  b.sw_lds = uint32_t(plan->swave_lds);
  const size_t lds = size_t(b.sw_lds) + 2 * kSwPad + size_t(plan->lds_pad_kb) * 1024;
#define MDSX_SWAVE(NT, UU, OCC)                                                                  \
  if (nt == NT && U == UU && occ == OCC) {                                                       \
    const void* fn = reinterpret_cast<const void*>(swave_decode_kernel<NT, UU, OCC>);            \
    if (lds > 64 * 1024 &&                                                                       \
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)) !=         \
            hipSuccess)                                                                          \
      return mdsx::fail(MDSX_E_HIP, "mdsx: swave_decode_kernel LDS attribute");                 \
    mdsx::set_last_kernel("swave_decode_kernel<" #NT ", " #UU ", " #OCC ">");                    \
    hipLaunchKernelGGL((swave_decode_kernel<NT, UU, OCC>), dim3(unsigned(waves)), dim3(64), lds, \
                       s, b);                                                                    \
    const int rc = hip_check(hipGetLastError(), "swave_decode_kernel launch");                   \
    return rc != MDSX_OK ? rc : launch_huge_rows(a, NT, s);                                      \
  }
  if (plan->swave_x) {  // measurement variants (nt, 6 KiB, the compiler's occupancy)
    if (!nt || U != 6 || occ != 0)
      return mdsx::fail(MDSX_E_ARG, "mdsx: swave variants: rnt=1, swkb=6, swocc=0 only");
    if ((plan->swave_x & 8) && a.nvar < 2)
      return mdsx::fail(MDSX_E_ARG, "mdsx: swave stamps need two ragged columns (src_abs space)");
#define MDSX_SWAVE_X(X)                                                                          \
  if (plan->swave_x == X) {                                                                      \
    mdsx::set_last_kernel("swave_decode_kernel<true, 6, 0, " #X ">");                            \
    hipLaunchKernelGGL((swave_decode_kernel<true, 6, 0, X>), dim3(unsigned(waves)), dim3(64),     \
                       lds, s, b);                                                               \
    const int rc = hip_check(hipGetLastError(), "swave_decode_kernel launch");                   \
    return rc != MDSX_OK ? rc : launch_huge_rows(a, true, s);                                    \
  }
    MDSX_SWAVE_X(1) MDSX_SWAVE_X(2) MDSX_SWAVE_X(3) MDSX_SWAVE_X(4) MDSX_SWAVE_X(7)
    MDSX_SWAVE_X(8) MDSX_SWAVE_X(16) MDSX_SWAVE_X(32) MDSX_SWAVE_X(48) MDSX_SWAVE_X(64)
#undef MDSX_SWAVE_X
    return mdsx::fail(MDSX_E_ARG, "mdsx: swave variant out of range");
  }
  MDSX_SWAVE(true, 6, 0)
  MDSX_SWAVE(true, 6, 4)
  MDSX_SWAVE(true, 6, 6)
  MDSX_SWAVE(true, 4, 0)
  MDSX_SWAVE(true, 4, 6)
  MDSX_SWAVE(true, 8, 0)
  MDSX_SWAVE(true, 8, 4)
  MDSX_SWAVE(false, 6, 0)
#undef MDSX_SWAVE
  return mdsx::fail(MDSX_E_ARG,
                    "mdsx: swave: (nt, KiB, occupancy) of (1, 6, 0/4/6), (1, 4, 0/6), (1, 8, 0/4), "
                    "(0, 6, 0)");
}

}  // namespace mdsx_kernels
