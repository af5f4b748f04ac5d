// LDS-staged decode of ragged plans (gfx950): one workgroup per tile of rows, the tile's shard
// bytes read from HBM ONCE, straight into LDS, then every column written from LDS.
//
// The reference decodes one sample per call: MDSReader.get_sample_data reads the sample's byte
// range (streaming/base/format/mds/reader.py:128-149), decode_sample splits it at the u32 size
// heads of the variable columns and mds_decode returns each column's value
// (mds/reader.py:103-126, encodings.py:62-397,760-773). Here a tile's samples are contiguous in the
// shard file, so their bytes [begin(first row), end(last row)) are one range:
//
//   1. offsets pairs of the tile's rows (mds/reader.py:137-142), checked against the file;
//      final ragged output offsets = the scan pass's prefix + its tile-local offset;
//   2. the rows are cut into groups whose byte range fits the LDS stage (normally one group per
//      tile: the host sizes tiles to about half the stage, mdsx_plan_tile_rows_for); each group's
//      range is fetched with global_load_lds_dwordx4 (1 KiB per wave-instruction, no VGPRs), so
//      the column boundaries inside a sample, the heads and the str bytes re-read by the UTF-8
//      check cost no second HBM read;
//   3. size heads parsed from LDS (decode_sample's head loop), every column range checked;
//   4. each column written destination-major: lane k of the workgroup owns 16-byte-aligned output
//      chunk k of the group's contiguous output range of that column (fixed columns: rows x size;
//      ragged: the packed values), assembled from the LDS bytes of the row(s) it covers (two
//      aligned ds_read_b128 + v_alignbyte; binary search of the row), stored whole -- so every
//      store is a full, coalesced 16-byte store except the two chunks a group shares with its
//      neighbours (byte stores);
//   5. str rows checked for strict UTF-8 from LDS (what bytes.decode('utf-8') accepts,
//      encodings.py:80-81), four rows per wave, one per 16-lane group.
//
// A sample larger than the stage is copied straight from HBM (wave_copy, the 16-byte realigning
// wave copy; the str check runs inside that copy).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "mdsx_decode.h"
#include "mdsx_device.h"
#include "mdsx_internal.h"

namespace mdsx_kernels {
namespace {

// 16 bytes of the stage at byte position p (any alignment, -16 < p < cap: the stage has 16 bytes
// of slack on either side).
__device__ __forceinline__ uint4 lds16(const uint8_t* stage, int32_t p) {
  const uint4* q = reinterpret_cast<const uint4*>(stage + (p & ~15));
  return funnel16_lane(q[0], q[1], uint32_t(p & 15));
}

// u32 of the stage at byte position p (any alignment).
__device__ __forceinline__ uint32_t lds_u32(const uint8_t* stage, uint32_t p) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(stage + (p & ~3u));
  return alignbyte(q[1], q[0], p & 3u);
}

// Bytes [a, b) (0 <= a <= b <= 16) of `val` merged into `acc`.
__device__ __forceinline__ uint4 merge_bytes(uint4 acc, const uint4 val, uint32_t a, uint32_t b) {
  const uint4 m = byte_mask(a, b);
  return make_uint4((acc.x & ~m.x) | (val.x & m.x), (acc.y & ~m.y) | (val.y & m.y),
                    (acc.z & ~m.z) | (val.z & m.z), (acc.w & ~m.w) | (val.w & m.w));
}

// Strict UTF-8 of four staged rows per wave, one per 16-lane group: lane gl of a group checks
// aligned 16-byte chunks gl, gl + 16, ... of its row [p0, p0 + len) of the stage (bytes outside
// the row zeroed), the dword before each chunk passed along the group. Returns the group's
// verdict (uniform within the group).
__device__ __forceinline__ bool lds_utf8_bad(const uint8_t* stage, uint32_t p0, uint32_t len,
                                             int lane) {
  const int gl = lane & 15;
  const uint32_t d0 = p0, dend = p0 + len, dbeg = p0 & ~15u;
  const uint32_t nchunks = len ? (((dend + 15u) & ~15u) - dbeg) >> 4 : 0u;
  uint32_t maxc = nchunks;  // wave-uniform trip count
  maxc = max(maxc, uint32_t(__shfl_xor(int(maxc), 16)));
  maxc = max(maxc, uint32_t(__shfl_xor(int(maxc), 32)));
  bool bad = false;
  uint32_t carry = 0;
  for (uint32_t base = 0; base < maxc; base += 16) {
    const uint32_t k = base + uint32_t(gl);
    const uint32_t D = dbeg + 16u * k;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (k < nchunks) v = *reinterpret_cast<const uint4*>(stage + D);
    const uint4 vout = keep_range(v, D, d0, dend);
    uint32_t pw = __shfl_up(vout.w, 1, 16);
    if (gl == 0) pw = carry;
    carry = __shfl(vout.w, 15, 16);
    if (k < nchunks) bad |= utf8_chunk_bad(vout, pw, k == nchunks - 1);
  }
  const uint64_t m = __ballot(bad);
  return ((m >> (lane & 48)) & 0xffffull) != 0;
}

// Store the bytes of `v` (chunk at column byte D) that lie in [lo, hi): a whole 16-byte store
// when the chunk is inside, else one byte at a time (the group's two edge chunks).
template <bool kNT>
__device__ __forceinline__ void store_chunk(uint8_t* out, uint64_t D, uint64_t lo, uint64_t hi,
                                            const uint4 v) {
  if (D >= lo && D + 16 <= hi) {
    st16<kNT>(reinterpret_cast<uint64_t>(out) + D, v);
    return;
  }
  for (int b = 0; b < 16; ++b)
    if (D + b >= lo && D + b < hi) *gp(out + D + b) = uint8_t(byte_of(v, b));
}

struct StageLds {
  uint8_t* stage;    // [cap], 16 bytes of slack before and after
  int64_t* dst;      // [nvar][TR]  final ragged output offset of each row
  uint32_t* beg;     // [TR]        sample begin (file offset)
  uint32_t* end;     // [TR]        sample end
  uint32_t* src;     // [ncols][TR] stage position of each column of a row of the current group
  uint32_t* len;     // [nvar][TR]  ragged length of a row (0 if the row failed a check)
  uint8_t* ok;       // [TR]
};

__host__ __device__ __forceinline__ size_t stage_meta_bytes(int TR, int ncols, int nvar) {
  return size_t(TR) * (8 * size_t(nvar) + 8 + 4 * size_t(ncols) + 4 * size_t(nvar) + 1);
}

// The heads and column layout of row t from its sample bytes at stage position `pos`
// (MDSReader.decode_sample, mds/reader.py:111-125): the same rules as the scan pass, so a row's
// lengths here are the ones its output offsets were scanned from.
template <class HeadAt>
__device__ __forceinline__ bool row_layout(const DevArgs& a, const StageLds& L, int TR, int t,
                                           uint64_t pos, uint64_t size, HeadAt head) {
  if (4ull * a.nvar > size) return false;
  uint64_t p = pos + 4ull * a.nvar;
  for (int c = 0; c < a.ncols; ++c) {
    const DevCol& col = a.cols[c];
    uint64_t n = col.row_bytes;
    if (col.var_index >= 0) {
      n = head(col.var_index);
      L.len[col.var_index * TR + t] = uint32_t(n);
    }
    L.src[c * TR + t] = uint32_t(p);
    p += n;
  }
  return p <= pos + size;
}

// Huge rows (a sample larger than the stage), listed by stage_decode_kernel: one workgroup per
// row, straight from HBM (a separate launch, so the staged kernel keeps its registers for the
// common case). Fixed and bytes columns are split over the four waves at 16-byte-aligned
// destination points (wave_copy: the 16-byte realigning wave copy); str columns are copied and
// checked by one wave (the UTF-8 look-back runs through the whole row).
template <bool kNT>
__global__ __launch_bounds__(kBlock) void stage_huge_kernel(const DevArgs a) {
  const uint32_t* count = reinterpret_cast<const uint32_t*>(
      reinterpret_cast<const uint8_t*>(a.status) + kHugeCountOffset);
  const uint64_t* list = a.src_abs;  // (tile << 32 | row in tile) of every huge row
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t n = *count;
  for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {  // block-uniform
    const uint64_t entry = list[i];
    const TileView v = tile_view(a, uint32_t(entry >> 32));
    const uint32_t t = uint32_t(entry);
    const uint64_t row = v.d.row0 + v.r0 + t;
    uint32_t b = 0, e = 0;
    sample_range(v, v.r0 + t, &b, &e);  // checked by the staged kernel before listing the row
    const uint8_t* sample = v.shard + b;
    auto head = [&](int vi) { return load_u32_any(sample + 4u * uint32_t(vi)); };
    uint64_t pos = 4ull * a.nvar;
    bool ok = pos <= uint64_t(e - b);
    for (int c = 0; ok && c < a.ncols; ++c) {
      const DevCol& col = a.cols[c];
      pos += col.var_index >= 0 ? head(col.var_index) : col.row_bytes;
      ok = pos <= uint64_t(e - b);
    }
    if (!ok) {
      if (threadIdx.x == 0) report(a.status, MDSX_E_BOUNDS, v.shard_idx, int(v.r0 + t), -1);
      continue;
    }
    pos = 4ull * a.nvar;
    for (int c = 0; c < a.ncols; ++c) {
      const DevCol& col = a.cols[c];
      const uint64_t len = col.var_index >= 0 ? head(col.var_index) : col.row_bytes;
      const uint8_t* src = sample + pos;
      pos += len;
      if (len == 0) continue;
      uint8_t* out = static_cast<uint8_t*>(col.data);
      uint64_t d = row * col.row_bytes;
      if (col.var_index >= 0) {
        d = uint64_t(col.offsets[row]);  // final (written by the staged kernel)
        if (d + len > col.capacity) {
          if (threadIdx.x == 0) report(a.status, MDSX_E_CAPACITY, v.shard_idx, int(v.r0 + t), c);
          continue;
        }
      }
      if (col.kind == MDSX_KIND_STR && col.flags) {
        if (wave == 0) {
          const bool bad = wave_copy<true, 2, kNT>(src, out + d, len, lane);
          if (lane == 0 && bad) col.flags[row] = 1;
        }
        continue;
      }
      // quarter w: destination bytes [q_w, q_{w+1}), split at 16-byte-aligned output addresses
      const uint64_t D0 = reinterpret_cast<uint64_t>(out) + d;
      const uint64_t per = (((len + 3) / 4) + 15) & ~uint64_t(15);
      uint64_t q0 = wave == 0 ? 0 : ((D0 + per * uint64_t(wave)) & ~uint64_t(15)) - D0;
      uint64_t q1 = wave == 3 ? len : ((D0 + per * uint64_t(wave + 1)) & ~uint64_t(15)) - D0;
      q0 = std::min(q0, len);
      q1 = std::min(std::max(q1, q0), len);
      if (q1 > q0) wave_copy<false, 4, kNT>(src + q0, out + d + q0, q1 - q0, lane);
    }
  }
}

template <bool kNT>
__global__ __launch_bounds__(kBlock) void stage_decode_kernel(const DevArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int TR = a.tile_rows;
  const uint32_t cap = a.stage_bytes;
  StageLds L;
  L.stage = smem + 16;
  L.dst = reinterpret_cast<int64_t*>(smem + 16 + cap + 16);
  L.beg = reinterpret_cast<uint32_t*>(L.dst + a.nvar * TR);
  L.end = L.beg + TR;
  L.src = L.end + TR;
  L.len = L.src + a.ncols * TR;
  L.ok = reinterpret_cast<uint8_t*>(L.len + a.nvar * TR);
  __shared__ uint32_t s_first, s_gend, s_hi;

  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  const uint32_t tile = blockIdx.x;
  const TileView v = tile_view(a, tile);
  if (!v.table_ok) {
    if (t == 0 && tile == v.d.tile0) report(a.status, MDSX_E_HEADER, v.shard_idx, -1, -1);
    return;  // block-uniform
  }
  if (t == 0 && tile == v.d.tile0) {
    // header written by encode_joint_shard (mds/writer.py:133-144): u32 N, then N+1 offsets
    const uint32_t n = *reinterpret_cast<const uint32_t*>(v.shard);
    if (n != v.d.samples || v.offs[0] < v.hdr_end || v.offs[v.d.samples] > v.d.bytes)
      report(a.status, MDSX_E_HEADER, v.shard_idx, -1, -1);
  }
  const int nrows = int(v.nrows);

  // ---- 1. sample ranges, final ragged offsets
  if (t < nrows) {
    uint32_t b = 0, e = 0;
    const int rc = sample_range(v, v.r0 + t, &b, &e);
    L.beg[t] = b;
    L.end[t] = e;
    L.ok[t] = rc == MDSX_OK;
    if (rc != MDSX_OK) report(a.status, rc, v.shard_idx, int(v.r0 + t), -1);
    const uint64_t row = v.d.row0 + v.r0 + t;
    for (int c = 0; c < a.ncols; ++c) {
      const DevCol& col = a.cols[c];
      if (col.var_index < 0) continue;
      const int vi = col.var_index;
      // the scan pass left the scan-block-local offset in offsets[row]
      const int64_t off = a.tile_prefix[uint64_t(vi) * a.nscan + tile / a.scan_per] +
                          col.offsets[row];
      col.offsets[row] = off;
      L.dst[vi * TR + t] = off;
      L.len[vi * TR + t] = 0;
      if (col.flags) col.flags[row] = 0;
    }
  }
  __syncthreads();

  const uint32_t stage_lds = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)L.stage)));
  for (int ga = 0; ga < nrows;) {  // block-uniform loop over row groups
    // ---- 2. the group: rows from ga while every checked row's bytes fit the stage window that
    // starts at the first checked row
    if (t == 0) {
      s_first = uint32_t(nrows);
      s_gend = uint32_t(nrows);
      s_hi = 0;
    }
    __syncthreads();
    if (t >= ga && t < nrows && L.ok[t]) atomicMin(&s_first, uint32_t(t));
    __syncthreads();
    const int first = int(s_first);
    const uint32_t lo = first < nrows ? (L.beg[first] & ~15u) : 0u;
    if (t >= ga && t < nrows && L.ok[t] && !(L.beg[t] >= lo && L.end[t] - lo <= cap))
      atomicMin(&s_gend, uint32_t(t));
    __syncthreads();
    const int gb = int(s_gend);
    if (gb == ga) {  // row ga is checked and larger than the stage: stage_huge_kernel's
      if (t == 0) {
        uint32_t* count = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(a.status) +
                                                      kHugeCountOffset);
        a.src_abs[atomicAdd(count, 1u)] = (uint64_t(tile) << 32) | uint32_t(ga);
      }
      ++ga;
      __syncthreads();  // every thread has read s_first / s_gend before they are reset
      continue;
    }
    if (t >= ga && t < gb && L.ok[t]) atomicMax(&s_hi, (L.end[t] + 15u) & ~15u);
    __syncthreads();
    const uint32_t hi = first < gb ? s_hi : lo;

    // ---- the group's bytes [lo, hi) into the stage, 1 KiB per wave-instruction
    const uint32_t nchunks = (hi - lo) >> 4;
    const uint4* gsrc = reinterpret_cast<const uint4*>(v.shard + lo);
    for (uint32_t p = uint32_t(wave); p * 64 < nchunks; p += kBlock / 64) {
      const uint32_t k = min(p * 64 + uint32_t(lane), nchunks - 1);
      glds16<kNT>(gsrc + k, stage_lds + p * 1024u);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();

    // ---- 3. heads and column ranges of the group's rows, from the stage
    if (t >= ga && t < gb && L.ok[t]) {
      const uint32_t pos = L.beg[t] - lo;
      const bool fits = row_layout(a, L, TR, t, pos, uint64_t(L.end[t] - L.beg[t]),
                                   [&](int vi) { return lds_u32(L.stage, pos + 4u * vi); });
      if (!fits) {
        L.ok[t] = 0;
        for (int vi = 0; vi < a.nvar; ++vi) L.len[vi * TR + t] = 0;
        report(a.status, MDSX_E_BOUNDS, v.shard_idx, int(v.r0 + t), -1);
      }
    }
    __syncthreads();

    // ---- 4. every column, destination-major from the stage
    const uint64_t grow0 = v.d.row0 + v.r0 + ga;  // output row of the group's first row
    for (int c = 0; c < a.ncols; ++c) {
      const DevCol& col = a.cols[c];
      uint8_t* out = static_cast<uint8_t*>(col.data);
      const int vi = col.var_index;
      const uint32_t rb = col.row_bytes;
      uint64_t d0, d1;  // the group's output byte range of this column
      if (vi < 0) {
        d0 = grow0 * rb;
        d1 = d0 + uint64_t(gb - ga) * rb;
      } else {
        d0 = uint64_t(L.dst[vi * TR + ga]);
        d1 = uint64_t(L.dst[vi * TR + gb - 1]) + L.len[vi * TR + gb - 1];
        if (d1 > col.capacity) {  // block-uniform
          if (t == 0) report(a.status, MDSX_E_CAPACITY, v.shard_idx, int(v.r0 + ga), c);
          continue;
        }
      }
      if (d1 <= d0) continue;
      const uint64_t dbeg = d0 & ~uint64_t(15);
      const uint32_t nout = uint32_t(((d1 + 15) & ~uint64_t(15)) - dbeg) >> 4;
      for (uint32_t k = uint32_t(t); k < nout; k += kBlock) {
        const uint64_t D = dbeg + 16ull * k;
        const uint64_t x = D > d0 ? D : d0;  // first byte of the chunk this group owns
        // row j holding byte x: fixed by division, ragged by binary search of the offsets
        int j;
        if (vi < 0) {
          j = ga + int(d1 - d0 < (1ull << 32) ? uint64_t(uint32_t(x - d0) / rb) : (x - d0) / rb);
        } else {
          int l = ga, h = gb - 1;
          while (l < h) {
            const int m = (l + h + 1) >> 1;
            if (uint64_t(L.dst[vi * TR + m]) <= x) l = m; else h = m - 1;
          }
          j = l;
        }
        uint4 val = make_uint4(0, 0, 0, 0);
        for (; j < gb; ++j) {
          const uint64_t rd = vi < 0 ? grow0 * rb + uint64_t(j - ga) * rb
                                     : uint64_t(L.dst[vi * TR + j]);
          if (rd >= D + 16) break;
          const uint32_t rl = vi < 0 ? rb : L.len[vi * TR + j];
          const uint64_t pa = std::max(D, rd), pb = std::min(D + 16, rd + rl);
          if (pb <= pa || !L.ok[j]) continue;
          // the 16 stage bytes that line up with the chunk: stage byte of D within row j
          const uint4 piece = lds16(L.stage, int32_t(L.src[c * TR + j]) - int32_t(rd - D));
          if (pa == D && pb == D + 16) {
            val = piece;
            break;
          }
          val = merge_bytes(val, piece, uint32_t(pa - D), uint32_t(pb - D));
        }
        store_chunk<kNT>(out, D, d0, d1, val);
      }
    }

    // ---- 5. strict UTF-8 of the group's str rows, from the stage
    for (int c = 0; c < a.ncols; ++c) {
      const DevCol& col = a.cols[c];
      if (col.kind != MDSX_KIND_STR || !col.flags) continue;
      const int vi = col.var_index;
      for (int r0 = ga + wave * 4; r0 < gb; r0 += kBlock / 16) {
        const int r = min(r0 + (lane >> 4), gb - 1);
        const bool live = r0 + (lane >> 4) < gb && L.ok[r];
        const uint32_t n = live ? L.len[vi * TR + r] : 0u;
        const bool bad = lds_utf8_bad(L.stage, L.src[c * TR + r], n, lane);
        if ((lane & 15) == 0 && n && bad) col.flags[v.d.row0 + v.r0 + r] = 1;
      }
    }
    __syncthreads();  // the stage is refilled by the next group
    ga = gb;
  }
}

}  // namespace

size_t stage_lds_bytes(const mdsx_plan* plan, int tile_rows, uint32_t stage_bytes) {
  return ((16 + size_t(stage_bytes) + 16 + stage_meta_bytes(tile_rows, plan->ncols, plan->nvar) +
           15) & ~size_t(15));
}

int launch_stage_decode(const mdsx_plan* plan, const DevArgs& a, hipStream_t s) {
  int rc = hip_check(hipMemsetAsync(reinterpret_cast<uint8_t*>(a.status) + kHugeCountOffset, 0,
                                    sizeof(uint32_t), s),
                     "hipMemsetAsync");
  if (rc != MDSX_OK) return rc;
  const size_t lds = stage_lds_bytes(plan, a.tile_rows, a.stage_bytes);
  if (lds > 64 * 1024) {  // above the default dynamic-LDS limit of a launch
    rc = hip_check(hipFuncSetAttribute(reinterpret_cast<const void*>(
                                           plan->nontemporal ? stage_decode_kernel<true>
                                                             : stage_decode_kernel<false>),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)),
                   "hipFuncSetAttribute");
    if (rc != MDSX_OK) return rc;
  }
  // huge rows: at most one per workgroup of the staged kernel's tiles (usually none)
  const unsigned hgrid = unsigned(std::min<uint64_t>(a.ntiles, 1024));
  if (plan->nontemporal) {
    mdsx::set_last_kernel("stage_decode_kernel<true>");
    hipLaunchKernelGGL((stage_decode_kernel<true>), dim3(a.ntiles), dim3(kBlock), lds, s, a);
    rc = hip_check(hipGetLastError(), "stage_decode_kernel launch");
    if (rc == MDSX_OK)
      hipLaunchKernelGGL((stage_huge_kernel<true>), dim3(hgrid), dim3(kBlock), 0, s, a);
  } else {
    mdsx::set_last_kernel("stage_decode_kernel<false>");
    hipLaunchKernelGGL((stage_decode_kernel<false>), dim3(a.ntiles), dim3(kBlock), lds, s, a);
    rc = hip_check(hipGetLastError(), "stage_decode_kernel launch");
    if (rc == MDSX_OK)
      hipLaunchKernelGGL((stage_huge_kernel<false>), dim3(hgrid), dim3(kBlock), 0, s, a);
  }
  if (rc != MDSX_OK) return rc;
  return hip_check(hipGetLastError(), "stage_huge_kernel launch");
}

}  // namespace mdsx_kernels
