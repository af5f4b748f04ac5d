// Row-parallel decode of ragged plans with short samples (gfx950): a workgroup decodes one tile
// -- up to 256 consecutive samples of one shard -- from a single LDS copy of the tile's bytes, one
// thread per sample.
//
// The reference decodes one sample per call (MDSReader.get_sample_data, mds/reader.py:128-149;
// decode_sample, :103-126; mds_decode, encodings.py:760-773). The samples of a tile are one
// contiguous byte range of the shard (sample i ends where i + 1 starts), so the workgroup
//   1. copies the range into LDS once (global_load_lds_dwordx4, 1 KiB per wave-instruction, the
//      range started on a 128-byte line);
//   2. parses each sample's size heads and column boundaries from LDS, one thread per sample
//      (decode_sample's head loop; a sample whose offsets or columns do not fit counts zero
//      bytes and is reported, the scan pass's rule);
//   3. scans the ragged lengths across the tile (block scan) onto the tile's output base (from
//      the scan pass, stage_totals_kernel + the reduce-then-scan kernels);
//   4. writes every column: the thread of sample j owns the 16-byte-aligned output chunks whose
//      first byte is one of its own, assembles each from LDS with unaligned ds_read_b128 (a chunk
//      that runs past the sample's end takes the following samples' bytes), and stores it whole;
//      only the chunks a tile shares with its neighbours are stored a byte at a time;
//   5. checks its str values for strict UTF-8 from LDS (what bytes.decode('utf-8') accepts,
//      encodings.py:80-81) and writes its offsets and flags.
// Per-sample work is spread over lanes, not looped over by one wave: the per-sample scalar
// control of the streaming decode (mdsx_run.hip) is what bounds short samples there.
//
// A tile whose range exceeds the LDS stage is decoded in windows of samples that fit, each window
// a tile of its own for the edge chunks; a sample larger than the stage is copied straight from
// HBM by the workgroup's four waves.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "mdsx_decode.h"
#include "mdsx_device.h"
#include "mdsx_internal.h"

namespace mdsx_kernels {
namespace {

constexpr int kRowsBlock = 256;  // one thread per sample of a tile (<= 256 samples)
// LDS: 32 bytes before the stage (a chunk's read may start up to 15 bytes before a value) and
// 128 + 32 after it (the range starts on a 128-byte line; unaligned reads run past its end)
constexpr uint32_t kStageFront = 32;
constexpr uint32_t kStageSlack = 128 + 32;

__device__ __forceinline__ uint4 lds_read16(const lds_u8* p) {
  const u32x4 v = *(const MDSX_L u32x4*)p;
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Bytes [from, to) (0 <= from <= to <= 16) of chunk v stored at the aligned address D.
__device__ __forceinline__ void store_bytes(uint64_t D, const uint4 v, uint32_t from, uint32_t to) {
  for (uint32_t b = from; b < to; ++b) *gp_at<uint8_t>(D + b) = uint8_t(byte_of(v, int(b)));
}

// Per-column, per-sample tables of the window in LDS.
struct RowsTab {
  MDSX_L uint32_t* src;  // [ncols][TR] stage position of the column's first byte
  MDSX_L uint32_t* len;  // [ncols][TR] bytes (0: a sample that failed a check)
  MDSX_L uint64_t* dst;  // [ncols][TR] output byte of the column value, relative to its data
};

__host__ __device__ __forceinline__ size_t rows_tab_bytes(int TR, int ncols) {
  return size_t(TR) * size_t(ncols) * 16;
}

__host__ __device__ __forceinline__ size_t rows_lds_bytes(uint32_t cap, int TR, int ncols) {
  return kStageFront + size_t(cap) + kStageSlack + rows_tab_bytes(TR, ncols);
}

// The 16 output bytes at aligned column address D (absolute), from the window's samples r, r + 1,
// ... (stage bytes; a sample whose value is not in the stage leaves zeros) whose values cover
// them, starting at byte `from` of the chunk.
__device__ __forceinline__ uint4 assemble(const lds_u8* stage, const RowsTab& T, int base, int r,
                                          int gb, uint64_t data, uint64_t D, uint32_t from) {
  uint4 val = make_uint4(0, 0, 0, 0);
  uint64_t pos = D + from;
  for (; r < gb && pos < D + 16; ++r) {
    const uint32_t len = T.len[base + r];
    const uint64_t ds = data + T.dst[base + r];
    const uint64_t de = ds + len;
    if (de <= pos || len == 0) continue;
    const uint64_t a = max(pos, ds), b = min(D + 16, de);
    const uint4 v = lds_read16(stage + T.src[base + r] + uint32_t(a - ds) - uint32_t(a - D));
    val = merge_bytes(val, v, uint32_t(a - D), uint32_t(b - D));
    pos = b;
  }
  return val;
}

template <bool kNT>
__global__ __launch_bounds__(kRowsBlock) void rows_decode_kernel(const DevArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ DevCol s_cols[MDSX_MAX_COLUMNS];
  __shared__ int64_t s_wsum[kRowsBlock / 64];
  __shared__ uint64_t s_base[MDSX_MAX_COLUMNS];  // next output byte of each column (rel. data)
  __shared__ uint32_t s_skip[MDSX_MAX_COLUMNS];   // the tile's bytes exceed the column capacity
  __shared__ uint32_t s_gb, s_lo, s_hi, s_bdir;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  for (int c = t; c < a.ncols; c += kRowsBlock) s_cols[c] = a.cols[c];
  const MDSX_L DevCol* cols = (const MDSX_L DevCol*)s_cols;
  const uint32_t tile = blockIdx.x;
  const int TR = a.tile_rows;
  const int ncols = a.ncols, nvar = a.nvar;
  const uint32_t cap = a.rows_bytes;
  const lds_u8* stage = (const lds_u8*)(smem + kStageFront);
  RowsTab T;
  T.dst = (MDSX_L uint64_t*)(smem + kStageFront + cap + kStageSlack);
  T.src = (MDSX_L uint32_t*)(T.dst + size_t(ncols) * TR);
  T.len = T.src + size_t(ncols) * TR;
  const uint32_t stage_lds = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((const MDSX_L uint8_t*)(smem + kStageFront))));

  const TileView v = tile_view(a, tile);
  if (t == 0 && tile == v.d.tile0) {
    // header written by encode_joint_shard (mds/writer.py:133-144): u32 N, then N + 1 offsets
    if (!v.table_ok || *reinterpret_cast<const uint32_t*>(v.shard) != v.d.samples ||
        v.offs[0] < v.hdr_end || v.offs[v.d.samples] > v.d.bytes)
      report_decode(a, MDSX_E_HEADER, v.shard_idx, -1, -1);
  }
  if (!v.table_ok) return;  // block-uniform
  const int n = int(v.nrows);
  const uint64_t row0 = v.d.row0 + v.r0;
  // this thread's sample: offsets pair and file checks (mds/reader.py:137-148)
  uint32_t b = 0, e = 0;
  int rc = MDSX_OK;
  if (t < n) rc = sample_range(v, v.r0 + uint32_t(t), &b, &e);
  const bool in_range = t < n && rc == MDSX_OK;
  if (t < n && rc != MDSX_OK) report_decode(a, rc, v.shard_idx, int(v.r0 + t), -1);
  if (t < ncols) {
    const MDSX_L DevCol& col = cols[t];
    const int vi = col.var_index;
    uint32_t skip = 0;
    if (vi >= 0) {
      const uint64_t off = uint64_t(a.tile_prefix[uint64_t(vi) * a.nscan + tile]);
      s_base[t] = off;
      if (off + uint64_t(a.tile_total[uint64_t(vi) * a.nscan + tile]) > col.capacity) {
        report_decode(a, MDSX_E_CAPACITY, v.shard_idx, int(v.r0), t);
        skip = 1;
      }
    } else {
      s_base[t] = row0 * col.row_bytes;
    }
    s_skip[t] = skip;
  }

  for (int ga = 0; ga < n;) {  // block-uniform loop over windows
    // ---- the window: samples [ga, gb) whose bytes lie in [lo, lo + cap)
    __syncthreads();  // the previous window's readers of the stage and the tables are done
    if (t == 0) s_gb = uint32_t(n), s_lo = 0xffffffffu;
    __syncthreads();
    if (t >= ga && in_range) atomicMin(&s_lo, b);  // the window's first in-range byte
    __syncthreads();
    const uint32_t lo = s_lo;
    if (t >= ga && in_range && !(b >= lo && e - lo <= cap)) atomicMin(&s_gb, uint32_t(t));
    __syncthreads();
    int gb = int(s_gb);
    const bool direct = gb == ga;  // sample ga alone is larger than the stage: from HBM
    if (direct) gb = ga + 1;
    const uint32_t lo_al = lo & ~127u;
    // ---- 1. the window's bytes [lo_al, hi) into LDS, hi the largest end of its in-range samples
    if (t == 0) s_hi = 0;
    __syncthreads();
    if (t >= ga && t < gb && in_range) atomicMax(&s_hi, e);
    if (direct && t == ga) s_bdir = b;
    __syncthreads();
    const uint32_t hi = s_hi;
    if (!direct && lo != 0xffffffffu && hi > lo_al) {
      const uint32_t nq = (hi - lo_al + 15) >> 4;
      const uint4* src = reinterpret_cast<const uint4*>(v.shard + lo_al);
      for (uint32_t kb = uint32_t(wave); kb * 64 < nq; kb += kRowsBlock / 64) {
        const uint32_t k = kb * 64 + uint32_t(lane);
        if (k < nq) glds16<kNT>(src + k, stage_lds + kb * 1024u);  // lanes past nq write nothing
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();

    // ---- 2. column boundaries of this thread's sample (mds/reader.py:111-125)
    const bool mine = t >= ga && t < gb;
    bool ok = mine && in_range;
    uint32_t need = 4u * uint32_t(nvar);
    if (ok && need > e - b) ok = false;
    if (ok) {
      for (int c = 0; c < ncols; ++c) {
        const int vi = cols[c].var_index;
        need += vi >= 0 ? (direct ? load_u32_any(v.shard + b + 4u * uint32_t(vi))
                                  : *(const MDSX_L uint32_t*)(stage + (b - lo_al) + 4u * vi))
                        : cols[c].row_bytes;
      }
      if (need > e - b) ok = false;
    }
    if (mine && in_range && !ok) report_decode(a, MDSX_E_BOUNDS, v.shard_idx, int(v.r0 + t), -1);
    // ---- 3. offsets: lengths scanned across the window onto each column's base
    uint32_t rel = 4u * uint32_t(nvar);
    for (int c = 0; c < ncols; ++c) {
      const MDSX_L DevCol& col = cols[c];
      const int vi = col.var_index;
      uint32_t len = 0;
      if (ok)
        len = vi >= 0 ? (direct ? load_u32_any(v.shard + b + 4u * uint32_t(vi))
                                : *(const MDSX_L uint32_t*)(stage + (b - lo_al) + 4u * vi))
                      : col.row_bytes;
      uint64_t dst;
      if (vi >= 0) {
        int64_t total;
        const int64_t excl = block_exclusive_scan(mine ? int64_t(len) : 0, s_wsum, &total);
        dst = s_base[c] + uint64_t(excl);
        __syncthreads();  // every thread has read s_base[c]
        if (t == 0) s_base[c] += uint64_t(total);
        if (mine) *gp(col.offsets + row0 + t) = int64_t(dst);
      } else {
        dst = uint64_t(row0 + t) * col.row_bytes;
      }
      if (mine) {
        T.dst[c * TR + t] = dst;
        T.src[c * TR + t] = direct ? rel : (b - lo_al) + rel;  // direct: inside the sample
        T.len[c * TR + t] = len;
      }
      rel += len;
    }
    __syncthreads();

    // ---- 4. every column, destination-major per sample; 5. UTF-8
    for (int c = 0; c < ncols; ++c) {
      const MDSX_L DevCol& col = cols[c];
      if (s_skip[c]) continue;  // block-uniform
      const uint64_t data = reinterpret_cast<uint64_t>(col.data);
      const int base = c * TR;
      const bool utf8 = col.kind == MDSX_KIND_STR && col.flags != nullptr;
      // the window's output range of the column
      const uint64_t wbeg = data + T.dst[base + ga];
      const uint64_t wend = data + T.dst[base + gb - 1] + T.len[base + gb - 1];
      if (direct) {  // one sample larger than the stage: copied from HBM by the four waves
        const uint32_t len = T.len[base + ga];
        if (len == 0) continue;  // block-uniform
        const uint8_t* src = v.shard + s_bdir + T.src[base + ga];
        uint8_t* out = reinterpret_cast<uint8_t*>(data + T.dst[base + ga]);
        if (utf8) {  // one wave copies and validates
          if (wave == 0) {
            const bool bad = wave_copy<true, 2, kNT>(src, out, len, lane);
            if (lane == 0) *gp(col.flags + row0 + ga) = bad ? 1 : 0;
          }
          continue;
        }
        // quarter w: output bytes [q_w, q_w+1), split at 16-byte-aligned output addresses
        const uint64_t D0 = reinterpret_cast<uint64_t>(out);
        const uint64_t per = (((uint64_t(len) + 3) / 4) + 15) & ~uint64_t(15);
        uint64_t q0 = wave == 0 ? 0 : ((D0 + per * uint64_t(wave)) & ~uint64_t(15)) - D0;
        uint64_t q1 = wave == 3 ? len : ((D0 + per * uint64_t(wave + 1)) & ~uint64_t(15)) - D0;
        q0 = std::min<uint64_t>(q0, len);
        q1 = std::min<uint64_t>(std::max(q1, q0), len);
        if (q1 > q0) wave_copy<false, 4, kNT>(src + q0, out + q0, q1 - q0, lane);
        continue;
      }
      if (mine && T.len[base + t]) {
        const uint32_t len = T.len[base + t];
        const uint64_t ds = data + T.dst[base + t];
        const uint64_t de = ds + len;
        const uint32_t sp = T.src[base + t];
        // the chunk holding the window's first byte, shared with the previous window / tile
        if ((ds & 15) && ds == wbeg) {
          const uint64_t D = ds & ~uint64_t(15);
          const uint4 val = assemble(stage, T, base, t, gb, data, D, uint32_t(ds - D));
          store_bytes(D, val, uint32_t(ds - D), uint32_t(min(D + 16, wend) - D));
        }
        // the chunks whose first byte is one of this sample's
        for (uint64_t D = (ds + 15) & ~uint64_t(15); D < de; D += 16) {
          uint4 val;
          if (D + 16 <= de) {
            val = lds_read16(stage + sp + uint32_t(D - ds));
          } else {
            val = assemble(stage, T, base, t, gb, data, D, 0);
          }
          if (D + 16 <= wend) st16<kNT>(D, val);
          else store_bytes(D, val, 0, uint32_t(wend - D));
        }
      }
      if (utf8 && mine) {
        bool bad = false;
        const uint32_t len = T.len[base + t];
        const uint32_t sp = T.src[base + t];
        uint32_t pw = 0;
        for (uint32_t k = 0; k < len; k += 16) {
          uint4 vv = lds_read16(stage + sp + k);
          if (k + 16 > len) vv = keep_range(vv, 0, 0, len - k);
          bad |= utf8_chunk_bad(vv, pw, k + 16 >= len);
          pw = vv.w;
        }
        *gp(col.flags + row0 + t) = bad ? 1 : 0;
      }
    }
    ga = gb;
  }
}

}  // namespace

uint32_t rows_tile_rows_limit() { return kRowsBlock; }

int launch_rows_decode(const mdsx_plan* plan, const DevArgs& a, hipStream_t s) {
  if (a.tile_rows > kRowsBlock)
    return mdsx::fail(MDSX_E_ARG, "mdsx: row-parallel decode tiles hold at most 256 rows");
  const size_t lds = rows_lds_bytes(a.rows_bytes, a.tile_rows, a.ncols);
#define MDSX_ROWS_CASE(NT)                                                                   \
  if (bool(plan->rows_nt) == NT) {                                                           \
    if (lds > 64 * 1024) {                                                                   \
      const int rc = hip_check(                                                              \
          hipFuncSetAttribute(reinterpret_cast<const void*>(rows_decode_kernel<NT>),         \
                              hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)),         \
          "hipFuncSetAttribute");                                                            \
      if (rc != MDSX_OK) return rc;                                                          \
    }                                                                                        \
    mdsx::set_last_kernel("rows_decode_kernel<" #NT ">");                                   \
    hipLaunchKernelGGL((rows_decode_kernel<NT>), dim3(a.ntiles), dim3(kRowsBlock), lds, s, a); \
    return hip_check(hipGetLastError(), "rows_decode_kernel launch");                        \
  }
  MDSX_ROWS_CASE(true)
  MDSX_ROWS_CASE(false)
#undef MDSX_ROWS_CASE
  return MDSX_E_ARG;
}

}  // namespace mdsx_kernels
