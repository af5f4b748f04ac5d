// LDS-staged decode of ragged plans (gfx950): each tile's shard bytes are read from HBM ONCE,
// straight into LDS, and every column is written from there.
//
// The reference decodes one sample per call: MDSReader.get_sample_data reads the sample's byte
// range (streaming/base/format/mds/reader.py:128-149), decode_sample splits it at the u32 size
// heads of the variable columns and mds_decode returns each column's value
// (mds/reader.py:103-126, encodings.py:62-397,760-773). Here the samples of a tile (a few rows,
// sized by the host to about half the LDS stage: mdsx_plan_tile_rows_for) are contiguous in the
// shard file, so their bytes are one range.
//
// Pass 1 (stage_totals_kernel): the ragged bytes of every tile from the offsets table and the u32
// size heads, then scan_totals_kernel (mdsx_kernels.hip) turns them into each tile's output base.
//
// Pass 2 (stage_decode_kernel): a workgroup runs a software pipeline over a run of consecutive
// tiles. Wave 0 is the loader: while waves 1-3 decode tile k from one LDS stage buffer, the shard
// bytes of tile k + 1 are in flight into the other (global_load_lds_dwordx4: 1 KiB per
// wave-instruction, no VGPRs) and the offsets-table slice and output bases of tile k + 2 into a
// third metadata slot (global_load_lds_dword). The loads are issued from inline asm, invisible to
// the compiler; the loader, which stores nothing, retires them with one `s_waitcnt vmcnt(0)` per
// tile and a barrier publishes them, while the consumers' stores stay in flight. For tile k:
//
//   1. each row's offsets pair (mds/reader.py:137-142) checked against the file, its size heads
//      and column ranges parsed from LDS (decode_sample's head loop, mds/reader.py:111-125);
//   2. ragged output offsets = the tile's base + an exclusive scan of the rows' lengths;
//   3. every column written destination-major: lane k of the workgroup owns 16-byte-aligned output
//      chunk k of the tile's contiguous output range of that column (fixed columns: rows x size;
//      ragged: packed values), assembled from the LDS bytes of the row(s) it covers (two aligned
//      ds_read_b128 + v_alignbyte; the row by binary search), stored whole -- every store is a
//      full, coalesced 16-byte store except the two chunks a tile shares with its neighbours;
//   4. str rows checked for strict UTF-8 from LDS (what bytes.decode('utf-8') accepts,
//      encodings.py:80-81), four rows per wave, one per 16-lane group.
//
// So the heads, the column boundaries inside a sample and the str bytes the UTF-8 check reads cost
// no second HBM read, and no row edge costs a partial store. A tile larger than a stage buffer is
// decoded in row groups with synchronous loads; a sample larger than the stage is listed for
// stage_huge_kernel, which copies it straight from HBM.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "mdsx_decode.h"
#include "mdsx_device.h"
#include "mdsx_internal.h"

namespace mdsx_kernels {
namespace {

constexpr int kMetaSlots = 3;
// A stage_decode_kernel workgroup: 8 waves. Wave 0 is the loader: it issues every LDS-DMA and
// no global store, so it waits for its loads with vmcnt(0) without waiting for stores; waves 1-7
// (the consumers, consumer thread ct = threadIdx.x - 64) decode and store, and never wait for
// their stores inside the loop.
constexpr int kStageBlock = 512;
constexpr int kConsumers = kStageBlock - 64;


// 16 bytes of a stage buffer at byte position p (any alignment, -16 < p < cap: a buffer has 16
// bytes of slack on either side).
__device__ __forceinline__ uint4 lds16(const lds_u8* stage, int32_t p) {
  const MDSX_L uint4* q = reinterpret_cast<const MDSX_L uint4*>(stage + (p & ~15));
  return funnel16_lane(q[0], q[1], uint32_t(p & 15));
}

// u32 of a stage buffer at byte position p (any alignment).
__device__ __forceinline__ uint32_t lds_u32(const lds_u8* stage, uint32_t p) {
  const MDSX_L uint32_t* q = reinterpret_cast<const MDSX_L uint32_t*>(stage + (p & ~3u));
  return alignbyte(q[1], q[0], p & 3u);
}

// Strict UTF-8 of four staged rows per wave, one per 16-lane group: lane gl of a group checks
// aligned 16-byte chunks gl, gl + 16, ... of its row [p0, p0 + len) of the stage (bytes outside
// the row zeroed), the dword before each chunk passed along the group. Returns the group's
// verdict (uniform within the group).
__device__ __forceinline__ bool lds_utf8_bad(const lds_u8* stage, uint32_t p0, uint32_t len,
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
    if (k < nchunks) v = *reinterpret_cast<const MDSX_L uint4*>(stage + D);
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
// when the chunk is inside, else one byte at a time (the two chunks a tile shares).
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

// A tile as the pipeline sees it (built once per workgroup from the tile and shard tables).
struct TileDesc {
  uint64_t shard_off;  // shard file offset inside the batch buffer
  uint64_t row0;       // output row of the tile's first row
  uint32_t bytes;      // shard file size (< 4 GiB: u32 offsets)
  uint32_t r0;         // first row of the tile inside its shard
  uint32_t nrows;
  uint32_t samples;    // rows of the shard
  int32_t shard;       // batch shard index
  uint32_t table_ok;   // the shard's offsets table fits in its file
};

// Per-tile metadata, loaded by LDS-DMA two tiles ahead: the tile's slice of the offsets table
// (offs[r0 .. r0 + nrows]) and its output base in every ragged column (low / high dwords).
struct MetaSlot {
  uint32_t* offs;     // [TR + 1] (rounded up to 64 + 1 entries)
  uint32_t* base_lo;  // [64]
  uint32_t* base_hi;  // [64]
};

__host__ __device__ __forceinline__ uint32_t meta_slot_words(int TR) {
  return uint32_t(((TR + 1 + 63) / 64) * 64) + 128;
}

// Per-row layout of the tile being decoded.
struct RowLds {
  uint32_t* rel;   // [ncols][TR] byte offset of each column inside the row's sample
  uint32_t* len;   // [nvar][TR]  ragged length (0 where the row failed a check)
  int64_t* dst;    // [nvar][TR]  final ragged output offset
  int32_t* src;    // [ncols][TR] stage position of the column's first byte (-1: the row failed)
  uint32_t* rdst;  // [ncols][TR] output position of the column's first byte, relative to the
                   //             first 16-byte-aligned output chunk of the rows being written
  uint8_t* ok;     // [TR]
};

__host__ __device__ __forceinline__ size_t row_lds_bytes(int TR, int ncols, int nvar) {
  return size_t(TR) * (12 * size_t(ncols) + 4 * size_t(nvar) + 8 * size_t(nvar) + 1);
}

// Column layout of a sample of `size` bytes from its size heads (MDSReader.decode_sample,
// mds/reader.py:111-125): writes each column's offset inside the sample and each ragged column's
// length; false where the heads or the columns do not fit in the sample. The same rule as
// stage_totals_kernel, so a row's lengths here are the ones its tile base was summed from.
template <class HeadAt>
__device__ __forceinline__ bool row_layout(const DevArgs& a, const MDSX_L DevCol* cols,
                                           const RowLds& R, int TR, int t, uint64_t size,
                                           HeadAt head) {
  if (4ull * a.nvar > size) return false;
  uint64_t p = 4ull * a.nvar;
  for (int c = 0; c < a.ncols; ++c) {
    const MDSX_L DevCol& col = cols[c];
    uint64_t n = col.row_bytes;
    if (col.var_index >= 0) {
      n = head(col.var_index);
      R.len[col.var_index * TR + t] = uint32_t(n);
    }
    R.rel[c * TR + t] = uint32_t(p);
    p += n;
  }
  return p <= size;
}

// The rows of `td` from its metadata slot: sample range checks (mds/reader.py:137-148).
__device__ __forceinline__ int row_range(const TileDesc& td, const MetaSlot& m, int t,
                                         uint32_t* b, uint32_t* e) {
  *b = m.offs[t];
  *e = m.offs[t + 1];
  const uint64_t hdr_end = 4ull + 4ull * (uint64_t(td.samples) + 1ull);
  if (!(hdr_end <= *b && *b <= *e && *e <= td.bytes)) return MDSX_E_BOUNDS;
  if (*b == *e) return MDSX_E_EMPTY;
  return MDSX_OK;
}

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const uint8_t*)p)));
}

// Loader (wave 0): the offsets-table slice and output bases of tile `td` into metadata slot m.
__device__ __forceinline__ void load_meta(const DevArgs& a, const TileDesc& td, uint32_t tile,
                                          const MetaSlot& m, int lane) {
  if (!td.table_ok) return;
  const uint32_t* offs = reinterpret_cast<const uint32_t*>(a.batch + td.shard_off + 4) + td.r0;
  const uint32_t n = td.nrows + 1;
  const uint32_t lds_offs = lds_addr(m.offs);
  for (uint32_t i = 0; i < n; i += 64)
    glds4(offs + min(i + uint32_t(lane), n - 1), lds_offs + 4 * i);
  if (a.nvar) {
    const int vi = lane < a.nvar ? lane : 0;
    const uint32_t* base =
        reinterpret_cast<const uint32_t*>(a.tile_prefix + uint64_t(vi) * a.nscan + tile);
    glds4(base, lds_addr(m.base_lo));
    glds4(base + 1, lds_addr(m.base_hi));
  }
}

// Loader (wave 0): the byte range [lo, hi) of the tile's checked samples, and whether it fits a
// stage buffer of `cap` bytes.
__device__ __forceinline__ void tile_span(const TileDesc& td, const MetaSlot& m, uint32_t cap,
                                          int lane, uint32_t* lo, uint32_t* hi, bool* fits) {
  uint32_t mn = 0xffffffffu, mx = 0;
  if (td.table_ok) {
    for (uint32_t r = uint32_t(lane); r < td.nrows; r += 64) {
      uint32_t b, e;
      if (row_range(td, m, int(r), &b, &e) == MDSX_OK) {
        mn = min(mn, b);
        mx = max(mx, e);
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    mn = min(mn, uint32_t(__shfl_xor(int(mn), o)));
    mx = max(mx, uint32_t(__shfl_xor(int(mx), o)));
  }
  if (mn > mx) {  // no checked row: nothing to load
    *lo = *hi = 0;
    *fits = true;
    return;
  }
  *lo = mn & ~15u;
  *hi = (mx + 15u) & ~15u;
  *fits = *hi - *lo <= cap;
}

// Loader: bytes [lo, hi) of the shard into a stage buffer, 1 KiB per wave-instruction.
template <bool kNT>
__device__ __forceinline__ void load_bytes(const uint8_t* shard, uint32_t lo, uint32_t hi,
                                           uint32_t stage_lds, int lane) {
  const uint32_t n = (hi - lo) >> 4;
  const uint4* src = reinterpret_cast<const uint4*>(shard + lo);
  for (uint32_t p = 0; p * 64 < n; ++p)
    glds16<kNT>(src + min(p * 64 + uint32_t(lane), n - 1), stage_lds + p * 1024u);
}

// The output byte range [d0, d1) of column c for rows [ga, gb) of the tile.
__device__ __forceinline__ void column_range(const MDSX_L DevCol& col, const TileDesc& td,
                                             const RowLds& R, int TR, int ga, int gb,
                                             uint64_t* d0, uint64_t* d1) {
  const int vi = col.var_index;
  if (vi < 0) {
    *d0 = (td.row0 + uint32_t(ga)) * col.row_bytes;
    *d1 = *d0 + uint64_t(gb - ga) * col.row_bytes;
  } else {
    *d0 = uint64_t(R.dst[vi * TR + ga]);
    *d1 = uint64_t(R.dst[vi * TR + gb - 1]) + R.len[vi * TR + gb - 1];
  }
}

// Consumers: where each column of rows [ga, gb) sits in the stage (whose byte 0 is shard byte
// `lo`) and in the output (relative to the rows' first aligned output chunk of the column).
__device__ __forceinline__ void place_rows(const DevArgs& a, const MDSX_L DevCol* cols,
                                           const TileDesc& td, const RowLds& R, const MetaSlot& m,
                                           int TR, uint32_t lo, int ga, int gb) {
  for (int r = ga + int(threadIdx.x) - 64; r >= ga && r < gb; r += kConsumers) {
    for (int c = 0; c < a.ncols; ++c) {
      const MDSX_L DevCol& col = cols[c];
      uint64_t d0, d1;
      column_range(col, td, R, TR, ga, gb, &d0, &d1);
      const uint64_t rd = col.var_index < 0 ? d0 + uint64_t(r - ga) * col.row_bytes
                                            : uint64_t(R.dst[col.var_index * TR + r]);
      R.rdst[c * TR + r] = uint32_t(rd - (d0 & ~uint64_t(15)));
      R.src[c * TR + r] = R.ok[r] ? int32_t(m.offs[r] - lo + R.rel[c * TR + r]) : -1;
    }
  }
}

// Consumers: every column of rows [ga, gb) from the stage, destination-major: consumer lane k
// assembles 16-byte-aligned output chunk k of the rows' contiguous output range of the column
// from the stage bytes of the row(s) it covers (the row: division for fixed columns, binary
// search for ragged ones) and stores it whole; only the range's two edge chunks, shared with
// the neighbouring rows of other tiles, are stored a byte at a time.
template <bool kNT>
__device__ __forceinline__ void write_columns(const DevArgs& a, const MDSX_L DevCol* cols,
                                              const TileDesc& td, const RowLds& R, int TR,
                                              const lds_u8* stage, int ga, int gb) {
  const int ct = int(threadIdx.x) - 64;
  for (int c = 0; c < a.ncols; ++c) {
    const MDSX_L DevCol& col = cols[c];
    const int vi = col.var_index;
    const uint32_t rb = col.row_bytes;
    uint64_t d0, d1;
    column_range(col, td, R, TR, ga, gb, &d0, &d1);
    if (vi >= 0 && d1 > col.capacity) {  // block-uniform
      if (ct == 0) report_decode(a, MDSX_E_CAPACITY, td.shard, int(td.r0 + ga), c);
      continue;
    }
    if (d1 <= d0) continue;
    const uint64_t dbeg = d0 & ~uint64_t(15);
    uint8_t* out = static_cast<uint8_t*>(col.data) + dbeg;
    const uint32_t lo = uint32_t(d0 - dbeg), hi = uint32_t(d1 - dbeg);  // owned bytes
    const uint32_t nout = (hi + 15) >> 4;
    const uint32_t* rdst = R.rdst + c * TR;
    const int32_t* src = R.src + c * TR;
    for (uint32_t k = uint32_t(ct); k < nout; k += kConsumers) {
      const uint32_t D = 16u * k;
      const uint32_t x = max(D, lo);  // first byte of the chunk these rows own
      int j;
      if (vi < 0) {
        j = ga + int((x - lo) / rb);
      } else {
        int l = ga, h = gb - 1;
        while (l < h) {
          const int mid = (l + h + 1) >> 1;
          if (rdst[mid] <= x) l = mid; else h = mid - 1;
        }
        j = l;
      }
      uint32_t rd = rdst[j];
      uint32_t rl = vi < 0 ? rb : R.len[vi * TR + j];
      int32_t sp = src[j];
      uint4 val;
      if (sp >= 0 && D >= rd && D + 16 <= rd + rl) {  // inside one row: the common case
        val = lds16(stage, sp + int32_t(D - rd));
      } else {
        val = make_uint4(0, 0, 0, 0);
        for (;;) {
          const uint32_t pa = max(D, rd), pb = min(D + 16, rd + rl);
          if (pb > pa && sp >= 0)
            val = merge_bytes(val, lds16(stage, sp - int32_t(rd - D)), pa - D, pb - D);
          if (++j >= gb) break;
          rd = rdst[j];
          if (rd >= D + 16) break;
          rl = vi < 0 ? rb : R.len[vi * TR + j];
          sp = src[j];
        }
      }
      if (D >= lo && D + 16 <= hi) {
        st16<kNT>(reinterpret_cast<uint64_t>(out) + D, val);
      } else {
        for (uint32_t b = 0; b < 16; ++b)
          if (D + b >= lo && D + b < hi) *gp(out + D + b) = uint8_t(byte_of(val, int(b)));
      }
    }
  }
}

// Consumers: strict UTF-8 of the str rows in [ga, gb), from the stage (four rows per wave).
__device__ __forceinline__ void check_utf8(const DevArgs& a, const MDSX_L DevCol* cols,
                                           const TileDesc& td, const RowLds& R, int TR,
                                           const lds_u8* stage, int ga, int gb) {
  const int lane = threadIdx.x & 63, cw = int(threadIdx.x >> 6) - 1;
  for (int c = 0; c < a.ncols; ++c) {
    const MDSX_L DevCol& col = cols[c];
    if (col.kind != MDSX_KIND_STR || !col.flags) continue;
    const int vi = col.var_index;
    for (int r0 = ga + cw * 4; r0 < gb; r0 += kConsumers / 16) {
      const int r = min(r0 + (lane >> 4), gb - 1);
      const bool live = r0 + (lane >> 4) < gb && R.src[c * TR + r] >= 0;
      const uint32_t n = live ? R.len[vi * TR + r] : 0u;
      const bool bad = lds_utf8_bad(stage, live ? uint32_t(R.src[c * TR + r]) : 0u, n, lane);
      if ((lane & 15) == 0 && n && bad) col.flags[td.row0 + r] = 1;
    }
  }
}

// Exclusive scan of the rows' ragged lengths -> final offsets (tile base + scan) by wave 1 (up to
// four rows per lane), written out by the consumers with zeroed str flags. Block-uniform.
__device__ __forceinline__ void tile_offsets(const DevArgs& a, const MDSX_L DevCol* cols,
                                             const TileDesc& td, const RowLds& R,
                                             const MetaSlot& m, int TR) {
  const int t = threadIdx.x, lane = t & 63;
  const int n = td.table_ok ? int(td.nrows) : 0;
  if ((t >> 6) == 1) {
    const int per = (n + 63) / 64;
    const int r0 = lane * per, r1 = min(r0 + per, n);
    for (int vi = 0; vi < a.nvar; ++vi) {
      const uint32_t* len = R.len + vi * TR;
      int64_t sum = 0;
      for (int r = r0; r < r1; ++r) sum += len[r];
      int64_t incl = sum;
      for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(incl, o);
        if (lane >= o) incl += y;
      }
      int64_t run = int64_t((uint64_t(m.base_hi[vi]) << 32) | m.base_lo[vi]) + incl - sum;
      for (int r = r0; r < r1; ++r) {
        R.dst[vi * TR + r] = run;
        run += len[r];
      }
    }
  }
  __syncthreads();
  for (int r = t - 64; r >= 0 && r < n; r += kConsumers) {
    const uint64_t row = td.row0 + r;
    for (int c = 0; c < a.ncols; ++c) {
      const MDSX_L DevCol& col = cols[c];
      if (col.var_index < 0) continue;
      col.offsets[row] = R.dst[col.var_index * TR + r];
      if (col.flags) col.flags[row] = 0;
    }
  }
}

// A row that fails a check: no ragged bytes, its error reported.
__device__ __forceinline__ void fail_row(const DevArgs& a, const TileDesc& td, const RowLds& R,
                                         int TR, int t, int rc) {
  R.ok[t] = 0;
  for (int vi = 0; vi < a.nvar; ++vi) R.len[vi * TR + t] = 0;
  report_decode(a, rc, td.shard, int(td.r0 + t), -1);
}

}  // namespace

// Look-back status word of one (ragged column, block of tiles): flag in the top 2 bits (0 not yet
// published, 1 the block's own aggregate, 2 its inclusive prefix), a byte count below.
constexpr uint64_t kChainAgg = 1ull << 62, kChainIncl = 2ull << 62;
constexpr uint64_t kChainValue = (1ull << 62) - 1;

// One ragged column of a chained totals block: the block's tiles' exclusive prefixes (x: the
// tile's total at its first thread, 0 elsewhere) from a block scan plus the block's base from the
// look-back, written to tile_prefix; the last block also writes the column's total.
__device__ __forceinline__ void chained_prefix(const DevArgs& a, int vi, uint32_t block,
                                               uint32_t tile, int64_t x, bool head_thread,
                                               int64_t* s_wsum, int64_t* s_base) {
  typedef __attribute__((address_space(1))) uint64_t cu64;
  int64_t agg;
  const int64_t excl = block_exclusive_scan(x, s_wsum, &agg);
  const int t = threadIdx.x, lane = t & 63;
  const uint32_t nblocks = (a.ntiles + uint32_t(kBlock / a.tile_rows) - 1) /
                           uint32_t(kBlock / a.tile_rows);
  cu64* st = (cu64*)(a.chain + uint64_t(vi) * nblocks);
  if (t < 64) {  // wave 0: publish, then look back over the earlier blocks
    if (t == 0)
      __hip_atomic_store(st + block, (block == 0 ? kChainIncl : kChainAgg) | uint64_t(agg),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t base = 0;
    int64_t j = int64_t(block) - 1;
    bool done = block == 0;
    uint32_t polls = 0;
    while (!done) {  // wave-uniform
      const int64_t k = j - lane;
      const uint64_t w = k >= 0 ? __hip_atomic_load(st + k, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_AGENT)
                                : kChainIncl;
      const uint64_t incl = __ballot((w >> 62) == 2);
      const uint64_t none = __ballot((w >> 62) == 0);
      const uint64_t span = incl ? ((incl & (0 - incl)) << 1) - 1 : ~0ull;  // lanes <= first incl
      // an earlier block is still scanning its rows (it holds an earlier ticket, so it runs);
      // the bound only keeps a broken invariant from hanging the launch
      if ((none & span) != 0 && ++polls < (1u << 22)) {
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      if ((none & span) != 0 && lane == 0) report_decode(a, MDSX_E_HIP, -1, -1, -1);
      uint64_t v = ((span >> lane) & 1) ? (w & kChainValue) : 0;
      for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
      base += v;
      if (incl) done = true;
      else j -= 64;
    }
    if (t == 0) {
      if (block != 0)
        __hip_atomic_store(st + block, kChainIncl | (base + uint64_t(agg)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      *s_base = int64_t(base);
      if (block + 1 == nblocks) {  // the batch's last block: column totals
        for (int c = 0; c < a.ncols; ++c)
          if (a.cols[c].var_index == vi) a.cols[c].offsets[a.rows] = int64_t(base) + agg;
        if (a.totals) a.totals[vi] = int64_t(base) + agg;
      }
    }
  }
  __syncthreads();
  if (head_thread) a.tile_prefix[uint64_t(vi) * a.nscan + tile] = *s_base + excl;
  __syncthreads();  // s_base is reused by the next column
}

// Pass 1 of the staged decode: the ragged bytes of every tile (one thread per row; 256 / TR tiles
// per workgroup), with the staged kernel's row rule: a row whose range, heads or columns do not
// fit counts zero.
//
// kChained (tiles of <= 64 rows): the exclusive scan of the tile totals is done here too, in one
// pass -- workgroups take their block of tiles in ticket order, block-scan their tiles' totals
// and find the block's base by a decoupled look-back over the earlier blocks' status words (flag
// and value in one 8-byte word, agent-scope atomics) -- so no scan kernels follow.
template <bool kChained>
__global__ __launch_bounds__(kBlock) void stage_totals_kernel(const DevArgs a) {
  __shared__ int64_t s_part[kBlock / 64][MDSX_MAX_COLUMNS];
  __shared__ uint32_t s_bad[kBlock / 64];
  __shared__ int64_t s_wsum[kBlock / 64];
  __shared__ int64_t s_base;
  __shared__ uint32_t s_block;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int TR = a.tile_rows;
  uint32_t block = blockIdx.x;
  if constexpr (kChained) {
    if (t == 0) s_block = atomicAdd(a.ticket, 1u);
    __syncthreads();
    block = s_block;
  }
  const uint32_t tile = block * uint32_t(kBlock / TR) + uint32_t(t / TR);
  const bool tile_ok = tile < a.ntiles;
  TileView v;
  if (tile_ok) v = tile_view(a, tile);
  const bool in_tile = tile_ok && v.table_ok && (t % TR) < int(v.nrows);
  uint32_t b = 0, e = 0;
  bool ok = false, range_bad = false;
  if (in_tile) {
    range_bad = sample_range(v, v.r0 + t % TR, &b, &e) != MDSX_OK;
    ok = !range_bad && 4ull * a.nvar <= e - b;
  }
  const bool few = a.nvar <= kHeadRegs;
  Heads h;
  if (ok && few) h.load(v.shard + b, a.nvar);
  auto head = [&](int vi) -> uint32_t {
    return few ? h.get(vi) : load_u32_any(v.shard + b + 4u * uint32_t(vi));
  };
  if (ok) {
    uint64_t need = 4ull * a.nvar;
    for (int c = 0; c < a.ncols; ++c) {
      const DevCol& col = a.cols[c];
      need += col.var_index >= 0 ? head(col.var_index) : col.row_bytes;
    }
    ok = uint64_t(b) + need <= e;
  }
  for (int vi = 0; vi < a.nvar; ++vi) {
    int64_t x = ok ? int64_t(head(vi)) : 0;
    if (TR <= 64) {  // segments of TR lanes inside the wave
      for (int o = 1; o < TR; o <<= 1) x += __shfl_xor(x, o);
      if (tile_ok && t % TR == 0) a.tile_total[uint64_t(vi) * a.nscan + tile] = x;
      if constexpr (kChained) chained_prefix(a, vi, block, tile, tile_ok && t % TR == 0 ? x : 0,
                                             tile_ok && t % TR == 0, s_wsum, &s_base);
    } else {  // a tile spans TR / 64 waves
      for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
      if (lane == 0) s_part[wave][vi] = x;
    }
  }
  if (TR > 64) {
    __syncthreads();
    if (tile_ok && t % TR == 0) {
      for (int vi = 0; vi < a.nvar; ++vi) {
        int64_t sum = 0;
        for (int w = wave; w < wave + TR / 64; ++w) sum += s_part[w][vi];
        a.tile_total[uint64_t(vi) * a.nscan + tile] = sum;
      }
    }
  }
  // the run records of the streaming decode (tiles <= 32 rows) and the row-parallel decode
  if ((a.run_slots && TR < 64) || a.rows_bytes) {
    const uint64_t bad = __ballot(range_bad);
    // samples too large for the streaming decode's lean path (its ring holds a whole sample)
    const uint64_t big = __ballot(in_tile && !range_bad && a.seg_lim && e - b > a.seg_lim);
    bool tile_bad, tile_big = false;
    if (TR <= 64) {
      const uint64_t seg = TR == 64 ? ~0ull : ((1ull << TR) - 1) << (lane & ~(TR - 1));
      tile_bad = (bad & seg) != 0;  // this tile's lanes
      tile_big = (big & seg) != 0;
    } else {  // a tile spans TR / 64 waves
      if (lane == 0) s_bad[wave] = bad != 0;
      __syncthreads();
      tile_bad = false;
      for (int w = wave & ~(TR / 64 - 1); w < (wave & ~(TR / 64 - 1)) + TR / 64; ++w)
        tile_bad = tile_bad || s_bad[w];
    }
    if (tile_ok && t % TR == 0) {
      TileRun r;
      const bool fast = v.table_ok && v.nrows > 0 && !tile_bad;
      r.fast = fast ? (a.seg_lim && !tile_big ? 3 : 1) : 0;
      r.stream = v.d.offset + (fast ? v.offs[v.r0] : 0u);
      r.bytes = fast ? v.offs[v.r0 + v.nrows] - v.offs[v.r0] : 0u;
      r.offs = v.d.offset + 4ull + 4ull * v.r0;
      r.row0 = v.d.row0 + v.r0;
      r.shard = v.shard_idx;
      r.r0 = v.r0;
      r.nrows = uint16_t(v.nrows);
      r.shard_off = v.d.offset;
      a.tile_run[tile] = r;
      // header written by encode_joint_shard (mds/writer.py:133-144): u32 N, then N + 1 offsets
      if (tile == v.d.tile0 &&
          (!v.table_ok || *reinterpret_cast<const uint32_t*>(v.shard) != v.d.samples ||
           v.offs[0] < v.hdr_end || v.offs[v.d.samples] > v.d.bytes))
        report_decode(a, MDSX_E_HEADER, v.shard_idx, -1, -1);
    }
  }
}

namespace {

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
          if (threadIdx.x == 0) report_decode(a, MDSX_E_CAPACITY, v.shard_idx, int(v.r0 + t), c);
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
__global__ __launch_bounds__(kStageBlock) void stage_decode_kernel(const DevArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int TR = a.tile_rows;
  const uint32_t cap = a.stage_bytes;
  const uint32_t per_wg = a.stage_tiles;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint32_t tile0 = blockIdx.x * per_wg;
  const uint32_t ntiles = min(per_wg, a.ntiles - tile0);

  // LDS: two stage buffers (16 bytes of slack around each), the run's tile table, three
  // metadata slots, the decoded tile's row layout
  uint8_t* const stage[2] = {smem + 16, smem + 16 + cap + 32};
  TileDesc* s_td = reinterpret_cast<TileDesc*>(smem + 2 * (cap + 32));
  uint32_t* meta_base = reinterpret_cast<uint32_t*>(s_td + per_wg);
  const uint32_t mw = meta_slot_words(TR);
  auto meta = [&](uint32_t k) {
    uint32_t* p = meta_base + (k % kMetaSlots) * mw;
    return MetaSlot{p, p + (mw - 128), p + (mw - 64)};
  };
  RowLds R;
  R.dst = reinterpret_cast<int64_t*>(meta_base + kMetaSlots * mw);
  R.rel = reinterpret_cast<uint32_t*>(R.dst + a.nvar * TR);
  R.len = R.rel + a.ncols * TR;
  R.src = reinterpret_cast<int32_t*>(R.len + a.nvar * TR);
  R.rdst = reinterpret_cast<uint32_t*>(R.src + a.ncols * TR);
  R.ok = reinterpret_cast<uint8_t*>(R.rdst + a.ncols * TR);
  __shared__ uint32_t s_lo[2], s_fits[2];
  __shared__ uint32_t s_first, s_gend, s_ghi;
  // the column table in LDS: kernel-argument fields indexed by a loop variable compile to vector
  // loads, whose waits (vmcnt) would also wait for the consumers' stores in flight
  __shared__ DevCol s_cols[MDSX_MAX_COLUMNS];
  const MDSX_L DevCol* cols = (const MDSX_L DevCol*)s_cols;
  for (int c = t; c < a.ncols; c += kStageBlock) s_cols[c] = a.cols[c];

  // ---- the run's tiles (plain loads, before any LDS-DMA is in flight)
  for (uint32_t k = uint32_t(t); k < ntiles; k += kStageBlock) {
    const uint32_t tile = tile0 + k;
    const uint32_t si = a.tile_shard[tile];
    const mdsx_shard_desc d = a.shards[si];
    TileDesc td;
    td.shard_off = d.offset;
    td.r0 = (tile - d.tile0) * uint32_t(TR);
    td.nrows = d.samples > td.r0 ? min(uint32_t(TR), d.samples - td.r0) : 0u;
    td.row0 = d.row0 + td.r0;
    td.bytes = uint32_t(min(d.bytes, uint64_t(0xffffffffu)));
    td.samples = d.samples;
    td.shard = int32_t(si);
    td.table_ok = 4ull + 4ull * (uint64_t(d.samples) + 1ull) <= d.bytes ? 1u : 0u;
    s_td[k] = td;
    // header written by encode_joint_shard (mds/writer.py:133-144): u32 N, then N+1 offsets
    if (tile == d.tile0) {
      const uint8_t* shard = a.batch + d.offset;
      const uint32_t* offs = reinterpret_cast<const uint32_t*>(shard + 4);
      if (!td.table_ok || *reinterpret_cast<const uint32_t*>(shard) != d.samples ||
          offs[0] < 4ull + 4ull * (uint64_t(d.samples) + 1ull) || offs[d.samples] > d.bytes)
        report_decode(a, MDSX_E_HEADER, int(si), -1, -1);
    }
  }
  __syncthreads();

  const uint32_t stage_lds[2] = {lds_addr(stage[0]), lds_addr(stage[1])};
  // ---- prologue (loader): metadata of tiles 0 and 1, the bytes of tile 0
  if (wave == 0) {
    load_meta(a, s_td[0], tile0, meta(0), lane);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t lo, hi;
    bool fits;
    tile_span(s_td[0], meta(0), cap, lane, &lo, &hi, &fits);
    if (fits) load_bytes<kNT>(a.batch + s_td[0].shard_off, lo, hi, stage_lds[0], lane);
    if (lane == 0) s_lo[0] = lo, s_fits[0] = fits;
    if (ntiles > 1) load_meta(a, s_td[1], tile0 + 1, meta(1), lane);
  }

  // measurement only (stage_debug & 16): cycles per phase, summed over the workgroups by the
  // loader's lane 0 (slot 0: its wait for the DMA) and the first consumer (slots 1-6)
  const bool timed = (a.stage_debug & 16) != 0;
  uint64_t ph[7] = {0, 0, 0, 0, 0, 0, 0};
  uint64_t last = timed ? __builtin_readcyclecounter() : 0;
  auto stamp = [&](int i) {
    if (timed) {
      const uint64_t now = __builtin_readcyclecounter();
      ph[i] += now - last;
      last = now;
    }
  };
  for (uint32_t k = 0; k < ntiles; ++k) {
    // the bytes of tile k and the metadata of tile k + 1 have landed (the loader's loads; the
    // consumers' stores stay in flight)
    if (wave == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (wave == 0) stamp(0);
    __syncthreads();
    if (wave > 0) stamp(6);
    const uint32_t sb = k & 1;
    const TileDesc td = s_td[k];
    const MetaSlot m = meta(k);
    const int n = td.table_ok ? int(td.nrows) : 0;
    const lds_u8* st = (const lds_u8*)(stage[sb]);
    const uint32_t lo = s_lo[sb];
    const bool fits = s_fits[sb] != 0;
    if (wave == 0) {  // loader: tile k + 1's bytes, tile k + 2's metadata
      if (k + 1 < ntiles) {
        uint32_t nlo, nhi;
        bool nfits;
        tile_span(s_td[k + 1], meta(k + 1), cap, lane, &nlo, &nhi, &nfits);
        if (nfits && !(a.stage_debug & 1))
          load_bytes<kNT>(a.batch + s_td[k + 1].shard_off, nlo, nhi, stage_lds[sb ^ 1], lane);
        if (lane == 0) s_lo[sb ^ 1] = nlo, s_fits[sb ^ 1] = nfits;
      }
      if (k + 2 < ntiles) load_meta(a, s_td[k + 2], tile0 + k + 2, meta(k + 2), lane);
    }
    if (a.stage_debug & 8) {  // measurement only: skip the tile's decode
      __syncthreads();
      continue;
    }

    // ---- 1. ranges and column layout: from the stage, or (a tile larger than a stage buffer)
    // from HBM
    for (int r = t - 64; r >= 0 && r < n; r += kConsumers) {
      uint32_t b, e;
      const int rc = row_range(td, m, r, &b, &e);
      R.ok[r] = 1;
      const uint8_t* sample = a.batch + td.shard_off + b;
      if (rc != MDSX_OK) {
        fail_row(a, td, R, TR, r, rc);
      } else if (fits ? !row_layout(a, cols, R, TR, r, uint64_t(e - b),
                                    [&](int vi) { return lds_u32(st, b - lo + 4u * vi); })
                      : !row_layout(a, cols, R, TR, r, uint64_t(e - b), [&](int vi) {
                          return load_u32_any(sample + 4u * uint32_t(vi));
                        })) {
        fail_row(a, td, R, TR, r, MDSX_E_BOUNDS);
      }
    }
    __syncthreads();
    stamp(1);
    // ---- 2. ragged offsets
    tile_offsets(a, cols, td, R, m, TR);
    stamp(2);
    if (fits) {
      place_rows(a, cols, td, R, m, TR, lo, 0, n);
      __syncthreads();
      stamp(3);
      // ---- 3. columns; 4. UTF-8
      if (n && wave > 0) {
        if (!(a.stage_debug & 2)) write_columns<kNT>(a, cols, td, R, TR, st, 0, n);
        stamp(4);
        if (!(a.stage_debug & 4)) check_utf8(a, cols, td, R, TR, st, 0, n);
        stamp(5);
      }
    } else {
      // ---- a tile larger than a stage buffer: row groups that fit, loaded synchronously into
      // this tile's buffer (tile k + 1's stays in flight)
      for (int ga = 0; ga < n;) {  // block-uniform loop over row groups
        if (t == 0) s_first = uint32_t(n), s_gend = uint32_t(n), s_ghi = 0;
        __syncthreads();
        for (int r = t; r < n; r += kStageBlock)
          if (r >= ga && R.ok[r]) atomicMin(&s_first, uint32_t(r));
        __syncthreads();
        const int first = int(s_first);
        const uint32_t glo = first < n ? (m.offs[first] & ~15u) : 0u;
        for (int r = t; r < n; r += kStageBlock)
          if (r >= ga && R.ok[r] && !(m.offs[r] >= glo && m.offs[r + 1] - glo <= cap))
            atomicMin(&s_gend, uint32_t(r));
        __syncthreads();
        const int gb = int(s_gend);
        if (gb == ga) {  // row ga alone is larger than the stage: stage_huge_kernel's
          if (t == 64) {  // a consumer: the loader wave stores nothing
            uint32_t* count = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(a.status) +
                                                          kHugeCountOffset);
            a.src_abs[atomicAdd(count, 1u)] = (uint64_t(tile0 + k) << 32) | uint32_t(ga);
          }
          ++ga;
          __syncthreads();  // every thread has read s_first / s_gend before they are reset
          continue;
        }
        for (int r = t; r < gb; r += kStageBlock)
          if (r >= ga && R.ok[r]) atomicMax(&s_ghi, (m.offs[r + 1] + 15u) & ~15u);
        __syncthreads();
        const uint32_t ghi = first < gb ? s_ghi : glo;
        if (wave == 0) {
          load_bytes<kNT>(a.batch + td.shard_off + glo, 0, ghi - glo, stage_lds[sb], lane);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        place_rows(a, cols, td, R, m, TR, glo, ga, gb);
        __syncthreads();
        if (wave > 0) {
          write_columns<kNT>(a, cols, td, R, TR, st, ga, gb);
          check_utf8(a, cols, td, R, TR, st, ga, gb);
        }
        __syncthreads();  // the buffer is refilled by the next group
        ga = gb;
      }
    }
    __syncthreads();  // stage buffer sb and metadata slot k are refilled from the next tile on
  }
  if (timed && (t == 0 || t == 64)) {
    unsigned long long* acc = reinterpret_cast<unsigned long long*>(
        reinterpret_cast<uint8_t*>(a.status) + kStageTimeOffset);
    for (int i = t == 0 ? 0 : 1; i < (t == 0 ? 1 : 7); ++i) atomicAdd(acc + i, ph[i]);
  }
}

}  // namespace

size_t stage_lds_bytes(const mdsx_plan* plan, int tile_rows, uint32_t stage_bytes,
                       uint32_t tiles_per_wg) {
  const size_t bytes = 2 * (size_t(stage_bytes) + 32) + sizeof(TileDesc) * tiles_per_wg +
                       4 * size_t(kMetaSlots) * meta_slot_words(tile_rows) +
                       row_lds_bytes(tile_rows, plan->ncols, plan->nvar);
  return (bytes + 15) & ~size_t(15);
}

// Tiles per workgroup of the staged decode: runs long enough for the pipeline to fill, and
// enough workgroups (>= ~16 per CU) to balance the tail.
uint32_t stage_tiles_per_wg(uint32_t ntiles) {
  return std::max<uint32_t>(1, std::min<uint32_t>(64, ntiles / 4096));
}

int launch_stage_totals(const DevArgs& a, hipStream_t s, bool chained) {
  const unsigned grid = unsigned((uint64_t(a.ntiles) * a.tile_rows + kBlock - 1) / kBlock);
  if (chained)
    hipLaunchKernelGGL((stage_totals_kernel<true>), dim3(grid), dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((stage_totals_kernel<false>), dim3(grid), dim3(kBlock), 0, s, a);
  return hip_check(hipGetLastError(), "stage_totals_kernel launch");
}

int launch_stage_decode(const mdsx_plan* plan, const DevArgs& a, hipStream_t s) {
  // the huge-row count and (measurement only) the phase cycle sums
  int rc = hip_check(hipMemsetAsync(reinterpret_cast<uint8_t*>(a.status) + kHugeCountOffset, 0,
                                    kStatusBlock - kHugeCountOffset, s),
                     "hipMemsetAsync");
  if (rc != MDSX_OK) return rc;
  const size_t lds = stage_lds_bytes(plan, a.tile_rows, a.stage_bytes, a.stage_tiles);
  const void* fn = plan->nontemporal ? reinterpret_cast<const void*>(stage_decode_kernel<true>)
                                     : reinterpret_cast<const void*>(stage_decode_kernel<false>);
  if (lds > 64 * 1024) {  // above the default dynamic-LDS limit of a launch
    rc = hip_check(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)),
                   "hipFuncSetAttribute");
    if (rc != MDSX_OK) return rc;
  }
  const unsigned grid = (a.ntiles + a.stage_tiles - 1) / a.stage_tiles;
  if (plan->nontemporal) {
    mdsx::set_last_kernel("stage_decode_kernel<true>");
    hipLaunchKernelGGL((stage_decode_kernel<true>), dim3(grid), dim3(kStageBlock), lds, s, a);
  } else {
    mdsx::set_last_kernel("stage_decode_kernel<false>");
    hipLaunchKernelGGL((stage_decode_kernel<false>), dim3(grid), dim3(kStageBlock), lds, s, a);
  }
  rc = hip_check(hipGetLastError(), "stage_decode_kernel launch");
  if (rc != MDSX_OK) return rc;
  return launch_huge_rows(a, plan->nontemporal != 0, s);
}

int launch_huge_rows(const DevArgs& a, bool nt, hipStream_t s) {
  // one workgroup per listed row, 1024 at a time (usually none are listed)
  const unsigned hgrid = unsigned(std::min<uint64_t>(a.ntiles, 1024));
  if (nt)
    hipLaunchKernelGGL((stage_huge_kernel<true>), dim3(hgrid), dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL((stage_huge_kernel<false>), dim3(hgrid), dim3(kBlock), 0, s, a);
  return hip_check(hipGetLastError(), "stage_huge_kernel launch");
}

}  // namespace mdsx_kernels
