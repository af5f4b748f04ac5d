// Row-parallel decode of ragged plans with short samples (gfx950): a workgroup decodes one tile
// -- up to 256 consecutive samples of one shard -- from a single LDS copy of the tile's bytes, one
// thread per sample for the per-sample work and one thread per 16-byte output chunk for the copy.
//
// The reference decodes one sample per call (MDSReader.get_sample_data, mds/reader.py:128-149;
// decode_sample, :103-126; mds_decode, encodings.py:760-773). The samples of a tile are one
// contiguous byte range of the shard (sample i ends where i + 1 starts), so the workgroup
//   1. copies the range into LDS once (global_load_lds_dwordx4, 1 KiB per wave-instruction, the
//      range started on a 128-byte line). A tile the scan pass found clean and small enough
//      (its TileRun record, stage_totals_kernel) is copied straight from that record, in flight
//      together with the tile's offsets;
//   2. parses each sample's size heads and column boundaries from LDS, one thread per sample
//      (decode_sample's head loop; a sample whose offsets or columns do not fit counts zero
//      bytes and is reported, the scan pass's rule);
//   3. scans the ragged lengths across the tile (one block scan per pair of ragged columns, the
//      two 32-bit sums packed in one 64-bit word) onto the tile's output base (from the scan
//      pass), writes the offsets, and marks which sample holds the first byte of every output
//      chunk (the chunk map);
//   4. writes every column output-chunk-parallel: consecutive threads assemble consecutive
//      16-byte chunks of the column's output from LDS (unaligned ds_read_b128; a chunk spanning
//      several samples takes a piece of each) and store them whole; only the chunks a tile
//      shares with its neighbours are stored a byte at a time. The pieces of str values are
//      checked for strict UTF-8 on the way (what bytes.decode('utf-8') accepts,
//      encodings.py:80-81; the dword before a piece comes from the same value), a failing piece
//      marks its sample, and each sample's flag is written at the end.
// Per-sample work is spread over lanes, not looped over by one wave: the per-sample scalar
// control of the streaming decode (mdsx_run.hip) is what bounds short samples there.
//
// A tile whose range exceeds the LDS stage is decoded in windows of samples that fit, each window
// a tile of its own for the edge chunks; a sample larger than the stage is listed for the
// huge-row kernel (stage_huge_kernel, straight from HBM) once its offsets are written.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "mdsx_decode.h"
#include "mdsx_device.h"
#include "mdsx_internal.h"
#include "mdsx_ring.h"

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

// A u32 of the stage at an arbitrary byte position (unaligned ds_read_b32).
__device__ __forceinline__ uint32_t lds_u32(const lds_u8* p) { return *(const MDSX_L uint32_t*)p; }

// Bytes [from, to) (0 <= from <= to <= 16) of chunk v stored at the aligned address D.
__device__ __forceinline__ void store_bytes(uint64_t D, const uint4 v, uint32_t from, uint32_t to) {
  for (uint32_t b = from; b < to; ++b) *gp_at<uint8_t>(D + b) = uint8_t(byte_of(v, int(b)));
}

__host__ __device__ __forceinline__ uint32_t rows_map_len(uint32_t cap) { return cap / 16 + 4; }

// LDS of one workgroup: the stage, then per-column tables of the window ([ncols][TR] output
// byte of the value inside the window's output, stage byte, length), the UTF-8 marks ([ncols]
// [8] bits, one per sample) and the chunk maps ([nvar][map_len]: the sample holding the first
// window byte of each output chunk).
// (then, 16-byte aligned, the per-column workgroup state: write descriptors, column table, next
// output byte, window base and length, skip flag -- sized by ncols, so a narrow schema leaves room
// for more workgroups per CU)
__host__ __device__ __forceinline__ size_t rows_lds_tables(uint32_t cap, int TR, int ncols,
                                                           int nvar, int nstage) {
  return size_t(nstage) * (kStageFront + size_t(cap) + kStageSlack) +
         size_t(TR) * size_t(ncols) * 16 + size_t(ncols) * 32 + size_t(nvar) * rows_map_len(cap);
}
// One column's write descriptor: everything the write loop reads of the column, in one 32-byte
// record written once per window (one LDS round trip per chunk instead of the column table's,
// window base's and length's three: +0.8-1.3 % on short rows, profiles/r06/rows_var/).
struct __attribute__((aligned(16))) RowsDesc {
  uint64_t wout;  // the window's first output byte (absolute)
  uint32_t wlen;  // the window's output bytes
  uint32_t rb;    // fixed columns: bytes per row (ragged: 0)
  int32_t vi;     // ragged columns: the chunk map's index (fixed: 0)
  uint32_t utf8;  // str values checked
  uint32_t pad[2];
};

static_assert(sizeof(RowsDesc) == 32, "RowsDesc: two 16-byte LDS reads");

__host__ __device__ __forceinline__ size_t rows_lds_colstate(int ncols) {
  return size_t(ncols) * (sizeof(RowsDesc) + sizeof(DevCol) + 8 + 8 + 4 + 4 + 4);
}
__host__ __device__ __forceinline__ size_t rows_lds_bytes(uint32_t cap, int TR, int ncols,
                                                          int nvar, int nstage = 1) {
  return ((rows_lds_tables(cap, TR, ncols, nvar, nstage) + 15) & ~size_t(15)) +
         rows_lds_colstate(ncols);
}

template <bool kFence>
__device__ __forceinline__ void rows_barrier() {
  if constexpr (kFence) __syncthreads();
  else lds_barrier();
}

// Measurement only (MDSX_TUNE sdbg bit 64): shader-clock time of each phase of a tile (DMA wait;
// size heads + bounds; value records; scan + offsets + chunk maps; the barrier after them; column
// writes; flags), written by thread 0 of each tile's workgroup to src_abs[8 tile + k] (the
// huge-row list's space; plain stores, no shared counter).
__device__ __forceinline__ uint64_t shader_clock() {
  uint64_t c;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c)::"memory");
  return c;
}
__device__ __forceinline__ void prof_mark(const DevArgs& a, uint32_t tile, int k, uint64_t& ts) {
  const uint64_t now = shader_clock();
  if (threadIdx.x == 0) a.src_abs[8ull * tile + k] = now - ts;
  ts = now;
}

// The DMA of a clean run's bytes (its TileRun, stage_totals_kernel) into a stage: the range
// started on a 128-byte line, 1 KiB per wave-instruction, the waves taking turns.
template <bool kNT>
__device__ __forceinline__ void rows_dma(const DevArgs& a, const TileRun& run, uint32_t stage_lds,
                                         int wave, int lane) {
  const uint64_t lo_al = run.stream & ~uint64_t(127);
  const uint32_t nq = uint32_t((run.stream + run.bytes - lo_al + 15) >> 4);
  const uint4* src = reinterpret_cast<const uint4*>(a.batch + lo_al);
  for (uint32_t kb = uint32_t(wave); kb * 64 < nq; kb += kRowsBlock / 64) {
    const uint32_t k = kb * 64 + uint32_t(lane);
    if (k < nq) glds16<kNT>(src + k, stage_lds + kb * 1024u);  // lanes past nq write nothing
  }
}

// One value of the window: output byte inside the window's output of its column, bytes (0: a
// sample that failed a check), stage position of its first byte (read with one ds_read_b128).
struct RowsRec {
  uint32_t dst, len, src, pad;
};

struct RowsTab {
  MDSX_L RowsRec* rec;   // [ncols][TR]
  MDSX_L uint32_t* bad;  // [ncols][8]: UTF-8 failures of the tile's samples
  MDSX_L uint8_t* map;   // [nvar][map_len]
};

// Launch bound 4 waves per SIMD: the same 96 VGPRs as at 5 (occupancy is set by the LDS stage),
// scheduled 1.5 % faster on 32-256 and 256-1024-byte rows (two A/B runs); 6 spills (9 % slower).
//
// kPipe: the workgroup decodes a.rows_pipe consecutive tiles through two stages, the next clean
// tile's DMA (and its offsets) issued once this tile's column geometry is done, so it lands while
// this tile's columns are written; the barriers it crosses leave it in flight (lds_barrier).
// kFence (measurement only, MDSX_TUNE sdbg bit 128): __syncthreads() barriers, as before
// lds_barrier replaced them.
// kOcc: waves per SIMD the registers are bounded for (6: at most 80 VGPRs, so that six
// workgroups fit a CU where their LDS does).
// kFlat: the write loop over all columns' chunks at once (else one loop per column; measurement
// control, MDSX_TUNE sdbg bit 256).
template <bool kNT, bool kPipe, bool kProf = false, bool kFence = false, int kOcc = 4,
          bool kFlat = true>
__global__ __launch_bounds__(kRowsBlock, kOcc) void rows_decode_kernel(const DevArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ int64_t s_wsum[kRowsBlock / 64];
  __shared__ uint32_t s_gb, s_lo, s_hi;
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const uint32_t blk = (a.xcd_order & kXcdRows) ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const int TR = a.tile_rows;
  const int ncols = a.ncols, nvar = a.nvar;
  const uint32_t cap = a.rows_bytes;
  const uint32_t map_len = rows_map_len(cap);
  const uint32_t stage_stride = kStageFront + cap + kStageSlack;  // (16-byte multiple)
  constexpr int kStages = kPipe ? 2 : 1;
  RowsTab T;
  T.rec = (MDSX_L RowsRec*)(smem + kStages * stage_stride);
  T.bad = (MDSX_L uint32_t*)(T.rec + size_t(ncols) * TR);
  T.map = (MDSX_L uint8_t*)(T.bad + size_t(ncols) * 8);
  // the per-column workgroup state (rows_lds_colstate)
  MDSX_L uint8_t* cs = (MDSX_L uint8_t*)(
      smem + ((rows_lds_tables(cap, TR, ncols, nvar, kStages) + 15) & ~size_t(15)));
  MDSX_L RowsDesc* s_desc = (MDSX_L RowsDesc*)cs;
  MDSX_L DevCol* s_cols = (MDSX_L DevCol*)(s_desc + ncols);
  MDSX_L uint64_t* s_base = (MDSX_L uint64_t*)(s_cols + ncols);  // next output byte (rel. data)
  MDSX_L uint64_t* s_wbase = s_base + ncols;  // the window's first output byte (rel. data)
  MDSX_L uint32_t* s_wlen = (MDSX_L uint32_t*)(s_wbase + ncols);  // the window's output bytes
  MDSX_L uint32_t* s_skip = s_wlen + ncols;  // the tile's bytes exceed the column capacity
  MDSX_L uint32_t* s_ends = s_skip + ncols;  // the write loop's column ends (wide schemas)
  for (int c = t; c < ncols; c += kRowsBlock) s_cols[c] = a.cols[c];
  const MDSX_L DevCol* cols = s_cols;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((const MDSX_L uint8_t*)(smem + kStageFront))));
  const uint32_t per = kPipe ? a.rows_pipe : 1u;
  const uint32_t first = blk * per;
  const uint32_t last = kPipe ? min(first + per, a.ntiles) : first + 1u;
  auto fits = [&](const TileRun& r) { return r.fast && (r.stream & 127) + r.bytes <= cap; };
  // kPipe: whether the current tile's bytes and offsets are already on their way (prefetched)
  bool pre = false;
  uint32_t pb = 0, pe = 0;  // its offsets pair (this thread's sample)
  if constexpr (kPipe) {
    const TileRun r0_ = a.tile_run[first];
    if (fits(r0_)) {
      rows_dma<kNT>(a, r0_, lds0, wave, lane);
      if (t < int(r0_.nrows)) {
        const uint32_t* o = reinterpret_cast<const uint32_t*>(a.batch + r0_.offs);
        pb = o[t];
        pe = o[t + 1];
      }
      pre = true;
    }
  }

  uint32_t count = kPipe ? last - first : 1u;  // (1: the loop folds away)
  for (uint32_t it = 0; it < count; ++it) {  // block-uniform
  const uint32_t tile = first + it;
  const uint32_t sbuf = kPipe ? it & 1u : 0u;
  const lds_u8* stage = (const lds_u8*)(smem + kStageFront + sbuf * stage_stride);
  const uint32_t stage_lds = lds0 + sbuf * stage_stride;
  if (kPipe && it != 0) {
    // the previous tile's readers of the tables are done (its end barrier); its stores, this
    // tile's DMA and offsets retire here
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    rows_barrier<kFence>();
  }
  for (int i = t; i < ncols * 8; i += kRowsBlock) T.bad[i] = 0;
  constexpr bool prof = kProf;
  uint64_t ts = prof ? shader_clock() : 0;

  // ---- the tile: its run record (scan pass) or its shard's view
  const TileRun run = a.tile_run[tile];
  const bool fast = fits(run);  // block-uniform
  const uint8_t* frame;  // b / e below are byte positions relative to frame
  int n;
  uint64_t row0;
  uint32_t shard_idx, r0;
  uint32_t b = 0, e = 0;
  bool in_range = false;
  if (fast) {
    // one window: the DMA of the run's bytes goes out with the offsets loads
    n = run.nrows;
    row0 = run.row0;
    shard_idx = run.shard;
    r0 = run.r0;
    frame = a.batch + run.shard_off;
    if (kPipe && pre) {
      b = pb;
      e = pe;
    } else {
      rows_dma<kNT>(a, run, stage_lds, wave, lane);
      if (t < n) {
        const uint32_t* o = reinterpret_cast<const uint32_t*>(a.batch + run.offs);
        b = o[t];
        e = o[t + 1];
      }
    }
    in_range = t < n;  // run.fast: every sample of the run passed the file checks
  } else {
    const TileView v = tile_view(a, tile);
    if (!v.table_ok) {  // block-uniform; reported by the scan pass
      if constexpr (!kPipe) return;
      pre = false;  // (nothing was prefetched for the next tile either)
      continue;
    }
    n = int(v.nrows);
    row0 = v.d.row0 + v.r0;
    shard_idx = v.shard_idx;
    r0 = v.r0;
    frame = v.shard;
    int rc = MDSX_OK;
    if (t < n) rc = sample_range(v, v.r0 + uint32_t(t), &b, &e);
    in_range = t < n && rc == MDSX_OK;
    if (t < n && rc != MDSX_OK) report_decode(a, rc, shard_idx, int(r0 + t), -1);
  }
  if (t < ncols) {
    const MDSX_L DevCol& col = cols[t];
    const int vi = col.var_index;
    uint32_t skip = 0;
    if (vi >= 0) {
      const uint64_t off = uint64_t(a.tile_prefix[uint64_t(vi) * a.nscan + tile]);
      s_base[t] = off;
      if (off + uint64_t(a.tile_total[uint64_t(vi) * a.nscan + tile]) > col.capacity) {
        report_decode(a, MDSX_E_CAPACITY, shard_idx, int(r0), t);
        skip = 1;
      }
    }
    s_skip[t] = skip;
  }

  for (int ga = 0; ga < n;) {  // block-uniform loop over windows
    // ---- the window: samples [ga, gb) whose bytes lie in [lo, lo + cap)
    int gb;
    uint32_t lo_al;  // stage byte 0 = frame byte lo_al
    bool direct = false;
    if (fast) {
      gb = n;
      lo_al = uint32_t((run.stream & ~uint64_t(127)) - run.shard_off);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      rows_barrier<kFence>();  // the previous window's readers of the stage and the tables are done
      if (t == 0) s_gb = uint32_t(n), s_lo = 0xffffffffu, s_hi = 0;
      rows_barrier<kFence>();
      if (t >= ga && in_range) atomicMin(&s_lo, b);  // the window's first in-range byte
      rows_barrier<kFence>();
      const uint32_t lo = s_lo;
      if (t >= ga && in_range && !(b >= lo && e - lo <= cap)) atomicMin(&s_gb, uint32_t(t));
      rows_barrier<kFence>();
      gb = int(s_gb);
      direct = gb == ga;  // sample ga alone is larger than the stage: the huge-row kernel's
      if (direct) gb = ga + 1;
      lo_al = lo & ~127u;
      // ---- 1. the window's bytes [lo_al, hi) into LDS, hi the largest end of its samples
      if (t >= ga && t < gb && in_range) atomicMax(&s_hi, e);
      rows_barrier<kFence>();
      const uint32_t hi = s_hi;
      if (!direct && lo != 0xffffffffu && hi > lo_al) {
        const uint32_t nq = (hi - lo_al + 15) >> 4;
        const uint4* src = reinterpret_cast<const uint4*>(frame + lo_al);
        for (uint32_t kb = uint32_t(wave); kb * 64 < nq; kb += kRowsBlock / 64) {
          const uint32_t k = kb * 64 + uint32_t(lane);
          if (k < nq) glds16<kNT>(src + k, stage_lds + kb * 1024u);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
    }
    rows_barrier<kFence>();
    if constexpr (prof) prof_mark(a, tile, 0, ts);

    // ---- 2. column boundaries of this thread's sample (mds/reader.py:111-125)
    const bool mine = t >= ga && t < gb;
    const uint32_t sp = b - lo_al;  // stage position of the sample (not direct)
    // the column table lane-distributed (lane c: column c), read by readlane in the uniform
    // column loops below instead of an LDS round trip per column; up to four size heads read at
    // once (one unaligned ds_read_b128)
    const int lvi = lane < ncols ? int(cols[lane].var_index) : -1;
    const uint32_t lrb = lane < ncols ? cols[lane].row_bytes : 0u;
    uint4 h4 = make_uint4(0, 0, 0, 0);
    if (mine && in_range && !direct && nvar <= 4) h4 = lds_read16(stage + sp);
    auto head = [&](int vi) -> uint32_t {
      if (!direct && nvar <= 4)
        return vi == 0 ? h4.x : vi == 1 ? h4.y : vi == 2 ? h4.z : h4.w;
      return direct ? load_u32_any(frame + b + 4u * uint32_t(vi))
                    : lds_u32(stage + sp + 4u * uint32_t(vi));
    };
    bool ok = mine && in_range;
    uint64_t need = 4ull * uint64_t(nvar);
    if (ok && need > e - b) ok = false;
    // (the column facts are read across lanes here, where every lane is active; only the size
    // heads are read under the per-sample condition)
    for (int c = 0; c < ncols; ++c) {
      const int vi = __builtin_amdgcn_readlane(lvi, c);
      const uint32_t rbc = uint32_t(__builtin_amdgcn_readlane(int(lrb), c));
      uint32_t add = rbc;
      if (vi >= 0) add = ok ? head(vi) : 0u;
      need += add;
    }
    if (ok && need > e - b) ok = false;
    if (mine && in_range && !ok) report_decode(a, MDSX_E_BOUNDS, shard_idx, int(r0 + t), -1);
    if constexpr (prof) prof_mark(a, tile, 1, ts);
    // ---- 3. value lengths and stage positions; fixed columns' window output
    {
      uint32_t rel = 4u * uint32_t(nvar);
      for (int c = 0; c < ncols; ++c) {
        const int vi = __builtin_amdgcn_readlane(lvi, c);
        const uint32_t rb = uint32_t(__builtin_amdgcn_readlane(int(lrb), c));
        const uint32_t len = ok ? (vi >= 0 ? head(vi) : rb) : 0u;
        if (mine) {
          T.rec[c * TR + t].len = len;
          T.rec[c * TR + t].src = (direct ? 0u : sp) + rel;
          if (vi < 0) T.rec[c * TR + t].dst = uint32_t(t - ga) * rb;
        }
        if (vi < 0 && t == 0) {
          s_wbase[c] = (row0 + uint64_t(ga)) * rb;
          s_wlen[c] = uint32_t(gb - ga) * rb;
        }
        rel += len;
      }
    }
    if constexpr (prof) prof_mark(a, tile, 2, ts);
    // ragged lengths scanned across the window onto each column's base, two columns per scan;
    // offsets; chunk maps
    for (int c0 = 0; c0 < ncols;) {
      int c1 = c0;
      while (c1 < ncols && cols[c1].var_index < 0) ++c1;
      if (c1 >= ncols) break;
      int c2 = c1 + 1;
      while (c2 < ncols && cols[c2].var_index < 0) ++c2;
      const bool pair = c2 < ncols;
      const uint64_t len1 = mine ? T.rec[c1 * TR + t].len : 0u;
      const uint64_t len2 = (mine && pair) ? T.rec[c2 * TR + t].len : 0u;
      const uint64_t base1 = s_base[c1], base2 = pair ? s_base[c2] : 0;
      int64_t total, excl;
      // each half sums at most the window's bytes (< 2^32): no carry between the halves
      const int64_t x = int64_t(len1 | (len2 << 32));
      if (TR <= 64) {  // block-uniform: every sample of the tile is in wave 0 -- no barriers
        const uint32_t i1 = wave_incl_dpp(uint32_t(len1)), i2 = wave_incl_dpp(uint32_t(len2));
        excl = int64_t((uint64_t(i2 - uint32_t(len2)) << 32) | (i1 - uint32_t(len1)));
        total = int64_t((uint64_t(uint32_t(__builtin_amdgcn_readlane(int(i2), 63))) << 32) |
                        uint32_t(__builtin_amdgcn_readlane(int(i1), 63)));
      } else {
        excl = block_exclusive_scan<!kFence>(x, s_wsum, &total);
      }
      for (int h = 0; h < (pair ? 2 : 1); ++h) {
        const int c = h ? c2 : c1;
        const MDSX_L DevCol& col = cols[c];
        const uint32_t dst = uint32_t(uint64_t(excl) >> (32 * h));
        const uint32_t len = uint32_t(h ? len2 : len1);
        const uint64_t base = h ? base2 : base1;
        if (mine) {
          *gp(col.offsets + row0 + t) = int64_t(base + dst);
          T.rec[c * TR + t].dst = dst;
          if (len && !direct) {
            // chunk k of the window's output begins at window byte 16 k - head (head: the
            // window's misalignment); this sample holds the first byte of chunks [k0, k1)
            const uint32_t hd = uint32_t((reinterpret_cast<uint64_t>(col.data) + base) & 15);
            const uint32_t k0 = dst == 0 ? 0u : (dst + hd + 15) >> 4;
            const uint32_t k1 = (dst + len + hd + 15) >> 4;
            MDSX_L uint8_t* mp = T.map + size_t(col.var_index) * map_len;
            for (uint32_t k = k0; k < k1; ++k) mp[k] = uint8_t(t);
          }
        }
        if (t == 0) {
          const uint32_t tot = uint32_t(uint64_t(total) >> (32 * h));
          s_wbase[c] = base;
          s_wlen[c] = tot;
          s_base[c] = base + tot;
        }
      }
      c0 = pair ? c2 + 1 : c1 + 1;
    }
    // the columns' write descriptors (wave 0 only: its thread 0 wrote s_wbase / s_wlen above, and
    // one wave's LDS accesses take effect in program order; the barrier below publishes them)
    if (t < 64) {
      for (int c = t; c < ncols; c += 64) {
        const MDSX_L DevCol& col = cols[c];
        RowsDesc d;
        d.wout = reinterpret_cast<uint64_t>(col.data) + s_wbase[c];
        d.wlen = s_wlen[c];
        d.rb = col.var_index >= 0 ? 0u : col.row_bytes;
        d.vi = col.var_index >= 0 ? col.var_index : 0;
        d.utf8 = col.kind == MDSX_KIND_STR && col.flags != nullptr && !(a.stage_debug & 1);
        d.pad[0] = d.pad[1] = 0;
        s_desc[c] = d;
      }
    }
    if (direct && t == ga && ok) {  // copied by the huge-row kernel after this one
      if constexpr (prof) {
        // the stamps take the huge-row list's space: a batch with huge rows is refused there
        report_decode(a, MDSX_E_ARG, int(shard_idx), int(r0 + t), -1);
      } else {
        uint32_t* count = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(a.status) +
                                                      kHugeCountOffset);
        const uint32_t slot = atomicAdd(count, 1u);
        a.src_abs[slot] = (uint64_t(tile) << 32) | uint32_t(t);
      }
    }
    if constexpr (prof) prof_mark(a, tile, 3, ts);
    rows_barrier<kFence>();
    if constexpr (prof) prof_mark(a, tile, 4, ts);
    if constexpr (kPipe) {
      // the next clean tile's bytes and offsets, into the other stage (last read by the tile
      // before this one, whose readers passed this tile's first barrier), while this one's
      // columns are written
      if (gb == n) {
        pre = false;
        if (tile + 1 < last) {
          const TileRun nx = a.tile_run[tile + 1];
          if (fits(nx)) {
            rows_dma<kNT>(a, nx, lds0 + (sbuf ^ 1u) * stage_stride, wave, lane);
            if (t < int(nx.nrows)) {
              const uint32_t* o = reinterpret_cast<const uint32_t*>(a.batch + nx.offs);
              pb = o[t];
              pe = o[t + 1];
            }
            pre = true;
          }
        }
      }
    }

    // ---- 4. every column, output-chunk-parallel, str pieces checked on the way
    if (!direct) {
      // kFlat: the columns' output chunks as one index space -- consecutive threads take
      // consecutive chunks across the column ends, so a tile's writes take the fewest rounds of
      // the (latency-bound) chunk loop; lane c counts column c's chunks. Else a loop per column.
      // The loop is divergent (a lane leaves it after its last chunk), so nothing inside it reads
      // across lanes: a VGPR's inactive lanes are not preserved by the compiler (a spill reload or
      // a copy under a partial exec mask writes the active lanes only -- a 64-VGPR build faulted
      // reading the column ends with v_readlane inside the loop). The column ends
      // are read here, every lane active, into scalar registers (up to kEnds of them) or, for
      // wider schemas, into LDS (streaming_amd/isa_check.py checks the built code).
      constexpr int kEnds = 8;
      uint32_t total = 0;
      uint32_t ends[kEnds];
      if constexpr (kFlat) {
        // (a column with no bytes in the window has no chunks: a misaligned empty window would
        // otherwise count one, whose chunk-map entry no sample wrote)
        uint32_t cn = 0;
        if (lane < ncols && !s_skip[lane] && s_wlen[lane] != 0) {
          const uint64_t w = reinterpret_cast<uint64_t>(cols[lane].data) + s_wbase[lane];
          cn = uint32_t(((w & 15) + s_wlen[lane] + 15) >> 4);
        }
        const uint32_t cincl = wave_incl_u32(cn, lane, ncols);
#pragma unroll
        for (int j = 0; j < kEnds; ++j)
          ends[j] = j + 1 < ncols ? uint32_t(__builtin_amdgcn_readlane(int(cincl), j)) : ~0u;
        if (ncols > kEnds + 1 && lane < ncols) s_ends[lane] = cincl;  // (this wave reads its own)
        total = (a.stage_debug & 2) ? 0u : uint32_t(__builtin_amdgcn_readlane(int(cincl), ncols - 1));
      }
      for (int cl = 0; cl < (kFlat ? 1 : ncols); ++cl) {
        if (!kFlat && s_skip[cl]) continue;  // block-uniform
        const uint32_t kend = kFlat ? total
                                    : (a.stage_debug & 2) || s_wlen[cl] == 0 ? 0u
                                    : uint32_t(((((reinterpret_cast<uint64_t>(cols[cl].data) +
                                                   s_wbase[cl]) & 15) + s_wlen[cl] + 15) >> 4));
        for (uint32_t kw = uint32_t(t); kw < kend; kw += kRowsBlock) {
        const uint32_t kg = kw;
        // the chunk's column c and its index k inside the column
        int c = cl;
        uint32_t c0 = 0;
        if constexpr (kFlat) {
          if (ncols <= kEnds + 1) {  // uniform: the ends in scalar registers
#pragma unroll
            for (int j = 0; j < kEnds; ++j) {
              if (j + 1 >= ncols) break;  // (uniform: a narrow schema compares ncols - 1 ends)
              if (kg >= ends[j]) c = j + 1, c0 = ends[j];
            }
          } else {
            for (int j = 0; j + 1 < ncols; ++j) {
              const uint32_t e = s_ends[j];
              if (kg >= e) c = j + 1, c0 = e;
            }
          }
        }
        const uint32_t k = kg - c0;
        const int base = c * TR;
        // (measurement only, MDSX_TUNE sdbg: 1 no UTF-8 check, 2 no copy, 16 no stores)
        const RowsDesc d = s_desc[c];
        const bool utf8 = d.utf8 != 0;
        const uint64_t wout = d.wout;
        const uint32_t wlen = d.wlen, rb = d.rb;
        const MDSX_L uint8_t* mp = T.map + size_t(d.vi) * map_len;
        const uint64_t D0 = wout & ~uint64_t(15);
        const int32_t hd = int32_t(wout - D0);
        MDSX_L uint32_t* bad = T.bad + c * 8;
        {
          const int32_t P0 = int32_t(k * 16) - hd;  // window output byte of the chunk's byte 0
          int32_t pos = max(P0, 0);
          const int32_t end = min(P0 + 16, int32_t(wlen));
          const int r = rb ? ga + int(uint32_t(pos) / rb) : int(mp[k]);
          // the common chunk: one value (A) or two (A, then B from byte sB), straight-line
          const RowsRec qa = T.rec[base + r];
          const int32_t dsA = int32_t(qa.dst), deA = dsA + int32_t(qa.len);
          const lds_u8* pa = stage + (int32_t(qa.src) - dsA + P0);
          uint4 val = lds_read16(pa);
          const int32_t hiA = min(end, deA);
          bool simple = deA > pos;  // (a fixed column's failed sample: no bytes)
          uint32_t sB = 16;
          int32_t deL = deA;  // end of the chunk's last value
          if (simple && hiA < end) {
            const RowsRec qb = T.rec[base + r + 1];
            const int32_t dsB = int32_t(qb.dst), deB = dsB + int32_t(qb.len);
            simple = dsB == hiA && deB >= end;
            if (simple) {
              const uint4 vb = lds_read16(stage + (int32_t(qb.src) - dsB + P0));
              sB = uint32_t(hiA - P0);
              const uint4 m = byte_mask(0, sB);
              val = make_uint4((val.x & m.x) | (vb.x & ~m.x), (val.y & m.y) | (vb.y & ~m.y),
                               (val.z & m.z) | (vb.z & ~m.z), (val.w & m.w) | (vb.w & ~m.w));
              deL = deB;
            }
          }
          if (simple) {
            if (utf8) {
              // the chunk's bytes (others zero), A's dword before the chunk (bytes before A's
              // start zero); each value checked in its own context (utf8_chunk_err2); A's end at
              // sB and a value ending at the chunk's end checked for an open sequence
              const uint4 X = (pos > P0 || end < P0 + 16)
                                  ? keep_bytes(val, uint32_t(pos - P0), uint32_t(end - P0))
                                  : val;
              uint32_t pw = 0;
              if (pos > dsA) {
                pw = lds_u32(pa + (pos - P0) - 4);
                const int32_t nv = pos - dsA;  // A's bytes before the chunk
                if (nv < 4) pw &= ~((1u << (8 * (4 - nv))) - 1u);
              }
              // a chunk of ASCII with no lead byte before it cannot err, and no sequence is open
              // at its values' ends: the check is skipped when that holds for the whole wave
              // (measurement knob sdbg 32: always check)
              const bool plain = (((X.x | X.y | X.z | X.w) & 0x80808080u) | hi_c0(pw)) == 0;
              if (!__all(plain) || (a.stage_debug & 32)) {
                uint32_t e = utf8_chunk_err2(X, pw, sB);
                if (sB < 16 && utf8_open_at(X, pw, sB)) e |= 1u;
                if (end == P0 + 16 && end == deL) {
                  if (sB < 16) e |= utf8_open_at(keep_bytes(X, sB, 16), 0, 16) ? 2u : 0u;
                  else e |= utf8_open_at(X, pw, 16) ? 1u : 0u;
                }
                if (e & 1u) atomicOr(&bad[r >> 5], 1u << (r & 31));
                if (e & 2u) atomicOr(&bad[(r + 1) >> 5], 1u << ((r + 1) & 31));
              }
            }
          } else {
            // three or more values, an empty value, or a gap (a fixed column's failed sample
            // leaves zeros): piece by piece
            val = make_uint4(0, 0, 0, 0);
            for (int rr = r; rr < gb && pos < end; ++rr) {
              const RowsRec q = T.rec[base + rr];
              const int32_t ds = int32_t(q.dst);
              const int32_t de = ds + int32_t(q.len);
              if (de <= pos) continue;  // a sample with no bytes in this column
              if (ds >= end) break;
              const int32_t lo = max(pos, ds), hi = min(end, de);
              const lds_u8* p = stage + (int32_t(q.src) - ds + P0);
              const uint4 v = lds_read16(p);
              const uint4 pv = keep_bytes(v, uint32_t(lo - P0), uint32_t(hi - P0));
              val = make_uint4(val.x | pv.x, val.y | pv.y, val.z | pv.z, val.w | pv.w);
              if (utf8) {
                uint32_t pw = 0;
                if (lo > ds) {
                  pw = lds_u32(p + (lo - P0) - 4);
                  const int32_t nv = lo - ds;
                  if (nv < 4) pw &= ~((1u << (8 * (4 - nv))) - 1u);
                }
                // an ASCII piece after no lead byte cannot err nor end a sequence open (the
                // simple path's `plain`, per lane here; measurement knob sdbg 16384: always check)
                const bool ascii =
                    (((pv.x | pv.y | pv.z | pv.w) & 0x80808080u) | hi_c0(pw)) == 0 &&
                    !(a.stage_debug & 16384);
                if (!ascii && ((utf8_chunk_err2(pv, pw, 16) & 1u) ||
                               (hi == de && hi == P0 + 16 && utf8_open_at(pv, pw, 16))))
                  atomicOr(&bad[rr >> 5], 1u << (rr & 31));
              }
              pos = hi;
            }
          }
          const uint64_t D = D0 + 16ull * k;
          if ((a.stage_debug & 16) && val.x != 0x9e3779b9u) continue;
          if (P0 >= 0 && P0 + 16 <= int32_t(wlen)) st16<kNT>(D, val);
          else store_bytes(D, val, uint32_t(max(P0, 0) - P0), uint32_t(end - P0));
        }
        }
      }
      rows_barrier<kFence>();  // every piece's UTF-8 mark is in (a next tile's DMA may be in flight)
    }
    if constexpr (prof) prof_mark(a, tile, 5, ts);
    // ---- 5. flags (a sample listed for the huge-row kernel: set there when its value fails)
    if (mine) {
      for (int c = 0; c < ncols; ++c) {
        const MDSX_L DevCol& col = cols[c];
        if (col.kind == MDSX_KIND_STR && col.flags != nullptr && !s_skip[c])
          *gp(col.flags + row0 + t) = uint8_t((T.bad[c * 8 + (t >> 5)] >> (t & 31)) & 1u);
      }
    }
    if constexpr (prof) prof_mark(a, tile, 6, ts);
    ga = gb;
  }
  if constexpr (kPipe) rows_barrier<kFence>();  // this tile's readers of the tables and its stage are done
  }  // tile
}

}  // namespace

uint32_t rows_tile_rows_limit() { return kRowsBlock; }

int launch_rows_decode(const mdsx_plan* plan, const DevArgs& a, hipStream_t s) {
  if (a.tile_rows > kRowsBlock)
    return mdsx::fail(MDSX_E_ARG, "mdsx: row-parallel decode tiles hold at most 256 rows");
  // the huge-row list (samples larger than the stage) starts empty
  int rc = hip_check(hipMemsetAsync(reinterpret_cast<uint8_t*>(a.status) + kHugeCountOffset, 0,
                                    4, s),
                     "hipMemsetAsync");
  if (rc != MDSX_OK) return rc;
  const bool pipe = a.rows_pipe > 0;
  const size_t lds = rows_lds_bytes(a.rows_bytes, a.tile_rows, a.ncols, a.nvar, pipe ? 2 : 1);
  if (lds > 160 * 1024)
    return mdsx::fail(MDSX_E_ARG, "mdsx: row-parallel decode stage and tables exceed 160 KiB of LDS");
  const bool nt = plan->rows_nt != 0;
  const unsigned grid = pipe ? (a.ntiles + a.rows_pipe - 1) / a.rows_pipe : a.ntiles;
  // registers bounded for six waves per SIMD where six workgroups' stages fit a CU (measured:
  // +7 % on 32-256-byte samples, -1 % on 256-1024-byte ones)
  const int occ = plan->rows_occ ? plan->rows_occ : (a.rows_bytes <= 24 * 1024 ? 6 : 4);
#define MDSX_ROWS_CASE(NT, PIPE)                                                                \
  if (nt == NT && pipe == PIPE) {                                                               \
    if (lds > 64 * 1024) {                                                                      \
      rc = hip_check(hipFuncSetAttribute(reinterpret_cast<const void*>(                         \
                                             rows_decode_kernel<NT, PIPE>),                     \
                                         hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)), \
                     "hipFuncSetAttribute");                                                    \
      if (rc != MDSX_OK) return rc;                                                             \
    }                                                                                           \
    mdsx::set_last_kernel("rows_decode_kernel<" #NT ", " #PIPE ">");                            \
    hipLaunchKernelGGL((rows_decode_kernel<NT, PIPE>), dim3(grid), dim3(kRowsBlock), lds, s, a); \
  }
  if (a.stage_debug & 256) {  // measurement only: one write loop per column
    if (lds > 64 * 1024) {
      rc = hip_check(hipFuncSetAttribute(reinterpret_cast<const void*>(
                                             rows_decode_kernel<true, false, false, false, 4, false>),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)),
                     "hipFuncSetAttribute");
      if (rc != MDSX_OK) return rc;
    }
    mdsx::set_last_kernel("rows_decode_kernel<true, false, false, false, 4, false>");
    hipLaunchKernelGGL((rows_decode_kernel<true, false, false, false, 4, false>), dim3(a.ntiles),
                       dim3(kRowsBlock), lds, s, a);
  } else if (a.stage_debug & 128) {  // measurement only: __syncthreads() barriers
    if (lds > 64 * 1024) {
      rc = hip_check(hipFuncSetAttribute(
                         reinterpret_cast<const void*>(rows_decode_kernel<true, false, false, true>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)),
                     "hipFuncSetAttribute");
      if (rc != MDSX_OK) return rc;
    }
    mdsx::set_last_kernel("rows_decode_kernel<true, false, false, true>");
    hipLaunchKernelGGL((rows_decode_kernel<true, false, false, true>), dim3(a.ntiles),
                       dim3(kRowsBlock), lds, s, a);
  } else if (a.stage_debug & 64) {  // measurement only: the phase stamps (src_abs)
    // 8 stamps per tile in the huge-row list's space (nvar x rows words): refused where they
    // would run past it; a huge row in such a batch is reported (MDSX_E_ARG), not listed
    if (8ull * a.ntiles > uint64_t(a.nvar) * a.rows)
      return mdsx::fail(MDSX_E_ARG, "mdsx: row-decode stamps need 8 x tiles <= nvar x rows");
    if (lds > 64 * 1024) {
      rc = hip_check(hipFuncSetAttribute(
                         reinterpret_cast<const void*>(rows_decode_kernel<true, false, true>),
                         hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)),
                     "hipFuncSetAttribute");
      if (rc != MDSX_OK) return rc;
    }
    mdsx::set_last_kernel("rows_decode_kernel<true, false, true>");
    hipLaunchKernelGGL((rows_decode_kernel<true, false, true>), dim3(a.ntiles), dim3(kRowsBlock),
                       lds, s, a);
  } else if ((occ == 6 || occ == 8) && nt && !pipe) {
    const void* fn = occ == 6
                         ? reinterpret_cast<const void*>(rows_decode_kernel<true, false, false, false, 6>)
                         : reinterpret_cast<const void*>(rows_decode_kernel<true, false, false, false, 8>);
    if (lds > 64 * 1024) {
      rc = hip_check(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)),
                     "hipFuncSetAttribute");
      if (rc != MDSX_OK) return rc;
    }
    if (occ == 6) {
      mdsx::set_last_kernel("rows_decode_kernel<true, false, false, false, 6>");
      hipLaunchKernelGGL((rows_decode_kernel<true, false, false, false, 6>), dim3(a.ntiles),
                         dim3(kRowsBlock), lds, s, a);
    } else {
      mdsx::set_last_kernel("rows_decode_kernel<true, false, false, false, 8>");
      hipLaunchKernelGGL((rows_decode_kernel<true, false, false, false, 8>), dim3(a.ntiles),
                         dim3(kRowsBlock), lds, s, a);
    }
  } else {
    MDSX_ROWS_CASE(true, false)
    MDSX_ROWS_CASE(false, false)
    MDSX_ROWS_CASE(true, true)
    MDSX_ROWS_CASE(false, true)
  }
#undef MDSX_ROWS_CASE
  rc = hip_check(hipGetLastError(), "rows_decode_kernel launch");
  if (rc != MDSX_OK) return rc;
  return launch_huge_rows(a, nt, s);
}

}  // namespace mdsx_kernels
