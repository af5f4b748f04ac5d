// MI355X (gfx950, CDNA4) kernels of the MDS shard decoder, and the C ABI entry points that
// launch them (declared in include/mdsx.h).
//
// The reference decodes one sample per Python call: MDSReader.get_sample_data opens the shard,
// seeks into the u32 offsets table, reads [begin, end) (streaming/base/format/mds/reader.py:128-149),
// then decode_sample splits the columns with the u32 size head of the variable columns and calls
// mds_decode per column (mds/reader.py:103-126, encodings.py:760-773). Here whole shards are
// HBM-resident and decoded at once:
//
//   scan_tiles_kernel    one workgroup per tile of rows: offsets-table scan + u32 size heads ->
//                        per-row lengths of every ragged column, block exclusive scan (wave64
//                        shuffles + LDS), per-tile totals.                      (ragged plans only)
//   scan_chunks_kernel / scan_chunk_sums_kernel / scan_apply_kernel: exclusive scan of the
//                        per-block totals of every ragged column (reduce-then-scan).
//   decode_kernel        one workgroup per tile: per-row column boundaries into LDS; fixed columns
//                        of <= 16 bytes gathered one row per lane; larger fixed columns and long
//                        ragged rows copied one row per wave with 16-byte aligned loads and stores,
//                        the source realigned in registers (v_alignbyte funnel over the neighbour
//                        lane's chunk); medium ragged rows (a few hundred bytes) four per wave, one
//                        per 16-lane group; then the tile's str rows are UTF-8 checked from the
//                        L2-resident output, four rows per wave; for short-row ragged columns:
//                        final offsets, each row's source address and the row that starts every
//                        4 KiB output grain (for the gather kernel).
//   gather_ragged_kernel one workgroup per 16 KiB tile of a ragged column's packed output
//                        (destination-major): every lane writes whole aligned 16-byte chunks,
//                        assembled from the row(s) that cover them (binary search over the tile's
//                        rows staged in LDS), so short and long rows keep all 64 lanes busy; str
//                        columns are UTF-8 validated in the same pass, flagging rows Python's
//                        strict decoder would reject.
//
// Every load stays inside [shard - 32, shard + bytes + 32): the batch buffer carries
// MDSX_BATCH_PAD bytes of slack around its shards, and every sample range is checked against
// the shard before it is touched.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>

#include "mdsx_decode.h"
#include "mdsx_device.h"
#include "mdsx_internal.h"

namespace mdsx_kernels {

// ---------------------------------------------------------------------------------------------
// Pass 1a: per-row ragged lengths -> block-local exclusive offsets + per-block totals.
// One workgroup (a scan block) covers scan_per = 256 / tile_rows consecutive tiles (tile_rows <=
// 256, a power of two): one thread per row, one block-wide exclusive scan. Tiles are in output
// row order and a partial tile's missing rows count zero, so the scan is the output order; the
// decode adds the scan block's prefix. Totals per scan block, not per tile, keep pass 1b an
// eighth as long (32-row tiles).
// kRec (the one-sample-per-wave decode): every sample slot's record (sw_rec), its range errors and
// its shard's header checked here instead of in the decode (mds/reader.py:137-148,
// mds/writer.py:133-144).
template <bool kRec = false>
__global__ __launch_bounds__(kBlock) void scan_tiles_kernel(const DevArgs a) {
  __shared__ int64_t s_wsum[kBlock / 64];
  const int t = threadIdx.x;
  const int TR = a.tile_rows;
  const int per_block = kBlock / TR;
  const uint32_t tile = blockIdx.x * uint32_t(per_block) + uint32_t(t / TR);
  const int tt = t % TR;  // row of the tile
  const bool tile_ok = tile < a.ntiles;
  TileView v;
  if (tile_ok) v = tile_view(a, tile);
  const uint32_t i = tile_ok ? v.r0 + tt : 0;
  const bool in_tile = tile_ok && v.table_ok && tt < int(v.nrows);
  uint32_t b = 0, e = 0;
  bool ok = false;
  int rc = MDSX_OK;
  if (in_tile) {
    rc = sample_range(v, i, &b, &e);
    ok = rc == MDSX_OK && uint64_t(b) + 4ull * a.nvar <= e;
  }
  if constexpr (kRec) {
    if (tile_ok) {
      const uint64_t src = v.d.offset + b;
      const uint32_t z = !in_tile ? kSwIdle : rc != MDSX_OK ? kSwBad : e - b;
      a.sw_rec[uint64_t(tile) * uint32_t(TR) + uint32_t(tt)] =
          make_uint4(uint32_t(src), uint32_t(src >> 32) | (v.shard_idx << 8), z,
                     uint32_t(v.d.row0 + i));
      if (in_tile && rc != MDSX_OK) report_decode(a, rc, int(v.shard_idx), int(i), -1);
      // the shard header (mds/writer.py:133-144): u32 N, then N + 1 offsets
      if (tt == 0 && tile == v.d.tile0 &&
          (!v.table_ok || *reinterpret_cast<const uint32_t*>(v.shard) != v.d.samples ||
           v.offs[0] < v.hdr_end || v.offs[v.d.samples] > v.d.bytes))
        report_decode(a, MDSX_E_HEADER, int(v.shard_idx), -1, -1);
    }
  }
  const bool few = a.nvar <= kHeadRegs;  // heads in registers (else re-read per column)
  Heads h;
  if (ok && few) h.load(v.shard + b, a.nvar);
  auto head = [&](int vi) -> uint32_t {
    return few ? h.get(vi) : load_u32_any(v.shard + b + 4u * uint32_t(vi));
  };
  if (ok) {  // the whole sample must hold its heads and columns; else emit zero lengths
    uint64_t need = 4ull * a.nvar;
    for (int c = 0; c < a.ncols; ++c) {
      const DevCol& col = a.cols[c];
      need += col.var_index >= 0 ? head(col.var_index) : col.row_bytes;
    }
    ok = uint64_t(b) + need <= e;
  }
  for (int c = 0; c < a.ncols; ++c) {
    const DevCol& col = a.cols[c];
    if (col.var_index < 0) continue;
    const int vi = col.var_index;
    const int64_t len = ok ? int64_t(head(vi)) : 0;
    int64_t total;
    const int64_t excl = block_exclusive_scan(len, s_wsum, &total);
    if (in_tile) col.offsets[v.d.row0 + i] = excl;
    if (t == 0) a.tile_total[uint64_t(vi) * a.nscan + blockIdx.x] = total;
  }
}

// Pass 1b: exclusive scan of the scan-block totals of every ragged column (nscan entries each),
// reduce-then-scan over chunks of kScanChunk entries: scan_chunks_kernel sums each chunk,
// scan_chunk_sums_kernel scans the chunk sums (one workgroup per column; the column totals land
// in totals[] and offsets[rows]), scan_apply_kernel scans each chunk from its base.
constexpr uint32_t kScanPer = 16;                   // entries per thread
constexpr uint32_t kScanChunk = kBlock * kScanPer;  // entries per workgroup

__global__ __launch_bounds__(kBlock) void scan_chunks_kernel(const DevArgs a) {
  __shared__ int64_t s_wsum[kBlock / 64];
  const int vi = blockIdx.y;
  const int64_t* in = a.tile_total + uint64_t(vi) * a.nscan;
  const uint64_t lo = uint64_t(blockIdx.x) * kScanChunk + uint64_t(threadIdx.x) * kScanPer;
  int64_t x[kScanPer];
#pragma unroll
  for (uint32_t j = 0; j < kScanPer; ++j) x[j] = lo + j < a.nscan ? in[lo + j] : 0;
  int64_t run = 0;
#pragma unroll
  for (uint32_t j = 0; j < kScanPer; ++j) run += x[j];
  int64_t total;
  block_exclusive_scan(run, s_wsum, &total);
  if (threadIdx.x == 0) a.chunk_sum[uint64_t(vi) * a.nchunk + blockIdx.x] = total;
}

__global__ __launch_bounds__(kBlock) void scan_chunk_sums_kernel(const DevArgs a) {
  __shared__ int64_t s_wsum[kBlock / 64];
  const int vi = blockIdx.x;
  int64_t* sums = a.chunk_sum + uint64_t(vi) * a.nchunk;
  int64_t carry = 0;
  for (uint32_t base = 0; base < a.nchunk; base += kBlock) {  // in place: sums -> prefixes
    const uint32_t k = base + threadIdx.x;
    const int64_t x = k < a.nchunk ? sums[k] : 0;
    int64_t total;
    const int64_t excl = block_exclusive_scan(x, s_wsum, &total);
    if (k < a.nchunk) sums[k] = carry + excl;
    carry += total;
  }
  if (threadIdx.x == 0) {
    if (a.totals) a.totals[vi] = carry;
    for (int c = 0; c < a.ncols; ++c)
      if (a.cols[c].var_index == vi) a.cols[c].offsets[a.rows] = carry;
  }
}

__global__ __launch_bounds__(kBlock) void scan_apply_kernel(const DevArgs a) {
  __shared__ int64_t s_wsum[kBlock / 64];
  const int vi = blockIdx.y;
  const int64_t* in = a.tile_total + uint64_t(vi) * a.nscan;
  int64_t* out = a.tile_prefix + uint64_t(vi) * a.nscan;
  const uint64_t lo = uint64_t(blockIdx.x) * kScanChunk + uint64_t(threadIdx.x) * kScanPer;
  int64_t x[kScanPer];
#pragma unroll
  for (uint32_t j = 0; j < kScanPer; ++j) x[j] = lo + j < a.nscan ? in[lo + j] : 0;
  int64_t run = 0;
#pragma unroll
  for (uint32_t j = 0; j < kScanPer; ++j) run += x[j];
  int64_t total;
  int64_t base = a.chunk_sum[uint64_t(vi) * a.nchunk + blockIdx.x] +
                 block_exclusive_scan(run, s_wsum, &total);
#pragma unroll
  for (uint32_t j = 0; j < kScanPer; ++j) {
    if (lo + j < a.nscan) out[lo + j] = base;
    base += x[j];
  }
}
// ---------------------------------------------------------------------------------------------
// Long ragged rows through an LDS-DMA ring (kSlots > 0 in decode_kernel). Each wave streams its
// rows' source bytes into a private ring of kSlots 1 KiB slots with global_load_lds_dwordx4 (no
// VGPR destination, so the bytes in flight per CU are bounded by LDS, not by registers) running
// up to kSlots KiB ahead of the copy, across row boundaries; the copy side reads each slot and
// its successor back (lane k: chunks k and k + 1), realigns with v_alignbyte and writes aligned
// 16-byte chunks. The DMA is issued from inline asm, so the compiler neither counts nor waits
// for it: the ring waits with explicit `s_waitcnt vmcnt(n)`, n = the vector-memory operations
// this wave issued after the slot's DMA (DMAs, and stores certain to issue; any other store
// only makes the wait stricter). Only the issuing wave reads its slots, so its vmcnt orders the
// reads (MI355X_MICROARCH.md: nothing else orders a ds_read behind a pending LDS-DMA).
// One long-row job of a wave: row r of ragged column c, as aligned 16-byte chunks.
struct RingJob {
  const uint4* sal;  // first aligned source chunk
  uint64_t dbeg, d0, dend;
  uint32_t nchunks, nload, nslots, sh;
  int r, c;  // c < 0: no more jobs
};

__device__ __forceinline__ bool ring_column(const DevCol& col) {
  return col.var_index >= 0 && !col.gather && !col.group;
}

// Advance j to this wave's next (row, column) with bytes to copy (rows r, r + 4, ...).
__device__ __forceinline__ void ring_next(const DevArgs& a, const DevCol* cols, const TileView& v,
                                          int TR,
                                          const uint32_t* s_src, const uint64_t* s_vdst,
                                          const uint32_t* s_vlen, const uint8_t* s_ok,
                                          RingJob& j) {
  int r = j.r, c = j.c;
  for (;;) {
    if (r >= int(v.nrows)) {
      j.c = -1;
      return;
    }
    ++c;
    while (c < a.ncols && !ring_column(cols[c])) ++c;
    if (c >= a.ncols || !s_ok[r]) {
      r += kBlock / 64;
      c = -1;
      continue;
    }
    const int vi = cols[c].var_index;
    const uint32_t len = s_vlen[vi * TR + r];
    if (len == 0) continue;
    const uint64_t d0 = reinterpret_cast<uint64_t>(cols[c].data) + s_vdst[vi * TR + r];
    const uint64_t dend = d0 + len;
    const uint64_t dbeg = d0 & ~uint64_t(15);
    const uint64_t sfirst =
        reinterpret_cast<uint64_t>(v.shard + s_src[c * TR + r]) - (d0 - dbeg);
    j.r = r;
    j.c = c;
    j.d0 = d0;
    j.dend = dend;
    j.dbeg = dbeg;
    j.sh = uint32_t(sfirst & 15);
    j.sal = reinterpret_cast<const uint4*>(sfirst & ~uint64_t(15));
    j.nchunks = uint32_t((((dend + 15) & ~uint64_t(15)) - dbeg) >> 4);
    j.nload = j.nchunks + (j.sh ? 1u : 0u);
    j.nslots = (j.nload + 63) / 64;
    return;
  }
}

template <int kSlots, bool kNT>
__device__ __forceinline__ void ring_copy(const DevArgs& a, const DevCol* cols, const TileView& v,
                                          int TR,
                                          const uint32_t* s_src, const uint64_t* s_vdst,
                                          const uint32_t* s_vlen, const uint8_t* s_ok,
                                          const uint4* ring, uint32_t ring_lds, int wave,
                                          int lane) {
  RingJob P, Q;  // producer (DMA) and consumer (copy) cursors, wave-uniform
  P.r = wave;
  P.c = -1;
  ring_next(a, cols, v, TR, s_src, s_vdst, s_vlen, s_ok, P);
  if (P.c < 0) return;
  Q = P;
  uint32_t p = 0;           // next slot of job P to load
  uint32_t issued = 0, consumed = 0, ops = 0;
  uint32_t op_at = 0;       // lane i: `ops` when ring slot i was loaded
  auto pump = [&]() {
    while (P.c >= 0 && issued - consumed < uint32_t(kSlots)) {
      const uint32_t k = p * 64 + uint32_t(lane);
      const uint32_t slot = issued % kSlots;
      glds16<kNT>(P.sal + (k < P.nload ? k : 0u), ring_lds + slot * 1024u);
      if (lane == int(slot)) op_at = ops;
      ++ops;
      ++issued;
      if (++p == P.nslots) {
        p = 0;
        ring_next(a, cols, v, TR, s_src, s_vdst, s_vlen, s_ok, P);
      }
    }
  };
  pump();
  while (Q.c >= 0) {
    const bool head_partial = Q.dbeg < Q.d0 || Q.dbeg + 16 > Q.dend;
    const bool tail_partial = Q.nchunks > 1 && (Q.dend & 15) != 0;
    const uint32_t kf0 = Q.d0 > Q.dbeg ? 1u : 0u;            // full chunks: [kf0, kf1)
    const uint32_t kf1 = uint32_t((Q.dend - Q.dbeg) >> 4);
    for (uint32_t q = 0; q < Q.nslots; ++q) {
      const uint32_t x = consumed % kSlots;
      const uint32_t need = (Q.sh != 0 && q + 1 < Q.nslots) ? (consumed + 1) % kSlots : x;
      wait_vm_at_most(ops - __builtin_amdgcn_readlane(op_at, need) - 1);
      const uint32_t k0 = q * 64;
      if (k0 < Q.nchunks) {  // wave-uniform: the slot holds output chunks
        const uint32_t k = k0 + uint32_t(lane);
        const uint4 lo = ring[x * 64 + lane];
        uint4 out = lo;
        if (Q.sh != 0) {
          const uint4 hi = lane < 63 ? ring[x * 64 + lane + 1] : ring[need * 64];
          out = funnel16(lo, hi, Q.sh);
        }
        const uint64_t D = Q.dbeg + 16ull * k;
        if (k < Q.nchunks && D >= Q.d0 && D + 16 <= Q.dend) st16<kNT>(D, out);
        if (max(kf0, k0) < min(kf1, k0 + 64)) ++ops;  // that store was issued
        if (q == 0 && head_partial) wave_edge_store(out, 0, Q.dbeg, Q.d0, Q.dend, lane);
        if (tail_partial && Q.nchunks - 1 >= k0 && Q.nchunks - 1 < k0 + 64)
          wave_edge_store(out, int(Q.nchunks - 1 - k0), Q.dbeg + 16ull * (Q.nchunks - 1), Q.d0,
                          Q.dend, lane);
      }
      ++consumed;
      pump();
    }
    ring_next(a, cols, v, TR, s_src, s_vdst, s_vlen, s_ok, Q);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// Pass 2: per-row column boundaries; fixed columns decoded; ragged columns prepared for the
// destination-major gather (final offsets, per-row source addresses, gather-tile row map).
// kSingle: one pass, no scan kernels before it (mdsx_decode_shards_single): each tile
// block-scans its ragged lengths and finds its base by the look-back (lookback_bases,
// mdsx_decode.h; status word of one (ragged column, tile): flag in the top 2 bits -- 0 not yet
// published, 1 the tile's own aggregate, 2 the inclusive prefix -- and a byte count below).
// kSlots > 0: long ragged rows copied through the LDS-DMA ring (ring_copy) instead of wave_copy.
template <int kUnroll, bool kNT, bool kRagged, bool kEdges, bool kSingle, int kSlots = 0>
__global__ __launch_bounds__(kBlock) void decode_kernel(const DevArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int TR = a.tile_rows;
  uint64_t* s_vdst = reinterpret_cast<uint64_t*>(smem);                 // [nvar][TR]
  uint32_t* s_src = reinterpret_cast<uint32_t*>(s_vdst + a.nvar * TR);  // [ncols][TR]
  uint32_t* s_vlen = s_src + a.ncols * TR;                               // [nvar][TR]
  uint8_t* s_ok = reinterpret_cast<uint8_t*>(s_vlen + a.nvar * TR);     // [TR]
  __shared__ uint32_t s_tile;
  __shared__ int64_t s_wsum[kBlock / 64];
  __shared__ int64_t s_base[kSingle ? MDSX_MAX_COLUMNS : 1];

  const int t = threadIdx.x;
  const int lane = t & 63, wave = t >> 6;
  // Ring variant: the column table in LDS. Indexed by a loop variable, kernel-argument fields
  // compile to vector-memory loads, and the compiler waits for one with a vmcnt(0) that would
  // also drain the ring's LDS-DMA in flight. (The register-copy variants keep reading the
  // kernel arguments: measured faster on config B than the LDS table plus its barrier.)
  __shared__ DevCol s_cols[kSlots > 0 ? MDSX_MAX_COLUMNS : 1];
  const DevCol* const cols = kSlots > 0 ? s_cols : a.cols;
  if constexpr (kSlots > 0)
    for (int i = t; i < a.ncols; i += kBlock) s_cols[i] = a.cols[i];
  uint32_t tile = (!kSingle && (a.xcd_order & kXcdRegister)) ? xcd_block(blockIdx.x, gridDim.x)
                                                              : blockIdx.x;
  if constexpr (kSingle) {
    if (t == 0) s_tile = atomicAdd(a.ticket, 1u);
  }
  if constexpr (kSingle || kSlots > 0) __syncthreads();
  if constexpr (kSingle) tile = s_tile;
  const TileView v = tile_view(a, tile);

  if (!v.table_ok) {
    if (t == 0 && tile == v.d.tile0) report_decode(a, MDSX_E_HEADER, v.shard_idx, -1, -1);
    if constexpr (!kSingle) return;  // block-uniform (kSingle: the tile still publishes zeros)
  }
  if (t == 0 && tile == v.d.tile0 && v.table_ok) {
    // Header written by encode_joint_shard (mds/writer.py:133-144): u32 N, then N+1 offsets.
    const uint32_t n = *reinterpret_cast<const uint32_t*>(v.shard);
    const uint32_t first = v.offs[0];
    if (n != v.d.samples || first < v.hdr_end || v.offs[v.d.samples] > v.d.bytes)
      report_decode(a, MDSX_E_HEADER, v.shard_idx, -1, -1);
  }
  const int nrows = v.table_ok ? int(v.nrows) : 0;

  // ---- column boundaries of this lane's row (MDSReader.decode_sample, mds/reader.py:111-125).
  // A row failing any check keeps zero ragged lengths (the scan pass's rule).
  if (t < nrows) {
    const uint32_t i = v.r0 + t;
    uint32_t b = 0, e = 0;
    int rc = sample_range(v, i, &b, &e);
    bool ok = rc == MDSX_OK;
    if (ok && uint64_t(b) + 4ull * a.nvar > e) {
      ok = false;
      rc = MDSX_E_BOUNDS;
    }
    uint64_t pos = uint64_t(b) + 4ull * a.nvar;
    const bool few = a.nvar <= kHeadRegs;
    Heads h;
    if (kRagged && ok && few) h.load(v.shard + b, a.nvar);
    for (int c = 0; c < a.ncols; ++c) {
      const DevCol& col = cols[c];
      uint64_t len = col.row_bytes;
      if (col.var_index >= 0) {
        const int vi = col.var_index;
        len = !ok ? 0u : few ? h.get(vi) : load_u32_any(v.shard + b + 4u * uint32_t(vi));
        s_vlen[col.var_index * TR + t] = uint32_t(len);
      }
      s_src[c * TR + t] = uint32_t(pos);
      pos += len;
    }
    if (ok && pos > e) {
      ok = false;
      rc = MDSX_E_BOUNDS;
    }
    if (!ok) {
      for (int vi = 0; vi < a.nvar; ++vi) s_vlen[vi * TR + t] = 0;
      if (rc != MDSX_OK) report_decode(a, rc, v.shard_idx, int(i), -1);
    }
    s_ok[t] = ok ? 1 : 0;
  }

  if constexpr (kSingle) {
    // ---- this tile's ragged offsets: block scan of the lengths, then the look-back for the base
    __shared__ int64_t s_agg[MDSX_MAX_COLUMNS];
    __syncthreads();
    for (int vi = 0; vi < a.nvar; ++vi) {
      const int64_t x = t < nrows ? int64_t(s_vlen[vi * TR + t]) : 0;
      int64_t tot;
      const int64_t excl = block_exclusive_scan(x, s_wsum, &tot);
      if (t < nrows) s_vdst[vi * TR + t] = uint64_t(excl);
      if (t == 0) s_agg[vi] = tot;
    }
    __syncthreads();
    if (wave == 0) lookback_bases(a, tile, s_agg, s_base, v.shard_idx, lane, a.lookback, a.ntiles);
    __syncthreads();
    if (!v.table_ok) return;  // block-uniform; published its zero aggregates above
  }

  // ---- ragged columns: final offsets; the destination of this kernel's copies, or (gather
  // columns) the row's source address and the 4 KiB output grains whose first byte it holds.
  if (t < nrows) {
    const uint32_t i = v.r0 + t;
    const uint64_t row = v.d.row0 + i;
    bool ok = s_ok[t] != 0;
    for (int c = 0; c < a.ncols; ++c) {
      const DevCol& col = cols[c];
      if (col.var_index < 0) continue;
      const int vi = col.var_index;
      int64_t off;
      if constexpr (kSingle)
        off = s_base[vi] + int64_t(s_vdst[vi * TR + t]);
      else  // the scan pass left the scan-block-local offset in offsets[row]
        off = a.tile_prefix[uint64_t(vi) * a.nscan + tile / a.scan_per] + col.offsets[row];
      col.offsets[row] = off;
      s_vdst[vi * TR + t] = uint64_t(off);
      if (col.flags) col.flags[row] = 0;
      if (!ok) continue;
      const uint64_t len = s_vlen[vi * TR + t];
      if (uint64_t(off) + len > col.capacity) {
        report_decode(a, MDSX_E_CAPACITY, v.shard_idx, int(i), c);
        ok = false;
        continue;
      }
      if (!col.gather && !col.group) continue;
      a.src_abs[uint64_t(vi) * a.rows + row] = v.d.offset + s_src[c * TR + t];
      if (col.gather && len) {
        uint32_t* map = a.row_map + uint64_t(vi) * a.map_len;
        for (uint64_t g = (uint64_t(off) + kMapGrain - 1) / kMapGrain;
             g * kMapGrain < uint64_t(off) + len && g < a.map_len; ++g)
          map[g] = uint32_t(row);
      }
    }
    s_ok[t] = ok ? 1 : 0;
  }
  __syncthreads();

  // ---- small fixed columns: one row per lane
  if (t < int(v.nrows) && s_ok[t]) {
    const uint64_t row = v.d.row0 + v.r0 + t;
    for (int c = 0; c < a.ncols; ++c) {
      const DevCol& col = cols[c];
      if (col.var_index >= 0 || col.row_bytes > uint32_t(kSmallMax)) continue;
      gather_small(v.shard + s_src[c * TR + t],
                   static_cast<uint8_t*>(col.data) + row * col.row_bytes, col.row_bytes);
    }
  }

  // ---- large fixed columns and long-row ragged columns: one row per wave
  for (int r = wave; r < int(v.nrows); r += kBlock / 64) {
    if (!s_ok[r]) continue;  // wave-uniform
    const uint64_t row = v.d.row0 + v.r0 + r;
    for (int c = 0; c < a.ncols; ++c) {
      const DevCol& col = cols[c];
      const uint8_t* src = v.shard + s_src[c * TR + r];
      if (col.var_index < 0) {
        if (col.row_bytes <= uint32_t(kSmallMax)) continue;
        wave_copy<false, kUnroll, kNT, kEdges>(
            src, static_cast<uint8_t*>(col.data) + row * col.row_bytes, col.row_bytes, lane);
      } else if (kRagged && kSlots == 0 && !col.gather && !col.group) {
        const int vi = col.var_index;
        uint8_t* dst = static_cast<uint8_t*>(col.data) + s_vdst[vi * TR + r];
        const uint64_t len = s_vlen[vi * TR + r];
        // str rows: validated below, once the tile's rows are copied (the check fused into
        // the copy loop costs the kernel a wave per SIMD: 125 vs 87 VGPRs)
        wave_copy<false, kUnroll, kNT>(src, dst, len, lane);
      }
    }
  }

  if constexpr (kRagged && kSlots > 0) {
    if (a.any_wave_ragged) {  // launch-uniform
      const size_t head = (size_t(TR) * (12 * size_t(a.nvar) + 4 * size_t(a.ncols) + 1) + 15) &
                          ~size_t(15);
      const uint4* ring = reinterpret_cast<const uint4*>(smem + head) + wave * kSlots * 64;
      const uint32_t ring_lds = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(
          reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const uint4*)ring)));
      ring_copy<kSlots, kNT>(a, cols, v, TR, s_src, s_vdst, s_vlen, s_ok, ring, ring_lds,
                             __builtin_amdgcn_readfirstlane(wave), lane);
    }
  }

  // ---- medium-row ragged columns: four rows per wave, one per 16-lane group
  if constexpr (kRagged) {
    if (a.any_group) {  // launch-uniform
      const int g = lane >> 4;
      for (int r0 = wave * 4; r0 < int(v.nrows); r0 += kBlock / 16) {
        const int r = min(r0 + g, int(v.nrows) - 1);
        const bool live = r0 + g < int(v.nrows) && s_ok[r];
        for (int c = 0; c < a.ncols; ++c) {
          const DevCol& col = cols[c];
          if (!col.group) continue;
          const int vi = col.var_index;
          const uint8_t* src = v.shard + s_src[c * TR + r];
          uint8_t* dst = static_cast<uint8_t*>(col.data) + s_vdst[vi * TR + r];
          const uint32_t len = live ? s_vlen[vi * TR + r] : 0;
          if (a.str_cached && col.kind == MDSX_KIND_STR)  // re-read below for the UTF-8 check
            group_copy<kGroupUnroll, false>(src, dst, len, lane);
          else
            group_copy<kGroupUnroll, kNT>(src, dst, len, lane);
        }
      }
    }
  }

  // ---- strict UTF-8 of this tile's str rows (encodings.py:80-81), re-read from the packed
  // output while it is L2-resident: four rows per wave, one per 16-lane group
  if constexpr (kRagged) {
    if (!a.any_wave_str) return;  // launch-uniform
    __threadfence_block();
    __syncthreads();
    const int g = lane >> 4;
    for (int r0 = wave * 4; r0 < int(v.nrows); r0 += kBlock / 16) {
      const int r = min(r0 + g, int(v.nrows) - 1);
      const bool live = r0 + g < int(v.nrows) && s_ok[r];
      for (int c = 0; c < a.ncols; ++c) {
        const DevCol& col = cols[c];
        if (col.kind != MDSX_KIND_STR || !col.flags || col.gather) continue;
        const int vi = col.var_index;
        const uint64_t len = live ? s_vlen[vi * TR + r] : 0;
        // (the ring variant: 1 chunk per lane in flight, which keeps it at 72 VGPRs = 7 waves)
        const bool bad = group_utf8_bad<(kSlots > 0 ? 1 : 2)>(static_cast<const uint8_t*>(col.data),
                                           s_vdst[vi * TR + r], len, lane);
        if ((lane & 15) == 0 && len && bad) col.flags[v.d.row0 + v.r0 + r] = 1;
      }
    }
  }

}

// ---------------------------------------------------------------------------------------------
// Pass 3: ragged columns, destination-major. Rows of a gather tile are addressed through an
// accessor: staged in LDS when they fit (the common case), else read from global memory.
struct RowsLds {
  const int64_t* off;    // [n + 1]
  const uint64_t* src;   // [n]
  __device__ __forceinline__ int64_t o(int i) const { return off[i]; }
  __device__ __forceinline__ uint64_t s(int i) const { return src[i]; }
};

struct RowsGlobal {
  const int64_t* off;    // offsets + r0
  const uint64_t* src;   // src_abs + r0
  __device__ __forceinline__ int64_t o(int i) const { return off[i]; }
  __device__ __forceinline__ uint64_t s(int i) const { return src[i]; }
};

// Index (in [0, n)) of the row holding byte D: the last i with o(i) <= D.
template <class Rows>
__device__ __forceinline__ int find_row(const Rows& R, int n, int64_t D) {
  int lo = 0, hi = n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (R.o(mid) <= D) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// The 16 output bytes at column position D (D % 16 == 0), assembled from the rows covering them
// starting at row index j. Bytes past the column end are zero.
template <bool kNT, class Rows>
__device__ __forceinline__ uint4 assemble(const Rows& R, int n, int j, int64_t D,
                                          const uint8_t* batch) {
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (; j < n && R.o(j) < D + 16; ++j) {
    const int64_t ro = R.o(j), re = R.o(j + 1);
    const int64_t a = max(D, ro), b = min(D + 16, re);
    if (b <= a) continue;
    const uint64_t s0 = reinterpret_cast<uint64_t>(batch) + R.s(j) + uint64_t(D - ro);
    const uint4* al = reinterpret_cast<const uint4*>(s0 & ~uint64_t(15));
    const uint32_t sh = uint32_t(s0 & 15);
    const uint4 lo = ld16<kNT>(al);
    const uint4 hi = sh ? ld16<kNT>(al + 1) : make_uint4(0, 0, 0, 0);
    const uint4 val = sh ? funnel16_lane(lo, hi, sh) : lo;
    const uint4 m = byte_mask(uint32_t(a - D), uint32_t(b - D));
    acc = make_uint4((acc.x & ~m.x) | (val.x & m.x), (acc.y & ~m.y) | (val.y & m.y),
                     (acc.z & ~m.z) | (val.z & m.z), (acc.w & ~m.w) | (val.w & m.w));
  }
  return acc;
}

// Strict UTF-8 well-formedness (what bytes.decode('utf-8') accepts, encodings.py:80-81) of the
// 16 bytes at column position D, rows tracked from row index j; pw holds the 4 bytes before D.
// Flags every row with an invalid byte (rows are flagged 0 beforehand by decode_kernel).
template <class Rows>
__device__ __forceinline__ void utf8_check(const Rows& R, int n, int j, int64_t D, int64_t tot,
                                           const uint4 v, uint32_t pw, uint8_t* flags,
                                           uint64_t row0) {
  uint32_t p1 = (pw >> 24) & 0xffu, p2 = (pw >> 16) & 0xffu, p3 = (pw >> 8) & 0xffu;
  const bool ascii = ((v.x | v.y | v.z | v.w) & 0x80808080u) == 0;
  if (ascii && p1 < 0xC0u && p2 < 0xE0u && p3 < 0xF0u) return;
  // look-back bytes that precede the row start are not part of the row
  const int64_t dist = D - R.o(j);
  if (dist < 3) p3 = 0;
  if (dist < 2) p2 = 0;
  if (dist < 1) p1 = 0;
  int64_t rend = R.o(j + 1);
  bool bad = false;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int64_t P = D + k;
    if (P >= tot) break;
    if (P >= rend) {  // next non-empty row: flush the previous row's verdict, reset look-back
      if (bad) flags[row0 + j] = 1;
      bad = false;
      do {
        ++j;
        rend = R.o(j + 1);
      } while (P >= rend && j + 1 < n);
      p1 = p2 = p3 = 0;
    }
    const uint32_t b = byte_of(v, k);
    const bool cont = (b & 0xC0u) == 0x80u;
    const bool need = p1 >= 0xC0u || p2 >= 0xE0u || p3 >= 0xF0u;
    const int64_t left = rend - P;  // bytes from P to the row end, >= 1
    bad |= cont != need;
    bad |= b == 0xC0u || b == 0xC1u || b >= 0xF5u;
    bad |= (p1 == 0xE0u && b < 0xA0u) || (p1 == 0xEDu && b > 0x9Fu) ||
           (p1 == 0xF0u && b < 0x90u) || (p1 == 0xF4u && b > 0x8Fu);
    bad |= (b >= 0xC0u && left <= 1) || (b >= 0xE0u && left <= 2) || (b >= 0xF0u && left <= 3);
    p3 = p2;
    p2 = p1;
    p1 = b;
  }
  if (bad) flags[row0 + j] = 1;
}

// One output tile (kChunks x 4 KiB) of a ragged column. Chunk c = threadIdx.x + 256 k (k < kChunks),
// so the 64 lanes of a wave hold 64 consecutive chunks. A chunk inside one row (the common case)
// loads its aligned source chunk and takes the next one from the neighbour lane (same row, so the
// next 16 source bytes); lane 63 and chunks ending on a row end load it themselves. Chunks that
// straddle rows are assembled row by row.
template <bool kNT, int kGatherChunks, class Rows>
__device__ __forceinline__ void gather_tile(const DevArgs& a, const DevCol& col, const Rows& R,
                                            int n, uint64_t r0, int64_t T0, int64_t tot,
                                            uint32_t* s_edge) {
  const bool utf8 = col.kind == MDSX_KIND_STR && col.flags;
  uint8_t* out = static_cast<uint8_t*>(col.data);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint64_t base = reinterpret_cast<uint64_t>(a.batch);
  uint4 val[kGatherChunks], lo[kGatherChunks], hi[kGatherChunks];
  int jrow[kGatherChunks];
  uint32_t shift[kGatherChunks];
  bool single[kGatherChunks], need_hi[kGatherChunks];
  // phase 1: locate rows, issue every load
#pragma unroll
  for (int k = 0; k < kGatherChunks; ++k) {
    const int64_t D = T0 + 16 * (threadIdx.x + kBlock * k);
    const bool valid = D < tot;
    const int j = valid ? find_row(R, n, D) : 0;
    const int64_t ro = R.o(j), re = R.o(j + 1);
    const uint64_t s0 = base + R.s(j) + uint64_t(D - ro);
    const uint4* al = reinterpret_cast<const uint4*>(s0 & ~uint64_t(15));
    jrow[k] = j;
    shift[k] = uint32_t(s0 & 15);
    single[k] = valid && D + 16 <= re;
    const bool next_same = single[k] && D + 16 < re && lane != 63;  // lane+1 starts in row j
    need_hi[k] = single[k] && shift[k] != 0 && !next_same;
    lo[k] = valid ? ld16<kNT>(al) : make_uint4(0, 0, 0, 0);  // also feeds lane-1's funnel
    hi[k] = need_hi[k] ? ld16<kNT>(al + 1) : make_uint4(0, 0, 0, 0);
  }
  // phase 2: realign, assemble row-straddling chunks, store
#pragma unroll
  for (int k = 0; k < kGatherChunks; ++k) {
    const int64_t D = T0 + 16 * (threadIdx.x + kBlock * k);
    const uint4 nb = shfl_down1(lo[k]);
    if (single[k]) {
      const uint4 h = need_hi[k] ? hi[k] : nb;
      val[k] = shift[k] ? funnel16_lane(lo[k], h, shift[k]) : lo[k];
    } else if (D < tot) {
      val[k] = assemble<kNT>(R, n, jrow[k], D, a.batch);
    } else {
      val[k] = make_uint4(0, 0, 0, 0);
    }
    if (D < tot) {
      const uint64_t dst = reinterpret_cast<uint64_t>(out) + uint64_t(D);
      if (uint64_t(D) + 16 <= col.capacity) {
        st16<kNT>(dst, val[k]);
      } else {
        for (int b = 0; b < 16 && uint64_t(D) + b < col.capacity; ++b)
          out[D + b] = uint8_t(byte_of(val[k], b));
      }
    }
  }
  if (!utf8) return;
  // UTF-8: the 4 bytes before each chunk come from the previous lane (lane 0: the previous
  // wave's lane 63 through LDS; the tile's first chunk: assembled from its row).
#pragma unroll
  for (int k = 0; k < kGatherChunks; ++k)
    if (lane == 63) s_edge[k * (kBlock / 64) + wave] = val[k].w;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kGatherChunks; ++k) {
    const int c = threadIdx.x + kBlock * k;
    const int64_t D = T0 + 16 * c;
    uint32_t pw = __shfl_up(val[k].w, 1);
    if (lane == 0) {
      if (c == 0)
        pw = D > R.o(0) ? assemble<kNT>(R, 1, 0, D - 16, a.batch).w : 0u;
      else
        pw = s_edge[wave > 0 ? k * (kBlock / 64) + wave - 1 : (k - 1) * (kBlock / 64) + 3];
    }
    if (D < tot) utf8_check(R, n, jrow[k], D, tot, val[k], pw, col.flags, r0);
  }
}

template <bool kNT, int kGatherChunks>
__global__ __launch_bounds__(kBlock) void gather_ragged_kernel(const DevArgs a) {
  constexpr uint64_t kGatherTile = kMapGrain * kGatherChunks;
  __shared__ __attribute__((aligned(16))) int64_t s_off[kGatherRows + 1];
  __shared__ uint64_t s_src[kGatherRows];
  __shared__ uint32_t s_edge[kGatherChunks * (kBlock / 64)];
  // which ragged column / tile (block-uniform)
  int vi = 0;
  while (vi + 1 < a.nvar && blockIdx.x >= a.gather_block0[vi + 1]) ++vi;
  int ci = 0;
  while (a.cols[ci].var_index != vi) ++ci;
  const DevCol& col = a.cols[ci];
  const int64_t tot = col.offsets[a.rows];
  // a decode error other than per-sample ones (empty sample, range) leaves offsets unreliable
  const uint32_t kinds =
      *reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(a.status) + kErrKindsOffset);
  if (kinds & ~kRowLevelErrors) return;
  const uint32_t* map = a.row_map + uint64_t(vi) * a.map_len;
  const uint64_t* src = a.src_abs + uint64_t(vi) * a.rows;
  const uint64_t stride = a.gather_block0[vi + 1] - a.gather_block0[vi];
  for (uint64_t g = blockIdx.x - a.gather_block0[vi];; g += stride) {  // block-uniform loop
    const int64_t T0 = int64_t(g * kGatherTile);
    if (T0 >= tot || (g + 1) * kGatherChunks >= a.map_len) return;
    const uint64_t r0 = map[g * kGatherChunks];
    const uint64_t r1 =
        (T0 + int64_t(kGatherTile) < tot) ? uint64_t(map[(g + 1) * kGatherChunks]) : a.rows - 1;
    if (r0 >= a.rows || r1 >= a.rows || r1 < r0) return;  // never for a status-clean decode
    const int n = int(r1 - r0 + 1);
    __syncthreads();  // the previous tile's readers of s_off / s_src / s_edge
    if (n <= kGatherRows) {
      for (int i = threadIdx.x; i <= n; i += kBlock) {
        s_off[i] = col.offsets[r0 + i];
        if (i < n) s_src[i] = src[r0 + i];
      }
      __syncthreads();
      gather_tile<kNT, kGatherChunks>(a, col, RowsLds{s_off, s_src}, n, r0, T0, tot, s_edge);
    } else {
      gather_tile<kNT, kGatherChunks>(a, col, RowsGlobal{col.offsets + r0, src + r0}, n, r0,
                                      T0, tot, s_edge);
    }
  }
}

// ---------------------------------------------------------------------------------------------
struct Layout {
  uint64_t tile_total, tile_prefix, chunk_sum, tile_run, src_abs, row_map, sw_rec, map_len,
      total;
};

__host__ uint64_t round256(uint64_t x) { return (x + 255) & ~uint64_t(255); }

// Host code below uses std::min / std::max: HIP's global host min / max are int-only and
// truncate 64-bit sizes.
constexpr uint64_t kTicketOffset = 128;  // single-pass tile ticket, inside the status block

Layout workspace_layout(const mdsx_plan* plan, const mdsx_batch* b) {
  Layout L;
  const uint64_t nv = uint64_t(plan->nvar);
  L.map_len = b->bytes / kMapGrain + 8;
  L.tile_total = 256;
  L.tile_prefix = L.tile_total + round256(nv * b->ntiles * 8);
  L.chunk_sum = L.tile_prefix + round256(nv * b->ntiles * 8);
  L.tile_run = L.chunk_sum + round256(nv * (b->ntiles / kScanChunk + 1) * 8);
  L.src_abs = L.tile_run + round256(nv ? uint64_t(b->ntiles) * sizeof(TileRun) : 0);
  L.row_map = L.src_abs + round256(nv * b->rows * 8);
  L.sw_rec = L.row_map + round256(nv * L.map_len * 4);
  L.total = L.sw_rec + round256(use_swave_decode(plan, b->bytes, b->rows)
                                    ? uint64_t(b->ntiles) *
                                          uint64_t(b->tile_rows ? b->tile_rows
                                                                : uint32_t(plan->tile_rows)) * 16
                                    : 0);
  return L;
}

// mode_bytes (host, [ncols], may be null): the expected bytes of each ragged column, which pick
// its copy mode and size its gather grid; null = outs[c].capacity (the two-pass decode, where the
// capacity is the scanned total or close to it).
int build_args(const mdsx_plan* plan, const mdsx_batch* b, const mdsx_column_out* outs,
               void* d_workspace, uint64_t workspace_bytes, int64_t* d_totals, DevArgs* a,
               const uint64_t* mode_bytes = nullptr) {
  if (!plan || !b || !b->data || !b->shards || !b->tile_shard || !d_workspace ||
      b->nshards <= 0)
    return mdsx::fail(MDSX_E_ARG, "mdsx: null argument or empty batch");
  if (plan->ncols > 0 && !outs) return mdsx::fail(MDSX_E_ARG, "mdsx: outs is NULL");
  const Layout L = workspace_layout(plan, b);
  if (workspace_bytes < L.total)
    return mdsx::fail(MDSX_E_ARG, "mdsx: workspace smaller than mdsx_workspace_bytes()");
  std::memset(a, 0, sizeof(*a));
  a->batch = b->data;
  a->shards = b->shards;
  a->tile_shard = b->tile_shard;
  uint8_t* ws = static_cast<uint8_t*>(d_workspace);
  a->status = reinterpret_cast<mdsx_status*>(ws);
  a->tile_total = reinterpret_cast<int64_t*>(ws + L.tile_total);
  a->tile_prefix = reinterpret_cast<int64_t*>(ws + L.tile_prefix);
  a->chunk_sum = reinterpret_cast<int64_t*>(ws + L.chunk_sum);
  a->tile_run = reinterpret_cast<TileRun*>(ws + L.tile_run);
  a->src_abs = reinterpret_cast<uint64_t*>(ws + L.src_abs);
  a->row_map = reinterpret_cast<uint32_t*>(ws + L.row_map);
  a->sw_rec = reinterpret_cast<uint4*>(ws + L.sw_rec);
  a->lookback = reinterpret_cast<uint64_t*>(ws + L.tile_total);  // single pass: no tile totals
  a->ticket = reinterpret_cast<uint32_t*>(ws + kTicketOffset);
  a->map_len = L.map_len;
  a->totals = d_totals;
  a->rows = b->rows;
  a->ntiles = b->ntiles;
  const int tr = b->tile_rows ? int(b->tile_rows) : plan->tile_rows;
  if (tr < 1 || tr > kBlock || (tr & (tr - 1)))
    return mdsx::fail(MDSX_E_ARG, "mdsx: batch tile_rows must be a power of two in [1, 256]");
  a->stage_debug = uint32_t(plan->stage_debug);
  a->xcd_order = uint32_t(plan->xcd_order);
  a->rw_k = uint32_t(plan->rowwave_k);
  a->swave = use_swave_decode(plan, b->bytes, b->rows) ? 1u : 0u;
  a->run_slots = use_run_decode(plan, b->bytes, b->rows) && !a->swave ? uint32_t(plan->run_slots)
                                                                      : 0u;
  if (a->run_slots && plan->seg) {
    // lean path: a sample must fit the ring with a slot to spare (seg_decode_kernel)
    a->seg_lim = a->run_slots * 1024u - 1024u - 32u;
    for (int c = 0; c < plan->ncols; ++c)
      if (plan->cols[c].kind == MDSX_KIND_FIXED && plan->cols[c].row_bytes <= kSmallMax)
        a->seg_small += uint32_t(plan->cols[c].row_bytes);
  }
  a->rows_bytes = use_rows_decode(plan, b->bytes, b->rows)
                      ? rows_stage_bytes(plan, b->bytes / b->rows, tr)
                      : 0u;
  // (a batch tiled for another decode, too wide for the row-parallel workgroup's LDS: the register
  // decode)
  if (a->rows_bytes && rows_lds_bytes_est(plan, a->rows_bytes, uint64_t(tr)) > 160 * 1024)
    a->rows_bytes = 0;
  a->rows_pipe = a->rows_bytes ? uint32_t(plan->rows_pipe) : 0u;
  if (a->run_slots && tr > 32)
    return mdsx::fail(MDSX_E_ARG, "mdsx: streaming decode tiles hold at most 32 rows");
  // the staged and streaming decodes scan one total per tile; the register-copy decode one per
  // 256 rows
  a->scan_per = (a->run_slots || a->rows_bytes) ? 1u : uint32_t(kBlock / tr);
  a->nscan = (b->ntiles + a->scan_per - 1) / a->scan_per;
  a->nchunk = (a->nscan + kScanChunk - 1) / kScanChunk;
  a->nshards = b->nshards;
  a->ncols = plan->ncols;
  a->nvar = plan->nvar;
  a->tile_rows = tr;
  uint32_t gblocks = 0;
  const uint64_t tile = kMapGrain * uint64_t(plan->gather_chunks);
  for (int c = 0; c < plan->ncols; ++c) {
    const mdsx::ColumnSpec& s = plan->cols[c];
    DevCol& d = a->cols[c];
    d.data = outs[c].data;
    d.offsets = outs[c].offsets;
    d.flags = outs[c].flags;
    d.capacity = outs[c].capacity;
    d.row_bytes = uint32_t(s.row_bytes);
    d.kind = int8_t(s.kind);
    d.var_index = int8_t(s.var_index);
    const uint64_t expect =
        mode_bytes ? std::min(mode_bytes[c], outs[c].capacity) : outs[c].capacity;
    // Short ragged rows keep a wave's lanes busy only when copied destination-major.
    d.gather = s.kind != MDSX_KIND_FIXED && b->rows > 0 &&
               expect < uint64_t(plan->gather_min) * b->rows;
    // Medium rows (a few hundred bytes): four per wave, one per 16-lane group (decided below).
    d.group = s.kind != MDSX_KIND_FIXED && !d.gather && b->rows > 0 &&
              expect < uint64_t(plan->group_max) * b->rows;
    if (s.kind == MDSX_KIND_FIXED) {
      if (!d.data && b->rows > 0)
        return mdsx::fail(MDSX_E_ARG, "mdsx: null data pointer for a fixed column");
    } else {
      if (!d.offsets || (!d.data && d.capacity > 0))
        return mdsx::fail(MDSX_E_ARG, "mdsx: null offsets/data for a ragged column");
    }
  }
  for (int c = 0; c < plan->ncols; ++c) {
    const DevCol& d = a->cols[c];
    if (d.group) a->any_group = 1;
    if (d.kind != MDSX_KIND_FIXED && !d.gather && !d.group) a->any_wave_ragged = 1;
    if (d.kind == MDSX_KIND_STR && d.flags && !d.gather) a->any_wave_str = 1;
    a->str_cached = int16_t(plan->str_cached);
  }
  for (int v = 0; v < plan->nvar; ++v) {  // gather workgroups of each ragged column, in order
    a->gather_block0[v] = gblocks;
    for (int c = 0; c < plan->ncols; ++c)
      if (plan->cols[c].var_index == v && a->cols[c].gather) {
        // every workgroup loops over the column's tiles with the column's grid as its stride
        const uint64_t expect =
            mode_bytes ? std::min(mode_bytes[c], outs[c].capacity) : outs[c].capacity;
        gblocks += uint32_t(expect > tile ? (expect + tile - 1) / tile : 1);
      }
  }
  a->gather_block0[plan->nvar] = gblocks;
  return MDSX_OK;
}

int hip_check(hipError_t e, const char* what) {
  if (e == hipSuccess) return MDSX_OK;
  return mdsx::fail(MDSX_E_HIP, std::string(what) + ": " + hipGetErrorString(e));
}

// HBM roofline probe: the fastest plain stream measured on MI355X (scripts/microbench/
// copy_ceiling.hip): each workgroup copies a contiguous 256 KiB, 8 x 16 B per lane in flight,
// non-temporal. Reported next to the decode rate as the measured copy ceiling.
constexpr uint64_t kProbeBlock = 256 * 1024 / 16;  // 16-byte units per workgroup
__global__ __launch_bounds__(kBlock) void copy_probe_kernel(const uint4* __restrict__ src,
                                                            uint4* __restrict__ dst, uint64_t n) {
  const uint64_t b0 = uint64_t(blockIdx.x) * kProbeBlock;
  const uint64_t b1 = b0 + kProbeBlock < n ? b0 + kProbeBlock : n;
  for (uint64_t base = b0; base < b1; base += kBlock * 8) {
    uint4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint64_t i = base + u * kBlock + threadIdx.x;
      if (i < b1) v[u] = ld16<true>(src + i);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint64_t i = base + u * kBlock + threadIdx.x;
      if (i < b1) st16<true>(reinterpret_cast<uint64_t>(dst + i), v[u]);
    }
  }
}

// ---- All-fixed plans, one row per wave (MDSX_TUNE rw = waves per workgroup) ----------------
// decode_kernel reads a tile's offsets into LDS and meets them at a workgroup barrier before any
// row's bytes are requested, so every row's copy waits for two dependent memory round trips. In
// an all-fixed schema every sample has the same size, and the writer lays sample i at offsets[0]
// + i x size (mds/writer.py:133-144: the header, the shard's config bytes, then the samples back
// to back): this kernel requests the row's bytes from there once offsets[0] is known (one line
// per shard, read by every wave of it), the row's offsets pair beside them, and stores only once
// the pair confirms the address; a row whose pair says otherwise takes the checked path from its
// offsets (decode_kernel's rules and reports: mds/reader.py:137-142 ranges, a row too short for
// its columns). Reads of the predicted address stay inside the shard. One wave per row, kW waves per workgroup; the launch
// sets the workgroups per CU (unused LDS): fewer, longer-lived streams copy faster on MI355X.
// The large columns of one row, from column c on, from sample byte b of the shard (wave_copy).
template <int U, bool kNT>
__device__ __forceinline__ void rowwave_columns(const DevArgs& a, const TileView& v, uint32_t b,
                                                uint64_t row, int c, int lane) {
  uint32_t pos = 0;
  for (int j = 0; j < c; ++j) pos += a.cols[j].row_bytes;
  for (; c < a.ncols; ++c) {  // uniform
    const DevCol& col = a.cols[c];
    if (col.row_bytes > uint32_t(kSmallMax))
      wave_copy<false, U, kNT>(v.shard + b + pos,
                               static_cast<uint8_t*>(col.data) + row * col.row_bytes,
                               col.row_bytes, lane);
    pos += col.row_bytes;
  }
}

// kR consecutive rows per wave (1, 2 or 4; the tile's rows a multiple), all of their bytes in
// flight together. kOcc > 0: registers bounded for that many waves per SIMD. kX (measurement
// only, MDSX_TUNE rwx; correct only on the writer's layout with rw_k config bytes): bit 1 no
// offsets pair (every row taken as predicted), bit 2 offsets[0] not loaded (hdr_end + rw_k),
// bit 4 (outputs incomplete) no small column loaded or stored.
template <bool kNT, int kW, int kR = 1, int kOcc = 0, int kX = 0>
__global__ __launch_bounds__(64 * kW, kOcc > 0 ? kOcc : 1) void rowwave_decode_kernel(const DevArgs a) {
  constexpr int U = 4;  // 16-byte chunks per lane in flight: a column of up to 4 KiB in one step
  const int lane = threadIdx.x & 63;
  const uint32_t blk =
      (a.xcd_order & kXcdRegister) ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint32_t w =
      blk * kW + (kW == 1 ? 0u : uint32_t(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)));
  const uint32_t per = uint32_t(a.tile_rows) / kR;  // waves per tile
  const uint32_t tile = w / per, rw0 = (w - tile * per) * kR;
  if (tile >= a.ntiles) return;  // wave-uniform; no barrier in this kernel
  const TileView v = tile_view(a, tile);
  if (!v.table_ok) {
    if (rw0 == 0 && lane == 0 && tile == v.d.tile0)
      report_decode(a, MDSX_E_HEADER, v.shard_idx, -1, -1);
    return;
  }
  if (rw0 == 0 && lane == 0 && tile == v.d.tile0) {
    // the shard header (mds/writer.py:133-144): u32 N, then N + 1 offsets
    const uint32_t n = *reinterpret_cast<const uint32_t*>(v.shard);
    if (n != v.d.samples || v.offs[0] < v.hdr_end || v.offs[v.d.samples] > v.d.bytes)
      report_decode(a, MDSX_E_HEADER, v.shard_idx, -1, -1);
  }
  if (rw0 >= v.nrows) return;
  const uint32_t nr = min(uint32_t(kR), v.nrows - rw0);  // this wave's rows
  const uint32_t i0 = v.r0 + rw0;
  const uint64_t row0 = v.d.row0 + i0;
  // the row size, lane c's column offset inside the sample, the first large column
  const int ncols = a.ncols;
  uint32_t size = 0, coff = 0, rb = 0, coff_l = 0, rb_l = 0;
  int cl = -1;
  for (int c = 0; c < ncols; ++c) {  // uniform
    const uint32_t b = a.cols[c].row_bytes;
    if (lane == c) coff = size, rb = b;
    if (cl < 0 && b > uint32_t(kSmallMax)) cl = c, coff_l = size, rb_l = b;
    size += b;
  }
  const bool small = !(kX & 4) && lane < ncols && rb <= uint32_t(kSmallMax);
  // the writer's layout: offsets[0] (after the header and the shard's config bytes) + i x size
  const uint32_t o0 = (kX & 2) ? uint32_t(v.hdr_end) + a.rw_k
                              : __builtin_amdgcn_readfirstlane(v.offs[0]);  // (one line per shard)
  const bool spec0 = o0 >= v.hdr_end;
  // offsets[i0 .. i0 + nr], the rows' offsets pairs: every lane loads the same word and reads it
  // back with readfirstlane (an active lane's copy: no cross-lane read of a lane that may be
  // inactive where the register is reloaded)
  uint32_t obv[kR + 1];
#pragma unroll
  for (int k = 0; k <= kR; ++k)
    obv[k] = (kX & 1) ? o0 + (i0 + uint32_t(k)) * size : k <= int(nr) ? v.offs[i0 + uint32_t(k)] : 0u;
  // ---- requested together: the offsets, each row's small columns (lane c: column c) and first
  // large column's chunks (wave_copy's realigning layout), from the predicted addresses
  const uint64_t data_l = cl >= 0 ? reinterpret_cast<uint64_t>(a.cols[cl].data) : 0;
  uint4 o[kR];
  uint4 lo[kR][U];
  uint4 tail[kR];
  bool one[kR];
#pragma unroll
  for (int j = 0; j < kR; ++j) {
    const uint64_t pred = uint64_t(o0) + uint64_t(i0 + j) * size;
    const bool spec = j < int(nr) && spec0 && pred + size <= v.d.bytes;  // wave-uniform
    o[j] = spec && small ? small_load(v.shard + pred + coff, rb) : make_uint4(0, 0, 0, 0);
    const uint64_t d0 = data_l + (row0 + j) * rb_l, dend = d0 + rb_l;
    const uint64_t dbeg = d0 & ~uint64_t(15);
    const uint32_t nch = uint32_t((((dend + 15) & ~uint64_t(15)) - dbeg) >> 4);
    one[j] = spec && cl >= 0 && nch <= 64u * U;
    const uint64_t sfirst = reinterpret_cast<uint64_t>(v.shard + pred + coff_l) - (d0 - dbeg);
    const uint32_t nload = nch + ((sfirst & 15) ? 1u : 0u);
    const uint4* sal = reinterpret_cast<const uint4*>(sfirst & ~uint64_t(15));
    tail[j] = make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t k = uint32_t(u) * 64u + uint32_t(lane);
      lo[j][u] = one[j] && k < nload ? ld16<kNT>(sal + k) : make_uint4(0, 0, 0, 0);
    }
    if (one[j] && (sfirst & 15) && lane == 63 && 64u * U < nload) tail[j] = ld16<kNT>(sal + 64u * U);
  }
#pragma unroll
  for (int j = 0; j < kR; ++j) {
    if (j >= int(nr)) break;  // uniform
    const uint32_t i = i0 + j;
    const uint64_t row = row0 + j;
    const uint64_t pred = uint64_t(o0) + uint64_t(i) * size;
    const uint32_t b = __builtin_amdgcn_readfirstlane(obv[j]);
    const uint32_t e = __builtin_amdgcn_readfirstlane(obv[j + 1]);
    if (spec0 && pred + size <= v.d.bytes && b == pred && e >= b && e - b >= size &&
        e <= v.d.bytes) {  // the predicted address holds
      if (small) small_store(static_cast<uint8_t*>(a.cols[lane].data) + row * rb, o[j], rb);
      int c = cl;
      if (one[j]) {  // the first large column from the registers
        const uint64_t d0 = data_l + row * rb_l, dend = d0 + rb_l;
        const uint64_t dbeg = d0 & ~uint64_t(15);
        const uint32_t nch = uint32_t((((dend + 15) & ~uint64_t(15)) - dbeg) >> 4);
        const uint32_t sh = uint32_t((reinterpret_cast<uint64_t>(v.shard + pred + coff_l) -
                                      (d0 - dbeg)) & 15);
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const uint32_t k0 = uint32_t(u) * 64u;
          if (k0 >= nch) break;  // wave-uniform
          const uint32_t k = k0 + uint32_t(lane);
          uint4 out = lo[j][u];
          if (sh != 0) {
            uint4 hi = shfl_down1(lo[j][u]);
            const uint4 nxt = (u + 1 < U) ? readlane0(lo[j][u + 1 < U ? u + 1 : u]) : tail[j];
            if (lane == 63) hi = nxt;
            out = funnel16(lo[j][u], hi, sh);
          }
          const uint64_t D = dbeg + 16ull * k;
          if (k < nch && D >= d0 && D + 16 <= dend) st16<kNT>(D, out);
          if (k0 == 0 && (dbeg < d0 || dbeg + 16 > dend))
            wave_edge_store(out, 0, dbeg, d0, dend, lane);
          if (nch > 1 && (dend & 15) != 0 && nch - 1 >= k0 && nch - 1 < k0 + 64)
            wave_edge_store(out, int(nch - 1 - k0), dbeg + 16ull * (nch - 1), d0, dend, lane);
        }
        ++c;
      }
      if (c >= 0) rowwave_columns<U, kNT>(a, v, b, row, c, lane);  // the other large columns
      continue;
    }
    // ---- the checked path (decode_kernel's): the row's range and columns from its offsets
    uint32_t bb = 0, ee = 0;
    int rc = sample_range(v, i, &bb, &ee);
    if (rc == MDSX_OK && uint64_t(bb) + size > ee) rc = MDSX_E_BOUNDS;
    if (rc != MDSX_OK) {
      if (lane == 0) report_decode(a, rc, v.shard_idx, int(i), -1);
      continue;
    }
    if (small)
      gather_small(v.shard + bb + coff, static_cast<uint8_t*>(a.cols[lane].data) + row * rb, rb);
    rowwave_columns<U, kNT>(a, v, bb, row, 0, lane);
  }
}

// The same stream cut per wave: each wave copies its own contiguous kU x 1 KiB (64 lanes x 16 B,
// kU loads per lane in flight, then kU stores) -- the access shape of the config-B decode's row
// copy (one 4 KiB row per wave), which outruns the 256 KiB-per-workgroup loop above on MI355X.
// kXcd: workgroups dealt to the 8 XCDs in contiguous ranges (xcd_block), the tile order of the
// register decode (config B) -- the line two neighbouring workgroups share meets in one L2.
// kWaves: waves per workgroup.
template <int kU, bool kNTLoad, bool kNTStore, bool kXcd = false, int kWaves = kBlock / 64>
__global__ __launch_bounds__(64 * kWaves) void copy_wave_kernel(const uint4* __restrict__ src,
                                                                uint4* __restrict__ dst,
                                                                uint64_t n) {
  const uint32_t blk = kXcd ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint64_t w = uint64_t(blk) * kWaves + (threadIdx.x >> 6);
  const uint64_t b0 = w * (64 * kU) + (threadIdx.x & 63);
  uint4 v[kU];
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const uint64_t i = b0 + 64 * u;
    if (i < n) v[u] = ld16<kNTLoad>(src + i);
  }
#pragma unroll
  for (int u = 0; u < kU; ++u) {
    const uint64_t i = b0 + 64 * u;
    if (i < n) st16<kNTStore>(reinterpret_cast<uint64_t>(dst + i), v[u]);
  }
}


// ---------------------------------------------------------------------------------------------
// Batch gather by sample id: out[k] = column[idx[k]] for decoded columns, the
// device side of StreamingDataset.__iter__'s per-sample get_item over a worker's sample ids
// (dataset.py:1430-1473). One launch sequence per column.

constexpr int kGatherRowTile = 256;  // rows of the output per workgroup

// Where the rows come from. OneSrc: one decoded column, ids are its rows. MultiSrc: a device
// table of decoded columns (one per shard a batch touches), ids are source << 40 | row -- a
// batch over many shards in ONE launch sequence per column, rows in the caller's order (the
// reference's Spanner lookup, spanner.py:40-59, done by the caller).
struct OneSrc {
  const uint8_t* vals;
  const int64_t* off;
  const uint8_t* flags;
  uint64_t rows;
  __device__ __forceinline__ bool resolve(int64_t id, mdsx_gather_src* g, uint64_t* r) const {
    if (id < 0 || uint64_t(id) >= rows) return false;
    g->values = vals;
    g->offsets = off;
    g->flags = flags;
    *r = uint64_t(id);
    return true;
  }
};

struct MultiSrc {
  const mdsx_gather_src* table;
  uint32_t n;
  __device__ __forceinline__ bool resolve(int64_t id, mdsx_gather_src* g, uint64_t* r) const {
    const uint64_t s = uint64_t(id) >> MDSX_GATHER_SRC_SHIFT;
    if (id < 0 || s >= n) return false;
    *g = table[s];
    *r = uint64_t(id) & ((uint64_t(1) << MDSX_GATHER_SRC_SHIFT) - 1);
    return *r < g->rows;
  }
};

// Fixed column: one output row per wave (rows > 16 bytes) or per lane (<= 16 bytes).
template <bool kNT, class Src>
__global__ __launch_bounds__(kBlock) void gather_fixed_kernel(const Src S, uint32_t row_bytes,
                                                              const int64_t* idx, uint64_t m,
                                                              uint8_t* dst, mdsx_status* st) {
  const uint64_t k0 = uint64_t(blockIdx.x) * kGatherRowTile;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (row_bytes <= uint32_t(kSmallMax)) {
    const uint64_t k = k0 + threadIdx.x;
    if (k < m) {
      mdsx_gather_src g;
      uint64_t r;
      if (!S.resolve(idx[k], &g, &r)) {
        report(st, MDSX_E_BOUNDS, -1, int(k), -1);
      } else {
        const MDSX_G uint8_t* p = gp(static_cast<const uint8_t*>(g.values) + r * row_bytes);
        MDSX_G uint8_t* q = gp(dst + k * row_bytes);  // both rows aligned to row_bytes'
        switch (row_bytes) {                          // power-of-two factor
          case 1: *q = *p; break;
          case 2: *(MDSX_G uint16_t*)q = *(const MDSX_G uint16_t*)p; break;
          case 4: *(MDSX_G uint32_t*)q = *(const MDSX_G uint32_t*)p; break;
          case 8: *(MDSX_G uint64_t*)q = *(const MDSX_G uint64_t*)p; break;
          case 16: *(MDSX_G u32x4*)q = *(const MDSX_G u32x4*)p; break;
          default:
            for (uint32_t j = 0; j < row_bytes; ++j) q[j] = p[j];
        }
      }
    }
    return;
  }
  const bool aligned = (row_bytes & 15) == 0;
  for (int i = wave; i < kGatherRowTile; i += kBlock / 64) {
    const uint64_t k = k0 + i;
    if (k >= m) break;  // wave-uniform
    mdsx_gather_src g;
    uint64_t r;
    if (!S.resolve(idx[k], &g, &r)) {
      if (lane == 0) report(st, MDSX_E_BOUNDS, -1, int(k), -1);
      continue;
    }
    const uint8_t* src = static_cast<const uint8_t*>(g.values) + r * row_bytes;
    if (aligned)
      wave_copy<false, 4, kNT, false>(src, dst + k * row_bytes, row_bytes, lane);
    else
      wave_copy<false, 4, kNT, true, true>(src, dst + k * row_bytes, row_bytes, lane);
  }
}

// Ragged column, pass 1: selected lengths -> local exclusive offsets + per-tile totals.
template <class Src>
__global__ __launch_bounds__(kBlock) void gather_len_kernel(const Src S, const int64_t* idx,
                                                            uint64_t m, int64_t* dst_off,
                                                            int64_t* tile_total, mdsx_status* st) {
  __shared__ int64_t s_wsum[kBlock / 64];
  const uint64_t k = uint64_t(blockIdx.x) * kGatherRowTile + threadIdx.x;
  int64_t len = 0;
  if (k < m) {
    mdsx_gather_src g;
    uint64_t r;
    if (!S.resolve(idx[k], &g, &r))
      report(st, MDSX_E_BOUNDS, -1, int(k), -1);
    else
      len = g.offsets[r + 1] - g.offsets[r];
  }
  int64_t total;
  const int64_t excl = block_exclusive_scan(len, s_wsum, &total);
  if (k < m) dst_off[k] = excl;
  if (threadIdx.x == 0) tile_total[blockIdx.x] = total;
}

// Exclusive scan of n tile totals (one workgroup); total -> *out_total and dst_off[m].
__global__ __launch_bounds__(kBlock) void scan_tile_totals_kernel(const int64_t* in, int64_t* out,
                                                                  uint32_t n, int64_t* dst_off,
                                                                  uint64_t m, int64_t* out_total) {
  __shared__ int64_t s_wsum[kBlock / 64];
  int64_t carry = 0;
  for (uint32_t base = 0; base < n; base += kBlock) {
    const uint32_t k = base + threadIdx.x;
    const int64_t x = k < n ? in[k] : 0;
    int64_t total;
    const int64_t excl = block_exclusive_scan(x, s_wsum, &total);
    if (k < n) out[k] = carry + excl;
    carry += total;
  }
  if (threadIdx.x == 0) {
    dst_off[m] = carry;
    if (out_total) *out_total = carry;
  }
}

// Ragged column, pass 2: final offsets, flags, and the rows copied: one per wave, or (kGroup,
// rows of a few hundred bytes) four per wave, one per 16-lane group.
template <bool kNT, bool kGroup, class Src>
__global__ __launch_bounds__(kBlock) void gather_copy_kernel(
    const Src S, const int64_t* idx, uint64_t m, uint8_t* dst_vals, uint64_t capacity,
    int64_t* dst_off, uint8_t* dst_flags, const int64_t* tile_prefix, mdsx_status* st) {
  __shared__ const uint8_t* s_src[kGatherRowTile];
  __shared__ int64_t s_dst[kGatherRowTile];
  __shared__ int64_t s_len[kGatherRowTile];
  const uint64_t k0 = uint64_t(blockIdx.x) * kGatherRowTile;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  {
    const uint64_t k = k0 + threadIdx.x;
    int64_t len = -1;
    if (k < m) {
      const int64_t off = tile_prefix[blockIdx.x] + dst_off[k];
      dst_off[k] = off;
      s_dst[threadIdx.x] = off;
      mdsx_gather_src g;
      uint64_t r;
      if (S.resolve(idx[k], &g, &r)) {
        s_src[threadIdx.x] = static_cast<const uint8_t*>(g.values) + g.offsets[r];
        len = g.offsets[r + 1] - g.offsets[r];
        if (uint64_t(off + len) > capacity) {
          report(st, MDSX_E_CAPACITY, -1, int(k), -1);
          len = -1;
        }
        if (dst_flags) dst_flags[k] = g.flags ? g.flags[r] : 0;
      }
    }
    s_len[threadIdx.x] = len;
  }
  __syncthreads();
  // the source is a caller's tensor, not a padded batch: load only chunks touching the row
  if constexpr (kGroup) {
    const int g = lane >> 4;
    for (int r0 = wave * 4; r0 < kGatherRowTile; r0 += kBlock / 16) {
      if (k0 + r0 >= m) break;  // wave-uniform
      const int i = r0 + g;
      const bool live = k0 + i < m && s_len[i] > 0;
      group_copy<2, kNT, true>(live ? s_src[i] : dst_vals, live ? dst_vals + s_dst[i] : dst_vals,
                               live ? uint64_t(s_len[i]) : 0, lane);
    }
  } else {
    for (int i = wave; i < kGatherRowTile; i += kBlock / 64) {
      if (k0 + i >= m) break;
      const int64_t len = s_len[i];
      if (len <= 0) continue;  // wave-uniform
      wave_copy<false, 4, kNT, true, true>(s_src[i], dst_vals + s_dst[i], uint64_t(len), lane);
    }
  }
}


// ---------------------------------------------------------------------------------------------
// Dynamic ndarray columns ('ndarray', 'ndarray:<dtype>'): per-row header parse over the decoded
// ragged values -- NDArray.decode (encodings.py:270-305): [dtype id: u8 if dynamic]
// [ndim << 2 | shape dtype: u8][shape: ndim x u8/u16/u32/u64][values]. One row per lane.
__device__ __forceinline__ bool value_dtype_ok(uint32_t id) {
  return id == 8 || id == 9 || id == 16 || id == 17 || id == 18 || id == 32 || id == 33 ||
         id == 34 || id == 64 || id == 65 || id == 66;
}

__device__ __forceinline__ uint64_t read_uint(const uint8_t* p, int nbytes) {
  uint64_t v = 0;
  for (int b = 0; b < nbytes; ++b) v |= uint64_t(p[b]) << (8 * b);
  return v;
}

template <bool kShapes>
__global__ __launch_bounds__(kBlock) void ndarray_meta_kernel(
    const uint8_t* values, const int64_t* offsets, uint64_t rows, int dtype_id, uint8_t* out_dtype,
    uint8_t* out_ndim, int64_t* out_data_offset, int64_t* out_numel, uint8_t* out_bad,
    int32_t* max_ndim, int32_t shape_cols, int64_t* out_shape) {
  const uint64_t r = uint64_t(blockIdx.x) * kBlock + threadIdx.x;
  if (r >= rows) return;
  const int64_t b = offsets[r], e = offsets[r + 1];
  const uint8_t* p = values + b;
  const int64_t len = e - b;
  int64_t pos = 0;
  bool bad = false;
  uint32_t id = uint32_t(dtype_id);
  if (id == 0) {
    if (len < 1) bad = true;
    else id = p[pos++];
    if (!bad && !value_dtype_ok(id)) bad = true;
  }
  uint32_t ndim = 0, code = 0;
  if (!bad) {
    if (pos + 1 > len) bad = true;
    else {
      const uint32_t byte = p[pos++];
      ndim = byte >> 2;
      code = byte & 3;
    }
  }
  // shape = frombuffer(data[index:index + ndim * sbytes], shape dtype): a truncated header
  // yields fewer dims (or raises when the tail is not whole dims); the values then start past
  // the end and are empty.
  const int sbytes = 1 << code;
  const int64_t want = int64_t(ndim) * sbytes;
  if (!bad && want > len - pos) {
    if ((len - pos) % sbytes) bad = true;
    else ndim = uint32_t((len - pos) / sbytes);
  }
  // numpy's size rule (PyArray_NewFromDescr): zero dims make the array empty, the product of
  // the non-zero dims times the item size must fit in intp; dims above intp max raise.
  const int64_t item = int64_t(id >> 3);
  int64_t prod = item;
  bool zero = false;
  if (!bad) {
    for (uint32_t k = 0; k < ndim; ++k) {
      const uint64_t dim = read_uint(p + pos + k * sbytes, sbytes);
      if (kShapes && int32_t(k) < shape_cols) out_shape[r * shape_cols + k] = int64_t(dim);
      if (dim > uint64_t(INT64_MAX)) { bad = true; break; }
      if (dim == 0) { zero = true; continue; }
      if (__builtin_mul_overflow(prod, int64_t(dim), &prod)) { bad = true; break; }
    }
    pos = pos + want < len ? pos + want : len;
  }
  const int64_t numel = (bad || zero) ? 0 : prod / item;
  // frombuffer(data[index:], dtype).reshape(shape): the value bytes must be exactly numel items
  if (!bad && (len - pos) != numel * item) bad = true;
  if (kShapes) {
    for (int32_t k = int32_t(ndim); k < shape_cols; ++k) out_shape[r * shape_cols + k] = 1;
    return;
  }
  out_dtype[r] = uint8_t(bad ? 0 : id);
  out_ndim[r] = uint8_t(bad ? 0 : ndim);
  out_data_offset[r] = b + pos;
  out_numel[r] = bad ? 0 : numel;
  out_bad[r] = bad ? 1 : 0;
  if (!bad && max_ndim) atomicMax(max_ndim, int32_t(ndim));
}

}  // namespace mdsx_kernels

using namespace mdsx_kernels;

extern "C" {

uint64_t mdsx_workspace_bytes(const mdsx_plan* plan, const mdsx_batch* batch) {
  if (!plan || !batch) return 0;
  return workspace_layout(plan, batch).total;
}

}  // extern "C"

// Pass 1 of a ragged plan: tile totals, their scan, offsets and column totals.
static int scan_pass(const mdsx_plan* plan, const DevArgs& a, hipStream_t s) {
  int rc = MDSX_OK;
  if (a.ntiles > 0 && (a.run_slots || a.rows_bytes)) {
    // heads non-temporal for the row-parallel decode's short samples (plan->scan_nt -1: auto)
    const bool nt = plan->scan_nt >= 0 ? plan->scan_nt != 0 : a.run_slots == 0;
    rc = launch_stage_totals(a, nt, s);
    if (rc != MDSX_OK) return rc;
  } else if (a.ntiles > 0 && a.swave) {
    hipLaunchKernelGGL(scan_tiles_kernel<true>, dim3(a.nscan), dim3(kBlock), 0, s, a);
    rc = hip_check(hipGetLastError(), "scan_tiles_kernel launch");
    if (rc != MDSX_OK) return rc;
  } else if (a.ntiles > 0) {
    hipLaunchKernelGGL(scan_tiles_kernel<false>, dim3(a.nscan), dim3(kBlock), 0, s, a);
    rc = hip_check(hipGetLastError(), "scan_tiles_kernel launch");
    if (rc != MDSX_OK) return rc;
  }
  if (a.nchunk) {
    hipLaunchKernelGGL(scan_chunks_kernel, dim3(a.nchunk, plan->nvar), dim3(kBlock), 0, s, a);
    rc = hip_check(hipGetLastError(), "scan_chunks_kernel launch");
    if (rc != MDSX_OK) return rc;
  }
  hipLaunchKernelGGL(scan_chunk_sums_kernel, dim3(plan->nvar), dim3(kBlock), 0, s, a);
  rc = hip_check(hipGetLastError(), "scan_chunk_sums_kernel launch");
  if (rc != MDSX_OK || !a.nchunk) return rc;
  hipLaunchKernelGGL(scan_apply_kernel, dim3(a.nchunk, plan->nvar), dim3(kBlock), 0, s, a);
  return hip_check(hipGetLastError(), "scan_apply_kernel launch");
}

extern "C" {

int mdsx_scan_shards(const mdsx_plan* plan, const mdsx_batch* batch, const mdsx_column_out* outs,
                     void* d_workspace, uint64_t workspace_bytes, int64_t* d_totals,
                     void* stream) {
  DevArgs a;
  int rc = build_args(plan, batch, outs, d_workspace, workspace_bytes, d_totals, &a);
  if (rc != MDSX_OK) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  rc = hip_check(hipMemsetAsync(d_workspace, 0, kStatusBlock, s), "hipMemsetAsync");
  if (rc != MDSX_OK || plan->nvar == 0) return rc;
  return scan_pass(plan, a, s);
}

}  // extern "C"

// The decode kernel (single: with its own look-back scan) and, for gather columns, the
// destination-major copy.
static int launch_decode(const mdsx_plan* plan, const DevArgs& a, hipStream_t s, bool single,
                         const uint64_t* mode_bytes) {
  int rc = MDSX_OK;
  if (a.swave) {  // one sample per wave: the register decode's scan pass, then the decode
    if (single && (rc = scan_pass(plan, a, s)) != MDSX_OK) return rc;
    return launch_swave_decode(plan, a, s);
  }
  if (plan->nvar > 0 && (a.run_slots > 0 || a.rows_bytes > 0)) {
    // the streaming and row-parallel decodes have no single-pass form: their scan pass, then
    // the decode (a look-back across the ~1000 tiles in flight measured slower than the pass:
    // profiles/r03/negative/rows_single_pass)
    if (single && (rc = scan_pass(plan, a, s)) != MDSX_OK) return rc;
    return a.run_slots > 0 ? launch_run_decode(plan, a, s) : launch_rows_decode(plan, a, s);
  }
  const size_t lds =
      size_t(a.tile_rows) * (12 * size_t(plan->nvar) + 4 * size_t(plan->ncols) + 1) + 16;
  const size_t dlds = lds + size_t(plan->lds_pad_kb) * 1024;  // (+ unused pad: occupancy)
  // All-fixed plans of rows >= 3 KiB: one row per wave (rowwave_decode_kernel), its copy issued
  // before the row's offsets are known, registers bounded for 6 waves per SIMD -- config B, in
  // one process on each of three boxes: 6.22-6.23 / 6.66 vs 5.96 / 6.51 TB/s for decode_kernel
  // (5 waves per SIMD: 6.15 / 6.43; profiles/r05/rowwave/). By row size (fixed_rows.json):
  // ahead from 3 KiB rows (+2 % at 3 KiB, +7 % at 8 KiB), behind below (-5 % at 2.5 KiB, -12 %
  // at 2 KiB, -63 % at 256 B: decode_kernel's row per lane and four rows per workgroup win).
  uint64_t row_size = 0;
  for (int c = 0; c < plan->ncols; ++c) row_size += plan->cols[c].row_bytes;
  const int rw = plan->rowwave >= 0 ? plan->rowwave : (row_size >= 3072 ? 1 : 0);
  if (plan->nvar == 0 && rw > 0) {
    const size_t pad = size_t(plan->lds_pad_kb) * 1024;
    const int rr = plan->rowwave_rows;  // rows per wave
    // registers bounded for rowwave_occ waves per SIMD: built for the default shape (one row per
    // one-wave workgroup, non-temporal); other shapes take the compiler's bound
    const int occ = plan->nontemporal && rw == 1 && rr == 1 ? plan->rowwave_occ : 0;
    if (a.tile_rows % rr != 0)
      return mdsx::fail(MDSX_E_ARG, "mdsx: rowwave: tile rows not a multiple of rows per wave");
#define MDSX_ROWWAVE(NT, WV, R)                                                                \
  if (bool(plan->nontemporal) == NT && rw == WV && rr == R && occ == 0) {                      \
    const void* fn = reinterpret_cast<const void*>(rowwave_decode_kernel<NT, WV, R>);           \
    if (pad > 64 * 1024 &&                                                                     \
        hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(pad)) !=        \
            hipSuccess)                                                                        \
      return mdsx::fail(MDSX_E_HIP, "mdsx: rowwave_decode_kernel LDS attribute");             \
    mdsx::set_last_kernel(R == 1 ? "rowwave_decode_kernel<" #NT ", " #WV ">"                  \
                                 : "rowwave_decode_kernel<" #NT ", " #WV ", " #R ">");         \
    const uint64_t waves = uint64_t(a.ntiles) * uint64_t(a.tile_rows / R);                     \
    hipLaunchKernelGGL((rowwave_decode_kernel<NT, WV, R>), dim3(unsigned((waves + WV - 1) / WV)), \
                       dim3(64 * WV), pad, s, a);                                              \
    return hip_check(hipGetLastError(), "rowwave_decode_kernel launch");                       \
  }
    MDSX_ROWWAVE(true, 1, 1)
    MDSX_ROWWAVE(true, 2, 1)
    MDSX_ROWWAVE(true, 4, 1)
    MDSX_ROWWAVE(false, 1, 1)
    MDSX_ROWWAVE(false, 2, 1)
    MDSX_ROWWAVE(false, 4, 1)
    MDSX_ROWWAVE(true, 1, 2)
    MDSX_ROWWAVE(true, 1, 4)
    MDSX_ROWWAVE(true, 2, 2)
#define MDSX_ROWWAVE_OCC(OCC)                                                                   \
  if (occ == OCC) {                                                                            \
    if (pad > 64 * 1024 &&                                                                     \
        hipFuncSetAttribute(reinterpret_cast<const void*>(rowwave_decode_kernel<true, 1, 1, OCC>), \
                            hipFuncAttributeMaxDynamicSharedMemorySize, int(pad)) != hipSuccess) \
      return mdsx::fail(MDSX_E_HIP, "mdsx: rowwave_decode_kernel LDS attribute");             \
    mdsx::set_last_kernel("rowwave_decode_kernel<true, 1, 1, " #OCC ">");                      \
    const uint64_t waves = uint64_t(a.ntiles) * uint64_t(a.tile_rows);                         \
    hipLaunchKernelGGL((rowwave_decode_kernel<true, 1, 1, OCC>), dim3(unsigned(waves)), dim3(64), \
                       pad, s, a);                                                             \
    return hip_check(hipGetLastError(), "rowwave_decode_kernel launch");                       \
  }
    if (plan->rowwave_x) {  // measurement variants
#define MDSX_ROWWAVE_X(X)                                                                       \
  if (occ == 6 && plan->rowwave_x == X) {                                                      \
    if (pad > 64 * 1024 &&                                                                     \
        hipFuncSetAttribute(reinterpret_cast<const void*>(rowwave_decode_kernel<true, 1, 1, 6, X>), \
                            hipFuncAttributeMaxDynamicSharedMemorySize, int(pad)) != hipSuccess) \
      return mdsx::fail(MDSX_E_HIP, "mdsx: rowwave_decode_kernel LDS attribute");             \
    mdsx::set_last_kernel("rowwave_decode_kernel<true, 1, 1, 6, " #X ">");                     \
    hipLaunchKernelGGL((rowwave_decode_kernel<true, 1, 1, 6, X>),                               \
                       dim3(unsigned(uint64_t(a.ntiles) * uint64_t(a.tile_rows))), dim3(64), pad, \
                       s, a);                                                                  \
    return hip_check(hipGetLastError(), "rowwave_decode_kernel launch");                       \
  }
      MDSX_ROWWAVE_X(1)
      MDSX_ROWWAVE_X(2)
      MDSX_ROWWAVE_X(3)
      MDSX_ROWWAVE_X(4)
      MDSX_ROWWAVE_X(7)
#undef MDSX_ROWWAVE_X
      return mdsx::fail(MDSX_E_ARG, "mdsx: rowwave measurement variants: rw=1, rwocc=6 only");
    }
    MDSX_ROWWAVE_OCC(6)
    MDSX_ROWWAVE_OCC(7)
    MDSX_ROWWAVE_OCC(8)
#undef MDSX_ROWWAVE_OCC
#undef MDSX_ROWWAVE
    return mdsx::fail(MDSX_E_ARG, "mdsx: rowwave: 1, 2 or 4 waves per workgroup (rows per wave "
                                 "2 / 4: 1 wave, nt; 2 / 2 waves, nt)");
  }
  const bool nt = plan->nontemporal != 0, ragged = plan->nvar > 0;
  // Edge (partial 16-byte chunk) stores are only needed for ragged columns and for large fixed
  // columns whose row size is not a multiple of 16 (outputs are 256-byte aligned).
  bool edges = ragged;
  for (int c = 0; c < plan->ncols; ++c)
    if (plan->cols[c].kind == MDSX_KIND_FIXED && plan->cols[c].row_bytes > kSmallMax &&
        plan->cols[c].row_bytes % 16 != 0)
      edges = true;
#define MDSX_DECODE(U, NT, RG, ED, SG)                                                           \
  do {                                                                                           \
    mdsx::set_last_kernel("decode_kernel<" #U ", " #NT ", " #RG ", " #ED ", " #SG ", 0>");       \
    if (dlds > 64 * 1024 &&                                                                      \
        hipFuncSetAttribute(reinterpret_cast<const void*>(decode_kernel<U, NT, RG, ED, SG>),     \
                            hipFuncAttributeMaxDynamicSharedMemorySize, int(dlds)) != hipSuccess)\
      return mdsx::fail(MDSX_E_HIP, "mdsx: decode_kernel LDS attribute");                       \
    hipLaunchKernelGGL((decode_kernel<U, NT, RG, ED, SG>), dim3(a.ntiles), dim3(kBlock), dlds, s, \
                       a);                                                                       \
  } while (0)
#define MDSX_DECODE_U(U)                                                 \
  do {                                                                   \
    if (ragged && single) {                                              \
      if (nt) MDSX_DECODE(U, true, true, true, true);                    \
      else MDSX_DECODE(U, false, true, true, true);                      \
    } else if (ragged) {                                                 \
      if (nt) MDSX_DECODE(U, true, true, true, false);                   \
      else MDSX_DECODE(U, false, true, true, false);                     \
    } else if (edges) {                                                  \
      if (nt) MDSX_DECODE(U, true, false, true, false);                  \
      else MDSX_DECODE(U, false, false, true, false);                    \
    } else {                                                             \
      if (nt) MDSX_DECODE(U, true, false, false, false);                 \
      else MDSX_DECODE(U, false, false, false, false);                   \
    }                                                                    \
  } while (0)
#define MDSX_RING(U, K)                                                                    \
  do {                                                                                     \
    mdsx::set_last_kernel(std::string("decode_kernel<" #U ", ") + (nt ? "true" : "false") + \
                          ", true, true, " + (single ? "true" : "false") + ", " #K ">");     \
    const size_t rl = ((lds + 15) & ~size_t(15)) + size_t(kBlock / 64) * (K)*1024;         \
    if (single) {                                                                          \
      if (nt)                                                                              \
        hipLaunchKernelGGL((decode_kernel<U, true, true, true, true, K>), dim3(a.ntiles),  \
                           dim3(kBlock), rl, s, a);                                        \
      else                                                                                 \
        hipLaunchKernelGGL((decode_kernel<U, false, true, true, true, K>), dim3(a.ntiles), \
                           dim3(kBlock), rl, s, a);                                        \
    } else {                                                                               \
      if (nt)                                                                              \
        hipLaunchKernelGGL((decode_kernel<U, true, true, true, false, K>), dim3(a.ntiles), \
                           dim3(kBlock), rl, s, a);                                        \
      else                                                                                 \
        hipLaunchKernelGGL((decode_kernel<U, false, true, true, false, K>), dim3(a.ntiles), \
                           dim3(kBlock), rl, s, a);                                        \
    }                                                                                      \
  } while (0)
  // 16-byte chunks per lane in flight in the whole-wave row copy: enough for the longest rows
  // copied that way, no more (every extra chunk costs registers, and waves per SIMD). Measured
  // on 32-row tiles: 4 KiB blobs + ~340-byte strings 4.30 TB/s at 6 vs 4.19 at 4; rows of a few
  // hundred bytes (all copied four per wave) 2.17 at 2 vs 1.99 at 4.
  int unroll = plan->unroll;
  uint64_t widest = 0, widest_fixed = 0;  // bytes per row of the widest column copied by waves
  for (int c = 0; c < plan->ncols; ++c) {
    const DevCol& d = a.cols[c];
    if (d.kind == MDSX_KIND_FIXED) {
      widest_fixed =
          std::max(widest_fixed, uint64_t(d.row_bytes > uint32_t(kSmallMax) ? d.row_bytes : 0));
    } else if (!d.gather && !d.group && a.rows) {
      widest = std::max(
          widest, (mode_bytes ? std::min(mode_bytes[c], d.capacity) : d.capacity) / a.rows);
    }
  }
  if (ragged && a.any_wave_ragged && plan->ring_slots > 0) {
    // long ragged rows go through the LDS-DMA ring; the unroll serves large fixed columns only
    const int u = unroll ? unroll : widest_fixed >= 2048 ? 4 : 2;
    if (plan->ring_slots == 4) {
      if (u == 2) MDSX_RING(2, 4); else MDSX_RING(4, 4);
    } else if (plan->ring_slots == 6) {
      if (u == 2) MDSX_RING(2, 6); else MDSX_RING(4, 6);
    } else {
      if (u == 2) MDSX_RING(2, 8); else MDSX_RING(4, 8);
    }
  } else {
    widest = std::max(widest, widest_fixed);
    if (unroll == 0) unroll = !ragged ? 4 : widest == 0 ? 2 : widest >= 2048 ? 6 : 4;
    if (unroll == 6) MDSX_DECODE_U(6);
    else if (unroll == 2) MDSX_DECODE_U(2);
    else MDSX_DECODE_U(4);
  }
#undef MDSX_RING
#undef MDSX_DECODE_U
#undef MDSX_DECODE
  rc = hip_check(hipGetLastError(), "decode_kernel launch");
  if (rc != MDSX_OK || plan->nvar == 0) return rc;
  const uint32_t gblocks = a.gather_block0[plan->nvar];
  if (gblocks == 0) return MDSX_OK;
  const int gk = plan->gather_chunks;
#define MDSX_GATHER(NT, K) \
  hipLaunchKernelGGL((gather_ragged_kernel<NT, K>), dim3(gblocks), dim3(kBlock), 0, s, a)
  if (gk == 1) {
    if (nt) MDSX_GATHER(true, 1); else MDSX_GATHER(false, 1);
  } else if (gk == 4) {
    if (nt) MDSX_GATHER(true, 4); else MDSX_GATHER(false, 4);
  } else {
    if (nt) MDSX_GATHER(true, 2); else MDSX_GATHER(false, 2);
  }
#undef MDSX_GATHER
  return hip_check(hipGetLastError(), "gather_ragged_kernel launch");
}


extern "C" {

int mdsx_decode_shards(const mdsx_plan* plan, const mdsx_batch* batch,
                       const mdsx_column_out* outs, void* d_workspace, uint64_t workspace_bytes,
                       void* stream) {
  DevArgs a;
  int rc = build_args(plan, batch, outs, d_workspace, workspace_bytes, nullptr, &a);
  if (rc != MDSX_OK || a.ntiles == 0) return rc;
  return launch_decode(plan, a, static_cast<hipStream_t>(stream), false, nullptr);
}

int mdsx_decode_shards_single(const mdsx_plan* plan, const mdsx_batch* batch,
                              const mdsx_column_out* outs, const uint64_t* mode_bytes,
                              void* d_workspace, uint64_t workspace_bytes, int64_t* d_totals,
                              void* stream) {
  DevArgs a;
  int rc = build_args(plan, batch, outs, d_workspace, workspace_bytes, d_totals, &a, mode_bytes);
  if (rc != MDSX_OK) return rc;
  hipStream_t s = static_cast<hipStream_t>(stream);
  // status record + ticket (the first 256 bytes) and the look-back words, zeroed together
  const uint64_t zero = 256 + round256(uint64_t(plan->nvar) * a.ntiles * 8);
  rc = hip_check(hipMemsetAsync(d_workspace, 0, zero, s), "hipMemsetAsync");
  if (rc != MDSX_OK) return rc;
  if (a.ntiles == 0) {  // no rows: ragged offsets are the single 0
    for (int c = 0; c < plan->ncols; ++c)
      if (plan->cols[c].var_index >= 0 && outs[c].offsets) {
        rc = hip_check(hipMemsetAsync(outs[c].offsets, 0, 8, s), "hipMemsetAsync");
        if (rc != MDSX_OK) return rc;
      }
    if (d_totals && plan->nvar)
      rc = hip_check(hipMemsetAsync(d_totals, 0, 8 * size_t(plan->nvar), s), "hipMemsetAsync");
    return rc;
  }
  return launch_decode(plan, a, s, plan->nvar > 0, mode_bytes);
}

uint64_t mdsx_gather_workspace_bytes(uint64_t m) {
  const uint64_t tiles = (m + kGatherRowTile - 1) / kGatherRowTile;
  return 256 + 2 * ((tiles * 8 + 255) & ~uint64_t(255));
}

static int gather_ws(void* ws, uint64_t ws_bytes, uint64_t m, mdsx_status** st, int64_t** tt,
                     int64_t** tp) {
  if (!ws || ws_bytes < mdsx_gather_workspace_bytes(m))
    return mdsx::fail(MDSX_E_ARG, "mdsx_gather: workspace smaller than mdsx_gather_workspace_bytes");
  const uint64_t tiles = (m + kGatherRowTile - 1) / kGatherRowTile;
  uint8_t* b = static_cast<uint8_t*>(ws);
  *st = reinterpret_cast<mdsx_status*>(b);
  *tt = reinterpret_cast<int64_t*>(b + 256);
  *tp = reinterpret_cast<int64_t*>(b + 256 + ((tiles * 8 + 255) & ~uint64_t(255)));
  return MDSX_OK;
}

extern "C++" {
template <class Src>
static int gather_fixed_launch(const Src S, uint64_t row_bytes, const int64_t* idx, uint64_t m,
                               void* dst, void* d_workspace, uint64_t workspace_bytes,
                               void* stream) {
  mdsx_status* st;
  int64_t *tt, *tp;
  int rc = gather_ws(d_workspace, workspace_bytes, m, &st, &tt, &tp);
  if (rc != MDSX_OK) return rc;
  if (!idx || !dst || row_bytes == 0 || row_bytes >= (uint64_t(1) << 32))
    return mdsx::fail(MDSX_E_ARG, "mdsx_gather_fixed: bad argument");
  if (m == 0) return MDSX_OK;
  const unsigned grid = unsigned((m + kGatherRowTile - 1) / kGatherRowTile);
  hipLaunchKernelGGL((gather_fixed_kernel<true, Src>), dim3(grid), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), S, uint32_t(row_bytes), idx, m,
                     static_cast<uint8_t*>(dst), st);
  return hip_check(hipGetLastError(), "gather_fixed_kernel launch");
}

template <class Src>
static int gather_scan_launch(const Src S, const int64_t* idx, uint64_t m, int64_t* dst_offsets,
                              void* d_workspace, uint64_t workspace_bytes, int64_t* d_total,
                              void* stream) {
  mdsx_status* st;
  int64_t *tt, *tp;
  int rc = gather_ws(d_workspace, workspace_bytes, m, &st, &tt, &tp);
  if (rc != MDSX_OK) return rc;
  if (!dst_offsets || (m && !idx))
    return mdsx::fail(MDSX_E_ARG, "mdsx_gather_ragged_scan: bad argument");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned tiles = unsigned((m + kGatherRowTile - 1) / kGatherRowTile);
  if (tiles) {
    hipLaunchKernelGGL((gather_len_kernel<Src>), dim3(tiles), dim3(kBlock), 0, s, S, idx, m,
                       dst_offsets, tt, st);
    rc = hip_check(hipGetLastError(), "gather_len_kernel launch");
    if (rc != MDSX_OK) return rc;
  }
  hipLaunchKernelGGL(scan_tile_totals_kernel, dim3(1), dim3(kBlock), 0, s, tt, tp, tiles,
                     dst_offsets, m, d_total);
  return hip_check(hipGetLastError(), "scan_tile_totals_kernel launch");
}

template <class Src>
static int gather_copy_launch(const Src S, const int64_t* idx, uint64_t m, uint8_t* dst_values,
                              uint64_t dst_capacity, int64_t* dst_offsets, uint8_t* dst_flags,
                              void* d_workspace, uint64_t workspace_bytes, void* stream) {
  mdsx_status* st;
  int64_t *tt, *tp;
  int rc = gather_ws(d_workspace, workspace_bytes, m, &st, &tt, &tp);
  if (rc != MDSX_OK) return rc;
  if (!dst_offsets || (m && !idx) || (dst_capacity && !dst_values))
    return mdsx::fail(MDSX_E_ARG, "mdsx_gather_ragged_copy: bad argument");
  if (m == 0) return MDSX_OK;
  const unsigned tiles = unsigned((m + kGatherRowTile - 1) / kGatherRowTile);
  // rows averaging under 1 KiB: four per wave (as the decode's medium rows)
  const bool group = dst_capacity < uint64_t(1024) * m;
  if (group)
    hipLaunchKernelGGL((gather_copy_kernel<true, true, Src>), dim3(tiles), dim3(kBlock), 0,
                       static_cast<hipStream_t>(stream), S, idx, m, dst_values, dst_capacity,
                       dst_offsets, dst_flags, tp, st);
  else
    hipLaunchKernelGGL((gather_copy_kernel<true, false, Src>), dim3(tiles), dim3(kBlock), 0,
                       static_cast<hipStream_t>(stream), S, idx, m, dst_values, dst_capacity,
                       dst_offsets, dst_flags, tp, st);
  return hip_check(hipGetLastError(), "gather_copy_kernel launch");
}

}  // extern "C++"

int mdsx_gather_fixed(const void* src, uint64_t src_rows, uint64_t row_bytes, const int64_t* idx,
                      uint64_t m, void* dst, void* d_workspace, uint64_t workspace_bytes,
                      void* stream) {
  if (!src) return mdsx::fail(MDSX_E_ARG, "mdsx_gather_fixed: bad argument");
  return gather_fixed_launch(OneSrc{static_cast<const uint8_t*>(src), nullptr, nullptr, src_rows},
                             row_bytes, idx, m, dst, d_workspace, workspace_bytes, stream);
}

int mdsx_gather_ragged_scan(const int64_t* src_offsets, uint64_t src_rows, const int64_t* idx,
                            uint64_t m, int64_t* dst_offsets, void* d_workspace,
                            uint64_t workspace_bytes, int64_t* d_total, void* stream) {
  if (!src_offsets) return mdsx::fail(MDSX_E_ARG, "mdsx_gather_ragged_scan: bad argument");
  return gather_scan_launch(OneSrc{nullptr, src_offsets, nullptr, src_rows}, idx, m, dst_offsets,
                            d_workspace, workspace_bytes, d_total, stream);
}

int mdsx_gather_ragged_copy(const uint8_t* src_values, const int64_t* src_offsets,
                            const uint8_t* src_flags, uint64_t src_rows, const int64_t* idx,
                            uint64_t m, uint8_t* dst_values, uint64_t dst_capacity,
                            int64_t* dst_offsets, uint8_t* dst_flags, void* d_workspace,
                            uint64_t workspace_bytes, void* stream) {
  if (!src_offsets || (dst_capacity && !src_values))
    return mdsx::fail(MDSX_E_ARG, "mdsx_gather_ragged_copy: bad argument");
  return gather_copy_launch(OneSrc{src_values, src_offsets, src_flags, src_rows}, idx, m,
                            dst_values, dst_capacity, dst_offsets, dst_flags, d_workspace,
                            workspace_bytes, stream);
}

int mdsx_gather_fixed_multi(const mdsx_gather_src* srcs, uint32_t nsrc, uint64_t row_bytes,
                            const int64_t* idx, uint64_t m, void* dst, void* d_workspace,
                            uint64_t workspace_bytes, void* stream) {
  if (!srcs || nsrc == 0) return mdsx::fail(MDSX_E_ARG, "mdsx_gather_fixed_multi: no sources");
  return gather_fixed_launch(MultiSrc{srcs, nsrc}, row_bytes, idx, m, dst, d_workspace,
                             workspace_bytes, stream);
}

int mdsx_gather_ragged_scan_multi(const mdsx_gather_src* srcs, uint32_t nsrc, const int64_t* idx,
                                  uint64_t m, int64_t* dst_offsets, void* d_workspace,
                                  uint64_t workspace_bytes, int64_t* d_total, void* stream) {
  if (!srcs || nsrc == 0)
    return mdsx::fail(MDSX_E_ARG, "mdsx_gather_ragged_scan_multi: no sources");
  return gather_scan_launch(MultiSrc{srcs, nsrc}, idx, m, dst_offsets, d_workspace,
                            workspace_bytes, d_total, stream);
}

int mdsx_gather_ragged_copy_multi(const mdsx_gather_src* srcs, uint32_t nsrc, const int64_t* idx,
                                  uint64_t m, uint8_t* dst_values, uint64_t dst_capacity,
                                  int64_t* dst_offsets, uint8_t* dst_flags, void* d_workspace,
                                  uint64_t workspace_bytes, void* stream) {
  if (!srcs || nsrc == 0)
    return mdsx::fail(MDSX_E_ARG, "mdsx_gather_ragged_copy_multi: no sources");
  return gather_copy_launch(MultiSrc{srcs, nsrc}, idx, m, dst_values, dst_capacity, dst_offsets,
                            dst_flags, d_workspace, workspace_bytes, stream);
}


int mdsx_ndarray_meta(const uint8_t* values, const int64_t* offsets, uint64_t rows, int dtype_id,
                      uint8_t* out_dtype, uint8_t* out_ndim, int64_t* out_data_offset,
                      int64_t* out_numel, uint8_t* out_bad, int32_t* d_max_ndim, void* stream) {
  if (!offsets || (rows && (!values || !out_dtype || !out_ndim || !out_data_offset ||
                            !out_numel || !out_bad)))
    return mdsx::fail(MDSX_E_ARG, "mdsx_ndarray_meta: bad argument");
  if (dtype_id != 0 && !(dtype_id == 8 || dtype_id == 9 || dtype_id == 16 || dtype_id == 17 ||
                         dtype_id == 18 || dtype_id == 32 || dtype_id == 33 || dtype_id == 34 ||
                         dtype_id == 64 || dtype_id == 65 || dtype_id == 66))
    return mdsx::fail(MDSX_E_ENCODING, "mdsx_ndarray_meta: unknown dtype id");
  if (rows == 0) return MDSX_OK;
  const unsigned grid = unsigned((rows + kBlock - 1) / kBlock);
  hipLaunchKernelGGL((ndarray_meta_kernel<false>), dim3(grid), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), values, offsets, rows, dtype_id, out_dtype,
                     out_ndim, out_data_offset, out_numel, out_bad, d_max_ndim, 0, nullptr);
  return hip_check(hipGetLastError(), "ndarray_meta_kernel launch");
}

int mdsx_ndarray_shapes(const uint8_t* values, const int64_t* offsets, uint64_t rows,
                        int dtype_id, int32_t shape_cols, int64_t* out_shape, void* stream) {
  if (!offsets || shape_cols < 0 || (rows && shape_cols && (!values || !out_shape)))
    return mdsx::fail(MDSX_E_ARG, "mdsx_ndarray_shapes: bad argument");
  if (rows == 0 || shape_cols == 0) return MDSX_OK;
  const unsigned grid = unsigned((rows + kBlock - 1) / kBlock);
  hipLaunchKernelGGL((ndarray_meta_kernel<true>), dim3(grid), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), values, offsets, rows, dtype_id, nullptr,
                     nullptr, nullptr, nullptr, nullptr, nullptr, shape_cols, out_shape);
  return hip_check(hipGetLastError(), "ndarray_meta_kernel launch");
}

int mdsx_copy_probe_variant(const void* d_src, void* d_dst, uint64_t bytes, int variant,
                            void* stream) {
  if (!d_src || !d_dst || (bytes & 15) || (reinterpret_cast<uint64_t>(d_src) & 15) ||
      (reinterpret_cast<uint64_t>(d_dst) & 15))
    return mdsx::fail(MDSX_E_ARG, "mdsx_copy_probe: 16-byte aligned pointers and size required");
  const uint64_t n = bytes / 16;
  if (n == 0) return MDSX_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint4* src = static_cast<const uint4*>(d_src);
  uint4* dst = static_cast<uint4*>(d_dst);
  const uint64_t per4 = uint64_t(kBlock / 64) * 64 * 4, per8 = per4 * 2;
  switch (variant) {
    case 0:
      hipLaunchKernelGGL(copy_probe_kernel, dim3(unsigned((n + kProbeBlock - 1) / kProbeBlock)),
                         dim3(kBlock), 0, s, src, dst, n);
      break;
    case 1:
      hipLaunchKernelGGL((copy_wave_kernel<4, true, true>), dim3(unsigned((n + per4 - 1) / per4)),
                         dim3(kBlock), 0, s, src, dst, n);
      break;
    case 2:
      hipLaunchKernelGGL((copy_wave_kernel<4, false, true>), dim3(unsigned((n + per4 - 1) / per4)),
                         dim3(kBlock), 0, s, src, dst, n);
      break;
    case 3:
      hipLaunchKernelGGL((copy_wave_kernel<8, true, true>), dim3(unsigned((n + per8 - 1) / per8)),
                         dim3(kBlock), 0, s, src, dst, n);
      break;
    case 4:
      hipLaunchKernelGGL((copy_wave_kernel<4, false, false>),
                         dim3(unsigned((n + per4 - 1) / per4)), dim3(kBlock), 0, s, src, dst, n);
      break;
    case 5:
      hipLaunchKernelGGL((copy_wave_kernel<4, true, true, true>),
                         dim3(unsigned((n + per4 - 1) / per4)), dim3(kBlock), 0, s, src, dst, n);
      break;
    case 6:
      hipLaunchKernelGGL((copy_wave_kernel<8, true, true, true>),
                         dim3(unsigned((n + per8 - 1) / per8)), dim3(kBlock), 0, s, src, dst, n);
      break;
    case 7:
    case 8: {
      // as 1, with unused dynamic LDS so that only 2 (7) or 3 (8) workgroups -- 8 or 12 waves --
      // share a CU: fewer concurrent streams, each with its bytes in flight
      const int pad = variant == 7 ? 72 * 1024 : 50 * 1024;
      const void* fn = reinterpret_cast<const void*>(copy_wave_kernel<4, true, true>);
      if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, pad) != hipSuccess)
        return mdsx::fail(MDSX_E_HIP, "mdsx_copy_probe_variant: LDS attribute");
      hipLaunchKernelGGL((copy_wave_kernel<4, true, true>), dim3(unsigned((n + per4 - 1) / per4)),
                         dim3(kBlock), size_t(pad), s, src, dst, n);
      break;
    }
    case 9:
    case 10: {
      // one wave per workgroup, XCD-contiguous (the row-per-wave decode's shape); 10: unused LDS
      // so that 12 workgroups share a CU (a pure copy's best occupancy on MI355X,
      // scripts/microbench/ring_copy4.hip)
      const int pad = variant == 10 ? 13 * 1024 : 0;
      const uint64_t per1 = 64 * 4;
      hipLaunchKernelGGL((copy_wave_kernel<4, true, true, true, 1>),
                         dim3(unsigned((n + per1 - 1) / per1)), dim3(64), size_t(pad), s, src, dst,
                         n);
      break;
    }
    default:
      return mdsx::fail(MDSX_E_ARG, "mdsx_copy_probe_variant: variant 0..10");
  }
  return hip_check(hipGetLastError(), "copy probe launch");
}

int mdsx_copy_probe(const void* d_src, void* d_dst, uint64_t bytes, void* stream) {
  return mdsx_copy_probe_variant(d_src, d_dst, bytes, 1, stream);
}

// The host hand-off copy: a FEW workgroups striding over the bytes (8 x 16 B per lane in flight,
// non-temporal), enough for PCIe (~57 GB/s x a few us of latency = well under 1 MiB in flight)
// while leaving the CUs to the next batch's decode and to a blit-kernel H2D copy on another
// stream. (A grid covering the whole buffer -- 2048 workgroups for a 512 MiB batch, all resident
// for the ~10 ms of the transfer -- kept a concurrent H2D copy from starting until it ended.)
constexpr unsigned kToHostGrid = 64;
__global__ __launch_bounds__(kBlock) void copy_to_host_kernel(const uint4* __restrict__ src,
                                                              uint4* __restrict__ dst, uint64_t n) {
  const uint64_t stride = uint64_t(gridDim.x) * kBlock * 8;
  for (uint64_t base = uint64_t(blockIdx.x) * kBlock * 8; base < n; base += stride) {
    uint4 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint64_t i = base + u * kBlock + threadIdx.x;
      if (i < n) v[u] = ld16<true>(src + i);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const uint64_t i = base + u * kBlock + threadIdx.x;
      if (i < n) st16<true>(reinterpret_cast<uint64_t>(dst + i), v[u]);
    }
  }
}

int mdsx_copy_to_host(const void* d_src, void* h_dst, uint64_t bytes, void* stream) {
  if (!d_src || !h_dst || (bytes & 15) || (reinterpret_cast<uint64_t>(d_src) & 15) ||
      (reinterpret_cast<uint64_t>(h_dst) & 15))
    return mdsx::fail(MDSX_E_ARG,
                      "mdsx_copy_to_host: 16-byte aligned pointers and size required");
  const uint64_t n = bytes / 16;
  if (n == 0) return MDSX_OK;
  const uint64_t need = (n + uint64_t(kBlock) * 8 - 1) / (uint64_t(kBlock) * 8);
  const unsigned grid = unsigned(std::min<uint64_t>(need, kToHostGrid));
  hipLaunchKernelGGL(copy_to_host_kernel, dim3(grid), dim3(kBlock), 0,
                     static_cast<hipStream_t>(stream), static_cast<const uint4*>(d_src),
                     static_cast<uint4*>(h_dst), n);
  return hip_check(hipGetLastError(), "copy_to_host_kernel launch");
}

}  // extern "C"
