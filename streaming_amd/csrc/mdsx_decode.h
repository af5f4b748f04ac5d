// Decode-side structures shared by the decode kernels of libmdsx.so (mdsx_kernels.hip: scan,
// register-copy decode, gather; mdsx_stage.hip: the LDS-staged decode of ragged plans): the
// kernel argument block, the per-tile view of a shard and the block-wide scan.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mdsx_device.h"
#include "mdsx_internal.h"

namespace mdsx_kernels {

constexpr int kBlock = 256;                     // 4 waves
constexpr int kSmallMax = 16;                   // fixed columns <= 16 B: one row per lane
constexpr uint64_t kMapGrain = uint64_t(kBlock) * 16;  // 4 KiB: row-map granule of ragged outputs
constexpr int kGatherRows = 1024;               // rows of a gather tile staged in LDS
constexpr int kGroupUnroll = 2;                 // chunks per lane in flight in group_copy

struct DevCol {
  void* data;
  int64_t* offsets;
  uint8_t* flags;
  uint64_t capacity;
  uint32_t row_bytes;
  int8_t kind;
  int8_t var_index;
  int8_t gather;  // ragged column copied by gather_ragged_kernel (short rows) instead of waves
  int8_t group;   // ragged column of medium rows: four rows per wave (group_copy)
};

// One run (tile) of the streaming decode as the scan pass describes it (stage_totals_kernel), so
// that a wave starts streaming its run after one load instead of a chain of table loads.
struct TileRun {
  uint64_t stream;  // batch byte of the run's first sample (offsets[r0])
  uint64_t offs;    // batch byte of offsets[r0] (the run's slice of the shard's offsets table)
  uint64_t row0;    // output row of the run's first sample
  uint32_t bytes;   // offsets[r0 + nrows] - offsets[r0] (when fast)
  uint32_t shard;   // batch shard index
  uint32_t r0;      // first sample of the run inside its shard
  uint16_t nrows;
  uint16_t fast;    // bit 0: the table fits and every sample of the run passes the file checks;
                    // bit 1: also every sample is at most seg_lim bytes (the lean path takes it)
  uint64_t shard_off;  // batch byte of the shard
};
static_assert(sizeof(TileRun) == 48, "TileRun layout");

constexpr uint32_t kXcdSeg = 1, kXcdRegister = 2, kXcdRows = 4;  // DevArgs::xcd_order bits

struct DevArgs {
  const uint8_t* batch;
  const mdsx_shard_desc* shards;
  const uint32_t* tile_shard;
  mdsx_status* status;
  int64_t* tile_total;   // [nvar][nscan] ragged bytes of each scan block (scan_per tiles)
  int64_t* tile_prefix;  // [nvar][nscan] their exclusive prefix
  int64_t* chunk_sum;    // [nvar][nchunk] scan of tile_total in chunks of kScanChunk entries
  TileRun* tile_run;     // [ntiles] (streaming decode)
  int64_t* totals;       // [nvar] or null
  uint64_t* src_abs;     // [nvar][rows]  byte index into the batch of each row's ragged value
  uint32_t* row_map;     // [nvar][map_len] first row of every gather tile
  uint64_t* lookback;    // [nvar][ntiles] single-pass look-back status words
  uint32_t* ticket;      // single-pass tile ticket counter
  uint64_t map_len;
  uint64_t rows;
  uint32_t ntiles;
  uint32_t nscan;     // scan blocks: ceil(ntiles / scan_per)
  uint32_t nchunk;    // chunks of the totals scan
  uint32_t scan_per;  // tiles per scan block (kBlock / tile_rows)
  int32_t nshards;
  int32_t ncols;
  int32_t nvar;
  int32_t tile_rows;
  int16_t any_group;     // some ragged column uses group_copy
  int16_t any_wave_str;  // some str column is copied by decode_kernel (validated there)
  int16_t any_wave_ragged;  // some ragged column is copied one row per wave
  int16_t str_cached;  // plan->str_cached
  uint32_t stage_debug;  // measurement only (MDSX_TUNE sdbg): parts of the row-parallel decode skipped
  uint32_t run_slots;    // KiB of the streaming decode's per-wave ring (0: not the streaming decode)
  uint32_t rows_bytes;   // LDS stage of the row-parallel decode (0: not the row-parallel decode)
  uint32_t seg_lim;      // streaming decode, lean path: largest sample it takes (0: lean path off)
  uint32_t seg_small;    // lean path: bytes per row of the fixed columns of <= 16 bytes
  uint32_t xcd_order;    // kXcd* bits: decodes whose workgroups take XCD-contiguous tile ranges
  uint32_t rows_pipe;    // row-parallel decode: tiles per workgroup through two stages (0: one)
  uint32_t rw_k;         // (measurement only, rowwave kX bit 2: offsets[0] taken as hdr_end + rw_k)
  uint32_t swave;        // ragged plans of long samples: one sample per wave (mdsx_swave.hip)
  uint4* sw_rec;         // [ntiles x tile_rows] its per-sample records (scan_tiles_kernel<true>)
  uint32_t sw_lds;       // ... bytes of its per-wave LDS copy of the columns past the first
  uint32_t gather_block0[MDSX_MAX_COLUMNS + 1];  // first gather workgroup of each ragged column
  DevCol cols[MDSX_MAX_COLUMNS];
};


// The one-sample-per-wave decode's record of a sample slot (tile x tile_rows + row of the tile),
// written by its scan pass (scan_tiles_kernel<true>) so that a decode wave starts with ONE load
// instead of the tile -> shard -> offsets chain: x | y << 32 = the sample's first byte in the batch
// (bits 0-39) and its shard (bits 40-63); z = its bytes, or kSwIdle (no sample in the slot) /
// kSwBad (its offsets failed the file checks: reported by the scan pass); w = its output row.
constexpr uint32_t kSwIdle = 0xffffffffu, kSwBad = 0xfffffffeu;

// Per-shard facts shared by the scan and decode kernels.
struct TileView {
  const uint8_t* shard;
  const uint32_t* offs;  // offsets table (absolute file offsets), 4-byte aligned
  mdsx_shard_desc d;
  uint32_t shard_idx;
  uint32_t r0;     // first row (inside the shard) of this tile
  uint32_t nrows;  // rows of this tile
  uint64_t hdr_end;
  bool table_ok;   // the offsets table of `samples` rows fits in the file
};

// Workgroups are dealt round robin over the 8 XCDs (MI355X_MICROARCH.md, dispatch). Remapped, XCD
// k takes the k-th contiguous eighth of the blocks (the last n % 8 keep their place), so the line
// two neighbouring tiles share meets in one L2 instead of two. A bijection on [0, n).
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t n) {
  const uint32_t per = n >> 3;
  return b < per * 8u ? (b & 7u) * per + (b >> 3) : b;
}

__device__ __forceinline__ TileView tile_view(const DevArgs& a, uint32_t tile) {
  TileView v;
  v.shard_idx = a.tile_shard[tile];
  v.d = a.shards[v.shard_idx];
  v.shard = a.batch + v.d.offset;
  v.offs = reinterpret_cast<const uint32_t*>(v.shard + 4);
  v.r0 = (tile - v.d.tile0) * uint32_t(a.tile_rows);
  v.nrows = v.d.samples > v.r0 ? min(uint32_t(a.tile_rows), v.d.samples - v.r0) : 0u;
  v.hdr_end = 4ull + 4ull * (uint64_t(v.d.samples) + 1ull);
  v.table_ok = v.hdr_end <= v.d.bytes;
  return v;
}

// Range of sample i of the shard (mds/reader.py:137-142) and its validity. A sample with zero
// bytes is the reference's IndexError (mds/reader.py:145-148).
__device__ __forceinline__ int sample_range(const TileView& v, uint32_t i, uint32_t* b,
                                            uint32_t* e) {
  *b = v.offs[i];
  *e = v.offs[i + 1];
  if (!(v.hdr_end <= *b && *b <= *e && *e <= v.d.bytes)) return MDSX_E_BOUNDS;
  if (*b == *e) return MDSX_E_EMPTY;
  return MDSX_OK;
}

// A workgroup barrier for kernels whose waves exchange data through LDS only: the wave's LDS
// operations done, then s_barrier. __syncthreads()'s release fence also waits for every
// vector-memory operation of the wave (vmcnt(0)): its global stores acknowledged and any LDS-DMA
// load landed -- store latency on every barrier (measured in the row-parallel decode's phases)
// and no DMA left in flight across it.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Exclusive scan over the 256 threads of the block; *total gets the block sum. kRaw: LDS-only
// barriers (lds_barrier).
template <bool kRaw = false>
__device__ __forceinline__ int64_t block_exclusive_scan(int64_t x, int64_t* s_wsum,
                                                        int64_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int64_t incl = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int64_t y = __shfl_up(incl, o);
    if (lane >= o) incl += y;
  }
  if (lane == 63) s_wsum[w] = incl;
  if constexpr (kRaw) lds_barrier();
  else __syncthreads();
  int64_t base = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kBlock / 64; ++k) {
    const int64_t s = s_wsum[k];
    base += (k < w) ? s : 0;
    tot += s;
  }
  if constexpr (kRaw) lds_barrier();
  else __syncthreads();
  *total = tot;
  return base + incl - x;
}


// Byte offset, inside the workspace's 256-byte status block, of the staged decode's count of
// huge rows (listed in the src_abs region; mdsx_stage.hip).
constexpr uint64_t kHugeCountOffset = 192;
// Bit (-code) set for every kind of error a decode kernel reported (the status record keeps only
// the first): the gather pass runs when every error is a per-sample one (empty sample, range),
// which leaves its row zero-length and every offset consistent.
constexpr uint64_t kErrKindsOffset = 64;
constexpr uint32_t kRowLevelErrors = (1u << -MDSX_E_BOUNDS) | (1u << -MDSX_E_EMPTY);

__device__ __forceinline__ void report_decode(const DevArgs& a, int code, int shard, int row,
                                              int col) {
  report(a.status, code, shard, row, col);
  atomicOr(reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(a.status) + kErrKindsOffset),
           1u << ((-code) & 31));
}

constexpr uint64_t kStatusBlock = 256;

// Single-pass decode (the register decode's kSingle form): tiles are
// taken in dispatch order from a ticket counter, so every tile a workgroup waits on is held by a
// workgroup that is already running. Each tile publishes its ragged bytes per ragged column and
// finds its output base by a decoupled look-back over the earlier tiles' status words. Flag and
// value share one 8-byte word written and read with agent-scope atomics, so no fence orders them.
constexpr uint64_t kLbAggregate = 1ull << 62, kLbInclusive = 2ull << 62;
constexpr uint64_t kLbValue = (1ull << 62) - 1;
typedef __attribute__((address_space(1))) uint64_t gu64;

// The look-back, run by one whole wave for every ragged column at once: agg[vi] is this tile's
// ragged bytes of column vi, base[vi] receives the bytes of every earlier tile. The wave splits
// into segments of W lanes, one per column (groups of 64 / W columns in turn); lane k of a
// segment reads the status of tile j - k. A segment sums its window up to the nearest inclusive
// prefix (tiles before 0 read as an inclusive zero), retrying while a tile inside that span has
// not published yet, and steps back W tiles when the window holds no inclusive prefix. The
// batch's last tile writes the column totals (offsets[rows], totals).
// `words` / `nunits`: the status words ([nvar][nunits]) and units (tiles, or scan chunks) of the
// look-back.
__device__ __forceinline__ void lookback_bases(const DevArgs& a, uint32_t tile, const int64_t* agg,
                                               int64_t* base_out, uint32_t shard, int lane,
                                               uint64_t* words, uint32_t nunits) {
  const int nv = a.nvar;
  const int W = nv <= 1 ? 64 : nv <= 2 ? 32 : nv <= 4 ? 16 : 8;
  const int kk = lane & (W - 1);
  const int seg0 = lane & ~(W - 1);
  const uint64_t wmask = W == 64 ? ~0ull : (1ull << W) - 1;
  for (int g0 = 0; g0 < nv; g0 += 64 / W) {
    const int vi = g0 + lane / W;
    const bool mine = vi < nv;
    gu64* st = (gu64*)(words + uint64_t(mine ? vi : 0) * nunits);
    const uint64_t ag = mine ? uint64_t(agg[vi]) : 0;
    if (mine && kk == 0)
      __hip_atomic_store(st + tile, (tile == 0 ? kLbInclusive : kLbAggregate) | ag,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t base = 0;
    int64_t j = int64_t(tile) - 1;
    bool done = !mine || tile == 0;
    uint32_t polls = 0;
    while (__ballot(!done) != 0) {
      const int64_t k = j - kk;
      const uint64_t w = (!done && k >= 0) ? __hip_atomic_load(st + k, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT)
                                           : kLbInclusive;
      const uint64_t incl = (__ballot((w >> 62) == 2) >> seg0) & wmask;
      const uint64_t none = (__ballot((w >> 62) == 0) >> seg0) & wmask;
      const uint64_t span = incl ? ((incl & (0 - incl)) << 1) - 1 : wmask;  // lanes <= first
      // an earlier tile's workgroup is still scanning its rows (it is running: it holds a
      // ticket); the bound only keeps a broken invariant from hanging the launch
      const bool wait = !done && (none & span) != 0 && ++polls < (1u << 22);
      uint64_t x = (!done && !wait && ((span >> kk) & 1)) ? (w & kLbValue) : 0;
      for (int o = W >> 1; o > 0; o >>= 1) x += __shfl_xor(x, o);
      if (!done && !wait) {
        if ((none & span) != 0 && kk == 0) report_decode(a, MDSX_E_HIP, int(shard), -1, -1);
        base += x;
        if (incl) done = true;
        else j -= W;
      }
      if (__ballot(wait) != 0) __builtin_amdgcn_s_sleep(1);
    }
    if (mine && kk == 0) {
      if (tile != 0)
        __hip_atomic_store(st + tile, kLbInclusive | (base + ag), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
      base_out[vi] = int64_t(base);
      if (tile + 1 == nunits) {  // the batch's last unit: column totals
        for (int c = 0; c < a.ncols; ++c)
          if (a.cols[c].var_index == vi) a.cols[c].offsets[a.rows] = int64_t(base + ag);
        if (a.totals) a.totals[vi] = int64_t(base + ag);
      }
    }
  }
}

// The tile number of a single-pass workgroup (thread 0 draws the ticket; block-uniform).
__device__ __forceinline__ uint32_t draw_ticket(const DevArgs& a, uint32_t* s_tile) {
  if (threadIdx.x == 0) *s_tile = atomicAdd(a.ticket, 1u);
  __syncthreads();
  return __builtin_amdgcn_readfirstlane(*s_tile);
}

// The LDS-staged decode of ragged plans (mdsx_stage.hip). Pass 1: the ragged bytes of every tile
// (then scan_totals_kernel, one entry per tile: a.scan_per == 1). Pass 2: every column of every
// row from each tile's shard bytes staged once in LDS. Return MDSX_OK or a launch error.
int launch_stage_totals(const DevArgs& a, bool nt, hipStream_t s);
int launch_run_decode(const mdsx_plan* plan, const DevArgs& a, hipStream_t s);
int launch_rows_decode(const mdsx_plan* plan, const DevArgs& a, hipStream_t s);
// The samples listed (tile << 32 | row in tile, a.src_abs; count at kHugeCountOffset) as larger
// than an LDS stage: one workgroup each, straight from HBM (mdsx_stage.hip).
int launch_huge_rows(const DevArgs& a, bool nt, hipStream_t s);
// One sample per one-wave workgroup, the sample in registers (mdsx_swave.hip), after the register
// decode's scan pass (scan-block-local offsets in the offsets outputs, block bases in tile_prefix).
int launch_swave_decode(const mdsx_plan* plan, const DevArgs& a, hipStream_t s);

}  // namespace mdsx_kernels
