// Streaming decode of ragged plans (gfx950): every wave decodes one tile -- a run of consecutive
// samples of one shard -- by streaming the run's bytes through a private LDS ring ONCE, in file
// order, and writing every column from there.
//
// The reference decodes one sample per call: MDSReader.get_sample_data reads the sample's byte
// range (streaming/base/format/mds/reader.py:128-149), decode_sample splits it at the u32 size
// heads of the variable columns (mds/reader.py:103-126) and each column's decoder returns its
// value (encodings.py:62-397, 760-773). In an MDS shard the samples of a run are contiguous --
// sample i ends where sample i + 1 starts (offsets[i + 1]) -- so a run is one byte range.
//
// Pass 1 (stage_totals_kernel + the reduce-then-scan kernels, mdsx_stage.hip / mdsx_kernels.hip):
// each tile's ragged bytes from the offsets table and the heads, scanned into each tile's output
// base per ragged column.
//
// Pass 2 (run_decode_kernel): a wave keeps up to S KiB of its run in flight into its LDS ring
// (global_load_lds_dwordx4: 1 KiB per wave-instruction, no VGPR destination) and walks the run's
// samples in order, all control wave-uniform:
//   * the sample's size heads are read from the ring (decode_sample's head loop) and its column
//     boundaries checked against its size (mds/reader.py:111-125);
//   * each column's bytes are written destination-major: lane k of a group owns 16-byte-aligned
//     output chunk k of the column, realigned from two aligned ring chunks (v_alignbyte). The
//     outputs of a column are contiguous over the run, so the chunk a sample leaves partly filled
//     is carried (in the column's lane of a lane-distributed register) into the next sample's
//     first chunk: every store is a whole 16-byte chunk except the two a run shares with its
//     neighbours;
//   * str values are checked for strict UTF-8 on the same registers (what bytes.decode('utf-8')
//     accepts, encodings.py:80-81), no second read;
//   * ragged offsets and UTF-8 flags are collected in LDS and written once per run, coalesced.
// So every byte of the shard range is read from HBM once (the heads, the column boundaries and
// the str bytes the check reads come from the ring) and the outputs are written once in whole
// chunks. The ring waits are explicit `s_waitcnt vmcnt(n)`, n = the vector-memory operations this
// wave issued after the slot's load (its loads, and stores certain to have issued), as in the
// ring of mdsx_kernels.hip.
//
// A run with a sample whose offsets fail the file checks streams each good sample on its own
// (every bad one reported): the file order of the run no longer holds there.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "mdsx_decode.h"
#include "mdsx_device.h"
#include "mdsx_internal.h"
#include "mdsx_ring.h"

namespace mdsx_kernels {
namespace {

constexpr int kRunBlock = 256;  // 4 waves, one tile each
constexpr int kRunWaves = kRunBlock / 64;
constexpr int kRunMaxRows = 32;  // rows of a tile: one offsets-table entry per lane (+1)

// A wave's LDS: its ring (S KiB, stream byte p at p % S KiB), a 64-byte mirror of the ring's
// first bytes behind it (so a read that wraps is one contiguous read), offsets and flags of its run.
__host__ __device__ __forceinline__ uint32_t run_wave_lds(int S, int TR, int nvar) {
  return (uint32_t(S) * 1024u + kMirror + uint32_t(nvar) * uint32_t(TR) * 5u + 15u) & ~15u;
}

// The per-column state of a wave, lane-distributed (lane c: column c). Output positions are
// 32-bit and relative to the column's `base` (the run's first output byte of the column,
// rounded down to 16): a run lies inside one shard, so its outputs span < 4 GiB.
struct Cursors {
  uint32_t cur;  // next output byte of the column
  uint32_t cst;  // first output byte of the column's current contiguous stretch (bytes below it
                 // belong to another run)
  uint4 carry;   // the partly filled chunk at cur & ~15 (bytes below cur valid from cst on)
};

// Column facts, lane-distributed, read with v_readlane in the sample loop.
struct ColRegs {
  uint64_t base;   // the run's first output byte of the column, rounded down to 16
  uint32_t first;  // that byte, relative to base (0..15)
  uint32_t rb;     // fixed columns: bytes per row
  uint32_t meta;   // bits 0-7: ragged index + 1 (0: fixed); bit 8: str with UTF-8 flags;
                   // bit 9: skip (the run's bytes exceed the output capacity)
};

// Write out the partly filled chunk of column c (the bytes [max(cst, chunk), cur)).
__device__ __forceinline__ void flush(const Cursors& k, uint64_t base, int c, int lane) {
  const uint32_t cur = __builtin_amdgcn_readlane(k.cur, c);
  const uint32_t cst = __builtin_amdgcn_readlane(k.cst, c);
  if ((cur & 15) == 0) return;
  const uint32_t C = cur & ~15u;
  const uint32_t lo = max(cst, C);
  if (lo >= cur) return;
  wave_edge_store(k.carry, c, base + C, base + lo, base + cur, lane);
}

// Bytes [0, n) of `v` zeroed (n uniform, 0 <= n <= 16).
__device__ __forceinline__ uint4 zero_below(const uint4 v, uint32_t n) {
  const uint4 m = byte_mask(0, n);
  return make_uint4(v.x & ~m.x, v.y & ~m.y, v.z & ~m.z, v.w & ~m.w);
}

// Column c of one sample: output bytes [d, d + len) (relative to `base`) from stream bytes
// [sp, sp + len). Returns (utf8: a str column) whether the value is not well-formed UTF-8
// (wave-uniform). Everything but the per-lane chunk is wave-uniform: each chunk is one unaligned
// ring read, the carried bytes and the value's last partial chunk are handled under uniform
// branches.
template <int S, bool kNT>
__device__ __forceinline__ bool copy_segment(Stream& st, const lds_u8* ring, uint32_t ring_lds,
                                             Cursors& k, uint64_t base, int c, uint32_t d,
                                             uint32_t len, uint32_t sp, bool utf8, int lane) {
  if (uint32_t(__builtin_amdgcn_readlane(k.cur, c)) != d) {  // a gap (a skipped sample's fixed
    flush(k, base, c, lane);                                  // bytes): a new stretch
    if (lane == c) k.cst = d;
  }
  const uint32_t cst = __builtin_amdgcn_readlane(k.cst, c);
  const uint32_t dbeg = d & ~15u, dend = d + len;
  const uint32_t head = d & 15u;               // carried bytes in the first chunk
  const uint32_t tail = dend & 15u;            // bytes of the last chunk, if partial
  const uint32_t nch = (dend + 15 - dbeg) >> 4;  // chunks touched
  const uint32_t nfull = (dend - dbeg) >> 4;     // chunks completed by this value
  // the stretch's first chunk, when another run owns its leading bytes: index inside this value
  const uint32_t cchunk = cst & ~15u;
  const uint32_t kc = (cst & 15) && cchunk >= dbeg ? (cchunk - dbeg) >> 4 : 0xffffffffu;
  // chunk kk of the value holds stream bytes from s0 + 16 kk (s0 wraps below 0 only on the first
  // value of the stream: those bytes are the carried ones, replaced below)
  const uint32_t s0 = sp - head;
  const uint64_t out = base + dbeg;
  bool bad = false;
  uint32_t prev_w = 0;
  uint4 last = make_uint4(0, 0, 0, 0);
  // chunks per lane per step: 1 (a step waits for 1 KiB of the ring, the rest stays in flight;
  // measured 1 % faster than 2 on config C, profiles/r02/u1/)
  constexpr uint32_t U = 1;
  for (uint32_t g = 0; g < nch; g += 64 * U) {
    ensure<S, kNT>(st, ring, ring_lds, g ? s0 + 16u * g : sp, s0 + 16u * g + 64u * 16u * U + 15u,
                   lane);
    uint4 val[U];
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) val[u] = ring16<S>(ring, s0 + 16u * (g + 64 * u + lane));
    if (g == 0 && head) {  // the bytes carried from the column's previous value
      const uint4 carry = readlane4(k.carry, c);
      if (lane == 0) val[0] = merge_bytes(val[0], carry, 0, head);
    }
#pragma unroll
    for (uint32_t u = 0; u < U; ++u) {
      const uint32_t g0 = g + 64 * u;
      if (g0 >= nch) break;  // uniform
      const uint32_t kk = g0 + uint32_t(lane);
      // whole chunks are stored whole, except the stretch's shared first chunk (its own bytes)
      const uint32_t f1 = min(nfull, g0 + 64);
      const bool kc_here = kc >= g0 && kc < f1;
      if (kk < nfull && kk != kc) st16<kNT>(out + 16ull * kk, val[u]);
      if (f1 > g0 + (kc_here ? 1u : 0u)) ++st.ops;  // a store certain to have issued
      if (kc_here)
        wave_edge_store(val[u], int(kc - g0), base + cchunk, base + cst, base + cchunk + 16, lane);
      const bool last_here = nch - 1 < g0 + 64;
      if (utf8) {
        // this value's bytes only: the carried ones and those past its end zeroed
        uint4 vout = kk < nch ? val[u] : make_uint4(0, 0, 0, 0);
        if (g0 == 0 && head && lane == 0) vout = zero_below(vout, head);
        if (last_here && tail && kk == nch - 1) vout = keep_range(vout, 0, 0, tail);
        const uint32_t any8 = (vout.x | vout.y | vout.z | vout.w) & 0x80808080u;
        if (__any(any8 != 0) || hi_c0(prev_w)) {  // a byte >= 0x80 (or a sequence open before)
          uint32_t pw = __shfl_up(vout.w, 1);
          if (lane == 0) pw = prev_w;
          if (kk < nch) bad |= utf8_chunk_bad(vout, pw, kk == nch - 1);
        }
        prev_w = __builtin_amdgcn_readlane(vout.w, 63);
      }
      if (last_here && tail) last = readlane4(val[u], int(nch - 1 - g0));
    }
  }
  if (lane == c) {
    k.cur = dend;
    k.carry = last;  // the chunk at dend & ~15 (meaningful when dend is not aligned)
  }
  return utf8 ? __any(bad) : false;
}

// The general path of a wave's run: any run the scan pass described (a sample failing the file
// checks, or larger than the ring). `wl`: the wave's LDS (ring, mirror, offsets, flags).
template <int S, bool kNT>
__device__ __forceinline__ void run_body(const DevArgs& a, const MDSX_L DevCol* cols,
                                         uint32_t tile, const TileRun& r, uint8_t* wl, int lane) {
  const int TR = a.tile_rows;
  const int ncols = a.ncols, nvar = a.nvar;
  const lds_u8* ring = (const lds_u8*)wl;
  MDSX_L uint32_t* obuf = (MDSX_L uint32_t*)(wl + S * 1024 + kMirror);  // [nvar][TR]
  MDSX_L uint8_t* fbuf = (MDSX_L uint8_t*)(wl + S * 1024 + kMirror + nvar * TR * 4);  // [nvar][TR]
  const uint32_t ring_lds = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const MDSX_L uint8_t*)wl)));

  // the run as the scan pass described it (its header check too): the run's first S KiB in
  // flight at once, its offsets-table slice and output bases loaded meanwhile
  const bool fast = (r.fast & 1) != 0;
  const uint64_t batch = reinterpret_cast<uint64_t>(a.batch);
  const uint64_t shard = batch + (r.offs - 4ull - 4ull * r.r0);  // the shard file's first byte
  Stream st;
  // streams start on a 128-byte line: every 1 KiB slot load is 8 whole lines (a slot straddling
  // lines makes the next slot fetch the shared line again, measured +7% reads)
  uint64_t sbase = (batch + r.stream) & ~uint64_t(127);
  st.base = reinterpret_cast<const uint4*>(sbase);
  st.nq = 0;
  st.nslots = 0;
  st.issued = 0;
  st.ops = 0;
  st.op_at = 0;
  st.mirrored = 0xffffffffu;
  st.landed = 0;
  if (fast) {
    st.nq = uint32_t((batch + r.stream + r.bytes - sbase + 15) >> 4);
    st.nslots = (st.nq + 63) >> 6;
    pump<S, kNT>(st, ring_lds, 0, lane);
  }
  // a run with a sample failing the file checks (or a table past its file): each sample checked
  // against its shard, and streamed on its own
  uint64_t hdr_end = 0, fbytes = 0;
  if (!fast) {
    const TileView v = tile_view(a, tile);
    if (!v.table_ok) return;
    hdr_end = v.hdr_end;
    fbytes = v.d.bytes;
  }
  const int n = int(r.nrows);
  if (n == 0) return;
  const uint64_t row0 = r.row0;
  // this run's offsets-table slice: lane j holds offsets[r0 + j] (j <= n)
  const uint32_t ob = lane <= n ? *reinterpret_cast<const uint32_t*>(a.batch + r.offs + 4u * lane)
                                : 0u;

  // column facts and cursors at the run's first output byte, lane-distributed
  ColRegs cr = {0, 0, 0, 0};
  Cursors k;
  k.carry = make_uint4(0, 0, 0, 0);
  k.cur = 0;
  if (lane < ncols) {
    const MDSX_L DevCol& col = cols[lane];
    const uint64_t data = reinterpret_cast<uint64_t>(col.data);
    const int vi = col.var_index;
    uint64_t first = data + row0 * col.row_bytes;
    uint32_t meta = uint32_t(vi + 1) & 255u;
    if (vi >= 0) {
      const uint64_t off = uint64_t(a.tile_prefix[uint64_t(vi) * a.nscan + tile]);
      first = data + off;
      if (off + uint64_t(a.tile_total[uint64_t(vi) * a.nscan + tile]) > col.capacity) {
        report_decode(a, MDSX_E_CAPACITY, int(r.shard), int(r.r0), lane);
        meta |= 1u << 9;  // this run writes nothing of the column
      }
      if (col.kind == MDSX_KIND_STR && col.flags != nullptr) meta |= 1u << 8;
    }
    cr.base = first & ~uint64_t(15);
    cr.first = uint32_t(first & 15);
    cr.rb = col.row_bytes;
    cr.meta = meta;
    k.cur = cr.first;
  }
  k.cst = k.cur;


  for (int j = 0; j < n; ++j) {  // wave-uniform
    const uint32_t b = uint32_t(__builtin_amdgcn_readlane(int(ob), j));
    const uint32_t e = uint32_t(__builtin_amdgcn_readlane(int(ob), j + 1));
    const uint64_t srow = shard + b;  // the sample's first byte
    const uint32_t size = e - b;
    int rc = MDSX_OK;
    if (!fast) {  // the sample on its own: its own stream, once the previous one has landed
      if (!(hdr_end <= b && b <= e && e <= fbytes)) rc = MDSX_E_BOUNDS;
      else if (b == e) rc = MDSX_E_EMPTY;
      if (rc == MDSX_OK) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        sbase = srow & ~uint64_t(127);
        st.base = reinterpret_cast<const uint4*>(sbase);
        st.nq = uint32_t((srow + size - sbase + 15) >> 4);
        st.nslots = (st.nq + 63) >> 6;
        st.issued = 0;
        st.mirrored = 0xffffffffu;
        st.landed = 0;
        pump<S, kNT>(st, ring_lds, 0, lane);
      }
    }
    const uint32_t sp = uint32_t(srow - sbase);  // stream position of the sample
    // a sample that fits the ring with a slot to spare: all its bytes waited for at once (the
    // per-column waits then cost a compare each)
    if (rc == MDSX_OK && size + 16u <= uint32_t(S - 2) * 1024u)
      ensure<S, kNT>(st, ring, ring_lds, sp, sp + size + 15u, lane);
    // size heads: lane vi holds head vi
    uint32_t h = 0;
    if (rc == MDSX_OK && 4u * uint32_t(nvar) <= size && nvar > 0) {
      ensure<S, kNT>(st, ring, ring_lds, sp, sp + 4u * uint32_t(nvar) + 3u, lane);
      if (lane < nvar) h = ring_u32<S>(ring, sp + 4u * uint32_t(lane));
    }
    if (rc == MDSX_OK) {
      if (4u * uint32_t(nvar) > size) {
        rc = MDSX_E_BOUNDS;
      } else {
        uint64_t need = 4ull * uint32_t(nvar);
        for (int c = 0; c < ncols; ++c) {
          const int vi = int(__builtin_amdgcn_readlane(cr.meta, c) & 255u) - 1;
          need += vi >= 0 ? uint32_t(__builtin_amdgcn_readlane(int(h), vi))
                          : uint32_t(__builtin_amdgcn_readlane(cr.rb, c));
        }
        if (need > size) rc = MDSX_E_BOUNDS;
      }
    }
    if (rc != MDSX_OK && lane == 0) report_decode(a, rc, int(r.shard), int(r.r0 + j), -1);
    uint32_t rel = 4u * uint32_t(nvar);
    for (int c = 0; c < ncols; ++c) {
      const uint32_t meta = __builtin_amdgcn_readlane(cr.meta, c);
      const int vi = int(meta & 255u) - 1;
      const uint32_t rb = __builtin_amdgcn_readlane(cr.rb, c);
      const uint32_t len = rc != MDSX_OK ? 0u
                           : vi >= 0     ? uint32_t(__builtin_amdgcn_readlane(int(h), vi))
                                         : rb;
      const bool utf8 = (meta >> 8) & 1u;
      const uint32_t d = vi < 0 ? __builtin_amdgcn_readlane(cr.first, c) + uint32_t(j) * rb
                                : __builtin_amdgcn_readlane(k.cur, c);
      if (vi >= 0 && lane == 0) obuf[vi * TR + j] = d;
      bool bad = false;
      if (len && !((meta >> 9) & 1u))
        bad = copy_segment<S, kNT>(st, ring, ring_lds, k, readlane64(cr.base, c), c, d, len,
                                   sp + rel, utf8, lane);
      if (utf8 && lane == 0) fbuf[vi * TR + j] = bad ? 1 : 0;
      rel += len;
    }
  }
  // the partly filled last chunk of every column; the run's offsets and flags
  for (int c = 0; c < ncols; ++c) flush(k, readlane64(cr.base, c), c, lane);
  for (int c = 0; c < ncols; ++c) {
    const MDSX_L DevCol& col = cols[c];
    const int vi = col.var_index;
    if (vi < 0) continue;
    // offsets[row] = (base - data) + the row's position relative to base
    const int64_t obase = int64_t(readlane64(cr.base, c) - reinterpret_cast<uint64_t>(col.data));
    if (lane < n) *gp(col.offsets + row0 + lane) = obase + int64_t(obuf[vi * TR + lane]);
    if (col.kind == MDSX_KIND_STR && col.flags && lane < n)
      *gp(col.flags + row0 + lane) = fbuf[vi * TR + lane];
  }
}

template <int S, bool kNT>
__global__ __launch_bounds__(kRunBlock, 7) void run_decode_kernel(const DevArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  __shared__ DevCol s_cols[MDSX_MAX_COLUMNS];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  // the column table in LDS: kernel-argument fields indexed by a loop variable compile to vector
  // loads, whose waits would also wait for the ring's loads and the stores in flight
  for (int c = t; c < a.ncols; c += kRunBlock) s_cols[c] = a.cols[c];
  __syncthreads();
  const MDSX_L DevCol* cols = (const MDSX_L DevCol*)s_cols;
  const uint32_t tile = blockIdx.x * kRunWaves + uint32_t(wave);
  if (tile >= a.ntiles) return;  // wave-uniform; no barrier below
  uint8_t* wl = smem + size_t(wave) * run_wave_lds(S, a.tile_rows, a.nvar);
  run_body<S, kNT>(a, cols, tile, a.tile_run[tile], wl, lane);
}

// ---------------------------------------------------------------------------------------------
// The lean path (seg_decode_kernel) for the common run: every sample passes the file checks and
// fits the ring with a slot to spare (TileRun.fast bit 1, set by the scan pass). Per sample the
// wave waits ONCE, for all of the sample's bytes, and then has nothing left to wait for:
//   * the column geometry is lane-parallel -- lane c reads column c's size head from the ring,
//     a wave prefix sum places every column in the sample, one ballot checks the boundaries
//     (MDSReader.decode_sample, mds/reader.py:111-125);
//   * fixed columns of <= 16 bytes (the `int` / scalar columns) go to an LDS stage, one lane per
//     column, and leave the wave once per run, one row per lane;
//   * every wider column is copied destination-major (lane k: 16-byte output chunk k, one
//     unaligned ds_read_b128 from the ring, one whole-chunk store), the partly filled last chunk
//     carried into the next sample's first chunk; str values checked for strict UTF-8 on the same
//     registers (bytes.decode('utf-8'), encodings.py:80-81).
// Other runs take the general path (run_body). A sample failing the boundary check is reported
// (MDSX_E_BOUNDS) and decodes as empty ragged values and zeroed fixed values, the scan pass's
// zero-length rule.

// per-wave LDS of the lean path: the general path's, then the staged small fixed columns
__host__ __device__ __forceinline__ uint32_t seg_wave_lds(int S, int TR, int nvar,
                                                          uint32_t small) {
  return run_wave_lds(S, TR, nvar) + ((small * uint32_t(TR) + 15u) & ~15u);
}

// One value of a wide column, all of its stream bytes landed: output bytes [d, d + len) (relative
// to `base`) from stream bytes [p, p + len) (zeros when `zero`). `cst`: the run's first output
// byte of the column (bytes below it belong to the run before). `carry` (uniform): in, the partly
// filled chunk at d & ~15; out, the one at (d + len) & ~15. Returns (utf8) whether the value is
// not well-formed UTF-8 (wave-uniform).
template <int S, bool kNT>
__device__ __forceinline__ bool seg_copy(const lds_u8* ring, uint64_t base, uint32_t cst,
                                         uint32_t d, uint32_t len, uint32_t p, bool utf8,
                                         bool zero, uint4& carry, uint32_t& ops, int lane) {
  const uint32_t head = d & 15u, dbeg = d - head, dend = d + len;
  const uint32_t nch = (dend - dbeg + 15u) >> 4;  // chunks touched
  const uint32_t nfull = (dend - dbeg) >> 4;      // chunks completed by this value
  const uint32_t tail = dend & 15u;
  const bool shared0 = dbeg < cst;  // the run's first chunk of the column, shared with the run before
  const uint32_t s0 = p - head;     // stream byte of chunk 0's byte 0 (bytes below p: the carry's)
  const uint64_t out = base + dbeg;
  const uint4 z4 = make_uint4(0, 0, 0, 0);
  bool bad = false;
  uint32_t prev_w = 0;
  uint4 last = carry;
  for (uint32_t g = 0; g < nch; g += 64) {  // wave-uniform
    const uint32_t kk = g + uint32_t(lane);
    uint4 val = zero ? z4 : ring16<S>(ring, s0 + 16u * kk);
    if (g == 0 && head && lane == 0) val = splice_lo(carry, val, head);
    const bool skip0 = shared0 && g == 0;
    if (kk < nfull && !(skip0 && lane == 0)) st16<kNT>(out + 16ull * kk, val);
    if (min(nfull, g + 64u) > g + (skip0 ? 1u : 0u)) ++ops;  // that store was issued
    if (skip0 && nfull > 0) wave_edge_store(val, 0, out, base + cst, out + 16, lane);
    if (utf8) {
      // this value's bytes only: the carried ones and those past its end zeroed
      uint4 vout = kk < nch ? val : z4;
      if (g == 0 && head && lane == 0) vout = splice_lo(z4, vout, head);
      if (tail && kk == nch - 1) vout = splice_lo(vout, z4, tail);
      const uint32_t any8 = (vout.x | vout.y | vout.z | vout.w) & 0x80808080u;
      if (__any(any8 != 0) || hi_c0(prev_w)) {  // a byte >= 0x80 (or a sequence open before)
        uint32_t pw = uint32_t(__shfl_up(int(vout.w), 1));
        if (lane == 0) pw = prev_w;
        if (kk < nch) bad |= utf8_chunk_bad(vout, pw, kk == nch - 1);
      }
      prev_w = __builtin_amdgcn_readlane(vout.w, 63);
    }
    if (tail && nch - 1 - g < 64u) last = readlane4(val, int(nch - 1 - g));
  }
  carry = last;
  return utf8 ? __any(bad) != 0 : false;
}

// The column table of a lean-path workgroup, ahead of the waves' LDS (dynamic, ncols entries).
__host__ __device__ __forceinline__ uint32_t seg_cols_lds(int ncols) {
  return (uint32_t(ncols) * uint32_t(sizeof(DevCol)) + 15u) & ~15u;
}

// W waves per workgroup (one run each): fewer waves per workgroup waste less LDS per CU.
template <int S, bool kNT, int W>
__global__ __launch_bounds__(64 * W, 4) void seg_decode_kernel(const DevArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = W == 1 ? 0 : __builtin_amdgcn_readfirstlane(t >> 6);
  MDSX_L DevCol* s_cols = (MDSX_L DevCol*)smem;
  for (int c = t; c < a.ncols; c += 64 * W) s_cols[c] = a.cols[c];
  __syncthreads();
  const MDSX_L DevCol* cols = (const MDSX_L DevCol*)s_cols;
  const uint32_t tile = blockIdx.x * W + uint32_t(wave);
  if (tile >= a.ntiles) return;  // wave-uniform; no barrier below
  const int TR = a.tile_rows;
  const int ncols = a.ncols, nvar = a.nvar;
  uint8_t* wl = smem + seg_cols_lds(ncols) + size_t(wave) * seg_wave_lds(S, TR, nvar, a.seg_small);
  const TileRun r = a.tile_run[tile];
  if (!(r.fast & 2)) {
    run_body<S, kNT>(a, cols, tile, r, wl, lane);
    return;
  }
  const lds_u8* ring = (const lds_u8*)wl;
  MDSX_L uint32_t* obuf = (MDSX_L uint32_t*)(wl + S * 1024 + kMirror);  // [nvar][TR]
  MDSX_L uint8_t* fbuf = (MDSX_L uint8_t*)(wl + S * 1024 + kMirror + nvar * TR * 4);  // [nvar][TR]
  MDSX_L uint8_t* sbuf = (MDSX_L uint8_t*)(wl + run_wave_lds(S, TR, nvar));  // small columns
  const uint32_t ring_lds = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const MDSX_L uint8_t*)wl)));

  // the run's bytes: one range starting on a 128-byte line, its first S KiB in flight at once
  const uint64_t batch = reinterpret_cast<uint64_t>(a.batch);
  const uint64_t shard = batch + (r.offs - 4ull - 4ull * r.r0);  // the shard file's first byte
  const uint64_t sbase = (batch + r.stream) & ~uint64_t(127);
  Stream st;
  st.base = reinterpret_cast<const uint4*>(sbase);
  st.nq = uint32_t((batch + r.stream + r.bytes - sbase + 15) >> 4);
  st.nslots = (st.nq + 63) >> 6;
  st.issued = 0;
  st.ops = 0;
  st.op_at = 0;
  st.mirrored = 0xffffffffu;
  st.landed = 0;
  pump<S, kNT>(st, ring_lds, 0, lane);
  const int n = int(r.nrows);
  const uint64_t row0 = r.row0;
  // lane j holds offsets[r0 + j] (j <= n)
  const uint32_t ob = lane <= n ? *reinterpret_cast<const uint32_t*>(a.batch + r.offs + 4u * lane)
                                : 0u;

  // column facts and cursors, lane-distributed (lane c: column c)
  int vi = -1;
  uint32_t rb = 0, meta = 0, cur = 0;
  uint64_t base = 0;
  bool small = false, wide = false;
  if (lane < ncols) {
    const MDSX_L DevCol& col = cols[lane];
    vi = col.var_index;
    rb = col.row_bytes;
    const uint64_t data = reinterpret_cast<uint64_t>(col.data);
    uint64_t first = data + row0 * rb;
    bool skip = false;
    if (vi >= 0) {
      const uint64_t off = uint64_t(a.tile_prefix[uint64_t(vi) * a.nscan + tile]);
      first = data + off;
      if (off + uint64_t(a.tile_total[uint64_t(vi) * a.nscan + tile]) > col.capacity) {
        report_decode(a, MDSX_E_CAPACITY, int(r.shard), int(r.r0), lane);
        skip = true;  // this run writes nothing of the column
      }
      meta = uint32_t(vi + 1) & 255u;
      if (col.kind == MDSX_KIND_STR && col.flags != nullptr) meta |= 1u << 8;
    }
    small = vi < 0 && rb <= uint32_t(kSmallMax);
    wide = !small && !skip;
    base = first & ~uint64_t(15);
    cur = uint32_t(first & 15);
  }
  const uint32_t cst = cur;
  uint4 carry = make_uint4(0, 0, 0, 0);
  const uint32_t ssz = small ? rb * uint32_t(TR) : 0u;
  const uint32_t soff = ((wave_incl_u32(ssz, lane, ncols) - ssz));  // stage offset of the column
  const uint64_t wide_mask = __ballot(wide);
  const uint64_t small_mask = __ballot(small);
  const uint32_t hv = 4u * uint32_t(nvar);

  for (int j = 0; j < n;) {  // wave-uniform
    const uint32_t b = uint32_t(__builtin_amdgcn_readlane(int(ob), j));
    const uint32_t e = uint32_t(__builtin_amdgcn_readlane(int(ob), j + 1));
    const uint32_t size = e - b;
    const uint32_t sp = uint32_t(shard + b - sbase);  // stream position of the sample
    ensure<S, kNT>(st, ring, ring_lds, sp, sp + size + 15u, lane);  // ALL of the sample's bytes
    // column geometry, lane c: size head (ragged) or row size (fixed), place by prefix sum
    uint32_t len = 0;
    if (lane < ncols) len = vi >= 0 ? ring_u32<S>(ring, sp + 4u * uint32_t(vi)) : rb;
    const bool over = lane < ncols && len > size;
    const uint32_t lc = over ? 0u : len;
    const uint32_t incl = wave_incl_u32(lc, lane, ncols);
    const uint32_t total = uint32_t(__builtin_amdgcn_readlane(int(incl), ncols - 1));
    const bool ok = !__any(over) && hv <= size && total <= size - hv;
    if (!ok && lane == 0) report_decode(a, MDSX_E_BOUNDS, int(r.shard), int(r.r0 + j), -1);
    const uint32_t pos = sp + hv + incl - lc;  // stream position of the column's value
    const uint32_t clen = ok ? len : (vi >= 0 ? 0u : rb);
    if (small)
      lds_put(sbuf + soff + uint32_t(j) * rb, ok ? ring16<S>(ring, pos) : make_uint4(0, 0, 0, 0),
              rb);
    if (vi >= 0) {
      obuf[vi * TR + j] = cur;
      if ((meta >> 8) & 1u) fbuf[vi * TR + j] = 0;
    }
    // the wide columns, in column order = stream order
    uint64_t wm = wide_mask;
    while (wm) {
      const int c = __builtin_ctzll(wm);
      wm &= wm - 1;
      const uint32_t l = uint32_t(__builtin_amdgcn_readlane(int(clen), c));
      if (l == 0) continue;
      const uint32_t d = uint32_t(__builtin_amdgcn_readlane(int(cur), c));
      const uint32_t p = uint32_t(__builtin_amdgcn_readlane(int(pos), c));
      const uint32_t mc = uint32_t(__builtin_amdgcn_readlane(int(meta), c));
      const uint32_t cs = uint32_t(__builtin_amdgcn_readlane(int(cst), c));
      uint4 cy = (d & 15u) ? readlane4(carry, c) : make_uint4(0, 0, 0, 0);
      const bool utf8 = (mc >> 8) & 1u;
      const bool bad = seg_copy<S, kNT>(ring, readlane64(base, c), cs, d, l, p, utf8, !ok, cy,
                                        st.ops, lane);
      if (lane == c) {
        cur = d + l;
        carry = cy;
      }
      if (bad && lane == 0) fbuf[(int(mc & 255u) - 1) * TR + j] = 1;
      pump<S, kNT>(st, ring_lds, (p + l) >> 10, lane);  // the bytes before p + l are done
    }
    ++j;
  }
  // the partly filled last chunk of every wide column (bytes [max(cst, chunk), cur))
  for (uint64_t m = wide_mask; m; m &= m - 1) {
    const int c = __builtin_ctzll(m);
    const uint32_t cu = uint32_t(__builtin_amdgcn_readlane(int(cur), c));
    const uint32_t cs = uint32_t(__builtin_amdgcn_readlane(int(cst), c));
    if ((cu & 15u) == 0) continue;
    const uint32_t C = cu & ~15u;
    const uint32_t lo = max(cs, C);
    if (lo >= cu) continue;
    const uint64_t bs = readlane64(base, c);
    wave_edge_store(carry, c, bs + C, bs + lo, bs + cu, lane);
  }
  // the staged small fixed columns, one row per lane
  for (uint64_t m = small_mask; m; m &= m - 1) {
    const int c = __builtin_ctzll(m);
    const uint32_t w = cols[c].row_bytes;
    const uint32_t so = uint32_t(__builtin_amdgcn_readlane(int(soff), c));
    if (lane < n)
      lds_out(sbuf + so + uint32_t(lane) * w,
              static_cast<uint8_t*>(cols[c].data) + (row0 + uint64_t(lane)) * w, w);
  }
  // the run's ragged offsets and str flags
  for (int c = 0; c < ncols; ++c) {
    const MDSX_L DevCol& col = cols[c];
    const int v = col.var_index;
    if (v < 0) continue;
    // offsets[row] = (base - data) + the row's position relative to base
    const int64_t obase = int64_t(readlane64(base, c) - reinterpret_cast<uint64_t>(col.data));
    if (lane < n) *gp(col.offsets + row0 + lane) = obase + int64_t(obuf[v * TR + lane]);
    if (col.kind == MDSX_KIND_STR && col.flags && lane < n)
      *gp(col.flags + row0 + lane) = fbuf[v * TR + lane];
  }
}

}  // namespace

int launch_run_decode(const mdsx_plan* plan, const DevArgs& a, hipStream_t s) {
  const unsigned grid = (a.ntiles + kRunWaves - 1) / kRunWaves;
  const size_t lds = size_t(kRunWaves) * run_wave_lds(a.run_slots, a.tile_rows, a.nvar);
  if (a.tile_rows > kRunMaxRows)
    return mdsx::fail(MDSX_E_ARG, "mdsx: streaming decode tiles hold at most 32 rows");
  if (a.seg_lim) {
    const int W = plan->seg_waves;
    const size_t slds = seg_cols_lds(a.ncols) +
                        size_t(W) * seg_wave_lds(a.run_slots, a.tile_rows, a.nvar, a.seg_small);
    if (slds > 160 * 1024)
      return mdsx::fail(MDSX_E_ARG, "mdsx: streaming decode LDS exceeds 160 KiB");
    const unsigned sgrid = (a.ntiles + unsigned(W) - 1) / unsigned(W);
#define MDSX_SEG_CASE(S, NT, WV)                                                               \
  if (a.run_slots == S && bool(plan->run_nt) == NT && W == WV) {                               \
    if (slds > 64 * 1024) {                                                                    \
      const int rc = hip_check(                                                                \
          hipFuncSetAttribute(reinterpret_cast<const void*>(seg_decode_kernel<S, NT, WV>),     \
                              hipFuncAttributeMaxDynamicSharedMemorySize, int(slds)),          \
          "hipFuncSetAttribute");                                                              \
      if (rc != MDSX_OK) return rc;                                                            \
    }                                                                                          \
    mdsx::set_last_kernel("seg_decode_kernel<" #S ", " #NT ", " #WV ">");                     \
    hipLaunchKernelGGL((seg_decode_kernel<S, NT, WV>), dim3(sgrid), dim3(64 * WV), slds, s, a); \
    return hip_check(hipGetLastError(), "seg_decode_kernel launch");                           \
  }
#define MDSX_SEG_W(WV)         \
  MDSX_SEG_CASE(4, true, WV)   \
  MDSX_SEG_CASE(4, false, WV)  \
  MDSX_SEG_CASE(8, true, WV)   \
  MDSX_SEG_CASE(8, false, WV)  \
  MDSX_SEG_CASE(16, true, WV)  \
  MDSX_SEG_CASE(16, false, WV)
    MDSX_SEG_W(1)
    MDSX_SEG_W(2)
    MDSX_SEG_W(4)
#undef MDSX_SEG_W
#undef MDSX_SEG_CASE
    return mdsx::fail(MDSX_E_ARG, "mdsx: streaming decode ring of 4, 8 or 16 KiB");
  }
#define MDSX_RUN_CASE(S, NT)                                                              \
  if (a.run_slots == S && bool(plan->run_nt) == NT) {                                     \
    if (lds > 64 * 1024) {                                                                \
      const int rc = hip_check(                                                           \
          hipFuncSetAttribute(reinterpret_cast<const void*>(run_decode_kernel<S, NT>),    \
                              hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)),      \
          "hipFuncSetAttribute");                                                         \
      if (rc != MDSX_OK) return rc;                                                       \
    }                                                                                     \
    mdsx::set_last_kernel("run_decode_kernel<" #S ", " #NT ">");                         \
    hipLaunchKernelGGL((run_decode_kernel<S, NT>), dim3(grid), dim3(kRunBlock), lds, s, a); \
    return hip_check(hipGetLastError(), "run_decode_kernel launch");                      \
  }
  MDSX_RUN_CASE(4, true)
  MDSX_RUN_CASE(4, false)
  MDSX_RUN_CASE(8, true)
  MDSX_RUN_CASE(8, false)
  MDSX_RUN_CASE(16, true)
  MDSX_RUN_CASE(16, false)
#undef MDSX_RUN_CASE
  return mdsx::fail(MDSX_E_ARG, "mdsx: streaming decode ring of 4, 8 or 16 KiB");
}

}  // namespace mdsx_kernels
