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
// base per ragged column; each run's record says whether the lean path can take it.
//
// Pass 2, by default seg_decode_kernel (the lean path, below): one wait per sample, lane-parallel
// column geometry, for every run whose samples pass the file checks and fit the ring; the runs it
// does not take go to the general path, run_body (mdsx_run_body.h), which is also a kernel of its
// own (run_decode_kernel, MDSX_TUNE=seg=0) and is described here.
//
// The general path: a wave keeps up to S KiB of its run in flight into its LDS ring
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
#include <cstddef>
#include <cstdint>

#include "mdsx_decode.h"
#include "mdsx_device.h"
#include "mdsx_internal.h"
#include "mdsx_ring.h"
#include "mdsx_run_body.h"

namespace mdsx_kernels {
namespace {

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
// Measurement variants (kV bits, MDSX_TUNE sv): 2 releases the ring slots a value's 1 KiB step
// has consumed after each step (not after the whole value), so the next sample's slots go in
// flight while the value is still being written; 4 waits per 1 KiB step (not once per sample);
// 8 (ablation, outputs incomplete) stores no partial edge chunk; 32 touches the run's lines
// beyond the ring's first fill at the start (seg_decode_kernel); 128: the chunks in the run's
// first and last 128-byte line of the column (relative to base: outside [nlo, nhi)) -- lines
// the neighbouring runs write too -- store with the default policy, the others with kNT, so
// the two runs' pieces of a shared line can meet in L2 (and the stream's first and last ring
// slots load so); 256 the stores alone, 512 the loads alone; 1024 (with 256): the policy chosen
// per 64-chunk step (default when the step touches such a line), not per lane.
template <int S, bool kNT, int kV = 0>
__device__ __forceinline__ bool seg_copy(Stream& st, const lds_u8* ring, uint32_t ring_lds,
                                         uint64_t base, uint32_t cst, uint32_t d, uint32_t len,
                                         uint32_t p, bool utf8, bool zero, uint4& carry,
                                         int lane, uint32_t nlo = 0, uint32_t nhi = 0) {
  constexpr bool kE = (kV & (128 | 512)) != 0;
  constexpr bool kES = (kV & (128 | 256)) != 0;
  uint32_t& ops = st.ops;
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
    const uint32_t gend = min(s0 + 16u * (g + 64u), p + len);  // this step's stream bytes end
    if constexpr ((kV & 4) != 0)
      if (!zero) ensure<S, kNT, kE>(st, ring, ring_lds, g ? s0 + 16u * g : p, gend - 1u, lane);
    uint4 val = zero ? z4 : ring16<S>(ring, s0 + 16u * kk);
    if (g == 0 && head && lane == 0) val = splice_lo(carry, val, head);
    const bool skip0 = shared0 && g == 0;
    if (kk < nfull && !(skip0 && lane == 0)) {
      if constexpr (kES && (kV & 1024) != 0) {
        if (dbeg + 16u * g >= nlo && dbeg + 16u * min(g + 64u, nfull) <= nhi)  // wave-uniform
          st16<kNT>(out + 16ull * kk, val);
        else
          st16<false>(out + 16ull * kk, val);
      } else if constexpr (kES) {
        const uint32_t rk = dbeg + 16u * kk;
        if (rk >= nlo && rk + 16u <= nhi) st16<kNT>(out + 16ull * kk, val);
        else st16<false>(out + 16ull * kk, val);
      } else {
        st16<kNT>(out + 16ull * kk, val);
      }
    }
    if (min(nfull, g + 64u) > g + (skip0 ? 1u : 0u)) ++ops;  // that store was issued
    if ((kV & 8) == 0)
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
    if constexpr ((kV & 2) != 0) pump<S, kNT, kE>(st, ring_lds, gend >> 10, lane);
  }
  carry = last;
  return utf8 ? __any(bad) != 0 : false;
}

// The column table of a lean-path workgroup, ahead of the waves' LDS (dynamic, ncols entries;
// 256-byte pieces: the early prologue copies it with one 4-byte LDS-DMA load per lane and piece).
__host__ __device__ __forceinline__ uint32_t seg_cols_lds(int ncols) {
  return (uint32_t(ncols) * uint32_t(sizeof(DevCol)) + 255u) & ~255u;
}

// W waves per workgroup (one run each): fewer waves per workgroup waste less LDS per CU.
// Measurement only (kProf, MDSX_TUNE sdbg bit 64): shader-clock stamps per wave (run), written
// to src_abs[3 tile + k]: k 0 the wave's start to its first sample landed, 1 the later samples'
// ring waits, 2 the whole wave.
__device__ __forceinline__ uint64_t seg_clock() {
  uint64_t c;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(c)::"memory");
  return c;
}

// The run's bytes: one range starting on a 128-byte line, its first S KiB in flight at once.
template <int S, bool kNT, bool kE = false>
__device__ __forceinline__ uint64_t seg_stream_start(Stream& st, const TileRun& r, uint64_t batch,
                                                     uint32_t ring_lds, int lane) {
  const uint64_t sbase = (batch + r.stream) & ~uint64_t(127);
  st.base = reinterpret_cast<const uint4*>(sbase);
  st.nq = uint32_t((batch + r.stream + r.bytes - sbase + 15) >> 4);
  st.nslots = (st.nq + 63) >> 6;
  st.issued = 0;
  st.op_at = 0;
  st.mirrored = 0xffffffffu;
  st.landed = 0;
  pump<S, kNT, kE>(st, ring_lds, 0, lane);
  return sbase;
}

// kV (measurement variants, MDSX_TUNE sv; 0 the default): bit 1 -- the early prologue: the run's
// record loaded and its ring loads issued before the column table is in LDS (each wave copies the
// table itself by LDS-DMA and waits for exactly those loads; no workgroup barrier), so a wave's
// first sample waits for two dependent memory round trips instead of three; bits 2 and 4: seg_copy.
template <int S, bool kNT, int W, bool kProf = false, int kV = 0>
__global__ __launch_bounds__(64 * W, 4) void seg_decode_kernel(const DevArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr bool kE = (kV & (128 | 512)) != 0;  // boundary slots: default policy
  constexpr bool kES = (kV & (128 | 256)) != 0;  // boundary lines' stores: default policy
  const uint64_t t_start = kProf ? seg_clock() : 0;
  uint64_t t_wait = 0, t_first = 0;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = W == 1 ? 0 : __builtin_amdgcn_readfirstlane(t >> 6);
  MDSX_L DevCol* s_cols = (MDSX_L DevCol*)smem;
  // XCD-contiguous runs: the line two neighbouring runs share (read: a run starts on a 128-byte
  // line; written: partial output chunks) meets in one L2
  const uint32_t blk = (a.xcd_order & kXcdSeg) ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint32_t tile = blk * W + uint32_t(wave);
  const int TR = a.tile_rows;
  const int ncols = a.ncols, nvar = a.nvar;
  uint8_t* wl = smem + seg_cols_lds(ncols) + size_t(wave) * seg_wave_lds(S, TR, nvar, a.seg_small);
  const uint32_t ring_lds = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const MDSX_L uint8_t*)wl)));
  const uint64_t batch = reinterpret_cast<uint64_t>(a.batch);
  Stream st;
  st.ops = 0;
  uint64_t sbase = 0;
  TileRun r;
  if constexpr ((kV & 1) != 0) {
    if (tile >= a.ntiles) return;  // wave-uniform; no barrier below
    const uint32_t cbytes = uint32_t(ncols) * uint32_t(sizeof(DevCol));
    // the table in the kernel-argument segment (DevArgs is the kernel's only argument; taking
    // a.cols's address would copy the argument block to scratch)
    const uint8_t* csrc = (const uint8_t*)__builtin_amdgcn_kernarg_segment_ptr() +
                          offsetof(DevArgs, cols);
    const uint32_t cl = __builtin_amdgcn_readfirstlane(
        static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const MDSX_L uint8_t*)smem)));
    for (uint32_t q = 0; q < cbytes; q += 256u) {  // identical bytes from every wave
      glds4(csrc + q + 4u * uint32_t(lane), cl + q);
      ++st.ops;
    }
    r = a.tile_run[tile];
    if (r.fast & 2) sbase = seg_stream_start<S, kNT, kE>(st, r, batch, ring_lds, lane);
    wait_vm_exact16(st.issued);  // the table's loads landed (issued before the ring's)
  } else {
    for (int c = t; c < a.ncols; c += 64 * W) s_cols[c] = a.cols[c];
    __syncthreads();
    if (tile >= a.ntiles) return;  // wave-uniform; no barrier below
    r = a.tile_run[tile];
    if (r.fast & 2) sbase = seg_stream_start<S, kNT, kE>(st, r, batch, ring_lds, lane);
  }
  if constexpr ((kV & 32) != 0) {
    // the run's 128-byte lines beyond the ring's first fill, touched now (one 4-byte LDS-DMA
    // load each into a scratch word after the waves' LDS: the line lands in L2, nothing in a
    // register), so that the later ring loads of this run hit L2
    if (r.fast & 2) {
      const uint32_t beyond = st.nq > uint32_t(S) * 64u ? st.nq - uint32_t(S) * 64u : 0u;
      if (beyond) {
        const uint32_t lines = min((beyond + 7u) >> 3, 64u);
        const uint32_t scratch = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(
            reinterpret_cast<uintptr_t>((const MDSX_L uint8_t*)(smem + seg_cols_lds(ncols) +
                                                                 size_t(W) * seg_wave_lds(
                                                                     S, TR, nvar, a.seg_small)))));
        const uint8_t* line = reinterpret_cast<const uint8_t*>(st.base) + uint64_t(S) * 1024u +
                              128u * uint32_t(lane < int(lines) ? lane : 0);
        glds4(line, scratch);
        ++st.ops;
      }
    }
  }
  const MDSX_L DevCol* cols = (const MDSX_L DevCol*)s_cols;
  if (!(r.fast & 2)) {
    run_body<S, kNT>(a, cols, tile, r, wl, lane);
    return;
  }
  const lds_u8* ring = (const lds_u8*)wl;
  MDSX_L uint32_t* obuf = (MDSX_L uint32_t*)(wl + S * 1024 + kMirror);  // [nvar][TR]
  MDSX_L uint8_t* fbuf = (MDSX_L uint8_t*)(wl + S * 1024 + kMirror + nvar * TR * 4);  // [nvar][TR]
  MDSX_L uint8_t* sbuf = (MDSX_L uint8_t*)(wl + run_wave_lds(S, TR, nvar));  // small columns
  const uint64_t shard = batch + (r.offs - 4ull - 4ull * r.r0);  // the shard file's first byte
  const int n = int(r.nrows);
  const uint64_t row0 = r.row0;
  // lane j holds offsets[r0 + j] (j <= n)
  const uint32_t ob = lane <= n ? *reinterpret_cast<const uint32_t*>(a.batch + r.offs + 4u * lane)
                                : 0u;

  // column facts and cursors, lane-distributed (lane c: column c)
  int vi = -1;
  uint32_t rb = 0, meta = 0, cur = 0, nlo = 0, nhi = 0;
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
    if constexpr (kES) {  // the run's lines of the column no neighbouring run writes
      const uint64_t end = first + (vi >= 0 ? uint64_t(a.tile_total[uint64_t(vi) * a.nscan + tile])
                                            : uint64_t(n) * rb);
      nlo = uint32_t(((first + 127) & ~uint64_t(127)) - base);
      nhi = uint32_t(max(end & ~uint64_t(127), base) - base);
    }
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
    uint64_t t_w0 = 0;
    if constexpr (kProf) t_w0 = seg_clock();
    if constexpr ((kV & 4) != 0)  // the heads; every value's bytes are waited for step by step
      ensure<S, kNT, kE>(st, ring, ring_lds, sp, sp + min(size, hv) + 3u, lane);
    else
      ensure<S, kNT, kE>(st, ring, ring_lds, sp, sp + size + 15u, lane);  // ALL of the sample's bytes
    if constexpr (kProf) {
      const uint64_t now = seg_clock();
      if (j == 0) t_first = now - t_start;
      else t_wait += now - t_w0;
    }
    if constexpr ((kV & 64) != 0) {
      // (measurement only, outputs incomplete) column 0 alone -- a ragged column whose value
      // comes first after the heads (config C's `b`) -- copied through the ring; no geometry, no
      // other column, no str check (with bit 16: no per-run outputs either)
      const int c0 = 0;
      const uint32_t len0 = uint32_t(__builtin_amdgcn_readfirstlane(int(ring_u32<S>(ring, sp))));
      // (column 0 must be a ragged column whose head comes first, and writable; else nothing)
      const bool col0 = __builtin_amdgcn_readfirstlane(vi) == 0 && (wide_mask & 1ull);
      const uint32_t l = (col0 && hv + len0 <= size) ? len0 : 0u;
      const uint32_t d = uint32_t(__builtin_amdgcn_readlane(int(cur), c0));
      uint4 cy = (d & 15u) ? readlane4(carry, c0) : make_uint4(0, 0, 0, 0);
      if (vi == 0 && lane == 0) obuf[j] = d;
      seg_copy<S, kNT, 0>(st, ring, ring_lds, readlane64(base, c0),
                          uint32_t(__builtin_amdgcn_readlane(int(cst), c0)), d, l, sp + hv, false,
                          false, cy, lane);
      if (lane == c0) {
        cur = d + l;
        carry = cy;
      }
      pump<S, kNT, kE>(st, ring_lds, (sp + size) >> 10, lane);
      ++j;
      continue;
    }
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
    if constexpr ((kV & 4) == 0) {
      if (small)
        lds_put(sbuf + soff + uint32_t(j) * rb,
                ok ? ring16<S>(ring, pos) : make_uint4(0, 0, 0, 0), rb);
    }
    if (vi >= 0) {
      obuf[vi * TR + j] = cur;
      if ((meta >> 8) & 1u) fbuf[vi * TR + j] = 0;
    }
    // the wide columns (kV bit 4: and the small ones), in column order = stream order
    uint64_t wm = (kV & 4) ? (wide_mask | small_mask) : wide_mask;
    while (wm) {
      const int c = __builtin_ctzll(wm);
      wm &= wm - 1;
      const uint32_t p = uint32_t(__builtin_amdgcn_readlane(int(pos), c));
      if constexpr ((kV & 4) != 0) {
        if ((small_mask >> c) & 1ull) {
          const uint32_t w = uint32_t(__builtin_amdgcn_readlane(int(rb), c));
          if (ok) ensure<S, kNT, kE>(st, ring, ring_lds, p, p + w - 1u, lane);
          const uint4 v = ok ? ring16<S>(ring, p) : make_uint4(0, 0, 0, 0);
          if (lane == c) lds_put(sbuf + soff + uint32_t(j) * w, v, w);
          continue;
        }
      }
      const uint32_t l = uint32_t(__builtin_amdgcn_readlane(int(clen), c));
      if (l == 0) continue;
      const uint32_t d = uint32_t(__builtin_amdgcn_readlane(int(cur), c));
      const uint32_t mc = uint32_t(__builtin_amdgcn_readlane(int(meta), c));
      const uint32_t cs = uint32_t(__builtin_amdgcn_readlane(int(cst), c));
      uint4 cy = (d & 15u) ? readlane4(carry, c) : make_uint4(0, 0, 0, 0);
      const bool utf8 = (mc >> 8) & 1u;
      const bool bad = seg_copy<S, kNT, kV>(
          st, ring, ring_lds, readlane64(base, c), cs, d, l, p, utf8, !ok, cy, lane,
          kES ? uint32_t(__builtin_amdgcn_readlane(int(nlo), c)) : 0u,
          kES ? uint32_t(__builtin_amdgcn_readlane(int(nhi), c)) : 0u);
      if (lane == c) {
        cur = d + l;
        carry = cy;
      }
      if (bad && lane == 0) fbuf[(int(mc & 255u) - 1) * TR + j] = 1;
      pump<S, kNT, kE>(st, ring_lds, (p + l) >> 10, lane);  // the bytes before p + l are done
    }
    ++j;
  }
  // the partly filled last chunk of every wide column (bytes [max(cst, chunk), cur))
  for (uint64_t m = (kV & 8) ? 0ull : wide_mask; m; m &= m - 1) {
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
  // the staged small fixed columns, one row per lane (kV bit 16, ablation: none of the run's
  // per-row outputs -- small columns, offsets, flags -- is written)
  for (uint64_t m = (kV & 16) ? 0ull : small_mask; m; m &= m - 1) {
    const int c = __builtin_ctzll(m);
    const uint32_t w = cols[c].row_bytes;
    const uint32_t so = uint32_t(__builtin_amdgcn_readlane(int(soff), c));
    if (lane < n)
      lds_out(sbuf + so + uint32_t(lane) * w,
              static_cast<uint8_t*>(cols[c].data) + (row0 + uint64_t(lane)) * w, w);
  }
  // the run's ragged offsets and str flags
  for (int c = 0; c < ((kV & 16) ? 0 : ncols); ++c) {
    const MDSX_L DevCol& col = cols[c];
    const int v = col.var_index;
    if (v < 0) continue;
    // offsets[row] = (base - data) + the row's position relative to base
    const int64_t obase = int64_t(readlane64(base, c) - reinterpret_cast<uint64_t>(col.data));
    if (lane < n) *gp(col.offsets + row0 + lane) = obase + int64_t(obuf[v * TR + lane]);
    if (col.kind == MDSX_KIND_STR && col.flags && lane < n)
      *gp(col.flags + row0 + lane) = fbuf[v * TR + lane];
  }
  if constexpr (kProf) {
    if (lane == 0) {
      a.src_abs[3ull * tile] = t_first;
      a.src_abs[3ull * tile + 1] = t_wait;
      a.src_abs[3ull * tile + 2] = seg_clock() - t_start;
    }
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
                        size_t(W) * seg_wave_lds(a.run_slots, a.tile_rows, a.nvar, a.seg_small) +
                        ((plan->seg_var & 32) ? 256u : 0u) +  // (the touch variant's scratch)
                        size_t(plan->lds_pad_kb) * 1024u;     // (+ unused pad: occupancy)
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
  MDSX_SEG_CASE(7, true, WV)   \
  MDSX_SEG_CASE(7, false, WV)  \
  MDSX_SEG_CASE(8, true, WV)   \
  MDSX_SEG_CASE(8, false, WV)  \
  MDSX_SEG_CASE(16, true, WV)  \
  MDSX_SEG_CASE(16, false, WV)
    if (plan->seg_var) {  // measurement variants (7 KiB ring, nt, 2 waves)
      if (a.run_slots != 7 || !plan->run_nt || W != 2)
        return mdsx::fail(MDSX_E_ARG, "mdsx: seg variants: run=7, rnt=1, swg=2 only");
#define MDSX_SEG_V(V)                                                                         \
  if (plan->seg_var == V) {                                                                   \
    mdsx::set_last_kernel("seg_decode_kernel<7, true, 2, false, " #V ">");                   \
    hipLaunchKernelGGL((seg_decode_kernel<7, true, 2, false, V>), dim3(sgrid), dim3(128), slds, \
                       s, a);                                                                 \
    return hip_check(hipGetLastError(), "seg_decode_kernel launch");                          \
  }
      MDSX_SEG_V(1) MDSX_SEG_V(2) MDSX_SEG_V(3) MDSX_SEG_V(4) MDSX_SEG_V(8) MDSX_SEG_V(16)
      MDSX_SEG_V(7) MDSX_SEG_V(24) MDSX_SEG_V(32) MDSX_SEG_V(33) MDSX_SEG_V(80) MDSX_SEG_V(128)
      MDSX_SEG_V(256) MDSX_SEG_V(512) MDSX_SEG_V(1280)
#undef MDSX_SEG_V
      return mdsx::fail(MDSX_E_ARG, "mdsx: seg variant out of range");
    }
    if (plan->stage_debug & 64) {  // measurement only: the per-wave stamps (7 KiB ring, nt, 2)
      if (a.run_slots != 7 || !plan->run_nt || W != 2)
        return mdsx::fail(MDSX_E_ARG, "mdsx: seg stamps: run=7, rnt=1, swg=2 only");
      if (3ull * a.ntiles > uint64_t(a.nvar) * a.rows)  // the stamps' space: nvar x rows words
        return mdsx::fail(MDSX_E_ARG, "mdsx: seg stamps need 3 x tiles <= nvar x rows");
      mdsx::set_last_kernel("seg_decode_kernel<7, true, 2, true>");
      hipLaunchKernelGGL((seg_decode_kernel<7, true, 2, true>), dim3(sgrid), dim3(128), slds, s, a);
      return hip_check(hipGetLastError(), "seg_decode_kernel launch");
    }
    MDSX_SEG_W(1)
    MDSX_SEG_W(2)
    MDSX_SEG_W(4)
#undef MDSX_SEG_W
#undef MDSX_SEG_CASE
    return mdsx::fail(MDSX_E_ARG, "mdsx: streaming decode ring of 4, 7, 8 or 16 KiB");
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
  MDSX_RUN_CASE(7, true)
  MDSX_RUN_CASE(7, false)
  MDSX_RUN_CASE(8, true)
  MDSX_RUN_CASE(8, false)
  MDSX_RUN_CASE(16, true)
  MDSX_RUN_CASE(16, false)
#undef MDSX_RUN_CASE
  return mdsx::fail(MDSX_E_ARG, "mdsx: streaming decode ring of 4, 7, 8 or 16 KiB");
}

}  // namespace mdsx_kernels
