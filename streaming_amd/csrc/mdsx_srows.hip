// Streaming row-parallel decode of short ragged samples (gfx950): one wave decodes one tile --
// up to 256 consecutive samples of one shard -- by streaming the tile's bytes through a private
// LDS ring ONCE, in windows of up to 31 samples, lane-parallel per sample and output-chunk-
// parallel per column inside each window.
//
// The reference decodes one sample per call (MDSReader.get_sample_data, mds/reader.py:128-149;
// decode_sample, :103-126; mds_decode, encodings.py:760-773). The row-parallel decode
// (mdsx_rows.hip) stages a whole tile in LDS and holds it while the tile is parsed, scanned and
// written: at ~20 KiB per tile six tiles fit a CU, and a tile's bytes are in flight only during its
// first ~20 % (short rows ran at a third of HBM, parked on the tile's latency chain).
// Here the stage is a ring smaller than the tile (the verdict's "stream the tile's bytes through a
// per-workgroup ring smaller than the tile"): while the wave parses and writes window w, the
// bytes of the windows after it are landing in the ring's other slots, and a wave's LDS is the
// ring plus small per-window tables, so twice as many tiles stream per CU.
//
// Per window (samples [j0, j0 + m), their bytes at most seg_lim, every sample of the tile at most
// seg_lim: TileRun bit 1 from the scan pass, stage_totals_kernel):
//   1. lane j holds sample j0 + j's offsets pair (the tile's offsets are held lane-distributed);
//      the wave waits for the window's bytes (explicit vmcnt, mdsx_ring.h);
//   2. lane j parses its sample's size heads from the ring and checks the column boundaries
//      (mds/reader.py:111-125; a failing sample counts zero bytes and is reported, the scan
//      pass's rule), writes its value records (window output byte, bytes, stream position);
//   3. per ragged column a DPP wave scan places the values onto the column's running output
//      cursor; lane j writes the offsets and marks the chunk map (the sample holding the first
//      byte of each 16-byte output chunk); fixed columns of <= 16 bytes are written one row per
//      lane;
//   4. every wider column output-chunk-parallel: lane k assembles 16-byte output chunk k from the
//      ring (unaligned ds_read_b128, a piece of each value a chunk spans) and stores it whole; the
//      chunk a window leaves partly filled is carried (lane c of a register) into the next
//      window's first chunk, so only the two chunks a tile shares with its neighbours are stored
//      a byte at a time. str pieces are checked for strict UTF-8 on the way (bytes.decode('utf-8'),
//      encodings.py:80-81) and each sample's flag written per window;
//   5. the ring slots below the next window are released and refilled.
// Tiles the scan pass did not mark (a sample failing the file checks, or larger than seg_lim) are
// listed for the row-parallel kernel, launched after this one over the list only.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "mdsx_decode.h"
#include "mdsx_device.h"
#include "mdsx_internal.h"
#include "mdsx_ring.h"

namespace mdsx_kernels {
namespace {

// Value records per column of a window (lane j: sample j, lane j + 1: its end): 32 with the ring
// (windows of <= 31 samples), 64 when the samples are read from L2 (kL2, <= 63).
__host__ __device__ __forceinline__ int sr_rec(bool l2) { return l2 ? 64 : 32; }

// LDS: the workgroup's column table, then per wave: the ring (+ mirror) -- or (kL2) a 256-byte
// scratch the line touches land in --, [ncols][sr_rec] value records, [nvar][map_len] chunk maps,
// one UTF-8 word (two with kL2) per column.
__host__ __device__ __forceinline__ uint32_t sr_cols_lds(int ncols) {
  return (uint32_t(ncols) * uint32_t(sizeof(DevCol)) + 15u) & ~15u;
}
__host__ __device__ __forceinline__ uint32_t sr_map_len(uint32_t lim) { return lim / 16u + 8u; }
__host__ __device__ __forceinline__ uint32_t sr_wave_lds(int S, int ncols, int nvar, uint32_t lim,
                                                         bool l2) {
  return (l2 ? 256u : uint32_t(S) * 1024u + kMirror) + uint32_t(ncols) * uint32_t(sr_rec(l2)) * 16u +
         ((uint32_t(nvar) * sr_map_len(lim) + 15u) & ~15u) + ((uint32_t(ncols) * 8u + 15u) & ~15u);
}

// 16 / 4 bytes at any byte address of global memory (gfx950 loads unaligned dwordx4 / dword:
// scripts/microbench/unaligned_copy.hip, bit-exact at every offset).
__device__ __forceinline__ uint4 ldu16(const uint8_t* p) {
  u32x4 v;
  __builtin_memcpy(&v, (const MDSX_G uint8_t*)p, 16);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint32_t ldu32(const uint8_t* p) {
  uint32_t v;
  __builtin_memcpy(&v, (const MDSX_G uint8_t*)p, 4);
  return v;
}

struct SrRec {  // one value of a window: output byte (window-relative), bytes, stream position
  uint32_t dst, len, src, pad;
};

// the tile's offsets, lane-distributed: q selects offsets[64 q + lane] (wave-uniform q)
__device__ __forceinline__ uint32_t sel5(uint32_t o0, uint32_t o1, uint32_t o2, uint32_t o3,
                                         uint32_t o4, int q) {
  return q == 0 ? o0 : q == 1 ? o1 : q == 2 ? o2 : q == 3 ? o3 : o4;
}

// Bytes [from, to) of chunk v stored at the aligned address D (one lane, a byte at a time).
__device__ __forceinline__ void store_bytes_from(uint64_t D, const uint4 v, uint32_t from,
                                                 uint32_t to) {
  for (uint32_t k = from; k < to; ++k) *gp_at<uint8_t>(D + k) = uint8_t(byte_of(v, int(k)));
}

// n (1..16) bytes of v to global memory at q (q aligned to the largest power of two dividing n)
__device__ __forceinline__ void store_small(uint64_t q, const uint4 v, uint32_t n) {
  if (n == 8) {
    *gp_at<uint64_t>(q) = uint64_t(v.x) | (uint64_t(v.y) << 32);
  } else if (n == 4) {
    *gp_at<uint32_t>(q) = v.x;
  } else if (n == 16) {
    st16<false>(q, v);
  } else if (n == 2) {
    *gp_at<uint16_t>(q) = uint16_t(v.x);
  } else {
    for (uint32_t b = 0; b < n; ++b) *gp_at<uint8_t>(q + b) = uint8_t(byte_of(v, int(b)));
  }
}

// kL2: no ring -- the samples' bytes are read from global memory (their lines touched into L2
// when the window is laid out, the reads unaligned 16-byte loads), so a wave's LDS is its tables
// only and up to five waves per SIMD hold a tile each; windows of up to 63 samples, seg_lim bytes.
template <int S, bool kNT, int W, bool kL2>
__global__ __launch_bounds__(64 * W, kL2 ? 5 : 1) void srows_decode_kernel(const DevArgs a) {
  constexpr int kRec = kL2 ? 64 : 32;
  constexpr int kSrWin = kRec - 1;  // samples per window at most
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int t = threadIdx.x, lane = t & 63;
  const int wave = W == 1 ? 0 : __builtin_amdgcn_readfirstlane(t >> 6);
  MDSX_L DevCol* s_cols = (MDSX_L DevCol*)smem;
  for (int c = t; c < a.ncols; c += 64 * W) s_cols[c] = a.cols[c];
  __syncthreads();
  const MDSX_L DevCol* cols = (const MDSX_L DevCol*)s_cols;
  const uint32_t blk = (a.xcd_order & kXcdSeg) ? xcd_block(blockIdx.x, gridDim.x) : blockIdx.x;
  const uint32_t tile = blk * W + uint32_t(wave);
  if (tile >= a.ntiles) return;  // wave-uniform; no barrier below
  const TileRun r = a.tile_run[tile];
  if ((r.fast & 2) == 0) {  // the row-parallel kernel's: listed for it
    if (lane == 0) {
      uint32_t* count = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(a.status) +
                                                    kSrowsCountOffset);
      a.tile_list[atomicAdd(count, 1u)] = tile;
    }
    return;
  }
  const int ncols = a.ncols, nvar = a.nvar;
  const uint32_t lim = a.seg_lim;
  const uint32_t map_len = sr_map_len(lim);
  uint8_t* wl = smem + sr_cols_lds(ncols) + size_t(wave) * sr_wave_lds(S, ncols, nvar, lim, kL2);
  const lds_u8* ring = (const lds_u8*)wl;
  MDSX_L SrRec* rec = (MDSX_L SrRec*)(wl + (kL2 ? 256 : S * 1024 + kMirror));  // [ncols][kRec]
  MDSX_L uint8_t* map = (MDSX_L uint8_t*)(rec + ncols * kRec);  // [nvar][map_len]
  MDSX_L uint32_t* bad = (MDSX_L uint32_t*)(map + ((uint32_t(nvar) * map_len + 15u) & ~15u));
  const uint32_t ring_lds = __builtin_amdgcn_readfirstlane(
      static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const MDSX_L uint8_t*)wl)));
  const uint64_t batch = reinterpret_cast<uint64_t>(a.batch);
  const int n = int(r.nrows);
  // the tile's offsets (lane j: offsets[r0 + 64 q + j], q < 5: up to 257 values), issued before
  // the ring's loads so that their first use waits for them alone
  const uint32_t* offs = reinterpret_cast<const uint32_t*>(a.batch + r.offs);
  uint32_t o0 = lane <= n ? offs[lane] : 0u;
  uint32_t o1 = 64 + lane <= n ? offs[64 + lane] : 0u;
  uint32_t o2 = 128 + lane <= n ? offs[128 + lane] : 0u;
  uint32_t o3 = 192 + lane <= n ? offs[192 + lane] : 0u;
  uint32_t o4 = 256 + lane <= n ? offs[256 + lane] : 0u;
  // the tile's bytes: one range starting on a 128-byte line, its first S KiB in flight at once
  // (kL2: positions are bytes of the shard file, read from global memory)
  Stream st;
  const uint64_t sbase = (batch + r.stream) & ~uint64_t(127);
  const uint8_t* frame = a.batch + r.shard_off;
  uint32_t sp0 = 0;
  if constexpr (!kL2) {
    st.base = reinterpret_cast<const uint4*>(sbase);
    st.nq = uint32_t((batch + r.stream + r.bytes - sbase + 15) >> 4);
    st.nslots = (st.nq + 63) >> 6;
    st.issued = 0;
    st.ops = 0;
    st.op_at = 0;
    st.mirrored = 0xffffffffu;
    st.landed = 0;
    pump<S, kNT>(st, ring_lds, 0, lane);
    sp0 = uint32_t(batch + r.shard_off - sbase);  // stream position of file byte 0
  }
  // the source bytes: from the ring, or (kL2) from global memory at a shard-file position
  auto rd16 = [&](uint32_t p) -> uint4 {
    if constexpr (kL2) return ldu16(frame + p);
    else return ring16<S>(ring, p);
  };
  auto rd32 = [&](uint32_t p) -> uint32_t {
    if constexpr (kL2) return ldu32(frame + p);
    else return ring_u32<S>(ring, p);
  };
  uint32_t sink = 0;  // (kL2) the line touches' words, kept live until the tile's end
  uint32_t touch[4] = {0, 0, 0, 0};

  // column facts and cursors, lane-distributed (lane c: column c)
  int vi = -1;
  uint32_t rb = 0;
  uint64_t data = 0, cur = 0;  // cur: the column's next output byte (relative to its data)
  bool small = false, wide = false, utf8 = false, skip = false;
  if (lane < ncols) {
    const MDSX_L DevCol& col = cols[lane];
    vi = col.var_index;
    rb = col.row_bytes;
    data = reinterpret_cast<uint64_t>(col.data);
    if (vi >= 0) {
      cur = uint64_t(a.tile_prefix[uint64_t(vi) * a.nscan + tile]);
      if (cur + uint64_t(a.tile_total[uint64_t(vi) * a.nscan + tile]) > col.capacity) {
        report_decode(a, MDSX_E_CAPACITY, int(r.shard), int(r.r0), lane);
        skip = true;  // this tile writes no value of the column
      }
      utf8 = col.kind == MDSX_KIND_STR && col.flags != nullptr;
    } else {
      cur = r.row0 * uint64_t(rb);
    }
    small = vi < 0 && rb <= uint32_t(kSmallMax);
    wide = !small && !skip;
  }
  for (int i = lane; i < 2 * ncols; i += 64) bad[i] = 0;
  const uint64_t wide_mask = __ballot(wide);
  const uint64_t small_mask = __ballot(small);
  const uint64_t utf8_mask = __ballot(utf8 && !skip);
  // lane c: the partly filled chunk at (data + cur) & ~15 carried to the next window (pend), its
  // bytes [clo, cur & 15) this tile's (clo > 0: the tile's first chunk, shared with the tile
  // before)
  uint4 carry = make_uint4(0, 0, 0, 0);
  bool pend = false;
  uint32_t clo = 0;
  const uint32_t hv = 4u * uint32_t(nvar);
  const uint4 z4 = make_uint4(0, 0, 0, 0);

  for (int j0 = 0; j0 < n;) {  // wave-uniform
    // ---- 1. the window: lane j holds offsets[r0 + j0 + j]
    const int q0 = j0 >> 6, sh = j0 & 63;
    const int from = (lane + sh) & 63;
    const uint32_t va = uint32_t(__shfl(int(sel5(o0, o1, o2, o3, o4, q0)), from));
    const uint32_t vb = uint32_t(__shfl(int(sel5(o0, o1, o2, o3, o4, q0 + 1)), from));
    const uint32_t wo = lane + sh < 64 ? va : vb;
    const uint32_t ob = uint32_t(__builtin_amdgcn_readfirstlane(int(wo)));
    const bool fit = lane <= kSrWin && j0 + lane <= n && wo - ob <= lim;  // (kSrWin: uniform)
    const int m = __popcll(__ballot(fit)) - 1;  // samples of the window
    if (m < 1) {  // (every sample is at most seg_lim: TileRun bit 1; an exit every wave reaches)
      if (lane == 0) report_decode(a, MDSX_E_HIP, int(r.shard), int(r.r0) + j0, -1);
      return;
    }
    const uint32_t b = wo, e = uint32_t(__shfl(int(wo), (lane + 1) & 63));
    const bool mine = lane < m;
    const uint32_t sp = b + sp0;  // stream position of the sample
    const uint32_t wlo = ob + sp0;
    const uint32_t whi = uint32_t(__builtin_amdgcn_readlane(int(wo), m)) + sp0;
    uint4 h4 = z4;
    if constexpr (kL2) {
      // the size heads first, then the window's 128-byte lines touched into L2 (one word each):
      // the heads' wait leaves the touches in flight, and the chunk reads below hit L2
      if (mine && nvar <= 4) h4 = ldu16(frame + b);
      // (up to 4 x 8 KiB of lines, lim <= 32 KiB; each word folded into `sink` only after the
      // window is written, so no wait for a touch is placed before that)
      const uint64_t l0 = (reinterpret_cast<uint64_t>(frame) + wlo) & ~uint64_t(127);
      const uint64_t l1 = reinterpret_cast<uint64_t>(frame) + whi;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint64_t q = l0 + 128ull * uint64_t(lane + 64 * i);
        touch[i] = q < l1 ? *gp_at<const uint32_t>(q) : 0u;
      }
    } else {
      ensure<S, kNT>(st, ring, ring_lds, wlo, whi - 1u, lane);  // the window's bytes landed
      if (mine && nvar <= 4) h4 = ring16<S>(ring, sp);
    }

    // ---- 2. column boundaries (mds/reader.py:111-125), value records
    auto head = [&](int k) -> uint32_t {
      if (nvar <= 4) return k == 0 ? h4.x : k == 1 ? h4.y : k == 2 ? h4.z : h4.w;
      return rd32(sp + 4u * uint32_t(k));
    };
    bool ok = mine && hv <= e - b;
    uint64_t need = hv;
    for (int c = 0; c < ncols; ++c) {  // uniform
      const int v = __builtin_amdgcn_readlane(vi, c);
      const uint32_t w = uint32_t(__builtin_amdgcn_readlane(int(rb), c));
      need += v >= 0 ? (ok ? head(v) : 0u) : w;
    }
    ok = ok && need <= uint64_t(e - b);
    if (mine && !ok) report_decode(a, MDSX_E_BOUNDS, int(r.shard), int(r.r0) + j0 + lane, -1);
    {
      uint32_t rel = hv;
      for (int c = 0; c < ncols; ++c) {
        const int v = __builtin_amdgcn_readlane(vi, c);
        const uint32_t w = uint32_t(__builtin_amdgcn_readlane(int(rb), c));
        const uint32_t len = ok ? (v >= 0 ? head(v) : w) : 0u;
        if (mine) {
          rec[c * kRec + lane].len = len;
          rec[c * kRec + lane].src = sp + rel;
          rec[c * kRec + lane].dst = v >= 0 ? 0u : uint32_t(lane) * w;
        }
        rel += len;
      }
    }
    // ---- 3. ragged values placed by a wave scan; offsets; chunk maps. Small fixed columns.
    uint32_t wtot = 0;  // lane c: the window's output bytes of column c
    for (int c = 0; c < ncols; ++c) {  // uniform
      const int v = __builtin_amdgcn_readlane(vi, c);
      const uint32_t w = uint32_t(__builtin_amdgcn_readlane(int(rb), c));
      if (v < 0) {
        if (lane == c) wtot = uint32_t(m) * w;
        continue;
      }
      const uint32_t len = mine ? rec[c * kRec + lane].len : 0u;
      const uint32_t incl = wave_incl_dpp(len);
      const uint32_t ex = incl - len;
      const uint32_t tot = uint32_t(__builtin_amdgcn_readlane(int(incl), 63));
      const uint64_t cc = readlane64(cur, c);
      const MDSX_L DevCol& col = cols[c];
      if (mine) {
        *gp(col.offsets + r.row0 + uint64_t(j0 + lane)) = int64_t(cc + ex);
        rec[c * kRec + lane].dst = ex;
        if (len) {
          // chunk k of the window's output begins at window byte 16 k - hd; this sample holds
          // the first byte of chunks [k0, k1)
          const uint32_t hd = uint32_t((reinterpret_cast<uint64_t>(col.data) + cc) & 15u);
          const uint32_t k0 = ex == 0 ? 0u : (ex + hd + 15u) >> 4;
          const uint32_t k1 = (ex + len + hd + 15u) >> 4;
          MDSX_L uint8_t* mp = map + uint32_t(v) * map_len;
          for (uint32_t k = k0; k < k1; ++k) mp[k] = uint8_t(lane);
        }
      }
      if (lane == c) wtot = tot;
    }
    for (uint64_t mm = small_mask; mm; mm &= mm - 1) {
      const int c = __builtin_ctzll(mm);
      const uint32_t w = uint32_t(__builtin_amdgcn_readlane(int(rb), c));
      if (mine) {
        const MDSX_L SrRec& q = rec[c * kRec + lane];
        const uint4 v = q.len ? rd16(q.src) : z4;
        store_small(readlane64(data, c) + (r.row0 + uint64_t(j0 + lane)) * w, v, w);
      }
    }

    // ---- 4. every wider column, output-chunk-parallel, str pieces checked on the way
    for (uint64_t mm = wide_mask; mm; mm &= mm - 1) {
      const int c = __builtin_ctzll(mm);
      const uint32_t T = uint32_t(__builtin_amdgcn_readlane(int(wtot), c));
      if (T == 0) continue;
      const int v = __builtin_amdgcn_readlane(vi, c);
      const uint32_t w = v >= 0 ? 0u : uint32_t(__builtin_amdgcn_readlane(int(rb), c));
      const uint64_t wout = readlane64(data, c) + readlane64(cur, c);
      const uint64_t D0 = wout & ~uint64_t(15);
      const int32_t hd = int32_t(wout - D0);
      const uint32_t K = (uint32_t(hd) + T + 15u) >> 4;
      const bool chk = (utf8_mask >> c) & 1ull;
      const bool cpend = uint32_t(__builtin_amdgcn_readlane(int(pend), c)) != 0;
      const uint32_t cclo = uint32_t(__builtin_amdgcn_readlane(int(clo), c));
      const uint4 cy = readlane4(carry, c);
      const bool tail = ((uint32_t(hd) + T) & 15u) != 0;  // the last chunk is partly filled
      const MDSX_L uint8_t* mp = map + uint32_t(v >= 0 ? v : 0) * map_len;
      const int base = c * kRec;
      uint4 last = z4;
      uint32_t last_lo = 0;
      for (uint32_t kb = 0; kb < K; kb += 64) {  // wave-uniform
        const uint32_t k = kb + uint32_t(lane);
        uint4 val = z4;
        uint32_t lob = 0;  // the chunk's first byte of this tile
        if (k < K) {
          const int32_t P0 = int32_t(k * 16) - hd;  // window output byte of the chunk's byte 0
          int32_t pos = max(P0, 0);
          const int32_t end = min(P0 + 16, int32_t(T));
          const int rr = w ? int(uint32_t(pos) / w) : int(mp[k]);
          // the common chunk: one value (A) or two (A, then B from byte sB), straight-line
          const MDSX_L SrRec& qa = rec[base + rr];
          const int32_t dsA = int32_t(qa.dst), deA = dsA + int32_t(qa.len);
          const uint32_t pa = qa.src - uint32_t(dsA) + uint32_t(P0);  // stream pos. of byte 0
          val = rd16(pa);
          const int32_t hiA = min(end, deA);
          bool simple = deA > pos;  // (a fixed column's failed sample: no bytes)
          uint32_t sB = 16;
          int32_t deL = deA;  // end of the chunk's last value
          if (simple && hiA < end) {
            const MDSX_L SrRec& qb = rec[base + rr + 1];
            const int32_t dsB = int32_t(qb.dst), deB = dsB + int32_t(qb.len);
            simple = dsB == hiA && deB >= end;
            if (simple) {
              const uint4 vb4 = rd16(qb.src - uint32_t(dsB) + uint32_t(P0));
              sB = uint32_t(hiA - P0);
              const uint4 mk = byte_mask(0, sB);
              val = make_uint4((val.x & mk.x) | (vb4.x & ~mk.x), (val.y & mk.y) | (vb4.y & ~mk.y),
                               (val.z & mk.z) | (vb4.z & ~mk.z), (val.w & mk.w) | (vb4.w & ~mk.w));
              deL = deB;
            }
          }
          if (simple) {
            if (chk) {
              const uint4 X = (pos > P0 || end < P0 + 16)
                                  ? keep_bytes(val, uint32_t(pos - P0), uint32_t(end - P0))
                                  : val;
              uint32_t pw = 0;
              if (pos > dsA) {
                pw = rd32(pa + uint32_t(pos - P0) - 4u);
                const int32_t nv = pos - dsA;  // A's bytes before the chunk
                if (nv < 4) pw &= ~((1u << (8 * (4 - nv))) - 1u);
              }
              const bool plain = (((X.x | X.y | X.z | X.w) & 0x80808080u) | hi_c0(pw)) == 0;
              if (!plain) {
                uint32_t er = utf8_chunk_err2(X, pw, sB);
                if (sB < 16 && utf8_open_at(X, pw, sB)) er |= 1u;
                if (end == P0 + 16 && end == deL) {
                  if (sB < 16) er |= utf8_open_at(keep_bytes(X, sB, 16), 0, 16) ? 2u : 0u;
                  else er |= utf8_open_at(X, pw, 16) ? 1u : 0u;
                }
                if (er & 1u) atomicOr(&bad[2 * c + (rr >> 5)], 1u << (rr & 31));
                if (er & 2u) atomicOr(&bad[2 * c + ((rr + 1) >> 5)], 1u << ((rr + 1) & 31));
              }
            }
          } else {
            // three or more values, an empty value, or a gap (a fixed column's failed sample
            // leaves zeros): piece by piece
            val = z4;
            for (int q = rr; q < m && pos < end; ++q) {
              const MDSX_L SrRec& qq = rec[base + q];
              const int32_t ds = int32_t(qq.dst);
              const int32_t de = ds + int32_t(qq.len);
              if (de <= pos) continue;  // a sample with no bytes in this column
              if (ds >= end) break;
              const int32_t lo = max(pos, ds), hi = min(end, de);
              const uint32_t p = qq.src - uint32_t(ds) + uint32_t(P0);
              const uint4 pv = keep_bytes(rd16(p), uint32_t(lo - P0), uint32_t(hi - P0));
              val = make_uint4(val.x | pv.x, val.y | pv.y, val.z | pv.z, val.w | pv.w);
              if (chk) {
                uint32_t pw = 0;
                if (lo > ds) {
                  pw = rd32(p + uint32_t(lo - P0) - 4u);
                  const int32_t nv = lo - ds;
                  if (nv < 4) pw &= ~((1u << (8 * (4 - nv))) - 1u);
                }
                if ((utf8_chunk_err2(pv, pw, 16) & 1u) ||
                    (hi == de && hi == P0 + 16 && utf8_open_at(pv, pw, 16)))
                  atomicOr(&bad[2 * c + (q >> 5)], 1u << (q & 31));
              }
              pos = hi;
            }
          }
          // the chunk's bytes below the window's first output byte: the carried chunk's (its
          // bytes [clo, hd)) or the tile before's (not stored here)
          if (k == 0 && hd > 0) {
            if (cpend) {
              val = splice_lo(cy, val, uint32_t(hd));
              lob = cclo;
            } else {
              lob = uint32_t(hd);
            }
          }
          const uint64_t D = D0 + 16ull * k;
          if (!(tail && k == K - 1)) {  // (the last chunk, partly filled, is carried)
            if (lob == 0) st16<kNT>(D, val);
            else store_bytes_from(D, val, lob, 16);
          }
        }
        if (tail && K - 1 - kb < 64u) {
          last = readlane4(val, int(K - 1 - kb));
          last_lo = uint32_t(__builtin_amdgcn_readlane(int(lob), int(K - 1 - kb)));
        }
      }
      if (lane == c) {
        cur += T;
        pend = tail;
        carry = last;
        clo = last_lo;
      }
    }

    // ---- 5. str flags of the window; the ring slots below the next window
    for (uint64_t mm = utf8_mask; mm; mm &= mm - 1) {
      const int c = __builtin_ctzll(mm);
      const uint32_t word = bad[2 * c + (lane >> 5)];
      if (mine) *gp(cols[c].flags + r.row0 + uint64_t(j0 + lane)) = uint8_t((word >> (lane & 31)) & 1u);
    }
    for (int i = lane; i < 2 * ncols; i += 64) bad[i] = 0;
    if constexpr (!kL2) pump<S, kNT>(st, ring_lds, whi >> 10, lane);
    else sink ^= touch[0] ^ touch[1] ^ touch[2] ^ touch[3];
    j0 += m;
  }
  // the partly filled last chunk of every wide column (its bytes [clo, cur & 15))
  for (uint64_t mm = wide_mask; mm; mm &= mm - 1) {
    const int c = __builtin_ctzll(mm);
    if (uint32_t(__builtin_amdgcn_readlane(int(pend), c)) == 0) continue;
    const uint64_t wend = readlane64(data, c) + readlane64(cur, c);
    const uint64_t C = wend & ~uint64_t(15);
    wave_edge_store(carry, c, C, C + uint32_t(__builtin_amdgcn_readlane(int(clo), c)), wend,
                    lane);
  }
  if constexpr (kL2) asm volatile("" ::"v"(sink));  // (the touches' loads are not dead code)
}

}  // namespace

int launch_srows_decode(const mdsx_plan* plan, const DevArgs& a, hipStream_t s) {
  constexpr int W = 2;
  const bool l2 = plan->srows == 2;  // the samples read from L2, no ring
  const unsigned grid = (a.ntiles + W - 1) / W;
  const size_t lds = sr_cols_lds(a.ncols) + size_t(W) * sr_wave_lds(int(a.srows_slots), a.ncols,
                                                                     a.nvar, a.seg_lim, l2);
  if (lds > 160 * 1024)
    return mdsx::fail(MDSX_E_ARG, "mdsx: streaming row-parallel decode LDS exceeds 160 KiB");
  if (!l2 && a.seg_lim + 2048u > a.srows_slots * 1024u)
    return mdsx::fail(MDSX_E_ARG, "mdsx: streaming row-parallel window larger than its ring");
  const bool nt = plan->rows_nt != 0;
  if (l2) {
    const void* fn = nt ? reinterpret_cast<const void*>(srows_decode_kernel<0, true, W, true>)
                        : reinterpret_cast<const void*>(srows_decode_kernel<0, false, W, true>);
    if (lds > 64 * 1024) {
      const int rc = hip_check(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                   int(lds)), "hipFuncSetAttribute");
      if (rc != MDSX_OK) return rc;
    }
    mdsx::set_last_kernel(nt ? "srows_decode_kernel<0, true, 2, true>"
                             : "srows_decode_kernel<0, false, 2, true>");
    if (nt)
      hipLaunchKernelGGL((srows_decode_kernel<0, true, W, true>), dim3(grid), dim3(64 * W), lds, s, a);
    else
      hipLaunchKernelGGL((srows_decode_kernel<0, false, W, true>), dim3(grid), dim3(64 * W), lds, s, a);
    return hip_check(hipGetLastError(), "srows_decode_kernel launch");
  }
#define MDSX_SR_CASE(S, NT)                                                                     \
  if (a.srows_slots == S && nt == NT) {                                                         \
    if (lds > 64 * 1024) {                                                                      \
      const int rc = hip_check(                                                                 \
          hipFuncSetAttribute(reinterpret_cast<const void*>(srows_decode_kernel<S, NT, W, false>), \
                              hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)),            \
          "hipFuncSetAttribute");                                                               \
      if (rc != MDSX_OK) return rc;                                                             \
    }                                                                                           \
    mdsx::set_last_kernel("srows_decode_kernel<" #S ", " #NT ", 2, false>");                    \
    hipLaunchKernelGGL((srows_decode_kernel<S, NT, W, false>), dim3(grid), dim3(64 * W), lds, s, a); \
    return hip_check(hipGetLastError(), "srows_decode_kernel launch");                          \
  }
  MDSX_SR_CASE(6, true)
  MDSX_SR_CASE(6, false)
  MDSX_SR_CASE(8, true)
  MDSX_SR_CASE(8, false)
  MDSX_SR_CASE(12, true)
  MDSX_SR_CASE(12, false)
#undef MDSX_SR_CASE
  return mdsx::fail(MDSX_E_ARG, "mdsx: streaming row-parallel ring of 6, 8 or 12 KiB");
}

}  // namespace mdsx_kernels
