// The streaming decode's general path (run_body), used by both kernels of mdsx_run.hip: the
// general-path kernel (run_decode_kernel) and the lean path (seg_decode_kernel), which hands it
// the runs its fast form does not take. A wave streams its run -- consecutive samples of one
// shard -- through its LDS ring once, sample by sample, any sample size, samples failing the file
// checks reported one by one.
// (The reference: MDSReader.get_sample_data / decode_sample, streaming/base/format/mds/
// reader.py:103-149; column decoders, encodings.py:62-397, 760-773.)
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "mdsx_decode.h"
#include "mdsx_device.h"
#include "mdsx_internal.h"
#include "mdsx_ring.h"

namespace mdsx_kernels {

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

}  // namespace mdsx_kernels
