// The totals pass of the streaming and row-parallel decodes of ragged plans (gfx950), and the
// huge-row kernel of the row-parallel decode.
//
// The reference decodes one sample per call: MDSReader.get_sample_data reads the sample's byte
// range (streaming/base/format/mds/reader.py:128-149), decode_sample splits it at the u32 size
// heads of the variable columns and mds_decode returns each column's value
// (mds/reader.py:103-126, encodings.py:62-397,760-773). The device decodes (mdsx_run.hip,
// mdsx_rows.hip) write each ragged column packed, so a tile of consecutive samples needs its
// output base: stage_totals_kernel reads every sample's offsets pair and size heads, sums each
// tile's ragged bytes (a sample failing a check counts zero, the decodes' rule) and writes each
// tile's run record (stream range, offsets-table slice, whether every sample passes the file
// checks and fits the lean path's ring); the tile bases then come from the scan kernels
// (mdsx_kernels.hip). (A single-pass form -- the scan chained into this pass by a decoupled
// look-back over workgroups in ticket order -- measured no faster on config C and 16 % slower on
// short rows: with thousands of workgroups starting together the inclusive prefixes propagate
// one block at a time. The three scan kernels as one look-back launch over 4096-entry chunks:
// 0.2 % slower on config C, 1 % on short rows, round 4.)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "mdsx_decode.h"
#include "mdsx_device.h"
#include "mdsx_internal.h"

namespace mdsx_kernels {

// The totals pass: the ragged bytes of every tile (one thread per row; 256 / TR tiles
// per workgroup), with the staged kernel's row rule: a row whose range, heads or columns do not
// fit counts zero. kNT: the size heads loaded non-temporal (each costs a whole 128-byte line
// either way; measured 10 % faster at a 254-byte stride, 9 % slower at 4.3 KB:
// profiles/r05/scan_heads/).
template <bool kNT>
__global__ __launch_bounds__(kBlock) void stage_totals_kernel(const DevArgs a) {
  __shared__ int64_t s_part[kBlock / 64][MDSX_MAX_COLUMNS];
  __shared__ uint32_t s_bad[kBlock / 64], s_big[kBlock / 64];
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int TR = a.tile_rows;
  const uint32_t tile = blockIdx.x * uint32_t(kBlock / TR) + uint32_t(t / TR);
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
  if (ok && few) h.template load<kNT>(v.shard + b, a.nvar);
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
      if (lane == 0) s_bad[wave] = bad != 0, s_big[wave] = big != 0;
      __syncthreads();
      tile_bad = false;
      for (int w = wave & ~(TR / 64 - 1); w < (wave & ~(TR / 64 - 1)) + TR / 64; ++w)
        tile_bad = tile_bad || s_bad[w], tile_big = tile_big || s_big[w];
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

// Huge rows (a sample larger than the row-parallel decode's stage), listed by it: one workgroup
// per row, straight from HBM (a separate launch, so the row-parallel kernel keeps its registers
// for the common case). Fixed and bytes columns are split over the four waves at 16-byte-aligned
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
    sample_range(v, v.r0 + t, &b, &e);  // checked by the row-parallel kernel before listing it
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
        d = uint64_t(col.offsets[row]);  // final (written by the row-parallel kernel)
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

}  // namespace

int launch_stage_totals(const DevArgs& a, bool nt, hipStream_t s) {
  const unsigned grid = unsigned((uint64_t(a.ntiles) * a.tile_rows + kBlock - 1) / kBlock);
  if (nt)
    hipLaunchKernelGGL(stage_totals_kernel<true>, dim3(grid), dim3(kBlock), 0, s, a);
  else
    hipLaunchKernelGGL(stage_totals_kernel<false>, dim3(grid), dim3(kBlock), 0, s, a);
  return hip_check(hipGetLastError(), "stage_totals_kernel launch");
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
