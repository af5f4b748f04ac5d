// MI355X kernels of the MDS shard ENCODER: the reverse byte shuffle of the
// decoder. Columns in the decoder's output layout (fixed rows, ragged values + int64 offsets)
// become MDS shard files, byte-identical to the reference writer's:
//
//   shard = u32 N | u32 offsets[N + 1] (absolute) | config JSON | samples,
//   sample = u32 size of every variable column (column order) | every column's bytes
//   (MDSWriter.encode_sample + encode_joint_shard, streaming/base/format/mds/writer.py:92-144).
//
//   encode_sizes_kernel    one row per lane: cum[i] = bytes of samples 0..i-1, computed
//                          elementwise from the ragged offsets (no scan needed); row lengths
//                          checked (0 <= len < 2^32, the u32 head).
//   encode_headers_kernel  one workgroup per shard: N, offsets[N], the config bytes.
//   encode_kernel          one workgroup per tile of rows: offsets-table entries, u32 heads and
//                          fixed columns of <= 16 bytes one row per lane; larger fixed columns and
//                          ragged rows one row per wave through the realigning wave copy (aligned
//                          16-byte stores, partial chunks at row ends one byte per lane).
//
// The shard split (base/writer.py:248-269: flush when size_limit < shard + sample + 4) is a
// greedy prefix rule over cum, decided on the host from cum (O(shards) binary searches); the
// kernels write into a batch laid out exactly like a decode batch, so an encoded batch is
// decodable in place.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>

#include "mdsx_device.h"
#include "mdsx_internal.h"

namespace mdsx_kernels {
namespace {

constexpr int kEncBlock = 256;

struct EncCol {
  const uint8_t* data;
  const int64_t* offsets;
  uint64_t bytes;  // size of data (bounds of the ragged offsets)
  uint32_t row_bytes;
  int32_t var_index;
  int32_t group;  // ragged rows averaging < 1 KiB: four rows per wave (group_copy)
  int32_t pad_;
};

struct EncArgs {
  uint8_t* batch;
  uint64_t batch_bytes;
  const mdsx_shard_desc* shards;
  const uint32_t* tile_shard;
  mdsx_status* status;
  int64_t* cum;
  const uint8_t* config;
  uint64_t rows;
  uint32_t config_bytes;
  uint32_t ntiles;
  int32_t nshards;
  int32_t ncols;
  int32_t nvar;
  int32_t tile_rows;
  int64_t per_row_fixed;  // sum of fixed row bytes + 4 per variable column (the heads)
  EncCol cols[MDSX_MAX_COLUMNS];
};

// Up to 16 bytes (a register copy of one small value) to any byte address.
__device__ __forceinline__ void store_small(uint8_t* dst, const uint4 v, uint32_t n) {
  const uint64_t a = reinterpret_cast<uint64_t>(dst);
  if (n == 4 && (a & 3) == 0) {
    *reinterpret_cast<uint32_t*>(dst) = v.x;
  } else if (n == 8 && (a & 7) == 0) {
    *reinterpret_cast<uint2*>(dst) = make_uint2(v.x, v.y);
  } else {
    for (uint32_t j = 0; j < n; ++j) dst[j] = uint8_t(byte_of(v, int(j)));
  }
}

// One small fixed value (<= 16 bytes, source row aligned to its size's largest power of two).
__device__ __forceinline__ uint4 load_small(const uint8_t* p, uint32_t n) {
  uint4 v = make_uint4(0, 0, 0, 0);
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  switch ((n == 4 || n == 8 || n == 16) && (a & (n - 1)) == 0 ? n : 0u) {
    case 4: v.x = *reinterpret_cast<const uint32_t*>(p); break;
    case 8: {
      const uint2 w = *reinterpret_cast<const uint2*>(p);
      v.x = w.x; v.y = w.y;
      break;
    }
    case 16: v = *reinterpret_cast<const uint4*>(p); break;
    default: {
      uint32_t w[4] = {0, 0, 0, 0};
      for (uint32_t j = 0; j < n; ++j) w[j >> 2] |= uint32_t(p[j]) << (8 * (j & 3));
      v = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
  return v;
}

__global__ __launch_bounds__(kEncBlock) void encode_sizes_kernel(const EncArgs a) {
  const uint64_t i = uint64_t(blockIdx.x) * kEncBlock + threadIdx.x;
  if (i > a.rows) return;
  int64_t c = int64_t(i) * a.per_row_fixed;
  for (int k = 0; k < a.ncols; ++k) {
    const EncCol& col = a.cols[k];
    if (col.var_index < 0) continue;
    const int64_t o = col.offsets[i];
    c += o - col.offsets[0];
    // monotone offsets inside [0, bytes] keep every row's bytes inside the values buffer
    bool bad = o < 0 || uint64_t(o) > col.bytes;
    if (i < a.rows) {
      const int64_t len = col.offsets[i + 1] - o;
      bad = bad || len < 0 || len > int64_t(0xffffffffll);
    }
    if (bad) report(a.status, MDSX_E_ARG, -1, int(i), k);
  }
  a.cum[i] = c;
}

// Facts of shard s every encode kernel re-derives (and checks) before writing.
struct EncShard {
  mdsx_shard_desc d;
  uint64_t hdr;   // 4 + 4 (N + 1) + config bytes: where sample 0 starts
  int64_t base;   // cum[row0]
  bool ok;
};

__device__ __forceinline__ EncShard enc_shard(const EncArgs& a, uint32_t s) {
  EncShard e;
  e.d = a.shards[s];
  e.hdr = 4ull + 4ull * (uint64_t(e.d.samples) + 1) + a.config_bytes;
  e.ok = e.d.row0 + e.d.samples <= a.rows && e.d.offset + e.d.bytes <= a.batch_bytes;
  e.base = e.ok ? a.cum[e.d.row0] : 0;
  if (e.ok) e.ok = e.hdr + uint64_t(a.cum[e.d.row0 + e.d.samples] - e.base) == e.d.bytes &&
                   e.d.bytes < (uint64_t(1) << 32);
  return e;
}

__global__ __launch_bounds__(kEncBlock) void encode_headers_kernel(const EncArgs a) {
  if (a.status->code != 0) return;  // bad columns (encode_sizes): write nothing
  const uint32_t s = blockIdx.x;
  const EncShard e = enc_shard(a, s);
  if (!e.ok) {
    if (threadIdx.x == 0) report(a.status, MDSX_E_HEADER, int(s), -1, -1);
    return;
  }
  uint8_t* file = a.batch + e.d.offset;
  if (threadIdx.x == 0) {
    reinterpret_cast<uint32_t*>(file)[0] = e.d.samples;
    reinterpret_cast<uint32_t*>(file)[1 + e.d.samples] = uint32_t(e.d.bytes);
  }
  uint8_t* cfg = file + 4 + 4 * (uint64_t(e.d.samples) + 1);
  for (uint32_t j = threadIdx.x; j < a.config_bytes; j += kEncBlock) cfg[j] = a.config[j];
}

template <int kUnroll, bool kNT>
__global__ __launch_bounds__(kEncBlock) void encode_kernel(const EncArgs a) {
  extern __shared__ uint32_t s_pos[];  // [ncols][tile_rows]: column start inside the file
  __shared__ int s_bad;
  const int t = threadIdx.x;
  const int lane = t & 63;
  const int wave = t >> 6;
  const int TR = a.tile_rows;
  if (a.status->code != 0) return;
  const uint32_t tile = blockIdx.x;
  const uint32_t s = a.tile_shard[tile];
  if (s >= uint32_t(a.nshards)) {
    if (t == 0) report(a.status, MDSX_E_ARG, int(s), -1, -1);
    return;
  }
  const EncShard e = enc_shard(a, s);
  if (!e.ok || tile < e.d.tile0) return;  // reported by encode_headers_kernel
  const uint64_t r0 = uint64_t(tile - e.d.tile0) * TR;
  if (r0 >= e.d.samples) return;
  const int nrows = int(min(uint64_t(TR), uint64_t(e.d.samples) - r0));
  uint8_t* file = a.batch + e.d.offset;
  if (t == 0) s_bad = 0;
  __syncthreads();
  if (t < nrows) {
    const uint64_t i = r0 + t;
    const uint64_t g = e.d.row0 + i;
    const uint64_t start = e.hdr + uint64_t(a.cum[g] - e.base);
    const uint64_t end = e.hdr + uint64_t(a.cum[g + 1] - e.base);
    reinterpret_cast<uint32_t*>(file + 4)[i] = uint32_t(start);
    uint64_t pos = start + 4ull * a.nvar;
    bool bad = end > e.d.bytes;
    for (int c = 0; c < a.ncols; ++c) {
      const EncCol& col = a.cols[c];
      uint64_t len = col.row_bytes;
      if (col.var_index >= 0) {
        len = uint64_t(col.offsets[g + 1] - col.offsets[g]);
        if (!bad && start + 4ull * (col.var_index + 1) <= end)
          store_small(file + start + 4ull * col.var_index, make_uint4(uint32_t(len), 0, 0, 0), 4);
      }
      s_pos[c * TR + t] = uint32_t(pos);
      pos += len;
    }
    if (bad || pos != end) {
      s_bad = 1;
      report(a.status, MDSX_E_ARG, int(s), int(i), -1);
    }
  }
  __syncthreads();
  if (s_bad) return;
  // fixed columns of <= 16 bytes: one row per lane
  if (t < nrows) {
    const uint64_t g = e.d.row0 + r0 + t;
    for (int c = 0; c < a.ncols; ++c) {
      const EncCol& col = a.cols[c];
      if (col.var_index >= 0 || col.row_bytes == 0 || col.row_bytes > 16) continue;
      const uint4 v = load_small(col.data + g * col.row_bytes, col.row_bytes);
      store_small(file + s_pos[c * TR + t], v, col.row_bytes);
    }
  }
  // larger fixed columns and ragged rows: one row per wave; medium ragged rows four per wave
  for (int c = 0; c < a.ncols; ++c) {
    const EncCol& col = a.cols[c];
    const bool var = col.var_index >= 0;
    if (!var && col.row_bytes <= 16) continue;
    if (var && col.group) {
      const int gi = lane >> 4;
      for (int q0 = wave * 4; q0 < nrows; q0 += kEncBlock / 16) {
        const int r = q0 + gi;
        const bool live = r < nrows;
        const uint64_t g = e.d.row0 + r0 + uint64_t(live ? r : 0);
        const int64_t b = live ? col.offsets[g] : 0;
        const uint64_t len = live ? uint64_t(col.offsets[g + 1] - b) : 0;
        group_copy<2, kNT, true>(col.data + b, file + (live ? s_pos[c * TR + r] : 0), len, lane);
      }
      continue;
    }
    for (int r = wave; r < nrows; r += kEncBlock / 64) {
      const uint64_t g = e.d.row0 + r0 + r;
      const uint8_t* src;
      uint64_t len;
      if (var) {
        const int64_t b = col.offsets[g];
        src = col.data + b;
        len = uint64_t(col.offsets[g + 1] - b);
      } else {
        src = col.data + g * col.row_bytes;
        len = col.row_bytes;
      }
      wave_copy<false, kUnroll, kNT, true, true>(src, file + s_pos[c * TR + r], len, lane);
    }
  }
}

bool fill_args(const mdsx_plan* plan, const mdsx_column_in* cols, uint64_t rows, EncArgs* a) {
  std::memset(a, 0, sizeof(*a));
  a->rows = rows;
  a->ncols = plan->ncols;
  a->nvar = plan->nvar;
  a->tile_rows = plan->encode_tile_rows;
  int64_t fixed = 0;
  for (int c = 0; c < plan->ncols; ++c) {
    const mdsx::ColumnSpec& spec = plan->cols[c];
    EncCol& d = a->cols[c];
    d.data = static_cast<const uint8_t*>(cols[c].data);
    d.offsets = cols[c].offsets;
    d.bytes = cols[c].bytes;
    d.var_index = spec.var_index;
    if (spec.var_index >= 0) {
      if (!d.offsets || (rows && !d.data)) return false;
      d.group = rows && d.bytes < uint64_t(1024) * rows;
    } else {
      d.row_bytes = uint32_t(spec.row_bytes);
      fixed += spec.row_bytes;
      if (rows && spec.row_bytes && (!d.data || d.bytes < rows * uint64_t(spec.row_bytes)))
        return false;
    }
  }
  a->per_row_fixed = fixed + 4ll * plan->nvar;
  return true;
}

}  // namespace
}  // namespace mdsx_kernels

using namespace mdsx_kernels;

uint64_t mdsx_encode_workspace_bytes(void) { return 256; }

int mdsx_encode_sizes(const mdsx_plan* plan, const mdsx_column_in* cols, uint64_t rows,
                      int64_t* d_cum, void* d_workspace, uint64_t workspace_bytes,
                      void* stream) {
  if (!plan || !d_cum || !d_workspace || (plan->ncols && !cols))
    return mdsx::fail(MDSX_E_ARG, "mdsx_encode_sizes: null argument");
  if (workspace_bytes < mdsx_encode_workspace_bytes())
    return mdsx::fail(MDSX_E_ARG, "mdsx_encode_sizes: workspace too small");
  EncArgs a;
  if (!fill_args(plan, cols, rows, &a))
    return mdsx::fail(MDSX_E_ARG, "mdsx_encode_sizes: null data/offsets or short data for a column");
  a.status = static_cast<mdsx_status*>(d_workspace);
  a.cum = d_cum;
  hipStream_t s = static_cast<hipStream_t>(stream);
  int rc = hip_check(hipMemsetAsync(d_workspace, 0, sizeof(mdsx_status), s), "hipMemsetAsync");
  if (rc) return rc;
  const unsigned grid = unsigned((rows + 1 + kEncBlock - 1) / kEncBlock);
  hipLaunchKernelGGL(encode_sizes_kernel, dim3(grid), dim3(kEncBlock), 0, s, a);
  return hip_check(hipGetLastError(), "encode_sizes_kernel launch");
}

int mdsx_encode_shards(const mdsx_plan* plan, const mdsx_batch* batch, const mdsx_column_in* cols,
                       const int64_t* d_cum, const uint8_t* d_config, uint32_t config_bytes,
                       void* d_workspace, uint64_t workspace_bytes, void* stream) {
  if (!plan || !batch || !batch->data || !batch->shards || batch->nshards <= 0 || !d_cum ||
      !d_workspace || (config_bytes && !d_config) || (plan->ncols && !cols))
    return mdsx::fail(MDSX_E_ARG, "mdsx_encode_shards: null argument or empty batch");
  if (batch->ntiles && !batch->tile_shard)
    return mdsx::fail(MDSX_E_ARG, "mdsx_encode_shards: null tile table");
  if (workspace_bytes < mdsx_encode_workspace_bytes())
    return mdsx::fail(MDSX_E_ARG, "mdsx_encode_shards: workspace too small");
  EncArgs a;
  if (!fill_args(plan, cols, batch->rows, &a))
    return mdsx::fail(MDSX_E_ARG, "mdsx_encode_shards: null data/offsets or short data for a column");
  a.batch = const_cast<uint8_t*>(batch->data);  // the encoder writes the batch it is given
  a.batch_bytes = batch->bytes;
  a.shards = batch->shards;
  a.tile_shard = batch->tile_shard;
  a.status = static_cast<mdsx_status*>(d_workspace);
  a.cum = const_cast<int64_t*>(d_cum);
  a.config = d_config;
  a.config_bytes = config_bytes;
  a.ntiles = batch->ntiles;
  a.nshards = batch->nshards;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(encode_headers_kernel, dim3(unsigned(batch->nshards)), dim3(kEncBlock), 0,
                     s, a);
  int rc = hip_check(hipGetLastError(), "encode_headers_kernel launch");
  if (rc || batch->ntiles == 0) return rc;
  const size_t lds = size_t(plan->ncols) * plan->encode_tile_rows * sizeof(uint32_t);
  if (plan->nontemporal)
    hipLaunchKernelGGL((encode_kernel<4, true>), dim3(batch->ntiles), dim3(kEncBlock), lds, s, a);
  else
    hipLaunchKernelGGL((encode_kernel<4, false>), dim3(batch->ntiles), dim3(kEncBlock), lds, s, a);
  return hip_check(hipGetLastError(), "encode_kernel launch");
}
