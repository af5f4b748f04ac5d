// One sample's bytes decoded exactly as MDSReader.decode_sample slices them (gfx950):
// mdsx_decode_sample.
//
// The reference (streaming/base/format/mds/reader.py:103-126) reads the u32 size head of every
// variable column from data[idx:idx + 4] (a head cut short raises ValueError from numpy: `size, =
// np.frombuffer(...)`), then hands column c the slice data[idx:idx + size] -- a slice, so a head
// larger than what is left, or a sample shorter than its fixed columns, gives a SHORTER value, not
// an error; the column's decoder then returns it (bytes), decodes it (str: UnicodeDecodeError if
// the cut splits a sequence) or rejects it (numpy's frombuffer / reshape for int, scalars and static
// ndarrays). get_sample_data (mds/reader.py:128-149) already returns whatever the file holds in
// [begin, end). The whole-shard decodes check every sample and report the ones that do not fit
// (MDSX_E_BOUNDS): the per-sample path of a shard with such samples goes through here instead
// (streaming_amd/reader.py: get_item = decode_sample(get_sample_data(idx)), base/reader.py:310-320).
//
// One wave: lane c parses column c's head and size, a wave prefix places the columns, each
// column's clipped slice is copied (wave_copy) into `values`, packed in column order; meta gets
// (offset in values, clipped length) per column and a status word.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "mdsx_decode.h"
#include "mdsx_device.h"
#include "mdsx_internal.h"

namespace mdsx_kernels {
namespace {

struct SampleArgs {
  const uint8_t* data;  // the sample's first byte (the caller's buffer has 64 bytes of slack
                        // before and after it: the aligned loads of the copy)
  uint8_t* values;      // >= n bytes
  int64_t* meta;        // [2 ncols]: offset, clipped length; [2 ncols]: status
  uint32_t n;
  int32_t ncols;
  int32_t nvar;
  uint32_t row_bytes[MDSX_MAX_COLUMNS];
  int8_t var_index[MDSX_MAX_COLUMNS];
};

__global__ __launch_bounds__(64) void decode_sample_kernel(const SampleArgs a) {
  const int lane = threadIdx.x;
  const bool col = lane < a.ncols;
  const int vi = col ? a.var_index[lane] : -1;
  // the heads: data[4 vi : 4 vi + 4] (mds/reader.py:118)
  const bool short_head = vi >= 0 && 4ull * uint64_t(vi) + 4 > a.n;
  const uint64_t sm = __ballot(short_head);
  if (sm) {  // numpy raises at the first head (column order) cut short
    if (lane == 0) a.meta[2 * a.ncols] = 1 + __builtin_ctzll(sm);
    return;
  }
  const uint64_t size = !col ? 0 : vi >= 0 ? uint64_t(load_u32_any(a.data + 4u * uint32_t(vi)))
                                           : uint64_t(a.row_bytes[lane]);
  // column starts: 4 x nvar + the sizes before (mds/reader.py:122-125), then the slice's clip
  uint64_t incl = size;
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = uint64_t(__shfl_up(static_cast<unsigned long long>(incl), o));
    if (lane >= o) incl += y;
  }
  const uint64_t start = 4ull * uint64_t(a.nvar) + incl - size;
  const uint64_t s = start < a.n ? start : a.n;
  const uint64_t e = start + size < a.n ? start + size : a.n;
  const uint64_t len = e - s;
  uint64_t out = len;
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = uint64_t(__shfl_up(static_cast<unsigned long long>(out), o));
    if (lane >= o) out += y;
  }
  out -= len;
  if (col) {
    a.meta[2 * lane] = int64_t(out);
    a.meta[2 * lane + 1] = int64_t(len);
  }
  for (int c = 0; c < a.ncols; ++c) {  // uniform
    const uint64_t l = uint64_t(__shfl(static_cast<unsigned long long>(len), c));
    const uint64_t src = uint64_t(__shfl(static_cast<unsigned long long>(s), c));
    const uint64_t dst = uint64_t(__shfl(static_cast<unsigned long long>(out), c));
    if (l) wave_copy<false, 2, false>(a.data + src, a.values + dst, l, lane);
  }
  if (lane == 0) a.meta[2 * a.ncols] = 0;
}

}  // namespace
}  // namespace mdsx_kernels

using namespace mdsx_kernels;

extern "C" {

int mdsx_decode_sample(const mdsx_plan* plan, const uint8_t* d_data, uint32_t n, uint8_t* d_values,
                       int64_t* d_meta, void* stream) {
  if (!plan || !d_meta || (n > 0 && (!d_data || !d_values)))
    return mdsx::fail(MDSX_E_ARG, "mdsx_decode_sample: null argument");
  SampleArgs a;
  a.data = d_data;
  a.values = d_values;
  a.meta = d_meta;
  a.n = n;
  a.ncols = plan->ncols;
  a.nvar = plan->nvar;
  for (int c = 0; c < plan->ncols; ++c) {
    a.row_bytes[c] = uint32_t(plan->cols[c].row_bytes);
    a.var_index[c] = int8_t(plan->cols[c].var_index);
  }
  hipLaunchKernelGGL(decode_sample_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream),
                     a);
  return hip_check(hipGetLastError(), "decode_sample_kernel launch");
}

}  // extern "C"
