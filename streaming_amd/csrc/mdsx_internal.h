// Internal declarations shared by the host plan builder and the HIP kernels of libmdsx.so.
#pragma once

#include <cstdint>
#include <string>

#include "../../include/mdsx.h"

namespace mdsx {

// What the encoding string means (independent of the index's fixed/variable layout).
enum Semantic : int {
  SEM_BYTES = 0,          // 'bytes'
  SEM_STR = 1,            // 'str'
  SEM_SCALAR = 2,         // 'int', uint8..float64
  SEM_NDARRAY_STATIC = 3, // 'ndarray:<dtype>:<shape>'
  SEM_NDARRAY_DYN = 4,    // 'ndarray', 'ndarray:', 'ndarray:<dtype>'
  SEM_HOST_OBJECT = 5,    // pil, jpeg, png, list[*], jpeg_array, pkl, json, str_* (host decode)
};

struct ColumnSpec {
  std::string encoding;
  int semantic = SEM_BYTES;
  int kind = MDSX_KIND_BYTES;  // device layout class (from the index's column_sizes)
  int64_t row_bytes = 0;       // fixed size from the index, 0 for variable columns
  int64_t natural_size = -1;   // fixed size implied by the encoding, -1 if variable
  int elem_bytes = 1;          // dtype itemsize (1 for byte-like)
  int var_index = -1;          // position among the variable columns (head order), -1 if fixed
};

int fail(int code, const std::string& msg);
// Template name of the last decode kernel this thread launched (mdsx_last_kernel).
void set_last_kernel(const std::string& name);

}  // namespace mdsx

struct mdsx_plan {
  int ncols = 0;
  int nvar = 0;
  int tile_rows = 256;
  int encode_tile_rows = 16;  // rows per workgroup of the encode kernel
  int unroll = 0;       // 16-byte chunks per lane in flight in the row copy (2, 4 or 6); 0 =
                        // chosen per launch from the row sizes (mdsx_decode_shards)
  int nontemporal = 0;  // non-temporal loads/stores in the row copy
  int str_cached = 0;   // medium str rows stored temporally (the UTF-8 re-read then hits L2)
  int ring_slots = 0;   // long ragged rows through a per-wave LDS-DMA ring of this many KiB (0: off)
  int stage_kb = 0;     // ragged plans: LDS stage of the staged decode in KiB (0: register copy)
  int stage_tiles = 0;  // tiles per workgroup of the staged decode (0: per launch)
  int stage_debug = 0;  // measurement only: parts of the staged decode skipped (bits)
  int stage_fill = 70;  // percent of a stage buffer a tile's samples fill on average (tile sizing)
  int run_slots = 0;    // ragged plans: KiB of the streaming decode's per-wave LDS ring (0: off)
  int run_kb = 32;      // streaming decode: about this many KiB of samples per tile (tile sizing)
  int64_t run_min = 2048;  // streaming decode for batches whose samples average >= this many bytes
  int run_nt = 0;          // streaming decode: non-temporal ring loads and stores (measured: the
                           // temporal ones let L2 merge the partial stores at run edges)
  int rows_kb = 0;         // row-parallel decode of short samples: LDS stage in KiB (0: off)
  int rows_nt = 0;         // row-parallel decode: non-temporal loads and stores
  int gather_chunks = 2;  // 16-byte chunks per lane in the ragged gather (tile = 4 KiB x this)
  int gather_min = 256;   // ragged columns averaging fewer bytes per row use the gather kernel
  int group_max = 1024;   // ... fewer than this (and >= gather_min): four rows per wave
  int64_t fixed_sum = 0;
  bool safe = true;
  mdsx::ColumnSpec cols[MDSX_MAX_COLUMNS];
};

// Whether a batch of `bytes` shard bytes and `rows` samples decodes through the streaming decode
// (mdsx_run.hip): ragged plans whose samples average at least run_min bytes (config C's 4.4 KB
// samples: 4.76 vs 4.70 TB/s, 1.02x vs 1.15x traffic; short and medium rows stay on the
// register decode, measured 2x and 1.3x faster there).
inline bool use_run_decode(const mdsx_plan* p, uint64_t bytes, uint64_t rows) {
  return p->nvar > 0 && p->run_slots > 0 && rows > 0 && bytes / rows >= uint64_t(p->run_min);
}

// Whether a ragged batch of shorter samples decodes through the row-parallel decode
// (mdsx_rows.hip).
inline bool use_rows_decode(const mdsx_plan* p, uint64_t bytes, uint64_t rows) {
  return p->nvar > 0 && p->rows_kb > 0 && rows > 0 && !use_run_decode(p, bytes, rows);
}
