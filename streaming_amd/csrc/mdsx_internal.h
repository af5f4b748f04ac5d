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
const std::string& last_kernel_name();

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
  int stage_debug = 0;  // measurement only: parts of the row-parallel decode skipped (bits)
  int run_slots = 0;    // ragged plans: KiB of the streaming decode's per-wave LDS ring (0: off)
  int run_kb = 16;      // streaming decode: about this many KiB of samples per tile (tile sizing:
                        // runs of at most ~8 KiB; measured DESIGN.md §5, profiles/r03/run_size/)
  int64_t run_min = 3072;  // streaming decode for batches whose samples average >= this many bytes
  int run_nt = 0;          // streaming decode: non-temporal ring loads and stores (the lean path
                           // is faster with them; the general one alone was slower)
  int seg = 0;             // streaming decode: the lean path for clean runs of samples that fit
                           // the ring (seg_decode_kernel; others take the general path)
  int xcd_order = 3;       // bits: decodes whose XCDs each take a contiguous range of tiles
                           // (profiles/r03/xcd_order/): 1 the lean path (+3 % on config C), 2 the
                           // register decode (+1.1 % on config B); not 4, the row-parallel (-1 %)
  int rowwave = -1;        // all-fixed plans: one row per wave, this many waves per workgroup (0:
                           // decode_kernel; -1: 1 for rows of >= 3 KiB, else 0; MDSX_TUNE rw)
  int rowwave_occ = 6;     // ... registers bounded for this many waves per SIMD (MDSX_TUNE rwocc;
                           // 0: the compiler's choice, 85 VGPRs = 5 waves)
  int rowwave_rows = 1;    // ... rows per wave (MDSX_TUNE rwr: 1, 2, 4)
  int rowwave_x = 0;       // (measurement only) rowwave kX variants (MDSX_TUNE rwx, rwk)
  int rowwave_k = 0;
  int scan_nt = -1;        // the scan pass's head loads non-temporal (MDSX_TUNE snt; -1: for the
                           // row-parallel decode's batches)
  int lds_pad_kb = 0;      // dynamic LDS added per workgroup of the register and streaming decodes
                           // (KiB; MDSX_TUNE lpad): fewer workgroups per CU
  int seg_var = 0;         // lean path, measurement variants (MDSX_TUNE sv, bits; mdsx_run.hip)
  int seg_waves = 2;       // lean path: waves (runs) per workgroup (1, 2 or 4; 2: 18 waves per CU,
                           // +4 % on 3-5 KB samples, profiles/r03/seg_waves/)
  int rows_kb = 0;         // row-parallel decode of shorter samples: LDS stage in KiB (0: off,
                           // -1: sized per batch, rows_tile_rows / rows_stage_bytes)
  int rows_nt = 1;         // row-parallel decode: non-temporal loads and stores (measured faster)
  int rows_slack = 8;      // row-parallel decode: the stage holds (1 + 1/rows_slack) x a tile's
                           // average bytes (+ 1 KiB)
  int rows_occ = 0;        // row-parallel decode: waves per SIMD its registers are bounded for
                           // (4, 6 or 8; 0: 6 for stages up to 24 KiB -- short samples, +7 % --
                           // else 4)
  int rows_pipe = 0;       // row-parallel decode: tiles per workgroup, the next tile's DMA in
                           // flight while one is written (two stages; 0: one tile, one stage)
  int swave = -1;          // ragged batches of the streaming decode's sample sizes: one sample per
                           // one-wave workgroup, in registers, instead (mdsx_swave.hip; -1: when
                           // the samples average <= 4/5 of its register window, +3 % on config C,
                           // profiles/r06/swave/; 1: always; 0: never, MDSX_TUNE swave)
  int swave_kb = 6;        // ... KiB of a sample held in registers (4, 6 or 8; larger samples are
                           // copied straight from HBM)
  int swave_occ = 0;       // ... waves per SIMD its registers are bounded for (0: the compiler's;
                           // bounds that make it spill are not built: build.py refuses scratch)
  int swave_tile = 64;     // ... rows per tile (the scan pass's unit: 256 / this tiles per block)
  int swave_lds = 2048;    // ... bytes of its per-wave LDS copy of the columns past the first (a
                           // sample whose later columns span more takes the huge-row kernel)
  int swave_x = 0;         // ... measurement variants (MDSX_TUNE swx, bits; mdsx_swave.hip)
  int gather_chunks = 2;  // 16-byte chunks per lane in the ragged gather (tile = 4 KiB x this)
  int gather_min = 256;   // ragged columns averaging fewer bytes per row use the gather kernel
  int group_max = 1024;   // ... fewer than this (and >= gather_min): four rows per wave
  int64_t fixed_sum = 0;
  bool safe = true;
  mdsx::ColumnSpec cols[MDSX_MAX_COLUMNS];
};

// Whether a batch of `bytes` shard bytes and `rows` samples decodes through the streaming decode
// (mdsx_run.hip): ragged plans whose samples average at least run_min bytes (config C's 4.4 KB
// samples: 4.2 TB/s there vs 3.4 through the row-parallel decode; at 1.9 KB the row-parallel
// decode leads, 2.85 vs 2.26).
inline bool use_run_decode(const mdsx_plan* p, uint64_t bytes, uint64_t rows) {
  return p->nvar > 0 && p->run_slots > 0 && rows > 0 && bytes / rows >= uint64_t(p->run_min);
}

// Whether such a batch decodes one sample per wave instead (mdsx_swave.hip).
inline bool use_swave_decode(const mdsx_plan* p, uint64_t bytes, uint64_t rows) {
  if (p->swave == 0 || !use_run_decode(p, bytes, rows)) return false;
  return p->swave > 0 || bytes / rows <= uint64_t(p->swave_kb) * 1024 * 4 / 5;
}

// Whether a ragged batch of shorter samples decodes through the row-parallel decode
// (mdsx_rows.hip).
inline bool use_rows_decode(const mdsx_plan* p, uint64_t bytes, uint64_t rows) {
  return p->nvar > 0 && p->rows_kb != 0 && rows > 0 && !use_run_decode(p, bytes, rows);
}

// Row-parallel decode sizing. A workgroup's LDS: the stage, [ncols][tile rows] 16-byte value
// records, UTF-8 marks, one chunk map per ragged column, and the kernel's static arrays.
inline uint64_t rows_lds_bytes_est(const mdsx_plan* p, uint64_t stage, uint64_t tr) {
  const uint64_t nstage = p->rows_pipe > 0 ? 2 : 1;
  return 192 * nstage + stage * nstage + tr * uint64_t(p->ncols) * 16 + uint64_t(p->ncols) * 32 +
         uint64_t(p->nvar) * (stage / 16 + 4) + uint64_t(p->ncols) * 104 + 64;
}

// The stage a tile of tr samples of per_row bytes needs: (1 + 1/slack) of its average bytes plus
// 1 KiB (4..96 KiB; a tile that does not fit is decoded in windows). slack 8 by default.
inline uint64_t rows_auto_stage(uint64_t per_row, uint64_t tr, uint64_t slack = 8) {
  const uint64_t kb = (tr * per_row * (slack + 1) / slack + 1023) / 1024 + 1;
  return (kb < 4 ? 4 : kb > 96 ? 96 : kb) * 1024;
}

// Rows per tile: the largest power of two (<= 256) whose samples fill at most 8/9 of the target
// stage -- rows_kb, or by default 20 KiB for samples under 512 bytes (per-sample work dominates:
// five workgroups per CU) and 40 KiB above (three workgroups of larger tiles; measured)
// -- with the workgroup's LDS within the CU's 160 KiB.
inline int rows_tile_rows(const mdsx_plan* p, uint64_t per_row) {
  if (per_row == 0) per_row = 1;
  const uint64_t target = p->rows_kb > 0 ? uint64_t(p->rows_kb) * 1024
                                         : (per_row < 512 ? 20 : 40) * 1024ull;
  int tr = 1;
  while (tr < 256) {
    const uint64_t t2 = uint64_t(tr) * 2;
    const uint64_t stage = p->rows_kb > 0 ? target : rows_auto_stage(per_row, t2, p->rows_slack);
    if (t2 * per_row * 9 > target * 8 || rows_lds_bytes_est(p, stage, t2) > 160 * 1024) break;
    tr = int(t2);
  }
  return tr;
}

// The stage of a batch decoded in tiles of tr rows.
inline uint32_t rows_stage_bytes(const mdsx_plan* p, uint64_t per_row, int tr) {
  return p->rows_kb > 0 ? uint32_t(p->rows_kb) * 1024u
                        : uint32_t(rows_auto_stage(per_row ? per_row : 1, uint64_t(tr),
                                                   uint64_t(p->rows_slack)));
}
