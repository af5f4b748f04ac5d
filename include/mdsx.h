/*
 * mdsx.h — C ABI of the MI355X-native MDS shard decoder (libmdsx.so).
 *
 * This is the drop-in boundary for ONE hot path of mosaicml/streaming: the per-sample MDS decode
 * path under streaming/base (offsets-table scan, per-sample byte-range gather, per-column decode).
 * Every entry point below names the reference interface it replaces (paths relative to the
 * mosaicml/streaming repository root).
 *
 * Conventions
 *   - Plain C: pointers, sizes, ints. No torch / HIP C++ types in signatures; `stream` is a
 *     hipStream_t passed as void* (NULL = the default stream).
 *   - The library NEVER allocates or frees device memory and keeps no pointer after a call returns.
 *     The caller (the Python host layer, through the PyTorch caching allocator) owns the shard
 *     batch buffer, the descriptor tables, every output buffer and the workspace.
 *   - All device work is enqueued on `stream`; calls return once it is enqueued. Errors found by
 *     the kernels (malformed shards) are written to the mdsx_status record at the start of the
 *     workspace and read by the caller after the stream completes.
 *   - Functions are reentrant. The only global state is a thread-local last-error string.
 *
 * Return codes: MDSX_OK (0) or a negative MDSX_E_* value; mdsx_last_error() gives the message.
 */
#ifndef MDSX_H_
#define MDSX_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- return / status codes ------------------------------------------------------------------ */
#define MDSX_OK 0
#define MDSX_E_ARG (-1)      /* bad argument (null pointer, size mismatch, too many columns)        */
#define MDSX_E_ENCODING (-2) /* unsupported encoding string (encodings.py:697-714,770-772)      */
#define MDSX_E_HEADER (-3)   /* shard header inconsistent: num_samples != index `samples`, offsets
                                table past the file, offsets[N] != file size (mds/writer.py:133-144) */
#define MDSX_E_BOUNDS (-4)   /* a sample or column byte range leaves its sample / shard
                                (mds/reader.py:103-149 would slice short or raise)                 */
#define MDSX_E_HIP (-5)      /* a HIP runtime call failed                                         */
#define MDSX_E_CAPACITY (-6) /* a ragged output buffer is smaller than the bytes to be written     */
#define MDSX_E_EMPTY (-7)    /* a sample has zero bytes: reference raises IndexError
                                (mds/reader.py:145-148)                                            */

/* ---- column kinds (what the device does with a column) -------------------------------------- */
#define MDSX_KIND_FIXED 0 /* fixed-size column: int, uint8..float64, ndarray:<dtype>:<shape>.
                             Output: row-major [rows, row_bytes] bytes (a dtype[rows, *shape]
                             tensor). encodings.py:84-94,148-161,270-305,308-397                   */
#define MDSX_KIND_BYTES 1 /* variable-size raw bytes (encodings.py:62-70). Also used for every
                             encoding whose decoded value is a host Python object (pil, jpeg, png,
                             list[*], jpeg_array, pkl, json, str_int/_float/_decimal,
                             encodings.py:410-650): the device gathers the bytes, the host applies
                             the reference semantics.                                               */
#define MDSX_KIND_STR 2   /* variable-size UTF-8 text (encodings.py:73-81). Ragged bytes plus a
                             per-row flag set where bytes.decode('utf-8') would raise.               */
#define MDSX_KIND_NDARRAY 3 /* dynamic ndarray ('ndarray', 'ndarray:<dtype>'; encodings.py:97-305):
                             ragged bytes of the whole encoded value (header + values); the host
                             splits the small header.                                               */

#define MDSX_MAX_COLUMNS 64

typedef struct mdsx_plan mdsx_plan; /* opaque, host-side, immutable after creation               */

/* One shard of a device batch (see mdsx_batch). */
typedef struct mdsx_shard_desc {
  uint64_t offset;  /* byte offset of the shard file inside the batch buffer (multiple of 256)   */
  uint64_t bytes;   /* shard file size: index.json raw_data.bytes                               */
  uint64_t row0;    /* first output row of this shard in the batch                              */
  uint32_t samples; /* index.json `samples` (checked against the file header)                   */
  uint32_t tile0;   /* first tile of this shard in the batch's tile numbering                   */
} mdsx_shard_desc;

#define MDSX_BATCH_PAD 256

/* Output of one column. Device pointers. */
typedef struct mdsx_column_out {
  void* data;         /* FIXED: rows*row_bytes bytes. var kinds: packed values (uint8)          */
  int64_t* offsets;   /* var kinds: int64[rows + 1] byte offsets into data. NULL for FIXED      */
  uint8_t* flags;     /* STR: uint8[rows], 1 = invalid UTF-8 (decode would raise). Else NULL     */
  uint64_t capacity;  /* var kinds: bytes available at data (checked against the scanned total) */
} mdsx_column_out;

/* Error record at byte 0 of the workspace (zeroed by every scan/decode call). */
typedef struct mdsx_status {
  int32_t code;   /* 0 or the first MDSX_E_* found by a kernel                                  */
  int32_t shard;  /* batch shard index of that error                                            */
  int32_t row;    /* sample index inside the shard (-1: shard header)                           */
  int32_t column; /* column index (-1: whole sample)                                            */
} mdsx_status;

/* ---- version / diagnostics ------------------------------------------------------------------ */
const char* mdsx_version(void);
const char* mdsx_last_error(void); /* thread-local message of the last failing call            */
/* Template name of the decode kernel the calling thread's last mdsx_decode_shards(_single) call
 * launched, as rocprofv3 reports it (e.g. "decode_kernel<4, true, false, false, false, 0>"):
 * ties a measured launch to the kernel its profile names. Not part of the reference interface. */
const char* mdsx_last_kernel(void);

/* ---- plan: per-shard schema ------------------------------------------------------------------
 * Replaces the per-sample encoding dispatch: mds_decode -> _get_coder (encodings.py:697-714,
 * 760-773) and NDArray.from_str / _get_static_size (encodings.py:148-193), which the reference
 * re-parses for every column of every sample. Built once per schema from the shard's index.json
 * entry as read by MDSReader.from_json (mds/reader.py:59-86): column_encodings and column_sizes
 * (sizes: a positive byte count for fixed columns; 0 or negative for variable columns, mirroring
 * the `if size:` test of mds/reader.py:114). */
int mdsx_plan_create(const char* const* encodings, const int64_t* column_sizes, int ncols,
                     mdsx_plan** out);
void mdsx_plan_destroy(mdsx_plan* plan);
int mdsx_plan_num_columns(const mdsx_plan* plan);
int mdsx_plan_num_var(const mdsx_plan* plan);
/* Rows per tile for this schema (all-fixed plans: about 32 KiB of rows, >= 4; ragged plans: 32).
 * Tile t of shard s covers rows
 * [(t - tile0) * tile_rows, ...) of that shard; a shard has ceil(samples / tile_rows) tiles. */
int mdsx_plan_tile_rows(const mdsx_plan* plan);
/* Rows per tile the decoder wants for a batch of `rows` samples in `shard_bytes` bytes of shard
 * files (set as mdsx_batch.tile_rows and used to build its tile table), a power of two. Ragged
 * plans, by the decode the batch gets: samples averaging >= 3 KiB (streaming decode) about
 * 32 KiB of samples per tile, 1..32 rows; shorter ones (row-parallel decode) up to 256 rows
 * filling ~8/9 of a 20 KiB (samples < 512 B) or 40 KiB LDS stage; all-fixed plans:
 * mdsx_plan_tile_rows. */
int mdsx_plan_tile_rows_for(const mdsx_plan* plan, uint64_t shard_bytes, uint64_t rows);
/* Rows per tile of the encoder's batches (mdsx_encode_shards): its tile table is built with
 * this, not with mdsx_plan_tile_rows. */
int mdsx_plan_encode_tile_rows(const mdsx_plan* plan);
/* kind (MDSX_KIND_*), bytes per row for FIXED (0 for var), element size in bytes (dtype size;
 * 1 for byte-like kinds). */
int mdsx_plan_column(const mdsx_plan* plan, int col, int* kind, int64_t* row_bytes,
                     int* elem_bytes);
/* MDSReader.validate (mds/reader.py:88-101) + is_mds_encoding_safe (encodings.py:730-739):
 * returns 1 if every column is safe ('pkl' is not), 0 otherwise. */
int mdsx_plan_is_safe(const mdsx_plan* plan);

/* A device batch: one device buffer holding several shard files (each at a 256-byte-aligned
 * offset, at least MDSX_BATCH_PAD bytes of readable slack before the first and after the last
 * shard) plus its descriptor and tile tables. Host struct; the pointers are device pointers. */
typedef struct mdsx_batch {
  const uint8_t* data;            /* batch buffer                                                */
  uint64_t bytes;                 /* its size in bytes                                           */
  const mdsx_shard_desc* shards;  /* nshards descriptors                                         */
  const uint32_t* tile_shard;     /* ntiles entries: the shard of each tile. Tiles never cross
                                     shards: shard s owns tiles [tile0, tile0 + ceil(samples /
                                     tile_rows)) and tile t covers rows (t - tile0) * tile_rows.. */
  int32_t nshards;
  uint32_t ntiles;
  uint64_t rows;                  /* rows of the batch (sum of samples)                          */
  uint32_t tile_rows;             /* rows per tile of this batch's tile table (a power of two
                                     <= 256); 0 = mdsx_plan_tile_rows(plan)                       */
  uint32_t reserved;
} mdsx_batch;

/* ---- workspace ----------------------------------------------------------------------------- */
/* Bytes of device workspace (256-byte aligned) the scan and decode of `batch` need: the status
 * record, per-tile ragged sums, per-row source addresses and the gather-tile row map of every
 * ragged column. */
uint64_t mdsx_workspace_bytes(const mdsx_plan* plan, const mdsx_batch* batch);

/* ---- the hot path ---------------------------------------------------------------------------
 * Pass 1. Resets the status record in the workspace (for an all-fixed plan that is all it
 * does), then, for variable-size columns, replaces the per-sample head parse of
 * MDSReader.decode_sample (mds/reader.py:111-118) and the offsets-table read of
 * MDSReader.get_sample_data (mds/reader.py:128-149), over whole shards: reads offsets[] and every
 * sample's u32 size head, checks the ranges, and writes, for every ragged column, per-row local
 * offsets into outs[c].offsets (int64[rows + 1]; made final by pass 2) and the column total
 * (d_totals[v] for the v-th variable column, int64, device; outs[c].offsets[rows] as well) so
 * the caller can size the value buffers.
 *   outs        : HOST array of plan->ncols column outputs (device pointers inside); only
 *                 .offsets of variable columns is used by this pass
 *   d_workspace : device scratch of at least mdsx_workspace_bytes(plan, batch) bytes
 *   d_totals    : device int64[num_var] (may be NULL)                                          */
int mdsx_scan_shards(const mdsx_plan* plan, const mdsx_batch* batch, const mdsx_column_out* outs,
                     void* d_workspace, uint64_t workspace_bytes, int64_t* d_totals,
                     void* stream);

/* Pass 2. Replaces MDSReader.get_sample_data + decode_sample + mds_decode for every sample of
 * every shard in the batch (mds/reader.py:103-149, encodings.py:62-397,760-773): gathers each
 * column's bytes of every sample into its output -- fixed columns as dtype rows, ragged columns
 * as packed values at the final offsets -- and flags the str rows that are not well-formed UTF-8
 * (where the reference's bytes.decode('utf-8') raises). outs[c].capacity of a ragged column must
 * be at least its scanned total. mdsx_scan_shards must have run on the same stream with the same
 * batch and workspace (every plan: it resets the status record this pass reports into). */
int mdsx_decode_shards(const mdsx_plan* plan, const mdsx_batch* batch,
                       const mdsx_column_out* outs, void* d_workspace, uint64_t workspace_bytes,
                       void* stream);

/* Single-pass decode: passes 1 and 2 in one launch sequence, with no host round trip for the
 * totals. The register decode's tiles scan their own ragged lengths and find their bases by
 * decoupled look-back over the tiles before them (tiles are taken in dispatch order from a
 * ticket); streaming and row-parallel batches run their scan pass and decode back to back on the
 * stream (a look-back across their ~1000 tiles in flight measured slower than the scan pass).
 * Ragged outputs are sized BEFORE the totals are known: outs[c].capacity of a ragged
 * column is its allocation (an upper bound such as the batch's sample bytes); a column that
 * needs more reports MDSX_E_CAPACITY. offsets[rows] and d_totals (device int64[num_var], may be
 * NULL) receive the totals. Same outputs as mdsx_scan_shards + mdsx_decode_shards.
 *   mode_bytes : host uint64[num_columns] (may be NULL): the expected bytes of each ragged column
 *                (e.g. the previous batch's totals). It only picks the copy mode and the grid of
 *                the destination-major copy -- a wrong guess is slower, never wrong; NULL uses
 *                the capacities. Replaces the same reader path as the two passes. */
int mdsx_decode_shards_single(const mdsx_plan* plan, const mdsx_batch* batch,
                              const mdsx_column_out* outs, const uint64_t* mode_bytes,
                              void* d_workspace, uint64_t workspace_bytes, int64_t* d_totals,
                              void* stream);

/* One sample, exactly as MDSReader.decode_sample slices it (mds/reader.py:103-126): the per-sample
 * path for samples the whole-shard decodes report (a head larger than the sample, a sample shorter
 * than its fixed columns), where the reference clips each column's slice instead of raising.
 *   d_data   : device, the n bytes get_sample_data returned (mds/reader.py:128-149), with 64
 *              readable bytes before and after them
 *   d_values : device uint8[>= n]: every column's clipped slice, packed in column order
 *   d_meta   : device int64[2 ncols + 1]: per column (offset in d_values, clipped length), then a
 *              status: 0, or 1 + c when column c's u32 size head is cut short (the reference's
 *              ValueError from np.frombuffer; the per-column entries are then not written)
 * The caller applies each column's decoder to its slice (a short int / scalar / static ndarray
 * raises there, as numpy does in the reference). */
int mdsx_decode_sample(const mdsx_plan* plan, const uint8_t* d_data, uint32_t n, uint8_t* d_values,
                       int64_t* d_meta, void* stream);

/* ---- batch gather by sample id ---------------------------------------------
 * out[k] = column[idx[k]] over already-decoded columns: the device side of the reference's
 * per-sample iteration over a worker's sample ids (StreamingDataset.__iter__ ->
 * _each_sample_id -> get_item, dataset.py:1430-1473,1237-1293). idx: device int64[m] of rows of
 * the decoded batch (no -1 padding: the reference skips those ids). The caller zeroes the
 * 16-byte status record at the start of the workspace before a gather sequence; out-of-range
 * ids report MDSX_E_BOUNDS there. Ragged columns: mdsx_gather_ragged_scan writes dst_offsets
 * (int64[m + 1]) and the total (d_total, device int64, may be NULL), then
 * mdsx_gather_ragged_copy (same idx, workspace and stream) copies the values (and str flags). */
uint64_t mdsx_gather_workspace_bytes(uint64_t m);
int mdsx_gather_fixed(const void* src, uint64_t src_rows, uint64_t row_bytes, const int64_t* idx,
                      uint64_t m, void* dst, void* d_workspace, uint64_t workspace_bytes,
                      void* stream);
int mdsx_gather_ragged_scan(const int64_t* src_offsets, uint64_t src_rows, const int64_t* idx,
                            uint64_t m, int64_t* dst_offsets, void* d_workspace,
                            uint64_t workspace_bytes, int64_t* d_total, void* stream);
int mdsx_gather_ragged_copy(const uint8_t* src_values, const int64_t* src_offsets,
                            const uint8_t* src_flags, uint64_t src_rows, const int64_t* idx,
                            uint64_t m, uint8_t* dst_values, uint64_t dst_capacity,
                            int64_t* dst_offsets, uint8_t* dst_flags, void* d_workspace,
                            uint64_t workspace_bytes, void* stream);

/* Multi-source gather: one batch over the decoded columns of many shards in one launch sequence
 * per column, rows in the caller's order -- StreamingDataset.__iter__'s get_item over a worker's
 * ids (dataset.py:1430-1473, 1237-1293), whose Spanner lookup (spanner.py:40-59) gives each id's
 * shard and row. srcs: DEVICE array of nsrc sources (one decoded column of one shard each);
 * idx: device int64[m], each source << MDSX_GATHER_SRC_SHIFT | row. Same workspace, status,
 * scan/copy sequence and errors as the single-source calls above (an id whose source or row is
 * out of range reports MDSX_E_BOUNDS). As there, a ragged column's copy reads the tile prefixes
 * its scan left in the workspace: scan another column in between only on another workspace. */
#define MDSX_GATHER_SRC_SHIFT 40
typedef struct mdsx_gather_src {
  const void* values;      /* fixed: rows x row_bytes; ragged: packed values                    */
  const int64_t* offsets;  /* ragged: rows + 1 offsets into values; NULL for fixed columns      */
  const uint8_t* flags;    /* str: per-row invalid-UTF-8 flags, or NULL                         */
  uint64_t rows;
} mdsx_gather_src;
int mdsx_gather_fixed_multi(const mdsx_gather_src* srcs, uint32_t nsrc, uint64_t row_bytes,
                            const int64_t* idx, uint64_t m, void* dst, void* d_workspace,
                            uint64_t workspace_bytes, void* stream);
int mdsx_gather_ragged_scan_multi(const mdsx_gather_src* srcs, uint32_t nsrc, const int64_t* idx,
                                  uint64_t m, int64_t* dst_offsets, void* d_workspace,
                                  uint64_t workspace_bytes, int64_t* d_total, void* stream);
int mdsx_gather_ragged_copy_multi(const mdsx_gather_src* srcs, uint32_t nsrc, const int64_t* idx,
                                  uint64_t m, uint8_t* dst_values, uint64_t dst_capacity,
                                  int64_t* dst_offsets, uint8_t* dst_flags, void* d_workspace,
                                  uint64_t workspace_bytes, void* stream);

/* ---- dynamic ndarray columns ------------------------------------------------------------------
 * Header parse of NDArray.decode (encodings.py:270-305) over a decoded MDSX_KIND_NDARRAY column
 * (values with headers + offsets): per row the value dtype id (encodings.py:131-143; dtype_id
 * is the static one of 'ndarray:<dtype>' or 0 for 'ndarray'), ndim, byte offset of the values
 * inside `values`, element count, and out_bad = 1 where the reference's decode raises (unknown
 * dtype, header past the row, value bytes != numel x itemsize). d_max_ndim (device int32, may
 * be NULL) receives the largest ndim by atomicMax (caller zeroes it). mdsx_ndarray_shapes
 * writes the shapes as int64[rows, shape_cols], padded with 1. */
int mdsx_ndarray_meta(const uint8_t* values, const int64_t* offsets, uint64_t rows, int dtype_id,
                      uint8_t* out_dtype, uint8_t* out_ndim, int64_t* out_data_offset,
                      int64_t* out_numel, uint8_t* out_bad, int32_t* d_max_ndim, void* stream);
int mdsx_ndarray_shapes(const uint8_t* values, const int64_t* offsets, uint64_t rows,
                        int dtype_id, int32_t shape_cols, int64_t* out_shape, void* stream);

/* ---- shard encode (MDSWriter on the device) ----------------------------------------------------
 * The reverse of the decode: columns in the decoder's output layout -> MDS shard files,
 * byte-identical to the reference writer's. Replaces MDSWriter.encode_sample +
 * encode_joint_shard (streaming/base/format/mds/writer.py:92-144) for whole batches; the shard
 * split of Writer.write (streaming/base/format/base/writer.py:248-269) is decided by the caller
 * from the cumulative sample sizes (a greedy prefix rule, O(shards) binary searches). */
typedef struct mdsx_column_in {
  const void* data;        /* fixed: rows x row_bytes (row-major); variable: packed values */
  const int64_t* offsets;  /* variable: rows + 1 offsets into data (offsets[0] may be > 0);
                              fixed: NULL */
  uint64_t bytes;          /* size of data: bounds the variable offsets / fixed rows */
  uint64_t reserved;
} mdsx_column_in;

/* Workspace of the encode calls (status record at offset 0). */
uint64_t mdsx_encode_workspace_bytes(void);
/* d_cum (device int64[rows + 1]): cum[i] = bytes of samples 0..i-1 (heads included, the 4-byte
 * offsets-table entry not). Checks every variable column (monotone offsets inside [0, bytes],
 * lengths < 2^32: the u32 head) into the status record, which this call resets. */
int mdsx_encode_sizes(const mdsx_plan* plan, const mdsx_column_in* cols, uint64_t rows,
                      int64_t* d_cum, void* d_workspace, uint64_t workspace_bytes, void* stream);
/* Write every shard of `batch` (laid out as for decoding: shard s holds rows
 * [row0, row0 + samples) and must be exactly 4 + 4 (samples + 1) + config_bytes +
 * cum[row0 + samples] - cum[row0] bytes) into batch->data, which this call writes. d_config:
 * the shard config JSON (device). Does nothing if the status record already holds an error;
 * inconsistent descriptors are reported as MDSX_E_HEADER, never written through. */
int mdsx_encode_shards(const mdsx_plan* plan, const mdsx_batch* batch, const mdsx_column_in* cols,
                       const int64_t* d_cum, const uint8_t* d_config, uint32_t config_bytes,
                       void* d_workspace, uint64_t workspace_bytes, void* stream);

/* ---- shard-file hashing on the device ------------------------------------------
 * The xxHash digests the reference records per shard file in index.json (Writer._write_file,
 * streaming/base/format/base/writer.py:197-200, via get_hash, streaming/base/hashing.py:55-68)
 * and recomputes over the whole file to validate it (Stream._decompress_shard_part /
 * _prepare_shard_part, streaming/base/stream.py:333-340,403-411), computed over byte ranges
 * already resident in device memory. Algorithm ids name python-xxhash 3.x functions (xxHash
 * 0.8.2); `seed` is their `seed=` argument (the reference uses 0). hashlib algorithms stay on
 * the host. */
#define MDSX_HASH_XXH32 1
#define MDSX_HASH_XXH64 2
#define MDSX_HASH_XXH3_64 3
#define MDSX_HASH_XXH3_128 4 /* also xxhash.xxh128 */

typedef struct mdsx_segment {
  uint64_t offset; /* byte offset inside `data` (multiple of 16)                                 */
  uint64_t bytes;  /* length                                                                     */
} mdsx_segment;

/* Workspace for hashing `nseg` segments totalling `total_segment_bytes` (status record at 0). */
uint64_t mdsx_hash_workspace_bytes(int nseg, uint64_t total_segment_bytes);
/* Digest of every segment of `data` (device, 16-byte aligned) into d_digests (device
 * uint64[2 * nseg]: the hash value's low 64 bits, then its high 64 bits -- 0 except for
 * xxh3_128; xxh32 values are in the low 32 bits). d_segs: device table of nseg segments.
 * A segment outside [0, data_bytes) or not 16-byte aligned is reported as MDSX_E_BOUNDS in the
 * status record (and no digest is written); a workspace too small for the segments' 1 KiB
 * blocks as MDSX_E_CAPACITY. */
int mdsx_hash_segments(int algo, uint64_t seed, const uint8_t* data, uint64_t data_bytes,
                       const mdsx_segment* d_segs, int nseg, uint64_t* d_digests,
                       void* d_workspace, uint64_t workspace_bytes, void* stream);

/* ---- diagnostics ---------------------------------------------------------------------------
 * HBM roofline probe: a streaming 16-byte-per-lane device-to-device copy of `bytes` (multiple of
 * 16, 16-byte aligned pointers) on `stream`. Not part of the decode path: it measures what a
 * pure stream of the same bytes reaches on the device, reported beside the decode rate. */
int mdsx_copy_probe(const void* d_src, void* d_dst, uint64_t bytes, void* stream);
/* The probe's shapes, for measurement: 0 a 256 KiB loop per workgroup (8 loads per lane in
 * flight, non-temporal); 1 one 4 KiB piece per wave, non-temporal loads and stores (the shape of
 * the config-B row copy; what mdsx_copy_probe runs); 2 as 1 with plain loads; 3 as 1 with 8 KiB
 * per wave; 4 as 1 with plain loads and stores; 5 as 1 and 6 as 3 with the workgroups dealt
 * to the 8 XCDs in contiguous ranges (the register decode's tile order); 7 and 8 as 1 with
 * unused LDS per workgroup so that only 2 / 3 workgroups (8 / 12 waves) share a CU -- fewer
 * concurrent streams copy faster on MI355X (scripts/microbench/ring_copy3.hip); 9 as 5 with one
 * wave per workgroup, 10 as 9 with unused LDS so that 12 workgroups share a CU. The bench
 * reports the fastest variant of its run as the same-run copy ceiling. */
int mdsx_copy_probe_variant(const void* d_src, void* d_dst, uint64_t bytes, int variant,
                            void* stream);
/* Host hand-off copy: a 16-byte streaming kernel storing into PINNED host memory (a
 * device-accessible host pointer) over PCIe, `bytes` a multiple of 16, both pointers 16-byte
 * aligned; at most 64 workgroups striding over the bytes, so the CUs stay free for the next
 * batch's decode and H2D copy. A DMA-engine D2H and H2D do not overlap on this platform (they
 * serialise, measured); this copy runs beside the H2D (scripts/pcie_duplex.py), so a decoded
 * batch goes to the host while the next batch's shards come in. */
int mdsx_copy_to_host(const void* d_src, void* h_dst, uint64_t bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MDSX_H_ */
