// Host-side schema plan for the MDS decoder (part of libmdsx.so).
//
// Replaces the per-sample encoding dispatch of the reference: mds_decode -> _get_coder
// (streaming/base/format/mds/encodings.py:697-714,760-773), NDArray.from_str and
// _get_static_size (encodings.py:148-193) and the fixed/variable column split that
// MDSReader.decode_sample does per sample (mds/reader.py:111-118). The reference re-parses the
// encoding string for every column of every sample; here it is parsed once per schema.
#include <algorithm>
#include <cctype>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "mdsx_internal.h"

namespace mdsx {

thread_local std::string g_last_error;
thread_local std::string g_last_kernel;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

void set_last_kernel(const std::string& name) { g_last_kernel = name; }
const std::string& last_kernel_name() { return g_last_kernel; }

namespace {

// NDArray._int2value_dtype values (encodings.py:131-143) -> itemsize.
int value_dtype_size(const std::string& name) {
  if (name == "uint8" || name == "int8") return 1;
  if (name == "uint16" || name == "int16" || name == "float16") return 2;
  if (name == "uint32" || name == "int32" || name == "float32") return 4;
  if (name == "uint64" || name == "int64" || name == "float64") return 8;
  return 0;
}

std::string strip(const std::string& s) {
  size_t b = 0, e = s.size();
  while (b < e && std::isspace(static_cast<unsigned char>(s[b]))) ++b;
  while (e > b && std::isspace(static_cast<unsigned char>(s[e - 1]))) --e;
  return s.substr(b, e - b);
}

// Python int(str) for a decimal literal: optional sign, digits, single '_' between digits.
bool parse_py_int(const std::string& text, int64_t* out) {
  std::string s = strip(text);
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  if (i >= s.size()) return false;
  int64_t v = 0;
  bool prev_digit = false;
  for (; i < s.size(); ++i) {
    char c = s[i];
    if (c == '_') {
      if (!prev_digit || i + 1 >= s.size() || !std::isdigit(static_cast<unsigned char>(s[i + 1])))
        return false;
      prev_digit = false;
      continue;
    }
    if (!std::isdigit(static_cast<unsigned char>(c))) return false;
    if (v > (INT64_MAX - 9) / 10) return false;
    v = v * 10 + (c - '0');
    prev_digit = true;
  }
  *out = neg ? -v : v;
  return true;
}

std::vector<std::string> split(const std::string& s, char sep) {
  std::vector<std::string> parts;
  size_t start = 0;
  for (;;) {
    size_t p = s.find(sep, start);
    if (p == std::string::npos) {
      parts.push_back(s.substr(start));
      return parts;
    }
    parts.push_back(s.substr(start, p - start));
    start = p + 1;
  }
}

// Encodings whose decoded value is a host Python object (encodings.py:410-650). The device
// gathers their bytes; the host applies the reference semantics.
bool is_host_object_encoding(const std::string& name) {
  static const char* kNames[] = {"str_int", "str_float", "str_decimal", "pil",       "jpeg",
                                 "jpeg_array", "jpegarray", "png",       "list[pil]", "list[jpeg]",
                                 "list[png]", "pkl",       "json"};
  for (const char* n : kNames)
    if (name == n) return true;
  return false;
}

// Mirrors _get_coder (encodings.py:697-714): returns MDSX_OK and fills the column's natural
// encoding facts, or MDSX_E_ENCODING where the reference returns None or raises.
int parse_encoding(const std::string& enc, ColumnSpec* c) {
  size_t colon = enc.find(':');
  c->natural_size = -1;
  c->elem_bytes = 1;
  if (colon == std::string::npos) {
    if (enc == "bytes") {
      c->semantic = SEM_BYTES;
      return MDSX_OK;
    }
    if (enc == "str") {
      c->semantic = SEM_STR;
      return MDSX_OK;
    }
    if (enc == "int") {  // Int: int64 (encodings.py:84-94)
      c->semantic = SEM_SCALAR;
      c->natural_size = 8;
      c->elem_bytes = 8;
      return MDSX_OK;
    }
    if (enc == "ndarray") {  // dynamic dtype + shape
      c->semantic = SEM_NDARRAY_DYN;
      return MDSX_OK;
    }
    int sz = value_dtype_size(enc);
    if (sz) {  // Scalar family (encodings.py:308-397)
      c->semantic = SEM_SCALAR;
      c->natural_size = sz;
      c->elem_bytes = sz;
      return MDSX_OK;
    }
    if (is_host_object_encoding(enc)) {
      c->semantic = SEM_HOST_OBJECT;
      return MDSX_OK;
    }
    return fail(MDSX_E_ENCODING, "Unsupported encoding: " + enc + ".");
  }
  std::string name = enc.substr(0, colon);
  std::string config = enc.substr(colon + 1);
  if (name != "ndarray")  // only NDArray has from_str (encodings.py:173-193)
    return fail(MDSX_E_ENCODING, "Unsupported encoding: " + enc + ".");
  std::vector<std::string> args;
  if (!config.empty()) args = split(config, ':');
  if (args.size() > 2) return fail(MDSX_E_ENCODING, "Unsupported encoding: " + enc + ".");
  if (args.empty()) {
    c->semantic = SEM_NDARRAY_DYN;
    return MDSX_OK;
  }
  int sz = value_dtype_size(args[0]);
  if (!sz) return fail(MDSX_E_ENCODING, "Unsupported ndarray dtype in encoding: " + enc + ".");
  c->elem_bytes = sz;
  if (args.size() == 1) {  // static dtype, dynamic shape
    c->semantic = SEM_NDARRAY_DYN;
    return MDSX_OK;
  }
  int64_t count = 1;
  for (const std::string& d : split(args[1], ',')) {
    int64_t v = 0;
    if (!parse_py_int(d, &v) || v < 1)
      return fail(MDSX_E_ENCODING, "Bad ndarray shape in encoding: " + enc + ".");
    if (count > (int64_t(1) << 40) / v)
      return fail(MDSX_E_ENCODING, "ndarray shape too large in encoding: " + enc + ".");
    count *= v;
  }
  c->semantic = SEM_NDARRAY_STATIC;
  c->natural_size = count * sz;
  return MDSX_OK;
}

// Tuning knobs for measurements: MDSX_TUNE="tile=64,unroll=8,nt=1" (read at plan creation).
void apply_tuning(mdsx_plan* p) {
  const char* env = std::getenv("MDSX_TUNE");
  if (!env) return;
  for (const std::string& kv : split(env, ',')) {
    size_t eq = kv.find('=');
    if (eq == std::string::npos) continue;
    std::string key = strip(kv.substr(0, eq));
    int64_t v = 0;
    if (!parse_py_int(kv.substr(eq + 1), &v)) continue;
    if (key == "tile" && (v == 4 || v == 8 || v == 16 || v == 32 || v == 64 || v == 128 || v == 256)) {
      const int64_t per_row = 4 * int64_t(p->ncols) + 12 * int64_t(p->nvar);
      if (per_row * v <= 64 * 1024) p->tile_rows = int(v);
    } else if (key == "etile" && (v == 4 || v == 8 || v == 16 || v == 32 || v == 64 ||
                                  v == 128 || v == 256)) {
      if (4 * int64_t(p->ncols) * v <= 64 * 1024) p->encode_tile_rows = int(v);
    } else if (key == "gmin" && v >= 0) {
      p->gather_min = int(v);
    } else if (key == "gmax" && v >= 0) {
      p->group_max = int(v);
    } else if (key == "unroll" && (v == 2 || v == 4 || v == 6)) {
      p->unroll = int(v);
    } else if (key == "gk" && (v == 1 || v == 2 || v == 4)) {
      p->gather_chunks = int(v);
    } else if (key == "nt") {
      p->nontemporal = v ? 1 : 0;
    } else if (key == "strc") {
      p->str_cached = v ? 1 : 0;
    } else if (key == "ring" && (v == 0 || v == 4 || v == 6 || v == 8)) {
      p->ring_slots = int(v);
    } else if (key == "sdbg" && v >= 0) {
      p->stage_debug = int(v);
    } else if (key == "run" && (v == 0 || v == 4 || v == 7 || v == 8 || v == 16)) {
      p->run_slots = int(v);
    } else if (key == "rmin" && v >= 0) {
      p->run_min = v;
    } else if (key == "rnt") {
      p->run_nt = v ? 1 : 0;
    } else if (key == "rows" && v >= -1 && v <= 96) {
      p->rows_kb = int(v);
    } else if (key == "rslack" && v >= 2 && v <= 64) {
      p->rows_slack = int(v);
    } else if (key == "rocc" && (v == 4 || v == 6 || v == 8)) {
      p->rows_occ = int(v);
    } else if (key == "rpipe" && v >= 0 && v <= 1024) {
      p->rows_pipe = int(v);
    } else if (key == "rownt") {
      p->rows_nt = v ? 1 : 0;
    } else if (key == "swg" && (v == 1 || v == 2 || v == 4)) {
      p->seg_waves = int(v);
    } else if (key == "rw" && (v == 0 || v == 1 || v == 2 || v == 4)) {
      p->rowwave = int(v);
    } else if (key == "rwx" && v >= 0 && v <= 7) {
      p->rowwave_x = int(v);
    } else if (key == "rwk" && v >= 0 && v <= 65536) {
      p->rowwave_k = int(v);
    } else if (key == "snt" && v >= -1 && v <= 1) {
      p->scan_nt = int(v);
    } else if (key == "rwocc" && (v == 0 || v == 6 || v == 7 || v == 8)) {
      p->rowwave_occ = int(v);
    } else if (key == "rwr" && (v == 1 || v == 2 || v == 4)) {
      p->rowwave_rows = int(v);
    } else if (key == "lpad" && v >= 0 && v <= 150) {
      p->lds_pad_kb = int(v);
    } else if (key == "sv" && v >= 0 && v <= 2047) {
      p->seg_var = int(v);
    } else if (key == "seg") {
      p->seg = v ? 1 : 0;
    } else if (key == "xcd" || key == "xcdb" || key == "xcdr") {
      const int bit = key == "xcd" ? 1 : key == "xcdb" ? 2 : 4;  // kXcdSeg / Register / Rows
      p->xcd_order = v ? (p->xcd_order | bit) : (p->xcd_order & ~bit);
    } else if (key == "swave") {
      p->swave = v ? 1 : 0;
    } else if (key == "swkb" && (v == 4 || v == 6 || v == 8)) {
      p->swave_kb = int(v);
    } else if (key == "swlds" && v >= 1 && v <= 8) {
      p->swave_lds = int(v) * 1024;
    } else if (key == "swx" && v >= 0 && v <= 127) {
      p->swave_x = int(v);
    } else if (key == "swocc" && (v == 0 || v == 4 || v == 6)) {
      p->swave_occ = int(v);
    } else if (key == "swtile" && (v == 1 || v == 2 || v == 4 || v == 8 || v == 16 || v == 32 ||
                                   v == 64 || v == 128 || v == 256)) {
      p->swave_tile = int(v);
    } else if (key == "rkb" && v >= 1 && v <= 4096) {
      p->run_kb = int(v);
    }
  }
}

}  // namespace
}  // namespace mdsx

using namespace mdsx;

extern "C" {

const char* mdsx_last_error(void) { return g_last_error.c_str(); }

const char* mdsx_last_kernel(void) { return g_last_kernel.c_str(); }

#ifndef MDSX_SOURCE_SHA
#define MDSX_SOURCE_SHA "unknown"
#endif
// The library's version and the sha256 of the sources it was built from (streaming_amd/build.py
// source_sha): measurements key their profiles on it.
const char* mdsx_version(void) { return "mdsx 0.1.0 (gfx950) src " MDSX_SOURCE_SHA; }

int mdsx_plan_create(const char* const* encodings, const int64_t* column_sizes, int ncols,
                     mdsx_plan** out) {
  if (!out) return fail(MDSX_E_ARG, "mdsx_plan_create: out is NULL");
  *out = nullptr;
  if (ncols < 0 || ncols > MDSX_MAX_COLUMNS)
    return fail(MDSX_E_ARG, "mdsx_plan_create: ncols must be in [0, 64]");
  if (ncols > 0 && (!encodings || !column_sizes))
    return fail(MDSX_E_ARG, "mdsx_plan_create: null encodings or column_sizes");
  mdsx_plan* p = new (std::nothrow) mdsx_plan();
  if (!p) return fail(MDSX_E_ARG, "mdsx_plan_create: out of host memory");
  p->ncols = ncols;
  p->nvar = 0;
  p->fixed_sum = 0;
  p->safe = true;
  for (int i = 0; i < ncols; ++i) {
    ColumnSpec& c = p->cols[i];
    if (!encodings[i]) {
      delete p;
      return fail(MDSX_E_ARG, "mdsx_plan_create: null encoding string");
    }
    c.encoding = encodings[i];
    int rc = parse_encoding(c.encoding, &c);
    if (rc != MDSX_OK) {
      delete p;
      return rc;
    }
    if (c.encoding == "pkl") p->safe = false;  // _unsafe_encodings (encodings.py:685)
    // Layout follows the index's column_sizes exactly as MDSReader.decode_sample does
    // (`if size:` at mds/reader.py:114): a truthy size is a fixed column, anything else reads a
    // u32 size from the sample head.
    int64_t size = column_sizes[i];
    if (size > 0) {
      if (size >= (int64_t(1) << 32)) {
        delete p;
        return fail(MDSX_E_ENCODING, "column size past the u32 shard offset range");
      }
      c.kind = MDSX_KIND_FIXED;
      c.row_bytes = size;
      c.var_index = -1;
      p->fixed_sum += size;
    } else {
      c.row_bytes = 0;
      c.var_index = p->nvar++;
      if (c.semantic == SEM_STR)
        c.kind = MDSX_KIND_STR;
      else if (c.semantic == SEM_NDARRAY_DYN)
        c.kind = MDSX_KIND_NDARRAY;
      else
        c.kind = MDSX_KIND_BYTES;
    }
  }
  // Tile = rows of one workgroup. All-fixed plans: about 32 KiB of rows per tile (>= 4 rows),
  // so the resident workgroups stream through a narrow window of the shard buffer -- measured
  // on config B (4 KiB rows): 4-8-row tiles 5.87 TB/s, 16: 5.66, 64: 5.52, and the plain copy
  // probe 5.42 on the same box (scripts/tune_decode.py). Ragged plans on the register decode:
  // 32-row tiles (256-1024-byte blobs + 64-256-code-point strings: 2.08 vs 1.97 TB/s at 16 rows;
  // 32-256-byte rows 0.87 vs 0.76; long samples go to the streaming decode, which sizes its own
  // tiles, mdsx_plan_tile_rows_for). LDS per tile: a u32
  // source offset per (row, column), and per ragged column a u32 length and a u64 destination
  // offset per row (<= 16.4 KiB at 64 columns and 64 rows).
  if (p->nvar == 0) {
    const int64_t per_row = p->fixed_sum > 0 ? p->fixed_sum : 1;
    int tr = 4;
    while (tr < 256 && int64_t(tr) * 2 * per_row <= 32 * 1024) tr *= 2;
    p->tile_rows = tr;
  } else {
    p->tile_rows = 32;
  }
  // Encoder tiles: 16 rows (config B encode 5.06 TB/s vs 4.94 at 8 and 4.76 at 64; config C
  // 4.12 vs 3.74 at 64).
  p->encode_tile_rows = 16;
  p->nontemporal = 1;  // shard bytes are read once and outputs written once: stream them
  // Long ragged rows (one per wave) through a 4 KiB LDS-DMA ring per wave: config C 1.96 vs
  // 2.13 ms from registers, 1-3 KiB blobs + 200-400-code-point strings 1.67 vs 1.89; 6 and 8
  // slots lose the waves per CU their LDS costs (scripts/tune_decode.py, ring=0/4/6/8).
  p->ring_slots = p->nvar > 0 ? 4 : 0;
  // Medium str rows written with temporal stores, so the UTF-8 check's re-read of the packed
  // output hits L2 instead of HBM: config C 1.94-2.01 vs 2.06-2.10 ms; 1-3 KiB blobs + 200-400-
  // code-point strings 1.51 vs 1.56 ms (tune/strc_*.json).
  p->str_cached = 1;
  // Ragged batches of long samples decode through the streaming decode (mdsx_run.hip): every
  // shard byte read once, whole-chunk stores (use_run_decode). Its lean path (seg_decode_kernel:
  // one wait per sample, lane-parallel column geometry) needs a sample to fit the per-wave ring
  // with a slot to spare, so the ring is 8 KiB; non-temporal ring loads and stores. Config C
  // (scan + decode, three boxes, interleaved in one process each): 5.37 / 4.94 / 4.88 TB/s
  // against 4.69 / 4.62 / 4.60 for the round-2 streaming decode (4 KiB ring, temporal);
  // 16 KiB rings lose half the waves per CU (3.8-3.9 TB/s) (profiles/r03/ab/).
  p->run_slots = p->nvar > 0 ? 7 : 0;
  p->seg = 1;
  p->run_nt = 1;
  // ... and shorter samples through the row-parallel decode (mdsx_rows.hip), its tiles and stage
  // sized per batch (rows_tile_rows).
  p->rows_kb = p->nvar > 0 ? -1 : 0;
  // Its shard loads and output stores non-temporal: 1-3 % faster on 0.25-2.5 KB samples
  // (profiles/r02/rows_nt_crossover.jsonl).
  p->rows_nt = 1;
  apply_tuning(p);
  *out = p;
  return MDSX_OK;
}

void mdsx_plan_destroy(mdsx_plan* plan) { delete plan; }

int mdsx_plan_num_columns(const mdsx_plan* plan) { return plan ? plan->ncols : MDSX_E_ARG; }

int mdsx_plan_num_var(const mdsx_plan* plan) { return plan ? plan->nvar : MDSX_E_ARG; }

int mdsx_plan_tile_rows(const mdsx_plan* plan) { return plan ? plan->tile_rows : MDSX_E_ARG; }

int mdsx_plan_tile_rows_for(const mdsx_plan* plan, uint64_t shard_bytes, uint64_t rows) {
  if (!plan) return MDSX_E_ARG;
  if (use_swave_decode(plan, shard_bytes, rows)) return plan->swave_tile;
  if (use_run_decode(plan, shard_bytes, rows)) {
    // streaming decode: about run_kb KiB of samples per tile (one wave's run), 1..32 rows
    const uint64_t per_row = std::max<uint64_t>(1, shard_bytes / rows);
    int tr = 1;
    while (tr < 32 && uint64_t(tr) * 2 * per_row <= uint64_t(plan->run_kb) * 1024) tr *= 2;
    return tr;
  }
  if (use_rows_decode(plan, shard_bytes, rows))
    return rows_tile_rows(plan, shard_bytes / rows);
  return plan->tile_rows;
}

int mdsx_plan_encode_tile_rows(const mdsx_plan* plan) {
  return plan ? plan->encode_tile_rows : MDSX_E_ARG;
}

int mdsx_plan_column(const mdsx_plan* plan, int col, int* kind, int64_t* row_bytes,
                     int* elem_bytes) {
  if (!plan || col < 0 || col >= plan->ncols)
    return fail(MDSX_E_ARG, "mdsx_plan_column: bad plan or column");
  const ColumnSpec& c = plan->cols[col];
  if (kind) *kind = c.kind;
  if (row_bytes) *row_bytes = c.row_bytes;
  if (elem_bytes) *elem_bytes = c.elem_bytes;
  return MDSX_OK;
}

int mdsx_plan_is_safe(const mdsx_plan* plan) { return plan && plan->safe ? 1 : 0; }

}  // extern "C"
