// Host check of the row-parallel decode's per-chunk UTF-8 logic (mdsx_rows.hip, phase 4): the
// device helpers (byte masks, the nibble-table check utf8_lookup_err / utf8_chunk_err2 /
// utf8_open_at) are pasted in from streaming_amd/csrc/mdsx_device.h by tests/test_utf8_chunks.py
// (at the placeholder below), with host stand-ins for the two gfx950 intrinsics (v_alignbyte_b32,
// v_perm_b32). Random runs of values (mostly well-formed text with injected bad bytes, and raw
// bytes) are laid out at every output misalignment, walked chunk by chunk exactly as the kernel
// does (one or two values per chunk straight-line, piece by piece otherwise), and each value's
// verdict is compared with a strict decoder (what bytes.decode('utf-8') accepts).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>
#define __device__
#define __forceinline__ inline
struct uint4 {
  uint32_t x, y, z, w;
};
static inline uint4 make_uint4(uint32_t x, uint32_t y, uint32_t z, uint32_t w) { return {x, y, z, w}; }
// v_perm_b32: byte k of {s0 (high), s1 (low)} for selector values 0..7
static uint32_t perm_emu(uint32_t s0, uint32_t s1, uint32_t sel) {
  const uint64_t d = (uint64_t(s0) << 32) | s1;
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) {
    const uint32_t k = (sel >> (8 * i)) & 0xff;
    const uint32_t b = k < 8 ? uint32_t(d >> (8 * k)) & 0xff : (k == 12 ? 0u : 0xffu);
    r |= b << (8 * i);
  }
  return r;
}
#define __builtin_amdgcn_perm perm_emu
static inline uint32_t alignbyte(uint32_t hi, uint32_t lo, uint32_t r) {
  return uint32_t(((uint64_t(hi) << 32) | lo) >> (8 * (r & 3)));
}
using std::max;
using std::min;
@DEVICE_CODE@
static uint4 and4(uint4 a, uint4 m) { return {a.x & m.x, a.y & m.y, a.z & m.z, a.w & m.w}; }
// Strict UTF-8 as Python's decoder accepts it: no overlong forms, surrogates or code points above
// U+10FFFF, no truncated sequences.
static bool valid(const uint8_t* s, int n) {
  int i = 0;
  while (i < n) {
    const uint8_t c = s[i];
    if (c < 0x80) {
      ++i;
      continue;
    }
    int need;
    uint32_t cp;
    if (c >= 0xC2 && c <= 0xDF) need = 1, cp = c & 0x1F;
    else if (c >= 0xE0 && c <= 0xEF) need = 2, cp = c & 0x0F;
    else if (c >= 0xF0 && c <= 0xF4) need = 3, cp = c & 0x07;
    else return false;
    for (int k = 1; k <= need; ++k) {
      if (i + k >= n || (s[i + k] & 0xC0) != 0x80) return false;
      cp = (cp << 6) | (s[i + k] & 0x3F);
    }
    if (need == 2 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) return false;
    if (need == 3 && (cp < 0x10000 || cp > 0x10FFFF)) return false;
    i += need + 1;
  }
  return true;
}

static std::mt19937 rng(1);
static const uint8_t kPool[] = {0x00, 0x41, 0x7F, 0x80, 0x8F, 0x90, 0x9F, 0xA0, 0xBF, 0xC0, 0xC1, 0xC2,
                                0xDF, 0xE0, 0xE1, 0xED, 0xEE, 0xEF, 0xF0, 0xF1, 0xF4, 0xF5, 0xFF};

// Raw bytes, mostly the interesting ones.
static void gen_raw(uint8_t* s, int n) {
  for (int i = 0; i < n; ++i) s[i] = (rng() & 3) ? kPool[rng() % sizeof(kPool)] : uint8_t(rng());
}

// Well-formed text (1- to `widths`-byte code points, cut at n bytes), one bad byte a third of
// the time.
static void gen_text(uint8_t* s, int n, int widths = 4) {
  int i = 0;
  while (i < n) {
    const int w = rng() % widths;
    uint32_t cp;
    if (w == 0) cp = 0x20 + rng() % 95;
    else if (w == 1) cp = 0x80 + rng() % 0x780;
    else if (w == 2) cp = 0x800 + rng() % 0xF000, cp += (cp >= 0xD800 && cp < 0xE000) ? 0x800 : 0;
    else cp = 0x10000 + rng() % 0x100000;
    uint8_t b[4];
    int k;
    if (cp < 0x80) b[0] = cp, k = 1;
    else if (cp < 0x800) b[0] = 0xC0 | (cp >> 6), b[1] = 0x80 | (cp & 63), k = 2;
    else if (cp < 0x10000)
      b[0] = 0xE0 | (cp >> 12), b[1] = 0x80 | ((cp >> 6) & 63), b[2] = 0x80 | (cp & 63), k = 3;
    else
      b[0] = 0xF0 | (cp >> 18), b[1] = 0x80 | ((cp >> 12) & 63), b[2] = 0x80 | ((cp >> 6) & 63),
      b[3] = 0x80 | (cp & 63), k = 4;
    for (int j = 0; j < k && i < n; ++j) s[i++] = b[j];
  }
  if (n > 0 && rng() % 3 == 0) s[rng() % n] = kPool[rng() % sizeof(kPool)];
}

// The dword before byte `at` of the stage, bytes before the value's start (`from`) zero.
static uint32_t dword_before(const std::vector<uint8_t>& st, int at, int from) {
  uint32_t pw;
  memcpy(&pw, st.data() + at - 4, 4);
  const int nv = at - from;
  if (nv < 4) pw &= ~((1u << (8 * (4 - nv))) - 1u);
  return pw;
}

static long nsimple = 0, nslow = 0;

// The values V laid out back to back in the window's output, its first byte at byte hd of an
// aligned chunk; each chunk checked as mdsx_rows.hip does. Returns each value's "bad" verdict.
static std::vector<bool> run_chunks(const std::vector<std::vector<uint8_t>>& V, int hd) {
  const int nv = int(V.size());
  std::vector<int> ds(nv), len(nv);
  std::vector<uint8_t> st(32, 0xEE);  // the stage: junk around the values (output = stage order)
  for (int i = 0; i < nv; ++i) {
    ds[i] = int(st.size()) - 32, len[i] = int(V[i].size());
    st.insert(st.end(), V[i].begin(), V[i].end());
  }
  const int wlen = int(st.size()) - 32;
  st.resize(st.size() + 32, 0xEE);
  std::vector<bool> bad(nv, false);
  auto read16 = [&](int at) {
    uint4 v;
    memcpy(&v, st.data() + 32 + at, 16);
    return v;
  };
  for (int k = 0; wlen > 0 && k * 16 < hd + wlen; ++k) {  // (no chunks when no bytes, as the kernel)
    const int P0 = 16 * k - hd, end = std::min(P0 + 16, wlen);
    int pos = std::max(P0, 0);
    int r = 0;  // the chunk map: the value holding byte pos
    while (!(ds[r] <= pos && pos < ds[r] + len[r])) ++r;
    const int dsA = ds[r], deA = dsA + len[r], hiA = std::min(end, deA);
    uint4 val = read16(P0);
    bool simple = deA > pos;
    uint32_t sB = 16;
    int deL = deA;
    if (simple && hiA < end) {
      const int dsB = ds[r + 1], deB = dsB + len[r + 1];
      simple = dsB == hiA && deB >= end;
      if (simple) sB = hiA - P0, deL = deB;  // (the stage is the output order: val holds B too)
    }
    if (simple) {
      ++nsimple;
      const uint4 X = (pos > P0 || end < P0 + 16) ? keep_bytes(val, pos - P0, end - P0) : val;
      const uint32_t pw = pos > dsA ? dword_before(st, 32 + pos, 32 + dsA) : 0u;
      uint32_t e = utf8_chunk_err2(X, pw, sB);
      if (sB < 16 && utf8_open_at(X, pw, sB)) e |= 1;
      if (end == P0 + 16 && end == deL) {
        if (sB < 16) e |= utf8_open_at(keep_bytes(X, sB, 16), 0, 16) ? 2 : 0;
        else e |= utf8_open_at(X, pw, 16) ? 1 : 0;
      }
      if (e & 1) bad[r] = true;
      if (e & 2) bad[r + 1] = true;
    } else {
      ++nslow;
      for (int rr = r; rr < nv && pos < end; ++rr) {
        const int d0 = ds[rr], d1 = d0 + len[rr];
        if (d1 <= pos) continue;
        if (d0 >= end) break;
        const int lo = std::max(pos, d0), hi = std::min(end, d1);
        const uint4 pv = keep_bytes(val, lo - P0, hi - P0);
        const uint32_t pw = lo > d0 ? dword_before(st, 32 + lo, 32 + d0) : 0u;
        // (an ASCII piece after no lead byte is skipped, as the kernel does)
        const bool ascii = (((pv.x | pv.y | pv.z | pv.w) & 0x80808080u) | hi_c0(pw)) == 0;
        if (!ascii && ((utf8_chunk_err2(pv, pw, 16) & 1) ||
                       (hi == d1 && hi == P0 + 16 && utf8_open_at(pv, pw, 16))))
          bad[rr] = true;
        pos = hi;
      }
    }
  }
  return bad;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 100000;
  long total = 0, mismatches = 0;
  for (int it = 0; it < iters; ++it) {
    std::vector<std::vector<uint8_t>> V(1 + rng() % 12);
    for (size_t i = 0; i < V.size(); ++i) {
      const int n = (rng() % 5 == 0) ? rng() % 4 : 1 + rng() % 40;  // some empty and tiny values
      V[i].resize(n);
      if (n) {
        const int kind = int((it + i) % 3);
        kind == 0 ? gen_raw(V[i].data(), n) : kind == 1 ? gen_text(V[i].data(), n)
                                                      : gen_text(V[i].data(), n, 2);
      }
    }
    const int hd = rng() % 16;
    const std::vector<bool> bad = run_chunks(V, hd);
    for (size_t i = 0; i < V.size(); ++i) {
      ++total;
      const bool ok = valid(V[i].data(), int(V[i].size()));
      if (bad[i] == !ok) continue;
      if (++mismatches <= 8) {
        printf("mismatch: value %zu of %zu, head %d, flagged %d, valid %d:", i, V.size(), hd,
               int(bad[i]), int(ok));
        for (uint8_t c : V[i]) printf(" %02X", c);
        printf("\n");
      }
    }
  }
  printf("values %ld mismatches %ld (simple chunks %ld, slow %ld)\n", total, mismatches, nsimple, nslow);
  return mismatches == 0 ? 0 : 1;
}
