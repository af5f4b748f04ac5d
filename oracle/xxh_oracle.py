"""ORACLE -- test infrastructure only. NOT part of the product and never on the product path.

A pure-Python restatement of the xxHash family the reference exposes as shard-file checksums
(SURVEY.md §8f-4): ``streaming/base/hashing.py:14-68`` collects ``xxhash.algorithms_available``
(python-xxhash 3.x, bundling the xxHash C library 0.8.2; the reference pins ``xxhash>=3.0.0,<4``
in ``setup.py``) next to hashlib's, and ``get_hash(algo, data)`` returns
``xxhash.<algo>(data).hexdigest()``. ``Writer._write_file`` (``base/writer.py:197-200``) records
these digests in ``index.json``; ``Stream._decompress_shard_part`` / ``_prepare_shard_part``
(``stream.py:333-340,403-411``) recompute them over the whole shard file to validate it.

Restated from the published xxHash specification (doc/xxhash_spec.md of xxHash 0.8.2 and the
reference implementation's XXH3 long-input loop):

* ``xxh32``  -- 4 lanes over 16-byte stripes, rotl 13, avalanche 15/13/16
* ``xxh64``  -- 4 lanes over 32-byte stripes, rotl 31, merge rounds, avalanche 33/29/32
* ``xxh3_64`` / ``xxh3_128`` (= ``xxh128``) -- short-input paths (0, 1-3, 4-8, 9-16, 17-128,
  129-240 bytes) and the long-input path: 8 accumulators, 64-byte stripes, 1 KiB blocks (16
  stripes with the default 192-byte secret) each followed by a scramble; seeded long inputs use
  the secret derived from the seed.

Only ``tests/`` import this module. Pinned by ``tests/test_hash_oracle.py``: the reference's own
known answer (``tests/test_hashing.py:34-41``: ``xxh3_64(b'hello') == '9555e8555c62dcfd'``), the
``index.json`` digests the reference writer recorded in ``tests/golden/`` and the python-xxhash
package (the reference's own dependency) on every length 0..2100 and on seeded inputs.
"""

from __future__ import annotations

import struct

__all__ = ['xxh32', 'xxh64', 'xxh3_64', 'xxh3_128', 'hexdigest', 'SECRET', 'derive_secret',
           'block_sums', 'ALGOS']

M32 = (1 << 32) - 1
M64 = (1 << 64) - 1

P32_1, P32_2, P32_3, P32_4, P32_5 = 0x9E3779B1, 0x85EBCA77, 0xC2B2AE3D, 0x27D4EB2F, 0x165667B1
P64_1 = 0x9E3779B185EBCA87
P64_2 = 0xC2B2AE3D27D4EB4F
P64_3 = 0x165667B19E3779F9
P64_4 = 0x85EBCA77C2B2AE63
P64_5 = 0x27D4EB2F165667C5
PMX1 = 0x165667919E3779F9
PMX2 = 0x9FB21C651E98DF25

# The default XXH3 secret (kSecret, 192 bytes).
SECRET = bytes.fromhex(
    'b8fe6c3923a44bbe7c01812cf721ad1cded46de9839097db7240a4a4b7b3671f'
    'cb79e64eccc0e578825ad07dccff7221b8084674f743248ee03590e6813a264c'
    '3c2852bb91c300cb88d0658b1b532ea371644897a20df94e3819ef46a9deacd8'
    'a8fa763fe39c343ff9dcbbc7c70b4f1d8a51e04bcdb45931c89f7ec9d9787364'
    'eac5ac8334d3ebc3c581a0fffa1363eb170ddd51b7f0da49d316552629d4689e'
    '2b16be587d47a1fc8ff8b8d17ad031ce45cb3a8f95160428afd7fbcabb4b407e')
assert len(SECRET) == 192

STRIPE = 64
BLOCK = 1024  # (192 - 64) // 8 = 16 stripes per block


def _u32(b: bytes, i: int) -> int:
    return struct.unpack_from('<I', b, i)[0]


def _u64(b: bytes, i: int) -> int:
    return struct.unpack_from('<Q', b, i)[0]


def _rotl32(x: int, r: int) -> int:
    return ((x << r) | (x >> (32 - r))) & M32


def _rotl64(x: int, r: int) -> int:
    return ((x << r) | (x >> (64 - r))) & M64


def _swap32(x: int) -> int:
    return int.from_bytes(x.to_bytes(4, 'little'), 'big')


def _swap64(x: int) -> int:
    return int.from_bytes(x.to_bytes(8, 'little'), 'big')


# ------------------------------------------------------------------------------------- XXH32
def xxh32(data: bytes, seed: int = 0) -> int:
    n = len(data)
    seed &= M32
    i = 0
    if n >= 16:
        v = [(seed + P32_1 + P32_2) & M32, (seed + P32_2) & M32, seed, (seed - P32_1) & M32]
        while i + 16 <= n:
            for k in range(4):
                v[k] = (_rotl32((v[k] + _u32(data, i + 4 * k) * P32_2) & M32, 13) * P32_1) & M32
            i += 16
        h = (_rotl32(v[0], 1) + _rotl32(v[1], 7) + _rotl32(v[2], 12) + _rotl32(v[3], 18)) & M32
    else:
        h = (seed + P32_5) & M32
    h = (h + n) & M32
    while i + 4 <= n:
        h = (_rotl32((h + _u32(data, i) * P32_3) & M32, 17) * P32_4) & M32
        i += 4
    while i < n:
        h = (_rotl32((h + data[i] * P32_5) & M32, 11) * P32_1) & M32
        i += 1
    h ^= h >> 15
    h = (h * P32_2) & M32
    h ^= h >> 13
    h = (h * P32_3) & M32
    h ^= h >> 16
    return h


# ------------------------------------------------------------------------------------- XXH64
def _round64(acc: int, lane: int) -> int:
    acc = (acc + lane * P64_2) & M64
    return (_rotl64(acc, 31) * P64_1) & M64


def _merge64(h: int, v: int) -> int:
    h ^= _round64(0, v)
    return (h * P64_1 + P64_4) & M64


def _avalanche64(h: int) -> int:
    h ^= h >> 33
    h = (h * P64_2) & M64
    h ^= h >> 29
    h = (h * P64_3) & M64
    h ^= h >> 32
    return h


def xxh64(data: bytes, seed: int = 0) -> int:
    n = len(data)
    seed &= M64
    i = 0
    if n >= 32:
        v = [(seed + P64_1 + P64_2) & M64, (seed + P64_2) & M64, seed, (seed - P64_1) & M64]
        while i + 32 <= n:
            for k in range(4):
                v[k] = _round64(v[k], _u64(data, i + 8 * k))
            i += 32
        h = (_rotl64(v[0], 1) + _rotl64(v[1], 7) + _rotl64(v[2], 12) + _rotl64(v[3], 18)) & M64
        for k in range(4):
            h = _merge64(h, v[k])
    else:
        h = (seed + P64_5) & M64
    h = (h + n) & M64
    while i + 8 <= n:
        h ^= _round64(0, _u64(data, i))
        h = (_rotl64(h, 27) * P64_1 + P64_4) & M64
        i += 8
    if i + 4 <= n:
        h ^= (_u32(data, i) * P64_1) & M64
        h = (_rotl64(h, 23) * P64_2 + P64_3) & M64
        i += 4
    while i < n:
        h ^= (data[i] * P64_5) & M64
        h = (_rotl64(h, 11) * P64_1) & M64
        i += 1
    return _avalanche64(h)


# -------------------------------------------------------------------------------------- XXH3
def _fold(a: int, b: int) -> int:
    p = a * b
    return (p & M64) ^ (p >> 64)


def _avalanche3(h: int) -> int:
    h ^= h >> 37
    h = (h * PMX1) & M64
    return h ^ (h >> 32)


def _rrmxmx(h: int, n: int) -> int:
    h ^= _rotl64(h, 49) ^ _rotl64(h, 24)
    h = (h * PMX2) & M64
    h ^= (h >> 35) + n
    h = (h * PMX2) & M64
    return h ^ (h >> 28)


def _mix16(data: bytes, i: int, sec: bytes, s: int, seed: int) -> int:
    return _fold(_u64(data, i) ^ ((_u64(sec, s) + seed) & M64),
                 _u64(data, i + 8) ^ ((_u64(sec, s + 8) - seed) & M64))


def derive_secret(seed: int) -> bytes:
    """XXH3_initCustomSecret: the secret of a seeded long input."""
    seed &= M64
    out = bytearray()
    for i in range(0, 192, 16):
        out += struct.pack('<QQ', (_u64(SECRET, i) + seed) & M64, (_u64(SECRET, i + 8) - seed) & M64)
    return bytes(out)


INIT_ACC = (P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1)


def _accumulate_stripe(acc: list, data: bytes, i: int, sec: bytes, s: int) -> None:
    for k in range(8):
        v = _u64(data, i + 8 * k)
        dk = v ^ _u64(sec, s + 8 * k)
        acc[k ^ 1] = (acc[k ^ 1] + v) & M64
        acc[k] = (acc[k] + (dk & M32) * (dk >> 32)) & M64


def _scramble(acc: list, sec: bytes) -> None:
    for k in range(8):
        a = acc[k]
        a ^= a >> 47
        a ^= _u64(sec, 128 + 8 * k)
        acc[k] = (a * P32_1) & M64


def block_sums(block: bytes, sec: bytes = SECRET) -> list:
    """The per-block sums of the long loop: acc after one block = scramble(acc + sums) (the
    accumulate step is a sum over the block's stripes). The device computes these in parallel."""
    s = [0] * 8
    for j in range(16):
        _accumulate_stripe(s, block, j * STRIPE, sec, 8 * j)
    return s


def _long_accs(data: bytes, sec: bytes) -> list:
    n = len(data)
    acc = list(INIT_ACC)
    nb = (n - 1) // BLOCK
    for b in range(nb):
        for j in range(16):
            _accumulate_stripe(acc, data, b * BLOCK + j * STRIPE, sec, 8 * j)
        _scramble(acc, sec)
    stripes = ((n - 1) - BLOCK * nb) // STRIPE
    for j in range(stripes):
        _accumulate_stripe(acc, data, nb * BLOCK + j * STRIPE, sec, 8 * j)
    _accumulate_stripe(acc, data, n - STRIPE, sec, 192 - STRIPE - 7)
    return acc


def _merge_accs(acc: list, sec: bytes, s: int, start: int) -> int:
    r = start & M64
    for k in range(4):
        r = (r + _fold(acc[2 * k] ^ _u64(sec, s + 16 * k), acc[2 * k + 1] ^ _u64(sec, s + 16 * k + 8))) & M64
    return _avalanche3(r)


def xxh3_64(data: bytes, seed: int = 0) -> int:
    n = len(data)
    seed &= M64
    k = SECRET
    if n <= 16:
        if n > 8:
            bf1 = ((_u64(k, 24) ^ _u64(k, 32)) + seed) & M64
            bf2 = ((_u64(k, 40) ^ _u64(k, 48)) - seed) & M64
            lo = _u64(data, 0) ^ bf1
            hi = _u64(data, n - 8) ^ bf2
            return _avalanche3((n + _swap64(lo) + hi + _fold(lo, hi)) & M64)
        if n >= 4:
            s = seed ^ (_swap32(seed & M32) << 32)
            x = (_u32(data, n - 4) + (_u32(data, 0) << 32)) ^ (((_u64(k, 8) ^ _u64(k, 16)) - s) & M64)
            return _rrmxmx(x, n)
        if n > 0:
            c = (data[0] << 16) | (data[n >> 1] << 24) | data[n - 1] | (n << 8)
            return _avalanche64(c ^ (((_u32(k, 0) ^ _u32(k, 4)) + seed) & M64))
        return _avalanche64(seed ^ _u64(k, 56) ^ _u64(k, 64))
    if n <= 128:
        acc = (n * P64_1) & M64
        if n > 32:
            if n > 64:
                if n > 96:
                    acc += _mix16(data, 48, k, 96, seed) + _mix16(data, n - 64, k, 112, seed)
                acc += _mix16(data, 32, k, 64, seed) + _mix16(data, n - 48, k, 80, seed)
            acc += _mix16(data, 16, k, 32, seed) + _mix16(data, n - 32, k, 48, seed)
        acc += _mix16(data, 0, k, 0, seed) + _mix16(data, n - 16, k, 16, seed)
        return _avalanche3(acc & M64)
    if n <= 240:
        acc = (n * P64_1) & M64
        for i in range(8):
            acc += _mix16(data, 16 * i, k, 16 * i, seed)
        acc = _avalanche3(acc & M64)
        for i in range(8, n // 16):
            acc += _mix16(data, 16 * i, k, 16 * (i - 8) + 3, seed)
        acc += _mix16(data, n - 16, k, 136 - 17, seed)
        return _avalanche3(acc & M64)
    sec = derive_secret(seed) if seed else SECRET
    return _merge_accs(_long_accs(data, sec), sec, 11, n * P64_1)


def _mix32(lo: int, hi: int, data: bytes, i1: int, i2: int, sec: bytes, s: int, seed: int):
    lo = (lo + _mix16(data, i1, sec, s, seed)) & M64
    lo ^= (_u64(data, i2) + _u64(data, i2 + 8)) & M64
    hi = (hi + _mix16(data, i2, sec, s + 16, seed)) & M64
    hi ^= (_u64(data, i1) + _u64(data, i1 + 8)) & M64
    return lo, hi


def xxh3_128(data: bytes, seed: int = 0) -> int:
    """Returns the 128-bit value (high64 << 64 | low64)."""
    n = len(data)
    seed &= M64
    k = SECRET
    if n <= 16:
        if n > 8:
            bfl = ((_u64(k, 32) ^ _u64(k, 40)) - seed) & M64
            bfh = ((_u64(k, 48) ^ _u64(k, 56)) + seed) & M64
            ilo = _u64(data, 0)
            ihi = _u64(data, n - 8)
            m = (ilo ^ ihi ^ bfl) * P64_1
            mlo, mhi = m & M64, m >> 64
            mlo = (mlo + ((n - 1) << 54)) & M64
            ihi ^= bfh
            mhi = (mhi + ihi + (ihi & M32) * (P32_2 - 1)) & M64
            mlo ^= _swap64(mhi)
            h = mlo * P64_2
            hlo, hhi = h & M64, h >> 64
            hhi = (hhi + mhi * P64_2) & M64
            return (_avalanche3(hhi) << 64) | _avalanche3(hlo)
        if n >= 4:
            s = seed ^ (_swap32(seed & M32) << 32)
            x = _u32(data, 0) + (_u32(data, n - 4) << 32)
            x ^= ((_u64(k, 16) ^ _u64(k, 24)) + s) & M64
            m = x * ((P64_1 + (n << 2)) & M64)
            mlo, mhi = m & M64, m >> 64
            mhi = (mhi + (mlo << 1)) & M64
            mlo ^= mhi >> 3
            mlo ^= mlo >> 35
            mlo = (mlo * PMX2) & M64
            mlo ^= mlo >> 28
            return (_avalanche3(mhi) << 64) | mlo
        if n > 0:
            cl = (data[0] << 16) | (data[n >> 1] << 24) | data[n - 1] | (n << 8)
            ch = _rotl32(_swap32(cl), 13)
            lo = cl ^ (((_u32(k, 0) ^ _u32(k, 4)) + seed) & M64)
            hi = ch ^ (((_u32(k, 8) ^ _u32(k, 12)) - seed) & M64)
            return (_avalanche64(hi) << 64) | _avalanche64(lo)
        return ((_avalanche64(seed ^ _u64(k, 80) ^ _u64(k, 88)) << 64)
                | _avalanche64(seed ^ _u64(k, 64) ^ _u64(k, 72)))
    if n <= 240:
        lo, hi = (n * P64_1) & M64, 0
        if n <= 128:
            rounds = []
            if n > 32:
                if n > 64:
                    if n > 96:
                        rounds.append((48, n - 64, 96))
                    rounds.append((32, n - 48, 64))
                rounds.append((16, n - 32, 32))
            rounds.append((0, n - 16, 0))
            for i1, i2, s in rounds:
                lo, hi = _mix32(lo, hi, data, i1, i2, k, s, seed)
        else:
            for i in range(4):
                lo, hi = _mix32(lo, hi, data, 32 * i, 32 * i + 16, k, 32 * i, seed)
            lo, hi = _avalanche3(lo), _avalanche3(hi)
            for i in range(4, n // 32):
                lo, hi = _mix32(lo, hi, data, 32 * i, 32 * i + 16, k, 3 + 32 * (i - 4), seed)
            lo, hi = _mix32(lo, hi, data, n - 16, n - 32, k, 136 - 17 - 16, (-seed) & M64)
        rlo = (lo + hi) & M64
        rhi = (lo * P64_1 + hi * P64_4 + ((n - seed) & M64) * P64_2) & M64
        return (((-_avalanche3(rhi)) & M64) << 64) | _avalanche3(rlo)
    sec = derive_secret(seed) if seed else SECRET
    acc = _long_accs(data, sec)
    lo = _merge_accs(acc, sec, 11, n * P64_1)
    hi = _merge_accs(acc, sec, 192 - 64 - 11, ~(n * P64_2) & M64)
    return (hi << 64) | lo


ALGOS = {'xxh32': (xxh32, 4), 'xxh64': (xxh64, 8), 'xxh3_64': (xxh3_64, 8),
         'xxh3_128': (xxh3_128, 16), 'xxh128': (xxh3_128, 16)}


def hexdigest(algo: str, data: bytes, seed: int = 0) -> str:
    """``xxhash.<algo>(data, seed).hexdigest()``: the big-endian hex of the hash value."""
    fn, width = ALGOS[algo]
    return f'{fn(data, seed):0{2 * width}x}'
