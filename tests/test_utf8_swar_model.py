"""CPU model of the device's SWAR UTF-8 validator (mdsx_kernels.hip: utf8_dword_err /
utf8_chunk_bad) checked against Python's strict decoder -- the reference's Str.decode
(streaming/base/format/mds/encodings.py:80-81) -- on random byte strings built from the
interesting bytes (leads, continuations, overlong / surrogate / >U+10FFFF boundaries)."""

import random

import pytest

M = 0xffffffff


def _al(x, p, r):
    return ((x << 32 | p) >> (8 * r)) & M


def _hc0(y):
    return y & (y << 1) & 0x80808080


def _he0(y):
    return y & (y << 1) & (y << 2) & 0x80808080


def _hf0(y):
    return y & (y << 1) & (y << 2) & (y << 3) & 0x80808080


def _z(v):
    return (~((((v & 0x7F7F7F7F) + 0x7F7F7F7F) & M) | v)) & 0x80808080


def dword_err(x, p):
    p1, p2, p3 = _al(x, p, 3), _al(x, p, 2), _al(x, p, 1)
    cont = x & ~(x << 1) & 0x80808080
    need = _hc0(p1) | _he0(p2) | _hf0(p3)
    e = need ^ cont
    e |= _z((x & 0xFEFEFEFE) ^ 0xC0C0C0C0)
    e |= ((x & 0x7F7F7F7F) + 0x0B0B0B0B) & x & 0x80808080
    b5 = (x << 2) & 0x80808080
    b45 = ((x << 2) | (x << 3)) & 0x80808080
    e |= _z(p1 ^ 0xE0E0E0E0) & ~b5 & 0x80808080
    e |= _z(p1 ^ 0xEDEDEDED) & b5
    e |= _z(p1 ^ 0xF0F0F0F0) & ~b45 & 0x80808080
    e |= _z(p1 ^ 0xF4F4F4F4) & b45
    return e & M


def segment_bad(seg, off):
    """The device's verdict for a segment starting `off` bytes into a 16-byte chunk."""
    buf = bytes(off) + seg
    buf += bytes((-len(buf)) % 16)
    pw, err, n = 0, 0, len(buf) // 16
    for c in range(n):
        d = [int.from_bytes(buf[16 * c + 4 * m:16 * c + 4 * m + 4], 'little') for m in range(4)]
        e = dword_err(d[0], pw) | dword_err(d[1], d[0]) | dword_err(d[2], d[1]) | \
            dword_err(d[3], d[2])
        if c == n - 1:
            e |= dword_err(0, d[3])
        err |= e
        pw = d[3]
    return n > 0 and err != 0


ALPHABET = [
    b'a', b'\x80', b'\xbf', b'\xc0', b'\xc1', b'\xc2', b'\xdf', b'\xe0', b'\xe1', b'\xed', b'\xee',
    b'\xef', b'\xf0', b'\xf1', b'\xf4', b'\xf5', b'\xff', b'\x90', b'\x9f', b'\xa0', b'\x8f',
    'é'.encode(), '€'.encode(), '\U0001F600'.encode(), '\U0010FFFF'.encode(),
    '퟿'.encode(), b'\x00'
]


@pytest.mark.parametrize('seed', range(4))
def test_swar_model_matches_python_decoder(seed):
    rng = random.Random(seed)
    for _ in range(20_000):
        seg = b''.join(rng.choice(ALPHABET) for _ in range(rng.randrange(0, 12)))
        try:
            seg.decode('utf-8')
            ok = True
        except UnicodeDecodeError:
            ok = False
        assert segment_bad(seg, rng.randrange(16)) == (not ok), seg
