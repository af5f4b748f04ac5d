"""The row-parallel decode's per-chunk UTF-8 check, on the host (no GPU).

mdsx_rows.hip checks str values 16 output bytes at a time: a chunk holding one or two values is
checked in one pass with each value in its own context (utf8_chunk_err2, the nibble-table check
utf8_lookup_err) plus an open-sequence test where a value ends (utf8_open_at); other chunks go
piece by piece. tests/native/utf8_chunks.cpp walks random runs of values chunk by chunk the same
way, with the device helpers pasted in from mdsx_device.h (host stand-ins for v_alignbyte_b32 and
v_perm_b32), and compares every value's verdict with a strict decoder -- what
``bytes.decode('utf-8')`` accepts (encodings.py:80-81 in the reference).
"""

import re
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
DEVICE_H = ROOT / 'streaming_amd' / 'csrc' / 'mdsx_device.h'
HARNESS = ROOT / 'tests' / 'native' / 'utf8_chunks.cpp'


def _section(text: str, start: str, end: str) -> str:
    i = text.index(start)
    return text[i:text.index(end, i)]


def _device_code() -> str:
    h = DEVICE_H.read_text()
    parts = [
        _section(h, '// 0xFF in byte i of the result', '// Bytes [a, b) (0 <= a <= b <= 16) of `val`'),
        _section(h, '__device__ __forceinline__ uint32_t hi_c0', '// Error bits of dword x'),
        _section(h, '// ---- The same check by nibble tables', '// Bytes of a 16-byte chunk at address D'),
    ]
    return '\n'.join(parts)


@pytest.fixture(scope='module')
def harness(tmp_path_factory):
    gxx = shutil.which('g++')
    if gxx is None:
        pytest.skip('g++ not available')
    d = tmp_path_factory.mktemp('utf8')
    src = d / 'utf8_chunks.cpp'
    src.write_text(HARNESS.read_text().replace('@DEVICE_CODE@', _device_code()))
    exe = d / 'utf8_chunks'
    subprocess.run([gxx, '-O2', '-std=c++17', '-o', str(exe), str(src)], check=True)
    return exe


def test_chunk_checks_match_a_strict_decoder(harness):
    out = subprocess.run([str(harness), '60000'], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    m = re.search(r'values (\d+) mismatches (\d+) \(simple chunks (\d+), slow (\d+)\)', out.stdout)
    assert m, out.stdout
    values, bad, simple, slow = map(int, m.groups())
    assert bad == 0
    assert values > 300_000 and simple > 0 and slow > 0  # both chunk paths exercised
