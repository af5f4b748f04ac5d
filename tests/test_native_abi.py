"""libmdsx.so loads on a CPU-only host, exports every symbol include/mdsx.h declares, and its
host-side plan builder parses schemas like the reference's _get_coder (no GPU calls here)."""

import ctypes
import os
import re

import pytest

from streaming_amd import _native
from streaming_amd.decoder import Plan
from tests import golden_util as gu

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'include',
                      'mdsx.h')


def _declared_functions():
    text = open(HEADER).read()
    text = re.sub(r'/\*.*?\*/', '', text, flags=re.S)
    return sorted(set(re.findall(r'\b(mdsx_[a-z_]+)\s*\(', text)))


def test_header_matches_binding_list():
    assert _declared_functions() == sorted(_native.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = _native.lib()
    for name in _declared_functions():
        assert hasattr(lib, name), name
    assert lib.mdsx_version().startswith(b'mdsx')


def test_library_built_from_these_sources():
    """The loaded library names the sources it was built from (bench.py keys profiles on it); a
    stale build (sources edited since) fails here instead of being measured."""
    from streaming_amd import build
    if os.environ.get('MDSX_LIBRARY'):
        pytest.skip('another build selected by MDSX_LIBRARY')
    version = _native.lib().mdsx_version().decode()
    assert version.endswith(' src ' + build.source_sha()), version


def test_struct_layouts():
    assert ctypes.sizeof(_native.ShardDesc) == 32
    assert ctypes.sizeof(_native.ColumnOut) == 32
    assert ctypes.sizeof(_native.Status) == 16
    assert ctypes.sizeof(_native.Batch) == 56


@pytest.mark.parametrize('name', gu.ALL_SETS)
def test_plan_for_every_golden_schema(name):
    info = gu.index(name)['shards'][0]
    plan = Plan(info['column_names'], info['column_encodings'], info['column_sizes'])
    assert len(plan.columns) == len(info['column_names'])
    for col, size in zip(plan.columns, info['column_sizes']):
        assert col.is_fixed == bool(size)
        if size:
            assert col.row_bytes == size
    assert plan.num_var == sum(1 for s in info['column_sizes'] if not s)
    if plan.num_var:
        assert plan.tile_rows == 32
    else:  # about 32 KiB of rows per decode tile, 4..256 rows
        per_row = sum(info['column_sizes'])
        assert plan.tile_rows in (4, 8, 16, 32, 64, 128, 256)
        assert plan.tile_rows == 4 or plan.tile_rows * per_row <= 32 * 1024
        assert plan.tile_rows == 256 or 2 * plan.tile_rows * per_row > 32 * 1024
    assert plan.encode_tile_rows == 16


def test_config_b_tiles():
    plan = Plan(['id', 'x'], ['int32', 'ndarray:float32:1024'], [4, 4096])
    assert plan.tile_rows == 4 and plan.encode_tile_rows == 16


def test_plan_kinds():
    plan = Plan(['a', 'b', 'c', 'd', 'e', 'f'], ['int', 'bytes', 'str', 'ndarray', 'ndarray:int16',
                                                  'json'], [8, None, None, None, None, None])
    kinds = [c.kind for c in plan.columns]
    assert kinds == [_native.KIND_FIXED, _native.KIND_BYTES, _native.KIND_STR,
                     _native.KIND_NDARRAY, _native.KIND_NDARRAY, _native.KIND_BYTES]
    assert plan.is_safe
    assert not Plan(['p'], ['pkl'], [None]).is_safe


@pytest.mark.parametrize('enc', ['foo', 'int:3', 'bytes:1', 'ndarray:float32:', 'ndarray:float33',
                                 'ndarray:float32:0', 'ndarray:float32:2:3:4', 'ndarray:int8:-1'])
def test_plan_rejects_unsupported_encodings(enc):
    with pytest.raises(ValueError):
        Plan(['a'], [enc], [None])


@pytest.mark.parametrize('enc,size', [('ndarray:uint8:3', 3), ('ndarray:float32:1, 2', 8),
                                      ('ndarray:int16:+2,3', 12), ('ndarray:uint8:1_0', 10),
                                      ('ndarray:', None), ('ndarray:float64', None)])
def test_plan_accepts_python_int_shapes(enc, size):
    plan = Plan(['a'], [enc], [size])
    assert plan.columns[0].is_fixed == (size is not None)


def test_workspace_bytes():
    lib = _native.lib()
    plan = Plan(['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None])
    b = _native.Batch()
    b.data, b.shards, b.tile_shard = 1, 1, 1
    b.bytes, b.nshards, b.ntiles, b.rows = 1 << 20, 1, 100, 6400
    r = lambda x: (x + 255) // 256 * 256
    # status block, per-tile totals and prefixes, chunk sums of their scan, the streaming
    # decode's 48-byte run records, per-row addresses (also the staged decode's huge-row list),
    # row map
    want = 256 + 2 * r(2 * 100 * 8) + r(2 * (100 // 4096 + 1) * 8) + r(100 * 48) + \
        r(2 * 6400 * 8) + r(2 * ((1 << 20) // 4096 + 8) * 4)
    assert lib.mdsx_workspace_bytes(plan.handle, ctypes.byref(b)) == want
    fixed = Plan(['id', 'x'], ['int32', 'ndarray:float32:1024'], [4, 4096])
    assert lib.mdsx_workspace_bytes(fixed.handle, ctypes.byref(b)) == 256


def test_too_many_columns():
    with pytest.raises(ValueError):
        Plan([f'c{i}' for i in range(65)], ['int'] * 65, [8] * 65)


def test_tile_rows_for_sizes_ragged_tiles_to_the_decode(monkeypatch):
    """Ragged plans: batches of long samples (>= 3 KiB on average) decode one sample per wave
    (64-row scan tiles) while they average <= 4/5 of its 6 KiB register window, else go to the
    streaming decode, whose tiles hold 16-32 KiB of samples (1..32 rows); shorter samples to the row-parallel
    decode, whose tiles fill at most 8/9 of a 20 KiB (samples < 512 B) or 40 KiB stage (1..256
    rows, the workgroup's LDS within 160 KiB); the register decode and all-fixed plans: the plan's
    tile size whatever the batch."""
    from streaming_amd.decoder import Plan
    c = Plan(['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None])
    assert c.tile_rows_for(1 << 26, (1 << 26) // 100) == 128  # 100-byte samples: row-parallel
    assert c.tile_rows_for(1 << 26, (1 << 26) // 50) == 256
    assert c.tile_rows_for(1 << 26, (1 << 26) // 250) == 64
    assert c.tile_rows_for(1 << 26, (1 << 26) // 1000) == 32
    assert c.tile_rows_for(1 << 26, (1 << 26) // 2000) == 16
    assert c.tile_rows_for(1 << 26, 15_700) == 64  # ~4.3 KB samples: one per wave, 64-row scan
    assert c.tile_rows_for(1 << 26, 12_000) == 2  # ~5.6 KB: past 4/5 of the window, streaming
    assert c.tile_rows_for(1 << 26, (1 << 26) // 2048) == 16
    assert c.tile_rows_for(1 << 26, 10) == 1  # 6.7 MB samples: one per tile
    wide = Plan([f'c{i:02d}' for i in range(64)], ['str'] * 64, [None] * 64)
    assert wide.tile_rows_for(1 << 26, 1 << 20) == 64  # 64 columns: the tables bound the tile
    monkeypatch.setenv('MDSX_TUNE', 'rows=18')
    assert Plan(['b'], ['bytes'], [None]).tile_rows_for(1 << 26, (1 << 26) // 100) == 128
    monkeypatch.setenv('MDSX_TUNE', 'swave=0')  # never one sample per wave: 2-row runs
    assert Plan(['b'], ['bytes'], [None]).tile_rows_for(1 << 26, 15_700) == 2
    monkeypatch.setenv('MDSX_TUNE', 'swave=1')  # always, whatever the sample size
    assert Plan(['b'], ['bytes'], [None]).tile_rows_for(1 << 26, 12_000) == 64
    assert Plan(['b'], ['bytes'], [None]).tile_rows_for(1 << 26, (1 << 26) // 100) == 128
    monkeypatch.setenv('MDSX_TUNE', 'swave=1,swtile=256')
    assert Plan(['b'], ['bytes'], [None]).tile_rows_for(1 << 26, 15_700) == 256
    monkeypatch.setenv('MDSX_TUNE', 'run=4,rkb=256,swave=0')
    assert Plan(['b'], ['bytes'], [None]).tile_rows_for(1 << 26, 15_700) == 32
    monkeypatch.setenv('MDSX_TUNE', 'run=0,rows=0')  # the register decode: the plan's tiles
    c = Plan(['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None])
    assert c.tile_rows_for(1 << 26, 15_700) == c.tile_rows == 32
    assert c.tile_rows_for(1 << 26, (1 << 26) // 100) == 32
    b = Plan(['id', 'x'], ['int32', 'ndarray:float32:1024'], [4, 4096])
    assert b.tile_rows_for(1 << 26, 16_352) == b.tile_rows


def test_batch_tiles_from_the_buffer_bytes_the_decode_choice_reads():
    """The C side picks the decode (streaming vs row-parallel) and the stage from batch->bytes,
    the padded buffer size; the batch's tile table must be sized from the same count (ADVICE
    round 2). Small shards whose samples average just under the streaming threshold unpadded
    (3000 bytes) and above it padded (each shard rounded up to 256 bytes)."""
    from streaming_amd.decoder import Plan, make_batch
    c = Plan(['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None])
    sizes, samples = [3000] * 64, [1] * 64
    b = make_batch(c, sizes, samples, device='cpu')
    assert sum(sizes) // sum(samples) < 3072 <= b.buffer.numel() // sum(samples)
    assert b.tile_rows == c.tile_rows_for(b.buffer.numel(), sum(samples))
