"""GPU parity: device header parse of dynamic ndarray columns (``mdsx_ndarray_meta`` /
``mdsx_ndarray_shapes``) against the oracle's NDArray.decode restatement
(``oracle/mds_oracle.py:_ndarray_decode``, reference ``encodings.py:270-305``).

Per row the device reports dtype id, shape, the value bytes' offset and ``bad``; the bar is the
oracle's result on the same row bytes: same dtype and shape, same value bytes, and ``bad``
exactly where the oracle raises.
"""

import numpy as np
import pytest
import torch

from oracle import mds_oracle
from streaming_amd.decoder import (Plan, RaggedColumn, decode_batch, ndarray_meta, stage_shards)
from streaming_amd.encodings import VALUE_DTYPES
from tests import golden_util as gu

pytestmark = pytest.mark.gpu

_IDS = {v: k for k, v in VALUE_DTYPES.items()}


@pytest.fixture(scope='module', autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')


def _check_against_oracle(col: RaggedColumn, encoding: str, dtype_id: int):
    meta = ndarray_meta(col, dtype_id)
    values = col.values.cpu().numpy().tobytes()
    offs = col.offsets.cpu().numpy()
    dt, nd, do, ne, bad = (t.cpu().numpy() for t in (meta.dtype, meta.ndim, meta.data_offset,
                                                      meta.numel, meta.bad))
    shape = meta.shape.cpu().numpy()
    nbad = 0
    for i in range(len(col)):
        row = values[offs[i]:offs[i + 1]]
        try:
            ref = mds_oracle.mds_decode(encoding, row)
        except Exception:  # the reference's decode raises on this row
            assert bad[i] == 1, f'row {i}: oracle raises, device says ok'
            nbad += 1
            continue
        assert bad[i] == 0, f'row {i}: device flags a row the oracle decodes'
        assert VALUE_DTYPES[int(dt[i])] == ref.dtype.name, i
        assert int(nd[i]) == ref.ndim, i
        assert tuple(int(x) for x in shape[i, :nd[i]]) == ref.shape, i
        assert np.all(shape[i, nd[i]:] == 1), i
        assert int(ne[i]) == ref.size, i
        got = values[do[i]:do[i] + ref.nbytes]
        assert got == ref.tobytes(), i
        if ref.size and i % 7 == 0:
            t = meta.row(col, i).cpu().numpy()
            assert t.shape == ref.shape and t.tobytes() == ref.tobytes()
    return nbad


def test_dynamic_golden_columns():
    name = 'dynamic'
    idx = gu.index(name)
    info0 = idx['shards'][0]
    plan = Plan(info0['column_names'], info0['column_encodings'], info0['column_sizes'])
    data = [gu.shard_bytes(name, s) for s in idx['shards']]
    decoded = decode_batch(plan, stage_shards(data, [s['samples'] for s in idx['shards']], plan))
    seen = 0
    for col_name, enc in zip(info0['column_names'], info0['column_encodings']):
        if not enc.startswith('ndarray'):
            continue
        parts = enc.split(':')
        dtype_id = _IDS[parts[1]] if len(parts) > 1 else 0
        assert _check_against_oracle(decoded[col_name], enc, dtype_id) == 0
        seen += 1
    assert seen == 3


def _ragged(rows):
    offs = np.zeros(len(rows) + 1, np.int64)
    offs[1:] = np.cumsum([len(r) for r in rows])
    vals = np.frombuffer(b''.join(rows), np.uint8) if offs[-1] else np.zeros(0, np.uint8)
    return RaggedColumn(torch.from_numpy(vals.copy()).cuda(), torch.from_numpy(offs).cuda())


def _header(dtype_id, shape, code, static):
    h = b'' if static else bytes([dtype_id])
    h += bytes([(len(shape) << 2) | code])
    sdt = ('<u1', '<u2', '<u4', '<u8')[code]
    return h + np.asarray(shape, dtype=sdt).tobytes()


@pytest.mark.parametrize('static', [None, 'float32', 'int16', 'uint8'])
def test_malformed_and_edge_rows(static):
    rng = np.random.default_rng(11 if static is None else len(static))
    rows = []
    for i in range(3000):
        name = static or VALUE_DTYPES[list(VALUE_DTYPES)[i % len(VALUE_DTYPES)]]
        dtid = _IDS[name]
        item = np.dtype(name).itemsize
        ndim = int(rng.integers(0, 5))
        shape = [int(rng.integers(0, 5)) for _ in range(ndim)]
        code = int(rng.integers(0, 4))
        numel = int(np.prod(shape)) if ndim else 1
        body = rng.bytes(numel * item)
        kind = i % 10
        if kind == 0:      # value bytes one item short / long
            body = body[:-item] if body else body + rng.bytes(item)
        elif kind == 1:    # truncated shape
            hdr = _header(dtid, shape, code, static)
            rows.append(hdr[:max(0, len(hdr) - 1 - int(rng.integers(0, 3)))])
            continue
        elif kind == 2 and static is None:  # unknown dtype id
            rows.append(bytes([int(rng.choice([0, 1, 7, 10, 19, 35, 67, 255]))]) +
                        _header(dtid, shape, code, True) + body)
            continue
        elif kind == 3:    # ragged byte count (not a multiple of the item size)
            body = body + b'\x00' if item > 1 else body
        elif kind == 4:    # a zero dim with a huge other dim (empty array, numpy accepts)
            shape = [0, 2**40 + 3] if code == 3 else [0, 200]
            body = b''
        elif kind == 5:    # product overflows intp
            shape, code, body = [2**40, 2**40], 3, rng.bytes(16)
        rows.append(_header(dtid, shape, code, static) + body)
    rows += [b'', b'\x00', b'\x04', bytes([_IDS['float64'], 0]) + b'\x00' * 8]
    enc = f'ndarray:{static}' if static else 'ndarray'
    nbad = _check_against_oracle(_ragged(rows), enc, _IDS[static] if static else 0)
    assert 0 < nbad < len(rows)


def test_empty_column():
    meta = ndarray_meta(_ragged([]), 0)
    assert meta.shape.shape == (0, 0) and meta.bad.numel() == 0
