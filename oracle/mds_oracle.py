"""ORACLE -- test infrastructure only. NOT part of the product and never on the product path.

A CPU restatement of mosaicml/streaming's per-sample MDS read path, used as the checker of the
GPU decoder and as the CPU baseline timed by ``bench.py`` (``cpu_baseline.kind = "port"``).
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module.

Restated from (paths relative to the mosaicml/streaming repository):

* ``OracleMDSReader.get_sample_data``  <- ``streaming/base/format/mds/reader.py:128-149``
  (open, seek to the u32 offsets pair, read, IndexError on empty data)
* ``OracleMDSReader.decode_sample``    <- ``streaming/base/format/mds/reader.py:103-126``
  (u32 size head of the variable columns, then one slice per column)
* ``mds_decode``                       <- ``streaming/base/format/mds/encodings.py:760-773``
  with the per-encoding decoders of ``encodings.py:62-397`` (Bytes, Str, Int, NDArray, scalars)
* ``writer_split``                     <- ``Writer.write`` (``streaming/base/format/base/
  writer.py:248-269``): flush when ``size_limit < shard_size + sample + 4``, per sample
* ``encode_sample_from_columns`` / ``encode_joint_shard`` <- ``MDSWriter.encode_sample`` /
  ``encode_joint_shard`` (``streaming/base/format/mds/writer.py:92-117,133-144``) over columns in
  the device format (the checker of the device encoder)
* ``decode_shard_columns``             <- the reader applied to every sample of a shard, written
  in the device decoder's output format (fixed columns as row bytes, ragged columns as packed
  values + int64 offsets + a UTF-8 validity flag per row for ``str``)

Parity pinning: ``tests/golden/make_golden.py`` generated the fixtures under ``tests/golden/``
by running the REAL reference (imported offline in the build container) and recording its
decoded values; ``tests/test_oracle_golden.py`` checks this oracle against every one of them.
"""

from __future__ import annotations

import hashlib
import json
import os
from typing import Any, Optional

import numpy as np

__all__ = [
    'OracleMDSReader', 'ReferenceCostMDSReader', 'mds_decode', 'mds_decode_reference_cost',
'decode_shard_columns', 'decode_fixed_shard_vectorized',
    'column_digests', 'utf8_is_valid', 'load_index', 'writer_split', 'encode_sample_from_columns',
    'encode_joint_shard'
]

_VALUE_DTYPES = {
    8: 'uint8',
    9: 'int8',
    16: 'uint16',
    17: 'int16',
    18: 'float16',
    32: 'uint32',
    33: 'int32',
    34: 'float32',
    64: 'uint64',
    65: 'int64',
    66: 'float64',
}
_SHAPE_DTYPES = {0: 'uint8', 1: 'uint16', 2: 'uint32', 3: 'uint64'}
_SCALARS = ('uint8', 'uint16', 'uint32', 'uint64', 'int8', 'int16', 'int32', 'int64', 'float16',
            'float32', 'float64')


def _ndarray_decode(config: str, data: bytes) -> np.ndarray:
    # NDArray.from_str (encodings.py:173-193) then NDArray.decode (encodings.py:270-305).
    args = config.split(':') if config else []
    dtype = args[0] if len(args) >= 1 else None
    shape = tuple(int(x) for x in args[1].split(',')) if len(args) >= 2 else None
    index = 0
    if not dtype:
        dtype = _VALUE_DTYPES[data[index]]
        index += 1
    if not shape:
        byte = data[index]
        index += 1
        ndim, code = byte >> 2, byte % 4
        size = ndim * 2**code
        shape = np.frombuffer(data[index:index + size], _SHAPE_DTYPES[code])
        index += size
    return np.frombuffer(data[index:], dtype).reshape(shape)


def mds_decode(encoding: str, data: bytes) -> Any:
    """Decode one column value (encodings.py:760-773) for the device-decoded encodings."""
    name, _, config = encoding.partition(':')
    if name == 'bytes' and not config:
        return data
    if name == 'str' and not config:
        return data.decode('utf-8')
    if name == 'int' and not config:
        return int(np.frombuffer(data, np.int64)[0])
    if name in _SCALARS and not config:
        return np.frombuffer(data, name)[0]
    if name == 'ndarray':
        return _ndarray_decode(config, data)
    raise ValueError(f'oracle does not decode encoding {encoding!r}')


def load_index(dirname: str, split: Optional[str] = None) -> dict[str, Any]:
    with open(os.path.join(dirname, split or '', 'index.json')) as f:
        return json.load(f)


class OracleMDSReader:
    """Per-sample reader over one shard, same algorithm as the reference MDSReader.

    ``data``: the shard file's bytes, read from memory instead of the file (the same reads:
    ``fp.read(n)`` from ``begin`` is ``data[begin:begin + n]``)."""

    def __init__(self, dirname: str, split: Optional[str], info: dict[str, Any],
                 data: Optional[bytes] = None) -> None:
        self.filename = os.path.join(dirname or '', split or '', info['raw_data']['basename'])
        self.column_names = info['column_names']
        self.column_encodings = info['column_encodings']
        self.column_sizes = info['column_sizes']
        self.samples = info['samples']
        self.data = data

    def get_sample_data(self, idx: int) -> bytes:
        offset = (1 + idx) * 4
        if self.data is not None:
            begin, end = np.frombuffer(self.data[offset:offset + 8], np.uint32)
            n = int(end - begin)  # (numpy uint32: wraps where end < begin, as the reference's)
            data = self.data[int(begin):int(begin) + n]
        else:
            with open(self.filename, 'rb', 0) as fp:
                fp.seek(offset)
                pair = fp.read(8)
                begin, end = np.frombuffer(pair, np.uint32)
                fp.seek(begin)
                data = fp.read(end - begin)
        if not data:
            raise IndexError(f'Relative sample index {idx} is not present.')
        return data

    def split_sample(self, data: bytes) -> list[bytes]:
        """Per-column byte slices of one sample (the first half of decode_sample)."""
        sizes, idx = [], 0
        for size in self.column_sizes:
            if size:
                sizes.append(size)
            else:
                size, = np.frombuffer(data[idx:idx + 4], np.uint32)
                sizes.append(int(size))
                idx += 4
        parts = []
        for size in sizes:
            parts.append(data[idx:idx + size])
            idx += size
        return parts

    def decode_sample(self, data: bytes) -> dict[str, Any]:
        return {
            name: mds_decode(enc, part)
            for name, enc, part in zip(self.column_names, self.column_encodings,
                                       self.split_sample(data))
        }

    def get_item(self, idx: int) -> dict[str, Any]:
        return self.decode_sample(self.get_sample_data(idx))

    def __len__(self) -> int:
        return self.samples


class _CostNDArray:
    """``NDArray`` construction as ``_get_coder`` -> ``NDArray.from_str`` does it on EVERY call
    (encodings.py:148-193): split the config, parse the shape, assert the dtype and dims, and
    compute the static size with ``np.prod`` (its decode is the oracle's)."""

    def __init__(self, config: str) -> None:
        args = config.split(':') if config else []
        assert len(args) in {0, 1, 2}
        dtype = args[0] if len(args) >= 1 else None
        shape = tuple(map(int, args[1].split(','))) if len(args) >= 2 else None
        if dtype is not None:
            assert dtype in _VALUE_DTYPES.values()
        if shape is not None:
            for dim in shape:
                assert 1 <= dim
        self.size = None if dtype is None or shape is None else \
            int(np.prod(shape)) * getattr(np, dtype)().nbytes
        self.config = config


def mds_decode_reference_cost(encoding: str, data: bytes) -> Any:
    """``mds_decode`` (encodings.py:760-773) with the per-call coder construction of
    ``_get_coder`` (encodings.py:697-714): a fresh coder object per column per sample (``cls()``,
    ``Scalar.__init__`` computing ``dtype().nbytes``, ``NDArray.from_str``), as the reference
    reader pays it. Same values as :func:`mds_decode`; used for the CPU baseline timing."""
    index = encoding.find(':')
    if index == -1:
        if encoding in _SCALARS:
            getattr(np, encoding)().nbytes  # Scalar.__init__ (encodings.py:308-313)
        elif encoding not in ('bytes', 'str', 'int'):
            raise ValueError(f'oracle does not decode encoding {encoding!r}')
        return mds_decode(encoding, data)
    name, config = encoding[:index], encoding[index + 1:]
    if name != 'ndarray':
        raise ValueError(f'oracle does not decode encoding {encoding!r}')
    coder = _CostNDArray(config)
    return _ndarray_decode(coder.config, data)


class ReferenceCostMDSReader(OracleMDSReader):
    """:class:`OracleMDSReader` whose ``decode_sample`` pays the reference's per-call coder
    construction (:func:`mds_decode_reference_cost`): the CPU baseline of ``bench.py``."""

    def decode_sample(self, data: bytes) -> dict[str, Any]:
        return {
            name: mds_decode_reference_cost(enc, part)
            for name, enc, part in zip(self.column_names, self.column_encodings,
                                       self.split_sample(data))
        }


def utf8_is_valid(data: bytes) -> bool:
    try:
        data.decode('utf-8')
        return True
    except UnicodeDecodeError:
        return False


def decode_shard_columns(dirname: str, split: Optional[str], info: dict[str, Any],
                         data: Optional[bytes] = None) -> dict[str, Any]:
    """Every sample of a shard through the per-sample reader, in the device output format.

    Returns ``{name: ('fixed', rows_bytes[N, size]) | ('ragged', values, offsets, flags)}``
    where ``flags`` is a uint8 array for ``str`` columns (1 = decode raises) else None.
    ``data``: the shard file's bytes (read from memory, OracleMDSReader).
    """
    r = OracleMDSReader(dirname, split, info, data=data)
    n = r.samples
    parts = [r.split_sample(r.get_sample_data(i)) for i in range(n)]
    out: dict[str, Any] = {}
    for c, (name, enc, size) in enumerate(zip(r.column_names, r.column_encodings, r.column_sizes)):
        col = [p[c] for p in parts]
        if size:
            arr = np.frombuffer(b''.join(col), np.uint8).reshape(n, size) if n else np.zeros(
                (0, size), np.uint8)
            out[name] = ('fixed', arr)
        else:
            lens = np.array([len(x) for x in col], np.int64)
            offsets = np.concatenate([np.zeros(1, np.int64), np.cumsum(lens)])
            values = np.frombuffer(b''.join(col), np.uint8)
            flags = None
            if enc == 'str':
                flags = np.array([0 if utf8_is_valid(x) else 1 for x in col], np.uint8)
            out[name] = ('ragged', values, offsets, flags)
    return out


def decode_fixed_shard_vectorized(shard: bytes, column_sizes: list[int]) -> list[np.ndarray]:
    """All-fixed schema: the same per-column slices for every sample, with numpy indexing.

    Equivalent to ``decode_shard_columns`` for schemas with no variable columns (checked by
    tests on small shards); used for full-size parity checks where a per-sample loop is slow.
    """
    buf = np.frombuffer(shard, np.uint8)
    n = int(buf[:4].view(np.uint32)[0])
    offs = buf[4:4 + 4 * (n + 1)].view(np.uint32).astype(np.int64)
    starts = offs[:-1]
    cols, pos = [], 0
    for size in column_sizes:
        col = np.empty((n, size), np.uint8)
        ramp = np.arange(size, dtype=np.int64)[None, :]
        for lo in range(0, n, 1024):  # bounded index arrays
            hi = min(n, lo + 1024)
            col[lo:hi] = buf[starts[lo:hi, None] + pos + ramp]
        cols.append(col)
        pos += size
    return cols


def column_digests(columns: dict[str, Any]) -> dict[str, dict[str, str]]:
    """sha256 of each column's device-format arrays."""
    out = {}
    for name, col in columns.items():
        if col[0] == 'fixed':
            out[name] = {'rows': hashlib.sha256(np.ascontiguousarray(col[1]).tobytes()).hexdigest()}
        else:
            d = {
                'values': hashlib.sha256(np.ascontiguousarray(col[1]).tobytes()).hexdigest(),
                'offsets': hashlib.sha256(np.ascontiguousarray(col[2]).tobytes()).hexdigest(),
            }
            if col[3] is not None:
                d['flags'] = hashlib.sha256(np.ascontiguousarray(col[3]).tobytes()).hexdigest()
            out[name] = d
    return out


def writer_split(sample_sizes, size_limit: Optional[int], extra_per_shard: int,
                 extra_per_sample: int = 4) -> list[int]:
    """Samples per shard, one sample at a time as ``Writer.write`` does
    (base/writer.py:248-269, ``_reset_cache`` :147-152, ``finish`` :289-314)."""
    shards, count, cur = [], 0, extra_per_shard
    for size in sample_sizes:
        new = int(size) + extra_per_sample
        if size_limit and size_limit < cur + new:
            shards.append(count)  # flush_shard, even with nothing cached
            count, cur = 0, extra_per_shard
        count += 1
        cur += new
    if count:
        shards.append(count)
    return shards


def encode_sample_from_columns(columns: list, row: int) -> bytes:
    """``encode_sample`` (mds/writer.py:92-117) of row ``row``: ``columns`` in column order,
    each ``('fixed', uint8[rows, size])`` or ``('var', values uint8, offsets int64)``."""
    heads, body = [], []
    for col in columns:
        if col[0] == 'fixed':
            body.append(col[1][row].tobytes())
        else:
            v = col[1][int(col[2][row]):int(col[2][row + 1])].tobytes()
            heads.append(len(v))
            body.append(v)
    return np.array(heads, np.uint32).tobytes() + b''.join(body)


def encode_joint_shard(config: bytes, samples: list) -> bytes:
    """``encode_joint_shard`` (mds/writer.py:133-144)."""
    n = np.uint32(len(samples))
    sizes = list(map(len, samples))
    offsets = np.array([0] + sizes).cumsum().astype(np.uint32)
    offsets += len(n.tobytes()) + len(offsets.tobytes()) + len(config)
    return n.tobytes() + offsets.tobytes() + config + b''.join(samples)
