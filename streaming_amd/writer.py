"""MDSWriter: writes MDS shards + ``index.json`` byte-identical to the reference writer.

Restates the format producer of the reference (``streaming/base/format/mds/writer.py:18-144``,
``streaming/base/format/base/writer.py:30-314``) for local output directories: the on-disk
layout is the spec the device decoder parses, and the writer is how synthetic shards are made on
a GPU box that has no copy of the reference. Remote upload (``CloudUploader``) is out of scope;
``out`` must be a local directory.

Shard layout (``encode_joint_shard``, mds/writer.py:133-144)::

    u32 N | u32 offsets[N+1] (absolute) | config JSON (sort_keys) | sample 0 | ... | sample N-1

Sample layout (``encode_sample``, mds/writer.py:92-117)::

    u32 size of each variable column, in column order | column payloads in column order

Columns are in sorted-name order (mds/writer.py:76).

:func:`encode_fixed_shard` is the vectorised form of the same layout for all-fixed schemas,
used to build large synthetic shards quickly (bit-identical to the per-sample writer).
"""

from __future__ import annotations

import hashlib
import json
import logging
import os
import shutil
from types import TracebackType
from typing import Any, Optional, Sequence, Union

import numpy as np

from streaming_amd.compression import compress, get_compression_extension, is_compression
from streaming_amd.encodings import get_mds_encoded_size, get_mds_encodings, is_mds_encoding, \
    mds_encode

__all__ = ['MDSWriter', 'bytes_to_int', 'encode_fixed_shard', 'shard_config_bytes',
           'get_index_basename']

logger = logging.getLogger(__name__)


def get_index_basename() -> str:
    """``index.json`` (streaming/base/format/index.py:9-15)."""
    return 'index.json'


_UNITS = {
    'kb': 1024,
    'mb': 1024**2,
    'gb': 1024**3,
    'tb': 1024**4,
    'pb': 1024**5,
    'eb': 1024**6,
    'zb': 1024**7,
    'yb': 1024**8
}


def bytes_to_int(value: Union[int, float, str]) -> int:
    """Human-readable byte size to int (streaming/base/util.py:74-123)."""
    if isinstance(value, (int, float)):
        return int(value)
    text = value.lower().strip()
    for suffix, mult in _UNITS.items():
        if text.endswith(suffix):
            try:
                return int(float(text[:-len(suffix)]) * mult)
            except ValueError:
                break
    else:
        if text.endswith('b') and text[:-1].isdigit():
            return int(text[:-1])
        if text.isdigit():
            return int(text)
    raise ValueError(f'Unsupported value/suffix {text}. Supported suffix are '
                     f'{["b"] + list(_UNITS)}.')


def _hash(algo: str, data: bytes) -> str:
    if algo in hashlib.algorithms_available and hasattr(hashlib, algo) and \
            not algo.startswith('shake_'):
        return getattr(hashlib, algo)(data).hexdigest()
    import xxhash
    if algo in xxhash.algorithms_available:  # type: ignore[attr-defined]
        return getattr(xxhash, algo)(data).hexdigest()
    raise ValueError(f'{algo} is not a supported hash algorithm.')


def _is_hash(algo: str) -> bool:
    try:
        _hash(algo, b'')
        return True
    except (ValueError, ImportError):
        return False


def shard_config_bytes(column_names: Sequence[str], column_encodings: Sequence[str],
                       column_sizes: Sequence[Optional[int]], compression: Optional[str],
                       hashes: Sequence[str], size_limit: Optional[int]) -> bytes:
    """The config JSON embedded in every shard (mds/writer.py:86-88, base/writer.py:229-241)."""
    obj = {
        'version': 2,
        'format': 'mds',
        'compression': compression,
        'hashes': list(hashes),
        'size_limit': size_limit,
        'column_names': list(column_names),
        'column_encodings': list(column_encodings),
        'column_sizes': list(column_sizes),
    }
    return json.dumps(obj, sort_keys=True).encode('utf-8')


def encode_fixed_shard(config: bytes, columns: Sequence[np.ndarray]) -> bytes:
    """Vectorised ``encode_joint_shard`` for an all-fixed schema.

    Args:
        config: shard config JSON bytes.
        columns: per column (in column order) a C-contiguous array whose leading dimension is
            the sample count; row i's bytes are that column's encoded value of sample i.
    """
    n = int(columns[0].shape[0]) if columns else 0
    rows = [np.ascontiguousarray(c).reshape(n, -1).view(np.uint8) for c in columns]
    sample = sum(r.shape[1] for r in rows)
    header = 4 + 4 * (n + 1) + len(config)
    out = np.empty(header + n * sample, np.uint8)
    out[:4] = np.frombuffer(np.uint32(n).tobytes(), np.uint8)
    offsets = header + sample * np.arange(n + 1, dtype=np.uint64)
    if n and offsets[-1] >= 1 << 32:
        raise ValueError('shard larger than the u32 offset range')
    out[4:4 + 4 * (n + 1)] = offsets.astype(np.uint32).view(np.uint8)
    out[4 + 4 * (n + 1):header] = np.frombuffer(config, np.uint8)
    body = out[header:].reshape(n, sample)
    pos = 0
    for r in rows:
        body[:, pos:pos + r.shape[1]] = r
        pos += r.shape[1]
    return out.tobytes()


class MDSWriter:
    """Writes a streaming MDS dataset to a local directory.

    Args mirror the reference (mds/writer.py:56-90, base/writer.py:66-143):
        columns (Dict[str, str]): column name -> encoding.
        out (str): local output directory.
        keep_local (bool): accepted for API compatibility (output is always local).
        compression (str, optional): ``None``, ``'zstd'``, ``'zstd:<level>'``, ``'gz'``,
            ``'gz:<level>'``, ``'bz2'``, ``'bz2:<level>'``.
        hashes (List[str], optional): sorted hash algorithms recorded per shard file.
        size_limit (int | str, optional): shard size limit (default ``1 << 26``).
        exist_ok (bool): remove an existing non-empty ``out`` first.
    """

    format = 'mds'
    extra_bytes_per_sample = 4

    def __init__(self,
                 *,
                 columns: dict[str, str],
                 out: Union[str, tuple[str, str]],
                 keep_local: bool = False,
                 compression: Optional[str] = None,
                 hashes: Optional[list[str]] = None,
                 size_limit: Optional[Union[int, str]] = 1 << 26,
                 **kwargs: Any) -> None:
        compression = compression or None
        if compression and not is_compression(compression):
            raise ValueError(f'Invalid compression: {compression}.')
        hashes = hashes or []
        if list(hashes) != sorted(hashes):
            raise ValueError('Hashes must be unique and in sorted order.')
        for algo in hashes:
            if not _is_hash(algo):
                raise ValueError(f'Invalid hash: {algo}.')
        size_limit_value = None
        if size_limit:
            size_limit_value = bytes_to_int(size_limit)
            if size_limit_value < 0:
                raise ValueError(f'`size_limit` must be greater than zero, instead, '
                                 f'found as {size_limit_value}.')
            if size_limit_value >= 2**32:
                raise ValueError(f'`size_limit` must be less than 2**32, instead, '
                                 f'found as {size_limit_value}. This is because sample '
                                 f'byte offsets are stored with uint32.')
        invalid = [k for k in kwargs if k not in ('progress_bar', 'max_workers', 'retry', 'exist_ok')]
        if invalid:
            raise ValueError(f'Invalid Writer argument(s): {invalid} ')
        if isinstance(out, tuple):
            if out[1]:
                raise ValueError('remote upload is out of scope for streaming_amd.MDSWriter')
            out = out[0]
        local = os.path.expanduser(out)
        if os.path.exists(local) and os.listdir(local):
            if kwargs.get('exist_ok', False):
                shutil.rmtree(local)
            else:
                raise FileExistsError(f'Directory is not empty: {local}')
        os.makedirs(local, exist_ok=True)
        self.local = local
        self.keep_local = keep_local
        self.compression = compression
        self.hashes = list(hashes)
        self.size_limit = size_limit_value
        self.shards: list[dict[str, Any]] = []

        self.columns = columns
        self.column_names: list[str] = []
        self.column_encodings: list[str] = []
        self.column_sizes: list[Optional[int]] = []
        for name in sorted(columns):
            encoding = columns[name]
            if not is_mds_encoding(encoding):
                raise TypeError(f'MDSWriter passed column `{name}` with encoding `{encoding}` ' +
                                f'is unsupported. Supported encodings are {get_mds_encodings()}')
            self.column_names.append(name)
            self.column_encodings.append(encoding)
            self.column_sizes.append(get_mds_encoded_size(encoding))
        self.config_data = shard_config_bytes(self.column_names, self.column_encodings,
                                              self.column_sizes, self.compression, self.hashes,
                                              self.size_limit)
        self.extra_bytes_per_shard = 4 + 4 + len(self.config_data)
        self._reset_cache()

    def _reset_cache(self) -> None:
        self.new_samples: list[bytes] = []
        self.new_shard_size = self.extra_bytes_per_shard
        self._dev_pending: list = []  # open shard's rows from write_columns (device columns)

    def get_config(self) -> dict[str, Any]:
        return json.loads(self.config_data)

    def encode_sample(self, sample: dict[str, Any]) -> bytes:
        """Sample -> bytes (mds/writer.py:92-117)."""
        sizes, data = [], []
        for key, encoding, size in zip(self.column_names, self.column_encodings,
                                       self.column_sizes):
            datum = mds_encode(encoding, sample[key])
            if size is None:
                sizes.append(len(datum))
            elif size != len(datum):
                raise KeyError(f'Unexpected data size; was this data typed with the correct ' +
                               f'encoding ({encoding})?')
            data.append(datum)
        return np.array(sizes, np.uint32).tobytes() + b''.join(data)

    def encode_joint_shard(self) -> bytes:
        """Cached samples -> shard file bytes (mds/writer.py:133-144)."""
        n = len(self.new_samples)
        sizes = np.array([0] + [len(s) for s in self.new_samples], np.int64)
        offsets = (np.cumsum(sizes) + 4 + 4 * (n + 1) + len(self.config_data)).astype(np.uint32)
        return (np.uint32(n).tobytes() + offsets.tobytes() + self.config_data +
                b''.join(self.new_samples))

    def write(self, sample: dict[str, Any]) -> None:
        """Cache a sample, flushing a shard first if it would pass size_limit
        (base/writer.py:248-269)."""
        if self._dev_pending:
            raise ValueError('write: rows from write_columns are pending in the open shard')
        new_sample = self.encode_sample(sample)
        new_size = len(new_sample) + self.extra_bytes_per_sample
        if self.size_limit and self.size_limit < self.new_shard_size + new_size:
            self.flush_shard()
            self._reset_cache()
        self.new_samples.append(new_sample)
        self.new_shard_size += new_size

    def write_columns(self, columns: dict[str, Any]) -> None:
        """Write a batch of rows given as device columns, encoded on the GPU.

        ``columns``: name -> fixed tensor ``[rows, ...]`` (the column's encoded bytes per row,
        e.g. ``int32[rows]`` or ``float32[rows, 1024]``) or ``RaggedColumn`` (each row's encoded
        bytes, ``mds_encode`` output). Produces the same shards as :meth:`write` called per row
        (the split of ``Writer.write``, base/writer.py:248-269); the open shard's rows stay on
        the device until more rows arrive or :meth:`finish`. See ``streaming_amd.encoder``.
        """
        from streaming_amd.encoder import concat_columns, encode_batch, slice_columns
        from streaming_amd.reader import get_plan
        if self.new_samples:
            raise ValueError('write_columns: rows cached by write() are pending in the open shard')
        plan = get_plan(self.column_names, self.column_encodings, self.column_sizes)
        fresh = not self.shards and not self._dev_pending
        cols = concat_columns(self._dev_pending + [columns])
        enc, consumed = encode_batch(plan, cols, self.config_data, self.size_limit, fresh=fresh,
                                     final=False)
        self._write_encoded(enc)
        first = next(iter(cols.values()))
        rows = len(first) if not hasattr(first, 'shape') else int(first.shape[0])
        self._dev_pending = [slice_columns(cols, consumed, rows)] if consumed < rows else []

    def _flush_device(self) -> None:
        from streaming_amd.encoder import concat_columns, encode_batch
        from streaming_amd.reader import get_plan
        plan = get_plan(self.column_names, self.column_encodings, self.column_sizes)
        enc, _ = encode_batch(plan, concat_columns(self._dev_pending), self.config_data,
                              self.size_limit, fresh=not self.shards, final=True)
        self._dev_pending = []
        self._write_encoded(enc)

    def _write_encoded(self, enc: Any) -> None:
        if enc is None:
            return
        for s, (b, e) in enumerate(enc.bounds):
            self._write_shard_file(enc.shard_bytes(s), e - b)

    def write_encoded_shard(self, raw: bytes, samples: int) -> None:
        """Write an already-encoded shard file (e.g. from :func:`encode_fixed_shard`)."""
        self._write_shard_file(raw, samples)

    def _name_next_shard(self) -> tuple[str, Optional[str]]:
        raw = f'shard.{len(self.shards):05}.{self.format}'
        if self.compression:
            return raw, f'{raw}.{get_compression_extension(self.compression)}'
        return raw, None

    def _file_info(self, data: bytes, basename: str) -> dict[str, Any]:
        return {
            'basename': basename,
            'bytes': len(data),
            'hashes': {algo: _hash(algo, data) for algo in self.hashes}
        }

    def _write_shard_file(self, raw_data: bytes, samples: int) -> None:
        raw_name, zip_name = self._name_next_shard()
        raw_info = self._file_info(raw_data, raw_name)
        if zip_name:
            zip_data = compress(self.compression, raw_data)
            zip_info = self._file_info(zip_data, zip_name)
            data, name = zip_data, zip_name
        else:
            zip_info, data, name = None, raw_data, raw_name
        with open(os.path.join(self.local, name), 'wb') as f:
            f.write(data)
        obj = {'samples': samples, 'raw_data': raw_info, 'zip_data': zip_info}
        obj.update(self.get_config())
        self.shards.append(obj)

    def flush_shard(self) -> None:
        self._write_shard_file(self.encode_joint_shard(), len(self.new_samples))

    def _write_index(self) -> None:
        if self.new_samples:
            raise RuntimeError('Internal error: not all samples have been written.')
        with open(os.path.join(self.local, get_index_basename()), 'w') as out:
            json.dump({'version': 2, 'shards': self.shards}, out, sort_keys=True)

    def finish(self) -> None:
        """Flush the last shard and write ``index.json`` (base/writer.py:289-314)."""
        if self._dev_pending:
            self._flush_device()
        if self.new_samples:
            self.flush_shard()
            self._reset_cache()
        self._write_index()

    def __enter__(self) -> 'MDSWriter':
        return self

    def __exit__(self, exc_type: Optional[type[BaseException]], exc: Optional[BaseException],
                 traceback: Optional[TracebackType]) -> None:
        self.finish()
