"""Whole-file shard compression codecs used by the writer and by the host prepare step.

Mirrors the reference's names, extensions and default levels (``streaming/base/compression.py:
79-166``, ``get_compression_extension``/``compress``/``decompress`` at ``:210-258``) for the
codecs available in this image: ``zstd`` (system ``libzstd.so.1`` through ctypes; the reference
binds the ``zstd`` pip package), ``gz`` and ``bz2`` (standard library). ``br`` and ``snappy``
need packages that are not installed and raise ``ValueError`` like an unknown codec.

Decompression is the host stage in front of the device decoder (config E: host decompress ->
pinned H2D -> device decode). ``decompress_into`` writes straight into a caller buffer (e.g. a
pinned staging tensor) to avoid one host copy.
"""

from __future__ import annotations

import bz2
import ctypes
import ctypes.util
import gzip
import threading
from typing import Optional

import numpy as np

__all__ = [
    'compress', 'decompress', 'decompress_into', 'get_compression_extension', 'get_compressions',
    'is_compression', 'zstd_available', 'zstd_frame_content_size'
]

_families = {
    # extension: (default level, levels)
    'bz2': (9, list(range(1, 10))),
    'gz': (9, list(range(10))),
    'zstd': (3, list(range(1, 23))),
}

_zstd_lock = threading.Lock()
_zstd: Optional[ctypes.CDLL] = None
_ZSTD_CONTENTSIZE_UNKNOWN = (1 << 64) - 1
_ZSTD_CONTENTSIZE_ERROR = (1 << 64) - 2


def _libzstd() -> ctypes.CDLL:
    global _zstd
    if _zstd is None:
        with _zstd_lock:
            if _zstd is None:
                name = ctypes.util.find_library('zstd') or 'libzstd.so.1'
                handle = ctypes.CDLL(name)
                handle.ZSTD_compressBound.restype = ctypes.c_size_t
                handle.ZSTD_compressBound.argtypes = [ctypes.c_size_t]
                handle.ZSTD_compress.restype = ctypes.c_size_t
                handle.ZSTD_compress.argtypes = [
                    ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                    ctypes.c_int
                ]
                handle.ZSTD_decompress.restype = ctypes.c_size_t
                handle.ZSTD_decompress.argtypes = [
                    ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t
                ]
                handle.ZSTD_getFrameContentSize.restype = ctypes.c_ulonglong
                handle.ZSTD_getFrameContentSize.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
                handle.ZSTD_isError.restype = ctypes.c_uint
                handle.ZSTD_isError.argtypes = [ctypes.c_size_t]
                handle.ZSTD_getErrorName.restype = ctypes.c_char_p
                handle.ZSTD_getErrorName.argtypes = [ctypes.c_size_t]
                _zstd = handle
    return _zstd


def zstd_available() -> bool:
    try:
        _libzstd()
        return True
    except OSError:
        return False


def _all_algos() -> set[str]:
    algos = set()
    for ext, (_, levels) in _families.items():
        if ext == 'zstd' and not zstd_available():
            continue
        algos.add(ext)
        algos.update(f'{ext}:{lvl}' for lvl in levels)
    return algos


def get_compressions() -> set[str]:
    return _all_algos()


def is_compression(algo: Optional[str]) -> bool:
    return algo in _all_algos()


def _split(algo: str) -> tuple[str, int]:
    if not is_compression(algo):
        raise ValueError(f'{algo} is not a supported compression algorithm.')
    ext, _, lvl = algo.partition(':')
    return ext, int(lvl) if lvl else _families[ext][0]


def get_compression_extension(algo: str) -> str:
    return _split(algo)[0]


def _zstd_err(code: int) -> str:
    return _libzstd().ZSTD_getErrorName(code).decode()


def zstd_frame_content_size(data: bytes) -> int:
    z = _libzstd()
    size = z.ZSTD_getFrameContentSize(data, len(data))
    if size in (_ZSTD_CONTENTSIZE_UNKNOWN, _ZSTD_CONTENTSIZE_ERROR):
        raise ValueError('zstd frame without a known content size')
    return int(size)


def compress(algo: Optional[str], data: bytes) -> bytes:
    if algo is None:
        return data
    ext, level = _split(algo)
    if ext == 'gz':
        return gzip.compress(data, level)
    if ext == 'bz2':
        return bz2.compress(data, level)
    z = _libzstd()
    bound = z.ZSTD_compressBound(len(data))
    out = ctypes.create_string_buffer(bound)
    n = z.ZSTD_compress(out, bound, data, len(data), level)
    if z.ZSTD_isError(n):
        raise ValueError(f'zstd compress failed: {_zstd_err(n)}')
    return out.raw[:n]


def decompress_into(algo: str, data: bytes, out: np.ndarray) -> int:
    """Decompress into ``out`` (a writable uint8 array, e.g. a pinned staging view)."""
    ext, _ = _split(algo)
    if ext != 'zstd':
        raw = decompress(algo, data)
        out[:len(raw)] = np.frombuffer(raw, np.uint8)
        return len(raw)
    z = _libzstd()
    if not out.flags.c_contiguous or out.dtype != np.uint8:
        raise ValueError('out must be a contiguous uint8 array')
    n = z.ZSTD_decompress(out.ctypes.data, out.nbytes, data, len(data))
    if z.ZSTD_isError(n):
        raise ValueError(f'zstd decompress failed: {_zstd_err(n)}')
    return int(n)


def decompress(algo: Optional[str], data: bytes) -> bytes:
    if algo is None:
        return data
    ext, _ = _split(algo)
    if ext == 'gz':
        return gzip.decompress(data)
    if ext == 'bz2':
        return bz2.decompress(data)
    out = np.empty(zstd_frame_content_size(data), np.uint8)
    n = decompress_into(algo, data, out)
    return out[:n].tobytes()
