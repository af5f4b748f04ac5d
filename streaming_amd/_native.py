"""ctypes binding of libmdsx.so, the C ABI declared in ``include/mdsx.h``.

The library is the product path: there is no CPU fallback. If it is missing or fails to load,
every decode entry point raises :class:`NativeLibraryError`.

This module imports torch before loading the library so that the HIP runtime torch ships
(``libamdhip64.so.7``) is the one the library binds to: one runtime, one device context.
"""

from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

import torch  # noqa: F401  (must be loaded before libmdsx.so, see module docstring)

__all__ = [
    'NativeLibraryError', 'MDSX_OK', 'MDSX_E_ARG', 'MDSX_E_ENCODING', 'MDSX_E_HEADER',
    'MDSX_E_BOUNDS', 'MDSX_E_HIP', 'MDSX_E_CAPACITY', 'MDSX_E_EMPTY', 'KIND_FIXED', 'KIND_BYTES',
    'KIND_STR', 'KIND_NDARRAY', 'ShardDesc', 'ColumnOut', 'Batch', 'Status', 'lib', 'lib_path',
    'EXPORTED_SYMBOLS', 'raise_for_code', 'Segment', 'HASH_XXH32', 'HASH_XXH64', 'HASH_XXH3_64',
    'HASH_XXH3_128'
]

MDSX_OK = 0
MDSX_E_ARG = -1
MDSX_E_ENCODING = -2
MDSX_E_HEADER = -3
MDSX_E_BOUNDS = -4
MDSX_E_HIP = -5
MDSX_E_CAPACITY = -6
MDSX_E_EMPTY = -7

KIND_FIXED = 0
KIND_BYTES = 1
KIND_STR = 2
KIND_NDARRAY = 3

MAX_COLUMNS = 64
BATCH_PAD = 256
GATHER_SRC_SHIFT = 40  # MDSX_GATHER_SRC_SHIFT: multi-source gather ids are source << 40 | row

# Every function include/mdsx.h declares (checked by tests/test_native_abi.py).
EXPORTED_SYMBOLS = (
    'mdsx_version',
    'mdsx_last_error',
    'mdsx_last_kernel',
    'mdsx_plan_create',
    'mdsx_plan_destroy',
    'mdsx_plan_num_columns',
    'mdsx_plan_num_var',
    'mdsx_plan_tile_rows',
    'mdsx_plan_tile_rows_for',
    'mdsx_plan_column',
    'mdsx_plan_is_safe',
    'mdsx_workspace_bytes',
    'mdsx_scan_shards',
    'mdsx_decode_shards',
    'mdsx_decode_shards_single',
    'mdsx_decode_sample',
    'mdsx_copy_probe',
    'mdsx_copy_probe_variant',
    'mdsx_copy_to_host',
    'mdsx_gather_workspace_bytes',
    'mdsx_gather_fixed',
    'mdsx_gather_ragged_scan',
    'mdsx_gather_ragged_copy',
    'mdsx_gather_fixed_multi',
    'mdsx_gather_ragged_scan_multi',
    'mdsx_gather_ragged_copy_multi',
    'mdsx_ndarray_meta',
    'mdsx_ndarray_shapes',
    'mdsx_plan_encode_tile_rows',
    'mdsx_encode_workspace_bytes',
    'mdsx_encode_sizes',
    'mdsx_encode_shards',
    'mdsx_hash_workspace_bytes',
    'mdsx_hash_segments',
)

HASH_XXH32 = 1
HASH_XXH64 = 2
HASH_XXH3_64 = 3
HASH_XXH3_128 = 4


class NativeLibraryError(RuntimeError):
    """libmdsx.so is missing or could not be loaded (the decoder has no CPU fallback)."""


class ShardDesc(ctypes.Structure):
    """``mdsx_shard_desc``."""
    _fields_ = [('offset', ctypes.c_uint64), ('bytes', ctypes.c_uint64), ('row0', ctypes.c_uint64),
                ('samples', ctypes.c_uint32), ('tile0', ctypes.c_uint32)]


class ColumnOut(ctypes.Structure):
    """``mdsx_column_out``."""
    _fields_ = [('data', ctypes.c_void_p), ('offsets', ctypes.c_void_p), ('flags', ctypes.c_void_p),
                ('capacity', ctypes.c_uint64)]


class ColumnIn(ctypes.Structure):
    """``mdsx_column_in``."""
    _fields_ = [('data', ctypes.c_void_p), ('offsets', ctypes.c_void_p), ('bytes', ctypes.c_uint64),
                ('reserved', ctypes.c_uint64)]


class Batch(ctypes.Structure):
    """``mdsx_batch``."""
    _fields_ = [('data', ctypes.c_void_p), ('bytes', ctypes.c_uint64), ('shards', ctypes.c_void_p),
                ('tile_shard', ctypes.c_void_p), ('nshards', ctypes.c_int32),
                ('ntiles', ctypes.c_uint32), ('rows', ctypes.c_uint64),
                ('tile_rows', ctypes.c_uint32), ('reserved', ctypes.c_uint32)]


class Status(ctypes.Structure):
    """``mdsx_status``."""
    _fields_ = [('code', ctypes.c_int32), ('shard', ctypes.c_int32), ('row', ctypes.c_int32),
                ('column', ctypes.c_int32)]


class Segment(ctypes.Structure):
    """``mdsx_segment``."""
    _fields_ = [('offset', ctypes.c_uint64), ('bytes', ctypes.c_uint64)]


assert ctypes.sizeof(ShardDesc) == 32
assert ctypes.sizeof(ColumnOut) == 32
assert ctypes.sizeof(Batch) == 56

_here = os.path.dirname(os.path.abspath(__file__))
# MDSX_LIBRARY: another build of the library (measurement A/B of kernel variants in one run)
lib_path = os.environ.get('MDSX_LIBRARY') or os.path.join(_here, 'lib', 'libmdsx.so')

_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None


def _declare(handle: ctypes.CDLL) -> None:
    c_int, c_u32, c_u64, vp = ctypes.c_int, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_void_p
    handle.mdsx_version.restype = ctypes.c_char_p
    handle.mdsx_version.argtypes = []
    handle.mdsx_last_error.restype = ctypes.c_char_p
    handle.mdsx_last_error.argtypes = []
    handle.mdsx_last_kernel.restype = ctypes.c_char_p
    handle.mdsx_last_kernel.argtypes = []
    handle.mdsx_plan_create.restype = c_int
    handle.mdsx_plan_create.argtypes = [
        ctypes.POINTER(ctypes.c_char_p),
        ctypes.POINTER(ctypes.c_int64), c_int,
        ctypes.POINTER(vp)
    ]
    handle.mdsx_plan_destroy.restype = None
    handle.mdsx_plan_destroy.argtypes = [vp]
    for name in ('mdsx_plan_num_columns', 'mdsx_plan_num_var', 'mdsx_plan_tile_rows',
                 'mdsx_plan_is_safe'):
        fn = getattr(handle, name)
        fn.restype = c_int
        fn.argtypes = [vp]
    handle.mdsx_plan_tile_rows_for.restype = c_int
    handle.mdsx_plan_tile_rows_for.argtypes = [vp, c_u64, c_u64]
    handle.mdsx_plan_column.restype = c_int
    handle.mdsx_plan_column.argtypes = [
        vp, c_int,
        ctypes.POINTER(c_int),
        ctypes.POINTER(ctypes.c_int64),
        ctypes.POINTER(c_int)
    ]
    pb = ctypes.POINTER(Batch)
    handle.mdsx_workspace_bytes.restype = c_u64
    handle.mdsx_workspace_bytes.argtypes = [vp, pb]
    handle.mdsx_scan_shards.restype = c_int
    handle.mdsx_scan_shards.argtypes = [vp, pb, ctypes.POINTER(ColumnOut), vp, c_u64, vp, vp]
    handle.mdsx_decode_shards.restype = c_int
    handle.mdsx_decode_shards.argtypes = [vp, pb, ctypes.POINTER(ColumnOut), vp, c_u64, vp]
    handle.mdsx_decode_shards_single.restype = c_int
    handle.mdsx_decode_shards_single.argtypes = [
        vp, pb, ctypes.POINTER(ColumnOut), ctypes.POINTER(c_u64), vp, c_u64, vp, vp
    ]
    handle.mdsx_decode_sample.restype = c_int
    handle.mdsx_decode_sample.argtypes = [vp, vp, c_u32, vp, vp, vp]
    handle.mdsx_copy_probe.restype = c_int
    handle.mdsx_copy_probe.argtypes = [vp, vp, c_u64, vp]
    handle.mdsx_copy_probe_variant.restype = c_int
    handle.mdsx_copy_probe_variant.argtypes = [vp, vp, c_u64, c_int, vp]
    handle.mdsx_copy_to_host.restype = c_int
    handle.mdsx_copy_to_host.argtypes = [vp, vp, c_u64, vp]
    handle.mdsx_ndarray_meta.restype = c_int
    handle.mdsx_ndarray_meta.argtypes = [vp, vp, c_u64, c_int, vp, vp, vp, vp, vp, vp, vp]
    handle.mdsx_ndarray_shapes.restype = c_int
    handle.mdsx_ndarray_shapes.argtypes = [vp, vp, c_u64, c_int, ctypes.c_int32, vp, vp]
    handle.mdsx_plan_encode_tile_rows.restype = c_int
    handle.mdsx_plan_encode_tile_rows.argtypes = [vp]
    handle.mdsx_encode_workspace_bytes.restype = c_u64
    handle.mdsx_encode_workspace_bytes.argtypes = []
    handle.mdsx_encode_sizes.restype = c_int
    handle.mdsx_encode_sizes.argtypes = [vp, ctypes.POINTER(ColumnIn), c_u64, vp, vp, c_u64, vp]
    handle.mdsx_encode_shards.restype = c_int
    handle.mdsx_encode_shards.argtypes = [
        vp, ctypes.POINTER(Batch), ctypes.POINTER(ColumnIn), vp, vp, ctypes.c_uint32, vp, c_u64, vp
    ]
    handle.mdsx_hash_workspace_bytes.restype = c_u64
    handle.mdsx_hash_workspace_bytes.argtypes = [c_int, c_u64]
    handle.mdsx_hash_segments.restype = c_int
    handle.mdsx_hash_segments.argtypes = [c_int, c_u64, vp, c_u64, vp, c_int, vp, vp, c_u64, vp]
    handle.mdsx_gather_workspace_bytes.restype = c_u64
    handle.mdsx_gather_workspace_bytes.argtypes = [c_u64]
    handle.mdsx_gather_fixed.restype = c_int
    handle.mdsx_gather_fixed.argtypes = [vp, c_u64, c_u64, vp, c_u64, vp, vp, c_u64, vp]
    handle.mdsx_gather_ragged_scan.restype = c_int
    handle.mdsx_gather_ragged_scan.argtypes = [vp, c_u64, vp, c_u64, vp, vp, c_u64, vp, vp]
    handle.mdsx_gather_ragged_copy.restype = c_int
    handle.mdsx_gather_ragged_copy.argtypes = [
        vp, vp, vp, c_u64, vp, c_u64, vp, c_u64, vp, vp, vp, c_u64, vp
    ]
    handle.mdsx_gather_fixed_multi.restype = c_int
    handle.mdsx_gather_fixed_multi.argtypes = [vp, c_u32, c_u64, vp, c_u64, vp, vp, c_u64, vp]
    handle.mdsx_gather_ragged_scan_multi.restype = c_int
    handle.mdsx_gather_ragged_scan_multi.argtypes = [vp, c_u32, vp, c_u64, vp, vp, c_u64, vp, vp]
    handle.mdsx_gather_ragged_copy_multi.restype = c_int
    handle.mdsx_gather_ragged_copy_multi.argtypes = [
        vp, c_u32, vp, c_u64, vp, c_u64, vp, vp, vp, c_u64, vp
    ]


def lib() -> ctypes.CDLL:
    """Load (once) and return libmdsx.so.

    Raises:
        NativeLibraryError: if the shared library is absent or cannot be loaded.
    """
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(lib_path):
                raise NativeLibraryError(
                    f'libmdsx.so not found at {lib_path}: build it with '
                    f'`python -c "import __graft_entry__ as g; g.build()"` '
                    f'(or python -m streaming_amd.build). There is no CPU fallback.')
            try:
                handle = ctypes.CDLL(lib_path)
            except OSError as e:
                raise NativeLibraryError(f'failed to load {lib_path}: {e}') from e
            _declare(handle)
            _lib = handle
    return _lib


def last_error() -> str:
    msg = lib().mdsx_last_error()
    return msg.decode('utf-8', 'replace') if msg else ''


def check_fork() -> None:
    """Raise a clear error in a process forked after its parent initialised the GPU.

    A ``torch.utils.data.DataLoader`` worker started with the default ``fork`` context inherits
    a parent that has touched the GPU (training code usually has) and cannot use the GPU itself.
    The device readers decode inside the worker, so such loaders need
    ``multiprocessing_context='spawn'`` (or ``'forkserver'``)."""
    if torch.cuda._is_in_bad_fork():
        raise RuntimeError(
            'streaming_amd: this process was forked after its parent initialised the GPU, so it '
            'cannot decode shards on the GPU. Create the DataLoader with '
            "multiprocessing_context='spawn' (or 'forkserver'), e.g. DataLoader(dataset, "
            "num_workers=4, multiprocessing_context='spawn').")


def require_gpu() -> None:
    """Fail loudly where a decode would need the GPU and there is none: the package has no CPU
    fallback (its only CPU decoder is the test oracle, which it never calls)."""
    if not torch.cuda.is_available():
        raise RuntimeError('streaming_amd decodes MDS shards on the GPU (HIP, gfx950), and no GPU '
                           'is visible to this process.')


def last_kernel() -> str:
    """Template name of the decode kernel this thread launched last (rocprofv3's name)."""
    name = lib().mdsx_last_kernel()
    return name.decode() if name else ''


def raise_for_code(code: int, where: str) -> None:
    """Map an MDSX_E_* code to the exception type the reference raises for that condition."""
    if code == MDSX_OK:
        return
    msg = f'{where}: {last_error()}'
    if code == MDSX_E_ENCODING:
        raise ValueError(msg)
    if code == MDSX_E_ARG:
        raise ValueError(msg)
    if code == MDSX_E_EMPTY:
        raise IndexError(msg)
    if code in (MDSX_E_HEADER, MDSX_E_BOUNDS):
        raise ValueError(msg)
    raise RuntimeError(f'{msg} (mdsx code {code})')
