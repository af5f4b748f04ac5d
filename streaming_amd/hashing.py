"""Shard-file checksums: the reference's hashing interface plus xxHash on the device.

Host side mirrors ``streaming/base/hashing.py:14-68`` (same names, argument meaning and errors):
``get_hashes()`` / ``is_hash(algo)`` / ``get_hash(algo, data)`` over hashlib and python-xxhash.

Device side: :func:`hash_device` / :func:`hash_batch` compute the xxHash
family over byte ranges already resident in HBM through ``mdsx_hash_segments`` (libmdsx.so,
``streaming_amd/csrc/mdsx_hash.hip``), returning the same hex digests ``get_hash`` returns, and
:func:`validate_batch` is the device counterpart of the checksum step of
``Stream._prepare_shard_part`` (``stream.py:401-411``): same two ``ValueError`` messages. The
hashlib algorithms (sha*, md5, blake2*) are not offered on the device.
"""

from __future__ import annotations

import hashlib
from typing import Any, Callable, Optional, Sequence

import numpy as np
import torch

from streaming_amd import _native

__all__ = ['get_hashes', 'is_hash', 'get_hash', 'DEVICE_HASHES', 'is_device_hash', 'hash_device',
           'hash_batch', 'validate_batch', 'DeviceHasher', 'hex_digests']


def _collect() -> dict[str, Callable[[bytes], Any]]:
    """hashing.py:14-27: hashlib's algorithms (not shake_*) plus xxhash's."""
    hashes = {}
    for algo in hashlib.algorithms_available:
        if hasattr(hashlib, algo) and not algo.startswith('shake_'):
            hashes[algo] = getattr(hashlib, algo)
    try:
        import xxhash
    except ImportError:  # the reference requires it; without it only hashlib is offered
        return hashes
    for algo in xxhash.algorithms_available:  # type: ignore[attr-defined]
        hashes[algo] = getattr(xxhash, algo)
    return hashes


_hashes = _collect()


def get_hashes() -> set[str]:
    """Supported hash algorithm names (hashing.py:34-40)."""
    return set(_hashes)


def is_hash(algo: str) -> bool:
    """Whether ``algo`` is supported (hashing.py:43-52)."""
    return algo in _hashes


def get_hash(algo: str, data: bytes) -> str:
    """Hex digest of ``data`` (hashing.py:55-68). Raises ``ValueError`` on unknown algorithms."""
    if not is_hash(algo):
        raise ValueError(f'{algo} is not a supported hash algorithm.')
    return _hashes[algo](data).hexdigest()


# name -> (mdsx algorithm id, hex digits of the digest)
DEVICE_HASHES = {
    'xxh32': (_native.HASH_XXH32, 8),
    'xxh64': (_native.HASH_XXH64, 16),
    'xxh3_64': (_native.HASH_XXH3_64, 16),
    'xxh3_128': (_native.HASH_XXH3_128, 32),
    'xxh128': (_native.HASH_XXH3_128, 32),
}


def is_device_hash(algo: str) -> bool:
    """Whether ``algo`` can be computed on the device."""
    return algo in DEVICE_HASHES


class DeviceHasher:
    """Reusable workspace + tables for hashing segments of device buffers on one device."""

    def __init__(self, device: torch.device) -> None:
        self.device = device
        self._ws = torch.empty(0, dtype=torch.uint8, device=device)

    def launch(self, algo: str, data: torch.Tensor, segments: Sequence[tuple[int, int]],
               seed: int = 0) -> tuple[torch.Tensor, torch.Tensor]:
        """Enqueue the hash of every segment on the current stream. Returns the device digests
        (uint64 [n, 2] as int64) and the status record tensor (read after the stream syncs)."""
        if algo not in DEVICE_HASHES:
            raise ValueError(f'{algo} is not a device hash algorithm '
                             f'(device: {sorted(DEVICE_HASHES)}).')
        if data.dtype != torch.uint8 or not data.is_contiguous() or data.device != self.device:
            raise ValueError('data must be a contiguous uint8 tensor on the hasher device')
        lib = _native.lib()
        algo_id = DEVICE_HASHES[algo][0]
        n = len(segments)
        segs = np.asarray(segments, dtype=np.uint64).reshape(n, 2)
        total = int(segs[:, 1].sum()) if n else 0
        need = int(lib.mdsx_hash_workspace_bytes(n, total))
        if self._ws.numel() < need:
            self._ws = torch.empty(need, dtype=torch.uint8, device=self.device)
        d_segs = torch.from_numpy(segs.view(np.int64).copy()).to(self.device, non_blocking=False)
        digests = torch.zeros((max(n, 1), 2), dtype=torch.int64, device=self.device)
        stream = torch.cuda.current_stream(self.device).cuda_stream
        code = lib.mdsx_hash_segments(algo_id, int(seed) & ((1 << 64) - 1), data.data_ptr(),
                                      data.numel(), d_segs.data_ptr(), n, digests.data_ptr(),
                                      self._ws.data_ptr(), self._ws.numel(), stream)
        _native.raise_for_code(code, 'mdsx_hash_segments')
        self._keep = d_segs  # alive until the launch has been consumed
        return digests[:n], self._ws[:16]


_hashers: dict[torch.device, DeviceHasher] = {}


def _hasher(device: torch.device) -> DeviceHasher:
    if device not in _hashers:
        _hashers[device] = DeviceHasher(device)
    return _hashers[device]


def _status_check(status: torch.Tensor) -> None:
    st = _native.Status.from_buffer_copy(status.cpu().numpy().tobytes())
    if st.code == _native.MDSX_E_BOUNDS:
        raise ValueError(f'hash segment {st.shard} lies outside the buffer or is not 16-byte '
                         f'aligned')
    if st.code != 0:
        raise ValueError(f'mdsx_hash_segments reported error {st.code}')


def hex_digests(algo: str, digests: Any) -> list[str]:
    """``get_hash``-format hex strings of device digests (int64 [n, 2] tensor or array)."""
    if isinstance(digests, torch.Tensor):
        digests = digests.cpu().numpy()
    width = DEVICE_HASHES[algo][1]
    out = []
    for lo, hi in np.ascontiguousarray(digests).view(np.uint64).reshape(-1, 2):
        value = (int(hi) << 64) | int(lo)
        out.append(f'{value:0{width}x}')
    return out


def hash_device(algo: str, data: torch.Tensor, segments: Sequence[tuple[int, int]],
                seed: int = 0) -> list[str]:
    """Hex digests (``get_hash`` format) of ``data[offset:offset + bytes]`` for each segment,
    computed on the device. ``data``: contiguous uint8 device tensor; offsets multiples of 16."""
    digests, status = _hasher(data.device).launch(algo, data, segments, seed)
    _status_check(status)
    return hex_digests(algo, digests)


def hash_batch(batch: Any, algo: str, seed: int = 0) -> list[str]:
    """Digest of every shard file of a resident :class:`~streaming_amd.decoder.DeviceBatch`."""
    return hash_device(algo, batch.buffer, list(zip(batch.offsets, batch.sizes)), seed)


def validate_batch(batch: Any, algo: str, expected: Sequence[Optional[dict[str, str]]],
                   filenames: Optional[Sequence[str]] = None) -> None:
    """Checksum step of ``Stream._prepare_shard_part`` (``stream.py:401-411``) for every shard of a
    resident batch: ``expected[s]`` is the shard's ``raw_data.hashes`` from index.json."""
    filenames = filenames or [f'shard {s}' for s in range(batch.nshards)]
    for hashes in expected:
        hashes = hashes or {}
        if algo not in hashes:
            raise ValueError(
                f'Hash algorithm `{algo}` chosen for data ' +
                f'validation does not match with those provided during dataset ' +
                f'creation `{sorted(hashes.keys())}`. Provide one of those.')
    got = hash_batch(batch, algo)
    for digest, hashes, name in zip(got, expected, filenames):
        if digest != hashes[algo]:
            raise ValueError(f'Checksum failure: {name}')


