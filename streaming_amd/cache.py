"""Bounded LRU of decoded shards (device tensors + their host copy).

The reference keeps nothing decoded: every ``get_item`` re-opens the shard file and decodes one
sample (``streaming/base/format/mds/reader.py:128-149``), so its memory is bounded by the disk
cache that ``StreamingDataset`` manages (``cache_limit``, ``evict_shard`` /
``evict_coldest_shard``, ``dataset.py:1113-1140``; ``Reader.evict``,
``format/base/reader.py:128-134``). The device reader decodes a whole shard at a time; this cache
bounds what those decodes keep resident, with two separate bounds:

* ``limit_bytes`` -- decoded outputs in device memory, **per device**: entries are counted
  against the device they were decoded on, so readers on two GPUs sharing one cache object (the
  process-wide default) each get the full bound on their own GPU. The decodes of a ``DataLoader``
  run in its worker processes, each with its own copy of the cache; inside a worker the bound is
  split evenly over the loader's ``num_workers`` (``torch.utils.data.get_worker_info``), so the
  workers of one loader together stay within it on their GPU;
* ``host_limit_bytes`` -- the host copies ``get_item`` slices samples from, per cache object.

When a device's bound is exceeded, that device's least recently used shards are dropped (their
tensors return to the PyTorch caching allocator) and are decoded again from their files on next
use; the host bound drops the least recently used host-holding entries. The most recently used
shard of each device is always kept, even when it alone exceeds a bound (a warning says so once):
repeated reads of one shard never decode it twice. So ``limit_bytes=0`` keeps exactly one decoded
shard per device (the one last used), not none.

``clear()`` and ``discard()`` also cancel decodes in flight: their owner hands the result to the
callers waiting on it but does not insert it.

A miss decodes OUTSIDE the cache lock: readers of other shards keep hitting (and decoding) while
one shard decodes; concurrent first touches of the same shard wait for the one decode in flight.

Entries are keyed by the reader object; a reader's ``evict()`` / ``release()`` drops its entry.
"""

from __future__ import annotations

import os
import threading
import warnings
from collections import OrderedDict
from typing import Any, Callable, Optional

__all__ = ['DecodedShardCache', 'default_cache', 'DEFAULT_CACHE_BYTES', 'worker_share']

# 16 GiB of decoded shards per device unless configured (MDSX_DECODED_CACHE_BYTES); host copies
# get the same bound per process unless configured (MDSX_DECODED_HOST_BYTES).
DEFAULT_CACHE_BYTES = int(os.environ.get('MDSX_DECODED_CACHE_BYTES', 16 << 30))
DEFAULT_HOST_BYTES = int(os.environ.get('MDSX_DECODED_HOST_BYTES', DEFAULT_CACHE_BYTES))


def worker_share() -> int:
    """How many processes share one cache bound: the DataLoader's ``num_workers`` inside a worker
    process, else 1."""
    try:
        from torch.utils.data import get_worker_info
    except ImportError:  # pragma: no cover - torch is a dependency
        return 1
    info = get_worker_info()
    return max(1, int(info.num_workers)) if info is not None else 1


class _InFlight:
    """One decode in progress: the threads that touch the same key meanwhile wait for it."""

    def __init__(self) -> None:
        self.done = threading.Event()
        self.value: Any = None
        self.error: Optional[BaseException] = None
        self.cancelled = False  # clear() / discard() ran meanwhile: do not insert the result


class DecodedShardCache:
    """LRU of decoded shards, bounded by ``limit_bytes`` of device memory per device (split over
    the DataLoader workers sharing the device) and ``host_limit_bytes`` of host copies."""

    def __init__(self, limit_bytes: int = DEFAULT_CACHE_BYTES,
                 host_limit_bytes: Optional[int] = None) -> None:
        if limit_bytes < 0:
            raise ValueError(f'limit_bytes must be >= 0, got {limit_bytes}')
        if host_limit_bytes is None:
            host_limit_bytes = limit_bytes if limit_bytes != DEFAULT_CACHE_BYTES else \
                DEFAULT_HOST_BYTES
        if host_limit_bytes < 0:
            raise ValueError(f'host_limit_bytes must be >= 0, got {host_limit_bytes}')
        self.limit_bytes = int(limit_bytes)
        self.host_limit_bytes = int(host_limit_bytes)
        self._lock = threading.RLock()
        # key -> [value, device bytes, host bytes, device]
        self._entries: 'OrderedDict[int, list]' = OrderedDict()
        self._inflight: dict[int, _InFlight] = {}
        self._device_bytes: dict[Any, int] = {}
        self._host_bytes = 0
        self._warned = False
        self.hits = 0
        self.misses = 0
        self.evictions = 0

    # -- bounds --------------------------------------------------------------------------------
    def device_limit(self) -> int:
        """This process's device-byte bound: ``limit_bytes`` split over the DataLoader workers."""
        return self.limit_bytes // worker_share()

    @property
    def resident_bytes(self) -> int:
        """Device bytes of the decoded shards held (all devices)."""
        return sum(self._device_bytes.values())

    def device_bytes(self, device: Any = None) -> int:
        """Device bytes of the decoded shards held on ``device``."""
        return self._device_bytes.get(device, 0)

    @property
    def resident_host_bytes(self) -> int:
        """Host bytes of the host copies held."""
        return self._host_bytes

    def __len__(self) -> int:
        return len(self._entries)

    def __contains__(self, key: int) -> bool:
        return key in self._entries

    # -- access --------------------------------------------------------------------------------
    def get(self, key: int) -> Optional[Any]:
        with self._lock:
            hit = self._entries.get(key)
            if hit is None:
                return None
            self._entries.move_to_end(key)
            return hit[0]

    def lookup(self, key: int) -> Optional[Any]:
        """The value for ``key`` if it is cached (a hit, made the most recently used), else None
        (not counted as a miss: the caller goes on to :meth:`get_or_create`)."""
        with self._lock:
            hit = self._entries.get(key)
            if hit is None:
                return None
            self._entries.move_to_end(key)
            self.hits += 1
            return hit[0]

    def get_or_create(self, key: int, create: Callable[[], tuple]) -> Any:
        """The value for ``key``, made by ``create() -> (value, device bytes[, device])`` on a
        miss.

        ``create`` runs without the cache lock held; a second caller of the same key waits for
        it (and gets its error, if it raised). A ``clear()`` / ``discard(key)`` meanwhile cancels
        the insertion (the callers still get the value)."""
        with self._lock:
            hit = self._entries.get(key)
            if hit is not None:
                self._entries.move_to_end(key)
                self.hits += 1
                return hit[0]
            flight = self._inflight.get(key)
            owner = flight is None
            if owner:
                flight = self._inflight[key] = _InFlight()
                self.misses += 1
            else:
                self.hits += 1
        if not owner:
            flight.done.wait()
            if flight.error is not None:
                raise flight.error
            return flight.value
        try:
            made = create()
            value, nbytes = made[0], made[1]
            device = made[2] if len(made) > 2 else None
        except BaseException as e:
            with self._lock:
                self._inflight.pop(key, None)
            flight.error = e
            flight.done.set()
            raise
        with self._lock:
            self._inflight.pop(key, None)
            if not flight.cancelled:
                self.put(key, value, nbytes, device=device)
        flight.value = value
        flight.done.set()
        return value

    def __getstate__(self) -> dict:
        # a copy in another process (a spawned DataLoader worker) starts empty, with the same bounds
        return {'limit_bytes': self.limit_bytes, 'host_limit_bytes': self.host_limit_bytes}

    def __setstate__(self, state: dict) -> None:
        self.__init__(state['limit_bytes'], state.get('host_limit_bytes'))

    def put(self, key: int, value: Any, nbytes: int, host_bytes: int = 0,
            device: Any = None) -> None:
        """Insert (or replace) ``key`` as the most recently used entry of ``device`` and evict
        down to the bounds; the entry itself is kept even when it alone exceeds one."""
        with self._lock:
            self._drop(key)
            self._entries[key] = [value, int(nbytes), int(host_bytes), device]
            self._device_bytes[device] = self._device_bytes.get(device, 0) + int(nbytes)
            self._host_bytes += int(host_bytes)
            self._shrink(key)

    def set_host_bytes(self, key: int, host_bytes: int) -> None:
        """Count a resident entry's host copy (added after its decode) and evict to the bounds."""
        with self._lock:
            hit = self._entries.get(key)
            if hit is None:
                return
            self._host_bytes += int(host_bytes) - hit[2]
            hit[2] = int(host_bytes)
            self._entries.move_to_end(key)
            self._shrink(key)

    def _shrink(self, newest: int) -> None:
        """Evict to the bounds after ``newest`` was inserted or grew: the device bound over the
        entries of its device, the host bound over every entry; ``newest`` itself stays."""
        dev_limit = self.device_limit()
        device = self._entries[newest][3]
        for key in [k for k, e in self._entries.items() if e[3] == device and k != newest]:
            if self._device_bytes.get(device, 0) <= dev_limit:
                break
            self._drop(key)
            self.evictions += 1
        for key in [k for k, e in self._entries.items() if e[2] and k != newest]:
            if self._host_bytes <= self.host_limit_bytes:
                break
            self._drop(key)
            self.evictions += 1
        over_dev = self._device_bytes.get(device, 0) > dev_limit
        if (over_dev or self._host_bytes > self.host_limit_bytes) and not self._warned:
            self._warned = True
            warnings.warn(f'streaming_amd: one decoded shard ({self._device_bytes.get(device, 0)} '
                          f'device bytes, {self._host_bytes} host bytes) exceeds the decoded-shard '
                          f'cache bound ({dev_limit} device bytes for this process, '
                          f'{self.host_limit_bytes} host bytes); it is kept while it is the most '
                          f'recently used')

    def _drop(self, key: int) -> None:
        hit = self._entries.pop(key, None)
        if hit is not None:
            self._device_bytes[hit[3]] -= hit[1]
            self._host_bytes -= hit[2]

    def discard(self, key: int) -> None:
        """Drop ``key`` (and cancel the insertion of a decode of it in flight)."""
        with self._lock:
            self._drop(key)
            flight = self._inflight.get(key)
            if flight is not None:
                flight.cancelled = True

    def clear(self) -> None:
        """Drop every entry (and cancel the insertion of every decode in flight)."""
        with self._lock:
            self._entries.clear()
            self._device_bytes.clear()
            self._host_bytes = 0
            for flight in self._inflight.values():
                flight.cancelled = True


_default: Optional[DecodedShardCache] = None
_default_lock = threading.Lock()


def default_cache() -> DecodedShardCache:
    """The process-wide cache readers share unless given their own."""
    global _default
    with _default_lock:
        if _default is None:
            _default = DecodedShardCache(DEFAULT_CACHE_BYTES)
        return _default
