"""Bounded LRU of decoded shards (device tensors + their host copy).

The reference keeps nothing decoded: every ``get_item`` re-opens the shard file and decodes one
sample (``streaming/base/format/mds/reader.py:128-149``), so its memory is bounded by the disk
cache that ``StreamingDataset`` manages (``cache_limit``, ``evict_shard`` /
``evict_coldest_shard``, ``dataset.py:1113-1140``; ``Reader.evict``,
``format/base/reader.py:128-134``). The device reader decodes a whole shard at a time; this cache
bounds what those decodes keep resident, with two separate bounds:

* ``limit_bytes`` -- decoded outputs in device memory, **per device**. The decodes of a
  ``DataLoader`` run in its worker processes, each with its own copy of the cache; inside a worker
  the bound is split evenly over the loader's ``num_workers`` (``torch.utils.data.
  get_worker_info``), so the workers of one loader together stay within it on their GPU;
* ``host_limit_bytes`` -- the host copies ``get_item`` slices samples from, per process.

When either bound is exceeded the least recently used shards are dropped (their tensors return to
the PyTorch caching allocator) and are decoded again from their files on next use. The most
recently used shard is always kept, even when it alone exceeds a bound (a warning says so once):
repeated reads of one shard never decode it twice.

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
        # key -> [value, device bytes, host bytes]
        self._entries: 'OrderedDict[int, list]' = OrderedDict()
        self._inflight: dict[int, _InFlight] = {}
        self._bytes = 0
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
        """Device bytes of the decoded shards held."""
        return self._bytes

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

    def get_or_create(self, key: int, create: Callable[[], tuple[Any, int]]) -> Any:
        """The value for ``key``, made by ``create() -> (value, device bytes)`` on a miss.

        ``create`` runs without the cache lock held; a second caller of the same key waits for
        it (and gets its error, if it raised)."""
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
            value, nbytes = create()
        except BaseException as e:
            with self._lock:
                self._inflight.pop(key, None)
            flight.error = e
            flight.done.set()
            raise
        with self._lock:
            self._inflight.pop(key, None)
            self.put(key, value, nbytes)
        flight.value = value
        flight.done.set()
        return value

    def __getstate__(self) -> dict:
        # a copy in another process (a spawned DataLoader worker) starts empty, with the same bounds
        return {'limit_bytes': self.limit_bytes, 'host_limit_bytes': self.host_limit_bytes}

    def __setstate__(self, state: dict) -> None:
        self.__init__(state['limit_bytes'], state.get('host_limit_bytes'))

    def put(self, key: int, value: Any, nbytes: int, host_bytes: int = 0) -> None:
        """Insert (or replace) ``key`` as the most recently used entry and evict down to the
        bounds; the entry itself is kept even when it alone exceeds one."""
        with self._lock:
            self.discard(key)
            self._entries[key] = [value, int(nbytes), int(host_bytes)]
            self._bytes += int(nbytes)
            self._host_bytes += int(host_bytes)
            self._shrink()

    def set_host_bytes(self, key: int, host_bytes: int) -> None:
        """Count a resident entry's host copy (added after its decode) and evict to the bounds."""
        with self._lock:
            hit = self._entries.get(key)
            if hit is None:
                return
            self._host_bytes += int(host_bytes) - hit[2]
            hit[2] = int(host_bytes)
            self._entries.move_to_end(key)
            self._shrink()

    def _shrink(self) -> None:
        dev_limit = self.device_limit()
        while len(self._entries) > 1 and (self._bytes > dev_limit or
                                          self._host_bytes > self.host_limit_bytes):
            _, (_, old, old_host) = self._entries.popitem(last=False)
            self._bytes -= old
            self._host_bytes -= old_host
            self.evictions += 1
        if (self._bytes > dev_limit or self._host_bytes > self.host_limit_bytes) and \
                not self._warned:
            self._warned = True
            warnings.warn(f'streaming_amd: one decoded shard ({self._bytes} device bytes, '
                          f'{self._host_bytes} host bytes) exceeds the decoded-shard cache bound '
                          f'({dev_limit} device bytes for this process, {self.host_limit_bytes} '
                          f'host bytes); it is kept while it is the most recently used')

    def discard(self, key: int) -> None:
        with self._lock:
            hit = self._entries.pop(key, None)
            if hit is not None:
                self._bytes -= hit[1]
                self._host_bytes -= hit[2]

    def clear(self) -> None:
        with self._lock:
            self._entries.clear()
            self._bytes = 0
            self._host_bytes = 0


_default: Optional[DecodedShardCache] = None
_default_lock = threading.Lock()


def default_cache() -> DecodedShardCache:
    """The process-wide cache readers share unless given their own."""
    global _default
    with _default_lock:
        if _default is None:
            _default = DecodedShardCache(DEFAULT_CACHE_BYTES)
        return _default
