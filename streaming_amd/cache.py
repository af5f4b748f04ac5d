"""Bounded, per-process LRU of decoded shards (device tensors + their host copy).

The reference keeps nothing decoded: every ``get_item`` re-opens the shard file and decodes one
sample (``streaming/base/format/mds/reader.py:128-149``), so its memory is bounded by the disk
cache that ``StreamingDataset`` manages (``cache_limit``, ``evict_shard`` /
``evict_coldest_shard``, ``dataset.py:1113-1140``; ``Reader.evict``,
``format/base/reader.py:128-134``). The device reader decodes a whole shard at a time; this cache
bounds what those decodes keep resident: when the bytes of the shards held exceed the limit, the
least recently used shards are dropped (their tensors return to the PyTorch caching allocator)
and are decoded again from their files on next use.

Entries are keyed by the reader object; a reader's ``evict()`` / ``release()`` drops its entry.
"""

from __future__ import annotations

import os
import threading
from collections import OrderedDict
from typing import Any, Callable, Optional

__all__ = ['DecodedShardCache', 'default_cache', 'DEFAULT_CACHE_BYTES']

# 16 GiB of decoded shards per process unless configured (MDSX_DECODED_CACHE_BYTES).
DEFAULT_CACHE_BYTES = int(os.environ.get('MDSX_DECODED_CACHE_BYTES', 16 << 30))


class DecodedShardCache:
    """LRU of decoded shards, bounded by ``limit_bytes`` (device bytes of the decoded outputs).

    A single shard larger than the limit is still decoded and returned, but not kept.
    """

    def __init__(self, limit_bytes: int = DEFAULT_CACHE_BYTES) -> None:
        if limit_bytes < 0:
            raise ValueError(f'limit_bytes must be >= 0, got {limit_bytes}')
        self.limit_bytes = int(limit_bytes)
        self._lock = threading.RLock()
        self._entries: 'OrderedDict[int, tuple[Any, int]]' = OrderedDict()
        self._bytes = 0
        self.hits = 0
        self.misses = 0
        self.evictions = 0

    @property
    def resident_bytes(self) -> int:
        return self._bytes

    def __len__(self) -> int:
        return len(self._entries)

    def __contains__(self, key: int) -> bool:
        return key in self._entries

    def get(self, key: int) -> Optional[Any]:
        with self._lock:
            hit = self._entries.get(key)
            if hit is None:
                return None
            self._entries.move_to_end(key)
            return hit[0]

    def get_or_create(self, key: int, create: Callable[[], tuple[Any, int]]) -> Any:
        """The value for ``key``, made by ``create() -> (value, nbytes)`` on a miss."""
        with self._lock:
            value = self.get(key)
            if value is not None:
                self.hits += 1
                return value
            self.misses += 1
            value, nbytes = create()
            self.put(key, value, nbytes)
            return value

    def __getstate__(self) -> dict:
        # a copy in another process (a spawned DataLoader worker) starts empty, with the same bound
        return {'limit_bytes': self.limit_bytes}

    def __setstate__(self, state: dict) -> None:
        self.__init__(state['limit_bytes'])

    def put(self, key: int, value: Any, nbytes: int) -> None:
        with self._lock:
            self.discard(key)
            if nbytes > self.limit_bytes:
                return
            while self._entries and self._bytes + nbytes > self.limit_bytes:
                _, (_, old) = self._entries.popitem(last=False)
                self._bytes -= old
                self.evictions += 1
            self._entries[key] = (value, int(nbytes))
            self._bytes += int(nbytes)

    def update(self, key: int, value: Any, nbytes: int) -> None:
        """Replace the value of a resident key (e.g. add its host copy) and re-count its bytes."""
        with self._lock:
            if key in self._entries:
                self.put(key, value, nbytes)

    def discard(self, key: int) -> None:
        with self._lock:
            hit = self._entries.pop(key, None)
            if hit is not None:
                self._bytes -= hit[1]

    def clear(self) -> None:
        with self._lock:
            self._entries.clear()
            self._bytes = 0


_default: Optional[DecodedShardCache] = None
_default_lock = threading.Lock()


def default_cache() -> DecodedShardCache:
    """The process-wide cache readers share unless given their own."""
    global _default
    with _default_lock:
        if _default is None:
            _default = DecodedShardCache(DEFAULT_CACHE_BYTES)
        return _default
