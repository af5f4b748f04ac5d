"""Global sample index -> (shard, index inside the shard).

Same mapping as the reference's ``Spanner`` (``streaming/base/spanner.py:10-59``), computed with
one ``searchsorted`` over the shard boundaries instead of span lists; batched lookups
(:meth:`Spanner.locate`) map a whole vector of sample ids at once for the device gather.
"""

from __future__ import annotations

from bisect import bisect_right

import numpy as np
from numpy.typing import NDArray

__all__ = ['Spanner']


class Spanner:
    """Args:
        shard_sizes: samples in each shard.
        span_size: kept for API compatibility with the reference (unused).
    """

    def __init__(self, shard_sizes: NDArray[np.int64], span_size: int = 1 << 10) -> None:
        self.shard_sizes = np.asarray(shard_sizes, np.int64)
        self.span_size = span_size
        self.num_samples = int(self.shard_sizes.sum())
        self.shard_bounds = np.concatenate([np.zeros(1, np.int64), self.shard_sizes.cumsum()])
        self._bounds = self.shard_bounds.tolist()  # (per-sample lookups: bisect on python ints)

    def __getitem__(self, index: int) -> tuple[int, int]:
        if not (0 <= index < self.num_samples):
            raise IndexError(f'Invalid sample index `{index}`: 0 <= {index} < {self.num_samples}')
        shard = bisect_right(self._bounds, index) - 1
        return shard, int(index) - self._bounds[shard]

    def locate(self, indices: NDArray[np.int64]) -> tuple[NDArray[np.int64], NDArray[np.int64]]:
        """Vectorised ``__getitem__``: (shard ids, indices inside the shards)."""
        idx = np.asarray(indices, np.int64)
        if idx.size and (idx.min() < 0 or idx.max() >= self.num_samples):
            raise IndexError(f'Invalid sample index in batch: 0 <= ids < {self.num_samples}')
        shards = np.searchsorted(self.shard_bounds, idx, side='right') - 1
        return shards, idx - self.shard_bounds[shards]
