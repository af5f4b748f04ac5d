"""A read-only list of items that can be fancy indexed like a numpy array.

Same indexing contract as the reference's ``Array`` (``streaming/base/array.py:12-110``):
subclasses provide ``size`` and ``get_item(0 <= idx < size)``; ``__getitem__`` accepts an int,
a slice, a list (recursively) or a numpy array (recursively).
"""

from __future__ import annotations

from typing import Any, Iterator, Union

import numpy as np
from numpy.typing import NDArray

__all__ = ['Array']


class Array:
    """Fancy-indexable read-only sequence."""

    @property
    def size(self) -> int:
        raise NotImplementedError

    def get_item(self, idx: int) -> Any:
        raise NotImplementedError

    def _each_slice_index(self, at: slice) -> Iterator[int]:
        # Slice bounds as array.py:44-76 resolves them (negative indices wrap once).
        size = self.size
        start = 0 if at.start is None else at.start
        if at.start is not None and -size <= start < 0:
            start += size
        stop = size if at.stop is None else at.stop
        if at.stop is not None and -size <= stop < 0:
            stop += size
        step = 1 if at.step is None else at.step
        if step > 0:
            start, stop = max(start, 0), min(stop, size)
        else:
            stop, start = max(stop, -1), min(start, size - 1)
        yield from range(start, stop, step)

    def __getitem__(self, at: Union[int, slice, list, NDArray[np.int64]]) -> Any:
        if isinstance(at, (int, np.integer)):
            if -self.size <= at < 0:
                at += self.size
            return self.get_item(at)
        if isinstance(at, slice):
            return [self.get_item(i) for i in self._each_slice_index(at)]
        if isinstance(at, (list, np.ndarray)):
            return [self.__getitem__(sub) for sub in at]
        raise ValueError(f'Unsupported argument type passed to __getitem__: {type(at)}.')
