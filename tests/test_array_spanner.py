"""Host-side index plumbing the device reader keeps from the reference: ``Array`` fancy indexing
(``streaming/base/array.py:12-110``) and ``Spanner`` (``streaming/base/spanner.py:10-59``).

The cases restate the reference's own tests (``tests/test_array.py``: ints from both ends and
out of range, every slice with start / stop in {-142 .. 142} and steps +-1, +-3, the named slice
list, nested lists and 1-3-d index arrays, all checked against numpy indexing of the same range;
``tests/test_spanner.py``: 19 shards of 5..95 samples, every global index, and out-of-range ids).
"""

import numpy as np
import pytest

from streaming_amd.array import Array
from streaming_amd.spanner import Spanner


class Range(Array):
    """``Array`` over 0..n-1 (get_item asserts the contract 0 <= idx < size)."""

    def __init__(self, n: int) -> None:
        self.n = n

    @property
    def size(self) -> int:
        return self.n

    def get_item(self, idx: int) -> int:
        assert 0 <= idx < self.n
        return idx


def _same_as_numpy(index) -> None:
    ref = np.arange(100)
    try:
        want = ref[index]
        want = want.tolist() if isinstance(want, np.ndarray) else want
    except Exception:
        want = None
    try:
        got = Range(100)[index]
    except Exception:
        got = None
    assert got == want, index


BOUNDS = [-142, -100, -99, -42, -1, 0, 42, 99, 100, 142]
NAMED_SLICES = [
    slice(0), slice(0, 0), slice(0, 1), slice(1, 2, 3), slice(2, 3, 1), slice(0, 6, 2),
    slice(0, 10), slice(10, 10), slice(10, 20, 2), slice(20, 10, -1), slice(1337, 42, -3),
    slice(-3, 3), slice(1337, 42, -5), slice(1337, 4, -5), slice(1337, -4, -5),
    slice(1337, -42, -5), slice(1337, -1337, -5), slice(1338, 42, -5), slice(-1337, 42, 5),
    slice(-1337, 42, -5)
]


def test_ints_both_ends_and_out_of_range():
    for i in list(range(-100, 100)) + list(range(-400, 400, 10)):
        _same_as_numpy(i)
        _same_as_numpy(np.int64(i))


@pytest.mark.parametrize('step', [-3, -1, 1, 3])
def test_every_slice(step):
    for start in BOUNDS:
        for stop in BOUNDS:
            _same_as_numpy(slice(start, stop, step))


def test_open_bounds_follow_the_reference_not_numpy():
    """array.py:50-75 resolves an omitted start to 0 and an omitted stop to size whatever the
    step, so a negative step with an open bound is not numpy's reversed range."""
    r = Range(100)
    assert r[::1] == list(range(100)) and r[:10] == list(range(10)) and r[90:] == list(range(90, 100))
    assert r[::-1] == [] and r[42::-1] == [] and r[:-142:-1] == [0]
    assert r[:0:-1] == [] and r[-1::-1] == []


def test_named_slices_and_their_index_lists():
    r = Range(100)
    for s in NAMED_SLICES:
        _same_as_numpy(s)
        as_list = list(r._each_slice_index(s))
        _same_as_numpy(as_list)
        _same_as_numpy(np.array(as_list, dtype=np.int64))


@pytest.mark.parametrize('shape', [(5, 4), (3, 3, 4), (3, 4), (3, 2, 3)])
def test_nested_lists_and_arrays(shape):
    idx = (np.arange(int(np.prod(shape))) * 2 + 7).reshape(shape)
    assert Range(100)[idx.tolist()] == np.arange(100)[idx].tolist()
    _same_as_numpy(idx)


def test_unsupported_index_type():
    with pytest.raises(ValueError):
        Range(10)['3']


def test_spanner_every_index():
    sizes = np.arange(5, 100, 5)
    sp = Spanner(sizes, 7)
    g = 0
    for shard, n in enumerate(sizes):
        for k in range(n):
            assert sp[g] == (shard, k)
            g += 1
    ids = np.arange(g)
    shards, local = sp.locate(ids)
    want = [sp[int(i)] for i in ids]
    assert list(zip(shards.tolist(), local.tolist())) == want


@pytest.mark.parametrize('index', [-10, -1, 2000, 950])
def test_spanner_invalid_index(index):
    sp = Spanner(np.arange(5, 100, 5), 7)  # 950 samples
    with pytest.raises(IndexError, match='Invalid sample index'):
        sp[index]
    with pytest.raises(IndexError, match='Invalid sample index'):
        sp.locate(np.array([0, index]))
