"""The device encoder's shard split (``streaming_amd.encoder.split_shards``, a prefix rule over
cumulative sizes) against the reference writer's per-sample greedy loop (oracle
``writer_split``, base/writer.py:248-269), and the oracle loop against the host MDSWriter."""

import numpy as np
import pytest

from oracle import mds_oracle
from streaming_amd.encoder import split_shards


def _cum4(sizes):
    cum = np.zeros(len(sizes) + 1, np.int64)
    cum[1:] = np.cumsum(np.asarray(sizes, np.int64) + 4)
    return cum


@pytest.mark.parametrize('seed', range(40))
def test_split_matches_writer_loop(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(1, 3000))
    mode = seed % 4
    if mode == 0:
        sizes = rng.integers(1, 200, n)
    elif mode == 1:
        sizes = np.full(n, int(rng.integers(1, 5000)))
    elif mode == 2:  # some samples above the limit
        sizes = np.where(rng.random(n) < 0.05, 50_000, rng.integers(0, 3000, n))
    else:
        sizes = rng.integers(0, 10, n)
    limit = [None, 1 << 12, 1 << 14, 3000, 100][seed % 5]
    extra = 8 + int(rng.integers(50, 400))
    bounds = split_shards(_cum4(sizes), limit, extra, fresh=True)
    assert [e - b for b, e in bounds] == mds_oracle.writer_split(sizes, limit, extra)
    assert bounds[0][0] == 0 and bounds[-1][1] == n
    assert all(bounds[i][1] == bounds[i + 1][0] for i in range(len(bounds) - 1))


def test_oversized_first_sample_flushes_empty_shard():
    sizes = [10_000, 10, 10, 10_000, 10_000, 5]
    extra = 200
    assert mds_oracle.writer_split(sizes, 4096, extra) == [0, 1, 2, 1, 1, 1]
    assert [e - b for b, e in split_shards(_cum4(sizes), 4096, extra)] == [0, 1, 2, 1, 1, 1]
    # a continuing writer (samples already cached) never flushes an empty shard
    assert [e - b for b, e in split_shards(_cum4(sizes), 4096, extra, fresh=False)] == \
        [1, 2, 1, 1, 1]


def test_oracle_split_matches_host_writer(tmp_path):
    from streaming_amd.writer import MDSWriter
    rng = np.random.default_rng(5)
    sizes = np.where(rng.random(500) < 0.02, 9000, rng.integers(0, 900, 500))
    sizes[0] = 9000
    with MDSWriter(columns={'b': 'bytes'}, out=str(tmp_path), size_limit=4096) as w:
        for s in sizes:
            w.write({'b': bytes(int(s))})
        extra = w.extra_bytes_per_shard
        size_of = [len(w.encode_sample({'b': bytes(int(s))})) for s in sizes]
    got = [sh['samples'] for sh in w.shards]
    assert got == mds_oracle.writer_split(size_of, 4096, extra)
    assert got[0] == 0


def test_empty_and_unlimited():
    assert split_shards(np.zeros(1, np.int64), 1 << 26, 300) == []
    assert split_shards(_cum4([5, 6, 7]), None, 300) == [(0, 3)]
