"""Device-reader lifecycle without a GPU: the bounded decoded-shard cache (LRU by bytes), eviction
semantics (``evict()`` removes the files and the decoded copy; ``get_item`` then raises
``FileNotFoundError`` as the reference's per-sample ``open`` does, mds/reader.py:137-139, which
drives ``StreamingDataset.get_item``'s prepare-and-retry loop, dataset.py:1274-1291), and the
clear error for a DataLoader worker forked after the parent initialised the GPU."""

import os
import shutil

import pytest
import torch

from streaming_amd import _native
from streaming_amd.cache import DecodedShardCache
from streaming_amd.local import LocalDataset
from streaming_amd.reader import MDSReader
from tests import golden_util as gu


def test_lru_bounds_bytes_and_evicts_oldest():
    c = DecodedShardCache(100)
    c.put(1, 'a', 40)
    c.put(2, 'b', 40)
    assert c.resident_bytes == 80 and len(c) == 2
    assert c.get(1) == 'a'  # 1 is now the most recent
    c.put(3, 'c', 40)  # evicts 2 (least recently used)
    assert 2 not in c and 1 in c and 3 in c
    assert c.resident_bytes == 80 and c.evictions == 1
    c.put(1, 'a2', 90)  # replaced and grown: evicts the others to fit
    assert c.get(1) == 'a2' and c.resident_bytes == 90 and len(c) == 1
    with pytest.warns(UserWarning):
        c.put(4, 'd', 150)  # larger than the limit: kept as the only (most recent) entry
    assert 4 in c and 1 not in c and c.resident_bytes == 150
    c.discard(4)
    assert c.resident_bytes == 0 and len(c) == 0


def test_get_or_create_counts_hits():
    c = DecodedShardCache(10)
    made = []
    assert c.get_or_create(7, lambda: (made.append(1) or 'x', 5)) == 'x'
    assert c.get_or_create(7, lambda: (made.append(1) or 'y', 5)) == 'x'
    assert len(made) == 1 and c.hits == 1 and c.misses == 1
    with pytest.raises(ValueError):
        DecodedShardCache(-1)


def _copy_dataset(tmp_path, name):
    dst = tmp_path / name
    shutil.copytree(os.path.join(gu.GOLDEN, name), dst)
    return str(dst)


def test_evict_removes_files_then_get_item_raises_file_not_found(tmp_path):
    d = _copy_dataset(tmp_path, 'sequence')
    ds = LocalDataset(d, decoded_cache_bytes=1 << 20)
    shard = ds.shards[0]
    path = os.path.join(d, shard.raw_data.basename)
    assert os.path.exists(path)
    assert shard.evict() == shard.raw_data.bytes  # bytes removed, as Reader.evict returns
    assert not os.path.exists(path)
    with pytest.raises(FileNotFoundError):
        shard.get_item(0)  # no GPU needed: the missing file is found before any decode
    with pytest.raises(FileNotFoundError):
        ds[0]
    assert shard.evict() == 0  # nothing left to remove


def test_readers_share_a_dataset_cache(tmp_path):
    d = _copy_dataset(tmp_path, 'kat')
    ds = LocalDataset(d, decoded_cache_bytes=12345)
    assert ds.cache is not None and ds.cache.limit_bytes == 12345
    assert all(s.cache is ds.cache for s in ds.shards)
    other = LocalDataset(d)
    assert other.shards[0].cache is not ds.cache  # default: the process-wide cache


def test_forked_worker_gets_a_clear_error(monkeypatch, tmp_path):
    monkeypatch.setattr(torch.cuda, '_is_in_bad_fork', lambda: True)
    with pytest.raises(RuntimeError, match="multiprocessing_context='spawn'"):
        _native.check_fork()
    d = _copy_dataset(tmp_path, 'kat')
    info = gu.index('kat')['shards'][0]
    r = MDSReader.from_json(d, None, info)
    with pytest.raises(RuntimeError, match='forked after its parent initialised the GPU'):
        r.decode_shard()
