"""Device-reader lifecycle on the GPU (ADVICE / VERDICT round 1): eviction releases the decoded
shard and turns later reads into FileNotFoundError; the decoded-shard cache stays within its bound
while a dataset is read; a malformed sample fails only its own reads; spawned DataLoader workers
decode in their own processes; the shard pipeline raises on a malformed early batch."""

import json
import os
import shutil

import numpy as np
import pytest
import torch

from oracle import mds_oracle
from streaming_amd.local import LocalDataset
from streaming_amd.pipeline import ShardPipeline, shard_files_from_index
from streaming_amd.reader import get_plan
from tests import golden_util as gu

pytestmark = pytest.mark.gpu

A = os.path.join(gu.GOLDEN, 'config_a')


def _copy(tmp_path, name='config_a'):
    d = tmp_path / name
    shutil.copytree(os.path.join(gu.GOLDEN, name), d)
    return str(d)


def _oracle_item(dirname, info, i):
    return mds_oracle.OracleMDSReader(dirname, None, info).get_item(i)


def test_evict_releases_decoded_shard_then_file_not_found(tmp_path):
    d = _copy(tmp_path)
    ds = LocalDataset(d, decoded_cache_bytes=64 << 20)
    r = ds.shards[3]
    info = gu.index('config_a')['shards'][3]
    assert r.get_item(2) == _oracle_item(A, info, 2)
    held = ds.cache.resident_bytes
    assert held > 0 and r._key in ds.cache
    r.evict()
    assert r._key not in ds.cache and ds.cache.resident_bytes < held
    with pytest.raises(FileNotFoundError):
        r.get_item(2)
    with pytest.raises(FileNotFoundError):
        r.decode_shard()


def test_cache_bound_holds_while_reading(tmp_path):
    limit = 24 << 10  # a few decoded shards of config A
    ds = LocalDataset(A, decoded_cache_bytes=limit)
    idx = gu.index('config_a')['shards']
    rng = np.random.default_rng(5)
    starts = np.concatenate([[0], np.cumsum([s['samples'] for s in idx])])
    for gid in rng.integers(0, len(ds), 300):
        s = int(np.searchsorted(starts, gid, side='right') - 1)
        assert ds[int(gid)] == _oracle_item(A, idx[s], int(gid - starts[s]))
        assert ds.cache.resident_bytes <= limit
    assert ds.cache.evictions > 0 and ds.cache.hits > 0


def _corrupt_empty_sample(path, k):
    """Sample k of the shard made empty (offsets[k + 1] = offsets[k]; sample k + 1 then spans
    both samples' bytes)."""
    with open(path, 'r+b') as f:
        f.seek(4 * (1 + k))
        begin = f.read(4)
        f.seek(4 * (2 + k))
        f.write(begin)


def test_malformed_sample_fails_only_its_own_reads(tmp_path):
    d = _copy(tmp_path)
    info = gu.index('config_a')['shards'][0]
    path = os.path.join(d, info['raw_data']['basename'])
    _corrupt_empty_sample(path, 5)
    ds = LocalDataset(d, decoded_cache_bytes=1 << 20)
    r = ds.shards[0]
    with pytest.raises(IndexError):
        r.get_item(5)
    for i in range(info['samples']):
        if i == 5:
            continue
        assert r.get_item(i) == _oracle_item(d, info, i), i  # the reference's bytes, sample i
    # the batch path: a batch holding the bad sample raises, the others decode
    good = [i for i in range(info['samples']) if i != 5]
    out = next(iter(ds.iter_batches(good, len(good))))
    assert out['number'].cpu().tolist() == [_oracle_item(d, info, i)['number'] for i in good]
    with pytest.raises(IndexError):
        next(iter(ds.iter_batches([4, 5], 2)))


def test_dataloader_spawn_workers():
    ds = LocalDataset(A, decoded_cache_bytes=1 << 20)
    loader = torch.utils.data.DataLoader(ds, batch_size=50, num_workers=2, collate_fn=list,
                                         multiprocessing_context='spawn')
    idx = gu.index('config_a')['shards']
    want = [_oracle_item(A, info, i) for info in idx for i in range(info['samples'])]
    got = [s for batch in loader for s in batch]
    assert got == want


def test_pipeline_raises_on_malformed_first_batch(tmp_path):
    d = _copy(tmp_path)
    idx = json.load(open(os.path.join(d, 'index.json')))
    _corrupt_empty_sample(os.path.join(d, idx['shards'][1]['raw_data']['basename']), 2)
    info = idx['shards'][0]
    plan = get_plan(info['column_names'], info['column_encodings'], info['column_sizes'])
    pipe = ShardPipeline(plan, shard_files_from_index(d, idx), shards_per_batch=4, depth=2)
    it = iter(pipe)
    with pytest.raises(IndexError):
        next(it)  # the first batch holds shard 1: raised before it is handed out
    pipe.close()


class _CacheProbe(torch.utils.data.Dataset):
    """A dataset reporting, with each sample, its worker's decoded-shard cache occupancy."""

    def __init__(self, ds):
        self.ds = ds

    def __len__(self):
        return len(self.ds)

    def __getitem__(self, i):
        c = self.ds.cache
        sample = self.ds[i]
        return os.getpid(), c.resident_bytes, c.device_limit(), sample


def test_dataloader_workers_share_the_device_bound():
    """Spawned workers each hold an equal share of the decoded-shard bound, so the loader's
    workers together never keep more device bytes than the bound."""
    bound = 24 << 10  # a few decoded shards of config A
    ds = LocalDataset(A, decoded_cache_bytes=bound)
    loader = torch.utils.data.DataLoader(_CacheProbe(ds), batch_size=50, num_workers=2,
                                         collate_fn=list, multiprocessing_context='spawn')
    peak, limits, got = {}, set(), []
    for batch in loader:
        for pid, resident, limit, sample in batch:
            peak[pid] = max(peak.get(pid, 0), resident)
            limits.add(limit)
            got.append(sample)
    idx = gu.index('config_a')['shards']
    assert got == [_oracle_item(A, info, i) for info in idx for i in range(info['samples'])]
    assert len(peak) == 2 and limits == {bound // 2}
    assert sum(peak.values()) <= bound, peak
