"""Device batches in the reference's sample order: the sample ids the real
reference's generate_work laid out for config A (tests/golden/order), per worker, from the start
of the epoch and resumed mid-epoch, gathered on the GPU through LocalDataset.iter_batches
(shards decoded on demand through a bounded decoded-shard cache) must be the reference's samples
in the reference's order, bit-exact: the recorded __iter__ digests for single-worker settings,
the oracle's values at every id for all settings."""

import pytest
import torch

from streaming_amd.local import LocalDataset
from streaming_amd.order import worker_sample_ids
from tests import golden_util as gu
from tests.test_order import digest, fixture_ids, oracle_rows, settings

pytestmark = pytest.mark.gpu

BATCH = 16


def _rows(batch):
    nums = batch['number'].cpu().tolist()
    col = batch['words']
    vals, offs = col.values.cpu().numpy(), col.offsets.cpu().numpy()
    words = [vals[offs[i]:offs[i + 1]].tobytes().decode('utf-8') for i in range(batch.rows)]
    assert col.flags is None or int(col.flags.sum()) == 0
    return nums, words


def _iterate(ds, ids):
    numbers, words = [], []
    for b in ds.iter_batches(ids, BATCH):
        n, w = _rows(b)
        assert len(n) <= BATCH
        numbers += n
        words += w
    return numbers, words


@pytest.mark.parametrize('name', ['noshuffle_w1', 'py1e_w1'])
@pytest.mark.parametrize('tag', ['start', 'resume'])
def test_reference_iteration_digest(name, tag):
    s = settings()[name]
    ds = LocalDataset(gu.GOLDEN + '/config_a', decoded_cache_bytes=1 << 20)
    ids = worker_sample_ids(fixture_ids()[f'{name}.{tag}'], 0, 0, 0)
    numbers, words = _iterate(ds, ids)
    assert len(numbers) == s[f'iter_{tag}_count']
    assert digest(numbers, words) == s[f'iter_{tag}_sha256']
    assert ds.cache.resident_bytes <= ds.cache.limit_bytes


@pytest.mark.parametrize('name', ['py1s_n1r2w2', 'py1br_n2r2w1'])
@pytest.mark.parametrize('tag', ['start', 'resume'])
def test_every_worker_in_order(name, tag):
    s = settings()[name]
    nodes, rpn, wpr = s['world']
    onum, owords = oracle_rows()
    # a cache smaller than one shard's decoded bytes: every shard decoded again on each visit
    ds = LocalDataset(gu.GOLDEN + '/config_a', decoded_cache_bytes=4096)
    for n in range(nodes):
        for r in range(rpn):
            for w in range(wpr):
                ids = worker_sample_ids(fixture_ids()[f'{name}.{tag}'], n, r, w)
                ids = ids[ids != -1]
                numbers, words = _iterate(ds, ids)
                assert numbers == onum[ids].tolist()
                assert words == [owords[i] for i in ids]


def test_missing_shard_raises_file_not_found(tmp_path):
    import shutil
    d = tmp_path / 'a'
    shutil.copytree(gu.GOLDEN + '/config_a', d)
    ds = LocalDataset(str(d), decoded_cache_bytes=1 << 20)
    first = next(iter(ds.iter_batches(list(range(20)), 20)))
    assert first.rows == 20
    ds.shards[0].evict()  # files gone, decoded copy dropped
    with pytest.raises(FileNotFoundError):
        next(iter(ds.iter_batches([0, 1], 2)))
    torch.cuda.synchronize()
