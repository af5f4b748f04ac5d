"""device_iter on the GPU: StreamingDataset.__iter__'s control flow yielding
device batches, the rows gathered on the device from the shards' decoded columns, must give the
reference's own iteration -- the sha256 digests its __iter__ recorded on config A
(tests/golden/order), from the epoch start and after a mid-epoch checkpoint -- through the
iteration surface of a stand-in dataset (tests/standin_dataset.py; the same loop over the real
StreamingDataset is checked in the build container, tests/test_plugin_reference.py)."""

import pytest
import torch

from streaming_amd.local import LocalDataset
from streaming_amd.order import worker_sample_ids
from streaming_amd.plugin import DeviceBatches, device_iter
from tests import golden_util as gu
from tests.standin_dataset import StandInDataset
from tests.test_order import digest, fixture_ids, settings

pytestmark = pytest.mark.gpu


def _rows(batches):
    numbers, words, sizes = [], [], []
    for b in batches:
        assert b.sample_ids is not None and len(b.sample_ids) == b.rows
        numbers += b['number'].cpu().tolist()
        col = b['words']
        vals, offs = col.values.cpu().numpy(), col.offsets.cpu().numpy()
        words += [vals[offs[i]:offs[i + 1]].tobytes().decode('utf-8') for i in range(b.rows)]
        sizes.append(b.rows)
    return numbers, words, sizes


@pytest.mark.parametrize('name', ['noshuffle_w1', 'py1e_w1'])
def test_device_iter_start_and_resume(name):
    s = settings()[name]
    ids = fixture_ids()
    ds = LocalDataset(gu.GOLDEN + '/config_a', decoded_cache_bytes=1 << 20)

    def work(epoch, sample_in_epoch):
        tag = 'start' if sample_in_epoch == 0 else 'resume'
        assert sample_in_epoch in (0, s['resume_at'])
        return worker_sample_ids(ids[f'{name}.{tag}'], 0, 0, 0)

    standin = StandInDataset(ds.shards, work)
    numbers, words, sizes = _rows(device_iter(standin, 16))
    assert len(numbers) == s['iter_start_count']
    assert digest(numbers, words) == s['iter_start_sha256']
    assert all(n == 16 for n in sizes[:-1])
    assert (standin._shard_access_times > 0).all()  # get_item's access-time touch
    # a checkpoint of the samples handed out, then a new iteration resumes there
    batches = DeviceBatches(standin, 16)
    it = iter(batches)
    while batches.num_samples_yielded < s['resume_at']:
        next(it)
    assert batches.num_samples_yielded == s['resume_at']
    standin._iterator.exit()
    standin.load_state_dict({'epoch': 0, 'sample_in_epoch': s['resume_at']})
    numbers, words, _ = _rows(device_iter(standin, 16))
    assert len(numbers) == s['iter_resume_count']
    assert digest(numbers, words) == s['iter_resume_sha256']
    torch.cuda.synchronize()


def test_device_iter_reprepares_an_evicted_shard(tmp_path):
    import shutil
    d = tmp_path / 'a'
    shutil.copytree(gu.GOLDEN + '/config_a', d)
    ds = LocalDataset(str(d), decoded_cache_bytes=1 << 20)
    ids = worker_sample_ids(fixture_ids()['noshuffle_w1.start'], 0, 0, 0)
    backup = tmp_path / 'shard0'
    shutil.copy(ds.shards[0]._filename(), backup)

    class Restoring(StandInDataset):
        def prepare_shard(self, shard_id, blocking=True):  # the reference downloads it again
            super().prepare_shard(shard_id, blocking)
            if shard_id == 0 and blocking:
                shutil.copy(backup, ds.shards[0]._filename())

    standin = Restoring(ds.shards, lambda e, s: ids)
    ds.shards[0].evict()  # gone before the first batch needs it
    numbers, _, _ = _rows(device_iter(standin, 16))
    assert len(numbers) == 10_000 and 0 in standin.prepared


def _loader_cases():
    from tests.test_plugin_iter import CASES
    return CASES


@pytest.mark.parametrize('name,rank', _loader_cases())
def test_device_iter_multi_worker_loader(name, rank):
    """device_iter(num_workers=W): the W worker partitions gathered on the GPU and interleaved as
    torch's DataLoader returns them give, on each rank, the samples and batch sizes the REAL
    reference's StreamingDataLoader(num_workers=W) yielded (tests/golden/order/loader.json), and
    DeviceBatches checkpoints (this rank's count times the ranks, // replication) and resumes as
    it does -- on one stream and on two streams drawn by proportion under every batching method
    (random, stratified, per_stream, device_per_stream), and with replication=2."""
    from tests.test_plugin_iter import _standin, loader_settings, stream_dirs
    st = loader_settings()[name]
    pr = st['per_rank'][rank]
    bs, W = st['kwargs']['batch_size'], st['workers']
    shards = []
    for d in stream_dirs(st):  # the dataset's shards: stream by stream, as StreamingDataset's
        shards += LocalDataset(gu.GOLDEN + '/' + d, decoded_cache_bytes=1 << 20).shards

    class _DS:
        pass

    ds = _DS()
    ds.shards = shards
    standin = _standin(name, rank, ds.shards)
    numbers, words, sizes = _rows(device_iter(standin, bs, num_workers=W))
    assert sizes == pr['start_batch_sizes']
    assert digest(numbers, words) == pr['iter_start_sha256']
    standin = _standin(name, rank, ds.shards)
    loader = DeviceBatches(standin, bs, num_workers=W)
    it = iter(loader)
    for _ in range(st['resume_batches']):
        next(it)
    state = loader.state_dict()
    assert state['sample_in_epoch'] == st['state_dict']['sample_in_epoch']
    standin._iterator.exit()
    standin = _standin(name, rank, ds.shards)
    standin.load_state_dict(state)
    numbers, words, sizes = _rows(device_iter(standin, bs, num_workers=W))
    assert sizes == pr['resume_batch_sizes']
    assert digest(numbers, words) == pr['iter_resume_sha256']
    torch.cuda.synchronize()
