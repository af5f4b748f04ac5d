"""device_iter / DeviceBatches host logic on CPU (rows read by the oracle in place of the device
gather; the device gather itself is tests/test_device_plugin_iter.py):

* ``loader_batches`` on the ids the real reference's ``generate_work`` recorded reproduces, for
  every rank, what the reference's ``StreamingDataLoader(num_workers=W)`` yielded
  (tests/golden/order/loader.json, recorded by tests/golden/make_loader_fixtures.py);
* ``device_iter(num_workers=W)`` driven over a stand-in of the reference's iteration surface
  gives the same samples, batch sizes and checkpoint (``DeviceBatches.state_dict`` counts this
  rank's samples times the ranks, ``dataloader.py:74-84``), and resumes there;
* a dataset lacking a private piece of the iteration fails at entry with one ``TypeError``;
* each sample's shard access time is stamped before its batch is gathered (``dataset.py:1270``).
"""

import json
import os

import numpy as np
import pytest

from oracle.mds_oracle import OracleMDSReader
from streaming_amd.order import loader_batches
from streaming_amd.plugin import DeviceBatches, device_iter
from tests import golden_util as gu
from tests.standin_dataset import StandInDataset
from tests.test_order import digest, oracle_rows

ORDER = os.path.join(gu.GOLDEN, 'order')


def loader_settings():
    with open(os.path.join(ORDER, 'loader.json')) as f:
        return {s['name']: s for s in json.load(f)['settings']}


def loader_ids():
    return dict(np.load(os.path.join(ORDER, 'loader.npz'), allow_pickle=False))


CASES = [(name, rank) for name, st in loader_settings().items() for rank in range(st['ranks'])]


@pytest.mark.parametrize('name,rank', CASES)
@pytest.mark.parametrize('tag', ['start', 'resume'])
def test_loader_batches_reproduce_the_reference_loader(name, rank, tag):
    st = loader_settings()[name]
    pr = st['per_rank'][rank]
    ids = loader_ids()[f'{name}.r{rank}.{tag}']
    prank = _parallel_rank(st, rank)
    batches = loader_batches(ids, 0, prank, st['workers'], st['kwargs']['batch_size'])
    flat = np.concatenate(batches)
    numbers, words = stream_rows(st)
    assert [len(b) for b in batches] == pr[f'{tag}_batch_sizes']
    assert digest(numbers[flat], [words[i] for i in flat]) == pr[f'iter_{tag}_sha256']


def stream_dirs(st):
    """The golden dirs of a loader setting's streams, in the dataset's shard order."""
    return [s['dir'] for s in st.get('streams', [])] or ['config_a']


def _parallel_rank(st, rank):
    """The rank a replicated rank iterates as (world.py:117-148, one node)."""
    return rank // (st['kwargs'].get('replication') or 1)


_ROWS = {}


def stream_rows(st):
    """(number, words) of every sample of the setting's streams in global id order (oracle)."""
    key = tuple(stream_dirs(st))
    if key not in _ROWS:
        numbers, words = [], []
        for d in key:
            for info in gu.index(d)['shards']:
                r = OracleMDSReader(os.path.join(gu.GOLDEN, d), None, info)
                for i in range(info['samples']):
                    s = r.get_item(i)
                    numbers.append(s['number'])
                    words.append(s['words'])
        _ROWS[key] = (np.array(numbers, np.int64), words)
    return _ROWS[key]


class OracleGather:
    """``DeviceSampleGather``'s interface with the rows read by the CPU oracle."""

    def __init__(self, readers):
        self.shards = readers
        self.starts = np.concatenate([[0], np.cumsum([r.samples for r in readers])])
        self.calls = []

    def locate(self, ids):
        ids = np.asarray(ids, np.int64)
        shard = np.searchsorted(self.starts, ids, side='right') - 1
        return shard, ids - self.starts[shard]

    def gather(self, ids):
        shard, loc = self.locate(ids)
        self.calls.append(shard)
        return [self.shards[int(s)].get_item(int(i)) for s, i in zip(shard, loc)]


def _readers(dirs=('config_a', )):
    return [OracleMDSReader(os.path.join(gu.GOLDEN, d), None, info) for d in dirs
            for info in gu.index(d)['shards']]


def _standin(name, rank, readers):
    """A stand-in whose generate_work returns what the reference's recorded for this setting's
    World (the replicated one under ``replication``)."""
    st = loader_settings()[name]
    ids = loader_ids()
    resume_at = st['state_dict']['sample_in_epoch']
    rep = st['kwargs'].get('replication')

    def epoch_work(world, epoch, sample_in_epoch):
        assert world.workers_per_rank == st['workers']
        assert world.rank == _parallel_rank(st, rank)
        assert world.num_ranks == st['ranks'] // (rep or 1) and epoch == 0
        assert sample_in_epoch in (0, resume_at)
        return ids[f'{name}.r{rank}.{"start" if sample_in_epoch == 0 else "resume"}']

    return StandInDataset(readers, None, epoch_work, world=(1, st['ranks'], rank),
                          batch_size=st['kwargs']['batch_size'], replication=rep,
                          batching_method=st['kwargs'].get('batching_method', 'random'))


def _digest(batches):
    numbers = [r['number'] for b in batches for r in b]
    words = [r['words'] for b in batches for r in b]
    return digest(numbers, words)


@pytest.mark.parametrize('name,rank', CASES)
def test_device_iter_workers_start_checkpoint_resume(name, rank):
    st = loader_settings()[name]
    pr = st['per_rank'][rank]
    bs, W = st['kwargs']['batch_size'], st['workers']
    readers = _readers(stream_dirs(st))
    ds = _standin(name, rank, readers)
    batches = list(device_iter(ds, bs, num_workers=W, gather=OracleGather(readers)))
    assert [len(b) for b in batches] == pr['start_batch_sizes']
    assert _digest(batches) == pr['iter_start_sha256']
    # checkpoint after the fixture's batches, as StreamingDataLoader.state_dict
    ds = _standin(name, rank, readers)
    loader = DeviceBatches(ds, bs, num_workers=W, gather=OracleGather(readers))
    it = iter(loader)
    for _ in range(st['resume_batches']):
        next(it)
    state = loader.state_dict()
    assert state['sample_in_epoch'] == st['state_dict']['sample_in_epoch']
    ds._iterator.exit()
    ds = _standin(name, rank, readers)
    ds.load_state_dict(state)
    resumed = list(device_iter(ds, bs, num_workers=W, gather=OracleGather(readers)))
    assert [len(b) for b in resumed] == pr['resume_batch_sizes']
    assert _digest(resumed) == pr['iter_resume_sha256']


def test_replicated_ranks_see_the_same_samples():
    """replication=2 over two ranks: the reference's loaders yielded the same samples on both
    ranks of a replication group, and so do the recorded partitions device_iter lays out."""
    for name, st in loader_settings().items():
        if not st['kwargs'].get('replication'):
            continue
        a, b = st['per_rank']
        assert a['iter_start_sha256'] == b['iter_start_sha256'], name
        assert a['iter_resume_sha256'] == b['iter_resume_sha256'], name
        ids = loader_ids()
        assert np.array_equal(ids[f'{name}.r0.start'], ids[f'{name}.r1.start']), name


def test_multi_stream_batching_methods_recorded():
    """The loader fixture covers every batching method the reference dispatches
    (batching/__init__.py:21-26) on a two-stream dataset, and replication."""
    sts = loader_settings().values()
    methods = {st['kwargs'].get('batching_method', 'random') for st in sts if st.get('streams')}
    assert methods == {'random', 'stratified', 'per_stream', 'device_per_stream'}
    assert any(st['kwargs'].get('replication') == 2 for st in sts)


def test_state_dict_divides_by_replication():
    readers = _readers()
    ds = _standin('py1s_r2w2', 0, readers)
    ds.replication = 2
    loader = DeviceBatches(ds, 8, num_workers=2, gather=OracleGather(readers))
    it = iter(loader)
    for _ in range(5):
        next(it)
    assert loader.state_dict()['sample_in_epoch'] == 5 * 8 * 2 // 2
    ds._iterator.exit()


@pytest.mark.parametrize('missing', ['_ready_thread', '_resume_incr_epoch', '_get_work'])
def test_missing_iteration_internals_fail_at_entry(missing):
    readers = _readers()

    class Renamed(StandInDataset):
        pass

    setattr(Renamed, missing, None)  # as if the installed reference renamed it
    ds = Renamed(readers, lambda e, s: np.arange(10), world=(1, 1, 0))
    with pytest.raises(TypeError, match=missing) as e:
        next(device_iter(ds, 4, gather=OracleGather(readers)))
    assert '0.14.0.dev0' in str(e.value)
    assert not hasattr(ds, '_iterator')  # nothing started


def test_workers_need_generate_work_and_world(monkeypatch):
    import tests.standin_dataset as standin
    readers = _readers()
    monkeypatch.delattr(standin, 'generate_work')
    ds = _standin('py1e_r1w2', 0, readers)
    with pytest.raises(TypeError, match='generate_work'):
        next(device_iter(ds, 16, num_workers=2, gather=OracleGather(readers)))
    # one worker uses _get_work, not generate_work
    ds = StandInDataset(readers, lambda e, s: np.arange(40), world=(1, 1, 0))
    assert sum(len(b) for b in device_iter(ds, 16, gather=OracleGather(readers))) == 40


def test_access_times_stamped_before_the_gather():
    """The reference stamps each sample's shard as it is read; device_iter stamps each id as it
    joins the pending batch, so a cache_limit eviction in the prepare thread sees the shards of
    the batch being assembled as recently used."""
    readers = _readers()
    ids = np.arange(0, 10_000, 97)  # spans every shard

    class Checking(OracleGather):

        def gather(self, ids_):
            shard, _ = self.locate(ids_)
            assert (ds._shard_access_times[np.unique(shard)] > 0).all()
            return super().gather(ids_)

    ds = StandInDataset(readers, lambda e, s: ids, world=(1, 1, 0))
    n = sum(len(b) for b in device_iter(ds, 32, gather=Checking(readers)))
    assert n == ids.size
