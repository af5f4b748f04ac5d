"""The reference's sample order on config A (tests/golden/order, recorded from the real
reference's generate_work and __iter__ by tests/golden/make_order_fixtures.py), host side:

* the recorded ids, walked per worker with the -1 padding skipped and read through the CPU oracle,
  reproduce the reference's own iteration digests (from the start and resumed from a state_dict);
* every epoch covers each sample once (resumed: the rest of the epoch);
* global id -> (shard, local id) as the reference's Spanner.
The device side (the same ids gathered on the GPU) is tests/test_device_order.py."""

import hashlib
import json
import os

import numpy as np
import pytest

from oracle import mds_oracle
from streaming_amd.order import DeviceSampleGather, worker_sample_ids
from tests import golden_util as gu

ORDER = os.path.join(gu.GOLDEN, 'order')


def settings():
    with open(os.path.join(ORDER, 'config_a.json')) as f:
        return {s['name']: s for s in json.load(f)['settings']}


def fixture_ids():
    return dict(np.load(os.path.join(ORDER, 'config_a.npz'), allow_pickle=False))


def digest(numbers, words) -> str:
    """make_order_fixtures.digest: int64 number + UTF-8 words per sample, in order."""
    h = hashlib.sha256()
    for n, w in zip(numbers, words):
        h.update(np.int64(n).tobytes())
        h.update(w.encode('utf-8') if isinstance(w, str) else bytes(w))
    return h.hexdigest()


_ORACLE = {}


def oracle_rows():
    """(number, words) of every config-A sample in global order, from the CPU oracle."""
    if not _ORACLE:
        d = os.path.join(gu.GOLDEN, 'config_a')
        numbers, words = [], []
        for info in gu.index('config_a')['shards']:
            r = mds_oracle.OracleMDSReader(d, None, info)
            for i in range(info['samples']):
                s = r.get_item(i)
                numbers.append(s['number'])
                words.append(s['words'])
        _ORACLE['rows'] = (np.array(numbers, np.int64), words)
    return _ORACLE['rows']


@pytest.mark.parametrize('name', ['noshuffle_w1', 'py1e_w1'])
@pytest.mark.parametrize('tag', ['start', 'resume'])
def test_recorded_ids_reproduce_reference_iteration(name, tag):
    s = settings()[name]
    ids = worker_sample_ids(fixture_ids()[f'{name}.{tag}'], 0, 0, 0)
    ids = ids[ids != -1]  # _each_sample_id (dataset.py:1463-1466)
    numbers, words = oracle_rows()
    assert len(ids) == s[f'iter_{tag}_count']
    assert digest(numbers[ids], [words[i] for i in ids]) == s[f'iter_{tag}_sha256']


@pytest.mark.parametrize('name', ['noshuffle_w1', 'py1e_w1', 'py1s_n1r2w2', 'py1br_n2r2w1'])
def test_epoch_covers_every_sample_once(name):
    s, z = settings()[name], fixture_ids()
    nodes, rpn, wpr = s['world']
    for tag, expect in (('start', s['epoch_size']), ('resume', s['epoch_size'] - s['resume_at'])):
        ids = np.concatenate([worker_sample_ids(z[f'{name}.{tag}'], n, r, w)
                              for n in range(nodes) for r in range(rpn) for w in range(wpr)])
        ids = ids[ids != -1]
        assert ids.size == expect and np.unique(ids).size == expect
        assert ids.min() >= 0 and ids.max() < s['epoch_size']


class _Shard:
    def __init__(self, samples):
        self.samples = samples


def test_locate_matches_spanner():
    counts = [3, 0, 5, 1, 7]
    g = DeviceSampleGather([_Shard(c) for c in counts])
    ids = np.arange(sum(counts))
    shard, local = g.locate(ids)
    want = [(s, i) for s, c in enumerate(counts) for i in range(c)]
    assert list(zip(shard.tolist(), local.tolist())) == want
    with pytest.raises(IndexError):
        g.locate(np.array([16]))
    with pytest.raises(IndexError):
        g.locate(np.array([-2]))


def test_gather_sources_refuses_host_columns_and_bad_arguments():
    """Argument checks of the multi-source gather, all before any kernel launch (CPU)."""
    import torch
    from streaming_amd.decoder import DecodedBatch, RaggedColumn, gather_sources
    host = DecodedBatch({'x': torch.zeros(4, dtype=torch.int32),
                         's': RaggedColumn(torch.zeros(8, dtype=torch.uint8),
                                           torch.arange(5, dtype=torch.int64) * 2, None)}, 4)
    with pytest.raises(ValueError, match='not on the GPU'):
        gather_sources([host], np.zeros(2, np.int64), np.arange(2))
    with pytest.raises(ValueError, match='not on the GPU'):
        host.gather([0, 1])
    with pytest.raises(ValueError, match='differ in length'):
        gather_sources([host], np.zeros(2, np.int64), np.arange(3))
    with pytest.raises(ValueError, match='no sources'):
        gather_sources([], np.zeros(0, np.int64), np.zeros(0, np.int64))
