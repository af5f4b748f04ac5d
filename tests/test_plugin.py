"""The Stream plugin swaps reference MDS readers for device readers with identical fields
(a stub Stream base stands in for the reference's; no GPU calls)."""

import os

import pytest
from types import SimpleNamespace

from streaming_amd.plugin import make_device_stream, to_device_reader
from streaming_amd.reader import MDSReader
from tests import golden_util as gu


def _ref_like_reader(info, dirname):
    fi = lambda f: None if f is None else SimpleNamespace(**f)  # noqa: E731
    return SimpleNamespace(dirname=dirname, split='', column_encodings=info['column_encodings'],
                           column_names=info['column_names'], column_sizes=info['column_sizes'],
                           compression=info['compression'], hashes=info['hashes'],
                           raw_data=fi(info['raw_data']), zip_data=fi(info['zip_data']),
                           samples=info['samples'], size_limit=info['size_limit'])


class FakeStream:
    """Stands in for streaming.base.stream.Stream: get_shards returns reference-like readers."""

    def __init__(self, local):
        self.local = local

    def get_shards(self, world, allow_unsafe_types):
        idx = gu.index('zstd')
        return [_ref_like_reader(info, self.local) for info in idx['shards']] + ['json-reader']


def test_device_stream_swaps_mds_readers():
    cls = make_device_stream(FakeStream)
    assert issubclass(cls, FakeStream)
    d = os.path.join(gu.GOLDEN, 'zstd')
    shards = cls(d).get_shards(world=None, allow_unsafe_types=False)
    assert shards[-1] == 'json-reader'  # non-MDS readers unchanged
    idx = gu.index('zstd')
    for r, info in zip(shards[:-1], idx['shards']):
        assert isinstance(r, MDSReader)
        assert r.samples == info['samples'] and len(r) == info['samples']
        assert r.column_names == info['column_names']
        assert r.column_sizes == info['column_sizes']
        assert r.raw_data.basename == info['raw_data']['basename']
        assert r.zip_data.bytes == info['zip_data']['bytes']
        assert r.compression == 'zstd'
        assert r.get_raw_size() == info['raw_data']['bytes']
        assert r.get_persistent_size(keep_zip=True) == \
            info['raw_data']['bytes'] + info['zip_data']['bytes']


def test_to_device_reader_idempotent():
    info = gu.index('kat')['shards'][0]
    r = to_device_reader(_ref_like_reader(info, os.path.join(gu.GOLDEN, 'kat')))
    assert to_device_reader(r) is r


def test_pipeline_validate_hash_algorithm_checks():
    """Unknown / unrecorded validate_hash algorithms raise the reference's ValueErrors before any
    device work (stream.py:401-408, hashing.py:65-66)."""
    from streaming_amd.decoder import Plan
    from streaming_amd.pipeline import ShardPipeline, shard_files_from_index
    d = os.path.join(gu.GOLDEN, 'zstd')
    idx = gu.index('zstd')
    info = idx['shards'][0]
    plan = Plan(info['column_names'], info['column_encodings'], info['column_sizes'])
    files = shard_files_from_index(d, idx)
    with pytest.raises(ValueError, match='not a supported hash algorithm'):
        ShardPipeline(plan, files, validate_hash='fake')
    with pytest.raises(ValueError, match='does not match with those provided'):
        ShardPipeline(plan, files, validate_hash='xxh3_64')
