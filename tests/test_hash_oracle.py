"""The xxHash oracle (``oracle/xxh_oracle.py``) pinned against the reference's own vectors:
its known answer (``tests/test_hashing.py:34-41``), the digests the reference writer recorded in
the golden ``index.json`` files, and python-xxhash (the reference's dependency,
``hashing.py:9,23-26``) on every length 0..1100 plus block-boundary lengths and seeds. Also the
host mirror of ``streaming/base/hashing.py`` (``streaming_amd.hashing``)."""

import json
import os
import random

import pytest

from oracle import xxh_oracle as X
from streaming_amd import hashing
from tests import golden_util as gu

xxhash = pytest.importorskip('xxhash')

ALGOS = ('xxh32', 'xxh64', 'xxh3_64', 'xxh3_128', 'xxh128')


def test_reference_known_answer():
    # tests/test_hashing.py:34-41 of the reference
    assert X.hexdigest('xxh3_64', b'hello') == '9555e8555c62dcfd'
    assert hashing.get_hash('xxh3_64', b'hello') == '9555e8555c62dcfd'
    assert hashing.get_hash('md5', b'hello') == '5d41402abc4b2a76b9719d911017c592'


def test_golden_index_digests():
    d = os.path.join(gu.GOLDEN, 'zstd')
    idx = json.load(open(os.path.join(d, 'index.json')))
    checked = 0
    for shard in idx['shards']:
        zip_info = shard['zip_data']
        data = open(os.path.join(d, zip_info['basename']), 'rb').read()
        assert X.hexdigest('xxh64', data) == zip_info['hashes']['xxh64']
        checked += 1
    assert checked == len(idx['shards'])


def test_golden_index_xxh3_digests():
    """The xxh3_64 / xxh128 digests the reference writer recorded for the zstd_xxh3 set (zip
    files and, decompressed, raw shards): what the pipeline's device validation compares with."""
    from streaming_amd.compression import decompress
    d = os.path.join(gu.GOLDEN, 'zstd_xxh3')
    idx = json.load(open(os.path.join(d, 'index.json')))
    for shard in idx['shards']:
        zdata = open(os.path.join(d, shard['zip_data']['basename']), 'rb').read()
        raw = decompress(shard['compression'], zdata)
        assert len(raw) == shard['raw_data']['bytes']
        for algo in ('xxh3_64', 'xxh128'):
            assert X.hexdigest(algo, zdata) == shard['zip_data']['hashes'][algo]
            assert X.hexdigest(algo, raw) == shard['raw_data']['hashes'][algo]


@pytest.mark.parametrize('algo', ALGOS)
def test_every_short_length_vs_xxhash(algo):
    rng = random.Random(7)
    fn = getattr(xxhash, algo)
    for n in range(0, 1100):
        data = rng.randbytes(n)
        assert X.hexdigest(algo, data) == fn(data).hexdigest(), n


@pytest.mark.parametrize('algo', ALGOS)
@pytest.mark.parametrize('n', [1023, 1024, 1025, 1087, 1088, 1089, 2047, 2048, 2049, 4096 + 63,
                               16384, 16385, 40000])
def test_block_boundaries_and_seeds(algo, n):
    rng = random.Random(n)
    data = rng.randbytes(n)
    fn = getattr(xxhash, algo)
    for seed in (0, 1, rng.getrandbits(64)):
        s = seed & 0xFFFFFFFF if algo == 'xxh32' else seed
        assert X.hexdigest(algo, data, s) == fn(data, seed=s).hexdigest(), (n, seed)


def test_block_sums_restate_the_long_loop():
    # acc after a block == scramble(acc + block_sums): the split the device kernels rely on
    rng = random.Random(3)
    block = rng.randbytes(1024)
    acc = list(X.INIT_ACC)
    direct = list(acc)
    for j in range(16):
        X._accumulate_stripe(direct, block, 64 * j, X.SECRET, 8 * j)
    X._scramble(direct, X.SECRET)
    sums = X.block_sums(block)
    split = [(a + s) & X.M64 for a, s in zip(acc, sums)]
    X._scramble(split, X.SECRET)
    assert split == direct


def test_host_mirror_interface():
    assert hashing.is_hash('xxh128') and hashing.is_hash('sha384')
    assert not hashing.is_hash('') and not hashing.is_hash('fake')
    for algo in ('', 'sha3'):
        with pytest.raises(ValueError):
            hashing.get_hash(algo, b'hello')
    assert set(hashing.DEVICE_HASHES) <= hashing.get_hashes()
    assert {'xxh32', 'xxh64', 'xxh3_64', 'xxh3_128', 'xxh128', 'sha1', 'md5'} <= hashing.get_hashes()
