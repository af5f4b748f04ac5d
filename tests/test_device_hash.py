"""GPU parity of shard-file hashing on the device (``mdsx_hash_segments``,
``streaming_amd.hashing``) -- SURVEY.md §8f-4.

Bar: the same hex digests as the reference's ``get_hash`` (``hashing.py:55-68``, i.e.
python-xxhash): every length 0..2100 in one launch (all short paths, block and stripe
boundaries), seeded inputs, the digests the reference writer recorded in the golden
``index.json`` (zip files and their decompressed shards), full-size 64 MiB config-B shards, and
the oracle restatement on the same inputs. Misplaced segments raise instead of faulting.
"""

import json
import os

import numpy as np
import pytest
import torch

from oracle import xxh_oracle as X
from streaming_amd import hashing
from streaming_amd.compression import decompress
from streaming_amd.decoder import Plan, stage_shards
from streaming_amd.synth import fixed_b_batch_on_device
from tests import golden_util as gu

xxhash = pytest.importorskip('xxhash')

pytestmark = pytest.mark.gpu

ALGOS = ('xxh32', 'xxh64', 'xxh3_64', 'xxh3_128', 'xxh128')


@pytest.fixture(scope='module', autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')


def _pack(chunks):
    """Place byte strings at 16-byte aligned offsets of one device buffer."""
    segs, pos = [], 0
    for c in chunks:
        segs.append((pos, len(c)))
        pos = (pos + len(c) + 15) & ~15
    host = np.zeros(pos + 16, np.uint8)
    for (off, n), c in zip(segs, chunks):
        host[off:off + n] = np.frombuffer(c, np.uint8)
    return torch.from_numpy(host).cuda(), segs


def _xx(algo, data, seed=0):
    return getattr(xxhash, algo)(data, seed=seed).hexdigest()


@pytest.mark.parametrize('algo', ALGOS)
@pytest.mark.parametrize('seed', [0, 0x9E3779B97F4A7C15])
def test_every_length_one_launch(algo, seed):
    rng = np.random.default_rng(11)
    chunks = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in range(2101)]
    buf, segs = _pack(chunks)
    s = seed & 0xFFFFFFFF if algo == 'xxh32' else seed
    got = hashing.hash_device(algo, buf, segs, seed=s)
    want = [_xx(algo, c, s) for c in chunks]
    bad = [n for n, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, f'{algo} seed={seed}: lengths {bad[:20]}'


@pytest.mark.parametrize('algo', ALGOS)
def test_block_boundaries_vs_oracle(algo):
    rng = np.random.default_rng(5)
    lens = [241, 1023, 1024, 1025, 1087, 1088, 1089, 2047, 2048, 2049, 131071, 131072, 131073,
            131072 + 1024 + 1, 1 << 20, (1 << 20) + 17]
    chunks = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    buf, segs = _pack(chunks)
    got = hashing.hash_device(algo, buf, segs)
    for n, g, c in zip(lens, got, chunks):
        assert g == _xx(algo, c), n
        if n <= 4096:
            assert g == X.hexdigest(algo, c), n


def test_same_range_many_times_and_reordered():
    rng = np.random.default_rng(2)
    data = rng.integers(0, 256, 300_000, dtype=np.uint8)
    buf = torch.from_numpy(data).cuda()
    segs = [(0, 300_000), (16, 200_000), (0, 300_000), (4096, 0), (299_984, 16), (160, 1025)]
    for algo in ALGOS:
        got = hashing.hash_device(algo, buf, segs)
        want = [_xx(algo, data[o:o + n].tobytes()) for o, n in segs]
        assert got == want, algo


def test_golden_zip_and_raw_digests():
    """The reference writer's own index.json digests (xxh64 of each .zstd file and of the raw
    shard it decompresses to)."""
    d = os.path.join(gu.GOLDEN, 'zstd')
    idx = json.load(open(os.path.join(d, 'index.json')))
    zips, raws, want_zip, want_raw = [], [], [], []
    for shard in idx['shards']:
        z = open(os.path.join(d, shard['zip_data']['basename']), 'rb').read()
        zips.append(z)
        raws.append(decompress('zstd', z))
        want_zip.append(shard['zip_data']['hashes']['xxh64'])
        want_raw.append(shard['raw_data']['hashes']['xxh64'])
    buf, segs = _pack(zips)
    assert hashing.hash_device('xxh64', buf, segs) == want_zip
    info0 = idx['shards'][0]
    plan = Plan(info0['column_names'], info0['column_encodings'], info0['column_sizes'])
    batch = stage_shards(raws, [s['samples'] for s in idx['shards']], plan)
    assert hashing.hash_batch(batch, 'xxh64') == want_raw
    hashing.validate_batch(batch, 'xxh64', [s['raw_data']['hashes'] for s in idx['shards']])
    with pytest.raises(ValueError, match='does not match with those provided'):
        hashing.validate_batch(batch, 'xxh3_64', [s['raw_data']['hashes'] for s in idx['shards']])
    bad = [dict(s['raw_data']['hashes']) for s in idx['shards']]
    bad[1]['xxh64'] = '0' * 16
    with pytest.raises(ValueError, match='Checksum failure: shard 1'):
        hashing.validate_batch(batch, 'xxh64', bad)


@pytest.mark.parametrize('algo', ['xxh3_64', 'xxh128', 'xxh64', 'xxh32'])
def test_full_size_config_b_shards(algo):
    """4 full 64 MiB shards + the partial last one of config B, resident in HBM."""
    syn = fixed_b_batch_on_device(16352 * 4 + 777, seed=3, keep_sources=False)
    b = syn.batch
    got = hashing.hash_batch(b, algo)
    host = b.buffer.cpu().numpy()
    want = [_xx(algo, host[o:o + n].tobytes()) for o, n in zip(b.offsets, b.sizes)]
    assert got == want


def test_bad_segments_raise():
    buf = torch.zeros(4096, dtype=torch.uint8, device='cuda')
    with pytest.raises(ValueError):
        hashing.hash_device('xxh3_64', buf, [(8, 100)])  # not 16-byte aligned
    with pytest.raises(ValueError):
        hashing.hash_device('xxh3_64', buf, [(0, 5000)])  # past the buffer
    with pytest.raises(ValueError):
        hashing.hash_device('sha1', buf, [(0, 10)])  # host-only algorithm
    assert hashing.hash_device('xxh3_64', buf, []) == []
    # the hasher is reusable after an error
    assert hashing.hash_device('xxh3_64', buf, [(0, 4096)]) == [_xx('xxh3_64', bytes(4096))]


@pytest.mark.parametrize('algo', ['xxh3_64', 'xxh128'])
def test_uneven_large_segments_repeated(algo):
    """Segments of very different lengths (uneven chain lengths and chunk counts), hashed
    several times in a row on the same workspace: every call must see only its own block sums."""
    rng = np.random.default_rng(9)
    lens = [int(x) for x in rng.integers(1 << 10, 24 << 20, 24)] + [40 << 20, 300, 5000]
    chunks = [rng.integers(0, 256, n, dtype=np.uint8).tobytes() for n in lens]
    buf, segs = _pack(chunks)
    want = [_xx(algo, c) for c in chunks]
    for rep in range(3):
        order = rng.permutation(len(segs))
        got = hashing.hash_device(algo, buf, [segs[i] for i in order])
        assert got == [want[i] for i in order], rep
