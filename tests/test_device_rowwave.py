"""GPU parity of the one-row-per-wave decode of all-fixed plans (``rowwave_decode_kernel``,
``MDSX_TUNE rw=1|2|4``, occupancy by ``lpad``): it reads each row from where the writer puts it
(offsets[0] + row x row size, mds/writer.py:133-144) and stores only once the row's offsets pair
confirms that address; any other layout takes its checked path. Against the golden digests, the
oracle, and the register decode (``decode_kernel``) on shards whose layout is not the writer's:
a gap before the first sample, junk after some samples, a short sample, offsets past the file."""

import numpy as np
import pytest
import torch

from oracle import mds_oracle
from streaming_amd.decoder import Plan, decode_batch, stage_shards
from tests import golden_util as gu
from tests.test_device_decode import _device_digests

pytestmark = pytest.mark.gpu

MODES = {
    'rw0': 'rw=0',  # decode_kernel (rows of >= 3 KiB take the row-per-wave kernel by default)
    'rw1': 'rw=1',  # registers bounded for 6 waves per SIMD (the default)
    'rw1_occ0': 'rw=1,rwocc=0',  # ... the compiler's choice (5)
    'rw1_occ8': 'rw=1,rwocc=8',  # ... 8 (spills)
    'rw1_rows2': 'rw=1,rwr=2,rwocc=0',  # two rows per wave
    'rw1_rows4': 'rw=1,rwr=4,rwocc=0',
    'rw1_pad': 'rw=1,rwocc=0,lpad=12',  # 12 waves per CU
    'rw2': 'rw=2,rwocc=0,lpad=24',
    'rw2_rows2': 'rw=2,rwr=2,rwocc=0',
    'rw4': 'rw=4,rwocc=0',
    'rw1_temporal': 'rw=1,rwocc=0,nt=0',
}
FIXED_SETS = [n for n in gu.ALL_SETS
              if all(s is not None for s in gu.index(n)['shards'][0]['column_sizes'])]
# an odd mix: a 4-byte and an 8-byte small column, a 37-byte, a 1000-byte and a 4100-byte row
# (the last beyond one 4 KiB step: copied after the check)
NAMES = ['id', 'odd', 'y', 'mid', 'big']
ENCS = ['int32', 'ndarray:uint8:37', 'float64', 'ndarray:uint8:1000', 'ndarray:uint8:4100']
SIZES = [4, 37, 8, 1000, 4100]


@pytest.fixture(scope='module', autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')


def _decode(monkeypatch, tune, shards, names=NAMES, encs=ENCS, sizes=SIZES):
    monkeypatch.setenv('MDSX_TUNE', tune)
    plan = Plan(names, encs, sizes)
    counts = [int(np.frombuffer(s[:4], np.uint32)[0]) for s in shards]
    return decode_batch(plan, stage_shards(shards, counts, plan))


def _rows(rng, n):
    return [rng.bytes(sum(SIZES)) for _ in range(n)]


def _shard(samples, gap=b'', junk=None):
    """The writer's layout (mds/writer.py:133-144), with `gap` bytes before the first sample and
    junk[i] bytes after sample i."""
    body = [s + (junk[i] if junk else b'') for i, s in enumerate(samples)]
    return mds_oracle.encode_joint_shard(gap, body)


def _want(samples):
    cols, pos = [], 0
    for size in SIZES:
        cols.append(np.stack([np.frombuffer(s[pos:pos + size], np.uint8) for s in samples]))
        pos += size
    return cols


def _check(dec, samples):
    for name, want in zip(NAMES, _want(samples)):
        got = dec[name]
        have = got.reshape(got.shape[0], -1).view(torch.uint8).cpu().numpy()
        assert np.array_equal(have, want), name


@pytest.mark.parametrize('mode', sorted(MODES))
@pytest.mark.parametrize('name', FIXED_SETS)
def test_golden_sets(monkeypatch, mode, name):
    idx = gu.index(name)
    info = idx['shards'][0]
    monkeypatch.setenv('MDSX_TUNE', MODES[mode])
    plan = Plan(info['column_names'], info['column_encodings'], info['column_sizes'])
    data = [gu.shard_bytes(name, s) for s in idx['shards']]
    dec = decode_batch(plan, stage_shards(data, [s['samples'] for s in idx['shards']], plan))
    assert _device_digests(plan, dec) == gu.manifest()[name]['columns']


@pytest.mark.parametrize('mode', sorted(MODES))
def test_layouts(monkeypatch, mode):
    """The writer's layout, with and without config bytes before the first sample (every row on
    the fast path), junk after some samples (the rows behind it checked), in one batch of shards
    of 1..300 rows; the same bytes as the oracle and as the register decode."""
    rng = np.random.default_rng(5)
    sets = [_rows(rng, n) for n in (1, 2, 7, 300, 64)]
    shards = [_shard(sets[0]), _shard(sets[1], gap=b'\x00' * 12), _shard(sets[2]),
              _shard(sets[3], junk=[rng.bytes(int(i % 97 == 5) * 3) for i in range(300)]),
              _shard(sets[4], gap=b'\x01' * 4, junk=[rng.bytes(i % 5) for i in range(64)])]
    dec = _decode(monkeypatch, MODES[mode], shards)
    _check(dec, [s for rows in sets for s in rows])
    for shard, rows in zip(shards, sets):  # each shard alone, against the vectorized oracle
        one = _decode(monkeypatch, MODES[mode], [shard])
        for name, want in zip(NAMES, mds_oracle.decode_fixed_shard_vectorized(shard, SIZES)):
            got = one[name]
            assert np.array_equal(got.reshape(got.shape[0], -1).view(torch.uint8).cpu().numpy(),
                                  want), (mode, name)
    base = _decode(monkeypatch, 'rw=0', shards)
    for name in NAMES:
        assert torch.equal(base[name], dec[name]), name


def _oracle_malformed(shard):
    """The samples the reference reader cannot return whole, by the oracle's restatement of it
    (mds/reader.py:103-149): IndexError where it raises one (an empty read), else the samples
    whose fixed columns it would slice short (decode_sample's data[idx:idx + size]) -- where the
    whole-batch decode raises ValueError instead of returning a truncated row."""
    n = int(np.frombuffer(shard[:4], np.uint32)[0])
    r = mds_oracle.OracleMDSReader(None, None, {'raw_data': {'basename': ''},
                                               'column_names': NAMES, 'column_encodings': ENCS,
                                               'column_sizes': SIZES, 'samples': n}, data=shard)
    bad = {}
    for i in range(n):
        try:
            parts = r.split_sample(r.get_sample_data(i))
        except IndexError:
            bad[i] = IndexError
            continue
        if any(len(p) != size for p, size in zip(parts, SIZES)):
            bad[i] = ValueError
    return bad


def _raises_like(monkeypatch, mode, shards, exact=True):
    with pytest.raises(Exception) as want:
        _decode(monkeypatch, 'rw=0', shards)
    with pytest.raises(type(want.value)) as got:
        _decode(monkeypatch, MODES[mode], shards)
    if exact:  # (one failing row: the same report; several: whichever lands first)
        assert str(got.value) == str(want.value)
    # anchored on the oracle: the failing sample is one the reference cannot return whole, and
    # the exception type is the one the batch path maps its failure to
    if exact:
        bad = _oracle_malformed(shards[0])
        rows = [int(w) for w in str(got.value).replace(',', ' ').replace(')', ' ').split()
                if w.isdigit()]
        assert any(row in bad and isinstance(got.value, bad[row]) for row in rows), \
            (str(got.value), bad)


@pytest.mark.parametrize('mode', sorted(MODES))
def test_malformed_rows_report_like_the_register_decode(monkeypatch, mode):
    rng = np.random.default_rng(8)
    rows = _rows(rng, 40)
    # one sample two bytes short of the row size (mds/reader.py: a column past the sample)
    short = [s if i != 17 else s[:-2] for i, s in enumerate(rows)]
    _raises_like(monkeypatch, mode, [_shard(short)])
    # an empty sample (the reference's IndexError)
    empty = [s if i != 3 else b'' for i, s in enumerate(rows)]
    _raises_like(monkeypatch, mode, [_shard(empty)])
    # the last offset past the file: the header check (and the last row's range); the reference
    # reads every sample whole here (its read stops at the file's end), the batch path refuses
    # the shard (malformed shards)
    bad = bytearray(_shard(rows))
    bad[4 + 4 * 40:4 + 4 * 41] = np.uint32(len(bad) + 100).tobytes()
    assert _oracle_malformed(bytes(bad)) == {}
    _raises_like(monkeypatch, mode, [bytes(bad)], exact=False)
