"""GPU parity of the device shard encoder (``mdsx_encode_*``, ``streaming_amd.encoder``,
``MDSWriter.write_columns``) -- SURVEY.md §8f-3.

Bar: byte-identical shard files. Checked against (1) the reference writer's own shards (every
golden set decoded on the device and re-encoded must reproduce its files and shard split),
(2) the oracle restatement of ``encode_sample`` / ``encode_joint_shard`` / ``Writer.write`` on
seeded random schemas, (3) the host MDSWriter (``write`` per sample) for whole directories, and
(4) full-size config B / C batches (the encoded shards equal the synthetic writer's).
"""

import json
import os

import numpy as np
import pytest
import torch

from oracle import mds_oracle
from streaming_amd import MDSWriter
from streaming_amd.decoder import Plan, RaggedColumn, decode_batch, stage_shards
from streaming_amd.encoder import encode_batch, slice_columns
from streaming_amd.encodings import mds_encode
from streaming_amd.synth import fixed_b_batch_on_device, var_c_shards
from streaming_amd.writer import shard_config_bytes
from tests import golden_util as gu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')


def _config(info):
    return shard_config_bytes(info['column_names'], info['column_encodings'],
                              info['column_sizes'], info.get('compression'),
                              info.get('hashes', []), info.get('size_limit'))


@pytest.mark.parametrize('name', gu.ALL_SETS)
def test_golden_reencode_reproduces_reference_shards(name):
    idx = gu.index(name)
    info0 = idx['shards'][0]
    plan = Plan(info0['column_names'], info0['column_encodings'], info0['column_sizes'])
    data = [gu.shard_bytes(name, s) for s in idx['shards']]
    decoded = decode_batch(plan, stage_shards(data, [s['samples'] for s in idx['shards']], plan))
    enc, consumed = encode_batch(plan, decoded.columns, _config(info0), info0['size_limit'])
    assert consumed == decoded.rows
    assert [e - b for b, e in enc.bounds] == [s['samples'] for s in idx['shards']]
    for s, want in enumerate(data):
        assert enc.shard_bytes(s) == want, f'{name}: shard {s} differs'


_ENCS = ['bytes', 'str', 'int', 'float64', 'uint8', 'int16', 'ndarray:float32:3', 'ndarray:uint8:37',
         'ndarray', 'ndarray:int32', 'json']


def _random_samples(rng, n, encs):
    out = []
    for i in range(n):
        s = {}
        for k, enc in enumerate(encs):
            name = f'c{k:02}'
            if enc == 'bytes':
                s[name] = rng.bytes(int(rng.integers(0, 300)) if i % 11 else 0)
            elif enc == 'str':
                s[name] = ''.join(chr(int(c)) for c in rng.integers(0x20, 0x2FF,
                                                                    int(rng.integers(0, 40))))
            elif enc == 'int':
                s[name] = int(rng.integers(-2**62, 2**62))
            elif enc in ('float64', 'uint8', 'int16'):
                s[name] = np.frombuffer(rng.bytes(np.dtype(enc).itemsize), enc)[0]
            elif enc.startswith('ndarray:') and enc.count(':') == 2:
                _, dt, shape = enc.split(':')
                shp = tuple(int(x) for x in shape.split(','))
                s[name] = np.frombuffer(rng.bytes(int(np.prod(shp)) * np.dtype(dt).itemsize),
                                        dt).reshape(shp)
            elif enc == 'ndarray':
                s[name] = rng.integers(0, 100, tuple(int(x) for x in rng.integers(1, 4, 2)))
            elif enc == 'ndarray:int32':
                s[name] = rng.integers(-5, 5, int(rng.integers(1, 9))).astype(np.int32)
            elif enc == 'json':
                s[name] = {'i': i, 'v': [float(rng.standard_normal())]}
        out.append(s)
    return out


def _device_columns(plan, samples, dev='cuda'):
    """Device columns of the samples' encoded bytes (what write_columns takes)."""
    cols = {}
    for c in plan.columns:
        enc = [mds_encode(c.encoding, s[c.name]) for s in samples]
        if c.is_fixed:
            dtype, shape = c.tensor_view()
            raw = np.frombuffer(b''.join(enc), np.uint8).reshape(len(samples), c.row_bytes)
            cols[c.name] = torch.from_numpy(raw.copy()).to(dev).view(dtype).reshape(
                (len(samples), ) + shape)
        else:
            offs = np.zeros(len(samples) + 1, np.int64)
            offs[1:] = np.cumsum([len(e) for e in enc])
            vals = np.frombuffer(b''.join(enc), np.uint8) if offs[-1] else np.zeros(0, np.uint8)
            cols[c.name] = RaggedColumn(torch.from_numpy(vals.copy()).to(dev),
                                        torch.from_numpy(offs).to(dev))
    return cols


@pytest.mark.parametrize('seed', range(8))
def test_random_schema_vs_oracle(seed):
    rng = np.random.default_rng(100 + seed)
    k = int(rng.integers(1, len(_ENCS) + 1))
    encs = list(rng.choice(_ENCS, k, replace=False))
    names = [f'c{i:02}' for i in range(k)]
    sizes = [{'int': 8, 'float64': 8, 'uint8': 1, 'int16': 2, 'ndarray:float32:3': 12,
              'ndarray:uint8:37': 37}.get(e) for e in encs]
    plan = Plan(names, encs, sizes)
    samples = _random_samples(rng, int(rng.integers(1, 4000)), encs)
    if seed % 3 == 0:
        samples = samples[:1] * 1 + samples  # duplicates are fine
    limit = [1 << 12, 1 << 14, 1 << 16, None][seed % 4]
    cfg = shard_config_bytes(names, encs, sizes, None, [], limit)
    cols = _device_columns(plan, samples)
    enc, consumed = encode_batch(plan, cols, cfg, limit)
    assert consumed == len(samples)
    # oracle: encode_sample per row, Writer.write split, encode_joint_shard per shard
    host_cols = []
    for c in plan.columns:
        v = cols[c.name]
        if c.is_fixed:
            host_cols.append(('fixed', v.reshape(len(samples), -1).contiguous().view(
                torch.uint8).cpu().numpy()))
        else:
            host_cols.append(('var', v.values.cpu().numpy(), v.offsets.cpu().numpy()))
    rows = [mds_oracle.encode_sample_from_columns(host_cols, i) for i in range(len(samples))]
    counts = mds_oracle.writer_split([len(r) for r in rows], limit, 8 + len(cfg))
    assert [e - b for b, e in enc.bounds] == counts
    row = 0
    for s, n in enumerate(counts):
        assert enc.shard_bytes(s) == mds_oracle.encode_joint_shard(cfg, rows[row:row + n]), s
        row += n


def test_write_columns_matches_host_writer(tmp_path):
    rng = np.random.default_rng(7)
    columns = {'a': 'bytes', 'b': 'int', 'c': 'str', 'd': 'ndarray:float32:4', 'e': 'ndarray'}
    samples = []
    for s in _random_samples(rng, 3000, ['bytes', 'int', 'str', 'ndarray:float32:4', 'ndarray']):
        samples.append({'a': s['c00'], 'b': s['c01'], 'c': s['c02'], 'd': s['c03'],
                        'e': s['c04']})
    samples[0]['a'] = rng.bytes(20_000)  # oversized first sample: an empty shard first
    samples[1500]['a'] = rng.bytes(30_000)
    kw = dict(columns=columns, size_limit=1 << 14, hashes=['sha1', 'xxh64'], compression='zstd')
    host_dir, dev_dir = str(tmp_path / 'host'), str(tmp_path / 'dev')
    with MDSWriter(out=host_dir, **kw) as w:
        for s in samples:
            w.write(s)
    with MDSWriter(out=dev_dir, **kw) as w:
        plan = Plan(w.column_names, w.column_encodings, w.column_sizes)
        cols = _device_columns(plan, samples)
        lo = 0
        for hi in (1, 700, 701, 2999, 3000):  # batches of 1, 699, 1, 2298, 1 rows
            w.write_columns(slice_columns(cols, lo, hi))
            lo = hi
    with open(os.path.join(host_dir, 'index.json')) as f:
        host_index = json.load(f)
    with open(os.path.join(dev_dir, 'index.json')) as f:
        dev_index = json.load(f)
    assert dev_index == host_index
    assert host_index['shards'][0]['samples'] == 0
    assert sorted(os.listdir(host_dir)) == sorted(os.listdir(dev_dir))
    for name in os.listdir(host_dir):
        with open(os.path.join(host_dir, name), 'rb') as f1, \
                open(os.path.join(dev_dir, name), 'rb') as f2:
            assert f1.read() == f2.read(), name


def test_alignment_sweep():
    """Ragged rows of every length 0..300 from values at every 16-byte phase, next to a
    37-byte fixed column: every source/destination alignment of the realigning copy."""
    plan = Plan(['a', 'b'], ['bytes', 'ndarray:uint8:37'], [None, 37])
    rng = np.random.default_rng(3)
    lens = np.tile(np.arange(301), 2)
    rng.shuffle(lens)
    rows = len(lens)
    for phase in (0, 1, 7, 15):
        pool = torch.from_numpy(np.frombuffer(rng.bytes(int(lens.sum()) + phase),
                                              np.uint8).copy()).cuda()
        offs = np.zeros(rows + 1, np.int64)
        offs[1:] = np.cumsum(lens)
        offs += phase
        a = RaggedColumn(pool, torch.from_numpy(offs).cuda())
        b = torch.from_numpy(np.frombuffer(rng.bytes(rows * 37), np.uint8).reshape(rows, 37).copy()
                             ).cuda()
        cfg = shard_config_bytes(['a', 'b'], ['bytes', 'ndarray:uint8:37'], [None, 37], None, [],
                                 1 << 14)
        enc, _ = encode_batch(plan, {'a': a, 'b': b}, cfg, 1 << 14)
        host = [('var', pool.cpu().numpy(), offs), ('fixed', b.cpu().numpy())]
        samples = [mds_oracle.encode_sample_from_columns(host, i) for i in range(rows)]
        counts = mds_oracle.writer_split([len(s) for s in samples], 1 << 14, 8 + len(cfg))
        row = 0
        for s, n in enumerate(counts):
            assert enc.shard_bytes(s) == mds_oracle.encode_joint_shard(cfg, samples[row:row + n])
            row += n


def test_bad_columns_raise():
    plan = Plan(['a', 'b'], ['bytes', 'int'], [None, 8])
    vals = torch.zeros(100, dtype=torch.uint8, device='cuda')
    ints = torch.zeros(3, dtype=torch.int64, device='cuda')
    cfg = b'{}'
    for offs in ([0, 10, 5, 20], [0, 10, 20, 101], [-1, 0, 0, 0]):
        col = RaggedColumn(vals, torch.tensor(offs, dtype=torch.int64, device='cuda'))
        with pytest.raises(ValueError):
            encode_batch(plan, {'a': col, 'b': ints}, cfg, 1 << 20)
    col = RaggedColumn(vals, torch.tensor([0, 1, 2, 3], dtype=torch.int64, device='cuda'))
    with pytest.raises(ValueError):
        encode_batch(plan, {'a': col, 'b': ints[:2]}, cfg, 1 << 20)
    with pytest.raises(TypeError):
        encode_batch(plan, {'a': vals[:3], 'b': ints}, cfg, 1 << 20)


def test_config_b_full_reencode():
    synth = fixed_b_batch_on_device(1_000_000, seed=5)
    cfg = shard_config_bytes(synth.plan.names, ['int32', 'ndarray:float32:1024'], [4, 4096], None,
                             [], 1 << 26)
    enc, consumed = encode_batch(synth.plan, {'id': synth.sources['id'], 'x': synth.sources['x']},
                                 cfg, 1 << 26)
    assert consumed == 1_000_000
    assert [e - b for b, e in enc.bounds] == synth.samples_per_shard
    for s in range(len(enc)):
        o = synth.batch.offsets[s]
        assert torch.equal(enc.shard(s), synth.batch.buffer[o:o + synth.batch.sizes[s]]), s


def test_config_c_reencode():
    shards, counts, _ = var_c_shards(100_000, seed=9)
    plan = Plan(['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None])
    decoded = decode_batch(plan, stage_shards(shards, counts, plan))
    cfg = shard_config_bytes(['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None], None, [],
                             1 << 26)
    enc, _ = encode_batch(plan, decoded.columns, cfg, 1 << 26)
    assert [e - b for b, e in enc.bounds] == counts
    for s, want in enumerate(shards):
        got = enc.shard(s)
        assert got.numel() == len(want)
        assert torch.equal(got, torch.from_numpy(np.frombuffer(want, np.uint8).copy()).cuda()), s
