"""GPU parity tests: the HIP decoder (through the C ABI) against the reference's golden outputs
and against the oracle (CPU restatement of the reference reader) on seeded inputs.

Bar: bit-exact for every column (floats compared as bit patterns), byte-identical UTF-8 and the
same error behaviour (UnicodeDecodeError on the same rows, IndexError on empty samples).
"""

import hashlib
import json
import os

import numpy as np
import pytest
import torch

from oracle import mds_oracle
from streaming_amd import LocalDataset, MDSReader, MDSWriter
from streaming_amd.decoder import (BatchDecoder, Plan, RaggedColumn, decode_batch, output_bytes,
                                   stage_shards)
from streaming_amd.synth import fixed_b_batch_on_device, var_c_shards
from tests import golden_util as gu

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')


def _device_digests(plan, decoded):
    out = {}
    for col in plan.columns:
        v = decoded.columns[col.name]
        if isinstance(v, RaggedColumn):
            d = {
                'values': hashlib.sha256(v.values.cpu().numpy().tobytes()).hexdigest(),
                'offsets': hashlib.sha256(v.offsets.cpu().numpy().tobytes()).hexdigest(),
            }
            if v.flags is not None:
                d['flags'] = hashlib.sha256(v.flags.cpu().numpy().tobytes()).hexdigest()
            out[col.name] = d
        else:
            raw = v.reshape(v.shape[0], -1).view(torch.uint8).cpu().numpy()
            out[col.name] = {'rows': hashlib.sha256(raw.tobytes()).hexdigest()}
    return out


def _decode_golden(name):
    idx = gu.index(name)
    info0 = idx['shards'][0]
    plan = Plan(info0['column_names'], info0['column_encodings'], info0['column_sizes'])
    data = [gu.shard_bytes(name, s) for s in idx['shards']]
    batch = stage_shards(data, [s['samples'] for s in idx['shards']], plan)
    return plan, decode_batch(plan, batch)


@pytest.mark.parametrize('name', gu.ALL_SETS)
def test_golden_batch_decode_matches_reference(name):
    plan, decoded = _decode_golden(name)
    assert _device_digests(plan, decoded) == gu.manifest()[name]['columns']


@pytest.mark.parametrize('name', gu.ALL_SETS)
def test_golden_per_shard_decode_matches_reference(name):
    idx = gu.index(name)
    m = gu.manifest()[name]['columns']
    parts = {}
    for info in idx['shards']:
        plan = Plan(info['column_names'], info['column_encodings'], info['column_sizes'])
        batch = stage_shards([gu.shard_bytes(name, info)], [info['samples']], plan)
        dec = decode_batch(plan, batch)
        for col in plan.columns:
            parts.setdefault(col.name, []).append(dec.columns[col.name])
    for cname, vals in parts.items():
        if isinstance(vals[0], RaggedColumn):
            values = np.concatenate([v.values.cpu().numpy() for v in vals])
            offs, base = [np.zeros(1, np.int64)], 0
            for v in vals:
                o = v.offsets.cpu().numpy()
                offs.append(o[1:] + base)
                base += int(o[-1])
            assert hashlib.sha256(values.tobytes()).hexdigest() == m[cname]['values']
            assert hashlib.sha256(np.concatenate(offs).tobytes()).hexdigest() == \
                m[cname]['offsets']
        else:
            rows = np.concatenate(
                [v.reshape(v.shape[0], -1).view(torch.uint8).cpu().numpy() for v in vals])
            assert hashlib.sha256(rows.tobytes()).hexdigest() == m[cname]['rows']


@pytest.mark.parametrize('name', gu.ITEM_SETS)
def test_golden_get_item_matches_reference(name):
    ds = LocalDataset(os.path.join(gu.GOLDEN, name))
    expected = gu.items(name)
    assert len(ds) == len(expected)
    for i, rec in enumerate(expected):
        shard_id, k = ds.spanner[i]
        reader = ds.shards[shard_id]
        if any(want['t'] == 'error' for want in rec.values()):
            with pytest.raises(UnicodeDecodeError):  # the reference raises for the whole sample
                reader[k]
            continue
        sample = reader[k]
        assert list(sample) == list(rec)
        for c, want in rec.items():
            assert gu.value_record(sample[c]) == want, (name, i, c)


def test_kat_values():
    ds = LocalDataset(os.path.join(gu.GOLDEN, 'kat'))
    assert ds[0] == {'s': 'hé', 'a': -2, 'b': b'\x00\x01\x02'}
    assert ds[1] == {'s': '', 'a': 7, 'b': b''}
    assert type(ds[0]['a']) is int
    dec = ds.decode_all()
    assert dec['a'].cpu().tolist() == [-2, 7]
    assert dec['s'].offsets.cpu().tolist() == [0, 3, 3]
    assert bytes(dec['s'].values.cpu().numpy()) == 'hé'.encode()
    assert dec['s'].flags.cpu().tolist() == [0, 0]
    assert dec['b'].offsets.cpu().tolist() == [0, 3, 3]


def test_bad_utf8_flags_match_python_decoder():
    plan, dec = _decode_golden('bad_utf8')
    flags = dec['s'].flags.cpu().tolist()
    want = [0 if mds_oracle.utf8_is_valid(b) else 1 for b in __import__(
        'tests.golden.make_golden', fromlist=['BAD_UTF8']).BAD_UTF8]
    assert flags == want


def test_decode_sample_on_device():
    d = os.path.join(gu.GOLDEN, 'scalars')
    info = gu.index('scalars')['shards'][0]
    reader = MDSReader.from_json(d, None, info)
    oracle = mds_oracle.OracleMDSReader(d, None, info)
    for i in range(info['samples']):
        data = reader.get_sample_data(i)
        assert data == oracle.get_sample_data(i)
        got = reader.decode_sample(data)
        want = oracle.decode_sample(data)
        for c in want:
            assert gu.value_record(got[c]) == gu.value_record(want[c])


def test_config_b_full_size_round_trip():
    """BASELINE config B: 1M samples, 62 x 64 MiB shards, decoded in one device batch."""
    synth = fixed_b_batch_on_device(1_000_000, seed=11)
    assert len(synth.samples_per_shard) == 62
    assert synth.samples_per_shard[0] == 16352
    dec = BatchDecoder(synth.plan, synth.batch)
    out = dec.run()
    dec.check()
    assert torch.equal(out['id'], synth.sources['id'])
    assert torch.equal(out['x'].view(torch.int32), synth.sources['x'].view(torch.int32))
    # second run over the same outputs (no stale state)
    out['x'].zero_()
    dec.run()
    dec.check()
    assert torch.equal(out['x'].view(torch.int32), synth.sources['x'].view(torch.int32))
    assert output_bytes(synth.plan, out) == 1_000_000 * 4100


def test_config_c_full_shards_round_trip(tmp_path):
    """BASELINE config C schema at full 64 MiB shard size (3 shards), vs the source columns and vs
    the oracle reading the shard files (every sample)."""
    shards, counts, src = var_c_shards(45_000, seed=5)
    assert len(counts) == 3 and counts[0] > 14_000
    names = ['b', 'n', 's']
    plan = Plan(names, ['bytes', 'int', 'str'], [None, 8, None])
    batch = stage_shards(shards, counts, plan)
    dec = decode_batch(plan, batch)
    assert np.array_equal(dec['n'].cpu().numpy(), src['n'])
    b = dec['b']
    assert np.array_equal(b.offsets.cpu().numpy(), np.concatenate([[0], np.cumsum(src['b_len'])]))
    assert np.array_equal(b.values.cpu().numpy(), src['b_pool'])
    s = dec['s']
    assert np.array_equal(s.offsets.cpu().numpy(), np.concatenate([[0], np.cumsum(src['s_len'])]))
    assert np.array_equal(s.values.cpu().numpy(), src['s_pool'])
    assert int(s.flags.sum()) == 0
    assert dec.rows == 45_000
    # the same decode against the oracle reading the three shard files, every sample
    want = {c: [] for c in names}
    for k, (data, n) in enumerate(zip(shards, counts)):
        (tmp_path / f'shard.{k:05d}.mds').write_bytes(data)
        info = {'column_names': names, 'column_encodings': ['bytes', 'int', 'str'],
                'column_sizes': [None, 8, None], 'samples': n,
                'raw_data': {'basename': f'shard.{k:05d}.mds'}}
        for c, v in mds_oracle.decode_shard_columns(str(tmp_path), None, info).items():
            want[c].append(v)
    assert np.array_equal(dec['n'].cpu().numpy().view(np.uint8).reshape(-1, 8),
                          np.concatenate([v[1] for v in want['n']]))
    for c, col in (('b', b), ('s', s)):
        assert np.array_equal(col.values.cpu().numpy(), np.concatenate([v[1] for v in want[c]]))
        assert np.array_equal(np.diff(col.offsets.cpu().numpy()),
                              np.concatenate([np.diff(v[2]) for v in want[c]]))
    assert np.array_equal(s.flags.cpu().numpy(), np.concatenate([v[3] for v in want['s']]))
    # and the oracle's per-sample reader (reference value types) at both ends of the first shard
    info = {'column_names': names, 'column_encodings': ['bytes', 'int', 'str'],
            'column_sizes': [None, 8, None], 'samples': counts[0],
            'raw_data': {'basename': 'shard.00000.mds'}}
    ref = mds_oracle.OracleMDSReader(str(tmp_path), None, info)
    bo, so = b.offsets.cpu().numpy(), s.offsets.cpu().numpy()
    bv, sv, nv = b.values.cpu().numpy(), s.values.cpu().numpy(), dec['n'].cpu().numpy()
    for i in list(range(50)) + [counts[0] - 1]:
        item = ref.get_item(i)
        assert item['n'] == int(nv[i])
        assert item['b'] == bv[bo[i]:bo[i + 1]].tobytes()
        assert item['s'] == sv[so[i]:so[i + 1]].tobytes().decode('utf-8')


def _random_dataset(tmp_path, seed):
    rng = np.random.default_rng(seed)
    choices = ['bytes', 'str', 'int', 'uint8', 'int16', 'float32', 'float64', 'ndarray:uint8:3',
               'ndarray:float32:5', 'ndarray:int8:33', 'ndarray:uint16:64', 'ndarray',
               'ndarray:int32']
    ncols = int(rng.integers(1, 7))
    name_pad = 'q' * int(rng.integers(0, 16))  # shifts the config length: every alignment
    cols = {f'{name_pad}c{k}': choices[int(rng.integers(0, len(choices)))] for k in range(ncols)}
    samples = []
    for _ in range(int(rng.integers(1, 700))):
        s = {}
        for c, enc in cols.items():
            if enc == 'bytes':
                s[c] = rng.bytes(int(rng.choice([0, 1, 15, 16, 17, int(rng.integers(0, 3000))])))
            elif enc == 'str':
                from tests.golden.make_golden import random_text
                s[c] = random_text(rng, 0, int(rng.choice([3, 40, 500])))
            elif enc == 'int':
                s[c] = int(rng.integers(-2**63, 2**63 - 1))
            elif enc in ('uint8', 'int16', 'float32', 'float64'):
                s[c] = np.frombuffer(rng.bytes(np.dtype(enc).itemsize), enc)[0]
            elif enc.count(':') == 2:
                _, dt, shape = enc.split(':')
                n = int(shape)
                s[c] = np.frombuffer(rng.bytes(n * np.dtype(dt).itemsize), dt)
            else:
                dt = enc.split(':')[1] if ':' in enc else 'float16'
                shape = tuple(int(rng.integers(1, 9)) for _ in range(int(rng.integers(1, 4))))
                s[c] = np.frombuffer(rng.bytes(int(np.prod(shape)) * np.dtype(dt).itemsize),
                                     dt).reshape(shape)
        samples.append(s)
    out = tmp_path / f'r{seed}'
    with MDSWriter(columns=cols, out=str(out), size_limit=int(rng.choice([1 << 12, 1 << 16,
                                                                          1 << 20]))) as w:
        for s in samples:
            w.write(s)
    return str(out)


@pytest.mark.parametrize('seed', range(12))
def test_random_schemas_match_oracle(tmp_path, seed):
    d = _random_dataset(tmp_path, seed)
    idx = json.load(open(os.path.join(d, 'index.json')))
    ds = LocalDataset(d)
    dec = ds.decode_all()
    rows = 0
    oracle_cols = {}
    for info in idx['shards']:
        for c, v in mds_oracle.decode_shard_columns(d, None, info).items():
            oracle_cols.setdefault(c, []).append(v)
        rows += info['samples']
    assert dec.rows == rows
    for c, parts in oracle_cols.items():
        got = dec[c]
        if parts[0][0] == 'fixed':
            want = np.concatenate([p[1] for p in parts])
            have = got.reshape(got.shape[0], -1).view(torch.uint8).cpu().numpy()
            assert np.array_equal(have, want), c
        else:
            want_v = np.concatenate([p[1] for p in parts])
            lens = np.concatenate([np.diff(p[2]) for p in parts])
            assert np.array_equal(got.values.cpu().numpy(), want_v), c
            assert np.array_equal(np.diff(got.offsets.cpu().numpy()), lens), c
            if parts[0][3] is not None:
                assert np.array_equal(got.flags.cpu().numpy(),
                                      np.concatenate([p[3] for p in parts])), c
    # per-sample host objects equal the oracle's per-sample decode
    for i in range(0, len(ds), max(1, len(ds) // 25)):
        shard_id, k = ds.spanner[i]
        want = mds_oracle.OracleMDSReader(d, None, idx['shards'][shard_id]).get_item(k)
        got = ds[i]
        for c in want:
            assert gu.value_record(got[c]) == gu.value_record(want[c])


def test_alignment_sweep():
    """Every source/destination byte alignment of the realigning copy, lengths 0..300."""
    rng = np.random.default_rng(7)
    shards, counts = [], []
    plan = None
    for pad in range(16):
        name = 'a' * (pad + 1)
        cols = {name: 'bytes', 'z' + name: 'str'}
        lens = list(range(0, 301)) + [int(x) for x in rng.integers(0, 5000, 50)]
        rows = [{name: rng.bytes(n), 'z' + name: 'é' * (n % 97) + 'x' * (n % 3)} for n in lens]
        import tempfile
        with tempfile.TemporaryDirectory() as t:
            with MDSWriter(columns=cols, out=t, size_limit=None) as w:
                for r in rows:
                    w.write(r)
            idx = json.load(open(os.path.join(t, 'index.json')))
            info = idx['shards'][0]
            raw = open(os.path.join(t, info['raw_data']['basename']), 'rb').read()
            p = Plan(info['column_names'], info['column_encodings'], info['column_sizes'])
            dec = decode_batch(p, stage_shards([raw], [info['samples']], p))
            b = dec[name]
            vals = b.values.cpu().numpy()
            offs = b.offsets.cpu().numpy()
            for k, r in enumerate(rows):
                assert vals[offs[k]:offs[k + 1]].tobytes() == r[name]
            s = dec['z' + name]
            vals = s.values.cpu().numpy()
            offs = s.offsets.cpu().numpy()
            for k, r in enumerate(rows):
                assert vals[offs[k]:offs[k + 1]].tobytes().decode() == r['z' + name]
            assert int(s.flags.sum()) == 0


# ---- error behaviour on malformed shards (must raise, never fault) -------------------------


def _kat_shard():
    info = gu.index('kat')['shards'][0]
    return bytearray(gu.shard_bytes('kat', info)), info


def _decode_raw(raw, info, samples=None):
    plan = Plan(info['column_names'], info['column_encodings'], info['column_sizes'])
    batch = stage_shards([bytes(raw)], [samples if samples is not None else info['samples']], plan)
    return decode_batch(plan, batch)


def test_error_offsets_past_file():
    raw, info = _kat_shard()
    raw[8:12] = np.uint32(10_000_000).tobytes()  # offsets[1] far past the file
    with pytest.raises(ValueError):
        _decode_raw(raw, info)


def test_error_head_larger_than_sample():
    raw, info = _kat_shard()
    start = int(np.frombuffer(bytes(raw[4:8]), np.uint32)[0])
    raw[start:start + 4] = np.uint32(0x7fffffff).tobytes()  # bytes column claims 2 GiB
    with pytest.raises(ValueError):
        _decode_raw(raw, info)


def test_error_sample_count_mismatch():
    raw, info = _kat_shard()
    with pytest.raises(ValueError):
        _decode_raw(raw, info, samples=1)


def test_error_empty_sample_is_index_error():
    raw = np.uint32(1).tobytes() + np.array([12, 12], np.uint32).tobytes()
    info = {'column_names': ['a'], 'column_encodings': ['bytes'], 'column_sizes': [None],
            'samples': 1}
    with pytest.raises(IndexError):
        _decode_raw(raw, info)


def test_error_table_past_file():
    raw = np.uint32(5).tobytes() + np.array([12, 12], np.uint32).tobytes()
    info = {'column_names': ['a'], 'column_encodings': ['bytes'], 'column_sizes': [None],
            'samples': 5}
    with pytest.raises(ValueError):
        _decode_raw(raw, info)


def test_missing_shard_file_raises_file_not_found(tmp_path):
    d = tmp_path / 'kat'
    import shutil
    shutil.copytree(os.path.join(gu.GOLDEN, 'kat'), d)
    ds = LocalDataset(str(d))
    os.remove(d / 'shard.00000.mds')
    with pytest.raises(FileNotFoundError):
        ds[0]


def _decode_rows(tmp_path, cols, rows, **kw):
    with MDSWriter(columns=cols, out=str(tmp_path / 'ds'), **kw) as w:
        for r in rows:
            w.write(r)
    ds = LocalDataset(str(tmp_path / 'ds'))
    return ds, ds.decode_all()


def test_ragged_many_tiny_rows(tmp_path):
    """Gather tiles holding thousands of empty / 1-byte rows (rows read from global memory)."""
    rng = np.random.default_rng(9)
    pieces = [b'', b'a', 'é'.encode(), b'\xc3', b'\x80', '€'.encode()]
    rows = []
    for i in range(6000):
        k = int(rng.integers(0, len(pieces))) if i % 7 == 0 else 0
        rows.append({'s': pieces[k], 'b': pieces[(k + 1) % len(pieces)] * (i % 3)})
    ds, dec = _decode_rows(tmp_path, {'s': 'str', 'b': 'bytes'}, rows, size_limit=None)
    s, b = dec['s'], dec['b']
    sv, so = s.values.cpu().numpy(), s.offsets.cpu().numpy()
    bv, bo = b.values.cpu().numpy(), b.offsets.cpu().numpy()
    flags = s.flags.cpu().numpy()
    for i, r in enumerate(rows):
        assert sv[so[i]:so[i + 1]].tobytes() == r['s']
        assert bv[bo[i]:bo[i + 1]].tobytes() == r['b']
        assert flags[i] == (0 if mds_oracle.utf8_is_valid(r['s']) else 1), i


def test_ragged_row_spanning_many_tiles(tmp_path):
    """One 150 KB str row (19 gather tiles) with an error deep inside, between valid rows."""
    big = ('ab€' * 30000).encode()
    bad = bytearray(big)
    bad[100001] = 0xFF
    rows = [{'s': 'x' * 5}, {'s': big}, {'s': bytes(bad)}, {'s': big[:-1]}, {'s': 'ok'}]
    ds, dec = _decode_rows(tmp_path, {'s': 'str'}, rows, size_limit=None)
    s = dec['s']
    sv, so = s.values.cpu().numpy(), s.offsets.cpu().numpy()
    for i, r in enumerate(rows):
        want = r['s'] if isinstance(r['s'], bytes) else r['s'].encode()
        assert sv[so[i]:so[i + 1]].tobytes() == want
    # big[:-1] cuts a 3-byte euro sign: truncated sequence at the row end
    assert s.flags.cpu().tolist() == [0, 0, 1, 1, 0]
