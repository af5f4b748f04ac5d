"""The oracle (CPU restatement of the reference reader) against the reference's golden outputs.

Pins oracle/mds_oracle.py: every golden set was decoded by the REAL reference when it was
generated (tests/golden/make_golden.py); the oracle must reproduce those outputs exactly.
"""

import hashlib
import os
import shutil

import numpy as np
import pytest

from oracle import mds_oracle
from tests import golden_util as gu

DEVICE_ENCODINGS = ('bytes', 'str', 'int', 'ndarray', 'uint8', 'uint16', 'uint32', 'uint64',
                    'int8', 'int16', 'int32', 'int64', 'float16', 'float32', 'float64')


def _local_copy(name, tmp_path):
    """Directory with raw shard files (decompressing compressed-only sets)."""
    idx = gu.index(name)
    if all(os.path.exists(os.path.join(gu.GOLDEN, name, s['raw_data']['basename']))
           for s in idx['shards']):
        return os.path.join(gu.GOLDEN, name), idx
    out = tmp_path / name
    out.mkdir()
    for info in idx['shards']:
        (out / info['raw_data']['basename']).write_bytes(gu.shard_bytes(name, info))
    shutil.copy(os.path.join(gu.GOLDEN, name, 'index.json'), out / 'index.json')
    return str(out), idx


def test_kat_shard_sha256():
    m = gu.manifest()
    assert m['kat']['shards'][0]['sha256'] == \
        '17b064fd07ffeb2e18af6169edc30aaa41a2e79f528161bd19dfb18fc8a4ccd0'
    raw = gu.shard_bytes('kat', gu.index('kat')['shards'][0])
    assert hashlib.sha256(raw).hexdigest() == m['kat']['shards'][0]['sha256']
    assert len(raw) == 255
    assert np.frombuffer(raw[:16], np.uint32).tolist() == [2, 217, 239, 255]


def test_config_a_content_digest():
    # ordered content sha256 over (int64 number, utf8 words) of config A.
    m = gu.manifest()
    assert m['config_a']['content_sha256'] == \
        'd82947a049275803b171bc1e385e105354b2137e0e2268c64a620bbba39e60c2'
    h = hashlib.sha256()
    d = os.path.join(gu.GOLDEN, 'config_a')
    for info in gu.index('config_a')['shards']:
        r = mds_oracle.OracleMDSReader(d, None, info)
        for i in range(len(r)):
            s = r.get_item(i)
            h.update(np.int64(s['number']).tobytes())
            h.update(s['words'].encode('utf-8'))
    assert h.hexdigest() == m['config_a']['content_sha256']


@pytest.mark.parametrize('name', gu.ALL_SETS)
def test_oracle_columns_match_reference_digests(name, tmp_path):
    d, idx = _local_copy(name, tmp_path)
    m = gu.manifest()[name]
    per_col = {}
    for info in idx['shards']:
        assert hashlib.sha256(open(os.path.join(d, info['raw_data']['basename']),
                                   'rb').read()).hexdigest() == \
            next(s['sha256'] for s in m['shards'] if s['basename'] == info['raw_data']['basename'])
        cols = mds_oracle.decode_shard_columns(d, None, info)
        for c, v in cols.items():
            per_col.setdefault(c, []).append(v)
    merged = {}
    for c, parts in per_col.items():
        if parts[0][0] == 'fixed':
            merged[c] = ('fixed', np.concatenate([p[1] for p in parts]))
        else:
            values = np.concatenate([p[1] for p in parts])
            offs, base = [np.zeros(1, np.int64)], 0
            for p in parts:
                offs.append(p[2][1:] + base)
                base += int(p[2][-1])
            flags = None if parts[0][3] is None else np.concatenate([p[3] for p in parts])
            merged[c] = ('ragged', values, np.concatenate(offs), flags)
    assert mds_oracle.column_digests(merged) == m['columns']


@pytest.mark.parametrize('name', gu.ITEM_SETS)
def test_oracle_items_match_reference(name):
    idx = gu.index(name)
    expected = gu.items(name)
    d = os.path.join(gu.GOLDEN, name)
    k = 0
    for info in idx['shards']:
        r = mds_oracle.OracleMDSReader(d, None, info)
        for i in range(len(r)):
            parts = r.split_sample(r.get_sample_data(i))
            for c, enc, part in zip(r.column_names, r.column_encodings, parts):
                if enc.split(':')[0] not in DEVICE_ENCODINGS:
                    continue
                try:
                    rec = gu.value_record(mds_oracle.mds_decode(enc, part))
                except UnicodeDecodeError:
                    rec = {'t': 'error', 'exc': 'UnicodeDecodeError'}
                assert rec == expected[k][c], (name, k, c)
            k += 1
    assert k == len(expected)


def test_vectorized_fixed_matches_per_sample():
    name = 'config_b_small'
    idx = gu.index(name)
    d = os.path.join(gu.GOLDEN, name)
    for info in idx['shards']:
        cols = mds_oracle.decode_shard_columns(d, None, info)
        raw = gu.shard_bytes(name, info)
        vec = mds_oracle.decode_fixed_shard_vectorized(raw, info['column_sizes'])
        for (c, v), arr in zip(cols.items(), vec):
            assert np.array_equal(v[1], arr)


def test_oracle_empty_sample_raises_index_error(tmp_path):
    # get_sample_data raises IndexError on zero-byte samples (mds/reader.py:145-148).
    raw = np.uint32(1).tobytes() + np.array([12, 12], np.uint32).tobytes()
    (tmp_path / 'shard.00000.mds').write_bytes(raw)
    info = {'raw_data': {'basename': 'shard.00000.mds'}, 'column_names': ['a'],
            'column_encodings': ['bytes'], 'column_sizes': [None], 'samples': 1}
    r = mds_oracle.OracleMDSReader(str(tmp_path), None, info)
    with pytest.raises(IndexError):
        r.get_sample_data(0)
