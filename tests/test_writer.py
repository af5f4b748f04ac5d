"""streaming_amd.MDSWriter writes byte-identical shards and index.json to the reference writer
(pinned by the golden sets the reference wrote)."""

import hashlib
import json
import os

import numpy as np
import pytest

from streaming_amd.writer import MDSWriter, bytes_to_int, encode_fixed_shard, shard_config_bytes
from tests import golden_util as gu
from tests.golden import make_golden as mg


class NumberAndSay:
    """Restatement of regression/synthetic_dataset.py:80-158 (legacy np.random stream)."""
    ones = ('zero one two three four five six seven eight nine ten eleven twelve thirteen '
            'fourteen fifteen sixteen seventeen eighteen nineteen').split()
    tens = 'twenty thirty forty fifty sixty seventy eighty ninety'.split()

    def say(self, i):
        if i < 0:
            return ['negative'] + self.say(-i)
        if i <= 19:
            return [self.ones[i]]
        if i < 100:
            return [self.tens[i // 10 - 2]] + ([self.ones[i % 10]] if i % 10 else [])
        if i < 1_000:
            return [self.ones[i // 100], 'hundred'] + (self.say(i % 100) if i % 100 else [])
        if i < 1_000_000:
            return self.say(i // 1_000) + ['thousand'] + (self.say(i % 1_000) if i % 1_000 else [])
        return self.say(i // 1_000_000) + ['million'] + (self.say(i % 1_000_000)
                                                         if i % 1_000_000 else [])

    def samples(self, n, seed):
        np.random.seed(seed)
        out = []
        for _ in range(n):
            sign = (np.random.random() < 0.8) * 2 - 1
            mag = 10**np.random.uniform(1, 4) - 10
            number = sign * int(mag**2)
            out.append({'number': number, 'words': ' '.join(self.say(number))})
        return out


GENERATORS = {
    'kat': mg.gen_kat,
    'sequence': mg.gen_sequence,
    'config_b_small': mg.gen_config_b_small,
    'config_c_small': mg.gen_config_c_small,
    'scalars': mg.gen_scalars,
    'dynamic': mg.gen_dynamic,
    'bad_utf8': mg.gen_bad_utf8,
    'zstd': mg.gen_zstd,
    'wide': mg.gen_wide,
    'config_a': lambda: ({'number': 'int', 'words': 'str'}, NumberAndSay().samples(10_000, 987),
                         {'size_limit': 10240}),
}


@pytest.mark.parametrize('name', sorted(GENERATORS))
def test_writer_is_byte_identical(name, tmp_path):
    cols, samples, kwargs = GENERATORS[name]()
    out = tmp_path / name
    with MDSWriter(columns=cols, out=str(out), **kwargs) as w:
        for s in samples:
            w.write(s)
    ours = json.load(open(out / 'index.json'))
    ref = gu.index(name)
    if kwargs.get('compression'):
        # Compressed bytes depend on the zstd build; compare everything else and the raw shards.
        for a, b in zip(ours['shards'], ref['shards']):
            assert a['raw_data'] == b['raw_data']
            assert a['zip_data']['basename'] == b['zip_data']['basename']
            a = dict(a, zip_data=None)
            b = dict(b, zip_data=None)
            assert a == b
        for info in ours['shards']:
            raw = gu.shard_bytes(name, info)  # the reference's compressed file, decompressed
            assert hashlib.sha1(raw).hexdigest() == info['raw_data']['hashes']['sha1']
            assert len(raw) == info['raw_data']['bytes']
    else:
        assert ours == ref
        for info in ours['shards']:
            mine = (out / info['raw_data']['basename']).read_bytes()
            theirs = open(os.path.join(gu.GOLDEN, name, info['raw_data']['basename']), 'rb').read()
            assert mine == theirs


def test_encode_fixed_shard_matches_writer(tmp_path):
    cols, samples, _ = mg.gen_config_b_small()
    with MDSWriter(columns=cols, out=str(tmp_path / 'w'), size_limit=None) as w:
        for s in samples:
            w.write(s)
    ref = (tmp_path / 'w' / 'shard.00000.mds').read_bytes()
    info = json.load(open(tmp_path / 'w' / 'index.json'))['shards'][0]
    config = shard_config_bytes(info['column_names'], info['column_encodings'],
                                info['column_sizes'], None, [], None)
    ids = np.array([s['id'] for s in samples], np.int32)
    xs = np.stack([s['x'] for s in samples])
    assert encode_fixed_shard(config, [ids, xs]) == ref


def test_shard_count_formula(tmp_path):
    # test_writer.py:59-99 of the reference: ceil(N / ((limit - 8 - len(cfg)) // (size + 4))).
    cols = {'id': 'int32', 'x': 'ndarray:float32:1024'}
    limit = 1 << 16
    with MDSWriter(columns=cols, out=str(tmp_path / 'o'), size_limit=limit) as w:
        for i in range(100):
            w.write({'id': np.int32(i), 'x': np.zeros(1024, np.float32)})
        cfg = len(w.config_data)
    per = (limit - 8 - cfg) // (4100 + 4)
    idx = json.load(open(tmp_path / 'o' / 'index.json'))
    assert len(idx['shards']) == -(-100 // per)


@pytest.mark.parametrize('text,value', [('100kb', 102400), ('1mb', 1 << 20), ('64', 64),
                                        ('12b', 12), (1 << 26, 1 << 26), ('1.5kb', 1536)])
def test_bytes_to_int(text, value):
    assert bytes_to_int(text) == value


def test_writer_rejects_bad_args(tmp_path):
    with pytest.raises(TypeError):
        MDSWriter(columns={'a': 'nope'}, out=str(tmp_path / 'a'))
    with pytest.raises(ValueError):
        MDSWriter(columns={'a': 'int'}, out=str(tmp_path / 'b'), size_limit=1 << 32)
    with pytest.raises(ValueError):
        MDSWriter(columns={'a': 'int'}, out=str(tmp_path / 'c'), hashes=['sha1', 'md5'])
    with pytest.raises(KeyError):
        with MDSWriter(columns={'a': 'int32'}, out=str(tmp_path / 'd')) as w:
            w.write({'a': b'123'})
