"""Synthetic config builders produce exactly what MDSWriter writes for the same samples."""

import json

import numpy as np

from streaming_amd.synth import CONFIG_C, shard_split, utf8_pool, var_c_shards
from streaming_amd.writer import MDSWriter


def test_utf8_pool_is_valid_utf8():
    rng = np.random.default_rng(0)
    pool, nbytes = utf8_pool(rng, 10_000)
    text = pool.tobytes().decode('utf-8')
    assert len(text) == 10_000
    assert [len(c.encode()) for c in text] == nbytes.tolist()


def test_var_c_matches_writer(tmp_path):
    shards, counts, src = var_c_shards(300, seed=3, size_limit=1 << 18)
    assert sum(counts) == 300 and len(counts) > 1
    b_off = np.concatenate([[0], np.cumsum(src['b_len'])])
    s_off = np.concatenate([[0], np.cumsum(src['s_len'])])
    with MDSWriter(columns=CONFIG_C, out=str(tmp_path / 'w'), size_limit=1 << 18) as w:
        for i in range(300):
            w.write({
                'n': int(src['n'][i]),
                'b': src['b_pool'][b_off[i]:b_off[i + 1]].tobytes(),
                's': src['s_pool'][s_off[i]:s_off[i + 1]].tobytes().decode('utf-8'),
            })
    idx = json.load(open(tmp_path / 'w' / 'index.json'))
    assert [s['samples'] for s in idx['shards']] == counts
    for info, mine in zip(idx['shards'], shards):
        assert (tmp_path / 'w' / info['raw_data']['basename']).read_bytes() == mine


def test_shard_split_rule():
    # size_limit < cur + size + 4 flushes; cur starts at 8 + len(config)
    assert shard_split(np.array([10, 10, 10]), 0, 8 + 14 + 14) == [2, 1]
    assert shard_split(np.array([10, 10, 10]), 0, 8 + 14 + 13) == [1, 1, 1]
    assert shard_split(np.array([10, 10, 10]), 0, None) == [3]
