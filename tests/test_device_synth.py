"""The benchmark's device-built workloads (bench.py): per-global-shard config B and C shards are
the files the (host, oracle-pinned) MDS writer produces for the same samples, decode bit-exact
to their sources, and do not depend on which rank builds them."""

import numpy as np
import pytest
import torch

from oracle import mds_oracle
from streaming_amd.decoder import decode_batch
from streaming_amd.synth import (CONFIG_C, _schema, fixed_b_batch_on_device, utf8_encode_device,
                                 var_c_batch_on_device, var_c_columns_on_device)
from streaming_amd.writer import shard_config_bytes

pytestmark = pytest.mark.gpu


def _shard(batch, s):
    o = batch.offsets[s]
    return batch.buffer[o:o + batch.sizes[s]].cpu().numpy().tobytes()


def test_utf8_encode_device_matches_python():
    rng = np.random.default_rng(5)
    cps = np.concatenate([rng.integers(0x20, 0x7F, 500), rng.integers(0x80, 0x800, 500),
                          rng.integers(0xE000, 0x10000, 500), rng.integers(0x10000, 0x110000, 500),
                          [0x7F, 0x80, 0x7FF, 0x800, 0xD7FF, 0xE000, 0xFFFF, 0x10000, 0x10FFFF]])
    out, nb = utf8_encode_device(torch.from_numpy(cps).cuda())
    want = ''.join(map(chr, cps.tolist())).encode('utf-8')
    assert out.cpu().numpy().tobytes() == want
    assert nb.cpu().tolist() == [len(chr(c).encode('utf-8')) for c in cps.tolist()]


def test_config_c_device_shards_are_writer_shards():
    size_limit = 1 << 20  # small shards, same generator and split rule as the benchmark's
    synth = var_c_batch_on_device([3, 11], seed=2000, size_limit=size_limit)
    names, encs, sizes = _schema(CONFIG_C)
    config = shard_config_bytes(names, encs, sizes, None, [], size_limit)
    cols = synth.sources
    n = cols['n'].cpu().numpy()
    b_vals, b_off = cols['b'].values.cpu().numpy(), cols['b'].offsets.cpu().numpy()
    s_vals, s_off = cols['s'].values.cpu().numpy(), cols['s'].offsets.cpu().numpy()
    row = 0
    for s, count in enumerate(synth.samples_per_shard):
        samples = []
        for i in range(row, row + count):  # column order b, n, s (sorted names)
            samples.append(mds_oracle.encode_sample_from_columns(
                [('var', b_vals, b_off), ('fixed', n.view(np.uint8).reshape(-1, 8)),
                 ('var', s_vals, s_off)], i))
            assert s_vals[s_off[i]:s_off[i + 1]].tobytes().decode('utf-8')  # valid UTF-8
        # the writer's flush rule puts exactly these rows in one shard
        sizes_ = [len(x) for x in samples]
        assert mds_oracle.writer_split(sizes_ + [10**9], size_limit, 8 + len(config))[0] == count
        assert _shard(synth.batch, s) == mds_oracle.encode_joint_shard(config, samples)
        row += count
    out = decode_batch(synth.plan, synth.batch)
    assert torch.equal(out['n'], cols['n'])
    for name in ('b', 's'):
        assert torch.equal(out[name].values, cols[name].values)
        assert torch.equal(out[name].offsets, cols[name].offsets - cols[name].offsets[0])
    assert int(out['s'].flags.sum()) == 0


def test_global_shards_independent_of_rank_split():
    a = var_c_batch_on_device([0, 1, 2], size_limit=1 << 20)
    b = var_c_batch_on_device([2], size_limit=1 << 20)
    assert _shard(a.batch, 2) == _shard(b.batch, 0)
    x = fixed_b_batch_on_device(0, seed=1000, size_limit=1 << 20, shard_ids=[4, 5])
    y = fixed_b_batch_on_device(0, seed=1000, size_limit=1 << 20, shard_ids=[5])
    assert _shard(x.batch, 1) == _shard(y.batch, 0)
    ids = np.frombuffer(_shard(y.batch, 0), np.uint8)
    out = decode_batch(y.plan, y.batch)
    per = y.samples_per_shard[0]
    assert out['id'].cpu().tolist() == list(range(5 * per, 6 * per))
    assert len(ids) == y.batch.sizes[0]


def test_full_size_config_c_columns_are_64mib_shards():
    parts, counts = var_c_columns_on_device([7])
    cols = parts[0]
    names, encs, sizes = _schema(CONFIG_C)
    config = shard_config_bytes(names, encs, sizes, None, [], 1 << 26)
    b_len = torch.diff(cols['b'].offsets)
    s_len = torch.diff(cols['s'].offsets)
    total = 8 + len(config) + int((8 + b_len + 8 + s_len + 4).sum())
    assert total <= 1 << 26
    assert (1 << 26) - total < 8 + 5120 + 8 + 4 * 256 + 4  # full: no room for a largest sample
    assert 15_000 < counts[0] < 16_500
