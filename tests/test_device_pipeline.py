"""GPU: the host pipeline (files / zstd -> pinned -> H2D -> decode) and the Stream plugin give
the reference's outputs."""

import hashlib
import os

import numpy as np
import pytest
import torch

from streaming_amd.decoder import Plan, RaggedColumn
from streaming_amd.pipeline import ShardPipeline, shard_files_from_index, to_host
from streaming_amd.plugin import make_device_stream
from tests import golden_util as gu
from tests.test_plugin import FakeStream, _ref_like_reader

pytestmark = pytest.mark.gpu


def _merge(parts):
    """Concatenate per-batch device outputs into reference-format column arrays."""
    merged = {}
    for name in parts[0]:
        vals = [p[name] for p in parts]
        if isinstance(vals[0], RaggedColumn):
            values = np.concatenate([v.values.cpu().numpy() for v in vals])
            offs, base = [np.zeros(1, np.int64)], 0
            for v in vals:
                o = v.offsets.cpu().numpy()
                offs.append(o[1:] + base)
                base += int(o[-1])
            merged[name] = (values, np.concatenate(offs))
        else:
            merged[name] = np.concatenate(
                [v.reshape(v.shape[0], -1).view(torch.uint8).cpu().numpy() for v in vals])
    return merged


@pytest.mark.parametrize('name,per,depth', [('zstd', 1, 2), ('config_c_small', 1, 2),
                                            ('config_a', 5, 2), ('config_a', 64, 2),
                                            ('wide', 3, 2), ('config_a', 7, 1), ('config_a', 3, 3)])
def test_pipeline_matches_reference(name, per, depth):
    d = os.path.join(gu.GOLDEN, name)
    idx = gu.index(name)
    info = idx['shards'][0]
    plan = Plan(info['column_names'], info['column_encodings'], info['column_sizes'])
    files = shard_files_from_index(d, idx)
    pipe = ShardPipeline(plan, files, shards_per_batch=per, depth=depth, workers=4)
    parts = []
    for b in pipe:
        parts.append({k: (RaggedColumn(v.values.clone(), v.offsets.clone()) if isinstance(
            v, RaggedColumn) else v.clone()) for k, v in b.columns.items()})
    pipe.close()
    m = gu.manifest()[name]['columns']
    for cname, v in _merge(parts).items():
        if isinstance(v, tuple):
            assert hashlib.sha256(v[0].tobytes()).hexdigest() == m[cname]['values']
            assert hashlib.sha256(v[1].tobytes()).hexdigest() == m[cname]['offsets']
        else:
            assert hashlib.sha256(v.tobytes()).hexdigest() == m[cname]['rows']


def test_to_host_handoff():
    d = os.path.join(gu.GOLDEN, 'kat')
    idx = gu.index('kat')
    info = idx['shards'][0]
    plan = Plan(info['column_names'], info['column_encodings'], info['column_sizes'])
    pipe = ShardPipeline(plan, shard_files_from_index(d, idx), workers=1)
    host = to_host(next(iter(pipe)))
    pipe.close()
    assert host['a'].tolist() == [-2, 7]
    vals, offs, flags = host['s']
    assert bytes(vals[offs[0]:offs[1]]).decode() == 'hé' and flags.tolist() == [0, 0]


@pytest.mark.parametrize('name,per,depth', [('config_a', 3, 2), ('config_c_small', 1, 2),
                                            ('zstd', 1, 1), ('wide', 2, 3)])
def test_iter_host_matches_reference(name, per, depth):
    """Host hand-off with the D2H overlapped (ShardPipeline.iter_host): every batch, in order,
    gives the reference's column digests once concatenated."""
    d = os.path.join(gu.GOLDEN, name)
    idx = gu.index(name)
    info = idx['shards'][0]
    plan = Plan(info['column_names'], info['column_encodings'], info['column_sizes'])
    pipe = ShardPipeline(plan, shard_files_from_index(d, idx), shards_per_batch=per, depth=depth,
                         workers=4)
    batches = list(pipe.iter_host())
    pipe.close()
    assert len(batches) == len(pipe.groups)
    m = gu.manifest()[name]['columns']
    for cname in batches[0]:
        if isinstance(batches[0][cname], tuple):
            values = np.concatenate([b[cname][0] for b in batches])
            offs, base = [np.zeros(1, np.int64)], 0
            for b in batches:
                offs.append(b[cname][1][1:] + base)
                base += int(b[cname][1][-1])
            assert hashlib.sha256(values.tobytes()).hexdigest() == m[cname]['values']
            assert hashlib.sha256(np.concatenate(offs).tobytes()).hexdigest() == \
                m[cname]['offsets']
        else:
            rows = np.concatenate([b[cname].reshape(b[cname].shape[0], -1).view(np.uint8)
                                   for b in batches])
            assert hashlib.sha256(rows.tobytes()).hexdigest() == m[cname]['rows']


@pytest.mark.parametrize('name', ['kat', 'scalars', 'bad_utf8'])
def test_plugin_stream_get_item(name):
    d = os.path.join(gu.GOLDEN, name)

    class Base(FakeStream):

        def get_shards(self, world, allow_unsafe_types):
            return [_ref_like_reader(info, self.local) for info in gu.index(name)['shards']]

    shards = make_device_stream(Base)(d).get_shards(None, False)
    expected = gu.items(name)
    k = 0
    for r in shards:
        for i in range(len(r)):
            rec = expected[k]
            if any(w['t'] == 'error' for w in rec.values()):
                with pytest.raises(UnicodeDecodeError):
                    r[i]
            else:
                s = r[i]
                assert {c: gu.value_record(v) for c, v in s.items()} == rec
            k += 1
    assert k == len(expected)


@pytest.mark.parametrize('name,algo', [('zstd', 'xxh64'), ('zstd', 'sha1'),
                                       ('zstd_xxh3', 'xxh3_64'), ('zstd_xxh3', 'xxh128')])
def test_pipeline_validate_hash(name, algo):
    """validate_hash as Stream._prepare_shard_part (stream.py:401-411; hashing.py:24-26): xxh3_64
    and xxh128 on the device over the resident batch (PIPELINE_DEVICE_HASHES), xxh64 and sha1 on
    the pipeline's host threads, in place in the pinned staging. The digests the reference writer
    recorded in index.json (tests/golden/make_golden.py) pass; a wrong one raises 'Checksum
    failure' before the batch is handed out."""
    from streaming_amd.pipeline import PIPELINE_DEVICE_HASHES
    d = os.path.join(gu.GOLDEN, name)
    idx = gu.index(name)
    info = idx['shards'][0]
    plan = Plan(info['column_names'], info['column_encodings'], info['column_sizes'])
    files = shard_files_from_index(d, idx)
    assert all(f.hashes.get(algo) for f in files)  # the reference's own digests
    pipe = ShardPipeline(plan, files, shards_per_batch=1, workers=2, validate_hash=algo)
    assert pipe._device_hash == (algo in PIPELINE_DEVICE_HASHES)
    parts = []
    for b in pipe:
        parts.append({k: (RaggedColumn(v.values.clone(), v.offsets.clone()) if isinstance(
            v, RaggedColumn) else v.clone()) for k, v in b.columns.items()})
    pipe.close()
    m = gu.manifest()[name]['columns']
    for cname, v in _merge(parts).items():
        if isinstance(v, tuple):
            assert hashlib.sha256(v[0].tobytes()).hexdigest() == m[cname]['values']
        else:
            assert hashlib.sha256(v.tobytes()).hexdigest() == m[cname]['rows']
    digest = files[-1].hashes[algo]
    files[-1].hashes = dict(files[-1].hashes, **{algo: digest[:-1] + ('0' if digest[-1] != '0'
                                                                      else '1')})
    pipe = ShardPipeline(plan, files, shards_per_batch=1, workers=2, validate_hash=algo)
    with pytest.raises(ValueError, match='Checksum failure'):
        for _ in pipe:
            pass
    pipe.close()


def _config_e_files(tmp, cfg):
    """Full-size config E: 64 MiB shards written with compression='zstd'
    (level 3, stream.py:319-351 / compression.py:243-258 decompress them); B-compressible
    (small integers as float32) or config C. Two full shards and a partial one."""
    from streaming_amd.compression import compress
    from streaming_amd.pipeline import ShardFile
    from streaming_amd.synth import config_b_samples_per_shard, var_c_shards
    from streaming_amd.writer import encode_fixed_shard, shard_config_bytes
    rng = np.random.default_rng(11)
    if cfg == 'B':
        names, encs, sizes = ['id', 'x'], ['int32', 'ndarray:float32:1024'], [4, 4096]
        config = shard_config_bytes(names, encs, sizes, 'zstd', [], 1 << 26)
        per = config_b_samples_per_shard()
        counts = [per, per, 1234]
        total = sum(counts)
        x = rng.integers(0, 256, (total, 1024)).astype(np.float32)
        first = np.concatenate([[0], np.cumsum(counts)])
        raws = [encode_fixed_shard(config, [np.arange(a, b, dtype=np.int32), x[a:b]])
                for a, b in zip(first[:-1], first[1:])]
        src = {'x': x}
    else:
        names, encs, sizes = ['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None]
        raws, counts, src = var_c_shards(34000, seed=12)
        assert len(counts) == 3 and max(len(r) for r in raws[:2]) > 60 << 20
    files = []
    for i, (raw, n) in enumerate(zip(raws, counts)):
        path = os.path.join(tmp, f'shard.{i:05}.mds.zstd')
        with open(path, 'wb') as f:
            f.write(compress('zstd', raw))
        files.append(ShardFile(path, len(raw), n, 'zstd', {}))
    return Plan(names, encs, sizes), files, counts, src


def _check_e_host(cfg, host, src, r0, r1):
    if cfg == 'B':
        assert np.array_equal(host['id'], np.arange(r0, r1, dtype=np.int32))
        assert np.array_equal(host['x'].view(np.uint32), src['x'][r0:r1].view(np.uint32))
        return
    assert np.array_equal(host['n'], src['n'][r0:r1])
    for name in ('b', 's'):
        lens = src[name + '_len']
        off = np.concatenate([[0], np.cumsum(lens)])
        vals, offs = host[name][0], host[name][1]
        assert np.array_equal(offs, off[r0:r1 + 1] - off[r0])
        assert np.array_equal(vals, src[name + '_pool'][off[r0]:off[r1]])
    assert not host['s'][2].any()


def _check_e_device(cfg, out, src, r0, r1):
    """The device hand-off compared on the device, against the sources uploaded."""
    dev = out.columns[next(iter(out.columns))]
    dev = (dev.offsets if isinstance(dev, RaggedColumn) else dev).device

    def same(got, exp):
        exp = torch.from_numpy(np.ascontiguousarray(exp)).to(dev)
        assert got.shape == exp.shape and torch.equal(got, exp)

    if cfg == 'B':
        same(out['id'], np.arange(r0, r1, dtype=np.int32))
        same(out['x'].view(torch.int32), src['x'][r0:r1].view(np.int32))
        return
    same(out['n'], src['n'][r0:r1])
    for name in ('b', 's'):
        off = np.concatenate([[0], np.cumsum(src[name + '_len'])])
        same(out[name].offsets, off[r0:r1 + 1] - off[r0])
        same(out[name].values, src[name + '_pool'][off[r0]:off[r1]])
    assert not bool(out['s'].flags.any())


@pytest.fixture(scope='module', params=['B', 'C'])
def config_e(request, tmp_path_factory):
    tmp = tmp_path_factory.mktemp(f'config_e_{request.param}')
    return (request.param, ) + _config_e_files(str(tmp), request.param)


@pytest.mark.parametrize('handoff,per,depth', [('device', 1, 2), ('device', 2, 2),
                                               ('iter_host', 1, 2), ('iter_host', 1, 3),
                                               ('to_host', 2, 1)])
def test_pipeline_full_size_config_e(config_e, handoff, per, depth):
    """Full 64 MiB zstd shards (config E) through host decompress -> pinned -> H2D -> device
    decode, bit-exact against the columns the shards were written from, with the device
    hand-off, the overlapped host hand-off (iter_host) and a blocking to_host."""
    cfg, plan, files, counts, src = config_e
    pipe = ShardPipeline(plan, files, shards_per_batch=per, depth=depth, workers=4)
    first = np.concatenate([[0], np.cumsum(counts)])
    if handoff == 'iter_host':
        outs = pipe.iter_host()
    elif handoff == 'to_host':
        outs = (to_host(b) for b in pipe)
    else:
        outs = iter(pipe)
    n = 0
    for gi, out in enumerate(outs):
        s0 = gi * per
        s1 = min(s0 + per, len(files))
        if handoff == 'device':
            _check_e_device(cfg, out, src, int(first[s0]), int(first[s1]))
        else:
            _check_e_host(cfg, out, src, int(first[s0]), int(first[s1]))
        n += 1
    pipe.close()
    assert n == len(pipe.groups)
