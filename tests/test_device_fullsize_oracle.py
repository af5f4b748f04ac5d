"""The bench's own workloads at full size, decoded on the GPU as bench.py builds and decodes them
(config B: 62 full 64 MiB shards, 1 013 824 samples; config C: 64 full shards, 963 880 samples),
checked against the oracle reading the same shard bytes -- not only against the encoded source
columns (bench.py's verify): EVERY sample of EVERY shard through the oracle's shard reader
(mds_oracle.decode_shard_columns over the shard's bytes: the reference's per-sample
get_sample_data + decode_sample, mds/reader.py:103-149), and the oracle's per-sample reader over
the shard FILE (OracleMDSReader.get_item: reference value types) on random samples of eight
shards spread over the batch."""

import numpy as np
import pytest
import torch

from oracle import mds_oracle

pytestmark = pytest.mark.gpu

N_FILES = 8  # shards written out for the per-sample reader
PER_FILE = 24  # random samples per written shard


def _workload(config):
    import bench
    from streaming_amd.decoder import BatchDecoder
    # (the plan and the batch's tiles are made under the caller's MDSX_TUNE)
    shard_ids = list(range(bench.SHARDS_PER_GPU[config]))
    synth, _ = bench.build_workload(config, shard_ids)
    dec = BatchDecoder(synth.plan, synth.batch)
    out = dec.run()
    dec.check()
    bench.verify(config, out, synth.sources)  # (raises on a mismatch with the sources)
    return synth, out


def _info(synth, s):
    names, encs, sizes = synth.plan.key
    return {'column_names': list(names), 'column_encodings': list(encs),
            'column_sizes': [sz or None for sz in sizes], 'samples': synth.batch.samples[s],
            'raw_data': {'basename': f'shard.{s:05d}.mds'}}


def _bytes(synth, s):
    b = synth.batch
    return b.buffer[b.offsets[s]:b.offsets[s] + b.sizes[s]].cpu().numpy().tobytes()


def _chosen(synth):
    n = synth.batch.nshards
    return sorted({round(i * (n - 1) / (N_FILES - 1)) for i in range(N_FILES)})


def test_config_b_full_size_vs_oracle(tmp_path):
    synth, out = _workload('B')
    b = synth.batch
    assert b.nshards == 62 and b.total_rows == 1_013_824
    ids = out['id'].cpu().numpy()
    x = out['x'].view(torch.uint8).view(b.total_rows, 4096)
    rng = np.random.default_rng(7)
    files = _chosen(synth)
    for s in range(b.nshards):  # every sample of every shard
        info, data = _info(synth, s), _bytes(synth, s)
        r0, n = b.row0[s], b.samples[s]
        xs = x[r0:r0 + n].cpu().numpy()
        want = mds_oracle.decode_shard_columns(None, None, info, data=data)
        assert np.array_equal(ids[r0:r0 + n].view(np.uint8).reshape(n, 4), want['id'][1]), s
        assert np.array_equal(xs, want['x'][1]), s
        if s in files:  # the per-sample reader over the file
            (tmp_path / info['raw_data']['basename']).write_bytes(data)
            ref = mds_oracle.OracleMDSReader(str(tmp_path), None, info)
            for i in rng.choice(n, PER_FILE, replace=False).tolist() + [0, n - 1]:
                item = ref.get_item(i)
                assert item['id'] == int(ids[r0 + i])
                assert item['x'].tobytes() == xs[i].tobytes()
            (tmp_path / info['raw_data']['basename']).unlink()


# config C through both decodes of its sample sizes: the default and the other one (the lean
# streaming decode / one sample per wave), each over the 4.3 GB batch (byte offsets past 2 and 4
# GiB)
@pytest.mark.parametrize('tune', ['', 'swave=0'])  # default: one sample per wave
def test_config_c_full_size_vs_oracle(tmp_path, monkeypatch, tune):
    monkeypatch.setenv('MDSX_TUNE', tune)
    synth, out = _workload('C')
    b = synth.batch
    assert b.nshards == 64 and b.total_rows == 963_880
    nv = out['n'].cpu().numpy()
    cols = {c: (out[c].values.cpu().numpy(), out[c].offsets.cpu().numpy()) for c in ('b', 's')}
    flags = out['s'].flags.cpu().numpy()
    rng = np.random.default_rng(11)
    files = _chosen(synth)
    for s in range(b.nshards):  # every sample of every shard
        info, data = _info(synth, s), _bytes(synth, s)
        r0, n = b.row0[s], b.samples[s]
        want = mds_oracle.decode_shard_columns(None, None, info, data=data)
        assert np.array_equal(nv[r0:r0 + n].view(np.uint8).reshape(n, 8), want['n'][1]), s
        for c, (vals, offs) in cols.items():
            o = offs[r0:r0 + n + 1]
            assert np.array_equal(vals[o[0]:o[-1]], want[c][1]), (s, c)
            assert np.array_equal(np.diff(o), np.diff(want[c][2])), (s, c)
        assert np.array_equal(flags[r0:r0 + n], want['s'][3]), s
        if s in files:  # the per-sample reader over the file
            (tmp_path / info['raw_data']['basename']).write_bytes(data)
            ref = mds_oracle.OracleMDSReader(str(tmp_path), None, info)
            for i in rng.choice(n, PER_FILE, replace=False).tolist() + [0, n - 1]:
                item = ref.get_item(i)
                k = r0 + i
                assert item['n'] == int(nv[k])
                bv, bo = cols['b']
                sv, so = cols['s']
                assert item['b'] == bv[bo[k]:bo[k + 1]].tobytes()
                assert item['s'] == sv[so[k]:so[k + 1]].tobytes().decode('utf-8')
            (tmp_path / info['raw_data']['basename']).unlink()
