"""GPU: batch gather by sample id against the oracle's per-sample decode."""

import os

import numpy as np
import pytest
import torch

from oracle import mds_oracle
from streaming_amd import LocalDataset
from streaming_amd.decoder import RaggedColumn
from streaming_amd.synth import fixed_b_batch_on_device
from tests import golden_util as gu

pytestmark = pytest.mark.gpu


def _oracle_rows(name):
    """Per-sample column bytes of a golden set through the oracle, in global order."""
    d = os.path.join(gu.GOLDEN, name)
    rows = []
    for info in gu.index(name)['shards']:
        r = mds_oracle.OracleMDSReader(d, None, info)
        for i in range(len(r)):
            rows.append(dict(zip(r.column_names, r.split_sample(r.get_sample_data(i)))))
    return rows


@pytest.mark.parametrize('name', ['config_b_small', 'config_c_small', 'scalars', 'bad_utf8',
                                  'wide', 'config_a'])
def test_gather_matches_oracle(name):
    rows = _oracle_rows(name)
    n = len(rows)
    rng = np.random.default_rng(len(name))
    ids = rng.integers(0, n, 3 * n + 5)
    ids[::7] = -1  # reference padding, skipped
    ds = LocalDataset(os.path.join(gu.GOLDEN, name))
    got = ds.decode_all().gather(ids)
    keep = ids[ids != -1]
    assert got.rows == len(keep)
    for cname, col in got.columns.items():
        if isinstance(col, RaggedColumn):
            vals, offs = col.values.cpu().numpy(), col.offsets.cpu().numpy()
            flags = col.flags.cpu().numpy() if col.flags is not None else None
            for k, r in enumerate(keep):
                assert vals[offs[k]:offs[k + 1]].tobytes() == rows[r][cname], (cname, k)
                if flags is not None:
                    assert flags[k] == (0 if mds_oracle.utf8_is_valid(rows[r][cname]) else 1)
        else:
            raw = col.reshape(col.shape[0], -1).view(torch.uint8).cpu().numpy()
            for k, r in enumerate(keep):
                assert raw[k].tobytes() == rows[r][cname], (cname, k)


def test_iter_batches_order():
    ds = LocalDataset(os.path.join(gu.GOLDEN, 'config_a'))
    ids = np.random.default_rng(0).permutation(len(ds))
    seen = []
    for b in ds.iter_batches(ids, 256):
        assert b.rows <= 256
        seen.extend(b['number'].cpu().tolist())
    want = [ds[int(i)]['number'] for i in ids[:500]]
    assert seen[:500] == want
    assert len(seen) == len(ds)


def test_gather_out_of_range_raises():
    ds = LocalDataset(os.path.join(gu.GOLDEN, 'kat'))
    with pytest.raises(IndexError):
        ds.decode_all().gather([0, 5])


def test_gather_config_b_full_size_permutation():
    synth = fixed_b_batch_on_device(1_000_000, seed=21)
    from streaming_amd.decoder import decode_batch
    dec = decode_batch(synth.plan, synth.batch)
    perm = torch.randperm(1_000_000, device=dec['x'].device)
    g = dec.gather(perm)
    assert torch.equal(g['id'], synth.sources['id'][perm])
    assert torch.equal(g['x'].view(torch.int32), synth.sources['x'].view(torch.int32)[perm])


@pytest.mark.parametrize('row', [4096 + 7, 300])
def test_ragged_gather_reads_only_inside_the_source_tensor(row):
    """The ragged gather copies from caller tensors with no padding: a row at the very start (or
    end) of a freshly mapped values allocation, landing at a misaligned destination, must be
    copied without touching bytes outside the tensor (it would fault). Long rows (one per wave)
    and medium rows (four per wave)."""
    from streaming_amd.decoder import DecodedBatch
    torch.cuda.empty_cache()
    n_bytes = (96 << 20) + 3  # its own segment, not a multiple of 16
    values = torch.randint(0, 256, (n_bytes, ), dtype=torch.uint8, device='cuda')
    lens = [5, 17, 1, 33] + [row] * ((n_bytes - (1 << 20)) // row)
    lens.append(n_bytes - sum(lens))
    offsets = torch.tensor(np.concatenate([[0], np.cumsum(lens)]), dtype=torch.int64,
                           device='cuda')
    col = RaggedColumn(values, offsets, None)
    n = len(lens)
    ids = [1, 0, 2, n - 1, 3, 0, n - 1] + list(range(4, n - 1))
    got = DecodedBatch({'v': col}, n).gather(ids)['v']
    v, o = got.values.cpu().numpy(), got.offsets.cpu().numpy()
    src, so = values.cpu().numpy(), offsets.cpu().numpy()
    for k, r in enumerate(ids):
        assert np.array_equal(v[o[k]:o[k + 1]], src[so[r]:so[r + 1]]), k


@pytest.mark.parametrize('name', ['config_b_small', 'config_c_small', 'config_a', 'bad_utf8',
                                  'dynamic'])
def test_gather_sources_matches_oracle(name):
    """Multi-source gather (mdsx_gather_*_multi): one launch sequence over every shard's decoded
    columns, rows in id order, against the oracle; also through DeviceSampleGather."""
    from streaming_amd.decoder import gather_sources
    rows = _oracle_rows(name)
    ds = LocalDataset(os.path.join(gu.GOLDEN, name))
    rng = np.random.default_rng(3 + len(name))
    ids = rng.integers(0, len(rows), 2 * len(rows) + 3)
    g = ds.sample_gather
    shard, local = g.locate(ids)
    sources = [ds.decode_all([s]) for s in range(len(ds.shards))]
    for got in (gather_sources(sources, shard, local), g.gather(ids)):
        assert got.rows == len(ids)
        for cname, col in got.columns.items():
            if isinstance(col, RaggedColumn):
                vals, offs = col.values.cpu().numpy(), col.offsets.cpu().numpy()
                flags = col.flags.cpu().numpy() if col.flags is not None else None
                for k, r in enumerate(ids):
                    assert vals[offs[k]:offs[k + 1]].tobytes() == rows[r][cname], (cname, k)
                    if flags is not None:
                        assert flags[k] == (0 if mds_oracle.utf8_is_valid(rows[r][cname]) else 1)
            else:
                raw = col.reshape(col.shape[0], -1).view(torch.uint8).cpu().numpy()
                for k, r in enumerate(ids):
                    assert raw[k].tobytes() == rows[r][cname], (cname, k)


def test_gather_sources_rejects_bad_ids():
    from streaming_amd.decoder import gather_sources
    ds = LocalDataset(os.path.join(gu.GOLDEN, 'config_c_small'))
    src = [ds.decode_all([0])]
    with pytest.raises(IndexError):
        gather_sources(src, np.array([0, 1]), np.array([0, 0]))  # no source 1
    with pytest.raises(IndexError):  # row past the source: found by the kernels
        gather_sources(src, np.array([0, 0]), np.array([0, src[0].rows]))


def test_gather_sources_config_b_full_size_four_sources():
    """1M config-B rows split into four sources (row-range views), permuted across them."""
    from streaming_amd.decoder import DecodedBatch, decode_batch, gather_sources
    synth = fixed_b_batch_on_device(1_000_000, seed=22)
    dec = decode_batch(synth.plan, synth.batch)
    cuts = [0, 250_000, 400_000, 999_999, 1_000_000]
    sources = [DecodedBatch({k: v[a:b] for k, v in dec.columns.items()}, b - a)
               for a, b in zip(cuts[:-1], cuts[1:])]
    perm = torch.randperm(1_000_000).numpy()
    src = np.searchsorted(np.array(cuts), perm, side='right') - 1
    g = gather_sources(sources, src, perm - np.array(cuts)[src])
    p = torch.from_numpy(perm).to(dec['x'].device)
    assert torch.equal(g['id'], synth.sources['id'][p])
    assert torch.equal(g['x'].view(torch.int32), synth.sources['x'].view(torch.int32)[p])
