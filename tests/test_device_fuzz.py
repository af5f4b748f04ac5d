"""GPU fuzz: random schemas and samples (every encoding the device decodes, empty and odd-sized
values, shards of 4 KiB .. 1 MiB) through every decode mode, and the multi-source gather, against
the oracle's reading of the same shard files.

The default run takes a few seeds; ``MDSX_FUZZ_SEEDS=N`` (and ``MDSX_FUZZ_START``) widens it, e.g.
``MDSX_FUZZ_SEEDS=400 python -m pytest tests/test_device_fuzz.py -m gpu``.
"""

import json
import os

import numpy as np
import pytest
import torch

from oracle import mds_oracle
from streaming_amd.decoder import (BatchDecoder, Plan, RaggedColumn, decode_batch, gather_sources,
                                   stage_shards)
from tests.test_device_decode import _random_dataset

pytestmark = pytest.mark.gpu

START = int(os.environ.get('MDSX_FUZZ_START', '1000'))
SEEDS = int(os.environ.get('MDSX_FUZZ_SEEDS', '6'))
MODES = {
    'default': '',  # long samples: one per wave (mdsx_swave.hip); streaming modes pin swave=0
    'seg_default': 'swave=0',
    'run': 'run=4,rmin=0,rkb=8,swave=0',  # the streaming decode whatever the sample size
    'seg': 'run=4,seg=1,rmin=0,rkb=8,swave=0',  # ... its lean path where a sample fits the ring
    'seg16': 'run=16,seg=1,rmin=0,rkb=64,swave=0',
    'seg7': 'run=7,seg=1,rmin=0,rkb=12,swave=0',  # a ring of 7 slots (modulo addressing)
    'seg7_v7': 'run=7,seg=1,rmin=0,rkb=12,sv=7,swave=0',  # early prologue, per-step release / waits
    'seg7_edge': 'run=7,seg=1,rmin=0,rkb=12,sv=128,swave=0',  # ... boundary lines, default policy
    'seg7_v3': 'run=7,seg=1,rmin=0,sv=3,swave=0',  # ... and per-step release, 2-sample runs
    'seg_wg4': 'run=8,seg=1,rmin=0,swg=4,swave=0',  # four waves per workgroup (the default is two)
    'swave': 'swave=1,rmin=0',  # one sample per wave, in registers (larger ones from HBM)
    'swave4': 'swave=1,rmin=0,swkb=4,swtile=2',
    'rows_small': 'rows=2,rmin=1000000000',  # row-parallel, 2 KiB stage (windows, huge rows)
    'rows_pipe': 'rows=4,rpipe=5,rmin=1000000000',  # ... two stages, next tile's DMA in flight
    'register': 'run=0,rows=0',  # the register decode (+ gather / groups per column)
    'rowwave': 'rw=1,lpad=12',  # all-fixed plans: one row per wave (others: as the default)
}
# the single pass (mdsx_decode_shards_single), fresh and re-run with known totals
SINGLE_MODES = {
    'single': '',  # streaming / row-parallel batches: scan pass + decode, no host round trip
    'single_rows_small': 'rows=2,rmin=1000000000',  # ... row-parallel in windows, huge rows
    'single_rows_pipe': 'rows=4,rpipe=5,rmin=1000000000',  # ... two stages per workgroup
    'single_register': 'run=0,rows=0',  # the register decode's single-pass form (look-back)
    'single_swave': 'swave=1,rmin=0',  # scan pass + one sample per wave
}


def _oracle(d, idx):
    cols = {}
    for info in idx['shards']:
        for c, v in mds_oracle.decode_shard_columns(d, None, info).items():
            cols.setdefault(c, []).append(v)
    return cols


def _check(got, parts, where):
    if parts[0][0] == 'fixed':
        want = np.concatenate([p[1] for p in parts])
        have = got.reshape(got.shape[0], -1).view(torch.uint8).cpu().numpy()
        assert np.array_equal(have, want), where
    else:
        assert np.array_equal(got.values.cpu().numpy(), np.concatenate([p[1] for p in parts])), \
            where
        lens = np.concatenate([np.diff(p[2]) for p in parts])
        assert np.array_equal(np.diff(got.offsets.cpu().numpy()), lens), where
        if parts[0][3] is not None:
            assert np.array_equal(got.flags.cpu().numpy(), np.concatenate([p[3] for p in parts])), \
                where


@pytest.mark.parametrize('seed', range(START, START + SEEDS))
def test_fuzz_decode_and_gather(tmp_path, monkeypatch, seed):
    d = _random_dataset(tmp_path, seed)
    idx = json.load(open(os.path.join(d, 'index.json')))
    info = idx['shards'][0]
    want = _oracle(d, idx)
    data = [open(os.path.join(d, s['raw_data']['basename']), 'rb').read() for s in idx['shards']]
    counts = [s['samples'] for s in idx['shards']]
    for mode, tune in MODES.items():
        monkeypatch.setenv('MDSX_TUNE', tune)
        plan = Plan(info['column_names'], info['column_encodings'], info['column_sizes'])
        dec = decode_batch(plan, stage_shards(data, counts, plan))
        assert dec.rows == sum(counts)
        for c, parts in want.items():
            _check(dec[c], parts, (seed, mode, c))
    for mode, tune in SINGLE_MODES.items():
        monkeypatch.setenv('MDSX_TUNE', tune)
        plan = Plan(info['column_names'], info['column_encodings'], info['column_sizes'])
        batch = stage_shards(data, counts, plan)
        dec = decode_batch(plan, batch, single=True)
        for c, parts in want.items():
            _check(dec[c], parts, (seed, mode, c))
        # a two-pass decoder re-running with its totals known
        bd = BatchDecoder(plan, batch)
        bd.run()
        bd.check()
        again = bd.run()
        bd.check()
        for c, parts in want.items():
            _check(again[c], parts, (seed, mode, 'rerun', c))
    # multi-source gather: one source per shard, random ids (repeats, every shard)
    monkeypatch.setenv('MDSX_TUNE', '')
    plan = Plan(info['column_names'], info['column_encodings'], info['column_sizes'])
    sources = [decode_batch(plan, stage_shards([b], [n], plan)) for b, n in zip(data, counts)]
    rng = np.random.default_rng(seed)
    starts = np.concatenate([[0], np.cumsum(counts)])
    ids = rng.integers(0, starts[-1], int(rng.integers(1, 3 * starts[-1] + 2)))
    src = np.searchsorted(starts, ids, side='right') - 1
    g = gather_sources(sources, src, ids - starts[src])
    for c, parts in want.items():
        if parts[0][0] == 'fixed':
            rows = np.concatenate([p[1] for p in parts])[ids]
            have = g[c].reshape(g[c].shape[0], -1).view(torch.uint8).cpu().numpy()
            assert np.array_equal(have, rows.reshape(len(ids), -1)), (seed, 'gather', c)
        else:
            vals = np.concatenate([p[1] for p in parts])
            offs = np.concatenate([[0], np.cumsum(np.concatenate([np.diff(p[2]) for p in parts]))])
            got = g[c]
            gv, go = got.values.cpu().numpy(), got.offsets.cpu().numpy()
            for k, i in enumerate(ids):
                assert np.array_equal(gv[go[k]:go[k + 1]], vals[offs[i]:offs[i + 1]]), \
                    (seed, 'gather', c, k)
            if parts[0][3] is not None:
                flags = np.concatenate([p[3] for p in parts])
                assert np.array_equal(got.flags.cpu().numpy(), flags[ids]), (seed, 'gather', c)
