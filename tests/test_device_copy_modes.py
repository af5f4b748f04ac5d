"""GPU parity of every ragged-column copy mode of the decoder, each forced through the
measurement knobs (MDSX_TUNE, read at plan creation).

* The default: ragged batches of long samples (>= 3 KiB on average) through the streaming decode
  (mdsx_run.hip), shorter ones through the row-parallel decode (mdsx_rows.hip).
* The streaming decode for every sample size, with small, default and large rings / tiles.
* The row-parallel decode for every sample size: a fixed 32 KiB stage, the per-batch sizing, and
  a 2 KiB stage (tiles in several windows, samples over 2 KiB through the huge-row kernel).
* The register-copy decode (run=0,rows=0): destination-major gather kernel (short rows), four rows
  per wave in 16-lane groups (medium rows), one row per wave (long rows), the last either from
  registers or through the per-wave LDS-DMA ring (8 or 4 slots).

Whatever mode a column gets, the bytes, offsets and UTF-8 flags must equal the reference's.
"""

import json
import os
import tempfile

import numpy as np
import pytest
import torch

from oracle import mds_oracle
from streaming_amd import MDSWriter
from streaming_amd.decoder import Plan, decode_batch, stage_shards
from streaming_amd.synth import var_c_shards
from tests import golden_util as gu
from tests.test_device_decode import _device_digests

pytestmark = pytest.mark.gpu

MODES = {
    'default': '',
    # the streaming decode's modes below pin swave=0: by default batches whose samples fit the
    # one-sample-per-wave register window decode there (mdsx_swave.hip, modes swave*)
    'seg_default': 'swave=0',  # the round-5 default for long samples (seg_decode_kernel<7,..>)
    'run': 'run=8,rmin=0,swave=0',  # the streaming decode (mdsx_run.hip) whatever the sample size
    'run4': 'run=4,rmin=0,rkb=4,swave=0',  # small ring, 1-2-row tiles
    'run16': 'run=16,rmin=0,rkb=1024,swave=0',  # 32-row tiles
    # the streaming decode's lean path (seg_decode_kernel) for runs whose samples fit its ring,
    # the general path for the others, in the same launch
    'seg4': 'run=4,seg=1,rmin=0,rkb=4,swave=0',
    'seg8': 'run=8,seg=1,rmin=0,swave=0',
    'seg7': 'run=7,seg=1,rmin=0,swave=0',  # a 7 KiB ring (not a power of two: modulo addressing)
    # ... the run's lines past the ring touched; shared boundary lines with the default policy
    'seg7_touch': 'run=7,seg=1,rmin=0,rnt=1,sv=32,swave=0',
    'seg7_edge': 'run=7,seg=1,rmin=0,rnt=1,sv=128,swave=0',
    'run7': 'run=7,rmin=0,swave=0',  # ... the general path through it
    'seg16': 'run=16,seg=1,rmin=0,rkb=1024,swave=0',
    'seg8_nt': 'run=8,seg=1,rmin=0,rnt=1,swave=0',
    'seg16_64k': 'run=16,seg=1,rmin=0,rkb=64,swave=0',
    'seg8_wg1': 'run=8,seg=1,rmin=0,swg=1,swave=0',  # one wave (run) per workgroup
    'seg8_wg4': 'run=8,seg=1,rmin=0,swg=4,swave=0',  # four (the default is two)
    'seg8_xcd0': 'run=8,seg=1,rmin=0,xcd=0,swave=0',  # runs in launch order (default: by XCD)
    # the lean path's measured variants (mdsx_run.hip kV): early prologue, per-step slot release,
    # per-step waits
    'seg7_v1': 'run=7,seg=1,rmin=0,sv=1,swave=0',
    'seg7_v3': 'run=7,seg=1,rmin=0,sv=3,swave=0',
    'seg7_v7': 'run=7,seg=1,rmin=0,sv=7,swave=0',
    # one sample per one-wave workgroup, the sample in registers (mdsx_swave.hip), for every
    # sample size: the default 6 KiB window (larger samples straight from HBM), 4 KiB, a 1-row
    # tile, launch order, temporal loads / stores, registers bounded for 4 / 6 waves per SIMD
    'swave': 'swave=1,rmin=0',
    'swave4': 'swave=1,rmin=0,swkb=4,swtile=1',
    'swave_xcd0': 'swave=1,rmin=0,xcd=0,swtile=256',
    'swave_temporal': 'swave=1,rmin=0,rnt=0',
    'swave_occ4': 'swave=1,rmin=0,swocc=4',
    'swave_occ6': 'swave=1,rmin=0,swocc=6',
    'rows': 'rows=32,rmin=1000000000',  # the row-parallel decode (mdsx_rows.hip) for every size
    'rows_auto': 'rows=-1,rmin=1000000000',  # ... its tiles and stage sized per batch
    'rows_small': 'rows=2,rmin=1000000000',  # a 2 KiB stage: windows and HBM-direct samples
    'rows_xcd': 'rows=-1,rmin=1000000000,xcdr=1',  # row-parallel tiles in XCD-contiguous ranges
    'rows_temporal': 'rows=-1,rownt=0,rmin=1000000000',  # temporal loads / stores (default: nt)
    # several tiles per workgroup through two stages, the next tile's DMA in flight
    'rows_pipe': 'rows=-1,rpipe=4,rmin=1000000000',
    'rows_pipe_small': 'rows=2,rpipe=3,rmin=1000000000',  # ... with windows and HBM-direct rows
    'rows_pipe_one': 'rows=8,rpipe=1,rmin=1000000000',  # one tile per workgroup, two stages
    'rows_occ6': 'rows=-1,rocc=6,rmin=1000000000',  # registers bounded for six waves per SIMD
    'rows_occ8': 'rows=12,rocc=8,rmin=1000000000',  # ... eight, smaller tiles
    # it lists; a 6 KiB ring (4 KiB windows) with small tiles and a 2 KiB fallback stage
    'gather': 'run=0,rows=0,gmin=1000000000',
    'group': 'run=0,rows=0,gmin=0,gmax=1000000000',
    'group_nt': 'run=0,rows=0,gmin=0,gmax=1000000000,strc=0',  # str rows streamed (non-temporal) too
    'wave': 'run=0,rows=0,gmin=0,gmax=0,ring=0',
    'wave_xcd0': 'run=0,rows=0,gmin=0,gmax=0,ring=0,xcdb=0',  # register tiles in launch order
    'ring': 'run=0,rows=0,gmin=0,gmax=0,ring=8',   # one row per wave through the LDS-DMA ring
    'ring4': 'run=0,rows=0,gmin=0,gmax=0,ring=4',
}


@pytest.fixture(scope='module', autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')


@pytest.fixture(params=sorted(MODES))
def mode(request, monkeypatch):
    monkeypatch.setenv('MDSX_TUNE', MODES[request.param])
    return request.param


def _plan(info):
    return Plan(info['column_names'], info['column_encodings'], info['column_sizes'])


@pytest.mark.parametrize('name', ['config_c_small', 'bad_utf8', 'config_a', 'dynamic', 'wide',
                                  'images', 'kat'])
def test_golden_sets(mode, name):
    idx = gu.index(name)
    plan = _plan(idx['shards'][0])
    data = [gu.shard_bytes(name, s) for s in idx['shards']]
    dec = decode_batch(plan, stage_shards(data, [s['samples'] for s in idx['shards']], plan))
    assert _device_digests(plan, dec) == gu.manifest()[name]['columns']


def test_alignment_sweep(mode):
    """All 16 source alignments x lengths 0..300 and up to 5000, bytes and 2-byte UTF-8 rows,
    in one shard per alignment; four rows of very different lengths share each wave."""
    rng = np.random.default_rng(11)
    for pad in range(16):
        name = 'a' * (pad + 1)
        cols = {name: 'bytes', 'z' + name: 'str'}
        lens = list(range(0, 301)) + [int(x) for x in rng.integers(0, 5000, 60)]
        rng.shuffle(lens)
        rows = [{name: rng.bytes(n), 'z' + name: 'é' * (n % 97) + 'x' * (n % 3)} for n in lens]
        with tempfile.TemporaryDirectory() as t:
            with MDSWriter(columns=cols, out=t, size_limit=None) as w:
                for r in rows:
                    w.write(r)
            info = json.load(open(os.path.join(t, 'index.json')))['shards'][0]
            raw = open(os.path.join(t, info['raw_data']['basename']), 'rb').read()
        p = _plan(info)
        dec = decode_batch(p, stage_shards([raw], [info['samples']], p))
        b, s = dec[name], dec['z' + name]
        bv, bo = b.values.cpu().numpy(), b.offsets.cpu().numpy()
        sv, so = s.values.cpu().numpy(), s.offsets.cpu().numpy()
        for k, r in enumerate(rows):
            assert bv[bo[k]:bo[k + 1]].tobytes() == r[name], (mode, pad, k)
            assert sv[so[k]:so[k + 1]].tobytes().decode() == r['z' + name], (mode, pad, k)
        assert int(s.flags.sum()) == 0


def test_invalid_utf8_rows_between_valid_ones(mode):
    """Bad sequences at every position of rows of 1..700 bytes: flags equal Python's decoder."""
    rng = np.random.default_rng(3)
    bad_bits = [b'\xc0\x80', b'\xed\xa0\x80', b'\xf4\x90\x80\x80', b'\xe2\x82', b'\x80', b'\xff']
    rows, want = [], []
    for k in range(1500):
        n = int(rng.integers(1, 700))
        body = bytearray(('ü' * n).encode()[:n])
        if k % 3 == 0:
            pos = int(rng.integers(0, n))
            body[pos:pos] = bad_bits[k % len(bad_bits)]
        data = bytes(body)
        rows.append(data)
        try:
            data.decode('utf-8')
            want.append(0)
        except UnicodeDecodeError:
            want.append(1)
    # write the raw bytes as 'str' values through the bytes encoding path of the writer
    with tempfile.TemporaryDirectory() as t:
        with MDSWriter(columns={'s': 'bytes', 'k': 'int'}, out=t, size_limit=None) as w:
            for k, r in enumerate(rows):
                w.write({'s': r, 'k': k})
        info = json.load(open(os.path.join(t, 'index.json')))['shards'][0]
        raw = open(os.path.join(t, info['raw_data']['basename']), 'rb').read()
    info = dict(info, column_encodings=['int', 'str'])  # columns are sorted: k, s
    p = _plan(info)
    dec = decode_batch(p, stage_shards([raw], [info['samples']], p))
    s = dec['s']
    v, o = s.values.cpu().numpy(), s.offsets.cpu().numpy()
    for k, r in enumerate(rows):
        assert v[o[k]:o[k + 1]].tobytes() == r
    assert s.flags.cpu().numpy().tolist() == want


def test_config_c_full_shards(mode):
    shards, counts, src = var_c_shards(32_000, seed=8)
    plan = Plan(['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None])
    dec = decode_batch(plan, stage_shards(shards, counts, plan))
    assert np.array_equal(dec['n'].cpu().numpy(), src['n'])
    assert np.array_equal(dec['b'].values.cpu().numpy(), src['b_pool'])
    assert np.array_equal(dec['s'].values.cpu().numpy(), src['s_pool'])
    assert np.array_equal(dec['s'].offsets.cpu().numpy(),
                          np.concatenate([[0], np.cumsum(src['s_len'])]))
    assert int(dec['s'].flags.sum()) == 0


def test_oracle_on_random_rows(mode, tmp_path):
    rng = np.random.default_rng(17)
    cols = {'a': 'bytes', 'b': 'str', 'c': 'int'}
    with MDSWriter(columns=cols, out=str(tmp_path), size_limit=1 << 16) as w:
        for _ in range(3000):
            w.write({'a': rng.bytes(int(rng.choice([0, 3, 64, 255, 256, 257, 900, 2000]))),
                     'b': 'abé中\U0001f600' * int(rng.integers(0, 60)),
                     'c': int(rng.integers(-2**40, 2**40))})
    idx = json.load(open(tmp_path / 'index.json'))
    plan = _plan(idx['shards'][0])
    data = [open(tmp_path / s['raw_data']['basename'], 'rb').read() for s in idx['shards']]
    dec = decode_batch(plan, stage_shards(data, [s['samples'] for s in idx['shards']], plan))
    base = {'a': 0, 'b': 0}
    row = 0
    for info in idx['shards']:
        want = mds_oracle.decode_shard_columns(str(tmp_path), None, info)
        n = info['samples']
        for c in ('a', 'b'):
            got = dec[c]
            offs = got.offsets.cpu().numpy()[row:row + n + 1]
            vals = got.values.cpu().numpy()[offs[0]:offs[-1]]
            assert np.array_equal(offs - offs[0], want[c][2]), (mode, c)
            assert np.array_equal(vals, want[c][1]), (mode, c)
            base[c] += len(vals)
        row += n
