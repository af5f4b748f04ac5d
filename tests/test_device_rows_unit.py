"""GPU parity of the row-parallel decode's single pass (``MDSX_TUNE runit=1``, mdsx_rows.hip
kUnit): no scan pass; units of 256 samples drawn from a ticket counter, each publishing the ragged
bytes of the unit ``rahead`` places on and finding its own output base by a look-back.

The decode tests of ``test_device_decode`` run here a third time, every ragged batch through the
unit form (``decode_batch`` switched to the single pass, the row-parallel decode forced for every
sample size): golden fixtures against the reference's digests, oracle comparisons, and the
malformed-shard errors (header, offsets past the file, heads larger than their sample, empty
samples). The tests below add what only the unit form has: a look-back over thousands of units
with every publication made ahead, the capacity check per tile, and bit-identity with the
two-pass decode on the short-row benchmark shape.
"""

import numpy as np
import pytest
import torch

import streaming_amd.decoder as D
import streaming_amd.local
import tests.test_device_decode as device_decode
from streaming_amd.decoder import BatchDecoder, Plan, RaggedColumn, stage_shards
from streaming_amd.synth import var_c_shards
from tests.test_device_decode import (test_alignment_sweep, test_error_empty_sample_is_index_error,
                                      test_error_head_larger_than_sample,
                                      test_error_offsets_past_file,
                                      test_error_sample_count_mismatch, test_error_table_past_file,
                                      test_golden_batch_decode_matches_reference,
                                      test_ragged_many_tiny_rows,
                                      test_ragged_row_spanning_many_tiles,
                                      test_random_schemas_match_oracle)

pytestmark = pytest.mark.gpu

UNIT = 'runit=1,rmin=1000000000'
_two_pass = D.decode_batch


def _single(plan, batch, check=True, single=True):
    return _two_pass(plan, batch, check=check, single=single)


@pytest.fixture(autouse=True)
def _unit_single_pass(monkeypatch):
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')
    monkeypatch.setenv('MDSX_TUNE', UNIT)
    for mod in (D, streaming_amd.local, device_decode):
        monkeypatch.setattr(mod, 'decode_batch', _single)


C_PLAN = (['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None])


def _equal(one, two):
    for name, x in one.columns.items():
        y = two.columns[name]
        if isinstance(x, RaggedColumn):
            assert torch.equal(x.offsets, y.offsets), name
            assert torch.equal(x.values, y.values), name
            if x.flags is not None:
                assert torch.equal(x.flags, y.flags), name
        else:
            assert torch.equal(x.reshape(x.shape[0], -1).view(torch.uint8),
                               y.reshape(y.shape[0], -1).view(torch.uint8)), name


@pytest.mark.parametrize('unit,ahead', [(1, 1), (1, 7), (1, 4096), (1, 100000), (2, 64),
                                        (4, 1), (4, 4096)])
def test_unit_short_rows_equal_two_pass(monkeypatch, unit, ahead):
    """The short-row benchmark shape (32-256-byte blobs, 8-64-code-point strings of 1-4-byte
    code points), 400k samples = 6250 tiles: bit-identical to scan + decode for units of one tile
    in workgroup order (runit=1) or from the ticket counter (2) and of four tiles (4), whether
    every unit publishes its own bytes (ahead >= units) or a later unit's."""
    shards, counts, src = var_c_shards(400_000, seed=61, blob_bytes=(32, 256), str_chars=(8, 64))
    monkeypatch.setenv('MDSX_TUNE', f'runit={unit},rmin=1000000000,rahead={ahead}')
    plan = Plan(*C_PLAN)
    batch = stage_shards(shards, counts, plan)
    one = _two_pass(plan, batch, single=True)
    monkeypatch.setenv('MDSX_TUNE', 'rmin=1000000000')
    two = _two_pass(Plan(*C_PLAN), batch, single=False)
    _equal(one, two)
    assert np.array_equal(one['b'].values.cpu().numpy(), src['b_pool'])
    assert np.array_equal(one['s'].values.cpu().numpy(), src['s_pool'])


def test_unit_repeated_runs_identical():
    """A decoder re-running the unit form (its ticket and look-back words reset each call)."""
    shards, counts, _ = var_c_shards(50_000, seed=62, blob_bytes=(32, 256), str_chars=(8, 64))
    plan = Plan(*C_PLAN)
    dec = BatchDecoder(plan, stage_shards(shards, counts, plan), single=True)
    first = dec.run()
    dec.check()
    ref = {k: (v.values.clone(), v.offsets.clone()) if isinstance(v, RaggedColumn) else v.clone()
           for k, v in first.columns.items()}
    for _ in range(3):
        out = dec.run()
        dec.check()
        for k, v in out.columns.items():
            if isinstance(v, RaggedColumn):
                assert torch.equal(v.values, ref[k][0]) and torch.equal(v.offsets, ref[k][1])
            else:
                assert torch.equal(v, ref[k])


def test_unit_capacity_overflow_reports_capacity():
    shards, counts, src = var_c_shards(3000, seed=63, blob_bytes=(32, 256), str_chars=(8, 64))
    plan = Plan(*C_PLAN)
    batch = stage_shards(shards, counts, plan)
    need = int(src['b_len'].sum())
    dec = BatchDecoder(plan, batch, capacities={'b': need - 1, 's': 1 << 24}, single=True)
    dec.run()
    with pytest.raises(RuntimeError, match='capacity'):
        dec.check()
    ok = BatchDecoder(plan, batch, capacities={'b': need, 's': int(src['s_len'].sum())},
                      single=True)
    out = ok.run()
    ok.check()
    assert np.array_equal(out['b'].values.cpu().numpy(), src['b_pool'])
