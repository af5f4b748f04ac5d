"""GPU parity of the single-pass decode (``mdsx_decode_shards_single``: one launch sequence with
no host round trip, outputs sized at the payload bound; the register decode scans its own ragged
lengths by decoupled look-back, streaming and row-parallel batches run their scan pass and decode
back to back).

The decode tests of ``test_device_decode`` / ``test_device_copy_modes`` are collected here a
second time with ``decode_batch`` switched to the single pass (every module that calls it), so
the same golden fixtures, oracle comparisons, copy modes and malformed-shard errors hold for
both paths; the tests below add what only the single pass has (capacity overflow, look-back over
tens of thousands of tiles, copy modes following the previous call's totals).
"""

import numpy as np
import pytest
import torch

import streaming_amd.decoder as D
import streaming_amd.local
import tests.test_device_copy_modes as copy_modes
import tests.test_device_decode as device_decode
from streaming_amd.decoder import BatchDecoder, Plan, RaggedColumn, decode_batch, stage_shards
from streaming_amd.synth import var_c_shards
from tests.test_device_copy_modes import mode  # noqa: F401  (fixture)
from tests.test_device_copy_modes import (test_alignment_sweep as test_modes_alignment_sweep,
                                          test_config_c_full_shards,
                                          test_golden_sets as test_modes_golden_sets,
                                          test_invalid_utf8_rows_between_valid_ones,
                                          test_oracle_on_random_rows)
from tests.test_device_decode import (test_alignment_sweep, test_error_empty_sample_is_index_error,
                                      test_error_head_larger_than_sample,
                                      test_error_offsets_past_file,
                                      test_error_sample_count_mismatch, test_error_table_past_file,
                                      test_golden_batch_decode_matches_reference,
                                      test_ragged_many_tiny_rows,
                                      test_ragged_row_spanning_many_tiles,
                                      test_random_schemas_match_oracle)

pytestmark = pytest.mark.gpu

_two_pass = D.decode_batch


def _single(plan, batch, check=True, single=True):
    return _two_pass(plan, batch, check=check, single=single)


@pytest.fixture(autouse=True)
def _single_pass(monkeypatch):
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')
    for mod in (D, streaming_amd.local, device_decode, copy_modes):
        monkeypatch.setattr(mod, 'decode_batch', _single)


def _columns_equal(a, b):
    for name, x in a.columns.items():
        y = b.columns[name]
        if isinstance(x, RaggedColumn):
            assert torch.equal(x.offsets, y.offsets), name
            assert torch.equal(x.values, y.values), name
            if x.flags is not None:
                assert torch.equal(x.flags, y.flags), name
        else:
            assert torch.equal(x.reshape(x.shape[0], -1).view(torch.uint8),
                               y.reshape(y.shape[0], -1).view(torch.uint8)), name


C_PLAN = (['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None])


@pytest.mark.parametrize('tune', ['', 'run=0,rows=0'])
def test_single_equals_two_pass_on_many_tiles(monkeypatch, tune):
    """160k rows of config C, both passes bit-identical: the default decodes, and the register
    decode's look-back over 5000 tiles per column."""
    monkeypatch.setenv('MDSX_TUNE', tune)
    shards, counts, src = var_c_shards(160_000, seed=41, blob_bytes=(0, 600))
    plan = Plan(*C_PLAN)
    batch = stage_shards(shards, counts, plan)
    one = _two_pass(plan, batch, single=True)
    two = _two_pass(plan, batch, single=False)
    _columns_equal(one, two)
    assert np.array_equal(one['b'].values.cpu().numpy(), src['b_pool'])
    assert np.array_equal(one['s'].values.cpu().numpy(), src['s_pool'])


def test_repeated_runs_follow_previous_totals():
    """The second and later calls pick copy modes from the last finished call's totals (the
    first from an even split of the bound): every call's outputs are identical."""
    shards, counts, _ = var_c_shards(20_000, seed=42)
    plan = Plan(*C_PLAN)
    batch = stage_shards(shards, counts, plan)
    dec = BatchDecoder(plan, batch, single=True)
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
    assert dec._mode[0] == int(first['b'].offsets[-1])  # modes now follow the real totals


def test_capacity_overflow_reports_capacity():
    shards, counts, src = var_c_shards(3000, seed=43)
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


def test_empty_batch_rows():
    """Shards of zero samples: offsets are the single 0 and the totals 0."""
    from streaming_amd.writer import shard_config_bytes
    import json
    plan = Plan(*C_PLAN)
    # a valid zero-sample shard: u32 0, offsets[1], config
    cfg = shard_config_bytes(['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None], None, [],
                             1 << 26)
    head = np.array([0, 8 + len(cfg)], np.uint32).tobytes()
    raw = head + cfg
    assert json.loads(cfg)['column_names'] == ['b', 'n', 's']
    batch = stage_shards([raw], [0], plan)
    out = _two_pass(plan, batch, single=True)
    assert out.rows == 0
    assert out['s'].offsets.cpu().tolist() == [0]
    assert out['b'].values.numel() == 0
