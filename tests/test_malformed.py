"""Malformed shards: the per-sample reader returns what the REAL reference returns, sample by
sample (values, or the exception type), on shards that break the MDS layout -- a size head past
its sample, a sample cut inside a str or a fixed column, junk between samples, a last offset past
the file, a cut file, an empty sample, end < begin (tests/golden/make_malformed.py recorded the
reference's outcomes; streaming/base/format/mds/reader.py:103-149).

The whole-shard decode (decode_shard, decode_all, device batches) is stricter, deliberately: a
shard with such a sample raises (ValueError; IndexError for an empty sample) instead of handing
out clipped values -- INTEGRATION.md §1. Both behaviours are asserted here.

CPU: the oracle's restatement against the fixtures. GPU: MDSReader.get_item and decode_shard."""
import json
import os
import warnings

import pytest

from oracle import mds_oracle
from tests import golden_util as gu

HERE = os.path.join(gu.GOLDEN, 'malformed')
OUTCOMES = json.load(open(os.path.join(HERE, 'outcomes.json')))
CASES = sorted(OUTCOMES)
# cases whose every sample the whole-shard decode reads as the reference does
CLEAN = {'junk_after'}
# cases whose shard header (the offsets table's last entry) does not match the file: the decode
# reports the shard, not a sample, so every device batch reading it raises
HEADER = {'file_cut', 'last_past_file'}


def _info(case):
    return json.load(open(os.path.join(HERE, case, 'index.json')))['shards'][0]


def _outcome(get, i):
    try:
        with warnings.catch_warnings():
            warnings.simplefilter('ignore')  # numpy's uint32 wrap of end - begin
            sample = get(i)
    except Exception as e:  # noqa: BLE001 -- the outcome is the exception
        return {'exc': type(e).__name__}
    return {'value': {k: gu.value_record(v) for k, v in sample.items()}}


def _want(case):
    return [{'exc': o['exc']} if 'exc' in o else o for o in OUTCOMES[case]]


def test_fixtures_cover_the_verdict_cases():
    assert {'head_over', 'junk_after', 'last_past_file', 'file_cut', 'fixed_short'} <= set(CASES)
    kinds = {o.get('exc', 'value') for c in CASES for o in OUTCOMES[c]}
    assert kinds == {'value', 'IndexError', 'ValueError', 'UnicodeDecodeError'}


@pytest.mark.parametrize('case', CASES)
def test_oracle_matches_reference_outcomes(case):
    r = mds_oracle.OracleMDSReader(HERE + '/' + case, None, _info(case))
    assert [_outcome(r.get_item, i) for i in range(len(r))] == _want(case)


@pytest.mark.parametrize('case', CASES)
def test_oracle_in_memory_matches_reference_outcomes(case):
    """The oracle reading the shard from memory (the full-size parity tests' form) reads as the
    reference reads the file: short reads at the end, end < begin wrapping to the end."""
    info = _info(case)
    data = open(os.path.join(HERE, case, info['raw_data']['basename']), 'rb').read()
    r = mds_oracle.OracleMDSReader(None, None, info, data=data)
    assert [_outcome(r.get_item, i) for i in range(len(r))] == _want(case)


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES)
def test_device_reader_matches_reference_outcomes(case):
    from streaming_amd.reader import MDSReader
    info = _info(case)
    r = MDSReader.from_json(os.path.join(HERE, case), None, info)
    try:
        assert [_outcome(r.get_item, i) for i in range(info['samples'])] == _want(case)
        # the whole-shard decode: strict where the reference clips
        if case in CLEAN:
            r.decode_shard()
        else:
            with pytest.raises(IndexError if case == 'empty' else ValueError):
                r.decode_shard()
    finally:
        r.release()


@pytest.mark.gpu
def test_decode_sample_equals_reference_slices():
    """decode_sample(data) on well-formed and cut sample bytes: the reference's slices."""
    from streaming_amd.reader import MDSReader
    info = _info('junk_after')
    r = MDSReader.from_json(os.path.join(HERE, 'junk_after'), None, info)
    o = mds_oracle.OracleMDSReader(os.path.join(HERE, 'junk_after'), None, info)
    for i in range(info['samples']):
        data = o.get_sample_data(i)
        for cut in range(len(data) + 1):
            assert _outcome(lambda _: r.decode_sample(data[:cut]), 0) == \
                _outcome(lambda _: o.decode_sample(data[:cut]), 0), (i, cut)


@pytest.mark.gpu
@pytest.mark.parametrize('case', CASES)
def test_device_batches_raise_only_for_refused_samples(case):
    """The batch path (iter_batches: a device gather of the decoded shard) on a malformed shard:
    a sample the reference raises for raises the same exception type; a sample the reference
    clips raises ValueError (the batch path hands out no clipped values) unless the decode took it
    whole (junk after it); every other sample is served -- except on a shard whose header does not
    match the file, where every batch raises."""
    from streaming_amd import LocalDataset
    ds = LocalDataset(os.path.join(HERE, case), decoded_cache_bytes=1 << 20)
    served = 0
    for i, want in enumerate(OUTCOMES[case]):
        got = _outcome(lambda j: next(iter(ds.iter_batches([j], 1))) and {}, i)
        if 'exc' in want:
            assert got == {'exc': want['exc']}, (case, i)
        elif 'exc' in got:
            assert case not in CLEAN and got == {'exc': 'ValueError'}, (case, i, got)
        else:
            served += 1
    if case in HEADER:
        assert served == 0, case
    else:
        assert served >= (len(OUTCOMES[case]) if case in CLEAN else 1), case
