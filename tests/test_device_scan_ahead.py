"""ScanAheadDecoder (streaming_amd.decoder): pass 1 of the next batch on a side stream beside
the current batch's pass 2. Every decode is compared with the one-stream two-pass decode of the
same batch (BatchDecoder, itself checked against the oracle in test_device_decode.py) and with
the encoded source columns; batches alternate so that a slot is rescanned with another batch's
bytes while the other slot decodes."""

import pytest
import torch

from streaming_amd.decoder import BatchDecoder, RaggedColumn, ScanAheadDecoder

pytestmark = pytest.mark.gpu


def _same(a, b):
    for name in a.columns:
        x, y = a.columns[name], b.columns[name]
        if isinstance(x, RaggedColumn):
            n = int(y.offsets[-1])
            assert torch.equal(x.offsets, y.offsets), name
            assert torch.equal(x.values[:n], y.values[:n]), name
            assert int(x.values.numel()) == n, name  # trimmed to the scanned total
            if x.flags is not None:
                assert torch.equal(x.flags, y.flags), name
        else:
            assert torch.equal(x, y), name


def _sources_equal(out, src):
    assert torch.equal(out['n'], src['n'])
    for name in ('b', 's'):
        assert torch.equal(out[name].values, src[name].values), name
        assert torch.equal(out[name].offsets - out[name].offsets[0], src[name].offsets), name


def _batches(blob, chars):
    from streaming_amd.synth import var_c_batch_on_device
    return [var_c_batch_on_device([g], seed=40 + 7 * g, size_limit=1 << 22, blob_bytes=blob,
                                  str_chars=chars) for g in range(3)]


@pytest.mark.parametrize('blob,chars', [((3072, 5120), (16, 256)), ((32, 256), (8, 64))],
                         ids=['streaming', 'row_parallel'])
def test_scan_ahead_alternating_batches(blob, chars):
    synths = _batches(blob, chars)
    plan = synths[0].plan
    want = []
    for s in synths:
        dec = BatchDecoder(plan, s.batch)
        out = dec.run()
        dec.check()
        want.append((dec, out))
    # upper-bound outputs (no capacities): the values are trimmed to the scanned totals
    sad = ScanAheadDecoder(plan, synths[0].batch)
    order = [0, 1, 2, 1, 0, 2, 2, 0]
    sad.scan(synths[order[0]].batch)
    for k, i in enumerate(order):
        if k + 1 < len(order):
            sad.scan(synths[order[k + 1]].batch)  # into the other slot, beside this decode
        got = sad.decode()
        sad.check()
        _same(got, want[i][1])
        _sources_equal(got, synths[i].sources)
    sad.close()


def test_scan_ahead_run_steps_and_events():
    synths = _batches((3072, 5120), (16, 256))[:1]
    s = synths[0]
    ref = BatchDecoder(s.plan, s.batch)
    ref_out = ref.run()
    ref.check()
    sad = ScanAheadDecoder(s.plan, s.batch, capacities=ref.capacities)
    n = 5
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(n)]
    for k in range(n):
        out = sad.run(ahead=k + 1 < n, events=evs[k])
    torch.cuda.synchronize()
    sad.check()
    _same(out, ref_out)
    _sources_equal(sad.result(), s.sources)
    assert all(e[0].elapsed_time(e[1]) > 0 for e in evs)
    assert all(e[2].elapsed_time(e[3]) > 0 for e in evs[:-1])
    with pytest.raises(RuntimeError, match='no scanned batch'):
        sad.decode()


def test_scan_ahead_slots_exhausted():
    s = _batches((3072, 5120), (16, 256))[0]
    sad = ScanAheadDecoder(s.plan, s.batch)
    sad.scan()
    sad.scan()
    with pytest.raises(RuntimeError, match='every slot'):
        sad.scan()
    sad.decode()
    sad.decode()
    sad.check()
    sad.close()


def test_scan_ahead_capacity_error():
    """Outputs too small for a batch: the decode reports MDSX_E_CAPACITY, never writes past."""
    s = _batches((3072, 5120), (16, 256))[0]
    caps = {'b': 1024, 's': 1024}
    sad = ScanAheadDecoder(s.plan, s.batch, capacities=caps)
    sad.scan()
    sad.decode()
    with pytest.raises(RuntimeError, match='capacity exceeded'):
        sad.check()


def test_scan_ahead_other_batch_gets_its_bound():
    """Capacities given for the constructor's batch: a slot built for another batch of the plan
    gets at least that batch's upper bound, so it decodes whole."""
    synths = _batches((3072, 5120), (16, 256))
    small = {'b': 1024, 's': 1024}
    sad = ScanAheadDecoder(synths[0].plan, synths[0].batch, capacities=small)
    sad.scan(synths[1].batch)
    got = sad.decode()
    sad.check()
    _sources_equal(got, synths[1].sources)
    sad.close()


def test_scan_ahead_dropped_with_a_scan_in_flight():
    """A decoder dropped while its side stream still scans: the slot tensors carry the side
    stream (record_stream) and the decoder waits for it, so their memory is not reused early."""
    synths = _batches((3072, 5120), (16, 256))
    sad = ScanAheadDecoder(synths[0].plan, synths[0].batch)
    sad.scan()
    del sad  # no close()
    fill = [torch.full((1 << 24,), 7, dtype=torch.uint8, device='cuda') for _ in range(8)]
    torch.cuda.synchronize()
    assert all(int(f[-1]) == 7 for f in fill)
    dec = BatchDecoder(synths[0].plan, synths[0].batch)
    out = dec.run()
    dec.check()
    _sources_equal(out, synths[0].sources)
