"""Gathers across streams: shards decoded on one stream, gathered on another,
then dropped from the cache while the gather may still run, and their memory handed out again on
the decode's stream. The gather must still read the decoded bytes (it waits for the decode's
stream and marks the sources in use by its own: decoder._on_current_stream)."""

import numpy as np
import pytest
import torch

from oracle import mds_oracle
from streaming_amd.decoder import gather_sources
from streaming_amd.local import LocalDataset
from tests import golden_util as gu

pytestmark = pytest.mark.gpu



@pytest.fixture(scope='module', autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')


@pytest.mark.parametrize('name', ['config_a', 'config_c_small'])
def test_gather_on_another_stream_survives_eviction(name):
    import os
    d = os.path.join(gu.GOLDEN, name)
    idx = gu.index(name)['shards']
    ds = LocalDataset(d, decoded_cache_bytes=1 << 30)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        decoded = [r.decode_shard() for r in ds.shards]
    counts = [s['samples'] for s in idx]
    rng = np.random.default_rng(11)
    starts = np.concatenate([[0], np.cumsum(counts)])
    ids = rng.integers(0, starts[-1], 3000)
    src = np.searchsorted(starts, ids, side='right') - 1
    out = gather_sources(decoded, src, ids - starts[src])
    del decoded
    ds.cache.clear()
    with torch.cuda.stream(side):  # the freed blocks go back to the side stream's pool
        junk = [torch.full((1 << 20, ), 0xA5, dtype=torch.uint8, device='cuda') for _ in range(32)]
    torch.cuda.synchronize()
    del junk
    want = {}
    for info in idx:
        for c, v in mds_oracle.decode_shard_columns(d, None, info).items():
            want.setdefault(c, []).append(v)
    for c, parts in want.items():
        got = out[c]
        if parts[0][0] == 'fixed':
            rows = np.concatenate([p[1] for p in parts])[ids]
            have = got.reshape(got.shape[0], -1).view(torch.uint8).cpu().numpy()
            assert np.array_equal(have, rows.reshape(len(ids), -1)), c
        else:
            vals = np.concatenate([p[1] for p in parts])
            offs = np.concatenate([[0], np.cumsum(np.concatenate([np.diff(p[2]) for p in parts]))])
            gv, go = got.values.cpu().numpy(), got.offsets.cpu().numpy()
            for k, i in enumerate(ids):
                assert np.array_equal(gv[go[k]:go[k + 1]], vals[offs[i]:offs[i + 1]]), (c, k)


def test_gather_output_carries_its_stream():
    """A gather's output made on one stream, gathered again on another: the
    output records the stream it was written on, so the second gather waits for it and marks it
    in use, and reads the first gather's rows even after they are freed and reused."""
    import os
    name = 'config_c_small'
    d = os.path.join(gu.GOLDEN, name)
    idx = gu.index(name)['shards']
    ds = LocalDataset(d, decoded_cache_bytes=1 << 30)
    decoded = [r.decode_shard() for r in ds.shards]
    counts = [s['samples'] for s in idx]
    starts = np.concatenate([[0], np.cumsum(counts)])
    rng = np.random.default_rng(12)
    ids = rng.integers(0, starts[-1], 2000)
    src = np.searchsorted(starts, ids, side='right') - 1
    side, other = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        first = gather_sources(decoded, src, ids - starts[src])
        assert first.stream == side
        again = first.gather(np.arange(first.rows))  # a DecodedBatch.gather output, same stream
        assert again.stream == side
    with torch.cuda.stream(other):
        sel = rng.integers(0, first.rows, 500)
        second = gather_sources([first], np.zeros(sel.size, np.int64), sel)
    del first
    with torch.cuda.stream(side):
        junk = [torch.full((1 << 20, ), 0x5A, dtype=torch.uint8, device='cuda') for _ in range(16)]
    torch.cuda.synchronize()
    del junk
    want = {}
    for info in idx:
        for c, v in mds_oracle.decode_shard_columns(d, None, info).items():
            want.setdefault(c, []).append(v)
    for c, parts in want.items():
        got = second[c]
        chosen = ids[sel]
        if parts[0][0] == 'fixed':
            rows = np.concatenate([p[1] for p in parts])[chosen]
            have = got.reshape(got.shape[0], -1).view(torch.uint8).cpu().numpy()
            assert np.array_equal(have, rows.reshape(len(chosen), -1)), c
        else:
            vals = np.concatenate([p[1] for p in parts])
            offs = np.concatenate([[0], np.cumsum(np.concatenate([np.diff(p[2]) for p in parts]))])
            gv, go = got.values.cpu().numpy(), got.offsets.cpu().numpy()
            for k, i in enumerate(chosen):
                assert np.array_equal(gv[go[k]:go[k + 1]], vals[offs[i]:offs[i + 1]]), (c, k)
