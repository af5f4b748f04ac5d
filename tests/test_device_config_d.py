"""Config D on the GPU (BASELINE.json configs[3]): one rank's full share of the
100M-sample, 8-GPU dataset -- 6 116 full 64 MiB config-B shards, global shard g owned by rank
g % 8 (``owned_shards``; the build's replacement for the reference's per-rank sample split,
``streaming/base/partition/orig.py:140-181``), generated from per-shard seeds exactly as
``bench.py --gpus 8`` does -- resident at once and decoded in ONE batch, bit-exact against the
encoded columns, and eight spread shards sample by sample against the oracle. Peak device memory: the shards (51 GB) + the decoded columns (51 GB) + one
shard's regenerated source at a time."""

import numpy as np
import pytest
import torch

from oracle import mds_oracle

from streaming_amd.decoder import decode_batch
from streaming_amd.distributed import owned_shards
from streaming_amd.synth import config_b_samples_per_shard, fixed_b_batch_on_device

pytestmark = pytest.mark.gpu

SHARDS_D, WORLD_D = 6116, 8
SEED_B = 1000  # bench.py's config-B seed


@pytest.fixture(scope='module', autouse=True)
def _needs_gpu():
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')


def test_config_d_rank0_share_bit_exact():
    per = config_b_samples_per_shard()
    assert per == 16352 and SHARDS_D == -(-100_000_000 // per)  # 100M samples, full shards
    mine = owned_shards(SHARDS_D, 0, WORLD_D)
    assert len(mine) == 765 and mine[:3] == [0, 8, 16] and mine[-1] == 6112
    # every shard owned exactly once over the 8 ranks
    assert sorted(g for r in range(WORLD_D) for g in owned_shards(SHARDS_D, r, WORLD_D)) == \
        list(range(SHARDS_D))
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    torch.zeros(1, device=dev)  # the context (the first GPU call of a fresh process)
    torch.cuda.empty_cache()
    torch.cuda.reset_peak_memory_stats(dev)
    synth = fixed_b_batch_on_device(0, seed=SEED_B, shard_ids=mine, keep_sources=False)
    batch = synth.batch
    assert batch.nshards == 765 and batch.total_rows == 765 * per
    out = decode_batch(synth.plan, batch)
    torch.cuda.synchronize(dev)
    ids, x = out['id'], out['x'].view(torch.uint8).view(-1, 4096)
    assert torch.equal(ids, synth.sources['id'])
    gen = torch.Generator(device=dev)
    for s, g in enumerate(mine):  # the x rows of shard g: its generator, seeded SEED_B + g
        gen.manual_seed(SEED_B + g)
        want = torch.randint(0, 256, (per, 4096), dtype=torch.uint8, device=dev, generator=gen)
        assert torch.equal(x[s * per:(s + 1) * per], want), g
        assert int(ids[s * per]) == g * per  # global sample ids of the 100M-sample layout
    # eight shards spread over the share: every sample against the oracle reading the shard's
    # bytes (the reference's per-sample get_sample_data + decode_sample, mds/reader.py:103-149)
    names, encs, sizes = synth.plan.key
    for s in sorted({round(k * (len(mine) - 1) / 7) for k in range(8)}):
        info = {'column_names': list(names), 'column_encodings': list(encs),
                'column_sizes': [sz or None for sz in sizes], 'samples': batch.samples[s],
                'raw_data': {'basename': f'shard.{mine[s]:05d}.mds'}}
        data = batch.buffer[batch.offsets[s]:batch.offsets[s] + batch.sizes[s]].cpu().numpy()
        want = mds_oracle.decode_shard_columns(None, None, info, data=data.tobytes())
        r0, n = batch.row0[s], batch.samples[s]
        assert np.array_equal(ids[r0:r0 + n].cpu().numpy().view(np.uint8).reshape(n, 4),
                              want['id'][1]), mine[s]
        assert np.array_equal(x[r0:r0 + n].cpu().numpy(), want['x'][1]), mine[s]
    peak = torch.cuda.max_memory_allocated(dev)
    assert peak < 106e9, peak  # shards + outputs (~102.7 GB) + one regenerated shard
    del out, ids, x, synth, batch
    torch.cuda.empty_cache()
