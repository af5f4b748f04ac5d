"""Device shard encoder throughput on config B / C columns resident in HBM.

    python scripts/bench_encode.py --config B --samples 1000000 --steps 20

One step = mdsx_encode_shards over the whole batch (headers + rows; the sizes pass and the host
split are set-up, timed separately). Verified byte-identical to the synthetic writer's shards
(config B) / the staged shards (config C) before timing. Prints one JSON line.
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from streaming_amd.decoder import Plan, RaggedColumn, decode_batch, stage_shards  # noqa: E402
from streaming_amd.encoder import BatchEncoder  # noqa: E402
from streaming_amd.synth import fixed_b_batch_on_device, var_c_shards  # noqa: E402
from streaming_amd.writer import shard_config_bytes  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', choices=['B', 'C'], default='B')
    ap.add_argument('--samples', type=int, default=1_000_000)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--tune', default=None, help='MDSX_TUNE knobs for the encode plan')
    args = ap.parse_args()
    if args.tune:
        os.environ['MDSX_TUNE'] = args.tune
    dev = torch.device('cuda', 0)
    if args.config == 'B':
        synth = fixed_b_batch_on_device(args.samples, seed=11)
        names, encs, sizes = ['id', 'x'], ['int32', 'ndarray:float32:1024'], [4, 4096]
        plan = Plan(names, encs, sizes)
        columns = {'id': synth.sources['id'], 'x': synth.sources['x']}
        ref = synth.batch
    else:
        names, encs, sizes = ['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None]
        plan = Plan(names, encs, sizes)
        shards, counts, _ = var_c_shards(args.samples, seed=12)
        ref = stage_shards(shards, counts, plan)
        columns = decode_batch(plan, ref).columns
    cfg = shard_config_bytes(names, encs, sizes, None, [], 1 << 26)
    t0 = time.perf_counter()
    enc = BatchEncoder(plan, columns, cfg, 1 << 26)
    setup_s = time.perf_counter() - t0
    out = enc.run()
    torch.cuda.synchronize(dev)
    for s in range(len(out)):
        o, r = out.batch.offsets[s], ref.offsets[s]
        if not torch.equal(out.shard(s), ref.buffer[r:r + ref.sizes[s]]):
            raise SystemExit(f'PARITY FAILURE: encoded shard {s} differs')
    for _ in range(args.warmup):
        enc.run(check=False)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    torch.cuda.synchronize(dev)
    for a, b in ev:
        a.record()
        enc.run(check=False)
        b.record()
    torch.cuda.synchronize(dev)
    if enc.status().code != 0:
        raise SystemExit('encode reported an error')
    ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
    col_bytes = sum((v.values.numel() + v.offsets.numel() * 8) if isinstance(v, RaggedColumn)
                    else v.numel() * v.element_size() for v in columns.values())
    shard_bytes = sum(out.batch.sizes)
    gbs = (col_bytes + shard_bytes) / ms / 1e6
    print(json.dumps({
        'metric': 'device MDS encode (columns -> shard files), HBM-resident',
        'config': args.config,
        'tune': args.tune,
        'tile_rows': plan.tile_rows,
        'samples': args.samples,
        'shards': len(out),
        'ms': ms,
        'samples_per_s': args.samples / ms * 1e3,
        'shard_gib_per_s': shard_bytes / ms * 1e3 / 2**30,
        'roofline': {'bound': 'hbm', 'achieved': gbs, 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                     'frac': gbs / HBM_PEAK_GBS,
                     'algorithmic_bytes_per_launch': col_bytes + shard_bytes},
        'setup_s': setup_s,
        'parity': 'byte-identical to the writer restatement',
    }))


if __name__ == '__main__':
    main()
