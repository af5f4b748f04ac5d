"""Output placement sweep (measurement): decode one resident batch into outputs placed at
different offsets of one large allocation, interleaved over rounds, and report each offset's
median scan + decode time. Identical kernels, only the output addresses move
(profiles/r03/noise_floor: ~5 % between identical decoders with their own buffers).

    python scripts/placement_sweep.py --config B --step-kib 4 --count 16 --rounds 4
"""

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from streaming_amd.decoder import BatchDecoder, Plan, output_bytes  # noqa: E402
from streaming_amd.synth import fixed_b_batch_on_device, var_c_batch_on_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='B')
    ap.add_argument('--shards', type=int, default=64)
    ap.add_argument('--step-kib', type=int, default=4)
    ap.add_argument('--count', type=int, default=16)
    ap.add_argument('--rounds', type=int, default=4)
    ap.add_argument('--iters', type=int, default=10)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    if args.config == 'B':
        synth = fixed_b_batch_on_device(1_000_000, seed=3)
        plan = Plan(['id', 'x'], ['int32', 'ndarray:float32:1024'], [4, 4096])
    else:
        synth = var_c_batch_on_device(list(range(args.shards)), seed=4)
        plan = Plan(['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None])
    batch = synth.batch
    dec = BatchDecoder(plan, batch)
    dec.run()
    dec.check()
    rows = batch.total_rows
    step = args.step_kib * 1024
    # one allocation holding every fixed column at each offset (fixed columns only: B)
    fixed = [c for c in plan.columns if c.is_fixed]
    need = sum(rows * c.row_bytes for c in fixed) + 256 * len(fixed)
    pool = torch.empty(need + step * args.count + 4096, dtype=torch.uint8, device=batch.device)
    base = (-pool.data_ptr()) % 4096  # offset 0 = a 4 KiB-aligned address
    layouts = []
    for k in range(args.count):
        off = base + k * step
        raws = {}
        for c in fixed:
            raws[c.name] = pool[off:off + rows * c.row_bytes].view(rows, c.row_bytes)
            off += (rows * c.row_bytes + 255) // 256 * 256
        layouts.append(raws)
    in_addr = batch.buffer.data_ptr()
    times = {k: [] for k in range(args.count)}
    for rnd in range(args.rounds):
        order = list(range(args.count))
        order = order[rnd % len(order):] + order[:rnd % len(order)]
        for k in order:
            dec._fixed_raw = dict(dec._fixed_raw, **layouts[k])
            evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)]
                   for _ in range(args.iters)]
            for e in evs:
                dec.run(e)
            torch.cuda.synchronize()
            times[k].extend(e[0].elapsed_time(e[2]) for e in evs)
    dec._fixed_raw = dict(dec._fixed_raw, **layouts[-1])
    out = dec.run()
    dec.check()
    if args.config == 'B':  # the last layout holds this last run's decode
        got = layouts[-1]['x'].view(torch.int32)
        assert torch.equal(got, synth.sources['x'].view(torch.int32).reshape(got.shape))
    R, W = batch.shard_bytes, output_bytes(plan, out)
    res = []
    for k in range(args.count):
        ms = float(np.median(times[k]))
        first = layouts[k][fixed[-1].name].data_ptr()
        res.append({'offset_kib': k * args.step_kib, 'out_minus_in_mod_1MiB_kib':
                    ((first - in_addr) % (1 << 20)) // 1024, 'median_ms': ms,
                    'GBps': (R + W) / ms / 1e6})
    print(json.dumps({'config': args.config, 'rows': rows, 'R': R, 'W': W,
                      'input_addr_mod_1MiB_kib': (in_addr % (1 << 20)) // 1024,
                      'results': res}, indent=1))


if __name__ == '__main__':
    main()
