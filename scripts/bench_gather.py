"""Device batch-gather throughput: rows of decoded, HBM-resident columns
selected by sample id (the reference's per-sample iteration over a worker's sample ids,
dataset.py:1430-1473), through the mdsx_gather_* C ABI.

    python scripts/bench_gather.py --config B --samples 1000000 --batch 0 --steps 10

One step gathers a random permutation of the decoded rows, in launches of ``--batch`` ids
(0 = all ids in one launch): fixed columns with mdsx_gather_fixed, ragged columns with
mdsx_gather_ragged_scan + mdsx_gather_ragged_copy (outputs pre-sized, no host sync inside the
step). Verified against torch indexing before timing. Prints one JSON line.
"""

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from streaming_amd import _native  # noqa: E402
from streaming_amd.decoder import (Plan, RaggedColumn, decode_batch, stage_shards)  # noqa: E402
from streaming_amd.synth import fixed_b_batch_on_device, var_c_shards  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', choices=['B', 'C'], default='B')
    ap.add_argument('--samples', type=int, default=1_000_000)
    ap.add_argument('--batch', type=int, default=0, help='ids per launch (0 = all)')
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device('cuda', 0)
    lib = _native.lib()
    if args.config == 'B':
        syn = fixed_b_batch_on_device(args.samples, seed=31, keep_sources=False)
        dec = decode_batch(syn.plan, syn.batch)
    else:
        plan = Plan(['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None])
        shards, counts, _ = var_c_shards(args.samples, seed=32)
        dec = decode_batch(plan, stage_shards(shards, counts, plan))
    rows = dec.rows
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    perm = torch.randperm(rows, device=dev, generator=gen)
    batch = args.batch or rows
    launches = [(lo, min(rows, lo + batch)) for lo in range(0, rows, batch)]
    ws = torch.zeros(int(lib.mdsx_gather_workspace_bytes(batch)), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    # outputs, sized once per launch
    plans = []
    moved = 0
    for name, col in dec.columns.items():
        if isinstance(col, RaggedColumn):
            lens = (col.offsets[1:] - col.offsets[:-1])[perm]
            per = []
            for lo, hi in launches:
                cap = int(lens[lo:hi].sum())
                per.append((torch.empty(hi - lo + 1, dtype=torch.int64, device=dev),
                            torch.empty(max(cap, 1), dtype=torch.uint8, device=dev), cap,
                            torch.zeros(hi - lo, dtype=torch.uint8, device=dev)
                            if col.flags is not None else None))
                moved += 2 * cap + 16 * (hi - lo)
            plans.append((name, col, True, per))
        else:
            rb = col[0].numel() * col.element_size()
            out = torch.empty((rows, ) + tuple(col.shape[1:]), dtype=col.dtype, device=dev)
            plans.append((name, col, False, (out, rb)))
            moved += 2 * rows * rb + 8 * rows

    def step():
        for name, col, ragged, p in plans:
            for k, (lo, hi) in enumerate(launches):
                idx = perm[lo:hi]
                m = hi - lo
                if ragged:
                    offs, vals, cap, flags = p[k]
                    lib.mdsx_gather_ragged_scan(col.offsets.data_ptr(), rows, idx.data_ptr(), m,
                                                offs.data_ptr(), ws.data_ptr(), ws.numel(), None,
                                                stream)
                    lib.mdsx_gather_ragged_copy(col.values.data_ptr(), col.offsets.data_ptr(),
                                                col.flags.data_ptr() if flags is not None else None,
                                                rows, idx.data_ptr(), m, vals.data_ptr(), cap,
                                                offs.data_ptr(),
                                                flags.data_ptr() if flags is not None else None,
                                                ws.data_ptr(), ws.numel(), stream)
                else:
                    out, rb = p
                    lib.mdsx_gather_fixed(col.data_ptr(), rows, rb, idx.data_ptr(), m,
                                          out[lo:hi].data_ptr(), ws.data_ptr(), ws.numel(),
                                          stream)

    step()
    torch.cuda.synchronize()
    if _native.Status.from_buffer_copy(ws[:16].cpu().numpy().tobytes()).code != 0:
        raise SystemExit('gather reported an error')
    # parity: torch indexing of the decoded columns
    for name, col, ragged, p in plans:
        if ragged:
            lo, hi = launches[-1]
            offs, vals, cap, flags = p[-1]
            ids = perm[lo:hi].cpu().numpy()
            so = col.offsets.cpu().numpy()
            sv = col.values.cpu().numpy()
            want = np.concatenate([sv[so[i]:so[i + 1]] for i in ids[:2000]])
            if not np.array_equal(vals[:len(want)].cpu().numpy(), want):
                raise SystemExit(f'PARITY FAILURE: {name}')
        else:
            out, _ = p
            # compare bit patterns (random float32 rows hold NaNs)
            if not torch.equal(out.reshape(rows, -1).view(torch.uint8),
                               col[perm].reshape(rows, -1).view(torch.uint8)):
                raise SystemExit(f'PARITY FAILURE: {name}')
    for _ in range(args.warmup):
        step()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(args.steps)]
    torch.cuda.synchronize()
    for e0, e1 in ev:
        e0.record()
        step()
        e1.record()
    torch.cuda.synchronize()
    ms = float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))
    gbs = moved / ms / 1e6
    print(json.dumps({
        'metric': 'device batch gather by sample id, HBM-resident',
        'config': args.config,
        'rows': rows,
        'ids_per_launch': batch,
        'launches_per_step': len(launches) * len(plans),
        'ms': ms,
        'samples_per_s': rows / ms * 1e3,
        'bytes_moved': moved,
        'GBps': gbs,
        'hbm_frac': gbs / HBM_PEAK_GBS,
        'parity': 'torch indexing of the decoded columns',
    }))


if __name__ == '__main__':
    main()
