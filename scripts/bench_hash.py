"""Device shard-file hashing throughput over config-B shards resident in HBM.

    python scripts/bench_hash.py --samples 1000000 --steps 10 [--algos xxh3_64,xxh128,xxh64]

One step = mdsx_hash_segments over every shard file of the batch (62 x 64 MiB at 1M samples).
Digests are checked against python-xxhash (the reference's get_hash, hashing.py:55-68) on the
host copy before timing. Prints one JSON line per algorithm, with the host xxhash rate on one
64 MiB shard (1 core) beside it.
"""

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from streaming_amd import hashing  # noqa: E402
from streaming_amd.synth import fixed_b_batch_on_device  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--samples', type=int, default=1_000_000)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--algos', default='xxh3_64,xxh128,xxh64,xxh32')
    ap.add_argument('--check', type=int, default=1, help='verify against python-xxhash')
    args = ap.parse_args()
    import xxhash
    dev = torch.device('cuda', 0)
    syn = fixed_b_batch_on_device(args.samples, seed=21, keep_sources=False)
    b = syn.batch
    segs = list(zip(b.offsets, b.sizes))
    total = sum(b.sizes)
    host = b.buffer.cpu().numpy() if args.check else None
    hasher = hashing.DeviceHasher(dev)
    for algo in args.algos.split(','):
        got = hashing.hash_batch(b, algo)
        if host is not None:
            want = [getattr(xxhash, algo)(host[o:o + n].tobytes()).hexdigest() for o, n in segs]
            if got != want:
                raise SystemExit(f'PARITY FAILURE: {algo}')
        for _ in range(args.warmup):
            hasher.launch(algo, b.buffer, segs)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(args.steps)]
        torch.cuda.synchronize(dev)
        for e0, e1 in ev:
            e0.record()
            hasher.launch(algo, b.buffer, segs)
            e1.record()
        torch.cuda.synchronize(dev)
        ms = float(np.median([e0.elapsed_time(e1) for e0, e1 in ev]))
        one = host[b.offsets[0]:b.offsets[0] + b.sizes[0]].tobytes() if host is not None else \
            bytes(b.sizes[0])
        fn = getattr(xxhash, algo)
        t0 = time.perf_counter()
        reps = 0
        while time.perf_counter() - t0 < 1.0:
            fn(one).hexdigest()
            reps += 1
        cpu_gbs = reps * len(one) / (time.perf_counter() - t0) / 1e9
        gbs = total / ms / 1e6
        print(json.dumps({
            'metric': 'device shard-file hash, HBM-resident',
            'algo': algo,
            'shards': len(segs),
            'bytes': total,
            'ms': ms,
            'GBps': gbs,
            'hbm_frac': gbs / HBM_PEAK_GBS,
            'parity': 'python-xxhash digests' if host is not None else 'unchecked',
            'cpu_baseline': {'GBps': cpu_gbs, 'cores': 1, 'kind': 'python-xxhash (reference '
                             'get_hash)', 'sample': f'one {len(one)} B shard x {reps}'},
        }), flush=True)


if __name__ == '__main__':
    main()
