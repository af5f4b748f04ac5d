"""Measurement: all-fixed schemas of several row sizes through decode_kernel (MDSX_TUNE rw=0) and
the row-per-wave decode (rw=1), in one process: where should the row-per-wave decode take over?
Shards are built in memory in the writer's layout (mds/writer.py:133-144: u32 N, N + 1 offsets,
the config bytes, the rows back to back): columns `id` int32 + `x` ndarray:uint8:(size - 4).

    python scripts/fixed_rows_ab.py [--sizes 260,516,1028,2052,4100] [--gib 1]
"""

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from streaming_amd.decoder import BatchDecoder, Plan, stage_shards  # noqa: E402
from streaming_amd.writer import shard_config_bytes  # noqa: E402


def shard(n, size, rng):
    names, encs, sizes = ['id', 'x'], ['int32', f'ndarray:uint8:{size - 4}'], [4, size - 4]
    config = shard_config_bytes(names, encs, sizes, None, [], 1 << 26)
    hdr = 4 + 4 * (n + 1)
    offs = (hdr + len(config) + size * np.arange(n + 1, dtype=np.int64)).astype(np.uint32)
    body = rng.integers(0, 256, n * size, dtype=np.uint8)
    return np.uint32(n).tobytes() + offs.tobytes() + config + body.tobytes(), (names, encs, sizes)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--sizes', default='260,516,1028,2052,4100')
    ap.add_argument('--gib', type=float, default=1.0)
    ap.add_argument('--iters', type=int, default=10)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--variants', default='rw=0;rw=1', help="MDSX_TUNE settings, ';'-separated")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    rng = np.random.default_rng(1)
    res = {}
    for size in [int(x) for x in args.sizes.split(',')]:
        per = ((64 << 20) - 4096) // (size + 4)
        nshards = max(1, int(args.gib * (1 << 30)) // (64 << 20))
        data, schema = zip(*[shard(per, size, rng) for _ in range(nshards)])
        names, encs, sizes = schema[0]
        outs, times = {}, {v: [] for v in args.variants.split(';')}
        batches = {}
        for tune in times:
            os.environ['MDSX_TUNE'] = tune
            plan = Plan(names, encs, sizes)
            batch = stage_shards(list(data), [per] * nshards, plan)
            dec = BatchDecoder(plan, batch)
            batches[tune] = dec
            outs[tune] = dec.run()
            dec.check()
        first = next(iter(outs.values()))
        for v in outs:
            for name in names:
                assert torch.equal(first[name], outs[v][name]), (size, v, name)
        nbytes = sum(len(d) for d in data) + sum(int(first[n].numel()) * first[n].element_size()
                                                 for n in names)
        for _ in range(args.rounds):
            for tune, dec in batches.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                dec.run()
                s.record()
                for _ in range(args.iters):
                    dec.run()
                e.record()
                torch.cuda.synchronize()
                times[tune].append(s.elapsed_time(e) / args.iters)
        res[size] = {t: round(nbytes / (float(np.median(v)) * 1e-3) / 1e9, 1) for t, v in times.items()}
        print(json.dumps({size: res[size]}), file=sys.stderr, flush=True)
        del outs, batches
        torch.cuda.empty_cache()
    print(json.dumps({'unit': 'GB/s of R + W (scan + decode per call)', 'results': res}, indent=1))


if __name__ == '__main__':
    main()
