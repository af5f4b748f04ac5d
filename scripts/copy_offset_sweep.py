"""Measurement: does the HBM copy rate depend on where the destination lies relative to the
source? One allocation holds a 4 GiB source and, at a sweep of offsets past it, the destination;
the copy probe (mdsx_copy_probe_variant, the bench's shapes) is timed per offset, the offsets
visited in rotated order over several rounds.

    python scripts/copy_offset_sweep.py [--gib 4] [--rounds 3]
"""

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from streaming_amd import _native  # noqa: E402

MIB = 1 << 20


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gib', type=int, default=4)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--iters', type=int, default=5)
    ap.add_argument('--variants', default='5,1')
    args = ap.parse_args()
    torch.cuda.set_device(0)
    lib = _native.lib()
    n = args.gib << 30
    offs_mib = [0, 1, 2, 3, 4, 6, 8, 16, 32, 64, 96, 128, 192, 256]
    big = torch.empty(2 * n + (max(offs_mib) + 2) * MIB, dtype=torch.uint8, device='cuda')
    big[:n].random_(0, 255)
    src = big[:n]
    stream = torch.cuda.current_stream().cuda_stream
    variants = [int(v) for v in args.variants.split(',')]
    times = {(o, v): [] for o in offs_mib for v in variants}
    for rnd in range(args.rounds):
        order = offs_mib[rnd % len(offs_mib):] + offs_mib[:rnd % len(offs_mib)]
        for o in order:
            dst = big[n + o * MIB:2 * n + o * MIB]
            for v in variants:
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                lib.mdsx_copy_probe_variant(src.data_ptr(), dst.data_ptr(), n, v, stream)
                s.record()
                for _ in range(args.iters):
                    lib.mdsx_copy_probe_variant(src.data_ptr(), dst.data_ptr(), n, v, stream)
                e.record()
                torch.cuda.synchronize()
                times[(o, v)].append(s.elapsed_time(e) / args.iters)
        print(json.dumps({'round': rnd}), file=sys.stderr, flush=True)
    res = {f'{o}MiB/v{v}': round(2 * n / float(np.median(t)) / 1e6, 1) for (o, v), t in times.items()}
    print(json.dumps({'gib': args.gib, 'src_ptr_mod_2MiB': src.data_ptr() % (2 * MIB),
                      'GBps': res}, indent=1))


if __name__ == '__main__':
    main()
