"""Measurement: does the decode kernel read the lines the scan pass just touched from the
Infinity Cache (MALL) when the batch is small enough? Per batch size, the decode kernel is timed
(HIP events) right after its scan pass, and after its scan pass plus a 2 GiB flush copy; also the
scan pass itself. If the decode right after the scan is clearly faster at small batches, a
windowed scan -> decode schedule would save HBM reads.

    python scripts/mall_reuse.py --shards 1,2,4,16 [--blob 32,256 --chars 8,64]
"""

import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from streaming_amd.decoder import BatchDecoder, Plan  # noqa: E402
from streaming_amd.synth import var_c_batch_on_device  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--shards', default='1,2,4,16')
    ap.add_argument('--blob', default='32,256')
    ap.add_argument('--chars', default='8,64')
    ap.add_argument('--iters', type=int, default=8)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    blob = tuple(int(x) for x in args.blob.split(','))
    chars = tuple(int(x) for x in args.chars.split(','))
    names = (['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None])
    flush_a = torch.empty(2 << 30, dtype=torch.uint8, device='cuda')
    flush_b = torch.empty_like(flush_a)
    res = {}
    for n in [int(x) for x in args.shards.split(',')]:
        synth = var_c_batch_on_device(list(range(n)), seed=4, str_chars=chars, blob_bytes=blob)
        plan = Plan(*names)
        dec = BatchDecoder(plan, synth.batch)
        dec.run()
        dec.check()
        s = torch.cuda.current_stream().cuda_stream
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        t = {'scan': [], 'decode_after_scan': [], 'decode_after_flush': [],
             'decode_after_decode': []}
        for _ in range(args.iters):
            flush_b.copy_(flush_a)
            ev[0].record()
            dec._scan(s)
            ev[1].record()
            dec._decode(s)
            ev[2].record()
            torch.cuda.synchronize()
            t['scan'].append(ev[0].elapsed_time(ev[1]))
            t['decode_after_scan'].append(ev[1].elapsed_time(ev[2]))
            dec._scan(s)
            flush_b.copy_(flush_a)
            ev[1].record()
            dec._decode(s)
            ev[2].record()
            torch.cuda.synchronize()
            t['decode_after_flush'].append(ev[1].elapsed_time(ev[2]))
            ev[1].record()
            dec._decode(s)
            ev[2].record()
            torch.cuda.synchronize()
            t['decode_after_decode'].append(ev[1].elapsed_time(ev[2]))
        dec.check()
        res[n] = {'bytes': int(synth.batch.shard_bytes), 'rows': int(synth.batch.total_rows),
                  **{k: round(float(np.median(v)) * 1e3, 1) for k, v in t.items()}}
        print(json.dumps({n: res[n]}), file=sys.stderr, flush=True)
        del dec, synth
        torch.cuda.empty_cache()
    print(json.dumps({'unit': 'us (median)', 'blob': args.blob, 'chars': args.chars,
                      'results': res}, indent=1))


if __name__ == '__main__':
    main()
