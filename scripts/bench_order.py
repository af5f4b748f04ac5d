"""Reference-order device batches: samples/s of ``LocalDataset.iter_batches``
over shuffled global ids, on one GPU.

Writes ``--shards`` config-C shard files (64 MiB, the reference writer's layout) to a temp
directory, then, in one process:
  * cold epoch: ids shuffled over the whole dataset, shards decoded on demand into the decoded
    cache as batches first touch them;
  * warm epochs: the same ids again (every shard resident), per batch size;
every batch checked against the fully decoded dataset gathered with the same ids (first batch of
each run bit-exact, all batches' row counts); then the per-sample ``get_item`` rate (the path
``StreamingDataset.get_item`` takes through a device reader). Prints one JSON object.
"""

import argparse
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from streaming_amd import LocalDataset, MDSWriter  # noqa: E402
from streaming_amd.decoder import RaggedColumn  # noqa: E402
from streaming_amd.synth import var_c_shards  # noqa: E402


def batch_bytes(b):
    n = 0
    for c in b.columns.values():
        if isinstance(c, RaggedColumn):
            n += c.values.numel() + c.offsets.numel() * 8 + (c.flags.numel() if c.flags is not None
                                                              else 0)
        else:
            n += c.numel() * c.element_size()
    return n


def same(a, b):
    for name, x in a.columns.items():
        y = b.columns[name]
        if isinstance(x, RaggedColumn):
            if not (torch.equal(x.values, y.values) and torch.equal(x.offsets, y.offsets)):
                return False
        elif not torch.equal(x, y):
            return False
    return True


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--shards', type=int, default=16)
    ap.add_argument('--batch', type=int, nargs='+', default=[256, 1024, 4096])
    ap.add_argument('--batches', type=int, default=200, help='timed batches per batch size')
    args = ap.parse_args()
    torch.cuda.set_device(0)
    tmp = tempfile.mkdtemp(prefix='mdsx_order_')
    try:
        data, counts, _ = var_c_shards(args.shards * 15_050, seed=7)
        data, counts = data[:args.shards], counts[:args.shards]
        with MDSWriter(out=tmp, columns={'b': 'bytes', 'n': 'int', 's': 'str'},
                       size_limit=1 << 26) as w:
            for raw, n in zip(data, counts):
                w.write_encoded_shard(raw, n)
        ds = LocalDataset(tmp, decoded_cache_bytes=1 << 40)
        total = len(ds)
        ids = np.random.default_rng(1).permutation(total).astype(np.int64)
        full = ds.decode_all()
        res = {'shards': args.shards, 'samples': total, 'runs': {}}
        # cold: shards decoded on demand as the shuffled batches first touch them
        bs = args.batch[0]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        nb = 0
        for i, b in enumerate(ds.iter_batches(ids[:bs * 50], bs)):
            nb += b.rows
        torch.cuda.synchronize()
        res['cold_50_batches'] = {'batch': bs, 'samples_per_s': nb / (time.perf_counter() - t0)}
        for bs in args.batch:
            m = min(args.batches, total // bs)
            sel = ids[:m * bs]
            first = next(iter(ds.iter_batches(sel[:bs], bs)))
            ok = same(first, full.gather(torch.from_numpy(sel[:bs])))
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rows = nbytes = 0
            for b in ds.iter_batches(sel, bs):
                rows += b.rows
                nbytes += batch_bytes(b)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            assert rows == m * bs
            res['runs'][str(bs)] = {'batches': m, 'ms_per_batch': dt / m * 1e3,
                                    'samples_per_s': rows / dt, 'out_GBps': nbytes / dt / 1e9,
                                    'first_batch_bit_exact': ok}
        # the per-sample drop-in path StreamingDataset.get_item takes (shard[idx] on a device
        # reader: the decoded shard's host copy, sliced per sample), shards already decoded
        n_items = min(20_000, total)
        for shard in ds.shards:  # first touch: the decoded shard's host copy (one D2H each)
            shard[0]
        t0 = time.perf_counter()
        for i in ids[:n_items]:
            ds.get_item(int(i))
        res['get_item'] = {'samples': n_items,
                           'samples_per_s': n_items / (time.perf_counter() - t0)}
        print(json.dumps(res, indent=1))
        assert all(r['first_batch_bit_exact'] for r in res['runs'].values())
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == '__main__':
    main()
