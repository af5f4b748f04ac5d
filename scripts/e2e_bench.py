"""End-to-end (host-inclusive) decode rates for DESIGN.md, on one GPU.

Writes synthetic shard files (config B, C, or E = B-compressible written with zstd) to a temp
directory (page cache), then measures, in one process:
  * host read (or zstd decompress) into pinned staging, all shards, `--workers` threads;
  * H2D of the staged batch; device-resident decode; D2H of the decoded columns;
  * the pipelined ShardPipeline (read/decompress -> pinned -> H2D -> decode), with and without
    the D2H hand-off.
Prints one JSON object.
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

from streaming_amd.compression import compress  # noqa: E402
from streaming_amd.hashing import get_hash  # noqa: E402
from streaming_amd.decoder import BatchDecoder, Plan, make_batch, output_bytes  # noqa: E402
from streaming_amd.pipeline import (PIPELINE_DEVICE_HASHES, ShardFile, ShardPipeline,  # noqa: E402
                                    _fill, to_host)
from streaming_amd.synth import var_c_shards  # noqa: E402
from streaming_amd.writer import encode_fixed_shard, shard_config_bytes  # noqa: E402


def make_files(cfg, samples, out, workers, hashes=()):
    rng = np.random.default_rng(5)
    files = []
    if cfg in ('B', 'E'):
        names, encs, sizes = ['id', 'x'], ['int32', 'ndarray:float32:1024'], [4, 4096]
        comp = 'zstd' if cfg == 'E' else None
        config = shard_config_bytes(names, encs, sizes, comp, [], 1 << 26)
        per = ((1 << 26) - 8 - len(config)) // (4100 + 4)
        shards = []
        for s0 in range(0, samples, per):
            n = min(per, samples - s0)
            if cfg == 'B':
                x = rng.integers(0, 2**32, (n, 1024), dtype=np.uint32)
            else:  # compressible: small integers as float32
                x = rng.integers(0, 256, (n, 1024)).astype(np.float32)
            shards.append((encode_fixed_shard(config, [np.arange(s0, s0 + n, dtype=np.int32), x]),
                           n))
    else:
        names, encs, sizes = ['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None]
        comp = None
        data, counts, _ = var_c_shards(samples, seed=6)
        shards = list(zip(data, counts))
    from concurrent.futures import ThreadPoolExecutor

    def write(i_raw):
        i, (raw, n) = i_raw
        path = os.path.join(out, f'shard.{i:05}.mds' + ('.zstd' if comp else ''))
        blob = compress('zstd', raw) if comp else raw
        with open(path, 'wb') as f:
            f.write(blob)
        digests = {algo: get_hash(algo, raw) for algo in hashes}  # index.json raw_data.hashes
        return ShardFile(path, len(raw), n, comp, digests), len(blob)

    with ThreadPoolExecutor(workers) as ex:
        res = list(ex.map(write, enumerate(shards)))
    return Plan(names, encs, sizes), [r[0] for r in res], sum(r[1] for r in res)


def _validate_runs(args, plan, files, raw_bytes, rows, algos, res):
    """The pipelined end-to-end run (device hand-off) with each shard's hash checked."""
    for algo in [None] + algos:
        pipe = ShardPipeline(plan, files, shards_per_batch=args.per_batch, depth=2,
                             workers=args.workers, validate_hash=algo)
        for _ in pipe:  # warm-up pass
            pass
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = sum(b.rows for b in pipe)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        pipe.close()
        assert n == rows
        where = 'device' if algo in PIPELINE_DEVICE_HASHES else 'host threads'
        res[f'e2e_validate_{algo or "none"}'] = {
            'samples_per_s': rows / dt, 'raw_GiBps': raw_bytes / dt / 2**30, 'seconds': dt,
            'hash_on': None if algo is None else where}


def _pipelined(args, plan, files, raw_bytes, rows, res):
    # 5. pipelined end to end: device hand-off; host hand-off with a blocking to_host per
    # batch; host hand-off with the D2H overlapped (ShardPipeline.iter_host)
    first_col = plan.columns[0].name
    for depth, mode in [(d, m) for d in args.depth for m in args.modes.split(',')]:
        pipe = ShardPipeline(plan, files, shards_per_batch=args.per_batch, depth=depth,
                             workers=args.workers)
        for b in (pipe.iter_host() if mode == 'd2h_overlap' else pipe):  # warm-up pass
            pass
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        if mode == 'd2h_overlap':
            for h in pipe.iter_host():
                v = h[first_col]
                n += (len(v[1]) - 1) if isinstance(v, tuple) else len(v)
        else:
            for b in pipe:
                n += b.rows
                if mode == 'd2h':
                    to_host(b)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        pipe.close()
        assert n == rows
        key = {'device': 'e2e_device_handoff', 'd2h': 'e2e_with_d2h',
               'd2h_overlap': 'e2e_with_d2h_overlapped'}[mode]
        if depth != 2:
            key += f'_depth{depth}'
        res[key] = {'samples_per_s': rows / dt, 'raw_GiBps': raw_bytes / dt / 2**30,
                    'seconds': dt}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='B', choices=['B', 'C', 'E'])
    ap.add_argument('--samples', type=int, default=1_000_000)
    ap.add_argument('--workers', type=int, default=16)
    ap.add_argument('--per-batch', type=int, default=8)
    ap.add_argument('--dir', default=None)
    ap.add_argument('--validate', default='',
                    help='comma-separated hash algorithms: also time the pipeline validating each '
                         '(ShardPipeline validate_hash; xxh3 on the device, the rest on the host '
                         'threads)')
    ap.add_argument('--skip-stages', action='store_true', help='only the pipelined runs')
    ap.add_argument('--depth', type=int, nargs='+', default=[2],
                    help='ShardPipeline depths of the pipelined runs')
    ap.add_argument('--modes', default='device,d2h,d2h_overlap',
                    help='pipelined runs: device, d2h (blocking to_host), d2h_overlap (iter_host)')
    args = ap.parse_args()
    algos = [a for a in args.validate.split(',') if a]
    torch.cuda.set_device(0)
    tmp = tempfile.mkdtemp(prefix='mdsx_e2e_', dir=args.dir)
    try:
        t0 = time.perf_counter()
        plan, files, file_bytes = make_files(args.config, args.samples, tmp, args.workers, algos)
        gen_s = time.perf_counter() - t0
        raw_bytes = sum(f.raw_bytes for f in files)
        rows = sum(f.samples for f in files)
        res = {'config': args.config, 'samples': rows, 'shards': len(files),
               'raw_bytes': raw_bytes, 'file_bytes': file_bytes, 'workers': args.workers,
               'host_cpus': len(os.sched_getaffinity(0)), 'generate_s': gen_s}
        if args.skip_stages:
            _pipelined(args, plan, files, raw_bytes, rows, res)
            _validate_runs(args, plan, files, raw_bytes, rows, algos, res)
            print(json.dumps(res, indent=1))
            return
        # 1. stage everything into one pinned buffer (page cache -> pinned), threads
        batch = make_batch(plan, [f.raw_bytes for f in files], [f.samples for f in files])
        pinned = torch.empty(batch.buffer.numel(), dtype=torch.uint8, pin_memory=True)
        view = pinned.numpy()
        from concurrent.futures import ThreadPoolExecutor
        with ThreadPoolExecutor(args.workers) as ex:
            for rep in range(2):  # first pass warms the page cache
                t0 = time.perf_counter()
                list(ex.map(lambda i: _fill(view[batch.offsets[i]:batch.offsets[i] +
                                                 files[i].raw_bytes], files[i]),
                            range(len(files))))
                read_s = time.perf_counter() - t0
        res['host_read_or_decompress_GBps'] = raw_bytes / read_s / 1e9
        # 2. H2D
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        batch.buffer.copy_(pinned, non_blocking=True)
        torch.cuda.synchronize()
        res['h2d_GBps'] = pinned.numel() / (time.perf_counter() - t0) / 1e9
        # 3. device-resident decode
        dec = BatchDecoder(plan, batch)
        out = dec.run()
        dec.check()
        for _ in range(3):
            dec.run()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            dec.run()
        torch.cuda.synchronize()
        dec_s = (time.perf_counter() - t0) / 10
        res['decode_resident_ms'] = dec_s * 1e3
        res['decode_resident_samples_per_s'] = rows / dec_s
        res['decode_resident_GiBps'] = raw_bytes / dec_s / 2**30
        W = output_bytes(plan, out)
        # 4. D2H of the outputs
        to_host(dec.result())
        t0 = time.perf_counter()
        to_host(dec.result())
        res['d2h_GBps'] = W / (time.perf_counter() - t0) / 1e9
        del dec, out, batch
        torch.cuda.empty_cache()
        _pipelined(args, plan, files, raw_bytes, rows, res)
        _validate_runs(args, plan, files, raw_bytes, rows, algos, res)
        print(json.dumps(res, indent=1))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == '__main__':
    main()
