"""End-to-end (host-inclusive) decode rates for DESIGN.md §7, on one GPU.

Writes synthetic shard files (config B, C, or E = B-compressible written with zstd,
``streaming/base/stream.py:319-351``, ``compression.py:243-258``) to a temp directory (page
cache), keeping the source columns, then measures in one process:

* the stages alone: host read (or zstd decompress) into pinned staging, H2D of the staged batch,
  device-resident decode, D2H of the decoded columns;
* the pipelined ShardPipeline (read/decompress -> pinned -> H2D -> decode) per (mode, depth):
  ``device`` (device hand-off), ``d2h`` (a blocking ``to_host`` per batch), ``d2h_overlap``
  (``ShardPipeline.iter_host``), and ``validate_<algo>`` (device hand-off with every shard's
  index.json digest checked).

Parity: every pipeline's first (untimed) pass compares every decoded batch bit-exact against the
source columns the shard files were written from (device hand-offs are copied to the host for
the comparison); a mismatch aborts the run. Timing: ``--passes`` timed passes per pipeline,
round-robin over the pipelines so that drift on the box reaches all of them alike; each entry
reports the median, min, max and spread ((max - min) / median) of the passes.

Prints one JSON object (``--out`` also writes it to a file).
"""

import argparse
import json
import os
import shutil
import statistics
import sys
import tempfile
import time
from concurrent.futures import ThreadPoolExecutor

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


class Sources:
    """The columns the shard files encode, sliced per run of consecutive shards."""

    def __init__(self, cfg, counts, cols):
        self.cfg = cfg
        self.first = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        self.cols = cols
        if cfg == 'C':
            self.b_off = np.concatenate([[0], np.cumsum(cols['b_len'])]).astype(np.int64)
            self.s_off = np.concatenate([[0], np.cumsum(cols['s_len'])]).astype(np.int64)

    def check(self, host, s0, s1):
        """Raise unless ``host`` (to_host / iter_host arrays) is shards [s0, s1) bit-exact."""
        r0, r1 = int(self.first[s0]), int(self.first[s1])
        if self.cfg == 'C':
            exp = {'n': self.cols['n'][r0:r1]}
            for name, off, pool in (('b', self.b_off, self.cols['b_pool']),
                                    ('s', self.s_off, self.cols['s_pool'])):
                exp[name] = (pool[off[r0]:off[r1]], off[r0:r1 + 1] - off[r0])
            _same(host['n'].view(np.uint8), exp['n'].view(np.uint8), 'n', s0)
            for name in ('b', 's'):
                got = host[name]
                _same(got[0], exp[name][0], name + '.values', s0)
                _same(got[1], exp[name][1], name + '.offsets', s0)
                if name == 's' and got[2].any():
                    raise AssertionError(f'batch at shard {s0}: str flagged invalid UTF-8')
        else:
            _same(host['id'], np.arange(r0, r1, dtype=np.int32), 'id', s0)
            _same(host['x'].reshape(r1 - r0, -1).view(np.uint32),
                  self.cols['x'][r0:r1].view(np.uint32), 'x', s0)


def _same(got, exp, what, s0):
    if got.shape != exp.shape or not np.array_equal(got, exp):
        raise AssertionError(f'batch at shard {s0}: column {what} differs from the source')


def make_files(cfg, samples, out, workers, hashes=()):
    rng = np.random.default_rng(5)
    if cfg in ('B', 'E'):
        names, encs, sizes = ['id', 'x'], ['int32', 'ndarray:float32:1024'], [4, 4096]
        comp = 'zstd' if cfg == 'E' else None
        config = shard_config_bytes(names, encs, sizes, comp, [], 1 << 26)
        per = ((1 << 26) - 8 - len(config)) // (4100 + 4)
        if cfg == 'B':
            x = rng.integers(0, 2**32, (samples, 1024), dtype=np.uint32)
        else:  # compressible: small integers as float32
            x = rng.integers(0, 256, (samples, 1024)).astype(np.float32)
        counts = [min(per, samples - s0) for s0 in range(0, samples, per)]
        first = np.concatenate([[0], np.cumsum(counts)])

        def raw_of(i):
            s0, s1 = int(first[i]), int(first[i + 1])
            return encode_fixed_shard(config, [np.arange(s0, s1, dtype=np.int32), x[s0:s1]])

        sources = Sources(cfg, counts, {'x': x})
    else:
        names, encs, sizes = ['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None]
        comp = None
        data, counts, cols = var_c_shards(samples, seed=6)
        sources = Sources(cfg, counts, cols)

        def raw_of(i):
            return data[i]

    def write(i):
        raw = raw_of(i)
        path = os.path.join(out, f'shard.{i:05}.mds' + ('.zstd' if comp else ''))
        blob = compress('zstd', raw) if comp else raw
        with open(path, 'wb') as f:
            f.write(blob)
        digests = {algo: get_hash(algo, raw) for algo in hashes}  # index.json raw_data.hashes
        return ShardFile(path, len(raw), counts[i], comp, digests), len(blob)

    with ThreadPoolExecutor(workers) as ex:
        res = list(ex.map(write, range(len(counts))))
    return Plan(names, encs, sizes), [r[0] for r in res], sum(r[1] for r in res), sources


def _stats(secs, raw_bytes, rows):
    med = statistics.median(secs)
    return {'raw_GiBps': raw_bytes / med / 2**30, 'samples_per_s': rows / med,
            'raw_GiBps_min': raw_bytes / max(secs) / 2**30,
            'raw_GiBps_max': raw_bytes / min(secs) / 2**30,
            'spread': (max(secs) - min(secs)) / med, 'seconds_median': med,
            'seconds': secs}


class Run:
    """One pipeline configuration: its verification pass, then timed passes."""

    def __init__(self, key, mode, depth, algo, args, plan, files):
        self.key, self.mode, self.depth, self.algo = key, mode, depth, algo
        self.pipe = ShardPipeline(plan, files, shards_per_batch=args.per_batch, depth=depth,
                                  workers=args.workers, validate_hash=algo)
        self.first_col = plan.columns[0].name
        self.secs = []

    def _batches(self):
        """Yields (host arrays or None, shard index of the batch's first shard)."""
        s0 = 0
        if self.mode == 'd2h_overlap':
            for h, g in zip(self.pipe.iter_host(), self.pipe.groups):
                yield h, s0
                s0 += len(g)
        else:
            for b, g in zip(self.pipe, self.pipe.groups):
                yield (to_host(b) if self.mode == 'd2h' else b), s0
                s0 += len(g)

    def verify(self, sources):
        n = 0
        for out, s0 in self._batches():
            host = out if isinstance(out, dict) else to_host(out)
            s1 = s0 + len(self.pipe.groups[n])
            sources.check(host, s0, s1)
            n += 1
        if n != len(self.pipe.groups):
            raise AssertionError(f'{self.key}: {n} batches of {len(self.pipe.groups)}')

    def timed(self, rows):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        n = 0
        for out, _ in self._batches():
            if isinstance(out, dict):
                v = out[self.first_col]
                n += (len(v[1]) - 1) if isinstance(v, tuple) else len(v)
            else:
                n += out.rows
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if n != rows:
            raise AssertionError(f'{self.key}: {n} rows of {rows}')
        self.secs.append(dt)

    def trace(self):
        """One more pass with the pipeline's step marks: per batch, host and device times (ms
        from the pass start)."""
        self.pipe.trace = []
        torch.cuda.synchronize()
        start = torch.cuda.Event(enable_timing=True)
        start.record()
        t0 = time.perf_counter()
        for _ in self._batches():
            pass
        torch.cuda.synchronize()
        rows = []
        for what, gi, t, ev in self.pipe.trace:
            rows.append([what, gi, round((t - t0) * 1e3, 3),
                         None if ev is None else round(start.elapsed_time(ev), 3)])
        self.pipe.trace = None
        return rows


def stages(args, plan, files, raw_bytes, rows, res):
    """The stages alone, each timed ``--passes`` times."""
    batch = make_batch(plan, [f.raw_bytes for f in files], [f.samples for f in files])
    pinned = torch.empty(batch.buffer.numel(), dtype=torch.uint8, pin_memory=True)
    view = pinned.numpy()
    secs = []
    with ThreadPoolExecutor(args.workers) as ex:
        for rep in range(args.passes + 1):  # the first pass warms the page cache
            t0 = time.perf_counter()
            list(ex.map(lambda i: _fill(view[batch.offsets[i]:batch.offsets[i] +
                                             files[i].raw_bytes], files[i]),
                        range(len(files))))
            if rep:
                secs.append(time.perf_counter() - t0)
    res['stage_host_read_or_decompress'] = _stats(secs, raw_bytes, rows)
    secs = []
    for rep in range(args.passes + 1):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        batch.buffer.copy_(pinned, non_blocking=True)
        torch.cuda.synchronize()
        if rep:
            secs.append(time.perf_counter() - t0)
    res['stage_h2d'] = _stats(secs, raw_bytes, rows)
    res['stage_h2d']['GBps_of_buffer'] = pinned.numel() / statistics.median(secs) / 1e9
    dec = BatchDecoder(plan, batch)
    out = dec.run()
    dec.check()
    for _ in range(3):
        dec.run()
    secs = []
    for _ in range(args.passes):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            dec.run()
        torch.cuda.synchronize()
        secs.append((time.perf_counter() - t0) / 10)
    res['stage_decode_resident'] = _stats(secs, raw_bytes, rows)
    W = output_bytes(plan, out)
    for _ in range(2):  # the pinned host blocks allocated once, then reused from torch's cache
        to_host(dec.result())
    secs = []
    for _ in range(args.passes):
        t0 = time.perf_counter()
        to_host(dec.result())
        secs.append(time.perf_counter() - t0)
    res['stage_d2h'] = _stats(secs, raw_bytes, rows)
    res['stage_d2h']['GBps_of_outputs'] = W / statistics.median(secs) / 1e9
    del dec, out, batch, pinned
    torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='B', choices=['B', 'C', 'E'])
    ap.add_argument('--samples', type=int, default=1_000_000)
    ap.add_argument('--workers', type=int, default=16)
    ap.add_argument('--per-batch', type=int, default=8)
    ap.add_argument('--passes', type=int, default=5, help='timed passes per pipeline (>= 5)')
    ap.add_argument('--dir', default=None)
    ap.add_argument('--validate', default='',
                    help='comma-separated hash algorithms: also time the pipeline validating each '
                         '(xxh3 on the device, the rest on the host threads), at each depth')
    ap.add_argument('--skip-stages', action='store_true', help='only the pipelined runs')
    ap.add_argument('--depth', type=int, nargs='+', default=[2, 3],
                    help='ShardPipeline depths of the pipelined runs')
    ap.add_argument('--modes', default='device,d2h,d2h_overlap',
                    help='pipelined runs: device, d2h (blocking to_host), d2h_overlap (iter_host)')
    ap.add_argument('--trace', default='', help='comma-separated run keys to trace once')
    ap.add_argument('--out', default=None, help='also write the JSON here')
    args = ap.parse_args()
    algos = [a for a in args.validate.split(',') if a]
    torch.cuda.set_device(0)
    tmp = tempfile.mkdtemp(prefix='mdsx_e2e_', dir=args.dir)
    try:
        t0 = time.perf_counter()
        plan, files, file_bytes, sources = make_files(args.config, args.samples, tmp,
                                                      args.workers, algos)
        gen_s = time.perf_counter() - t0
        raw_bytes = sum(f.raw_bytes for f in files)
        rows = sum(f.samples for f in files)
        res = {'config': args.config, 'samples': rows, 'shards': len(files),
               'raw_bytes': raw_bytes, 'file_bytes': file_bytes, 'workers': args.workers,
               'shards_per_batch': args.per_batch, 'passes': args.passes,
               'host_cpus': len(os.sched_getaffinity(0)), 'generate_s': gen_s,
               'parity': 'every pipeline\'s first pass bit-exact vs the source columns'}
        print(f'generated {len(files)} shards in {gen_s:.1f} s', file=sys.stderr, flush=True)
        if not args.skip_stages:
            stages(args, plan, files, raw_bytes, rows, res)
            print('stages done', file=sys.stderr, flush=True)
        names = {'device': 'e2e_device_handoff', 'd2h': 'e2e_with_d2h',
                 'd2h_overlap': 'e2e_with_d2h_overlapped'}
        runs = []
        for depth in args.depth:
            for mode in args.modes.split(','):
                runs.append(Run(f'{names[mode]}_depth{depth}', mode, depth, None, args, plan,
                                files))
        for algo in algos:
            where = 'device' if algo in PIPELINE_DEVICE_HASHES else 'host'
            for depth in args.depth:
                runs.append(Run(f'e2e_validate_{algo}_{where}_depth{depth}', 'device', depth,
                                algo, args, plan, files))
        for r in runs:
            r.verify(sources)
            print(f'{r.key}: verified', file=sys.stderr, flush=True)
        for p in range(args.passes):
            for r in (runs if p % 2 == 0 else runs[::-1]):
                r.timed(rows)
            print(f'pass {p} done', file=sys.stderr, flush=True)
        for r in runs:
            res[r.key] = _stats(r.secs, raw_bytes, rows)
        for key in [k for k in args.trace.split(',') if k]:
            res['trace_' + key] = next(r for r in runs if r.key == key).trace()
        for r in runs:
            r.pipe.close()
        text = json.dumps(res, indent=1)
        print(text)
        if args.out:
            os.makedirs(os.path.dirname(args.out) or '.', exist_ok=True)
            with open(args.out, 'w') as f:
                f.write(text + '\n')
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


if __name__ == '__main__':
    main()
