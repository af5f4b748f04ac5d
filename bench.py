"""Benchmark: device-resident MDS shard decode on MI355X (BASELINE.json metric).

One step = one decode of the rank's whole HBM-resident shard batch through libmdsx.so
(``mdsx_scan_shards`` + ``mdsx_decode_shards``): offsets-table scan, per-sample byte-range gather
and per-column decode of every sample of every shard, outputs materialised as torch tensors.

Default workload (N=1): BASELINE.json configs[1] = config B, 1M samples of
``{id: int32, x: ndarray:float32:1024}`` in 62 x 64 MiB shards. With
``--gpus N`` under torch.distributed.run every rank owns its own 1M-sample shard set
(per-GPU shard ownership, no collectives on the data path: weak scaling); the only
collectives are the timing barrier and the max-over-ranks reduction outside the timed region.

Prints ONE JSON line (rank 0) with the metric, a ``roofline`` object for the decode kernel
(algorithmic bytes R+W per launch / HIP-event kernel time, vs the 8 TB/s HBM3E peak) and a
``cpu_baseline`` object: the oracle's per-sample reader (a port of the reference algorithm,
oracle/mds_oracle.py) timed on one host core over a bounded sample of the same workload.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = 'decoded samples/sec + MDS GiB/s, device-resident, at 1/2/4/8 MI355X'
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s; 6.29 measured copy)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--config', choices=['B', 'C'], default='B')
    ap.add_argument('--samples', type=int, default=1_000_000, help='samples per GPU')
    ap.add_argument('--cpu-seconds', type=float, default=10.0,
                    help='CPU baseline time budget (0 disables)')
    ap.add_argument('--no-verify', action='store_true')
    return ap.parse_args()


def init_dist(args):
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        torch.cuda.set_device(local)
        torch.distributed.init_process_group('nccl', device_id=torch.device('cuda', local))
    else:
        torch.cuda.set_device(0)
    return world, rank, local


def barrier(world):
    if world > 1:
        torch.distributed.barrier()


def build_workload(args, rank, world):
    """Shards this rank owns, resident in HBM, plus what to verify them against."""
    from streaming_amd.synth import fixed_b_batch_on_device, var_c_shards
    from streaming_amd.decoder import Plan, stage_shards
    if args.config == 'B':
        synth = fixed_b_batch_on_device(args.samples, seed=1000 + rank,
                                        first_id=rank * args.samples)
        workload = (f'B: {args.samples} samples/GPU {{id:int32, x:ndarray:float32:1024}}, '
                    f'{len(synth.samples_per_shard)} x 64 MiB shards/GPU, HBM-resident')
        return synth.plan, synth.batch, synth.sources, workload
    shards, counts, src = var_c_shards(args.samples, seed=2000 + rank)
    plan = Plan(['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None])
    batch = stage_shards(shards, counts, plan)
    workload = (f'C: {args.samples} samples/GPU {{n:int, b:bytes U[3072,5120], s:str U[16,256] '
                f'cp}}, {len(counts)} x 64 MiB shards/GPU, HBM-resident')
    return plan, batch, src, workload


def verify(args, plan, out, sources):
    if args.config == 'B':
        ok = torch.equal(out['id'], sources['id']) and torch.equal(
            out['x'].view(torch.int32), sources['x'].view(torch.int32))
    else:
        ok = np.array_equal(out['n'].cpu().numpy(), sources['n'])
        ok &= np.array_equal(out['b'].values.cpu().numpy(), sources['b_pool'])
        ok &= np.array_equal(out['s'].values.cpu().numpy(), sources['s_pool'])
        ok &= int(out['s'].flags.sum()) == 0
    if not ok:
        raise SystemExit('PARITY FAILURE: decoded columns differ from the encoded sources')


def cpu_baseline(args):
    """Oracle per-sample reader (reference algorithm) on 1 host core, bounded sample."""
    from oracle.mds_oracle import OracleMDSReader
    from streaming_amd.synth import var_c_shards
    from streaming_amd.writer import encode_fixed_shard, shard_config_bytes
    tmp = tempfile.mkdtemp(prefix='mdsx_cpu_')
    if args.config == 'B':
        n = 16352
        names, encs, sizes = ['id', 'x'], ['int32', 'ndarray:float32:1024'], [4, 4096]
        config = shard_config_bytes(names, encs, sizes, None, [], 1 << 26)
        rng = np.random.default_rng(7)
        raw = encode_fixed_shard(config, [np.arange(n, dtype=np.int32),
                                          rng.integers(0, 2**32, (n, 1024), dtype=np.uint32)])
    else:
        shards, counts, _ = var_c_shards(16000, seed=7)
        raw, n = shards[0], counts[0]
        names, encs, sizes = ['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None]
    path = os.path.join(tmp, 'shard.00000.mds')
    with open(path, 'wb') as f:
        f.write(raw)
    info = {'raw_data': {'basename': 'shard.00000.mds'}, 'column_names': names,
            'column_encodings': encs, 'column_sizes': sizes, 'samples': n}
    reader = OracleMDSReader(tmp, None, info)
    offs = np.frombuffer(raw[4:4 + 4 * (n + 1)], np.uint32).astype(np.int64)
    sizes = np.diff(offs).tolist()
    done, nbytes, i = 0, 0, 0
    t0 = time.perf_counter()
    while True:
        reader.get_item(i)
        nbytes += sizes[i]
        done += 1
        i = i + 1 if i + 1 < n else 0
        if (done & 255) == 0 and time.perf_counter() - t0 >= args.cpu_seconds:
            break
    dt = time.perf_counter() - t0
    os.remove(path)
    os.rmdir(tmp)
    return {
        'value': done / dt,
        'unit': 'samples/s',
        'gib_per_s': nbytes / dt / 2**30,
        'cores': 1,
        'kind': 'port',
        'sample': (f'oracle per-sample MDSReader loop (open/seek/read + frombuffer per sample, '
                   f'mds/reader.py:103-149) over one 64 MiB config-{args.config} shard from '
                   f'page cache, {done} samples in {dt:.1f} s'),
    }


def main():
    args = parse_args()
    world, rank, local = init_dist(args)
    dev = torch.device('cuda', torch.cuda.current_device())
    from streaming_amd.decoder import BatchDecoder, output_bytes

    plan, batch, sources, workload = build_workload(args, rank, world)
    dec = BatchDecoder(plan, batch)
    out = dec.run()
    dec.check()
    if not args.no_verify:
        verify(args, plan, out, sources)
    for _ in range(args.warmup):
        dec.run()
    torch.cuda.synchronize(dev)

    K = args.steps
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(K)]
    barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(K):
        dec.run(events[k])
    torch.cuda.synchronize(dev)
    barrier(world)
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t.item())
    dec.check()
    if not args.no_verify:
        verify(args, plan, dec.result(), sources)

    decode_ms = [events[k][1].elapsed_time(events[k][2]) for k in range(K)]
    scan_ms = [events[k][0].elapsed_time(events[k][1]) for k in range(K)]
    kern_s = float(np.mean(decode_ms)) / 1e3
    R = batch.shard_bytes
    W = output_bytes(plan, dec.result())
    rows = batch.total_rows
    total_rows = rows * world
    value = total_rows * K / elapsed
    gibs = R * world * K / elapsed / 2**30
    achieved = (R + W) / kern_s / 1e9

    if rank == 0:
        cpu = cpu_baseline(args) if args.cpu_seconds > 0 else None
        line = {
            'metric': METRIC,
            'value': value,
            'unit': 'samples/s',
            'mds_gib_per_s': gibs,
            'n_gpus': world,
            'steps': K,
            'warmup': args.warmup,
            'ms_per_step': elapsed / K * 1e3,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'u8',
            'data': 'synthetic',
            'parity': 'bit-exact vs encoded source columns' if not args.no_verify else 'skipped',
            'config': {
                'workload': workload,
                'samples_per_gpu': rows,
                'shards_per_gpu': batch.nshards,
                'shard_bytes_per_gpu': R,
                'output_bytes_per_gpu': W,
                'parallelism': f'{world} GPU(s), per-GPU shard ownership, no data-path collectives',
            },
            'roofline': {
                'bound': 'hbm',
                'kernel': 'mdsx_kernels::decode_kernel',
                'achieved': achieved,
                'peak': HBM_PEAK_GBS,
                'unit': 'GB/s',
                'frac': achieved / HBM_PEAK_GBS,
                'traffic': None,
                'algorithmic_bytes_per_launch': R + W,
                'kernel_ms': kern_s * 1e3,
                'scan_ms': float(np.mean(scan_ms)),
            },
            'cpu_baseline': cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
