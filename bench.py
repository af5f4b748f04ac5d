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
oracle/mds_oracle.py) timed on 16 host cores (one process each, 2 s: ~32 s of CPU work) over a
bounded sample of the same workload.
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
    ap.add_argument('--cpu-seconds', type=float, default=2.0,
                    help='CPU baseline time budget (0 disables)')
    ap.add_argument('--cpu-procs', type=int, default=16,
                    help='CPU baseline processes (disjoint shard copies, one per core; 16 = the '
                         'host-core share of one GPU on the MI355X boxes)')
    ap.add_argument('--single', action='store_true',
                    help='ragged configs: single-pass decode (look-back scan inside the decode '
                    'kernel, outputs at the payload bound) instead of scan + decode')
    ap.add_argument('--no-verify', action='store_true')
    ap.add_argument('--no-copy-probe', dest='copy_probe', action='store_false',
                    help='skip the same-run copy-ceiling measurement')
    return ap.parse_args()


def init_dist(args):
    from streaming_amd.distributed import rank_info
    info = rank_info()
    world, rank, local = info.world_size, info.rank, info.local_rank
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


def _cpu_shard(config, seed):
    """One 64 MiB shard of the workload written to a temp dir (oracle reader input)."""
    from streaming_amd.synth import var_c_shards
    from streaming_amd.writer import encode_fixed_shard, shard_config_bytes
    if config == 'B':
        n = 16352
        names, encs, sizes = ['id', 'x'], ['int32', 'ndarray:float32:1024'], [4, 4096]
        cfg = shard_config_bytes(names, encs, sizes, None, [], 1 << 26)
        rng = np.random.default_rng(seed)
        raw = encode_fixed_shard(cfg, [np.arange(n, dtype=np.int32),
                                       rng.integers(0, 2**32, (n, 1024), dtype=np.uint32)])
    else:
        shards, counts, _ = var_c_shards(16000, seed=seed)
        raw, n = shards[0], counts[0]
        names, encs, sizes = ['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None]
    return raw, n, names, encs, sizes


def _cpu_worker(config, seed, seconds, q):
    """Oracle per-sample reader loop over one shard for `seconds` (one process = one core)."""
    from oracle.mds_oracle import OracleMDSReader
    raw, n, names, encs, sizes = _cpu_shard(config, seed)
    tmp = tempfile.mkdtemp(prefix='mdsx_cpu_')
    path = os.path.join(tmp, 'shard.00000.mds')
    with open(path, 'wb') as f:
        f.write(raw)
    info = {'raw_data': {'basename': 'shard.00000.mds'}, 'column_names': names,
            'column_encodings': encs, 'column_sizes': sizes, 'samples': n}
    reader = OracleMDSReader(tmp, None, info)
    offs = np.frombuffer(raw[4:4 + 4 * (n + 1)], np.uint32).astype(np.int64)
    row_bytes = np.diff(offs).tolist()
    for i in range(min(n, 256)):  # warm the page cache and the interpreter
        reader.get_item(i)
    done, nbytes, i = 0, 0, 0
    t0 = time.perf_counter()
    while True:
        reader.get_item(i)
        nbytes += row_bytes[i]
        done += 1
        i = i + 1 if i + 1 < n else 0
        if (done & 255) == 0 and time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    os.remove(path)
    os.rmdir(tmp)
    q.put((done, nbytes, dt))


def cpu_baseline(args):
    """The reference algorithm (oracle port) timed on host cores: `--cpu-procs` processes, each
    looping the per-sample reader over its own shard; aggregate samples/s."""
    import multiprocessing as mp
    procs = max(1, args.cpu_procs)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_cpu_worker, args=(args.config, 7 + k, args.cpu_seconds, q))
          for k in range(procs)]
    for p in ps:
        p.start()
    res = [q.get() for _ in ps]
    for p in ps:
        p.join()
    done = sum(r[0] for r in res)
    nbytes = sum(r[1] for r in res)
    dt = max(r[2] for r in res)
    return {
        'value': done / dt,
        'unit': 'samples/s',
        'gib_per_s': nbytes / dt / 2**30,
        'cores': procs,
        'kind': 'port',
        'sample': (f'oracle per-sample MDSReader loop (open/seek/read + frombuffer per sample, '
                   f'mds/reader.py:103-149; encodings.py:760-773) over a 64 MiB config-'
                   f'{args.config} shard from page cache per process, {procs} process(es), '
                   f'{done} samples in {dt:.1f} s ({done / dt / procs:.0f} samples/s per core)'),
    }


def committed_traffic(config):
    """Per-launch HBM bytes of the decode kernel from the newest committed rocprofv3 PMC run of
    this benchmark (FETCH_SIZE doubled per MI355X_MICROARCH.md §HBM, + WRITE_SIZE)."""
    import glob
    files = sorted(glob.glob(os.path.join(HERE, 'profiles', 'r*', f'pmc_bench_{config}_summary.json')))
    if not files:
        return None, None
    with open(files[-1]) as f:
        summ = json.load(f)
    return summ.get('hbm_traffic_bytes_per_launch'), os.path.relpath(files[-1], HERE)


def copy_ceiling(batch, dev, iters=10):
    """Median rate of a read+write streaming copy of the batch's shard bytes (GB/s)."""
    from streaming_amd import _native
    lib = _native.lib()
    src = batch.buffer
    dst = torch.empty_like(src)
    stream = torch.cuda.current_stream(dev)
    start = [torch.cuda.Event(enable_timing=True) for _ in range(iters + 1)]
    end = [torch.cuda.Event(enable_timing=True) for _ in range(iters + 1)]
    for i in range(iters + 1):
        start[i].record(stream)
        rc = lib.mdsx_copy_probe(src.data_ptr(), dst.data_ptr(), src.numel(), stream.cuda_stream)
        end[i].record(stream)
        if rc != 0:
            raise RuntimeError(f'mdsx_copy_probe failed: {lib.mdsx_last_error().decode()}')
    torch.cuda.synchronize(dev)
    if not torch.equal(src[-4096:], dst[-4096:]):
        raise RuntimeError('mdsx_copy_probe: copy mismatch')
    ms = float(np.median([start[i].elapsed_time(end[i]) for i in range(1, iters + 1)]))
    del dst
    return {'GBps': 2 * src.numel() / ms / 1e6, 'ms': ms, 'bytes_per_launch': 2 * src.numel()}


def main():
    args = parse_args()
    world, rank, local = init_dist(args)
    dev = torch.device('cuda', torch.cuda.current_device())
    from streaming_amd.decoder import BatchDecoder, output_bytes

    plan, batch, sources, workload = build_workload(args, rank, world)
    dec = BatchDecoder(plan, batch, single=args.single)
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
    from streaming_amd.distributed import max_over_ranks
    elapsed = max_over_ranks(t1 - t0, device=dev)
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

    copy = copy_ceiling(batch, dev) if args.copy_probe else None

    if rank == 0:
        cpu = cpu_baseline(args) if args.cpu_seconds > 0 else None
        traffic, traffic_src = committed_traffic(args.config)
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
                'traffic': traffic,
                'traffic_source': traffic_src,
                'algorithmic_bytes_per_launch': R + W,
                'kernel_ms': kern_s * 1e3,
                'scan_ms': float(np.mean(scan_ms)),
                # same-run streaming copy of the shard bytes (mdsx_copy_probe, the fastest copy
                # shape measured on this part): the practical HBM ceiling next to the 8 TB/s peak
                'copy_ceiling': copy,
                'frac_of_copy_ceiling': achieved / copy['GBps'] if copy else None,
            },
            'cpu_baseline': cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
