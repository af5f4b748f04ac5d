"""Benchmark: device-resident MDS shard decode on MI355X (BASELINE.json metric).

One step = one decode of the rank's whole HBM-resident shard batch through libmdsx.so
(``mdsx_scan_shards`` + ``mdsx_decode_shards``): offsets-table scan, per-sample byte-range gather
and per-column decode of every sample of every shard, outputs materialised as torch tensors.

Workloads (synthetic shards built on the device, bit-identical to the reference
writer's layout, verified against their sources before and after the timed region):

* config B (the headline line): ``{id: int32, x: ndarray:float32:1024}``, 62 full 64 MiB shards
  (1 013 824 samples) per GPU;
* config C (the ``config_c`` object of the same line): ``{n: int, b: bytes U[3072,5120], s: str}``,
  64 full 64 MiB shards (~1M samples) per GPU, written by the device MDS encoder.

Multi-GPU: the dataset is ``N x shards_per_gpu`` global shards; global shard ``g``
is generated from seed ``base + g`` and owned by rank ``g % N`` (``streaming_amd.distributed.
owned_shards``): weak scaling, no collective on the data path. ``python bench.py --gpus N``
starts N child processes itself (one per GPU, ``RANK`` / ``LOCAL_RANK`` / ``WORLD_SIZE`` /
``MASTER_*`` as ``torch.distributed.run`` sets them, the reference's env contract,
``streaming/base/distributed.py:23-56``) before anything touches the GPU; under
``torch.distributed.run`` it runs as the given rank. A world size different from ``--gpus`` is an
error. Only the timing barriers and the max-over-ranks reduction are collectives.

Rank 0 prints ONE JSON line with the metric, a ``roofline`` object per config (algorithmic bytes
R+W per launch / HIP-event kernel time on the launch stream, vs the 8 TB/s HBM3E peak and the
6.29 TB/s float4 copy the microarchitecture guide records; ``traffic`` from a committed
rocprofv3 PMC summary of the SAME workload and kernel, else null) and a ``cpu_baseline`` object
per config: the reference reader restated with its per-call coder construction
(``oracle/mds_oracle.py``, kind "port") timed on host cores, 1 core and all cores of the box's share.
"""

from __future__ import annotations

import argparse
import glob
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = 'decoded samples/sec + MDS GiB/s, device-resident, at 1/2/4/8 MI355X'
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
COPY_MEASURED_GBS = 6290.0  # MI355X_MICROARCH.md: float4 copy measured on MI355X
SEED_B, SEED_C = 1000, 2000
SHARDS_PER_GPU = {'B': 62, 'C': 64}


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    # untimed steps first: the decode reaches its steady rate after ~20 launches (config C 2 %
    # faster after 30 warm-up steps than after 3, profiles/r02/warmup.txt)
    ap.add_argument('--warmup', type=int, default=20)
    ap.add_argument('--config', choices=['B', 'C', 'BC'], default='BC',
                    help='B = headline line only; BC = B plus the config_c object')
    ap.add_argument('--shards', type=int, default=0,
                    help='shards per GPU (0: 62 for B, 64 for C = ~1M samples)')
    ap.add_argument('--cpu-seconds', type=float, default=2.0,
                    help='CPU baseline seconds per leg (0 disables)')
    ap.add_argument('--cpu-procs', type=int, default=0,
                    help='all-core CPU leg processes (0: the box share, see cpu_cores())')
    ap.add_argument('--single', action='store_true',
                    help='ragged configs: single-pass decode (look-back scan inside the decode '
                    'kernel) instead of scan + decode')
    ap.add_argument('--scan-ahead', action='store_true',
                    help='ragged configs: the next step\'s scan pass on a side stream beside this '
                    'step\'s decode (ScanAheadDecoder; measured no faster on MI355X, DESIGN.md '
                    '§9: the decode holds the CUs, so the scan competes instead of overlapping)')
    ap.add_argument('--no-verify', action='store_true')
    ap.add_argument('--no-copy-probe', dest='copy_probe', action='store_false',
                    help='skip the same-run copy-ceiling measurement')
    ap.add_argument('--dist', action='store_true',
                    help='set up the process group even for one rank (nccl = RCCL on the GPU): '
                         'runs the barrier / max-over-ranks / gather collectives of the N > 1 '
                         'path on a one-GPU box')
    ap.add_argument('--fresh-steps', type=int, default=6,
                    help='ragged configs: also time this many steps over two distinct resident '
                    'batches taken in turn, each with a decoder of its own (its sizing included: '
                    'the totals read back and the outputs allocated; and the single-pass form, '
                    'outputs at their upper bound); 0 disables')
    ap.add_argument('--dry-run', action='store_true',
                    help='no GPU: exercise the launcher, process group (gloo) and shard '
                    'ownership only (CPU test hook)')
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------------------------
# launcher: N fresh child processes, started before any GPU call of this process
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def launch(args, argv) -> int:
    """Run ``bench.py`` as ``--gpus`` ranks (one child process per GPU) and return the exit code
    (the first failing rank's, else 0). Rank 0's stdout is the benchmark line."""
    port = _free_port()
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus),
                   LOCAL_WORLD_SIZE=str(args.gpus), MASTER_ADDR='127.0.0.1',
                   MASTER_PORT=str(port))
        env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env, stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    while procs:
        for p in list(procs):
            code = p.poll()
            if code is None:
                continue
            procs.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in procs:  # one rank failed: the others would wait in a collective
                    q.kill()
        time.sleep(0.05)
    return rc


def init_dist(args):
    from streaming_amd.distributed import rank_info
    info = rank_info()
    world, rank, local = info.world_size, info.rank, info.local_rank
    if world != args.gpus:
        raise SystemExit(f'bench.py: --gpus {args.gpus} but WORLD_SIZE={world}')
    if (world > 1 or args.dist) and world == 1:  # --dist on one rank: its own rendezvous
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', str(_free_port()))
        os.environ.setdefault('RANK', '0')
        os.environ.setdefault('WORLD_SIZE', '1')
    if args.dry_run:
        if world > 1 or args.dist:
            torch.distributed.init_process_group('gloo')
        return world, rank, local, torch.device('cpu')
    if torch.cuda.device_count() < local + 1:
        raise SystemExit(f'bench.py: rank {rank} needs GPU {local}, '
                         f'{torch.cuda.device_count()} visible')
    torch.cuda.set_device(local)
    dev = torch.device('cuda', local)
    if world > 1 or args.dist:
        torch.distributed.init_process_group('nccl', device_id=dev)
    return world, rank, local, dev


def _dist_on() -> bool:
    return torch.distributed.is_available() and torch.distributed.is_initialized()


def barrier(world):
    if _dist_on():
        torch.distributed.barrier()


def gather_objects(world, obj):
    if not _dist_on():
        return [obj]
    out = [None] * world
    torch.distributed.all_gather_object(out, obj)
    return out


# ---------------------------------------------------------------------------------------------
# workloads
def shard_plan(args, config, rank, world):
    from streaming_amd.distributed import owned_shards
    per_gpu = args.shards or SHARDS_PER_GPU[config]
    total = per_gpu * world
    return owned_shards(total, rank, world), total


def build_workload(config, shard_ids):
    """This rank's shards (global ids ``shard_ids``) resident in HBM + their source columns."""
    from streaming_amd.synth import fixed_b_batch_on_device, var_c_batch_on_device
    if config == 'B':
        synth = fixed_b_batch_on_device(0, seed=SEED_B, shard_ids=shard_ids)
        desc = (f'B: {{id:int32, x:ndarray:float32:1024}}, {len(shard_ids)} full 64 MiB '
                f'shards/GPU ({synth.batch.total_rows} samples), HBM-resident')
    else:
        synth = var_c_batch_on_device(shard_ids, seed=SEED_C)
        desc = (f'C: {{n:int, b:bytes U[3072,5120], s:str U[16,256] code points of 1-4 UTF-8 '
                f'bytes}}, {len(shard_ids)} full 64 MiB shards/GPU ({synth.batch.total_rows} '
                f'samples), HBM-resident')
    return synth, desc


def verify(config, out, sources):
    if config == 'B':
        ok = torch.equal(out['id'], sources['id']) and torch.equal(
            out['x'].view(torch.int32), sources['x'].view(torch.int32))
    else:
        ok = torch.equal(out['n'], sources['n'])
        for name in ('b', 's'):
            ok &= torch.equal(out[name].offsets - out[name].offsets[0],
                              sources[name].offsets - sources[name].offsets[0])
            ok &= torch.equal(out[name].values, sources[name].values)
        ok &= int(out['s'].flags.sum()) == 0
    if not ok:
        raise SystemExit(f'PARITY FAILURE: config {config} decoded columns differ from the '
                         f'encoded sources')


def workload_key(config, batch, W):
    """What a committed PMC summary must match to be this run's traffic evidence."""
    return f'{config}:shards={batch.nshards}:rows={batch.total_rows}:R={batch.shard_bytes}:W={W}'


# ---------------------------------------------------------------------------------------------
# CPU baseline: the reference reader restated (oracle, per-call coder construction), host cores
def cpu_cores():
    """Processes for the all-core leg: the CPUs this process may run on
    (``len(os.sched_getaffinity(0))``), capped by the box's CPU share
    (``OMP_NUM_THREADS``, 16 per GPU on the MI355X boxes) -- returns (used, affinity, share)."""
    aff = len(os.sched_getaffinity(0))
    share = int(os.environ.get('OMP_NUM_THREADS', '0') or 0)
    return (min(aff, share) if share > 0 else aff), aff, share


def _cpu_worker(path, n, names, encs, sizes, seconds, q):
    """Per-sample reader loop over one shard file for ``seconds`` (one process = one core)."""
    from oracle.mds_oracle import ReferenceCostMDSReader
    info = {'raw_data': {'basename': os.path.basename(path)}, 'column_names': names,
            'column_encodings': encs, 'column_sizes': sizes, 'samples': n}
    reader = ReferenceCostMDSReader(os.path.dirname(path), None, info)
    with open(path, 'rb') as f:
        raw = f.read(4 + 4 * (n + 1))
    offs = np.frombuffer(raw[4:], np.uint32).astype(np.int64)
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
    q.put((done, nbytes, time.perf_counter() - t0))


def _cpu_leg(files, meta, procs, seconds):
    import multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_cpu_worker, args=(*files[k % len(files)], *meta, seconds, q))
          for k in range(procs)]
    for p in ps:
        p.start()
    res = [q.get(timeout=seconds + 300) for _ in ps]
    for p in ps:
        p.join()
    done = sum(r[0] for r in res)
    nbytes = sum(r[1] for r in res)
    dt = max(r[2] for r in res)
    return done / dt, nbytes / dt / 2**30, done, dt


def cpu_baseline(args, config, synth, tmpdir):
    """1-core and all-core legs over shard files copied from this rank's device workload."""
    used, aff, share = cpu_cores()
    procs = args.cpu_procs or used
    batch, plan = synth.batch, synth.plan
    nfiles = min(batch.nshards, max(procs, 1))
    files = []
    for s in range(nfiles):
        o = batch.offsets[s]
        path = os.path.join(tmpdir, f'{config}.{s:05d}', f'shard.{s:05d}.mds')
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, 'wb') as f:
            f.write(batch.buffer[o:o + batch.sizes[s]].cpu().numpy().tobytes())
        files.append((path, batch.samples[s]))
    meta = (plan.names, [c.encoding for c in plan.columns],
            [c.row_bytes if c.is_fixed else None for c in plan.columns])
    one = _cpu_leg(files, meta, 1, args.cpu_seconds)
    allc = _cpu_leg(files, meta, procs, args.cpu_seconds)
    return {
        'value': allc[0],
        'unit': 'samples/s',
        'gib_per_s': allc[1],
        'cores': procs,
        'kind': 'port',
        'one_core': {'value': one[0], 'unit': 'samples/s', 'gib_per_s': one[1]},
        'sample': (f'reference MDSReader.get_item restated (oracle ReferenceCostMDSReader: '
                   f'open/seek/read per sample, mds/reader.py:128-149; per-column coder built per '
                   f'call as _get_coder does, encodings.py:697-714,760-773) over full 64 MiB '
                   f'config-{config} shards of this workload copied to page-cached files: 1 '
                   f'process {one[2]} samples in {one[3]:.1f} s; {procs} processes '
                   f'(min(sched_getaffinity={aff}, box share OMP_NUM_THREADS={share or "unset"}))'
                   f', {allc[2]} samples in {allc[3]:.1f} s'),
    }


# ---------------------------------------------------------------------------------------------
# measurement
def src_sha() -> str:
    """sha256 (16 hex digits) of the sources the loaded libmdsx.so was built from (compiled into
    ``mdsx_version()`` by streaming_amd/build.py): profiles match on it."""
    from streaming_amd import _native
    version = _native.lib().mdsx_version().decode()
    return version.rsplit(' src ', 1)[1] if ' src ' in version else 'unknown'


def committed_traffic(key, kernel):
    """Per-launch HBM bytes of ``kernel`` on workload ``key`` from a committed rocprofv3 PMC
    summary (the L2's memory-side read and write requests by size, TCC_EA0_RDREQ_{32B,64B,128B}
    and TCC_EA0_WRREQ / _64B: scripts/pmc_summary.py), or (None, None) when no summary was taken
    on this exact workload, kernel and library sources."""
    build = src_sha()
    for path in sorted(glob.glob(os.path.join(HERE, 'profiles', 'r*', '**', 'pmc_*.json'),
                                 recursive=True), reverse=True):
        try:
            with open(path) as f:
                summ = json.load(f)
        except (OSError, ValueError):
            continue
        for e in summ.get('entries', []):
            if e.get('workload_key') == key and kernel and kernel in e.get('kernel', '') and \
                    e.get('src_sha') == build:
                return e.get('hbm_traffic_bytes_per_launch'), os.path.relpath(path, HERE)
    return None, None


COPY_VARIANTS = (1, 3, 4, 5, 6, 7, 8, 9, 10)  # include/mdsx.h mdsx_copy_probe_variant shapes


def copy_ceiling(batch, iters=10, dst=None):
    """The same-run copy ceiling: a read+write streaming copy of the batch's shard bytes in each
    probe shape (include/mdsx.h), interleaved launch by launch; the fastest shape's median (GB/s).
    ``dst``: the copy's destination (default: allocated here and freed)."""
    from streaming_amd import _native
    lib = _native.lib()
    src = batch.buffer
    if dst is None:
        dst = torch.empty_like(src)
    stream = torch.cuda.current_stream(src.device)
    ev = {v: [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(iters + 1)] for v in COPY_VARIANTS}
    for i in range(iters + 1):
        for v in COPY_VARIANTS:
            ev[v][i][0].record(stream)
            rc = lib.mdsx_copy_probe_variant(src.data_ptr(), dst.data_ptr(), src.numel(), v,
                                             stream.cuda_stream)
            ev[v][i][1].record(stream)
            if rc != 0:
                raise RuntimeError(f'mdsx_copy_probe failed: {lib.mdsx_last_error().decode()}')
    torch.cuda.synchronize(src.device)
    if not torch.equal(src[-4096:], dst[-4096:]):
        raise RuntimeError('mdsx_copy_probe: copy mismatch')
    ms = {v: float(np.median([a.elapsed_time(b) for a, b in ev[v][1:]])) for v in COPY_VARIANTS}
    best = min(ms, key=ms.get)
    del dst
    return {'GBps': 2 * src.numel() / ms[best] / 1e6, 'ms': ms[best], 'variant': best,
            'GBps_by_variant': {str(v): 2 * src.numel() / t / 1e6 for v, t in ms.items()},
            'bytes_per_launch': 2 * src.numel()}


BLOCKS = 3  # the K timed steps of each config, split into blocks interleaved across configs


class Leg:
    """One config's workload, decoder and timing records (built, checked and warmed up by
    :func:`prepare`; timed block by block by :func:`timed_block`)."""


def prepare(args, config, world, rank, dev):
    """Build this rank's workload, decode it once, verify it against its sources, warm up."""
    from streaming_amd import _native
    from streaming_amd.decoder import BatchDecoder, ScanAheadDecoder, output_bytes
    leg = Leg()
    leg.config = config
    leg.mine, leg.total_shards = shard_plan(args, config, rank, world)
    leg.synth, leg.desc = build_workload(config, leg.mine)
    plan, batch = leg.synth.plan, leg.synth.batch
    # --scan-ahead (ragged plans): each step's scan pass (pass 1) on a side stream beside the
    # previous step's decode (ScanAheadDecoder), outputs sized once from an exact two-pass decode
    leg.ahead = plan.num_var > 0 and not args.single and args.scan_ahead
    if leg.ahead:
        first = BatchDecoder(plan, batch)
        out = first.run()
        first.check()
        leg.kernel = _native.last_kernel()
        caps = first.capacities
        if not args.no_verify:
            verify(config, out, leg.synth.sources)
        del first, out
        leg.dec = ScanAheadDecoder(plan, batch, capacities=caps)
        out = leg.dec.run(ahead=False)
    else:
        leg.dec = BatchDecoder(plan, batch, single=args.single)
        out = leg.dec.run()
        leg.kernel = _native.last_kernel()
    leg.dec.check()
    if not args.no_verify:
        verify(config, out, leg.synth.sources)
    for k in range(args.warmup):
        step(leg, k, args.warmup, None)
    # the copy probe's destination, allocated (and the probe run once) before any timed block: a
    # large allocation made between blocks slowed the next config's first block by 9-12 %
    # (profiles/r05/final)
    leg.copy_dst = torch.empty_like(batch.buffer) if args.copy_probe else None
    if args.copy_probe:
        copy_ceiling(batch, iters=1, dst=leg.copy_dst)
    torch.cuda.synchronize(dev)
    leg.R = batch.shard_bytes
    leg.W = output_bytes(plan, leg.dec.result())
    leg.blocks = []
    leg.decode_ms, leg.scan_ms = [], []
    return leg


def step(leg, k, n, ev):
    """Step k of n: scan + decode of the batch (scan-ahead: this step's decode and, unless it
    is the block's last step, the next step's scan beside it). ``ev``: timing events."""
    if leg.ahead:
        leg.dec.run(ahead=k + 1 < n, events=ev)
    else:
        leg.dec.run(ev)


REWARM = 2  # untimed steps before each block: the other config's block left this one's buffers cold


def timed_block(args, leg, nsteps, world, dev):
    """``nsteps`` steps between barrier + synchronize on both sides, after REWARM untimed ones
    (interleaved with the other config's block and copy probe, a block's first launches ran 1-9 %
    slower: profiles/r05/final); the same-run copy ceiling right after them."""
    from streaming_amd.distributed import max_over_ranks
    for k in range(REWARM):
        step(leg, k, REWARM, None)
    nev = 4 if leg.ahead else 3
    events = [[torch.cuda.Event(enable_timing=True) for _ in range(nev)] for _ in range(nsteps)]
    span = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    stream = torch.cuda.current_stream(dev)  # the stream the decode kernels are launched on
    barrier(world)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    span[0].record(stream)
    for k in range(nsteps):
        step(leg, k, nsteps, events[k])
    span[1].record(stream)
    torch.cuda.synchronize(dev)
    barrier(world)
    t1 = time.perf_counter()
    elapsed = max_over_ranks(t1 - t0, device=dev)
    assert stream == torch.cuda.current_stream(dev)
    if leg.ahead:
        dec_ms = [e[0].elapsed_time(e[1]) for e in events]
        scan_ms = [e[2].elapsed_time(e[3]) for e in events[:-1]]
    else:
        dec_ms = [e[1].elapsed_time(e[2]) for e in events]
        scan_ms = [e[0].elapsed_time(e[1]) for e in events]
    leg.decode_ms += dec_ms
    leg.scan_ms += scan_ms
    copy = copy_ceiling(leg.synth.batch, dst=leg.copy_dst) if args.copy_probe else None
    kern = float(np.mean(dec_ms))
    achieved = (leg.R + leg.W) / kern / 1e6
    leg.blocks.append({
        'steps': nsteps,
        'elapsed_s': elapsed,
        'ms_per_step': elapsed / nsteps * 1e3,
        'kernel_ms': kern,
        'frac': achieved / HBM_PEAK_GBS,
        'step_ms_events': span[0].elapsed_time(span[1]) / nsteps,
        'step_frac': (leg.R + leg.W) / (span[0].elapsed_time(span[1]) / nsteps) / 1e6 /
                     HBM_PEAK_GBS,
        'copy_ceiling_GBps': copy['GBps'] if copy else None,
        'frac_of_same_run_copy': achieved / copy['GBps'] if copy else None,
        '_copy': copy,
    })


def rank_record(rank, leg_rows, shards, shard_ids, elapsed_s, K, blocks, R, W, decode_ms):
    """What one rank reports for the line's ``per_rank`` list: its step time, its decode kernel's
    time and fraction of the HBM peak, its step fraction and its own same-run copy ceiling (so an
    N-GPU line tells a slow rank from a slow box)."""
    kern_ms = float(np.mean(decode_ms)) if len(decode_ms) else None
    step_ms = (sum(b['step_ms_events'] * b['steps'] for b in blocks) / K) if blocks else None
    copies = [b['copy_ceiling_GBps'] for b in blocks if b.get('copy_ceiling_GBps')]
    achieved = (R + W) / kern_ms / 1e6 if kern_ms else None
    copy = float(np.median(copies)) if copies else None
    return {
        'rank': rank, 'ms_per_step': elapsed_s / K * 1e3, 'rows': leg_rows, 'shards': shards,
        'shard_ids': shard_ids,
        'kernel_ms': kern_ms,
        'frac': achieved / HBM_PEAK_GBS if achieved else None,
        'step_frac': (R + W) / step_ms / 1e6 / HBM_PEAK_GBS if step_ms else None,
        'copy_ceiling_GBps': copy,
        'frac_of_same_run_copy': achieved / copy if achieved and copy else None,
    }


def aggregate_ranks(per_rank):
    """min / median / max over the ranks of each per-rank figure, and the slowest rank."""
    out = {}
    for k in ('ms_per_step', 'kernel_ms', 'frac', 'step_frac', 'copy_ceiling_GBps',
              'frac_of_same_run_copy'):
        xs = [p[k] for p in per_rank if p.get(k) is not None]
        if xs:
            out[k] = {'min': float(np.min(xs)), 'median': float(np.median(xs)),
                      'max': float(np.max(xs))}
    out['slowest_rank'] = max(per_rank, key=lambda p: p['ms_per_step'])['rank']
    out['ranks'] = len(per_rank)
    return out


def block_sizes(k, n=BLOCKS):
    """K steps split into at most n blocks (sizes differ by at most one)."""
    n = max(1, min(n, k))
    return [k // n + (1 if i < k % n else 0) for i in range(n)]


def finish(args, leg, world, rank, tmpdir):
    """The config's result object from its blocks (+ the CPU baseline on rank 0)."""
    config, batch, plan = leg.config, leg.synth.batch, leg.synth.plan
    leg.dec.check()
    if leg.ahead:
        leg.dec.close()
    if not args.no_verify:
        verify(config, leg.dec.result(), leg.synth.sources)
    K = sum(b['steps'] for b in leg.blocks)
    elapsed = sum(b['elapsed_s'] for b in leg.blocks)
    rows = batch.total_rows
    per_rank = gather_objects(world, rank_record(
        rank, rows, len(leg.mine), f'{leg.mine[0]}..{leg.mine[-1]} step {world}' if leg.mine else '',
        elapsed, K, leg.blocks, leg.R, leg.W, leg.decode_ms))
    all_rows = sum(p['rows'] for p in per_rank)
    R, W = leg.R, leg.W
    kern_s = float(np.mean(leg.decode_ms)) / 1e3
    achieved = (R + W) / kern_s / 1e9
    step_s = sum(b['step_ms_events'] * b['steps'] for b in leg.blocks) / K / 1e3
    copies = [b['_copy'] for b in leg.blocks if b['_copy']]
    ratios = [b['frac_of_same_run_copy'] for b in leg.blocks if b['frac_of_same_run_copy']]
    copy = None
    if copies:  # the block whose copy ceiling is the median one, with every shape's rate
        copy = sorted(copies, key=lambda c: c['GBps'])[len(copies) // 2]
    key = workload_key(config, batch, W)
    traffic, traffic_src = committed_traffic(key, leg.kernel)
    spb = [b['ms_per_step'] for b in leg.blocks]
    blocks = [{k: v for k, v in b.items() if not k.startswith('_')} for b in leg.blocks]
    result = {
        'value': all_rows * K / elapsed,
        'unit': 'samples/s',
        'mds_gib_per_s': R * world * K / elapsed / 2**30,
        'ms_per_step': elapsed / K * 1e3,
        'ms_per_step_blocks': {'median': float(np.median(spb)), 'min': float(np.min(spb)),
                               'max': float(np.max(spb)), 'blocks': len(spb)},
        'blocks': blocks,
        'rewarm': REWARM,
        'config': {
            'workload': leg.desc,
            'workload_key': key,
            'samples_per_gpu': rows,
            'shards_per_gpu': batch.nshards,
            'shards_total': leg.total_shards,
            'shard_bytes_per_gpu': R,
            'output_bytes_per_gpu': W,
            'parallelism': f'{world} GPU(s), global shard g -> rank g % {world}, no data-path '
                           f'collectives',
            'blocks': (f'the K timed steps in {len(leg.blocks)} blocks interleaved with the other '
                       f'config\'s, each after {REWARM} untimed steps'),
            'step': ('scan pass of step k+1 on a side stream beside the decode of step k '
                     '(ScanAheadDecoder); both passes of every timed step inside the timed region'
                     if leg.ahead else 'scan pass then decode, one stream'),
        },
        'per_rank': per_rank,
        'per_rank_summary': aggregate_ranks(per_rank),
        'fresh_batch_ms_per_step': leg.fresh['fresh_batch_ms_per_step'] if leg.fresh else None,
        'fresh_batch': leg.fresh,
        'roofline': {
            'bound': 'hbm',
            'kernel': leg.kernel,
            'achieved': achieved,
            'peak': HBM_PEAK_GBS,
            'unit': 'GB/s',
            'frac': achieved / HBM_PEAK_GBS,
            'frac_blocks': [b['frac'] for b in leg.blocks],
            'traffic': traffic,
            'traffic_source': traffic_src,
            'src_sha': src_sha(),
            'algorithmic_bytes_per_launch': R + W,
            'algorithmic': {'R': R, 'W': W},
            'kernel_ms': kern_s * 1e3,
            'scan_ms': float(np.mean(leg.scan_ms)) if leg.scan_ms else 0.0,
            'scan_overlapped': leg.ahead,
            'step_frac': (R + W) / step_s / 1e9 / HBM_PEAK_GBS,
            'step_frac_blocks': [b['step_frac'] for b in leg.blocks],
            'frac_of_measured_copy': achieved / COPY_MEASURED_GBS,
            'frac_of_same_run_copy': float(np.median(ratios)) if ratios else None,
            'frac_of_same_run_copy_blocks': ratios,
            'copy_ceiling_same_run': copy,
        },
        'cpu_baseline': None,
    }
    # the reference reader restated, timed on rank 0's host cores at every N, after the GPU legs
    # (the other ranks wait for it at the next barrier, outside any timed region)
    if rank == 0 and args.cpu_seconds > 0:
        result['cpu_baseline'] = cpu_baseline(args, config, leg.synth, tmpdir)
    leg.dec = leg.synth = leg.copy_dst = None
    torch.cuda.empty_cache()
    return result


def fresh_batches(args, leg, world, dev):
    """Steps over TWO distinct resident batches of the config taken in turn (this rank's shards and
    as many other shards of the same workload, from their own seeds), each step with a decoder of
    its own, as a loader handed a new batch every step runs it: the two-pass decode pays the
    batch's sizing inside the step (scan pass, its totals read back to the host, the ragged outputs
    allocated, then the decode), the single-pass one allocates its ragged outputs at their upper
    bound and reads nothing back (``BatchDecoder(single=True)``). The headline's steps re-decode one
    batch whose outputs were sized once. Returns the ``fresh_batch`` object."""
    from streaming_amd.decoder import BatchDecoder, output_bytes
    from streaming_amd.distributed import max_over_ranks
    plan = leg.synth.plan
    synth2, _ = build_workload(leg.config, [g + leg.total_shards for g in leg.mine])
    pairs = [(leg.synth.batch, leg.synth.sources), (synth2.batch, synth2.sources)]
    rw = []
    for b, src in pairs:  # each batch decoded and checked once
        d = BatchDecoder(plan, b)
        out = d.run()
        d.check()
        verify(leg.config, out, src)
        rw.append(b.shard_bytes + output_bytes(plan, out))
        del d, out
    res = {'steps': args.fresh_steps,
           'batches': (f'2 distinct resident batches of {leg.synth.batch.nshards} shards, '
                       f'taken in turn; a new decoder per step (outputs from torch\'s caching '
                       f'allocator)'),
           'algorithmic_bytes_per_step': float(np.mean(rw))}
    for mode, single in (('two_pass', False), ('single_pass', True)):
        for k in range(2):  # warm: the allocator's pool holds both batches' outputs
            BatchDecoder(plan, pairs[k][0], single=single).run()
        barrier(world)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for k in range(args.fresh_steps):
            d = BatchDecoder(plan, pairs[k % 2][0], single=single)
            out = d.run()
        torch.cuda.synchronize(dev)
        barrier(world)
        elapsed = max_over_ranks(time.perf_counter() - t0, device=dev)
        d.check()
        if not args.no_verify:
            verify(leg.config, out, pairs[(args.fresh_steps - 1) % 2][1])
        del d, out
        ms = elapsed / args.fresh_steps * 1e3
        res[mode] = {'ms_per_step': ms, 'step_frac': float(np.mean(rw)) / ms / 1e6 / HBM_PEAK_GBS,
                     'samples_per_s': leg.synth.batch.total_rows * world / (ms / 1e3)}
    res['fresh_batch_ms_per_step'] = res['two_pass']['ms_per_step']
    del synth2, pairs
    torch.cuda.empty_cache()
    return res


def measure_all(args, configs, world, rank, dev, tmpdir):
    """Every config prepared, then BLOCKS timed blocks per config, interleaved (B1 C1 B2 C2 B3
    C3): each config's K steps are timed in blocks that fall on the same GPU phases."""
    legs = {c: prepare(args, c, world, rank, dev) for c in configs}
    for n in block_sizes(args.steps):
        for c in configs:
            timed_block(args, legs[c], n, world, dev)
    for c in configs:  # after every timed block of every config
        legs[c].fresh = fresh_batches(args, legs[c], world, dev) if (
            args.fresh_steps > 0 and legs[c].synth.plan.num_var > 0 and not legs[c].ahead) else None
    return {c: finish(args, legs[c], world, rank, tmpdir) for c in configs}


def dry_run(args, world, rank):
    """No GPU: the launcher's ranks, their process group and shard ownership (CPU test hook)."""
    lines = {}
    for config in ('B', 'C') if args.config == 'BC' else (args.config, ):
        mine, total = shard_plan(args, config, rank, world)
        lines[config] = gather_objects(world, {'rank': rank, 'shards': mine, 'total': total})
    # the N-GPU line's per-rank report, from made-up timings (rank r: 1 + r/10 ms per step)
    ms = 1.0 + rank / 10
    blocks = [{'steps': 2, 'step_ms_events': ms, 'copy_ceiling_GBps': 6000.0 + rank}]
    rec = rank_record(rank, 1000, len(mine), '', ms * 2e-3, 2, blocks, 4e9, 4e9, [ms * 0.9] * 2)
    per_rank = gather_objects(world, rec)
    barrier(world)
    if rank == 0:
        print(json.dumps({'dry_run': True, 'n_gpus': world, 'ownership': lines,
                          'per_rank': per_rank, 'per_rank_summary': aggregate_ranks(per_rank)}),
              flush=True)
    if _dist_on():
        torch.distributed.destroy_process_group()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    if args.gpus < 1:
        raise SystemExit('--gpus must be >= 1')
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        return launch(args, argv)  # before any GPU call in this process
    world, rank, local, dev = init_dist(args)
    if args.dry_run:
        dry_run(args, world, rank)
        return 0
    configs = ['B', 'C'] if args.config == 'BC' else [args.config]
    with tempfile.TemporaryDirectory(prefix='mdsx_cpu_') as tmpdir:
        results = measure_all(args, configs, world, rank, dev, tmpdir)
    head = results[configs[0]]
    if rank == 0:
        line = {
            'metric': METRIC,
            'value': head['value'],
            'unit': 'samples/s',
            'mds_gib_per_s': head['mds_gib_per_s'],
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': head['ms_per_step'],
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': 'u8',
            'data': 'synthetic (device-generated MDS shards, bit-identical to the reference '
                    'writer layout)',
            'parity': 'bit-exact vs encoded source columns' if not args.no_verify else 'skipped',
            'config': head['config'],
            'per_rank': head['per_rank'],
            'per_rank_summary': head['per_rank_summary'],
            'ms_per_step_blocks': head['ms_per_step_blocks'],
            'blocks': head['blocks'],
            'rewarm': head['rewarm'],
            # the timing barrier / max-over-ranks / report gather: a torch.distributed process
            # group ('nccl' = RCCL on ROCm) when one is up, else none (one process, no group)
            'process_group': (f'{torch.distributed.get_backend()}, {world} rank(s)'
                              if _dist_on() else None),
            'roofline': head['roofline'],
            'cpu_baseline': head['cpu_baseline'],
        }
        if 'C' in results and configs[0] != 'C':
            line['config_c'] = results['C']
        print(json.dumps(line), flush=True)
    if _dist_on():
        torch.distributed.destroy_process_group()
    return 0


if __name__ == '__main__':
    sys.exit(main())
