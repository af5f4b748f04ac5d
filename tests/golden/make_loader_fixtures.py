"""Record the REAL reference's multi-worker / multi-rank loader order on config A (build
container only).

    python tests/golden/make_loader_fixtures.py [--reference /root/reference]

The reference's usual setup is ``StreamingDataLoader(StreamingDataset(...), batch_size=B,
num_workers=W)`` in every rank: each DataLoader worker runs ``StreamingDataset.__iter__`` on its
own partition (``World.detect_workers``, ``streaming/base/world.py:150-163``; ``_get_work``,
``dataset.py:1012-1066``), torch interleaves the workers' batches, and the loader counts the
samples it hands out for ``state_dict`` (``dataloader.py:50-96``). For a few (shuffle, ranks,
workers) settings this script runs that setup in fresh subprocesses (one per rank, under
``RANK`` / ``WORLD_SIZE`` / ``LOCAL_WORLD_SIZE`` with a gloo rendezvous on 127.0.0.1 for two
ranks) and records, per rank:

* the sha256 of every sample the loader yields in epoch 0, in order (``int64 number`` + UTF-8
  ``words``, as ``make_order_fixtures.digest``), the sample count and the batch sizes;
* ``loader.state_dict()`` taken after ``resume_batches`` batches (mid-epoch), and then, in new
  processes, the same digest of a new loader after ``load_state_dict`` of that state;
* ``generate_work``'s ``[nodes, ranks per node, workers per rank, batches, batch]`` array for the
  setting's W-worker World, from the start and at the resumed ``sample_in_epoch`` -- the ids a
  one-process device iterator (``streaming_amd.plugin.device_iter(num_workers=W)``) lays out.

Output: ``tests/golden/order/loader.npz`` (ids) and ``tests/golden/order/loader.json``.
"""

from __future__ import annotations

import argparse
import hashlib
import json
import os
import shutil
import socket
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

# Two streams of config A's schema (config_a: 10 000 samples, config_a2: 3 000), each drawn by a
# proportion of the epoch (stream.py:92-140: config_a sub-sampled, config_a2 repeated).
TWO_STREAMS = [('config_a', {'proportion': 0.6}), ('config_a2', {'proportion': 0.4})]
_MS = dict(shuffle=True, shuffle_algo='py1e', shuffle_seed=23, num_canonical_nodes=2,
           batch_size=16, shuffle_block_size=1000)

SETTINGS = [
    # name, StreamingDataset kwargs, ranks (one node), DataLoader workers, resume after batches
    # [, streams: (golden dir, Stream kwargs) -- default the one local dir config_a]
    ('py1e_r1w2', dict(shuffle=True, shuffle_algo='py1e', shuffle_seed=17, num_canonical_nodes=2,
                       batch_size=16, shuffle_block_size=1000), 1, 2, 21),
    ('noshuffle_r1w3', dict(shuffle=False, num_canonical_nodes=1, batch_size=16), 1, 3, 10),
    ('py1s_r2w2', dict(shuffle=True, shuffle_algo='py1s', shuffle_seed=5, num_canonical_nodes=4,
                       batch_size=8, shuffle_block_size=2048), 2, 2, 25),
    # round 5: multi-stream datasets under every batching method (batching/__init__.py:21-26)
    ('ms_random_r1w2', dict(_MS, batching_method='random'), 1, 2, 15, TWO_STREAMS),
    ('ms_stratified_r1w2', dict(_MS, batching_method='stratified'), 1, 2, 12, TWO_STREAMS),
    ('ms_per_stream_r1w2', dict(_MS, batching_method='per_stream'), 1, 2, 10, TWO_STREAMS),
    ('ms_device_per_stream_r2w2', dict(_MS, batching_method='device_per_stream', batch_size=8),
     2, 2, 20, TWO_STREAMS),
    # replication: two ranks see the same samples (dataset.py:370-374, world.py:117-148)
    ('repl2_r2w2', dict(shuffle=True, shuffle_algo='py1s', shuffle_seed=5, num_canonical_nodes=2,
                        batch_size=8, shuffle_block_size=2048, replication=2), 2, 2, 25),
    ('ms_repl2_r2w2', dict(_MS, batching_method='per_stream', batch_size=8, replication=2), 2, 2,
     20, TWO_STREAMS),
]


def _free_port() -> int:
    """A free port below the kernel's ephemeral range (32768+), where no OS-assigned socket can
    take it before the reference's rank 0 binds its TCP store."""
    for port in range(24000 + 100 * (os.getpid() % 50), 32000):
        with socket.socket() as s:
            try:
                s.bind(('127.0.0.1', port))
            except OSError:
                continue
            return port
    raise RuntimeError('no free port')


def run_rank(spec: dict) -> None:
    """One rank of one phase (a subprocess): iterate the reference loader, write a JSON result."""
    from make_golden import boot_reference
    boot_reference(spec['reference'])
    from streaming.base.batching import generate_work
    from streaming.base.dataloader import StreamingDataLoader
    from streaming.base.dataset import StreamingDataset
    from streaming.base.stream import Stream
    from streaming.base.util import clean_stale_shared_memory
    from streaming.base.world import World

    rank, ranks, workers = spec['rank'], spec['ranks'], spec['workers']
    clean_stale_shared_memory()
    if spec['streams']:
        streams = [Stream(local=os.path.join(spec['local'], d), **kw) for d, kw in spec['streams']]
        ds = StreamingDataset(streams=streams, **spec['kwargs'])
    else:
        ds = StreamingDataset(local=spec['local'], **spec['kwargs'])
    bs = spec['kwargs']['batch_size']
    loader = StreamingDataLoader(ds, batch_size=bs, num_workers=workers)
    if spec['state'] is not None:
        loader.load_state_dict(spec['state'])
    h = hashlib.sha256()
    sizes, state = [], None
    for batch in loader:
        for n, w in zip(batch['number'].tolist(), batch['words']):
            h.update(np.int64(n).tobytes())
            h.update(w.encode('utf-8'))
        sizes.append(len(batch['words']))
        if spec['state'] is None and len(sizes) == spec['resume_batches']:
            state = loader.state_dict()
    epoch, sie = (0, 0) if spec['state'] is None else (spec['state']['epoch'],
                                                       spec['state']['sample_in_epoch'])
    # the partition World of this rank's W loader workers (replication: the replicated rank,
    # dataset.py:370-374), as device_iter lays it out (streaming_amd/plugin.py _loader_work)
    pw = ds._parallel_rank_world
    world = World(pw.num_nodes, pw.ranks_per_node, workers, pw.rank * workers)
    ids = generate_work(ds.batching_method, ds, world, epoch, sie)
    np.save(spec['ids_out'], ids.astype(np.int64), allow_pickle=False)
    with open(spec['out'], 'w') as f:
        json.dump({'sha256': h.hexdigest(), 'count': int(sum(sizes)), 'batch_sizes': sizes,
                   'state': state}, f)


def run_phase(args, name, kwargs, ranks, workers, resume_batches, local, state, work,
              streams=None):
    port = _free_port()
    procs, outs = [], []
    for rank in range(ranks):
        out = os.path.join(work, f'{name}.{rank}.{"resume" if state else "start"}.json')
        spec = {'reference': args.reference, 'rank': rank, 'ranks': ranks, 'workers': workers,
                'local': local, 'kwargs': kwargs, 'state': state, 'streams': streams,
                'resume_batches': resume_batches, 'out': out, 'ids_out': out + '.npy'}
        env = dict(os.environ, RANK=str(rank), WORLD_SIZE=str(ranks), LOCAL_RANK=str(rank),
                   LOCAL_WORLD_SIZE=str(ranks), MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port),
                   PYTHONDONTWRITEBYTECODE='1')
        procs.append(subprocess.Popen([sys.executable, __file__, '--rank-spec', json.dumps(spec)],
                                      env=env))
        outs.append(out)
    for p in procs:
        if p.wait(timeout=600) != 0:
            raise RuntimeError(f'{name}: a rank failed ({p.returncode})')
    res = []
    for out in outs:
        with open(out) as f:
            r = json.load(f)
        r['ids'] = np.load(out + '.npy', allow_pickle=False)
        res.append(r)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reference', default='/root/reference')
    ap.add_argument('--rank-spec', default=None)
    ap.add_argument('--only', default='', help='comma-separated settings to (re)record; the '
                    'others are kept from the existing fixture')
    args = ap.parse_args()
    if args.rank_spec:
        run_rank(json.loads(args.rank_spec))
        return
    out_dir = os.path.join(HERE, 'order')
    os.makedirs(out_dir, exist_ok=True)
    arrays, meta = {}, {'dataset': 'config_a', 'settings': []}
    only = set(filter(None, args.only.split(',')))
    if only:
        arrays = dict(np.load(os.path.join(out_dir, 'loader.npz'), allow_pickle=False))
        with open(os.path.join(out_dir, 'loader.json')) as f:
            meta = json.load(f)
        meta['settings'] = [e for e in meta['settings'] if e['name'] not in only]
        arrays = {k: v for k, v in arrays.items() if k.split('.')[0] not in only}
    work = tempfile.mkdtemp(prefix='loader_')
    try:
        for name, kwargs, ranks, workers, resume_batches, *rest in SETTINGS:
            if only and name not in only:
                continue
            streams = rest[0] if rest else None
            local = os.path.join(work, name)
            if streams:
                for d, _ in streams:
                    shutil.copytree(os.path.join(HERE, d), os.path.join(local, d))
            else:
                shutil.copytree(os.path.join(HERE, 'config_a'), local)
            start = run_phase(args, name, kwargs, ranks, workers, resume_batches, local, None,
                              work, streams)
            state = start[0]['state']
            assert all(r['state'] == state for r in start), [r['state'] for r in start]
            resumed = run_phase(args, name, kwargs, ranks, workers, resume_batches, local, state,
                                work, streams)
            entry = {'name': name, 'kwargs': kwargs, 'ranks': ranks, 'workers': workers,
                     'resume_batches': resume_batches, 'state_dict': state, 'per_rank': []}
            if streams:
                entry['streams'] = [{'dir': d, 'kwargs': kw} for d, kw in streams]
            for rank, (a, b) in enumerate(zip(start, resumed)):
                arrays[f'{name}.r{rank}.start'] = a['ids']
                arrays[f'{name}.r{rank}.resume'] = b['ids']
                entry['per_rank'].append({
                    'rank': rank, 'iter_start_sha256': a['sha256'], 'iter_start_count': a['count'],
                    'start_batch_sizes': a['batch_sizes'], 'iter_resume_sha256': b['sha256'],
                    'iter_resume_count': b['count'], 'resume_batch_sizes': b['batch_sizes']})
            meta['settings'].append(entry)
            print(name, state, [(r['count'], r['sha256'][:12]) for r in start + resumed],
                  flush=True)
    finally:
        shutil.rmtree(work, ignore_errors=True)
    order = [name for name, *_ in SETTINGS]
    meta['settings'].sort(key=lambda e: order.index(e['name']) if e['name'] in order else 99)
    np.savez_compressed(os.path.join(out_dir, 'loader.npz'), **arrays)
    with open(os.path.join(out_dir, 'loader.json'), 'w') as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
