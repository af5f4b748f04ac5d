"""Record the REAL reference's sample order on the golden config A dataset (build container only).

    python tests/golden/make_order_fixtures.py [--reference /root/reference]

Boots mosaicml/streaming offline exactly as make_golden.py does (stub codec/registry modules, no
bytecode written into the reference tree) and, for a few (shuffle, num_canonical_nodes, world,
batch size) settings, builds a ``StreamingDataset(local=<copy of tests/golden/config_a>)`` and
records:

* ``generate_work`` (``streaming/base/batching/__init__.py:28-45``) -- the epoch's sample ids as
  the reference lays them out, ``[nodes, ranks per node, workers per rank, batches, batch]``
  with ``-1`` padding, for every (node, rank, worker) of the setting's World -- from the start
  of the epoch and resumed mid-epoch (``sample_in_epoch`` > 0, what ``state_dict`` /
  ``load_state_dict`` resume from, ``dataset.py:778-856``);
* for the single-worker settings, the reference's own ``__iter__`` (``dataset.py:1475-1513``)
  from the start and after ``load_state_dict`` of a mid-epoch ``state_dict``: the sha256 of its
  yielded samples in order (``int64 number`` + UTF-8 ``words``), which pins that the recorded
  ids, read through ``_each_sample_id``'s ``-1`` skip, ARE the reference's stream.

Output: ``tests/golden/order/config_a.npz`` (ids) and ``tests/golden/order/config_a.json``
(settings, digests). The GPU test ``tests/test_device_order.py`` gathers the recorded ids on the
device and must reproduce the reference's samples in order, bit-exact.
"""

from __future__ import annotations

import argparse
import hashlib
import json
import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

SETTINGS = [
    # name, StreamingDataset kwargs, (nodes, ranks per node, workers per rank), resume at
    ('noshuffle_w1', dict(shuffle=False, num_canonical_nodes=1, batch_size=16), (1, 1, 1), 160),
    ('py1e_w1', dict(shuffle=True, shuffle_algo='py1e', shuffle_seed=17, num_canonical_nodes=2,
                     batch_size=16, shuffle_block_size=1000), (1, 1, 1), 336),
    ('py1s_n1r2w2', dict(shuffle=True, shuffle_algo='py1s', shuffle_seed=5, num_canonical_nodes=4,
                         batch_size=8, shuffle_block_size=2048), (1, 2, 2), 800),
    ('py1br_n2r2w1', dict(shuffle=True, shuffle_algo='py1br', shuffle_seed=3,
                          num_canonical_nodes=2, batch_size=32, shuffle_block_size=2000),
     (2, 2, 1), 1024),
]


def digest(samples) -> str:
    h = hashlib.sha256()
    for s in samples:
        h.update(np.int64(s['number']).tobytes())
        h.update(s['words'].encode('utf-8'))
    return h.hexdigest()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reference', default='/root/reference')
    args = ap.parse_args()
    from make_golden import boot_reference
    boot_reference(args.reference)
    from streaming.base.batching import generate_work
    from streaming.base.dataset import StreamingDataset
    from streaming.base.util import clean_stale_shared_memory
    from streaming.base.world import World

    out_dir = os.path.join(HERE, 'order')
    os.makedirs(out_dir, exist_ok=True)
    arrays, meta = {}, {'dataset': 'config_a', 'settings': []}
    work = tempfile.mkdtemp(prefix='order_')
    try:
        for name, kwargs, (nodes, rpn, wpr), resume_at in SETTINGS:
            clean_stale_shared_memory()
            local = os.path.join(work, name)
            shutil.copytree(os.path.join(HERE, 'config_a'), local)
            ds = StreamingDataset(local=local, **kwargs)
            entry = {'name': name, 'kwargs': kwargs, 'world': [nodes, rpn, wpr],
                     'resume_at': resume_at, 'epoch_size': int(ds.epoch_size)}
            for tag, sie in (('start', 0), ('resume', resume_at)):
                world = World(nodes, rpn, wpr, 0)
                ids = generate_work(ds.batching_method, ds, world, 0, sie)
                assert ids.shape[:3] == (nodes, rpn, wpr), ids.shape
                arrays[f'{name}.{tag}'] = ids.astype(np.int64)
                entry[f'{tag}_shape'] = list(ids.shape)
            if (nodes, rpn, wpr) == (1, 1, 1):
                samples = list(ds)  # the reference's own __iter__, epoch 0
                entry['iter_start_sha256'] = digest(samples)
                entry['iter_start_count'] = len(samples)
                state = ds.state_dict(num_samples=resume_at, from_beginning=True)
                del ds
                clean_stale_shared_memory()
                ds2 = StreamingDataset(local=local, **kwargs)
                ds2.load_state_dict(state)
                resumed = list(ds2)
                entry['state_dict'] = state
                entry['iter_resume_sha256'] = digest(resumed)
                entry['iter_resume_count'] = len(resumed)
                del ds2
            else:
                del ds
            meta['settings'].append(entry)
            print(name, {k: v for k, v in entry.items() if 'sha' in k or 'shape' in k}, flush=True)
    finally:
        clean_stale_shared_memory()
        shutil.rmtree(work, ignore_errors=True)
    np.savez_compressed(os.path.join(out_dir, 'config_a.npz'), **arrays)
    with open(os.path.join(out_dir, 'config_a.json'), 'w') as f:
        json.dump(meta, f, indent=1, sort_keys=True)


if __name__ == '__main__':
    main()
