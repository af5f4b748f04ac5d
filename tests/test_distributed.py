"""Multi-process (gloo, CPU) coverage of the N>1 path: per-rank shard ownership covers every
shard exactly once with imbalance <= 1; the ranks' owned shards, read with the oracle (CPU; this
container has no GPU) and put back in shard order, give the reference's ordered content digest of
config A (manifest.json ``content_sha256``, written by the real reference reader); and the
benchmark's max-over-ranks timing reduction."""

import hashlib
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import mds_oracle
from streaming_amd.distributed import max_over_ranks, owned_shards, sum_over_ranks
from tests import golden_util as gu


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        idx = gu.index('config_a')
        mine = owned_shards(len(idx['shards']), rank, world)
        d = os.path.join(gu.GOLDEN, 'config_a')
        samples = 0
        items = []
        for s in mine:
            r = mds_oracle.OracleMDSReader(d, None, idx['shards'][s])
            samples += len(r)
            items.extend((r.get_item(i)['number'], r.get_item(i)['words']) for i in range(len(r)))
        gathered = [None] * world
        dist.all_gather_object(gathered, (mine, samples, items))
        t = max_over_ranks(float(rank + 1))
        total = sum_over_ranks(float(samples))
        q.put((rank, gathered, t, total))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 4])
def test_per_rank_shard_ownership(world):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    idx = gu.index('config_a')
    n_shards = len(idx['shards'])
    for rank, gathered, t, total in results:
        assert t == float(world)  # max over ranks
        assert total == 10_000
        owned = [g[0] for g in gathered]
        flat = sorted(s for o in owned for s in o)
        assert flat == list(range(n_shards))
        sizes = [len(o) for o in owned]
        assert max(sizes) - min(sizes) <= 1
        # every rank's decoded numbers, re-ordered by shard, are the dataset in order
        by_shard = {}
        for o, g in zip(owned, gathered):
            pos = 0
            for s in o:
                n = idx['shards'][s]['samples']
                by_shard[s] = g[2][pos:pos + n]
                pos += n
        h = hashlib.sha256()
        count = 0
        for s in range(n_shards):
            for number, words in by_shard[s]:
                h.update(np.int64(number).tobytes())
                h.update(words.encode('utf-8'))
                count += 1
        assert count == 10_000
        assert h.hexdigest() == gu.manifest()['config_a']['content_sha256']


def test_owned_shards_rejects_bad_rank():
    with pytest.raises(ValueError):
        owned_shards(10, 3, 2)
