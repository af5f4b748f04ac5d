"""Multi-process (gloo, CPU) coverage of :class:`streaming_amd.exchange.OwnedShardGather`: per-GPU
shard ownership with a cross-rank row exchange keeps every rank's batches in the reference's order
while each shard is decoded by one rank only.

This container has no GPU, so the per-rank gather is a host stand-in over the oracle's per-sample
reader (``oracle/mds_oracle.py``, the reference's algorithm): the exchange protocol -- the request
all-gather, the failure agreement, the all-to-all of fixed bytes, ragged lengths / values / UTF-8
flags, and the reorder -- runs as on the GPU, with torch CPU ops in place of the device gather
kernels. The GPU tests (``tests/test_device_exchange.py``) run the same exchange over the HIP
decode and gather on two ranks sharing one MI355X.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import mds_oracle
from streaming_amd.decoder import DecodedBatch, RaggedColumn
from streaming_amd.synth import var_c_shards

NAMES, ENCS, SIZES = ['b', 'n', 's'], ['bytes', 'int', 'str'], [None, 8, None]


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


class _Shard:
    def __init__(self, samples):
        self.samples = samples

    def _filename(self):
        return __file__  # (exists: nothing to prepare)


class HostGather:
    """Stand-in for DeviceSampleGather on the host: the oracle's columns of each shard, decoded
    on first use (recorded in ``decoded``), rows gathered in the order asked. ``poison``: global
    ids whose gather raises IndexError (a malformed sample)."""

    def __init__(self, shards, counts, poison=()):
        self.data = shards
        self.shards = [_Shard(c) for c in counts]
        self.starts = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        self.decoded = set()
        self.cols = {}
        self.poison = set(poison)

    def locate(self, ids):
        ids = np.asarray(ids, np.int64)
        shard = np.searchsorted(self.starts, ids, side='right') - 1
        return shard, ids - self.starts[shard]

    def _decoded(self, g):
        if g not in self.cols:
            info = {'raw_data': {'basename': ''}, 'column_names': NAMES,
                    'column_encodings': ENCS, 'column_sizes': SIZES,
                    'samples': self.shards[g].samples}
            self.cols[g] = mds_oracle.decode_shard_columns(None, None, info, data=self.data[g])
            self.decoded.add(g)
        return self.cols[g]

    def gather(self, ids):
        ids = np.asarray(ids, np.int64)
        if self.poison & set(ids.tolist()):
            raise IndexError('Relative sample index is not present (poisoned id)')
        shard, local = self.locate(ids)
        cols = {}
        for name in NAMES:
            parts = [self._decoded(int(g))[name] for g in shard]
            if parts and parts[0][0] == 'fixed':
                rows = np.stack([p[1][i] for p, i in zip(parts, local)]) if len(ids) else \
                    np.zeros((0, 8), np.uint8)
                cols[name] = torch.from_numpy(rows.copy()).view(torch.int64).reshape(-1)
            else:
                vals = [p[1][p[2][i]:p[2][i + 1]] for p, i in zip(parts, local)]
                lens = np.array([v.size for v in vals], np.int64)
                offs = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
                flags = np.array([p[3][i] for p, i in zip(parts, local)], np.uint8) \
                    if parts and parts[0][3] is not None else np.zeros(len(ids), np.uint8)
                cols[name] = RaggedColumn(
                    torch.from_numpy(np.concatenate(vals) if vals else np.zeros(0, np.uint8)),
                    torch.from_numpy(offs), torch.from_numpy(flags) if name == 's' else None)
        return DecodedBatch(cols, len(ids))


def host_gather_sources(sources, src, rows, check=True):
    """gather_sources on host tensors (the test's stand-in for the mdsx_gather kernels)."""
    src = np.asarray(src, np.int64)
    rows = np.asarray(rows, np.int64)
    cols = {}
    for name, first in sources[0].columns.items():
        if isinstance(first, RaggedColumn):
            vals, lens, flags = [], [], []
            for s, r in zip(src, rows):
                c = sources[int(s)].columns[name]
                lo, hi = int(c.offsets[r]), int(c.offsets[r + 1])
                vals.append(c.values[lo:hi])
                lens.append(hi - lo)
                if c.flags is not None:
                    flags.append(c.flags[r:r + 1])
            offs = torch.zeros(len(lens) + 1, dtype=torch.int64)
            offs[1:] = torch.cumsum(torch.tensor(lens, dtype=torch.int64), 0)
            cols[name] = RaggedColumn(torch.cat(vals) if vals else first.values[:0], offs,
                                      torch.cat(flags) if flags else (
                                          first.flags[:0] if first.flags is not None else None))
        else:
            cols[name] = torch.stack([sources[int(s)].columns[name][int(r)]
                                      for s, r in zip(src, rows)]) if len(src) else first[:0]
    return DecodedBatch(cols, len(src))


def _same(a, b):
    assert a.rows == b.rows
    for name in NAMES:
        x, y = a.columns[name], b.columns[name]
        if isinstance(x, RaggedColumn):
            assert torch.equal(x.offsets, y.offsets), name
            assert torch.equal(x.values, y.values), name
            if x.flags is not None:
                assert torch.equal(x.flags, y.flags), name
        else:
            assert torch.equal(x, y), name


def _worker(rank, world, port, q, steps, capacity, poison_step):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import streaming_amd.exchange as ex
        ex.gather_sources = host_gather_sources  # (module global: the device gather stand-in)
        shards, counts, _ = var_c_shards(3000, seed=71, size_limit=1 << 17, str_chars=(0, 40),
                                         blob_bytes=(0, 300))
        starts = np.concatenate([[0], np.cumsum(counts)])
        poison = {int(starts[1] + 3)}  # shard 1: rank 1's when world is 2 or 3
        local = HostGather(shards, counts, poison=poison)
        full = HostGather(shards, counts)  # the batch every rank would gather alone
        og = ex.OwnedShardGather(local, capacity, group=None)
        results = []
        for k, ids in enumerate(steps[rank]):
            if k == poison_step:
                ids = list(ids[:-1]) + [int(starts[1] + 3)] if rank == 0 else ids
                try:
                    og.gather(ids)
                    results.append('no error')
                except IndexError:
                    results.append('IndexError')
                continue
            got = og.gather(ids)
            want = full.gather(np.asarray([i for i in ids if i != -1], np.int64))
            _same(got, want)
            results.append('ok')
        og.drain()  # (rank 0 runs out of batches first: it serves the others meanwhile)
        q.put((rank, results, sorted(local.decoded), og.owned(), len(counts)))
    finally:
        dist.destroy_process_group()


def _steps(world, nsteps, capacity, total, seed, avoid):
    """Random ids per rank and step (never ``avoid``: the poisoned id is asked for once)."""
    rng = np.random.default_rng(seed)
    out = []
    for r in range(world):
        rs = []
        for k in range(nsteps - 2 if r == 0 else nsteps):  # (rank 0: two batches fewer)
            n = int(rng.integers(1, capacity + 1)) if k != 2 else capacity
            ids = [i if i != avoid else i + 1 for i in rng.integers(0, total, n).tolist()]
            if k == 1:  # padding ids (-1) as the reference's partition leaves them
                ids[::5] = [-1] * len(ids[::5])
            rs.append(ids)
        out.append(rs)
    return out


@pytest.mark.parametrize('world', [2, 3])
def test_exchange_matches_local_gather(world):
    """Random batches (repeats, padding, every shard) on every rank: each rank's exchanged batch
    equals what it would gather alone; each shard is decoded by its owner only; a malformed sample
    in a shard one rank owns, asked for by another, raises on every rank (no rank left waiting in a
    collective), and the steps after it still exchange; a rank with fewer batches serves the
    others' requests (drain) until every rank is out."""
    shards, counts, _ = var_c_shards(3000, seed=71, size_limit=1 << 17, str_chars=(0, 40),
                                     blob_bytes=(0, 300))
    total = int(sum(counts))
    capacity, nsteps, poison_step = 48, 7, 3
    steps = _steps(world, nsteps, capacity, total, seed=world, avoid=int(counts[0]) + 3)
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, steps, capacity, poison_step))
             for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nshards = results[0][4]
    assert nshards >= 2 * world  # several shards per rank
    decoded_by = {}
    for rank, res, decoded, owned, _ in results:
        assert res[poison_step] == 'IndexError', (rank, res)
        assert all(x == 'ok' for i, x in enumerate(res) if i != poison_step), (rank, res)
        assert set(decoded) <= set(owned), (rank, decoded, owned)
        for g in decoded:
            decoded_by.setdefault(g, []).append(rank)
    assert all(len(v) == 1 for v in decoded_by.values())  # every shard decoded once
    assert len(decoded_by) > nshards // 2  # (the batches touched most shards)
