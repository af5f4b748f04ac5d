"""GPU parity of device_iter with the cross-rank exchange (``exchange=True``,
:class:`streaming_amd.exchange.OwnedShardGather`): two ranks, each decoding only the shards it
owns through the HIP decode and gathering each batch's rows from the owners, must still yield on
each rank the samples and batch sizes the REAL reference's ``StreamingDataLoader(num_workers=W)``
yielded there (``tests/golden/order/loader.json``, the digests ``test_device_plugin_iter`` checks
without the exchange) -- including the setting where the ranks get different numbers of batches
(``device_per_stream``: 813 and 812) and with ``replication=2`` (both ranks ask for the same rows).

The two ranks share the box's one MI355X over ``gloo`` (host-staged collectives; RCCL needs a GPU
per rank); the decode, the owners' gathers and the final reorder run the mdsx kernels.
"""

import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

CASES = ['py1s_r2w2', 'repl2_r2w2', 'ms_device_per_stream_r2w2', 'ms_repl2_r2w2']


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _rank(rank, world, port, name, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from streaming_amd.exchange import OwnedShardGather
        from streaming_amd.local import LocalDataset
        from streaming_amd.order import DeviceSampleGather
        from streaming_amd.plugin import device_iter
        from tests import golden_util as gu
        from tests.test_device_plugin_iter import _rows
        from tests.test_order import digest
        from tests.test_plugin_iter import _standin, loader_settings, stream_dirs
        st = loader_settings()[name]
        pr = st['per_rank'][rank]
        bs, W = st['kwargs']['batch_size'], st['workers']
        shards = []
        for d in stream_dirs(st):
            shards += LocalDataset(gu.GOLDEN + '/' + d, decoded_cache_bytes=1 << 20).shards
        og = OwnedShardGather(DeviceSampleGather(shards), bs)
        standin = _standin(name, rank, shards)
        numbers, words, sizes = _rows(device_iter(standin, bs, num_workers=W, gather=og))
        torch.cuda.synchronize()
        q.put((rank, sizes == pr['start_batch_sizes'],
               digest(numbers, words) == pr['iter_start_sha256'], sorted(og.decoded_shards),
               og.owned(), len(shards), None))
    except Exception as e:  # (reported, not left to the timeout)
        q.put((rank, False, False, [], [], 0, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('name', CASES)
def test_device_iter_exchange_matches_reference_loader(name):
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, name, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        results = sorted(q.get(timeout=150) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    decoded_by = {}
    for rank, sizes_ok, digest_ok, decoded, owned, nshards, err in results:
        assert err is None, (rank, err)
        assert sizes_ok and digest_ok, (name, rank)
        assert set(decoded) <= set(owned), (rank, decoded, owned)
        for g in decoded:
            decoded_by.setdefault(g, []).append(rank)
    assert all(len(v) == 1 for v in decoded_by.values())  # each shard decoded by one rank
    assert len(decoded_by) >= 2


def _rank_direct(rank, world, port, q):
    import numpy as np
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        from streaming_amd.decoder import RaggedColumn
        from streaming_amd.exchange import OwnedShardGather
        from streaming_amd.local import LocalDataset
        from streaming_amd.order import DeviceSampleGather
        from tests import golden_util as gu
        shards = LocalDataset(gu.GOLDEN + '/config_c_small', decoded_cache_bytes=1 << 24).shards
        alone = DeviceSampleGather(shards)
        # every shard owned by rank 0: rank 1 never sends (its empty columns come from the decode
        # of a shard of no samples), rank 0 serves every row both ask for
        og = OwnedShardGather(DeviceSampleGather(shards), 40, owner=lambda g: 0)
        rng = np.random.default_rng(rank)
        ok = True
        for step in range(5 if rank == 0 else 3):  # (rank 1 drains two steps early)
            ids = rng.integers(0, alone.num_samples, int(rng.integers(1, 41)))
            got, want = og.gather(ids), alone.gather(ids)
            for name, x in want.columns.items():
                y = got.columns[name]
                if isinstance(x, RaggedColumn):
                    ok = (ok and torch.equal(x.offsets, y.offsets) and
                          torch.equal(x.values, y.values))
                    if x.flags is not None:
                        ok = ok and torch.equal(x.flags, y.flags)
                else:
                    ok = ok and torch.equal(x, y)
        og.drain()
        torch.cuda.synchronize()
        q.put((rank, ok, sorted(og.decoded_shards), None))
    except Exception as e:
        q.put((rank, False, [], repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_exchange_rank_that_owns_nothing():
    """Two ranks, every shard owned by rank 0 (config C: ragged bytes and str columns and a fixed
    one): rank 1 decodes nothing and sends empty columns, both get the rows a gather alone gives,
    and rank 1 draining early still lets rank 0 finish."""
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need an MI355X (torch.cuda.is_available() is False)')
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_direct, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        results = sorted(q.get(timeout=150) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    (r0, ok0, dec0, e0), (r1, ok1, dec1, e1) = results
    assert e0 is None and e1 is None, (e0, e1)
    assert ok0 and ok1
    assert dec1 == [] and dec0
