"""Drop-in plugin for mosaicml/streaming's ``StreamingDataset``.

Two entry points:

* :func:`register_device_stream` -- the reader: every MDS shard of
  ``StreamingDataset(stream_name='mdsx')`` decodes on the GPU (per-sample ``__getitem__`` /
  ``__iter__`` keep the reference's host values);
* :func:`device_iter` / :class:`DeviceBatches` -- the iteration: ``StreamingDataset.__iter__``'s
  own control flow (epoch / resumption, this worker's ids from ``generate_work``, the prepare and
  ready threads, ``-1`` skipped) yielding device batches of the reference's samples in the
  reference's order, in place of ``map(__getitem__, ...)`` + ``default_collate``.

``StreamingDataset(stream_name=..., stream_config=...)`` builds its streams through the public
``streams_registry`` (``streaming/base/stream.py:515-522``, used at
``streaming/base/dataset.py:447-468``). :func:`make_device_stream` derives a ``Stream`` class whose
``get_shards`` (``stream.py:428-484``: index download/parse, ``reader_from_json``, ``validate``) is
the reference's own, with each MDS reader swapped for :class:`streaming_amd.reader.MDSReader`
(same ``Reader`` interface; samples decoded on the GPU a whole shard at a time). Readers of other
formats (JSONL, CSV) are returned unchanged.
"""

from __future__ import annotations

import os
import sys
from bisect import bisect_right
from concurrent.futures import ThreadPoolExecutor, wait
from threading import Event
from time import time_ns
from typing import Any, Callable, Iterator, Optional, Union

import numpy as np
import torch

from streaming_amd.decoder import DecodedBatch
from streaming_amd.reader import FileInfo, MDSReader

__all__ = ['to_device_reader', 'make_device_stream', 'register_device_stream', 'device_iter',
           'DeviceBatches']


def _file_info(f: Any) -> Optional[FileInfo]:
    if f is None:
        return None
    return FileInfo(f.basename, f.bytes, dict(f.hashes))


def to_device_reader(reader: Any, device: Union[str, torch.device, None] = None) -> Any:
    """The device-backed equivalent of a reference ``MDSReader`` (other readers unchanged)."""
    if isinstance(reader, MDSReader) or getattr(reader, 'column_encodings', None) is None:
        return reader
    return MDSReader(dirname=reader.dirname,
                     split=reader.split or None,
                     column_encodings=list(reader.column_encodings),
                     column_names=list(reader.column_names),
                     column_sizes=list(reader.column_sizes),
                     compression=reader.compression,
                     hashes=list(reader.hashes),
                     raw_data=_file_info(reader.raw_data),
                     samples=reader.samples,
                     size_limit=reader.size_limit,
                     zip_data=_file_info(reader.zip_data),
                     device=device)


def make_device_stream(stream_base: type, device: Union[str, torch.device, None] = None) -> type:
    """A subclass of the reference ``Stream`` whose shards decode on the GPU."""

    class DeviceStream(stream_base):  # type: ignore[misc, valid-type]
        """``Stream`` with MI355X-decoded MDS shards (``streaming_amd``)."""

        def get_shards(self, world: Any, allow_unsafe_types: bool) -> list:
            shards = super().get_shards(world, allow_unsafe_types)
            return [to_device_reader(s, device) for s in shards]

    DeviceStream.__name__ = 'DeviceStream'
    DeviceStream.__qualname__ = 'DeviceStream'
    return DeviceStream


def register_device_stream(name: str = 'mdsx',
                           device: Union[str, torch.device, None] = None) -> type:
    """Register the device stream in the reference's ``streams_registry`` under ``name``."""
    from streaming.base.stream import Stream, streams_registry  # the reference package
    cls = make_device_stream(Stream, device)
    streams_registry.register(name, func=cls)
    return cls


# What device_iter drives of StreamingDataset.__iter__ (dataset.py:1475-1513), by name. They are
# private to the reference; device_iter checks them up front against the installed version.
_ITER_METHODS = ('_resume_incr_epoch', '_prepare_thread', '_ready_thread', '_each_sample_id',
                 'on_exception', 'prepare_shard')
_ITER_STATE = ('_shard_access_times', '_unique_rank_world', '_parallel_rank_world')
_TESTED_REFERENCE = '0.14.0.dev0'  # mosaicml/streaming, streaming/_version.py:6


def _iteration_module(dataset: Any) -> Any:
    """The module that defines the dataset's iteration methods (any ``StreamingDataset``
    subclass, or a stand-in): it holds ``_Iterator``, ``generate_work`` and ``World``."""
    for klass in type(dataset).__mro__:
        if '_each_sample_id' in klass.__dict__:
            return sys.modules.get(klass.__module__)
    return None


def _require_iteration_surface(dataset: Any, num_workers: int) -> Any:
    """Check, before anything runs, that every private piece of ``StreamingDataset.__iter__``
    that :func:`device_iter` drives exists; one ``TypeError`` names all that are missing."""
    missing = [a for a in _ITER_METHODS if not callable(getattr(dataset, a, None))]
    missing += [a for a in _ITER_STATE if not hasattr(dataset, a)]
    if num_workers <= 1 and not callable(getattr(dataset, '_get_work', None)):
        missing.append('_get_work')
    mod = _iteration_module(dataset)
    needed = ['_Iterator'] + (['generate_work', 'World'] if num_workers > 1 else [])
    missing += [f'{getattr(mod, "__name__", "<module>")}.{n}' for n in needed
                if mod is None or not hasattr(mod, n)]
    if missing:
        top = sys.modules.get((getattr(mod, '__name__', '') or '').split('.')[0])
        version = getattr(top, '__version__', 'unknown')
        raise TypeError(f'device_iter: {type(dataset).__name__} lacks the StreamingDataset '
                        f'iteration internals it drives: {", ".join(missing)} (installed streaming '
                        f'{version}; device_iter follows mosaicml/streaming {_TESTED_REFERENCE})')
    return mod


def _gather_batch(dataset: Any, gather: Any, ids: list, retry: int) -> DecodedBatch:
    """The samples ``ids`` as one device batch, with ``StreamingDataset.get_item``'s contract
    (``dataset.py:1237-1293``): a background-thread failure stops the loop; a shard file found
    missing (``FileNotFoundError``, e.g. evicted meanwhile) is prepared again and the batch
    retried, up to ``retry`` times; the touched shards' access times are updated."""
    if hasattr(dataset, '_event') and dataset._event.is_set():
        raise RuntimeError('Background thread failed. Check other traceback.')
    ids = np.asarray(ids, np.int64)
    touched = np.unique(gather.locate(ids)[0])
    errors = []
    for _ in range(1 + retry):
        try:
            out = gather.gather(ids)
            break
        except FileNotFoundError as e:
            errors.append(str(e))
            for s in touched:
                if not os.path.exists(gather.shards[int(s)]._filename()):
                    dataset.prepare_shard(int(s))
    else:
        if hasattr(dataset, '_event'):
            dataset._event.set()
        if getattr(dataset, 'cache_limit', None):
            raise RuntimeError(f'{errors[-1]}. StreamingDataset repeatedly failed to download a '
                               f'shard. This may be due to thrashing caused by `cache_limit` '
                               f'being set too low.')
        raise RuntimeError(f'{errors[-1]}. Check if the shard file exists in your remote '
                           f'location or have you deleted the shard file from the local '
                           f'directory?')
    now = time_ns()
    for s in touched:
        dataset._shard_access_times[int(s)] = now
    if isinstance(out, DecodedBatch):
        out.sample_ids = ids
    return out


def device_iter(dataset: Any, batch_size: int, *, num_workers: int = 0, retry: int = 7,
                gather: Optional[Any] = None,
                exchange: Union[bool, Any, None] = None) -> Iterator[DecodedBatch]:
    """``StreamingDataset.__iter__`` (``dataset.py:1475-1513``) yielding DEVICE batches, in the
    order ``DataLoader(dataset, batch_size, num_workers=num_workers)`` yields them on this rank.

    The reference's own control flow, step for step: the previous epoch's iterator is exited,
    the worker world detected, the epoch incremented or resumed (``_resume_incr_epoch``: a
    ``load_state_dict`` checkpoint resumes mid-epoch, ``dataset.py:691-776``), the ids laid out
    (``_get_work`` / ``generate_work``, ``dataset.py:1012-1066``), and the ``_prepare_thread`` /
    ``_ready_thread`` started on the dataset's executor to download and ready shards ahead of the
    loop (``dataset.py:1313-1428``). The ids then come from ``_each_sample_id`` -- in order,
    ``-1`` skipped, each once its shard is ready -- and each batch's ids are gathered on the GPU
    from the shards' decoded columns (:class:`streaming_amd.order.DeviceSampleGather`: shards
    decoded on demand through the bounded decoded-shard cache, one launch sequence per column)
    instead of ``map(self.__getitem__, ...)`` and ``default_collate``. Each batch carries its
    ``sample_ids``.

    ``num_workers``: the loader being replaced. 0 or 1: this rank's one partition in batches of
    ``batch_size`` (the last may be short). W > 1: the W worker partitions of ``generate_work``
    for a World of W workers per rank (``world.py:150-163``), each cut into batches of its own,
    interleaved as torch's DataLoader returns them (:func:`streaming_amd.order.loader_batches`)
    -- all in this one process, which owns the GPU (the decode runs on the device; there is
    nothing for host workers to parallelise). Run it in every rank: under ``RANK`` /
    ``WORLD_SIZE`` each rank gets its own partition as with the reference.

    Checkpoints are ``StreamingDataLoader``'s (:class:`DeviceBatches`).

    The dataset's shards must be device readers (``stream_name='mdsx'``,
    :func:`register_device_stream`). ``gather``: what turns ids into a batch (default: a
    ``DeviceSampleGather`` over ``dataset.shards``); an object with ``gather(ids)``,
    ``locate(ids)`` and ``shards``.

    ``exchange``: ``True`` (the default process group) or a process group -- each shard is
    decoded by one rank of the group and every batch's rows are exchanged between the ranks
    (:class:`streaming_amd.exchange.OwnedShardGather`, RCCL ``all_to_all``), instead of every rank
    decoding every shard its batches touch. The batches are the same. Every rank of the group
    runs ``device_iter`` over the same epoch; a rank out of batches (or stopped early) keeps
    serving the others' requests until every rank is out.
    """
    if batch_size <= 0:
        raise ValueError('batch_size must be positive')
    ds = dataset
    workers = max(1, int(num_workers))
    mod = _require_iteration_surface(ds, workers)
    if gather is None:
        from streaming_amd.order import DeviceSampleGather
        bad = [i for i, s in enumerate(ds.shards) if not isinstance(s, MDSReader)]
        if bad:
            raise TypeError(f'device_iter: shard {bad[0]} is a {type(ds.shards[bad[0]]).__name__}, '
                            f'not a device reader (build the dataset with stream_name=\'mdsx\', '
                            f'streaming_amd.plugin.register_device_stream)')
        gather = DeviceSampleGather(ds.shards)
    if exchange:
        from streaming_amd.exchange import OwnedShardGather
        gather = OwnedShardGather(gather, batch_size, group=None if exchange is True else exchange,
                                  prepare=getattr(ds, 'prepare_shard', None))
    drain = getattr(gather, 'drain', None)
    try:
        yield from _device_iter(ds, mod, gather, batch_size, workers, retry)
    finally:
        if drain is not None:  # (every rank of the exchange group takes part until all are out)
            drain()


def _device_iter(ds: Any, mod: Any, gather: Any, batch_size: int, workers: int,
                 retry: int) -> Iterator[DecodedBatch]:
    # -- StreamingDataset.__iter__, dataset.py:1481-1510
    if hasattr(ds, '_iterator'):
        ds._iterator.exit()
    if not hasattr(ds, '_executor'):
        ds._executor = ThreadPoolExecutor()
    if not hasattr(ds, '_event'):
        ds._event = Event()
    elif ds._event.is_set():
        raise RuntimeError('Background thread failed. Check other traceback.')
    # this process is the rank's only iterating process: a one-worker world for the epoch
    # barrier of _resume_incr_epoch / _get_work
    ds._unique_worker_world = ds._unique_rank_world.detect_workers()
    ds._parallel_worker_world = ds._parallel_rank_world.detect_workers()
    epoch, sample_in_epoch = ds._resume_incr_epoch()
    if workers == 1:
        sample_ids = ds._get_work(epoch, sample_in_epoch)
        sizes = None
    else:
        sample_ids, sizes = _loader_work(ds, mod, workers, batch_size, epoch, sample_in_epoch)
    if not len(sample_ids):  # resumed at the end of the epoch: out of samples
        return
    ds._iterator = it = mod._Iterator(sample_ids)
    prepare_future = ds._executor.submit(ds._prepare_thread, it)
    prepare_future.add_done_callback(ds.on_exception)
    ready_future = ds._executor.submit(ds._ready_thread, it)
    ready_future.add_done_callback(ds.on_exception)
    # -- in place of `yield from map(self.__getitem__, self._each_sample_id(it))`
    stamp = _access_stamper(ds, gather)
    pending: list[int] = []
    k = 0
    want = sizes[0] if sizes else batch_size
    for sample_id in ds._each_sample_id(it):
        stamp(sample_id)  # get_item's access-time touch, as each sample is read (dataset.py:1270)
        pending.append(sample_id)
        if len(pending) == want:
            yield _gather_batch(ds, gather, pending, retry)
            pending = []
            k += 1
            want = sizes[k] if sizes and k < len(sizes) else batch_size
    if pending:
        yield _gather_batch(ds, gather, pending, retry)
    wait([prepare_future, ready_future], return_when='FIRST_EXCEPTION')
    it.exit()


def _loader_work(ds: Any, mod: Any, workers: int, batch_size: int, epoch: int,
                 sample_in_epoch: int) -> tuple[np.ndarray, list[int]]:
    """This rank's ids in a W-worker loader's order, and its batch sizes: ``generate_work``
    (what ``_get_work``'s local leader runs, ``dataset.py:1041-1052``) for a World of W workers
    per rank, then each worker's slice interleaved as the DataLoader returns them."""
    from streaming_amd.order import loader_batches
    if not isinstance(getattr(ds, 'batch_size', None), int):
        raise ValueError(f'Please pass `batch_size` to StreamingDataset. It should be ' +
                         f'set the same as the DataLoader, and is the number of samples ' +
                         f'per batch, for each device. It is necessary for ' +
                         f'deterministic resumption and optimal performance.')
    pw = ds._parallel_rank_world
    world = mod.World(num_nodes=pw.num_nodes, ranks_per_node=pw.ranks_per_node,
                      workers_per_rank=workers, worker=pw.rank * workers)
    epoch_ids = mod.generate_work(ds.batching_method, ds, world, epoch, sample_in_epoch)
    batches = loader_batches(epoch_ids, world.node, world.rank_of_node, workers, batch_size)
    ids = np.concatenate(batches) if batches else np.empty(0, np.int64)
    return ids, [len(b) for b in batches]


def _access_stamper(ds: Any, gather: Any) -> Callable[[int], None]:
    """Per sample id: stamp its shard's access time (``dataset.py:1270``) so the prepare
    thread's ``cache_limit`` eviction sees the shards of a pending batch as recently used."""
    times = ds._shard_access_times
    starts = getattr(gather, 'starts', None)
    if starts is not None:
        bounds = [int(x) for x in starts]

        def stamp(sid: int) -> None:
            times[bisect_right(bounds, sid) - 1] = time_ns()
    else:

        def stamp(sid: int) -> None:
            times[int(gather.locate(np.asarray([sid], np.int64))[0][0])] = time_ns()

    return stamp


class DeviceBatches:
    """An iterable of device batches over a ``StreamingDataset`` (one :func:`device_iter` per
    epoch) that checkpoints like ``StreamingDataLoader`` (``dataloader.py:50-96``): it counts
    the samples it hands out on this rank, and :meth:`state_dict` passes the global count --
    this rank's times the number of ranks, divided by ``replication`` when set -- to
    ``dataset.state_dict(num_samples, False)``."""

    def __init__(self, dataset: Any, batch_size: int, **kwargs: Any) -> None:
        self.dataset = dataset
        self.batch_size = batch_size
        self.kwargs = kwargs
        self.num_samples_yielded = 0

    def __iter__(self) -> Iterator[DecodedBatch]:
        self.num_samples_yielded = 0
        for batch in device_iter(self.dataset, self.batch_size, **self.kwargs):
            self.num_samples_yielded += len(batch)
            yield batch

    def state_dict(self) -> dict[str, Any]:
        """The dataset's checkpoint after the samples handed out so far this epoch."""
        num_ranks = int(getattr(self.dataset._unique_rank_world, 'num_ranks', 1))
        num_samples = self.num_samples_yielded * num_ranks
        replication = getattr(self.dataset, 'replication', None)
        if replication is not None:
            num_samples = num_samples // replication
        return self.dataset.state_dict(num_samples, False)

    def load_state_dict(self, obj: dict[str, Any]) -> None:
        self.dataset.load_state_dict(obj)
