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


def _iterator_class(dataset: Any) -> type:
    """The reference's ``_Iterator`` (``dataset.py:64-166``), from the module that defines the
    dataset's iteration methods (any ``StreamingDataset`` subclass, or a stand-in)."""
    for klass in type(dataset).__mro__:
        if '_each_sample_id' in klass.__dict__:
            mod = sys.modules[klass.__module__]
            if hasattr(mod, '_Iterator'):
                return mod._Iterator
    raise TypeError(f'{type(dataset).__name__} has no StreamingDataset iteration to follow')


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


def device_iter(dataset: Any, batch_size: int, *, retry: int = 7,
                gather: Optional[Any] = None) -> Iterator[DecodedBatch]:
    """``StreamingDataset.__iter__`` (``dataset.py:1475-1513``) yielding DEVICE batches.

    The reference's own control flow, step for step: the previous epoch's iterator is exited,
    the worker world detected, the epoch incremented or resumed (``_resume_incr_epoch``: a
    ``load_state_dict`` checkpoint resumes mid-epoch, ``dataset.py:691-776``), this worker's ids
    laid out by ``_get_work`` (``generate_work``, ``dataset.py:1012-1066``), and the
    ``_prepare_thread`` / ``_ready_thread`` started on the dataset's executor to download and
    ready shards ahead of the loop (``dataset.py:1313-1428``). The ids then come from
    ``_each_sample_id`` -- in order, ``-1`` skipped, each once its shard is ready -- and every
    ``batch_size`` of them (the last batch may be short) are gathered on the GPU from the
    shards' decoded columns (:class:`streaming_amd.order.DeviceSampleGather`: shards decoded
    on demand through the bounded decoded-shard cache, one launch sequence per column) instead
    of ``map(self.__getitem__, ...)`` and ``default_collate``. Each batch carries its
    ``sample_ids``.

    The dataset's shards must be device readers (``stream_name='mdsx'``,
    :func:`register_device_stream`). Run it in the process that owns the GPU (a ``DataLoader``
    with ``num_workers=0``, or no loader): the decode runs on the device, so there is nothing
    for host workers to parallelise. Checkpoints are the reference's: ``dataset.state_dict(
    num_samples, from_beginning)`` with the samples consumed so far, then ``load_state_dict`` and
    a new ``device_iter`` resume there.

    ``gather``: what turns ids into a batch (default: a ``DeviceSampleGather`` over
    ``dataset.shards``); an object with ``gather(ids)``, ``locate(ids)`` and ``shards``.
    """
    if batch_size <= 0:
        raise ValueError('batch_size must be positive')
    ds = dataset
    if gather is None:
        from streaming_amd.order import DeviceSampleGather
        bad = [i for i, s in enumerate(ds.shards) if not isinstance(s, MDSReader)]
        if bad:
            raise TypeError(f'device_iter: shard {bad[0]} is a {type(ds.shards[bad[0]]).__name__}, '
                            f'not a device reader (build the dataset with stream_name=\'mdsx\', '
                            f'streaming_amd.plugin.register_device_stream)')
        gather = DeviceSampleGather(ds.shards)
    Iterator_ = _iterator_class(ds)
    # -- StreamingDataset.__iter__, dataset.py:1481-1510
    if hasattr(ds, '_iterator'):
        ds._iterator.exit()
    if not hasattr(ds, '_executor'):
        ds._executor = ThreadPoolExecutor()
    if not hasattr(ds, '_event'):
        ds._event = Event()
    elif ds._event.is_set():
        raise RuntimeError('Background thread failed. Check other traceback.')
    ds._unique_worker_world = ds._unique_rank_world.detect_workers()
    ds._parallel_worker_world = ds._parallel_rank_world.detect_workers()
    epoch, sample_in_epoch = ds._resume_incr_epoch()
    sample_ids = ds._get_work(epoch, sample_in_epoch)
    if not len(sample_ids):  # resumed at the end of the epoch: out of samples
        return
    ds._iterator = it = Iterator_(sample_ids)
    prepare_future = ds._executor.submit(ds._prepare_thread, it)
    prepare_future.add_done_callback(ds.on_exception)
    ready_future = ds._executor.submit(ds._ready_thread, it)
    ready_future.add_done_callback(ds.on_exception)
    # -- in place of `yield from map(self.__getitem__, self._each_sample_id(it))`
    pending = []
    for sample_id in ds._each_sample_id(it):
        pending.append(sample_id)
        if len(pending) == batch_size:
            yield _gather_batch(ds, gather, pending, retry)
            pending = []
    if pending:
        yield _gather_batch(ds, gather, pending, retry)
    wait([prepare_future, ready_future], return_when='FIRST_EXCEPTION')
    it.exit()


class DeviceBatches:
    """An iterable of device batches over a ``StreamingDataset`` (one :func:`device_iter` per
    epoch), counting the samples it hands out so that :meth:`state_dict` checkpoints mid-epoch as
    ``StreamingDataLoader`` does (``dataloader.py:50-96``, single process)."""

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
        return self.dataset.state_dict(self.num_samples_yielded, False)

    def load_state_dict(self, obj: dict[str, Any]) -> None:
        self.dataset.load_state_dict(obj)
