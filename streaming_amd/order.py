"""Device batches in the reference's sample order.

``StreamingDataset.__iter__`` (``streaming/base/dataset.py:1475-1513``) takes this worker's slice
of the epoch's sample-id array that ``generate_work`` lays out (``batching/__init__.py:28-45``:
``[nodes, ranks per node, workers per rank, batches, batch]``, ``-1`` padding;
``dataset.py:1054-1056`` flattens the worker's slice), walks it skipping ``-1``
(``_each_sample_id``, ``dataset.py:1430-1473``) and fetches each id with ``get_item``
(``dataset.py:1237-1293``: ``spanner`` -> ``shard[idx]``). The DataLoader then collates runs of
``batch_size`` samples.

:class:`DeviceSampleGather` is the device side of that loop: the same ids, in the same order, as
device batches. For each batch the touched shards are decoded on demand through the readers'
bounded decoded-shard cache (:mod:`streaming_amd.cache`; a shard decoded once stays resident while
the cache holds it), then every column is gathered from all of them in one launch sequence
(``mdsx_gather_*_multi``: each id names its source shard and row), rows already in batch order.
:func:`streaming_amd.plugin.device_iter` drives it from the reference's own iteration. Resumption is the
reference's: ``state_dict`` / ``load_state_dict`` move ``sample_in_epoch``, and ``generate_work``
then hands out the rest of the epoch (``dataset.py:778-856``); this module takes those ids as they
come.

Errors follow ``get_item``: a missing shard file raises ``FileNotFoundError`` (the caller
re-prepares it, ``dataset.py:1274-1291``); a malformed sample raises for that sample only
(``IndexError`` for an empty one, ``ValueError`` for a range error); ``str`` values that are not
well-formed UTF-8 come back flagged in the column's ``flags`` (where ``bytes.decode('utf-8')``
raises, ``encodings.py:80-81``).
"""

from __future__ import annotations

import os
from typing import Iterator, Sequence, Union

import numpy as np
import torch

from streaming_amd.decoder import DecodedBatch, RaggedColumn, gather_sources
from streaming_amd.reader import MDSReader

__all__ = ['worker_sample_ids', 'loader_batches', 'concat_batches', 'DeviceSampleGather']


def worker_sample_ids(epoch_sample_ids: np.ndarray, node: int, rank_of_node: int,
                      worker_of_rank: int) -> np.ndarray:
    """One worker's portion of ``generate_work``'s array, flattened (``dataset.py:1054-1056``);
    the ``-1`` padding is kept (the iteration skips it)."""
    return np.asarray(epoch_sample_ids, np.int64)[node, rank_of_node, worker_of_rank].reshape(-1)


def loader_batches(epoch_sample_ids: np.ndarray, node: int, rank_of_node: int, workers: int,
                   batch_size: int) -> list[np.ndarray]:
    """The sample ids of each batch a ``DataLoader(dataset, batch_size, num_workers=workers)``
    over a ``StreamingDataset`` yields on one rank, in the loader's order.

    Each worker iterates its own slice of ``generate_work``'s array (``world.py:150-163``,
    ``dataset.py:1054-1056``), ``-1`` skipped (``_each_sample_id``), and the loader's fetcher
    cuts that stream into batches of ``batch_size`` consecutive samples (the last one may be
    short). Torch hands out batch index i to the workers round robin and returns them in index
    order, skipping a worker once it is exhausted (its remaining indices are dropped,
    ``torch/utils/data/dataloader.py`` ``_MultiProcessingDataLoaderIter``): batch k of every
    worker still running, worker by worker, for k = 0, 1, ... ``workers`` 0 (no worker
    processes) iterates as one worker."""
    workers = max(1, int(workers))
    arr = np.asarray(epoch_sample_ids, np.int64)
    per_worker = []
    for w in range(workers):
        ids = worker_sample_ids(arr, node, rank_of_node, w)
        ids = ids[ids != -1]
        per_worker.append([ids[lo:lo + batch_size] for lo in range(0, ids.size, batch_size)])
    out = []
    for k in range(max((len(b) for b in per_worker), default=0)):
        out.extend(b[k] for b in per_worker if k < len(b))
    return out


def concat_batches(parts: Sequence[DecodedBatch]) -> DecodedBatch:
    """Rows of ``parts`` one after the other (device tensors; ragged offsets rebased on the
    device, no host sync)."""
    if not parts:
        raise ValueError('concat_batches: no parts')
    if len(parts) == 1:
        return parts[0]
    cols: dict[str, Union[torch.Tensor, RaggedColumn]] = {}
    for name, first in parts[0].columns.items():
        xs = [p.columns[name] for p in parts]
        if isinstance(first, RaggedColumn):
            ends = torch.stack([x.offsets[-1] for x in xs])
            bases = torch.cumsum(ends, 0) - ends
            offs = [xs[0].offsets] + [x.offsets[1:] + b for x, b in zip(xs[1:], bases[1:])]
            vals = torch.cat([x.values for x in xs])  # gathered values: exactly offsets[-1]
            flags = torch.cat([x.flags for x in xs]) if first.flags is not None else None
            cols[name] = RaggedColumn(vals, torch.cat(offs), flags)
        else:
            cols[name] = torch.cat(xs)
    first = next(iter(cols.values()))
    dev = (first.offsets if isinstance(first, RaggedColumn) else first).device
    return DecodedBatch(cols, sum(p.rows for p in parts),
                        stream=torch.cuda.current_stream(dev) if dev.type == 'cuda' else None)


class DeviceSampleGather:
    """Device batches of global sample ids over a list of shards (``MDSReader``\\ s, in the
    dataset's shard order: global id -> (shard, local id) as ``Spanner``, ``spanner.py:40-59``).

    Args:
        shards: the dataset's readers (``LocalDataset.shards``, or the readers a device
            ``Stream`` returns).
    """

    def __init__(self, shards: Sequence[MDSReader]) -> None:
        self.shards = list(shards)
        counts = np.array([s.samples for s in self.shards], np.int64)
        self.starts = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        self.num_samples = int(self.starts[-1])

    def locate(self, ids: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        """(shard, local id) of each global id."""
        ids = np.asarray(ids, np.int64)
        bad = (ids < 0) | (ids >= self.num_samples)
        if bad.any():
            raise IndexError(f'Index {int(ids[bad][0])} out of range for dataset of '
                             f'{self.num_samples} samples')
        shard = np.searchsorted(self.starts, ids, side='right') - 1
        return shard, ids - self.starts[shard]

    def gather(self, sample_ids: Union[Sequence[int], np.ndarray, torch.Tensor]) -> DecodedBatch:
        """The samples ``sample_ids`` (global ids; ``-1`` skipped), in that order: the shards
        they touch decoded (or found in the cache), then every column gathered from all of them
        in one launch sequence (``mdsx_gather_*_multi``), rows already in batch order. The
        touched shards' decoded columns are held until the gather is queued, so a decoded-shard
        cache smaller than one batch's shards is exceeded for that long."""
        ids = np.asarray(torch.as_tensor(sample_ids).cpu().numpy() if isinstance(
            sample_ids, torch.Tensor) else sample_ids, np.int64).reshape(-1)
        ids = ids[ids != -1]
        if ids.size == 0:
            raise ValueError('gather: no samples')
        shard, local = self.locate(ids)
        touched, src = np.unique(shard, return_inverse=True)
        src = src.reshape(-1)
        decoded = []
        for j, s in enumerate(touched):
            reader = self.shards[int(s)]
            os.stat(reader._filename())  # FileNotFoundError once evicted (the reference's open())
            entry = reader._decode_entry()
            if entry.status.code != 0:  # raise only for the bad samples this batch reads
                for idx in np.unique(local[src == j]):
                    reader._check_row(entry, int(idx))
            decoded.append(entry.decoded)
        return gather_sources(decoded, src, local)

    def iter_batches(self, sample_ids: Union[Sequence[int], np.ndarray, torch.Tensor],
                     batch_size: int) -> Iterator[DecodedBatch]:
        """Device batches of ``batch_size`` samples over ``sample_ids`` (one worker's ids,
        flattened, ``-1`` skipped; the last batch may be short), in the reference's order."""
        if batch_size <= 0:
            raise ValueError('batch_size must be positive')
        ids = np.asarray(torch.as_tensor(sample_ids).cpu().numpy() if isinstance(
            sample_ids, torch.Tensor) else sample_ids, np.int64).reshape(-1)
        ids = ids[ids != -1]
        for lo in range(0, ids.size, batch_size):
            yield self.gather(ids[lo:lo + batch_size])
