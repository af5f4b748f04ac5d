"""Map-style dataset over local MDS shards, decoded on the GPU.

Same interface as the reference ``LocalDataset`` (``streaming/base/local.py:20-78``):
``LocalDataset(local, split)``, ``len``, ``size``, ``get_item(sample_id)`` and fancy
``__getitem__`` (host objects per sample). It adds the device batch API:

* :meth:`decode_all` -- stage every shard into one HBM buffer and decode them in one launch
  sequence (device tensors for the whole dataset);
* :meth:`shard_assignment` -- the shards a rank owns under per-GPU shard ownership
  (shard ``s`` -> rank ``s % world_size``), the multi-GPU layout of the decoder.
"""

from __future__ import annotations

from typing import Any, Iterator, Optional, Sequence, Union

import numpy as np
import torch
from torch.utils.data import Dataset

from streaming_amd.array import Array
from streaming_amd.cache import DecodedShardCache
from streaming_amd.decoder import DecodedBatch, decode_batch, stage_shards
from streaming_amd.distributed import owned_shards
from streaming_amd.order import DeviceSampleGather
from streaming_amd.reader import MDSReader, get_plan, load_index, reader_from_json
from streaming_amd.spanner import Spanner

__all__ = ['LocalDataset', 'shard_assignment']


def shard_assignment(num_shards: int, rank: int, world_size: int) -> list[int]:
    """Shards owned by ``rank``: round-robin, imbalance <= 1 shard, no data exchange."""
    return owned_shards(num_shards, rank, world_size)


class LocalDataset(Array, Dataset):
    """A dataset whose MDS shards reside locally.

    Args:
        local (str): dataset directory.
        split (str, optional): split sub-directory.
        device: CUDA device for decoding (default: current device).
        decoded_cache_bytes (int, optional): bound on the decoded shards this dataset's readers
            keep in device memory (per device, split over the DataLoader workers), and on their
            host copies (LRU; :mod:`streaming_amd.cache`). The most recently used shard of each
            device is always kept, so 0 keeps exactly one decoded shard per device. Default: the
            process-wide cache (``MDSX_DECODED_CACHE_BYTES``, 16 GiB).
    """

    def __init__(self, local: str, split: Optional[str] = None,
                 device: Union[str, torch.device, None] = None,
                 decoded_cache_bytes: Optional[int] = None) -> None:
        split = split or ''
        self.local = local
        self.split = split
        self.device = device
        self.cache = DecodedShardCache(decoded_cache_bytes) if decoded_cache_bytes is not None \
            else None
        obj = load_index(local, split)
        self.shards: list[MDSReader] = [
            reader_from_json(local, split, info, device=device, cache=self.cache)
            for info in obj['shards']
        ]
        self.num_samples = sum(shard.samples for shard in self.shards)
        self.spanner = Spanner(np.array([s.samples for s in self.shards], np.int64))

    def __len__(self) -> int:
        return self.num_samples

    @property
    def size(self) -> int:
        return self.num_samples

    def get_item(self, sample_id: int) -> dict[str, Any]:
        shard_id, index_in_shard = self.spanner[sample_id]
        return self.shards[shard_id][index_in_shard]

    def iter_batches(self, sample_ids: Union[Sequence[int], np.ndarray, torch.Tensor],
                     batch_size: int) -> Iterator[DecodedBatch]:
        """Device batches of ``batch_size`` samples in the order of ``sample_ids`` (global ids,
        ``-1`` padding skipped as the reference's ``_each_sample_id`` does,
        ``dataset.py:1430-1473``; e.g. one worker's slice of ``generate_work``'s ids,
        :func:`streaming_amd.order.worker_sample_ids`): the shards a batch touches are decoded on
        demand through the bounded decoded-shard cache and each batch is gathered on the device
        (:class:`streaming_amd.order.DeviceSampleGather`)."""
        return self.sample_gather.iter_batches(sample_ids, batch_size)

    @property
    def sample_gather(self) -> DeviceSampleGather:
        return DeviceSampleGather(self.shards)

    def decode_all(self, shard_ids: Optional[Sequence[int]] = None,
                   check: bool = True) -> DecodedBatch:
        """Decode the given shards (default: all) in one device batch.

        All shards of one batch must share a schema (one plan), as every shard of a writer does.
        """
        ids = list(range(len(self.shards))) if shard_ids is None else list(shard_ids)
        if not ids:
            raise ValueError('no shards to decode')
        readers = [self.shards[i] for i in ids]
        first = readers[0]
        for r in readers[1:]:
            if (r.column_names, r.column_encodings, r.column_sizes) != \
                    (first.column_names, first.column_encodings, first.column_sizes):
                raise ValueError('decode_all: shards with different schemas in one batch')
        plan = get_plan(first.column_names, first.column_encodings, first.column_sizes)
        data = [r.read_shard_bytes() for r in readers]
        batch = stage_shards(data, [r.samples for r in readers], plan, device=self.device)
        return decode_batch(plan, batch, check=check)
