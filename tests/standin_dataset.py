"""A stand-in for the private iteration surface of the reference's StreamingDataset that
``streaming_amd.plugin.device_iter`` drives (``dataset.py:64-166`` ``_Iterator``,
``_resume_incr_epoch``, ``_get_work``, ``_prepare_thread``, ``_ready_thread``,
``_each_sample_id``, ``prepare_shard``, ``on_exception``), for the GPU box where the reference
is absent. ``_get_work`` returns the ids the real reference's ``generate_work`` recorded
(tests/golden/order); the threads and the yield loop follow the reference's loops."""

from __future__ import annotations

from concurrent.futures import Future
from time import sleep

import numpy as np

TICK = 0.001


class _Iterator:
    """dataset.py:64-166, minus the shared-memory bookkeeping."""

    def __init__(self, sample_ids) -> None:
        self.sample_ids = sample_ids
        self.total = len(sample_ids)
        self.prepare_index = 0
        self.ready_index = 0
        self.yield_index = 0
        self._exit = False

    def exit(self) -> None:
        self._exit = True

    def should_exit(self) -> bool:
        return self._exit

    def on_exit(self) -> None:
        pass


class _World:

    def detect_workers(self) -> '_World':
        return self


class StandInDataset:

    def __init__(self, shards, work) -> None:
        """``work(epoch, sample_in_epoch)``: this worker's flattened ids (``-1`` padding kept)."""
        self.shards = shards
        self._work = work
        self._shard_access_times = np.zeros(len(shards), np.uint64)
        self._unique_rank_world = self._parallel_rank_world = _World()
        self.next_epoch = 0
        self._resume = None
        self.prepared = []

    def load_state_dict(self, obj) -> None:
        self._resume = (obj['epoch'], obj['sample_in_epoch'])

    def _resume_incr_epoch(self):
        if self._resume is not None:
            epoch, sample_in_epoch = self._resume
            self._resume = None
        else:
            epoch, sample_in_epoch = self.next_epoch, 0
        self.next_epoch = epoch + 1
        return epoch, sample_in_epoch

    def _get_work(self, epoch, sample_in_epoch):
        return self._work(epoch, sample_in_epoch)

    def prepare_shard(self, shard_id, blocking=True) -> None:
        self.prepared.append(shard_id)

    def _shard_of(self, sample_id):
        starts = np.cumsum([0] + [s.samples for s in self.shards])
        return int(np.searchsorted(starts, sample_id, side='right') - 1)

    def _prepare_thread(self, it) -> None:
        while not it.should_exit() and it.prepare_index < it.total:
            if self._event.is_set():
                break
            sid = it.sample_ids[it.prepare_index]
            if sid != -1:
                self.prepare_shard(self._shard_of(sid), False)
            it.prepare_index += 1
        it.on_exit()

    def _ready_thread(self, it) -> None:
        while not it.should_exit() and it.ready_index < it.total:
            if self._event.is_set():
                break
            if it.ready_index >= it.prepare_index:
                sleep(TICK)
                continue
            it.ready_index += 1
        it.on_exit()

    def _each_sample_id(self, it):
        while True:
            if it.should_exit() or it.yield_index == it.total or self._event.is_set():
                break
            if it.ready_index <= it.yield_index:
                sleep(TICK)
                continue
            sid = it.sample_ids[it.yield_index]
            if sid != -1:
                yield int(sid)
            it.yield_index += 1
        it.on_exit()

    def on_exception(self, future: Future) -> None:
        exc = future.exception()
        if exc:
            self._event.set()
            raise exc
