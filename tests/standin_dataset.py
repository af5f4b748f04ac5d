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


class World:
    """world.py:39-163 restated: node / rank / worker coordinates of one process."""

    def __init__(self, num_nodes, ranks_per_node, workers_per_rank, worker) -> None:
        self.node = worker // (ranks_per_node * workers_per_rank)
        self.num_nodes = num_nodes
        self.rank = worker // workers_per_rank
        self.num_ranks = num_nodes * ranks_per_node
        self.rank_of_node = self.rank % ranks_per_node
        self.ranks_per_node = ranks_per_node
        self.worker = worker
        self.workers_per_rank = workers_per_rank
        self.worker_of_rank = worker % workers_per_rank
        self.workers_per_node = ranks_per_node * workers_per_rank
        self.is_local_leader = not (worker % self.workers_per_node)

    def detect_workers(self) -> 'World':  # no DataLoader worker processes here
        return World(self.num_nodes, self.ranks_per_node, 1, self.rank)

    def replicate(self, replication: int) -> 'World':
        """world.py:117-148: the World of the replication group this rank iterates as."""
        rank = self.rank // replication
        num_ranks = self.num_ranks // replication
        worker = rank * self.workers_per_rank + self.worker_of_rank
        num_nodes = num_ranks // self.ranks_per_node if num_ranks % self.ranks_per_node == 0 else 1
        return World(num_nodes, num_ranks // num_nodes, self.workers_per_rank, worker)


def generate_work(batching_method, dataset, world, epoch, sample_in_epoch):
    """batching/__init__.py:28-45: the stand-in returns the epoch's recorded 5-D id array."""
    return dataset._epoch_work(world, epoch, sample_in_epoch)


class StandInDataset:

    def __init__(self, shards, work, epoch_work=None, world=(1, 1, 0), batch_size=None,
                 replication=None, batching_method='random') -> None:
        """``work(epoch, sample_in_epoch)``: this worker's flattened ids (``-1`` padding kept);
        ``epoch_work(world, epoch, sample_in_epoch)``: ``generate_work``'s 5-D array for a World
        (multi-worker iteration); ``world``: (nodes, ranks per node, rank); ``replication``: as
        StreamingDataset's (dataset.py:370-374: the parallel rank World replicated)."""
        self.shards = shards
        self._work = work
        self._epoch_work = epoch_work
        self.batch_size = batch_size
        self.batching_method = batching_method
        self.replication = replication
        self._shard_access_times = np.zeros(len(shards), np.uint64)
        nodes, rpn, rank = world
        self._unique_rank_world = World(nodes, rpn, 1, rank)
        self._parallel_rank_world = (self._unique_rank_world.replicate(replication)
                                     if replication is not None else World(nodes, rpn, 1, rank))
        self.next_epoch = 0
        self._resume = None
        self.prepared = []

    def state_dict(self, num_samples, from_beginning):
        """dataset.py:778-814, the fields the stand-in keeps."""
        return {'epoch': self.next_epoch - 1, 'sample_in_epoch': num_samples}

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
