"""End-to-end host path: shard files -> pinned staging -> HBM -> device decode (-> host).

The reference reads every sample from the local cache file with ``open``/``seek``/``read``
(``streaming/base/format/mds/reader.py:128-149``) after ``Stream.prepare_shard`` has downloaded
and, for compressed shards, decompressed the file (``streaming/base/stream.py:319-412``,
``compression.py:243-258``). :class:`ShardPipeline` is the device-side counterpart for a whole
set of shards:

1. host stage (thread pool): read each raw shard file -- or decompress its ``zip_data`` file
   (zstd through libzstd) -- straight into a pinned staging buffer laid out as a device batch;
2. H2D stage: one async copy per batch on a copy stream;
3. decode stage: scan + decode kernels on the compute stream, waiting on the copy event;
4. optional D2H of the decoded columns into pinned host memory (the host hand-off).

Batches of shards flow through a ring of ``depth`` staging/device slots, so reading and
decompressing batch i+1 overlaps the copy and decode of batch i.
"""

from __future__ import annotations

import logging
import os
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Iterator, Optional, Sequence, Union

import numpy as np
import torch

from streaming_amd.compression import decompress, decompress_into, get_compression_extension
from streaming_amd.decoder import (BatchDecoder, DecodedBatch, DeviceBatch, Plan, RaggedColumn,
                                   _layout, _tables)
from streaming_amd import _native
from streaming_amd.hashing import DeviceHasher, _status_check, get_hash, hex_digests, is_hash

__all__ = ['ShardFile', 'ShardPipeline', 'shard_files_from_index', 'to_host',
           'PIPELINE_DEVICE_HASHES']

# Validation hashes computed on the device by the pipeline (the rest on its host threads).
PIPELINE_DEVICE_HASHES = frozenset({'xxh3_64', 'xxh3_128', 'xxh128'})


@dataclass
class ShardFile:
    """One shard as the pipeline reads it."""
    path: str                      # raw file, or the compressed file if compression is set
    raw_bytes: int                 # decompressed size (index.json raw_data.bytes)
    samples: int
    compression: Optional[str] = None
    hashes: Optional[dict] = None  # index.json raw_data.hashes (digests of the raw shard file)


_log = logging.getLogger(__name__)

def shard_files_from_index(dirname: str, index: dict, split: Optional[str] = None,
                           prefer_raw: bool = True) -> list[ShardFile]:
    """ShardFiles of an index.json: the raw file when present, else the compressed one."""
    out = []
    for info in index['shards']:
        raw = os.path.join(dirname, split or '', info['raw_data']['basename'])
        z = info.get('zip_data')
        hashes = info['raw_data'].get('hashes') or {}
        if (prefer_raw and os.path.exists(raw)) or not z:
            out.append(ShardFile(raw, info['raw_data']['bytes'], info['samples'], None, hashes))
        else:
            out.append(
                ShardFile(os.path.join(dirname, split or '', z['basename']),
                          info['raw_data']['bytes'], info['samples'], info['compression'], hashes))
    return out


def _fill(view: np.ndarray, shard: ShardFile, host_hash: Optional[str] = None) -> None:
    """Read or decompress one shard into its slice of the pinned staging buffer (and check a
    hashlib digest of the raw bytes on the host when asked)."""
    if shard.compression:
        with open(shard.path, 'rb') as f:
            data = f.read()
        ext = get_compression_extension(shard.compression)
        if ext == 'zstd':
            n = decompress_into(shard.compression, data, view)
        else:
            raw = decompress(shard.compression, data)
            n = len(raw)
            view[:n] = np.frombuffer(raw, np.uint8)
    else:
        with open(shard.path, 'rb', buffering=0) as f:
            n = f.readinto(memoryview(view))
    if n != shard.raw_bytes:
        raise ValueError(f'{shard.path}: expected {shard.raw_bytes} raw bytes, got {n}')
    # hashed in place (a buffer, no copy): hashlib and xxhash release the GIL on large buffers,
    # so the pool threads hash in parallel (a bytes copy per shard serialised them: 3.7 GiB/s on
    # 16 threads, profiles/r02/e2e_validate.json)
    if host_hash and get_hash(host_hash, memoryview(view[:n])) != shard.hashes[host_hash]:
        raise ValueError(f'Checksum failure: {shard.path}')


def _fill_after(event: Optional[torch.cuda.Event], view: np.ndarray, shard: ShardFile,
                host_hash: Optional[str]) -> None:
    """Fill a staging slice once the slot's previous H2D copy (``event``) has completed."""
    if event is not None:
        event.synchronize()
    _fill(view, shard, host_hash)


class _Slot:

    def __init__(self, total: int, device: torch.device) -> None:
        self.host = torch.empty(total, dtype=torch.uint8, pin_memory=True)
        self.dev = torch.empty(total, dtype=torch.uint8, device=device)
        self.copied = torch.cuda.Event()
        self.decoded = torch.cuda.Event()
        self.handed: Optional[torch.cuda.Event] = None  # iter_host: D2H of its outputs queued
        self.hasher = DeviceHasher(device)
        self.decoder: Optional[BatchDecoder] = None
        self.key: Optional[tuple] = None


class ShardPipeline:
    """Stream shard files through the device decoder in batches of ``shards_per_batch``.

    Args:
        plan: the shards' schema (all shards of a pipeline share it).
        shards: shard files in order.
        shards_per_batch: shards decoded per device batch.
        depth: staging/device slots in flight (2 = double buffering). Default: enough slots
            for every worker thread to have a shard to read or decompress, ``ceil(workers /
            shards_per_batch) + 1`` and at least 2 (a slot is refilled only after its H2D copy,
            so with 16 threads and 8-shard batches two slots leave half the threads idle), two
            more when shards are compressed (decompression times vary shard to shard; spare
            slots absorb a slow one: config E, 16 threads, 8-shard batches, 2M samples: 16.5
            GiB/s at depth 2, 24.2 at depth 3 (15-24 % pass-to-pass spread), 24.1-24.9 at depth
            4 (6-18 %), 25.0 at depth 5 (3-4 %)). Memory: each slot holds the
            largest batch's shard bytes twice (pinned host + device) and its decoder's outputs
            on the device (about the batch's bytes again), so a slot costs ~2x the batch in
            device memory and 1x in pinned host memory; the automatic depth is capped so that
            the slots take at most half of the device memory free at construction (an explicit
            ``depth`` is taken as given). The chosen depth is logged (``logging`` INFO).
        workers: host threads reading / decompressing shards.
        device: CUDA device.
        validate_hash: check every shard against its index.json ``raw_data.hashes[algo]``
            before its batch is handed out, raising ``ValueError('Checksum failure: ...')`` like
            ``Stream._prepare_shard_part`` (``stream.py:401-411``). xxh3_64 / xxh128 run on the
            device over the resident batch (``streaming_amd.hashing``: 2.4-4.5 TB/s); every other
            algorithm -- hashlib's, and xxh64 / xxh32, whose one dependent chain per shard makes
            the device version slower than a host core -- on the host threads as
            the shards are read.
    """

    def __init__(self,
                 plan: Plan,
                 shards: Sequence[ShardFile],
                 shards_per_batch: int = 8,
                 depth: Optional[int] = None,
                 workers: int = 8,
                 device: Union[str, torch.device, None] = None,
                 validate_hash: Optional[str] = None) -> None:
        self.plan = plan
        self.shards = list(shards)
        self.validate_hash = validate_hash
        if validate_hash:
            if not is_hash(validate_hash):
                raise ValueError(f'{validate_hash} is not a supported hash algorithm.')
            for s in self.shards:
                if validate_hash not in (s.hashes or {}):
                    raise ValueError(
                        f'Hash algorithm `{validate_hash}` chosen for data ' +
                        f'validation does not match with those provided during dataset ' +
                        f'creation `{sorted((s.hashes or {}).keys())}`. Provide one of those.')
        self._device_hash = bool(validate_hash) and validate_hash in PIPELINE_DEVICE_HASHES
        self.per = max(1, shards_per_batch)
        dev = torch.device(device or 'cuda')
        if dev.index is None:
            dev = torch.device('cuda', torch.cuda.current_device())
        self.device = dev
        self.groups = [self.shards[i:i + self.per] for i in range(0, len(self.shards), self.per)]
        biggest = max((_layout([s.raw_bytes for s in g])[1] for g in self.groups), default=0)
        if depth is None:
            depth = max(2, -(-max(1, workers) // self.per) + 1)
            if any(s.compression for s in self.shards):
                depth += 2
            free = torch.cuda.mem_get_info(dev)[0]
            cap = max(2, int(free // 2 // max(2 * biggest, 1)))
            if depth > cap:
                depth = cap
            _log.info('ShardPipeline: depth %d (%d-shard batches up to %d bytes, %d workers)',
                      depth, self.per, biggest, workers)
        self.depth = max(1, depth)
        self.slots = [_Slot(biggest, dev) for _ in range(min(self.depth, len(self.groups)))]
        self.pool = ThreadPoolExecutor(max_workers=max(1, workers))
        self.copy_stream = torch.cuda.Stream(dev)
        self._lock = threading.Lock()
        # measurement only (scripts/e2e_bench.py --trace): a list collects (what, batch, host
        # seconds, timing event on the stream the step was queued on or None)
        self.trace: Optional[list] = None

    def _mark(self, what: str, gi: int, stream: Optional[torch.cuda.Stream] = None) -> None:
        if self.trace is None:
            return
        ev = None
        if stream is not None:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(stream)
        self.trace.append((what, gi, time.perf_counter(), ev))

    def _stage(self, slot: _Slot, group: Sequence[ShardFile], after: bool = False):
        """Read / decompress ``group`` into the slot's pinned buffer on the pool threads; with
        ``after``, each task first waits for the slot's previous H2D copy to complete."""
        sizes = [s.raw_bytes for s in group]
        offsets, total = _layout(sizes)
        view = slot.host.numpy()
        host_hash = self.validate_hash if self.validate_hash and not self._device_hash else None
        event = slot.copied if after else None
        futs = [
            self.pool.submit(_fill_after, event, view[o:o + s.raw_bytes], s, host_hash)
            for o, s in zip(offsets, group)
        ]
        return futs, sizes, offsets, total

    def _batch(self, slot: _Slot, group, sizes, offsets, total) -> DeviceBatch:
        samples = [s.samples for s in group]
        tr = self.plan.tile_rows_for(total, sum(samples))  # = the C side's batch->bytes
        raw, tile_shard, row0, rows, tiles = _tables(sizes, samples, offsets, tr)
        dev = self.device
        # small tables: pinned + async on the compute stream (no host wait on the device)
        descs = torch.from_numpy(raw).pin_memory().to(dev, non_blocking=True)
        tiles_t = (torch.from_numpy(tile_shard).pin_memory().to(dev, non_blocking=True)
                   if tiles else torch.zeros(1, dtype=torch.int32, device=dev))
        return DeviceBatch(slot.dev[:total], descs, tiles_t, offsets, sizes, samples, row0, tiles,
                           rows, tr)

    def __iter__(self) -> Iterator[DecodedBatch]:
        """Decoded batches in order (device tensors, valid until the slot is reused ``depth``
        batches later; clone or :func:`to_host` them to keep them)."""
        compute = torch.cuda.current_stream(self.device)
        pending = []  # (slot, futures, sizes, offsets, total, group)
        ngroups = len(self.groups)
        for i in range(min(len(self.slots), ngroups)):
            pending.append((self.slots[i], *self._stage(self.slots[i], self.groups[i]),
                            self.groups[i]))
        for gi in range(ngroups):
            slot, futs, sizes, offsets, total, group = pending.pop(0)
            for f in futs:
                f.result()
            self._mark('staged', gi)
            with torch.cuda.stream(self.copy_stream):
                self.copy_stream.wait_event(slot.decoded)  # device slot free again
                self._mark('h2d_start', gi, self.copy_stream)
                slot.dev[:total].copy_(slot.host[:total], non_blocking=True)
                slot.copied.record(self.copy_stream)
                self._mark('h2d_end', gi, self.copy_stream)
            compute.wait_event(slot.copied)
            # Restage this slot for batch gi + depth right away: the pool threads wait for this
            # copy to land, then refill the pinned buffer, while this loop moves on (copies are
            # queued back to back; host reads / decompression of later batches overlap).
            nxt = gi + len(self.slots)
            if nxt < ngroups:
                pending.append((slot, *self._stage(slot, self.groups[nxt], after=True),
                                self.groups[nxt]))
            batch = self._batch(slot, group, sizes, offsets, total)
            digests = None
            if self._device_hash:
                digests, hstatus = slot.hasher.launch(self.validate_hash, slot.dev[:total],
                                                      list(zip(offsets, sizes)))
            key = (tuple(sizes), tuple(s.samples for s in group))
            if slot.decoder is None or slot.key != key:
                slot.decoder = BatchDecoder(self.plan, batch)
                slot.key = key
            else:
                slot.decoder.batch = batch
                slot.decoder._abi = batch.abi()
                if self.plan.num_var:
                    slot.decoder._sized = False  # ragged totals differ per batch: re-size
            if slot.handed is not None:  # iter_host: this slot's last outputs are off the device
                compute.wait_event(slot.handed)
                slot.handed = None
            self._mark('decode_start', gi, compute)
            out = slot.decoder.run()
            slot.decoded.record(compute)
            self._mark('decode_end', gi, compute)
            if digests is not None:
                _status_check(hstatus)
                for got, shard in zip(hex_digests(self.validate_hash, digests), group):
                    if got != shard.hashes[self.validate_hash]:
                        raise ValueError(f'Checksum failure: {shard.path}')
            # a malformed sample fails its own batch, before the batch is handed out (the
            # reference raises when that sample is read); waits for this batch's decode, while
            # the next batches' reads and copies stay queued
            slot.decoder.check()
            self._mark('yield', gi)
            self._current = slot
            yield out

    def iter_host(self) -> Iterator[dict[str, Union[np.ndarray, tuple]]]:
        """Decoded batches handed to the host (numpy arrays as :func:`to_host` returns them), in
        order. Each batch's D2H copy runs on its own stream while the next batch's H2D copy is
        in flight, and the next decode waits for it (the outputs it reads belong to the slot); a
        batch is handed out once its copy has landed. The D2H is a kernel storing into pinned
        memory (``mdsx_copy_to_host``): two DMA-engine copies in opposite directions serialise
        on this platform, a kernel beside a DMA copy does not. Only the slot's next decode
        (``depth`` batches later), which rewrites the outputs being copied, waits for the copy
        (DESIGN.md §7)."""
        compute = torch.cuda.current_stream(self.device)
        d2h = torch.cuda.Stream(self.device)
        prev = None
        for gi, out in enumerate(self):
            host, done = _to_host_async(out, d2h, compute, self._mark if self.trace is not None
                                        else None, gi)
            self._current.handed = done  # the slot's outputs are reused by its next decode
            if prev is not None:
                prev[1].synchronize()
                self._mark('host_yield', gi - 1)
                yield _host_arrays(prev[0])
            prev = (host, done)
        if prev is not None:
            prev[1].synchronize()
            self._mark('host_yield', len(self.groups) - 1)
            yield _host_arrays(prev[0])

    def close(self) -> None:
        self.pool.shutdown(wait=True)


def _to_host_async(decoded: DecodedBatch, stream: torch.cuda.Stream,
                   after: torch.cuda.Stream, mark=None, gi: int = 0) -> tuple[dict, torch.cuda.Event]:
    """Queue the D2H copies of every column of ``decoded`` (pinned host tensors) on ``stream``,
    behind the work queued so far on ``after``; returns the host tensors and the copies' event."""
    ready = torch.cuda.Event()
    ready.record(after)
    stream.wait_event(ready)
    if mark is not None:
        mark('d2h_start', gi, stream)
    lib = _native.lib()
    out = {}
    with torch.cuda.stream(stream):
        for name, col in decoded.columns.items():
            parts = ([col.values, col.offsets] + ([col.flags] if col.flags is not None else [])
                     if isinstance(col, RaggedColumn) else [col])
            host = []
            for t in parts:
                t = t.contiguous()
                t.record_stream(stream)  # read on this stream (a kernel torch does not see)
                h = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                nbytes = t.numel() * t.element_size()
                body = nbytes & ~15
                if body and not (t.data_ptr() | h.data_ptr()) & 15:
                    # a kernel storing into the pinned buffer: it overlaps the DMA-engine H2D
                    # of the next batch, where a DMA-engine D2H would queue behind it
                    _native.raise_for_code(lib.mdsx_copy_to_host(
                        t.data_ptr(), h.data_ptr(), body, stream.cuda_stream), 'mdsx_copy_to_host')
                    if nbytes > body:
                        h.view(-1).view(torch.uint8)[body:].copy_(
                            t.view(-1).view(torch.uint8)[body:], non_blocking=True)
                else:
                    h.copy_(t, non_blocking=True)
                host.append(h)
            out[name] = host if isinstance(col, RaggedColumn) else host[0]
    if mark is not None:
        mark('d2h_end', gi, stream)
    done = torch.cuda.Event()
    done.record(stream)
    return out, done


def _host_arrays(out: dict) -> dict[str, Union[np.ndarray, tuple]]:
    res = {}
    for name, v in out.items():
        if isinstance(v, list):
            res[name] = tuple(x.numpy() for x in v)
        else:
            res[name] = v.view(torch.uint8).numpy() if v.dtype in (torch.uint16, torch.uint32,
                                                                   torch.uint64) else v.numpy()
    return res


def to_host(decoded: DecodedBatch, pin: bool = True) -> dict[str, Union[np.ndarray, tuple]]:
    """D2H hand-off of a decoded batch: numpy arrays (ragged columns as (values, offsets[, flags]))."""
    out = {}
    for name, col in decoded.columns.items():
        if isinstance(col, RaggedColumn):
            parts = [col.values, col.offsets] + ([col.flags] if col.flags is not None else [])
            host = []
            for t in parts:
                h = torch.empty(t.shape, dtype=t.dtype, pin_memory=pin)
                h.copy_(t, non_blocking=True)
                host.append(h)
            out[name] = host
        else:
            h = torch.empty(col.shape, dtype=col.dtype, pin_memory=pin)
            h.copy_(col, non_blocking=True)
            out[name] = h
    torch.cuda.current_stream().synchronize()
    return _host_arrays(out)
