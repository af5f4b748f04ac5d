"""Reference order without redundant decode: per-GPU shard ownership and a cross-GPU row exchange.

Within a node the reference interleaves ranks at single-sample granularity
(``streaming/base/partition/orig.py:140-163``): every rank's batches draw samples from every shard
of the node's range. :class:`streaming_amd.order.DeviceSampleGather` alone therefore decodes, on
each of R ranks, every shard its batches touch -- each shard R times, and each shard's bytes moved
to every GPU. :class:`OwnedShardGather` keeps the reference's order and decodes each
shard once: shard ``g`` is owned by rank ``g % R`` of the exchange group, which alone decodes it;
every step the ranks exchange the rows the others asked for (hard part 5).

One step, every rank of the group in lock-step (``device_iter`` calls ``gather`` once per batch on
every rank; the reference gives every rank the same number of samples per epoch):

1. the ranks' requested ids, all-gathered (``capacity`` ids per rank, ``-1`` padded);
2. each rank gathers, with the decode's own multi-source gather kernels (``mdsx_gather_*_multi``),
   the requested rows of the shards it owns -- for every requester, in the requester's order --
   decoding an owned shard on first use through the decoded-shard cache; a failure there (a
   missing file, a malformed sample) is agreed on by an all-reduce, so every rank raises and none
   waits in a collective;
3. the rows go to their requesters by ``all_to_all``: fixed columns as bytes (the row counts are
   known to every rank from step 1), ragged columns as per-row lengths, values and UTF-8 flags
   (one more small all-to-all carries the value byte counts);
4. each rank puts the received rows -- grouped by owner, each group in its own order -- back in
   request order with one gather (``mdsx_gather_*``).

Over RCCL (``nccl``) the device tensors travel GPU to GPU (xGMI within a node); over ``gloo`` they
are staged through host memory (CPU tests, or several ranks sharing one GPU). The bytes moved per
step are the batch's rows once, against every shard of the node decoded and moved to every GPU
without the exchange.
"""

from __future__ import annotations

import os
from typing import Any, Callable, Optional, Sequence, Union

import numpy as np
import torch
import torch.distributed as dist

from streaming_amd.decoder import DecodedBatch, RaggedColumn, gather_sources

__all__ = ['OwnedShardGather']

# failure kinds agreed on across the group (the first failing rank's kind wins by max)
_OK, _MISSING, _INDEX, _VALUE, _OTHER = 0, 1, 2, 3, 4
_KIND_OF = ((FileNotFoundError, _MISSING), (IndexError, _INDEX), (ValueError, _VALUE))
_TYPE_OF = {_MISSING: FileNotFoundError, _INDEX: IndexError, _VALUE: ValueError,
            _OTHER: RuntimeError}


def _kind(e: BaseException) -> int:
    for t, k in _KIND_OF:
        if isinstance(e, t):
            return k
    return _OTHER


class OwnedShardGather:
    """The ``gather`` / ``locate`` / ``shards`` object :func:`streaming_amd.plugin.device_iter`
    takes, with each shard decoded by one rank of ``group`` and the rows exchanged.

    Args:
        local: this rank's gather over the dataset's shards (a
            :class:`~streaming_amd.order.DeviceSampleGather`); only the shards this rank owns are
            ever gathered -- so decoded -- through it.
        capacity: the most ids one ``gather`` call takes on any rank (the batch size).
        group: the exchange group (default: the whole world). Each shard is decoded once per
            group; a node-local group keeps the exchange on xGMI.
        owner: shard index -> rank in ``group`` (default ``g % size``).
        prepare: called with a shard index before an owned shard is gathered when its file is
            missing (``StreamingDataset.prepare_shard``: the reference's download), so that the
            owner fetches what other ranks asked for.
    """

    def __init__(self, local: Any, capacity: int, group: Optional[Any] = None,
                 owner: Optional[Callable[[int], int]] = None,
                 prepare: Optional[Callable[[int], None]] = None) -> None:
        if capacity <= 0:
            raise ValueError('OwnedShardGather: capacity must be positive')
        self.local = local
        self.shards = local.shards
        self.starts = getattr(local, 'starts', None)
        self.capacity = int(capacity)
        self.group = group
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        n = len(self.shards)
        self.owners = np.array([owner(g) if owner else g % self.size for g in range(n)], np.int64)
        if n and (self.owners.min() < 0 or self.owners.max() >= self.size):
            raise ValueError('OwnedShardGather: owner out of the group')
        self.prepare = prepare
        backend = dist.get_backend(group)
        self.staged = backend != 'nccl'  # gloo: collectives on host tensors
        self.decoded_shards: set[int] = set()  # shards this rank has gathered from (decoded)
        self._proto: Optional[DecodedBatch] = None  # the schema's empty columns

    def owned(self) -> list[int]:
        """The shards this rank decodes."""
        return [int(g) for g in np.nonzero(self.owners == self.rank)[0]]

    def locate(self, ids: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
        return self.local.locate(ids)

    # -- collectives (host-staged under gloo)
    def _wire(self) -> torch.device:
        return (torch.device('cpu') if self.staged
                else torch.device('cuda', torch.cuda.current_device()))

    def _all_to_all(self, inp: torch.Tensor, in_splits: list[int],
                    out_splits: list[int]) -> torch.Tensor:
        wire = self._wire()
        x = inp.to(wire).contiguous()
        out = torch.empty(sum(out_splits), dtype=x.dtype, device=wire)
        dist.all_to_all_single(out, x, out_splits, in_splits, group=self.group)
        return out.to(inp.device)

    def gather(self, sample_ids: Union[Sequence[int], np.ndarray, torch.Tensor]) -> DecodedBatch:
        """This rank's samples ``sample_ids`` (global ids, ``-1`` skipped), in that order, with
        every rank of the group calling at the same step (a rank out of batches calls
        :meth:`drain` instead)."""
        ids = np.asarray(torch.as_tensor(sample_ids).cpu().numpy() if isinstance(
            sample_ids, torch.Tensor) else sample_ids, np.int64).reshape(-1)
        ids = ids[ids != -1]
        if ids.size > self.capacity:
            raise ValueError(f'OwnedShardGather: {ids.size} ids exceed the capacity '
                             f'{self.capacity}')
        return self._step(ids, False)[0]

    def drain(self) -> None:
        """For a rank out of batches: serve the rows other ranks still ask for from the shards
        it owns, until every rank of the group is out (the reference's ranks may differ by a batch
        per epoch, e.g. ``device_per_stream``). Every rank calls it once its iteration ends."""
        while not self._step(np.empty(0, np.int64), True)[1]:
            pass

    def _step(self, ids: np.ndarray, done: bool) -> tuple[Optional[DecodedBatch], bool]:
        # 1. every rank's request, and whether it is out of batches (the last slot)
        req = torch.full((self.capacity + 1,), -1, dtype=torch.int64)
        req[:ids.size] = torch.from_numpy(ids)
        req[-1] = 1 if done else 0
        dev = self._wire()
        parts = [torch.empty_like(req, device=dev) for _ in range(self.size)]
        dist.all_gather(parts, req.to(dev), group=self.group)
        reqs = [p.cpu().numpy() for p in parts]
        if all(r[-1] == 1 for r in reqs):
            return None, True
        reqs = [r[:-1] for r in reqs]
        reqs = [r[r != -1] for r in reqs]
        # 2. the rows this rank owns, for every requester in its order
        send_ids, send_rows = [], []
        for r in reqs:
            mine = r[self.owners[self.locate(r)[0]] == self.rank] if r.size else r
            send_ids.append(mine)
            send_rows.append(int(mine.size))
        kind, err, out, schema = _OK, None, None, None
        todo = np.concatenate(send_ids) if send_ids else np.empty(0, np.int64)
        try:
            if todo.size:
                shard = np.unique(self.locate(todo)[0])
                if self.prepare is not None:
                    for g in shard:
                        if not os.path.exists(self.shards[int(g)]._filename()):
                            self.prepare(int(g))
                out = schema = self.local.gather(todo)
                self.decoded_shards.update(int(g) for g in shard)
                if self._proto is None:
                    self._proto = _empty_like(out)
            else:
                schema = self._schema()
        except Exception as e:  # agreed on below, so no rank waits in a collective
            kind, err = _kind(e), e
        flag = torch.tensor([kind], dtype=torch.int64, device=dev)
        dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=self.group)
        agreed = int(flag.item())
        if agreed != _OK:
            if err is not None:
                raise err
            raise _TYPE_OF[agreed](f'OwnedShardGather: another shard owner failed (kind {agreed})')
        if done:  # (served the others; nothing to receive)
            self._exchange(out, send_rows, [0] * self.size, schema)
            return None, False
        # rows this rank receives from each owner (known from the requests alone)
        owner_of = self.owners[self.locate(ids)[0]] if ids.size else np.empty(0, np.int64)
        recv_rows = [int(np.count_nonzero(owner_of == s)) for s in range(self.size)]
        recv = self._exchange(out, send_rows, recv_rows, schema)
        # 4. back in request order: received rows come grouped by owner, each group in order
        base = np.concatenate([[0], np.cumsum(recv_rows)])[:-1]
        seen = np.zeros(self.size, np.int64)
        perm = np.empty(ids.size, np.int64)
        for i, s in enumerate(owner_of):
            perm[i] = base[s] + seen[s]
            seen[s] += 1
        return gather_sources([recv], np.zeros(ids.size, np.int64), perm), False

    def _exchange(self, out: Optional[DecodedBatch], send_rows: list[int], recv_rows: list[int],
                  schema: DecodedBatch) -> DecodedBatch:
        """3. the rows to their requesters, column by column (``out``: the rows this rank sends,
        requester by requester; None: none)."""
        cols: dict[str, Union[torch.Tensor, RaggedColumn]] = {}
        ragged = [n for n, c in schema.columns.items() if isinstance(c, RaggedColumn)]
        sent_bytes = {}
        if ragged:
            counts = torch.zeros((self.size, len(ragged)), dtype=torch.int64)
            for j, name in enumerate(ragged):
                col = out.columns[name] if out is not None else None
                ends = (col.offsets.cpu().numpy() if col is not None
                        else np.zeros(1, np.int64))
                bounds = np.concatenate([[0], np.cumsum(send_rows)])
                sent_bytes[name] = [int(ends[bounds[q + 1]] - ends[bounds[q]])
                                    for q in range(self.size)]
                counts[:, j] = torch.tensor(sent_bytes[name], dtype=torch.int64)
            got = self._all_to_all(counts.reshape(-1), [len(ragged)] * self.size,
                                   [len(ragged)] * self.size).reshape(self.size, len(ragged))
            recv_bytes = {name: [int(x) for x in got[:, j].tolist()]
                          for j, name in enumerate(ragged)}
        for name, proto in schema.columns.items():
            col = out.columns[name] if out is not None else None
            if isinstance(proto, RaggedColumn):
                lens = (torch.diff(col.offsets) if col is not None else
                        torch.zeros(0, dtype=torch.int64, device=proto.offsets.device))
                rlens = self._all_to_all(lens, send_rows, recv_rows)
                vals = col.values[:int(col.offsets[-1])] if col is not None else proto.values[:0]
                rvals = self._all_to_all(vals, sent_bytes[name], recv_bytes[name])
                rflags = None
                if proto.flags is not None:
                    fl = col.flags if col is not None else proto.flags[:0]
                    rflags = self._all_to_all(fl, send_rows, recv_rows)
                offs = torch.zeros(rlens.numel() + 1, dtype=torch.int64, device=rlens.device)
                torch.cumsum(rlens, 0, out=offs[1:])
                cols[name] = RaggedColumn(rvals, offs, rflags)
            else:
                x = col if col is not None else proto[:0]
                row_bytes = int(np.prod(x.shape[1:], dtype=np.int64)) * x.element_size()
                flat = x.contiguous().view(torch.uint8).reshape(-1)
                r = self._all_to_all(flat, [n * row_bytes for n in send_rows],
                                     [n * row_bytes for n in recv_rows])
                cols[name] = r.view(x.dtype).reshape(sum(recv_rows), *x.shape[1:])
        return DecodedBatch(cols, sum(recv_rows))

    def _schema(self) -> DecodedBatch:
        """Empty columns of the dataset's schema, for a rank that sends nothing this step: from
        an earlier step, else the decode of a shard of no samples under the readers' plan (no
        sample is read, so no malformed one can fail it); for a gather whose shards carry no
        plan, one sample of a shard this rank owns."""
        if self._proto is None:
            plan = getattr(self.shards[0], 'plan', None) if self.shards else None
            if plan is not None:
                from streaming_amd.decoder import decode_batch, stage_shards
                empty = np.array([0, 8], np.uint32).tobytes()  # count 0, offsets [8] (the end)
                dev = torch.device('cuda', torch.cuda.current_device())
                self._proto = decode_batch(plan, stage_shards([empty], [0], plan, device=dev))
            else:
                mine = [g for g in self.owned() if self.shards[g].samples] or [0]
                first = int(self.starts[mine[0]]) if self.starts is not None else 0
                self._proto = _empty_like(self.local.gather(np.array([first], np.int64)))
                self.decoded_shards.add(mine[0])
        return self._proto


def _empty_like(b: DecodedBatch) -> DecodedBatch:
    """No rows, the same columns (dtypes, row shapes, devices)."""
    cols: dict[str, Union[torch.Tensor, RaggedColumn]] = {}
    for name, c in b.columns.items():
        if isinstance(c, RaggedColumn):
            cols[name] = RaggedColumn(c.values[:0].clone(), c.offsets[:1].clone().zero_(),
                                      c.flags[:0].clone() if c.flags is not None else None)
        else:
            cols[name] = c[:0].clone()
    return DecodedBatch(cols, 0)
