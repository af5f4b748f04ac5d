"""Device MDS shard encoder: columns on the GPU -> MDS shard files.

The reverse byte shuffle of the decoder. The reference writes one sample at a time:
``MDSWriter.encode_sample`` (u32 heads of the variable columns, then every column's bytes;
``streaming/base/format/mds/writer.py:92-117``), ``Writer.write`` flushes a shard when
``size_limit < shard_size + sample_size + 4`` (``streaming/base/format/base/writer.py:248-269``)
and ``encode_joint_shard`` lays out ``N | offsets[N+1] | config | samples``
(``mds/writer.py:133-144``). Here whole batches of columns in the decoder's output layout
(fixed ``[rows, ...]`` tensors, :class:`RaggedColumn` values + offsets) are encoded by the
``mdsx_encode_*`` kernels into a device batch laid out like a decode batch (so it can be decoded
in place, or copied to files), byte-identical to the reference writer's shards.

The shard split is the reference's greedy rule restated as a prefix rule: with
``cum4[i]`` = bytes of samples ``0..i-1`` plus 4 per sample, a shard starting at row ``b`` takes
rows up to the last ``e`` with ``cum4[e] - cum4[b] <= size_limit - (8 + len(config))``, and at
least one row (the sample that triggered a flush is always appended). The writer's very first
sample, if alone too large, makes the reference flush an empty shard first; kept here.
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Optional, Sequence, Union

import numpy as np
import torch

from streaming_amd import _native
from streaming_amd._native import ColumnIn
from streaming_amd.decoder import (DeviceBatch, Plan, RaggedColumn, _check, _layout, _status_error,
                                   _tables)

__all__ = [
    'split_shards', 'EncodedBatch', 'BatchEncoder', 'encode_batch', 'concat_columns',
    'slice_columns'
]

Column = Union[torch.Tensor, RaggedColumn]


def split_shards(cum4: np.ndarray, size_limit: Optional[int], extra_per_shard: int,
                 fresh: bool = True) -> list[tuple[int, int]]:
    """Shard row ranges of the reference writer's greedy split.

    Args:
        cum4: int64[rows + 1], bytes of samples ``0..i-1`` plus 4 per sample (the
            ``extra_bytes_per_sample`` of ``MDSWriter``, ``mds/writer.py:54``).
        size_limit: shard size limit, or None / 0 for no limit.
        extra_per_shard: ``4 + 4 + len(config)`` (``mds/writer.py:79``).
        fresh: the writer has cached no sample yet (an oversized first sample then flushes an
            empty shard, as ``Writer.write`` does).

    Returns:
        ``[(begin, end), ...]`` covering ``[0, rows)``; the last range is the open shard.
    """
    rows = len(cum4) - 1
    if rows <= 0:
        return []
    if not size_limit:
        return [(0, rows)]
    cap = int(size_limit) - int(extra_per_shard)
    bounds = []
    if fresh and int(cum4[1] - cum4[0]) > cap:
        bounds.append((0, 0))
    b = 0
    while b < rows:
        e = int(np.searchsorted(cum4, cum4[b] + cap, side='right')) - 1
        e = min(max(e, b + 1), rows)
        bounds.append((b, e))
        b = e
    return bounds


@dataclass
class EncodedBatch:
    """Shards encoded on the device: ``batch`` holds shard ``s`` at
    ``batch.buffer[batch.offsets[s] : batch.offsets[s] + batch.sizes[s]]`` (decodable in
    place); ``bounds[s]`` = the input rows it holds."""
    batch: DeviceBatch
    bounds: list[tuple[int, int]]

    def __len__(self) -> int:
        return len(self.bounds)

    def shard(self, s: int) -> torch.Tensor:
        o = self.batch.offsets[s]
        return self.batch.buffer[o:o + self.batch.sizes[s]]

    def shard_bytes(self, s: int) -> bytes:
        return self.shard(s).cpu().numpy().tobytes()

    def decode_batch(self, plan: Plan) -> DeviceBatch:
        """The encoded shards as a decode batch of ``plan`` (same buffer, the tile table rebuilt
        for the decoder's tile size)."""
        b = self.batch
        tr = plan.tile_rows_for(int(b.buffer.numel()), sum(b.samples))  # C: batch->bytes
        if b.tile_rows == tr:
            return b
        raw, tile_shard, row0, rows, tiles = _tables(b.sizes, b.samples, b.offsets, tr)
        dev = b.device
        return DeviceBatch(b.buffer, torch.from_numpy(raw).to(dev),
                           torch.from_numpy(tile_shard).to(dev) if tiles else torch.zeros(
                               1, dtype=torch.int32, device=dev), b.offsets, b.sizes, b.samples,
                           row0, tiles, rows, tr)


def _row_count(plan: Plan, columns: dict[str, Column]) -> int:
    counts = {len(v) if isinstance(v, RaggedColumn) else int(v.shape[0]) for v in columns.values()}
    if len(counts) != 1:
        raise ValueError(f'columns differ in row count: {sorted(counts)}')
    missing = [c.name for c in plan.columns if c.name not in columns]
    if missing:
        raise KeyError(f'missing columns: {missing}')
    return counts.pop()


def _column_ins(plan: Plan, columns: dict[str, Column], rows: int):
    """``mdsx_column_in`` records in plan order (+ the tensors they point into)."""
    arr = (ColumnIn * max(len(plan.columns), 1))()
    keep = []
    for c in plan.columns:
        v = columns[c.name]
        rec = arr[c.index]
        if c.is_fixed:
            if isinstance(v, RaggedColumn):
                raise TypeError(f'column {c.name!r} ({c.encoding}) is fixed-size: pass a tensor')
            t = v.contiguous()
            nbytes = t.numel() * t.element_size()
            if nbytes != rows * c.row_bytes:
                raise ValueError(f'column {c.name!r}: {nbytes} bytes for {rows} rows of '
                                 f'{c.row_bytes} bytes')
            rec.data = t.data_ptr() if nbytes else None
            rec.bytes = nbytes
            keep.append(t)
        else:
            if not isinstance(v, RaggedColumn):
                raise TypeError(f'column {c.name!r} ({c.encoding}) is variable-size: pass a '
                                f'RaggedColumn (values, offsets)')
            vals = v.values.contiguous().view(torch.uint8)
            offs = v.offsets.contiguous()
            if offs.dtype != torch.int64 or offs.numel() != rows + 1:
                raise ValueError(f'column {c.name!r}: offsets must be int64[{rows + 1}]')
            rec.data = vals.data_ptr() if vals.numel() else None
            rec.offsets = offs.data_ptr()
            rec.bytes = vals.numel()
            keep += [vals, offs]
    return arr, keep


class BatchEncoder:
    """Sizes, shard split and batch layout of ``columns`` (computed once), then
    :meth:`run` launches the encode kernels (repeatable, e.g. for timing). Arguments as for
    :func:`encode_batch`."""

    def __init__(self,
                 plan: Plan,
                 columns: dict[str, Column],
                 config: bytes,
                 size_limit: Optional[int] = 1 << 26,
                 fresh: bool = True,
                 final: bool = True) -> None:
        lib = self._lib = _native.lib()
        self.plan = plan
        rows = _row_count(plan, columns)
        first = next(iter(columns.values()))
        dev = first.values.device if isinstance(first, RaggedColumn) else first.device
        self.stream = torch.cuda.current_stream(dev).cuda_stream
        self.ins, self._keep = _column_ins(plan, columns, rows)
        self.ws = torch.zeros(int(lib.mdsx_encode_workspace_bytes()), dtype=torch.uint8,
                              device=dev)
        self.cum = torch.empty(rows + 1, dtype=torch.int64, device=dev)
        _check(lib.mdsx_encode_sizes(plan.handle, self.ins, rows, self.cum.data_ptr(),
                                     self.ws.data_ptr(), self.ws.numel(), self.stream),
               'mdsx_encode_sizes')
        if plan.num_var:
            cum_host = self.cum.cpu().numpy()  # the split needs the sizes (host sync)
            st = self.status()
            if st.code != 0:
                raise ValueError(f'encode: bad variable column '
                                 f'{plan.columns[st.column].name!r} at row {st.row} (offsets not '
                                 f'monotone, outside the values, or a row of 2^32 bytes or more)')
        else:
            cum_host = np.arange(rows + 1, dtype=np.int64) * plan.fixed_row_bytes()
        cum4 = cum_host + 4 * np.arange(rows + 1, dtype=np.int64)
        bounds = split_shards(cum4, size_limit, 8 + len(config), fresh)
        if not final and bounds:
            bounds = bounds[:-1]
        self.bounds = bounds
        self.consumed = bounds[-1][1] if bounds else 0
        self.batch: Optional[DeviceBatch] = None
        if not bounds:
            return
        sizes = [8 + 4 * (e - b) + len(config) + int(cum_host[e] - cum_host[b]) for b, e in bounds]
        if max(sizes) >= 2**32:
            raise ValueError('encode: a shard of 4 GiB or more cannot hold u32 offsets')
        samples = [e - b for b, e in bounds]
        offsets, total = _layout(sizes)
        raw, tile_shard, row0, nrows, tiles = _tables(sizes, samples, offsets,
                                                      plan.encode_tile_rows)
        descs = torch.from_numpy(raw).to(dev)
        tiles_t = torch.from_numpy(tile_shard).to(dev) if tiles else torch.zeros(
            1, dtype=torch.int32, device=dev)
        self.batch = DeviceBatch(torch.empty(total, dtype=torch.uint8, device=dev), descs,
                                 tiles_t, offsets, sizes, samples, row0, tiles, nrows,
                                 plan.encode_tile_rows)
        self._abi = self.batch.abi()
        self.config = config
        self.cfg = torch.frombuffer(bytearray(config), dtype=torch.uint8).to(dev) \
            if config else None

    def status(self) -> _native.Status:
        return _native.Status.from_buffer_copy(self.ws[:16].cpu().numpy().tobytes())

    def run(self, check: bool = True) -> Optional[EncodedBatch]:
        if self.batch is None:
            return None
        _check(
            self._lib.mdsx_encode_shards(self.plan.handle, ctypes.byref(self._abi), self.ins,
                                         self.cum.data_ptr(),
                                         self.cfg.data_ptr() if self.cfg is not None else None,
                                         len(self.config), self.ws.data_ptr(), self.ws.numel(),
                                         self.stream), 'mdsx_encode_shards')
        if check:
            st = self.status()
            if st.code != 0:
                raise _status_error(st, self.plan)
        return EncodedBatch(self.batch, self.bounds)


def encode_batch(plan: Plan,
                 columns: dict[str, Column],
                 config: bytes,
                 size_limit: Optional[int] = 1 << 26,
                 fresh: bool = True,
                 final: bool = True,
                 check: bool = True) -> tuple[Optional[EncodedBatch], int]:
    """Encode rows of ``columns`` into MDS shards on the device.

    Args:
        plan: the schema (column order = sorted names, as ``MDSWriter`` writes).
        columns: name -> fixed tensor ``[rows, ...]`` or :class:`RaggedColumn` (raw encoded bytes
            of each row, i.e. what ``mds_encode`` returns for the column's encoding).
        config: the shard config JSON (``shard_config_bytes``).
        size_limit: shard size limit (``Writer.size_limit``).
        fresh: no sample was written before these rows (see :func:`split_shards`).
        final: also encode the last (open) shard; otherwise its rows are left over.

    Returns:
        ``(encoded, consumed)``: the encoded shards (None if there are none) and the number of
        leading rows they hold.
    """
    enc = BatchEncoder(plan, columns, config, size_limit, fresh, final)
    return enc.run(check), enc.consumed


def slice_columns(columns: dict[str, Column], begin: int, end: int) -> dict[str, Column]:
    """Rows ``[begin, end)`` of every column (views; ragged offsets keep their base)."""
    out = {}
    for name, v in columns.items():
        if isinstance(v, RaggedColumn):
            out[name] = RaggedColumn(v.values, v.offsets[begin:end + 1],
                                     v.flags[begin:end] if v.flags is not None else None)
        else:
            out[name] = v[begin:end]
    return out


def concat_columns(parts: Sequence[dict[str, Column]]) -> dict[str, Column]:
    """Row-wise concatenation of column dicts (ragged values re-packed, offsets rebased)."""
    if len(parts) == 1:
        return parts[0]
    out = {}
    for name in parts[0]:
        vs = [p[name] for p in parts]
        if isinstance(vs[0], RaggedColumn):
            vals, offs, base = [], [], 0
            for i, v in enumerate(vs):
                o0, o1 = int(v.offsets[0]), int(v.offsets[-1])
                vals.append(v.values[o0:o1])
                o = v.offsets - o0 + base
                offs.append(o if i == len(vs) - 1 else o[:-1])
                base += o1 - o0
            out[name] = RaggedColumn(torch.cat(vals), torch.cat(offs))
        else:
            out[name] = torch.cat(vs)
    return out
