"""Whole-shard device decode: plans, device shard batches and decoded columns.

This is the host side of the hot path. It replaces, for whole shards at once, the per-sample
chain ``Reader.get_item -> MDSReader.get_sample_data -> MDSReader.decode_sample -> mds_decode``
(``streaming/base/format/base/reader.py:310-320``, ``format/mds/reader.py:103-149``,
``format/mds/encodings.py:760-773``):

* :class:`Plan` -- the schema of a shard (``MDSReader.from_json``, ``mds/reader.py:59-86``),
  compiled once by ``mdsx_plan_create``;
* :class:`DeviceBatch` -- one or more shard files staged in a single HBM buffer
  (``mdsx_shard_desc`` table + tile table);
* :func:`decode_batch` / :class:`BatchDecoder` -- ``mdsx_scan_shards`` + ``mdsx_decode_shards``
  on the current torch stream, giving torch tensors: fixed columns as ``dtype[rows, *shape]``,
  ragged columns (bytes / str / dynamic ndarray / host-object encodings) as
  :class:`RaggedColumn` (packed ``uint8`` values + ``int64`` offsets [+ str validity flags]).

Every decode goes through libmdsx.so; there is no CPU path.
"""

from __future__ import annotations

import ctypes
import os
import math
from dataclasses import dataclass, field
from typing import Optional, Sequence, Union

import numpy as np
import torch

from streaming_amd import _native
from streaming_amd._native import (BATCH_PAD, KIND_BYTES, KIND_FIXED, KIND_NDARRAY, KIND_STR,
                                   Batch, ColumnOut, ShardDesc)
from streaming_amd.encodings import EncodingInfo, parse_encoding

__all__ = [
    'Plan', 'DeviceBatch', 'RaggedColumn', 'DecodedBatch', 'BatchDecoder', 'ScanAheadDecoder',
    'decode_batch',
    'make_batch', 'stage_shards', 'torch_dtype', 'output_bytes', 'NdarrayMeta', 'ndarray_meta'
]

_TORCH_DTYPES = {
    'uint8': torch.uint8,
    'int8': torch.int8,
    'uint16': torch.uint16,
    'int16': torch.int16,
    'float16': torch.float16,
    'uint32': torch.uint32,
    'int32': torch.int32,
    'float32': torch.float32,
    'uint64': torch.uint64,
    'int64': torch.int64,
    'float64': torch.float64,
}


def torch_dtype(name: str) -> torch.dtype:
    return _TORCH_DTYPES[name]


def _check(code: int, where: str) -> None:
    _native.raise_for_code(code, where)


@dataclass
class ColumnPlan:
    """One column of a :class:`Plan`."""
    index: int
    name: str
    encoding: str
    info: Optional[EncodingInfo]
    kind: int  # _native.KIND_*
    row_bytes: int  # fixed columns
    elem_bytes: int

    @property
    def is_fixed(self) -> bool:
        return self.kind == KIND_FIXED

    def tensor_view(self) -> tuple[torch.dtype, tuple[int, ...]]:
        """dtype and per-row shape of a fixed column's output tensor."""
        info = self.info
        if info is not None and info.dtype is not None and info.shape is not None and \
                info.size == self.row_bytes:
            return torch_dtype(info.dtype), tuple(info.shape)
        return torch.uint8, (self.row_bytes,)


class Plan:
    """A compiled MDS schema: ``mdsx_plan_create`` over (encodings, column_sizes).

    Args:
        column_names: shard column names (sorted, as written by ``MDSWriter``).
        column_encodings: encoding strings (``index.json`` ``column_encodings``).
        column_sizes: fixed sizes or None (``index.json`` ``column_sizes``).
    """

    def __init__(self, column_names: Sequence[str], column_encodings: Sequence[str],
                 column_sizes: Sequence[Optional[int]]) -> None:
        if not (len(column_names) == len(column_encodings) == len(column_sizes)):
            raise ValueError('column_names, column_encodings and column_sizes differ in length')
        self._lib = _native.lib()
        n = len(column_encodings)
        enc_bytes = [e.encode('utf-8') for e in column_encodings]
        encs = (ctypes.c_char_p * max(n, 1))(*enc_bytes)
        sizes = (ctypes.c_int64 * max(n, 1))(*[int(s) if s else 0 for s in column_sizes])
        handle = ctypes.c_void_p()
        _check(self._lib.mdsx_plan_create(encs, sizes, n, ctypes.byref(handle)),
               'mdsx_plan_create')
        self._handle = handle
        self.key = (tuple(column_names), tuple(column_encodings),
                    tuple(int(s) if s else 0 for s in column_sizes))
        self.columns: list[ColumnPlan] = []
        for i, (name, enc) in enumerate(zip(column_names, column_encodings)):
            kind, row_bytes, elem = ctypes.c_int(), ctypes.c_int64(), ctypes.c_int()
            _check(
                self._lib.mdsx_plan_column(handle, i, ctypes.byref(kind), ctypes.byref(row_bytes),
                                           ctypes.byref(elem)), 'mdsx_plan_column')
            try:
                info = parse_encoding(enc)
            except Exception:  # the C++ parser already accepted it; keep raw bytes semantics
                info = None
            self.columns.append(
                ColumnPlan(i, name, enc, info, kind.value, row_bytes.value, elem.value))
        self.num_var = self._lib.mdsx_plan_num_var(handle)
        self.tile_rows = self._lib.mdsx_plan_tile_rows(handle)
        self.encode_tile_rows = self._lib.mdsx_plan_encode_tile_rows(handle)
        self.is_safe = bool(self._lib.mdsx_plan_is_safe(handle))

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._handle

    @property
    def names(self) -> list[str]:
        return [c.name for c in self.columns]

    def tile_rows_for(self, shard_bytes: int, rows: int) -> int:
        """Rows per tile of a decode batch of ``rows`` samples in ``shard_bytes`` bytes of shard
        files (``mdsx_plan_tile_rows_for``: ragged plans size tiles to the LDS stage)."""
        tr = int(self._lib.mdsx_plan_tile_rows_for(self._handle, int(shard_bytes), int(rows)))
        _check(min(tr, 0), 'mdsx_plan_tile_rows_for')
        return tr

    def workspace_bytes(self, batch: 'DeviceBatch') -> int:
        return int(self._lib.mdsx_workspace_bytes(self._handle, ctypes.byref(batch.abi())))

    def fixed_row_bytes(self) -> int:
        return sum(c.row_bytes for c in self.columns if c.is_fixed)

    def __del__(self) -> None:
        handle = getattr(self, '_handle', None)
        if handle is not None and handle.value:
            try:
                self._lib.mdsx_plan_destroy(handle)
            except Exception:
                pass
            self._handle = ctypes.c_void_p()


@dataclass
class DeviceBatch:
    """Shard files resident in one device buffer, plus the descriptor and tile tables.

    Attributes:
        buffer: uint8 device tensor; shard s occupies ``buffer[offsets[s]:offsets[s]+sizes[s]]``.
        descs: device tensor holding ``nshards`` ``mdsx_shard_desc`` records.
        tile_shard: device int32 tensor (read as uint32), the shard of each tile.
    """
    buffer: torch.Tensor
    descs: torch.Tensor
    tile_shard: torch.Tensor
    offsets: list[int]
    sizes: list[int]
    samples: list[int]
    row0: list[int]
    ntiles: int
    total_rows: int
    tile_rows: int

    @property
    def nshards(self) -> int:
        return len(self.sizes)

    @property
    def shard_bytes(self) -> int:
        return int(sum(self.sizes))

    @property
    def device(self) -> torch.device:
        return self.buffer.device

    def abi(self) -> Batch:
        """The ``mdsx_batch`` view of this batch (device pointers)."""
        b = Batch()
        b.data = self.buffer.data_ptr()
        b.bytes = int(self.buffer.numel())
        b.shards = self.descs.data_ptr()
        b.tile_shard = self.tile_shard.data_ptr()
        b.nshards = self.nshards
        b.ntiles = self.ntiles
        b.rows = self.total_rows
        b.tile_rows = self.tile_rows
        return b


def _layout(sizes: Sequence[int]) -> tuple[list[int], int]:
    offsets, pos = [], BATCH_PAD
    for size in sizes:
        offsets.append(pos)
        pos = (pos + int(size) + 255) & ~255
    return offsets, pos + BATCH_PAD


def _tables(sizes: Sequence[int], samples: Sequence[int], offsets: Sequence[int],
            tile_rows: int) -> tuple[np.ndarray, np.ndarray, list[int], int, int]:
    descs = (ShardDesc * max(len(sizes), 1))()
    tile_shard, row0, rows, tiles = [], [], 0, 0
    for s, (size, n, off) in enumerate(zip(sizes, samples, offsets)):
        nt = math.ceil(int(n) / tile_rows)
        d = descs[s]
        d.offset, d.bytes, d.row0, d.samples, d.tile0 = off, int(size), rows, int(n), tiles
        row0.append(rows)
        tile_shard.extend([s] * nt)
        rows += int(n)
        tiles += nt
    raw = np.frombuffer(bytes(descs), np.uint8)[:32 * len(sizes)].copy()
    return raw, np.array(tile_shard, np.int32), row0, rows, tiles


def make_batch(plan: Plan,
               sizes: Sequence[int],
               samples: Sequence[int],
               device: Union[str, torch.device, None] = None) -> DeviceBatch:
    """Allocate a zeroed batch buffer laid out for shards of ``sizes`` bytes (filled by the
    caller at ``batch.offsets[s]``) with its descriptor and tile tables."""
    if len(sizes) != len(samples):
        raise ValueError('sizes and samples differ in length')
    if not len(sizes):
        raise ValueError('a batch needs at least one shard')
    device = torch.device(device or 'cuda')
    if device.type == 'cuda' and device.index is None:
        device = torch.device('cuda', torch.cuda.current_device())
    sizes = [int(x) for x in sizes]
    offsets, total = _layout(sizes)
    buffer = torch.zeros(total, dtype=torch.uint8, device=device)
    # tiles sized from the buffer's bytes, the batch->bytes the C side picks the decode from
    tr = plan.tile_rows_for(total, sum(int(n) for n in samples))
    raw, tile_shard, row0, rows, tiles = _tables(sizes, samples, offsets, tr)
    descs = torch.from_numpy(raw).to(device)
    tiles_t = torch.from_numpy(tile_shard).to(device) if tiles else torch.zeros(
        1, dtype=torch.int32, device=device)
    return DeviceBatch(buffer, descs, tiles_t, offsets, sizes, [int(n) for n in samples], row0,
                       tiles, rows, tr)


def stage_shards(shards: Sequence[Union[bytes, bytearray, memoryview, np.ndarray, torch.Tensor]],
                 samples: Sequence[int],
                 plan: Plan,
                 device: Union[str, torch.device, None] = None,
                 pin: bool = True) -> DeviceBatch:
    """Copy shard files into one device buffer (host -> pinned staging -> HBM).

    ``shards`` may also be uint8 device tensors already in HBM (copied device-to-device).
    """
    if len(shards) != len(samples):
        raise ValueError('shards and samples differ in length')
    sizes = [int(x.numel()) if isinstance(x, torch.Tensor) else len(memoryview(x).cast('B'))
             for x in shards]
    batch = make_batch(plan, sizes, samples, device)
    host = [(i, x) for i, x in enumerate(shards) if not isinstance(x, torch.Tensor)]
    if host:
        lo = batch.offsets[host[0][0]]
        hi = batch.offsets[host[-1][0]] + sizes[host[-1][0]]
        staging = torch.empty(hi - lo, dtype=torch.uint8,
                              pin_memory=pin and batch.device.type == 'cuda')
        view = staging.numpy()
        for i, x in host:
            o = batch.offsets[i] - lo
            view[o:o + sizes[i]] = np.frombuffer(memoryview(x).cast('B'), np.uint8)
        # one H2D over the staged span; gaps between shards are never read as sample bytes
        batch.buffer[lo:hi].copy_(staging, non_blocking=True)
    for i, x in enumerate(shards):
        if isinstance(x, torch.Tensor):
            batch.buffer[batch.offsets[i]:batch.offsets[i] + sizes[i]].copy_(
                x.reshape(-1).view(torch.uint8), non_blocking=True)
    if host:
        torch.cuda.current_stream(batch.device).synchronize()  # staging must outlive the copy
    return batch


@dataclass
class RaggedColumn:
    """A variable-size column: row i is ``values[offsets[i]:offsets[i+1]]``.

    ``flags`` (str columns) is 1 where the row is not well-formed UTF-8, i.e. where the reference's
    ``bytes.decode('utf-8')`` raises (encodings.py:80-81).
    """
    values: torch.Tensor
    offsets: torch.Tensor
    flags: Optional[torch.Tensor] = None

    def __len__(self) -> int:
        return int(self.offsets.numel()) - 1


@dataclass
class NdarrayMeta:
    """Per-row header facts of a dynamic ndarray column, parsed on the device
    (``mdsx_ndarray_meta`` / ``mdsx_ndarray_shapes``; NDArray.decode, encodings.py:270-305).

    Row i's values are ``values[data_offset[i] : data_offset[i] + numel[i] * itemsize]`` of
    dtype id ``dtype[i]`` (encodings.py:131-143) and shape ``shape[i, :ndim[i]]``; ``bad[i]`` is 1
    where the reference's decode raises.
    """
    dtype: torch.Tensor          # uint8[rows]
    ndim: torch.Tensor           # uint8[rows]
    data_offset: torch.Tensor    # int64[rows]
    numel: torch.Tensor          # int64[rows]
    bad: torch.Tensor            # uint8[rows]
    shape: torch.Tensor          # int64[rows, max_ndim] (padded with 1)

    def row(self, col: 'RaggedColumn', i: int) -> torch.Tensor:
        """Row i as a device tensor of its dtype and shape (a copy; values may be unaligned)."""
        if int(self.bad[i]):
            raise ValueError(f'row {i}: malformed ndarray')
        from streaming_amd.encodings import VALUE_DTYPES
        dt = torch_dtype(VALUE_DTYPES[int(self.dtype[i])])
        n = int(self.numel[i])
        item = torch.empty(0, dtype=dt).element_size()
        o = int(self.data_offset[i])
        shape = [int(d) for d in self.shape[i, :int(self.ndim[i])]]
        return col.values[o:o + n * item].clone().view(dt).reshape(shape)


def ndarray_meta(col: 'RaggedColumn', dtype_id: int = 0) -> NdarrayMeta:
    """Parse the headers of a decoded dynamic ndarray column on the device. ``dtype_id`` is the
    static value dtype id of ``ndarray:<dtype>`` columns, 0 for ``ndarray``."""
    lib = _native.lib()
    rows = len(col)
    dev = col.offsets.device
    stream = torch.cuda.current_stream(dev).cuda_stream
    u8 = dict(dtype=torch.uint8, device=dev)
    i64 = dict(dtype=torch.int64, device=dev)
    dtype, ndim, bad = (torch.empty(rows, **u8) for _ in range(3))
    data_offset, numel = torch.empty(rows, **i64), torch.empty(rows, **i64)
    max_ndim = torch.zeros(1, dtype=torch.int32, device=dev)
    vals = col.values.data_ptr() if col.values.numel() else None
    _check(
        lib.mdsx_ndarray_meta(vals, col.offsets.data_ptr(), rows, dtype_id, dtype.data_ptr(),
                              ndim.data_ptr(), data_offset.data_ptr(), numel.data_ptr(),
                              bad.data_ptr(), max_ndim.data_ptr(), stream), 'mdsx_ndarray_meta')
    width = int(max_ndim.item())  # sizes the shape table (host sync)
    shape = torch.ones((rows, width), **i64)
    _check(
        lib.mdsx_ndarray_shapes(vals, col.offsets.data_ptr(), rows, dtype_id, width,
                                shape.data_ptr() if shape.numel() else None, stream),
        'mdsx_ndarray_shapes')
    return NdarrayMeta(dtype, ndim, data_offset, numel, bad, shape)


@dataclass
class DecodedBatch:
    """Decoded columns of a :class:`DeviceBatch` (device tensors). ``stream``: the stream the
    columns were written on (the decode's, or the gather's that made them; None: unknown,
    taken as the reader's current stream)."""
    columns: dict[str, Union[torch.Tensor, RaggedColumn]]
    rows: int
    row0: list[int] = field(default_factory=list)
    stream: Optional[torch.cuda.Stream] = None
    sample_ids: Optional[np.ndarray] = None  # the global ids of the rows (device_iter batches)

    def __len__(self) -> int:
        return int(self.rows)

    def tensors(self) -> list[torch.Tensor]:
        out = []
        for col in self.columns.values():
            if isinstance(col, RaggedColumn):
                out += [t for t in (col.values, col.offsets, col.flags) if t is not None]
            else:
                out.append(col)
        return out

    def __getitem__(self, name: str) -> Union[torch.Tensor, RaggedColumn]:
        return self.columns[name]

    def gather(self, ids: Union[torch.Tensor, Sequence[int], np.ndarray],
               check: bool = True) -> 'DecodedBatch':
        """Rows ``ids`` of every column, in that order (the device batch gather of the
        reference's per-sample iteration over sample ids, ``dataset.py:1430-1473``; ids of -1,
        the reference's padding, are skipped). Runs the ``mdsx_gather_*`` kernels."""
        lib = _native.lib()
        first = next(iter(self.columns.values()))
        dev = first.values.device if isinstance(first, RaggedColumn) else first.device
        _require_device_columns([self])
        _on_current_stream([self], dev)
        idx = torch.as_tensor(ids, dtype=torch.int64).to(dev).reshape(-1)
        idx = idx[idx != -1].contiguous()
        m = int(idx.numel())
        ws = torch.zeros(int(lib.mdsx_gather_workspace_bytes(m)), dtype=torch.uint8, device=dev)
        stream = torch.cuda.current_stream(dev).cuda_stream
        out: dict[str, Union[torch.Tensor, RaggedColumn]] = {}
        for name, col in self.columns.items():
            if isinstance(col, RaggedColumn):
                offs = torch.empty(m + 1, dtype=torch.int64, device=dev)
                total = torch.zeros(1, dtype=torch.int64, device=dev)
                _check(
                    lib.mdsx_gather_ragged_scan(col.offsets.data_ptr(), self.rows,
                                                idx.data_ptr() if m else None, m, offs.data_ptr(),
                                                ws.data_ptr(), ws.numel(), total.data_ptr(),
                                                stream), 'mdsx_gather_ragged_scan')
                cap = int(total.item())  # sizes the values buffer (host sync)
                vals = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
                flags = torch.zeros(m, dtype=torch.uint8, device=dev) if col.flags is not None \
                    else None
                _check(
                    lib.mdsx_gather_ragged_copy(
                        col.values.data_ptr() if col.values.numel() else None,
                        col.offsets.data_ptr(), col.flags.data_ptr() if flags is not None else None,
                        self.rows, idx.data_ptr() if m else None, m,
                        vals.data_ptr() if cap else None, cap, offs.data_ptr(),
                        flags.data_ptr() if flags is not None else None, ws.data_ptr(),
                        ws.numel(), stream), 'mdsx_gather_ragged_copy')
                out[name] = RaggedColumn(vals[:cap], offs, flags)
            else:
                row_shape = tuple(col.shape[1:])
                dst = torch.empty((m, ) + row_shape, dtype=col.dtype, device=dev)
                row_bytes = col[0].numel() * col.element_size() if col.shape[0] else \
                    int(np.prod(row_shape, dtype=np.int64)) * col.element_size()
                if m:
                    _check(
                        lib.mdsx_gather_fixed(col.data_ptr(), self.rows, row_bytes, idx.data_ptr(),
                                              m, dst.data_ptr(), ws.data_ptr(), ws.numel(),
                                              stream), 'mdsx_gather_fixed')
                out[name] = dst
        if check:
            st = _native.Status.from_buffer_copy(ws[:16].cpu().numpy().tobytes())
            if st.code != 0:
                raise IndexError(f'sample id out of range at position {st.row} of the gather')
        return DecodedBatch(out, m, stream=torch.cuda.current_stream(dev))


def _require_device_columns(batches: Sequence['DecodedBatch']) -> None:
    """The gather kernels read their sources through device pointers: a host tensor's address
    must never reach them (it would fault the GPU), so CPU columns are refused here."""
    for b in batches:
        for name, col in b.columns.items():
            for t in ((col.values, col.offsets) if isinstance(col, RaggedColumn) else (col, )):
                if t.device.type != 'cuda':
                    raise ValueError(f'gather: column {name!r} is not on the GPU ({t.device}); '
                                     'the device gather reads decoded device tensors only')


def _on_current_stream(batches: Sequence['DecodedBatch'], dev: torch.device) -> None:
    """A gather reads its sources on the current stream. A source decoded on another stream:
    the current stream first waits for that stream's work (the decode), and its tensors are
    marked in use by the current stream (``record_stream``), so that freeing them -- a cache
    eviction -- cannot hand their memory to a new allocation on the decode's stream while the
    gather still reads it."""
    cur = torch.cuda.current_stream(dev)
    for b in batches:
        s = b.stream
        if s is None or s == cur:
            continue
        cur.wait_stream(s)
        for t in b.tensors():
            t.record_stream(cur)


def gather_sources(sources: Sequence[DecodedBatch], src: np.ndarray, rows: np.ndarray,
                   check: bool = True) -> DecodedBatch:
    """Output row k = row ``rows[k]`` of ``sources[src[k]]`` (decoded shards of one schema), for
    every column in ONE launch sequence (``mdsx_gather_*_multi``): the device side of the
    reference's per-sample ``get_item`` over a worker's ids across shards
    (``dataset.py:1430-1473``; ``Spanner``, ``spanner.py:40-59``, gives ``src`` / ``rows``).
    One host sync (the ragged totals that size the value buffers, read with the status)."""
    if not sources:
        raise ValueError('gather_sources: no sources')
    lib = _native.lib()
    src = np.asarray(src, np.int64).reshape(-1)
    rows = np.asarray(rows, np.int64).reshape(-1)
    if src.shape != rows.shape:
        raise ValueError('gather_sources: src and rows differ in length')
    m, nsrc = int(src.size), len(sources)
    _require_device_columns(sources)
    names = list(sources[0].columns)
    first = sources[0].columns[names[0]]
    dev = first.values.device if isinstance(first, RaggedColumn) else first.device
    _on_current_stream(sources, dev)
    # one upload: [ncols][nsrc] mdsx_gather_src records, then the packed ids
    table = np.zeros((len(names), nsrc, 4), np.uint64)
    for j, b in enumerate(sources):
        for c, name in enumerate(names):
            col = b.columns[name]
            if isinstance(col, RaggedColumn):
                table[c, j] = (col.values.data_ptr() if col.values.numel() else 0,
                               col.offsets.data_ptr(),
                               col.flags.data_ptr() if col.flags is not None else 0, b.rows)
            else:
                table[c, j] = (col.data_ptr(), 0, 0, b.rows)
    if m and (src.min() < 0 or src.max() >= nsrc or rows.min() < 0 or
              rows.max() >= (1 << _native.GATHER_SRC_SHIFT)):
        raise IndexError('gather_sources: source or row out of range')
    packed = (src.astype(np.uint64) << np.uint64(_native.GATHER_SRC_SHIFT)) | rows.astype(np.uint64)
    buf = torch.from_numpy(np.concatenate([table.reshape(-1), packed]).view(np.int64)).to(dev)
    tab = buf.data_ptr()
    idx = tab + table.size * 8
    ragged = [n for n in names if isinstance(sources[0].columns[n], RaggedColumn)]
    # a workspace per ragged column (its scan's tile prefixes are read by its copy, which runs
    # after every scan), fixed columns in the first; then the ragged totals
    wsb = int(lib.mdsx_gather_workspace_bytes(m))
    nws = max(len(ragged), 1)
    ws = torch.zeros(wsb * nws + 8 * nws, dtype=torch.uint8, device=dev)
    tot = wsb * nws
    stream = torch.cuda.current_stream(dev).cuda_stream
    out: dict[str, Union[torch.Tensor, RaggedColumn]] = {}
    offs = {}
    for c, name in enumerate(names):
        col = sources[0].columns[name]
        srcs = tab + c * nsrc * 32
        if isinstance(col, RaggedColumn):
            r = ragged.index(name)
            offs[name] = torch.empty(m + 1, dtype=torch.int64, device=dev)
            _check(lib.mdsx_gather_ragged_scan_multi(srcs, nsrc, idx if m else None, m,
                                                     offs[name].data_ptr(),
                                                     ws.data_ptr() + r * wsb, wsb,
                                                     ws.data_ptr() + tot + 8 * r, stream),
                   'mdsx_gather_ragged_scan_multi')
        else:
            row_shape = tuple(col.shape[1:])
            dst = torch.empty((m, ) + row_shape, dtype=col.dtype, device=dev)
            row_bytes = int(np.prod(row_shape, dtype=np.int64)) * col.element_size()
            if m:
                _check(lib.mdsx_gather_fixed_multi(srcs, nsrc, row_bytes, idx, m, dst.data_ptr(),
                                                   ws.data_ptr(), wsb, stream),
                       'mdsx_gather_fixed_multi')
            out[name] = dst
    # the one sync: the status records and the ragged totals together
    head = torch.cat([ws[r * wsb:r * wsb + 16] for r in range(nws)] +
                     [ws[tot:tot + 8 * len(ragged)]]).cpu().numpy()
    if check:
        for r in range(nws):
            st = _native.Status.from_buffer_copy(head[16 * r:16 * r + 16].tobytes())
            if st.code != 0:
                raise IndexError(f'sample id out of range at position {st.row} of the gather')
    caps = head[16 * nws:].view(np.int64)
    for c, name in enumerate(names):
        col = sources[0].columns[name]
        if not isinstance(col, RaggedColumn):
            continue
        cap = int(caps[ragged.index(name)])
        vals = torch.empty(max(cap, 1), dtype=torch.uint8, device=dev)
        flags = torch.zeros(m, dtype=torch.uint8, device=dev) if col.flags is not None else None
        _check(lib.mdsx_gather_ragged_copy_multi(
            tab + c * nsrc * 32, nsrc, idx if m else None, m, vals.data_ptr() if cap else None,
            cap, offs[name].data_ptr(), flags.data_ptr() if flags is not None else None,
            ws.data_ptr() + ragged.index(name) * wsb, wsb, stream), 'mdsx_gather_ragged_copy_multi')
        out[name] = RaggedColumn(vals[:cap], offs[name], flags)
    # (a source freed after this returns is reused in stream order: these kernels come first;
    # sources of another stream were marked in use by this one, _on_current_stream)
    return DecodedBatch({name: out[name] for name in names}, m,
                        stream=torch.cuda.current_stream(dev))


def _status_error(status: _native.Status, plan: Plan) -> Exception:
    code = status.code
    col = ''
    if 0 <= status.column < len(plan.columns):
        col = f', column {plan.columns[status.column].name!r}'
    where = f'shard {status.shard}, sample {status.row}{col}'
    if code == _native.MDSX_E_EMPTY:
        return IndexError(f'Relative sample index {status.row} is not present in shard '
                          f'{status.shard} (empty sample).')
    if code == _native.MDSX_E_HEADER:
        return ValueError(f'Malformed MDS shard header ({where}).')
    if code == _native.MDSX_E_BOUNDS:
        return ValueError(f'MDS sample or column out of bounds ({where}).')
    if code == _native.MDSX_E_CAPACITY:
        return RuntimeError(f'ragged output capacity exceeded ({where}).')
    return RuntimeError(f'mdsx device error {code} ({where}).')


class _PendingRagged(RaggedColumn):
    """A ragged column of a single-pass decode: ``values`` is the output buffer cut to the
    column's total, which is read back (one wait on the decode) the first time it is needed."""

    def __init__(self, buf: torch.Tensor, offsets: torch.Tensor, flags: Optional[torch.Tensor],
                 total) -> None:
        self._buf, self._total, self._values = buf, total, None
        self.offsets, self.flags = offsets, flags

    @property
    def values(self) -> torch.Tensor:
        if self._values is None:
            self._values = self._buf[:self._total()]
        return self._values

    @values.setter
    def values(self, v: torch.Tensor) -> None:
        self._values = v


def payload_bound(plan: Plan, batch: DeviceBatch) -> int:
    """Bytes any one ragged column of ``batch`` can hold at most: the sample bytes of its shards
    less every sample's column-size heads and fixed columns (mds/writer.py:133-144 layout)."""
    heads = sum(4 * (n + 2) for n in batch.samples)  # u32 count + N + 1 offsets
    per_row = 4 * plan.num_var + plan.fixed_row_bytes()
    return max(0, batch.shard_bytes - heads - per_row * batch.total_rows)


def _tune_knob(key: str) -> int:
    """An integer MDSX_TUNE knob the Python side reads (measurement only; 0 when unset)."""
    for kv in os.environ.get('MDSX_TUNE', '').split(','):
        k, _, v = kv.partition('=')
        if k.strip() == key and v.strip().isdigit():
            return int(v)
    return 0


class BatchDecoder:
    """Decode a :class:`DeviceBatch` on the device, reusing outputs across calls.

    ``run()`` enqueues the scan + decode kernels on the current torch stream with no host sync
    once the ragged capacities are known (first call, or given ``capacities``), so it can be
    timed / captured. ``check()`` synchronizes and raises the first kernel-reported error.

    ``single=True`` runs ``mdsx_decode_shards_single`` instead: one decode launch that scans its
    own ragged lengths (decoupled look-back), with ragged outputs allocated at their upper bound
    (:func:`payload_bound`) unless ``capacities`` are given -- no host round trip at all, the
    first call included. The exact ragged totals are read back only when a column's ``values``
    is first used. Copy modes follow the previous call's totals (the bound split evenly before
    any call has finished).
    """

    def __init__(self, plan: Plan, batch: DeviceBatch,
                 capacities: Optional[dict[str, int]] = None, single: bool = False) -> None:
        _native.check_fork()
        if batch.buffer.device.type != 'cuda':  # host addresses must never reach the kernels
            _native.require_gpu()
            raise ValueError(f'BatchDecoder: the shard batch is on {batch.buffer.device}, not '
                             'the GPU (stage_shards / make_batch put it there)')
        self.plan = plan
        self.batch = batch
        dev = batch.device
        self.device = dev
        rows = batch.total_rows
        self._abi = batch.abi()
        self.workspace = torch.zeros(max(plan.workspace_bytes(batch), 256), dtype=torch.uint8,
                                     device=dev)
        self.totals = torch.zeros(max(plan.num_var, 1), dtype=torch.int64, device=dev)
        self.outputs: dict[str, Union[torch.Tensor, RaggedColumn]] = {}
        self._fixed_raw: dict[str, torch.Tensor] = {}
        skew = _tune_knob('skew') * 1024  # measurement only: fixed outputs start this far in
        for col in plan.columns:
            if col.is_fixed:
                raw = torch.empty(rows * col.row_bytes + skew, dtype=torch.uint8,
                                  device=dev)[skew:].view(rows, col.row_bytes)
                self._fixed_raw[col.name] = raw
                dtype, shape = col.tensor_view()
                self.outputs[col.name] = raw.view(dtype).reshape((rows,) + shape)
            else:
                offsets = torch.empty(rows + 1, dtype=torch.int64, device=dev)
                flags = torch.zeros(rows, dtype=torch.uint8,
                                    device=dev) if col.kind == KIND_STR else None
                self.outputs[col.name] = RaggedColumn(torch.empty(0, dtype=torch.uint8,
                                                                  device=dev), offsets, flags)
        self._capacities = dict(capacities or {})
        self._outs = (ColumnOut * max(len(plan.columns), 1))()
        self._sized = plan.num_var == 0
        self.single = single
        if single and plan.num_var:
            bound = payload_bound(plan, batch)
            if not capacities:
                capacities = {c.name: bound for c in plan.columns if not c.is_fixed}
            self._capacities = dict(capacities)
            self._mode = (ctypes.c_uint64 * max(len(plan.columns), 1))()
            for c in plan.columns:
                self._mode[c.index] = 0 if c.is_fixed else bound // plan.num_var
            self._host_totals = torch.zeros(plan.num_var, dtype=torch.int64, pin_memory=True)
            self._totals_ready: Optional[torch.cuda.Event] = None
            self._totals_valid = False
        if capacities:
            self._resize(capacities)

    def _resize(self, capacities: dict[str, int]) -> None:
        for col in self.plan.columns:
            if col.is_fixed:
                continue
            need = int(capacities[col.name])
            rc = self.outputs[col.name]
            if rc.values.numel() < need:
                rc.values = torch.empty(max(need, 1), dtype=torch.uint8, device=self.device)
        self._sized = True

    def _fill_outs(self) -> None:
        for col in self.plan.columns:
            o = self._outs[col.index]
            out = self.outputs[col.name]
            if col.is_fixed:
                o.data, o.offsets, o.flags, o.capacity = self._fixed_raw[col.name].data_ptr(
                ), None, None, 0
            else:
                o.data = out.values.data_ptr() if out.values.numel() else None
                o.offsets = out.offsets.data_ptr()
                o.flags = out.flags.data_ptr() if out.flags is not None else None
                o.capacity = int(out.values.numel())

    def stream_tensors(self) -> list[torch.Tensor]:
        """The device tensors a pass reads or writes: the batch and its tables, the workspace,
        the totals and every output."""
        ts = [self.batch.buffer, self.batch.descs, self.batch.tile_shard, self.workspace,
              self.totals]
        for col in self.plan.columns:
            out = self.outputs[col.name]
            if isinstance(out, RaggedColumn):
                ts += [t for t in (out.values, out.offsets, out.flags) if t is not None]
            else:
                ts.append(self._fixed_raw[col.name])
        return ts

    def _scan(self, stream: int) -> None:
        _check(
            self.plan._lib.mdsx_scan_shards(self.plan.handle, ctypes.byref(self._abi), self._outs,
                                            self.workspace.data_ptr(), self.workspace.numel(),
                                            self.totals.data_ptr(), stream), 'mdsx_scan_shards')

    def _run_single(self, stream: int, events) -> DecodedBatch:
        if self._totals_ready is not None and self._totals_ready.query():
            vi = 0  # the last finished call's totals pick this call's copy modes
            for col in self.plan.columns:
                if not col.is_fixed:
                    self._mode[col.index] = int(self._host_totals[vi])
                    vi += 1
        if events is not None:
            events[0].record()
            events[1].record()
        _check(
            self.plan._lib.mdsx_decode_shards_single(self.plan.handle, ctypes.byref(self._abi),
                                                     self._outs, self._mode,
                                                     self.workspace.data_ptr(),
                                                     self.workspace.numel(),
                                                     self.totals.data_ptr(), stream),
            'mdsx_decode_shards_single')
        if events is not None:
            events[2].record()
        self._host_totals.copy_(self.totals[:self.plan.num_var], non_blocking=True)
        self._totals_ready = torch.cuda.Event()
        self._totals_ready.record()
        self._totals_valid = False
        return self.result()

    def _single_total(self, vi: int, cap: int):
        def total() -> int:
            if self._totals_ready is None:
                return 0
            if not self._totals_valid:
                self._totals_ready.synchronize()
                self._totals_valid = True
            return min(int(self._host_totals[vi]), cap)
        return total

    def run(self, events: Optional[Sequence[torch.cuda.Event]] = None) -> DecodedBatch:
        """Enqueue the decode of the whole batch; returns the (device) decoded columns.

        ``events``: optional three CUDA events recorded on the stream before the scan pass,
        between the scan and the decode kernel, and after the decode kernel (kernel timing; a
        single-pass decode records the first two together).
        """
        self._stream = torch.cuda.current_stream(self.device)
        stream = self._stream.cuda_stream
        self._fill_outs()
        if self.single and self.plan.num_var:
            return self._run_single(stream, events)
        if events is not None:
            events[0].record()
        self._scan(stream)  # resets the status record; ragged plans: offsets + totals
        if self.plan.num_var and not self._sized:
            totals = self.totals.cpu().tolist()  # host sync: size the ragged outputs once
            caps, vi = {}, 0
            for col in self.plan.columns:
                if not col.is_fixed:
                    caps[col.name] = int(totals[vi])
                    vi += 1
            self._capacities = caps
            self._resize(caps)
            self._fill_outs()
        if events is not None:
            events[1].record()
        self._decode(stream)
        if events is not None:
            events[2].record()
        return self.result()

    def _decode(self, stream: int) -> None:
        _check(
            self.plan._lib.mdsx_decode_shards(self.plan.handle, ctypes.byref(self._abi),
                                              self._outs, self.workspace.data_ptr(),
                                              self.workspace.numel(), stream),
            'mdsx_decode_shards')

    def result(self) -> DecodedBatch:
        cols: dict[str, Union[torch.Tensor, RaggedColumn]] = {}
        single = self.single and self.plan.num_var
        vi = 0
        for col in self.plan.columns:
            out = self.outputs[col.name]
            if isinstance(out, RaggedColumn) and single:
                out = _PendingRagged(out.values, out.offsets, out.flags,
                                     self._single_total(vi, int(out.values.numel())))
                vi += 1
            elif isinstance(out, RaggedColumn):
                cap = self._capacities.get(col.name, 0)
                out = RaggedColumn(out.values[:cap], out.offsets, out.flags)
            cols[col.name] = out
        return DecodedBatch(cols, self.batch.total_rows, list(self.batch.row0),
                            getattr(self, '_stream', None))

    @property
    def capacities(self) -> dict[str, int]:
        return dict(self._capacities)

    def status(self) -> _native.Status:
        raw = self.workspace[:16].cpu().numpy().tobytes()  # syncs the stream
        return _native.Status.from_buffer_copy(raw)

    def check(self) -> None:
        st = self.status()
        if st.code != 0:
            raise _status_error(st, self.plan)


class ScanAheadDecoder:
    """Decode a sequence of device batches of one plan with each batch's pass 1 (the offsets and
    size-head scan, ``mdsx_scan_shards``) enqueued on a side stream AHEAD of its pass 2
    (``mdsx_decode_shards``, on the current stream), so that it runs beside the previous batch's
    decode.

    The scan pass reads one line of size heads per sample and is latency-bound: alone it is
    ~4 % of a config-C step and ~14 % of a step over 32-256-byte rows, and it
    leaves most of HBM idle while it runs. Ahead of time it shares the GPU with a decode instead.

    Each of ``slots`` slots owns a workspace and outputs. ``scan(batch)`` takes a free slot and
    enqueues pass 1 of ``batch`` on the side stream behind everything queued so far on the
    current stream (so behind every reader of that slot's previous outputs); ``decode()``
    makes the current stream wait for the oldest scanned batch's pass 1, enqueues its pass 2
    and returns its outputs, valid until the next ``scan`` into that slot (with 2 slots: until
    the next call of :meth:`run`). Ragged outputs are allocated at ``capacities`` (default: the
    batch's :func:`payload_bound`, an upper bound, so no host round trip ever; a column that does
    not fit raises MDSX_E_CAPACITY at :meth:`check`); ragged ``values`` are trimmed to the
    scanned totals when first read.

    ``run(ahead)`` is one step over the decoder's own batch: the decode of the batch scanned
    before and, with ``ahead``, the scan for the next step beside it (the first call scans its
    own batch first).

    ``priority``: the side stream's priority (torch.cuda.Stream; lower is higher -- a scan whose
    workgroups are dispatched before the queued decode's as CUs free up).
    """

    def __init__(self, plan: Plan, batch: DeviceBatch,
                 capacities: Optional[dict[str, int]] = None, slots: int = 2,
                 priority: int = 0) -> None:
        if slots < 2:
            raise ValueError('ScanAheadDecoder: at least 2 slots (one scanned while one decodes)')
        self.plan = plan
        self.batch = batch
        self.device = batch.device
        self._caps = dict(capacities) if capacities else None
        self._slots = [self._new_slot(batch) for _ in range(slots)]
        self._side = torch.cuda.Stream(self.device, priority=priority)
        self._free = list(range(slots))
        self._pending: list[tuple[int, torch.cuda.Event, Optional[torch.cuda.Event]]] = []
        self._last: Optional[int] = None
        self._host_totals = [torch.zeros(max(plan.num_var, 1), dtype=torch.int64,
                                         pin_memory=True) for _ in range(slots)]
        self._totals_ready: list[Optional[torch.cuda.Event]] = [None] * slots

    def _new_slot(self, batch: DeviceBatch) -> BatchDecoder:
        caps = self._caps
        if self.plan.num_var and (caps is None or batch is not self.batch):
            # the given capacities fit the constructor's batch; another batch of the plan gets at
            # least its upper bound, so no column can overflow (MDSX_E_CAPACITY) however it sizes
            bound = payload_bound(self.plan, batch)
            caps = {c.name: max(bound, int((caps or {}).get(c.name, 0)))
                    for c in self.plan.columns if not c.is_fixed}
        dec = BatchDecoder(self.plan, batch, capacities=caps)
        dec._sized = True
        return dec

    def scan(self, batch: Optional[DeviceBatch] = None,
             events: Optional[Sequence[torch.cuda.Event]] = None) -> None:
        """Enqueue pass 1 of ``batch`` (default: the decoder's batch) into a free slot on the
        side stream. ``events``: two timing events recorded on the side stream around it."""
        if not self._free:
            raise RuntimeError('ScanAheadDecoder.scan: every slot holds a scanned batch; '
                               'decode() one first')
        si = self._free.pop(0)
        batch = self.batch if batch is None else batch
        dec = self._slots[si]
        if dec.batch is not batch:
            if batch.device != self.device:
                raise ValueError('ScanAheadDecoder: every batch must be on the decoder\'s device')
            dec = self._slots[si] = self._new_slot(batch)  # allocated on the current stream
        dec._fill_outs()
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.device))
        self._side.wait_event(ready)
        with torch.cuda.stream(self._side):
            if events is not None:
                events[0].record(self._side)
            dec._scan(self._side.cuda_stream)
            if events is not None:
                events[1].record(self._side)
        # the tensors the side stream's scan reads and writes were allocated on the current stream:
        # the caching allocator must not hand them out again before that scan is done
        for t in dec.stream_tensors():
            t.record_stream(self._side)
        done = torch.cuda.Event()
        done.record(self._side)
        self._pending.append((si, done, None))

    def decode(self, events: Optional[Sequence[torch.cuda.Event]] = None) -> DecodedBatch:
        """Enqueue pass 2 of the oldest scanned batch on the current stream; its outputs.
        ``events``: two timing events recorded on the current stream around the decode."""
        if not self._pending:
            raise RuntimeError('ScanAheadDecoder.decode: no scanned batch; scan() one first')
        si, done, _ = self._pending.pop(0)
        dec = self._slots[si]
        cur = torch.cuda.current_stream(self.device)
        cur.wait_event(done)
        if events is not None:
            events[0].record(cur)
        dec._stream = cur
        dec._decode(cur.cuda_stream)
        if events is not None:
            events[1].record(cur)
        if self.plan.num_var:
            self._host_totals[si].copy_(dec.totals[:self.plan.num_var], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(cur)
            self._totals_ready[si] = ev
        self._free.append(si)
        self._last = si
        return self._result(si)

    def run(self, ahead: bool = True, events: Optional[Sequence[torch.cuda.Event]] = None
            ) -> DecodedBatch:
        """One step over the decoder's batch. ``events``: four timing events -- around this
        step's decode on the current stream, then around the next step's scan on the side
        stream (left unrecorded without ``ahead``)."""
        if not self._pending:
            self.scan()
        if ahead:
            self.scan(events=events[2:4] if events is not None else None)
        return self.decode(events[0:2] if events is not None else None)

    def _result(self, si: int) -> DecodedBatch:
        dec = self._slots[si]
        cols: dict[str, Union[torch.Tensor, RaggedColumn]] = {}
        vi = 0
        for col in self.plan.columns:
            out = dec.outputs[col.name]
            if isinstance(out, RaggedColumn):
                out = _PendingRagged(out.values, out.offsets, out.flags,
                                     self._total(si, vi, int(out.values.numel())))
                vi += 1
            cols[col.name] = out
        return DecodedBatch(cols, dec.batch.total_rows, list(dec.batch.row0), dec._stream)

    def _total(self, si: int, vi: int, cap: int):
        ev = self._totals_ready[si]
        host = self._host_totals[si]

        def total() -> int:
            ev.synchronize()
            return min(int(host[vi]), cap)
        return total

    def result(self) -> DecodedBatch:
        """The outputs of the last decode."""
        if self._last is None:
            raise RuntimeError('ScanAheadDecoder.result: nothing decoded yet')
        return self._result(self._last)

    def check(self) -> None:
        """Synchronize and raise the first error the last decoded batch's kernels reported."""
        if self._last is not None:
            self._slots[self._last].check()

    def close(self) -> None:
        """Wait for the side stream (a scan ahead that will not be decoded) and drop it."""
        self._side.synchronize()
        self._pending.clear()
        self._free = list(range(len(self._slots)))

    def __del__(self) -> None:
        side = getattr(self, '_side', None)
        if side is not None and getattr(self, '_pending', None):
            try:  # a scan still in flight writes this decoder's slots
                side.synchronize()
            except Exception:  # noqa: BLE001 -- interpreter shutdown: nothing left to protect
                pass


def decode_batch(plan: Plan, batch: DeviceBatch, check: bool = True,
                 single: bool = False) -> DecodedBatch:
    """Decode every shard of ``batch`` (scan + decode, or ``single``: one look-back pass) and,
    by default, check the status."""
    dec = BatchDecoder(plan, batch, single=single)
    out = dec.run()
    if check:
        dec.check()
    return out


def output_bytes(plan: Plan, decoded: DecodedBatch) -> int:
    """W of SURVEY.md §8(d): bytes the decode writes (values, offsets, flags)."""
    total = 0
    for col in plan.columns:
        out = decoded.columns[col.name]
        if isinstance(out, RaggedColumn):
            total += int(out.values.numel()) + 8 * int(out.offsets.numel())
            if out.flags is not None:
                total += int(out.flags.numel())
        else:
            total += int(out.numel()) * out.element_size()
    return total


KINDS = {KIND_FIXED: 'fixed', KIND_BYTES: 'bytes', KIND_STR: 'str', KIND_NDARRAY: 'ndarray'}
