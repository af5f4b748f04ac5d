"""Synthetic MDS datasets of the BASELINE.json configs, built fast and bit-identical to what
:class:`streaming_amd.writer.MDSWriter` writes for the same samples.

* Config B -- ``{id: int32, x: ndarray:float32:1024}`` (every float bit pattern, NaN payloads
  included). :func:`fixed_b_batch_on_device` writes the shard files straight into an HBM batch
  buffer (header from the host, sample rows with torch copies on the device), so the benchmark
  does not push gigabytes through the host.
* Config C -- ``{n: int, b: bytes U[3072,5120], s: str U[16,256] code points of 1/2/3/4-byte
  UTF-8}``. :func:`var_c_shards` builds host shard files with vectorised value generation and
  one slice assignment per column per sample.

Shard boundaries follow the writer's size-limit rule (``streaming/base/format/base/writer.py:
263-269``): a sample starts a new shard when ``size_limit < shard_bytes + len(sample) + 4``.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Union

import numpy as np
import torch

from streaming_amd.decoder import DeviceBatch, Plan, make_batch
from streaming_amd.writer import shard_config_bytes

__all__ = ['CONFIG_B', 'CONFIG_C', 'fixed_b_batch_on_device', 'var_c_shards', 'shard_split',
           'utf8_pool', 'SynthShards']

CONFIG_B = {'id': 'int32', 'x': 'ndarray:float32:1024'}
CONFIG_C = {'n': 'int', 'b': 'bytes', 's': 'str'}


def _schema(columns: dict[str, str]):
    from streaming_amd.encodings import get_mds_encoded_size
    names = sorted(columns)
    encs = [columns[n] for n in names]
    sizes = [get_mds_encoded_size(e) for e in encs]
    return names, encs, sizes


def shard_split(sample_sizes: np.ndarray, config_len: int, size_limit: int) -> list[int]:
    """Samples per shard under the writer's flush rule."""
    counts, cur, n = [], 8 + config_len, 0
    for size in sample_sizes.tolist():
        new = size + 4
        if size_limit and size_limit < cur + new and n:
            counts.append(n)
            cur, n = 8 + config_len, 0
        cur += new
        n += 1
    if n:
        counts.append(n)
    return counts


def _fixed_header(n: int, sample_size: int, config: bytes) -> bytes:
    header = 4 + 4 * (n + 1) + len(config)
    offsets = (header + sample_size * np.arange(n + 1, dtype=np.int64)).astype(np.uint32)
    return np.uint32(n).tobytes() + offsets.tobytes() + config


@dataclass
class SynthShards:
    """A synthetic dataset as a device batch plus the source columns it encodes."""
    plan: Plan
    batch: DeviceBatch
    samples_per_shard: list[int]
    sources: dict[str, torch.Tensor]


def config_b_samples_per_shard(size_limit: int = 1 << 26) -> int:
    """Samples of a full config-B shard under the writer's size limit (16 352 at 64 MiB)."""
    names, encs, sizes = _schema(CONFIG_B)
    config = shard_config_bytes(names, encs, sizes, None, [], size_limit)
    return (size_limit - 8 - len(config)) // (sum(sizes) + 4)


def fixed_b_batch_on_device(num_samples: int,
                            seed: int = 0,
                            size_limit: int = 1 << 26,
                            device: Union[str, torch.device, None] = None,
                            keep_sources: bool = True,
                            first_id: int = 0,
                            shard_ids: Optional[list[int]] = None) -> SynthShards:
    """Config B shards written directly into a device batch buffer.

    ``x`` rows are uniform random bytes (every float32 bit pattern; ``torch.randint`` on the
    device, seeded), ``id`` is ``first_id + i``.

    With ``shard_ids``, the batch holds those shards of a larger dataset of full shards instead:
    global shard ``g`` has ids ``g * per ..`` and ``x`` drawn from a generator seeded
    ``seed + g``, so a shard's bytes do not depend on which rank builds it (``num_samples`` and
    ``first_id`` are then ignored).
    """
    names, encs, sizes = _schema(CONFIG_B)
    plan = Plan(names, encs, sizes)
    config = shard_config_bytes(names, encs, sizes, None, [], size_limit)
    sample = sum(sizes)
    per = (size_limit - 8 - len(config)) // (sample + 4) if size_limit else num_samples
    if shard_ids is not None:
        counts = [per] * len(shard_ids)
        firsts = [g * per for g in shard_ids]
        seeds = [seed + g for g in shard_ids]
    else:
        counts = [per] * (num_samples // per) + ([num_samples % per] if num_samples % per else [])
        firsts = [first_id + sum(counts[:s]) for s in range(len(counts))]
        seeds = [None] * len(counts)
    shard_sizes = [4 + 4 * (n + 1) + len(config) + n * sample for n in counts]
    batch = make_batch(plan, shard_sizes, counts, device)
    dev = batch.device
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    ids, xs = [], []
    for s, n in enumerate(counts):
        if seeds[s] is not None:
            gen.manual_seed(seeds[s])
        header = _fixed_header(n, sample, config)
        off = batch.offsets[s]
        batch.buffer[off:off + len(header)].copy_(torch.frombuffer(bytearray(header),
                                                                   dtype=torch.uint8))
        body = batch.buffer[off + len(header):off + shard_sizes[s]].view(n, sample)
        x = torch.randint(0, 256, (n, 4096), dtype=torch.uint8, device=dev, generator=gen)
        idv = torch.arange(firsts[s], firsts[s] + n, dtype=torch.int32, device=dev)
        body[:, :4].copy_(idv.view(torch.uint8).view(n, 4))
        body[:, 4:].copy_(x)
        ids.append(idv)
        if keep_sources:
            xs.append(x)
    sources = {'id': torch.cat(ids) if ids else torch.empty(0, dtype=torch.int32, device=dev)}
    if keep_sources:
        sources['x'] = torch.cat(xs).view(torch.float32) if xs else torch.empty(0, 1024)  # bits
    torch.cuda.synchronize(dev)
    return SynthShards(plan, batch, counts, sources)


def utf8_encode_device(cp: torch.Tensor) -> tuple[torch.Tensor, torch.Tensor]:
    """UTF-8 bytes of code points ``cp`` (int64, no surrogates) on the device: returns
    (packed bytes, bytes per code point)."""
    nb = 1 + (cp >= 0x80).long() + (cp >= 0x800).long() + (cp >= 0x10000).long()
    pos = torch.cumsum(nb, 0) - nb
    out = torch.empty(int(nb.sum()), dtype=torch.uint8, device=cp.device)
    lead = torch.where(nb == 1, cp,
                       torch.where(nb == 2, 0xC0 | (cp >> 6),
                                   torch.where(nb == 3, 0xE0 | (cp >> 12), 0xF0 | (cp >> 18))))
    out[pos] = lead.to(torch.uint8)
    for k in (1, 2, 3):  # continuation byte k of a sequence of nb bytes carries bits 6*(nb-1-k)
        m = nb > k
        shift = 6 * (nb[m] - 1 - k)
        out[pos[m] + k] = (0x80 | ((cp[m] >> shift) & 0x3F)).to(torch.uint8)
    return out, nb


def _ragged(lengths: torch.Tensor, values: torch.Tensor) -> 'RaggedColumn':
    from streaming_amd.decoder import RaggedColumn
    offsets = torch.zeros(lengths.numel() + 1, dtype=torch.int64, device=lengths.device)
    torch.cumsum(lengths, 0, out=offsets[1:])
    return RaggedColumn(values, offsets)


def var_c_columns_on_device(shard_ids: list[int],
                            seed: int = 2000,
                            size_limit: int = 1 << 26,
                            device: Union[str, torch.device, None] = None,
                            str_chars: tuple[int, int] = (16, 256),
                            blob_bytes: tuple[int, int] = (3072, 5120),
                            str_widths: int = 4):
    """Config C columns (``n: int``, ``b: bytes U[3072,5120]``, ``s: str`` of U[16,256] code
    points, 25 % each of 1/2/3/4-byte UTF-8) for full 64 MiB shards of a larger dataset, built
    on the device: global shard ``g`` draws from a generator seeded ``seed + g`` and holds
    exactly the rows the writer puts into one shard (``base/writer.py:263-269``). Returns
    (per-shard columns in decoder layout, rows per shard).

    Shards are separate writer runs (each starts a fresh shard), so the rows of shard ``g + 1``
    never move into shard ``g`` as one writer's greedy split of the concatenation could.
    ``str_widths`` < 4 draws code points of 1..str_widths UTF-8 bytes only (1: ASCII text)."""
    dev = torch.device(device or 'cuda')
    if dev.index is None:
        dev = torch.device('cuda', torch.cuda.current_device())
    names, encs, sizes = _schema(CONFIG_C)
    config = shard_config_bytes(names, encs, sizes, None, [], size_limit)
    cap = size_limit - 8 - len(config)
    rows_try = cap // (8 + blob_bytes[0] + 8 + str_chars[0] + 4) + 1
    gen = torch.Generator(device=dev)
    ns, bs, ss, counts = [], [], [], []
    for g in shard_ids:
        gen.manual_seed(seed + g)
        kw = dict(device=dev, generator=gen)
        b_len = torch.randint(blob_bytes[0], blob_bytes[1] + 1, (rows_try, ), **kw)
        chars = torch.randint(str_chars[0], str_chars[1] + 1, (rows_try, ), **kw)
        width = torch.randint(0, str_widths, (int(chars.sum()), ), **kw)
        lo = torch.tensor([0x20, 0x80, 0x800, 0x10000], device=dev)[width]
        hi = torch.tensor([0x7F, 0x800, 0x10000 - 0x800, 0x110000], device=dev)[width]
        cp = lo + (torch.rand(width.shape, dtype=torch.float64, **kw) * (hi - lo)).long()
        cp = torch.where((width == 2) & (cp >= 0xD800), cp + 0x800, cp)  # skip surrogates
        nb = 1 + (cp >= 0x80).long() + (cp >= 0x800).long() + (cp >= 0x10000).long()
        row_of_cp = torch.repeat_interleave(torch.arange(rows_try, device=dev), chars)
        s_len = torch.zeros(rows_try, dtype=torch.int64, device=dev).index_add_(0, row_of_cp, nb)
        cum4 = torch.cumsum(8 + b_len + 8 + s_len + 4, 0).cpu().numpy()
        n = int(np.searchsorted(cum4, cap, side='right'))
        b_len, s_len = b_len[:n], s_len[:n]
        ncp = int(chars[:n].sum())
        s_vals, _ = utf8_encode_device(cp[:ncp])
        b_vals = torch.randint(0, 256, (int(b_len.sum()), ), dtype=torch.uint8, **kw)
        nv = torch.randint(-2**62, 2**62, (n, ), dtype=torch.int64, **kw)
        ns.append(nv)
        bs.append(_ragged(b_len, b_vals))
        ss.append(_ragged(s_len, s_vals))
        counts.append(n)
    return [{'n': a, 'b': b, 's': s} for a, b, s in zip(ns, bs, ss)], counts


def var_c_batch_on_device(shard_ids: list[int],
                          seed: int = 2000,
                          size_limit: int = 1 << 26,
                          device: Union[str, torch.device, None] = None,
                          str_chars: tuple[int, int] = (16, 256),
                          blob_bytes: tuple[int, int] = (3072, 5120),
                          str_widths: int = 4) -> SynthShards:
    """Config C shards (``shard_ids`` of a dataset of full shards, see
    :func:`var_c_columns_on_device`) written by the device MDS encoder into one decode batch."""
    from streaming_amd.decoder import stage_shards
    from streaming_amd.encoder import concat_columns, encode_batch
    names, encs, sizes = _schema(CONFIG_C)
    plan = Plan(names, encs, sizes)
    config = shard_config_bytes(names, encs, sizes, None, [], size_limit)
    parts, counts = var_c_columns_on_device(shard_ids, seed, size_limit, device, str_chars,
                                            blob_bytes, str_widths)
    files = []
    for cols, n in zip(parts, counts):
        enc, consumed = encode_batch(plan, cols, config, size_limit)
        if enc is None or enc.bounds != [(0, n)] or consumed != n:
            raise RuntimeError('config C synth: a shard\'s rows do not fill exactly one shard')
        files.append(enc.shard(0))
    batch = stage_shards(files, counts, plan)
    del files
    torch.cuda.synchronize(batch.device)
    return SynthShards(plan, batch, counts, concat_columns(parts))


def utf8_pool(rng: np.random.Generator, count: int) -> tuple[np.ndarray, np.ndarray]:
    """``count`` random code points (25 % each of 1/2/3/4-byte UTF-8, no surrogates) encoded
    with numpy. Returns (utf-8 bytes, byte length per code point)."""
    width = rng.integers(0, 4, count)
    cp = np.empty(count, np.int64)
    m = width == 0
    cp[m] = rng.integers(0x20, 0x7F, int(m.sum()))
    m = width == 1
    cp[m] = rng.integers(0x80, 0x800, int(m.sum()))
    m = width == 2
    v = rng.integers(0x800, 0x10000 - 0x800, int(m.sum()))
    cp[m] = np.where(v >= 0xD800, v + 0x800, v)
    m = width == 3
    cp[m] = rng.integers(0x10000, 0x110000, int(m.sum()))
    nbytes = width + 1
    out = np.zeros((count, 4), np.uint8)
    # 1 byte
    m = nbytes == 1
    out[m, 0] = cp[m]
    m = nbytes == 2
    out[m, 0] = 0xC0 | (cp[m] >> 6)
    out[m, 1] = 0x80 | (cp[m] & 0x3F)
    m = nbytes == 3
    out[m, 0] = 0xE0 | (cp[m] >> 12)
    out[m, 1] = 0x80 | ((cp[m] >> 6) & 0x3F)
    out[m, 2] = 0x80 | (cp[m] & 0x3F)
    m = nbytes == 4
    out[m, 0] = 0xF0 | (cp[m] >> 18)
    out[m, 1] = 0x80 | ((cp[m] >> 12) & 0x3F)
    out[m, 2] = 0x80 | ((cp[m] >> 6) & 0x3F)
    out[m, 3] = 0x80 | (cp[m] & 0x3F)
    keep = np.arange(4)[None, :] < nbytes[:, None]
    return out[keep], nbytes


def var_c_shards(num_samples: int,
                 seed: int = 1,
                 size_limit: int = 1 << 26,
                 str_chars: tuple[int, int] = (16, 256),
                 blob_bytes: tuple[int, int] = (3072, 5120)) -> tuple[list[bytes], list[int], dict]:
    """Config C shard files (host bytes), identical to ``MDSWriter`` output for the same samples.

    Returns (shard files, samples per shard, source columns as numpy arrays: ``n`` int64,
    ``b_len``/``s_len`` byte lengths, ``b_pool``/``s_pool`` concatenated values).
    """
    rng = np.random.default_rng(seed)
    names, encs, sizes = _schema(CONFIG_C)  # b (var), n (8), s (var)
    config = shard_config_bytes(names, encs, sizes, None, [], size_limit)
    n_val = rng.integers(-2**62, 2**62, num_samples, dtype=np.int64)
    b_len = rng.integers(blob_bytes[0], blob_bytes[1] + 1, num_samples).astype(np.int64)
    b_pool = np.frombuffer(rng.bytes(int(b_len.sum())), np.uint8)
    chars = rng.integers(str_chars[0], str_chars[1] + 1, num_samples).astype(np.int64)
    s_pool, cp_bytes = utf8_pool(rng, int(chars.sum()))
    cp_end = np.cumsum(cp_bytes)
    char_end = np.cumsum(chars)
    s_end = cp_end[char_end - 1] if num_samples else np.zeros(0, np.int64)
    s_len = np.diff(np.concatenate([[0], s_end])).astype(np.int64)
    sample_sizes = 8 + b_len + 8 + s_len
    counts = shard_split(sample_sizes, len(config), size_limit)
    b_off = np.concatenate([[0], np.cumsum(b_len)])
    s_off = np.concatenate([[0], np.cumsum(s_len)])
    b_bytes, s_bytes = b_pool.tobytes(), s_pool.tobytes()
    n_bytes = n_val.tobytes()
    shards, row = [], 0
    for n in counts:
        rows = slice(row, row + n)
        sz = sample_sizes[rows]
        header = 4 + 4 * (n + 1) + len(config)
        offs = header + np.concatenate([[0], np.cumsum(sz)])
        buf = bytearray(int(offs[-1]))
        buf[0:4] = np.uint32(n).tobytes()
        buf[4:4 + 4 * (n + 1)] = offs.astype(np.uint32).tobytes()
        buf[4 + 4 * (n + 1):header] = config
        mv = memoryview(buf)
        heads = np.stack([b_len[rows], s_len[rows]], 1).astype(np.uint32).tobytes()
        for k in range(n):
            i = row + k
            p = int(offs[k])
            mv[p:p + 8] = heads[8 * k:8 * k + 8]
            p += 8
            lb = int(b_len[i])
            mv[p:p + lb] = b_bytes[b_off[i]:b_off[i] + lb]
            p += lb
            mv[p:p + 8] = n_bytes[8 * i:8 * i + 8]
            p += 8
            ls = int(s_len[i])
            mv[p:p + ls] = s_bytes[s_off[i]:s_off[i] + ls]
        shards.append(bytes(buf))
        row += n
    sources = {'n': n_val, 'b_len': b_len, 'b_pool': b_pool, 's_len': s_len, 's_pool': s_pool}
    return shards, counts, sources
