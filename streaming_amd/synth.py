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


def fixed_b_batch_on_device(num_samples: int,
                            seed: int = 0,
                            size_limit: int = 1 << 26,
                            device: Union[str, torch.device, None] = None,
                            keep_sources: bool = True,
                            first_id: int = 0) -> SynthShards:
    """Config B shards written directly into a device batch buffer.

    ``x`` rows are uniform random bytes (every float32 bit pattern; ``torch.randint`` on the
    device, seeded), ``id`` is ``first_id + i``.
    """
    names, encs, sizes = _schema(CONFIG_B)
    plan = Plan(names, encs, sizes)
    config = shard_config_bytes(names, encs, sizes, None, [], size_limit)
    sample = sum(sizes)
    per = (size_limit - 8 - len(config)) // (sample + 4) if size_limit else num_samples
    counts = [per] * (num_samples // per) + ([num_samples % per] if num_samples % per else [])
    shard_sizes = [4 + 4 * (n + 1) + len(config) + n * sample for n in counts]
    batch = make_batch(plan, shard_sizes, counts, device)
    dev = batch.device
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    ids_all = torch.arange(first_id, first_id + num_samples, dtype=torch.int32, device=dev)
    xs = []
    row = 0
    for s, n in enumerate(counts):
        header = _fixed_header(n, sample, config)
        off = batch.offsets[s]
        batch.buffer[off:off + len(header)].copy_(torch.frombuffer(bytearray(header),
                                                                   dtype=torch.uint8))
        body = batch.buffer[off + len(header):off + shard_sizes[s]].view(n, sample)
        x = torch.randint(0, 256, (n, 4096), dtype=torch.uint8, device=dev, generator=gen)
        body[:, :4].copy_(ids_all[row:row + n].view(torch.uint8).view(n, 4))
        body[:, 4:].copy_(x)
        if keep_sources:
            xs.append(x)
        row += n
    sources = {'id': ids_all}
    if keep_sources:
        sources['x'] = torch.cat(xs).view(torch.float32) if xs else torch.empty(0, 1024)  # bits
    torch.cuda.synchronize(dev)
    return SynthShards(plan, batch, counts, sources)


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
