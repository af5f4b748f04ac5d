"""Calibrate the CPU baseline's port against the REAL reference (build container only).

    python scripts/calibrate_cpu_baseline.py [--reference /root/reference] [--seconds 10]

Writes one config-B and one config-C 64 MiB shard (the synthetic generators of bench.py's
workloads, host side), then times on one core, on the same page-cached files:
  * the reference's MDSReader (reader_from_json + reader[i] over the shard, mds/reader.py:128-149 +
    decode_sample + mds_decode), booted offline as tests/golden/make_golden.py does;
  * the port bench.py's cpu_baseline leg runs on the GPU box (oracle ReferenceCostMDSReader).
Prints one JSON line per config: samples/s of each and their ratio (DESIGN.md §CPU baseline).
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(HERE, 'tests', 'golden'))


def b_shard():
    """One full config-B shard: id int32 = i, x = 1024 uint32-random float32 bit patterns."""
    from streaming_amd.synth import config_b_samples_per_shard
    from streaming_amd.writer import shard_config_bytes
    n = config_b_samples_per_shard()
    names, encs, sizes = ['id', 'x'], ['int32', 'ndarray:float32:1024'], [4, 4096]
    config = shard_config_bytes(names, encs, sizes, None, [], 1 << 26)
    rng = np.random.default_rng(0)
    x = rng.integers(0, 2**32, (n, 1024), dtype=np.uint32)
    rows = np.concatenate([np.arange(n, dtype=np.int32).view(np.uint8).reshape(n, 4),
                           x.view(np.uint8).reshape(n, 4096)], 1)
    header = 4 + 4 * (n + 1) + len(config)
    offs = header + 4100 * np.arange(n + 1, dtype=np.int64)
    data = (np.uint32(n).tobytes() + offs.astype(np.uint32).tobytes() + config + rows.tobytes())
    return data, n, dict(column_names=names, column_encodings=encs, column_sizes=sizes)


def c_shard():
    from streaming_amd.synth import var_c_shards
    shards, counts, _ = var_c_shards(20_000, seed=1)
    return shards[0], counts[0], dict(column_names=['b', 'n', 's'],
                                      column_encodings=['bytes', 'int', 'str'],
                                      column_sizes=[None, 8, None])


def index_entry(name, size, n, schema):
    return dict(schema, compression=None, format='mds', hashes=[],
                raw_data={'basename': name, 'bytes': size, 'hashes': {}}, samples=n,
                size_limit=1 << 26, version=2, zip_data=None)


def timed_loop(reader, n, seconds):
    t0, done = time.perf_counter(), 0
    while time.perf_counter() - t0 < seconds:
        for i in range(n):
            reader.get_item(i)  # what bench.py's leg times (Reader.get_item, base/reader.py:310-320)
            done += 1
            if done % 512 == 0 and time.perf_counter() - t0 >= seconds:
                break
    return done / (time.perf_counter() - t0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reference', default='/root/reference')
    ap.add_argument('--seconds', type=float, default=10.0)
    args = ap.parse_args()
    from make_golden import boot_reference
    _, ref_reader_from_json, _ = boot_reference(args.reference)
    from oracle.mds_oracle import ReferenceCostMDSReader
    tmp = tempfile.mkdtemp(prefix='calib_')
    for config, make in (('B', b_shard), ('C', c_shard)):
        data, n, schema = make()
        name = f'shard.{config}.mds'
        with open(os.path.join(tmp, name), 'wb') as f:
            f.write(data)
        info = index_entry(name, len(data), n, schema)
        ref = ref_reader_from_json(tmp, None, info)
        port = ReferenceCostMDSReader(tmp, None, info)
        for i in (0, n // 2, n - 1):  # same values
            a, b = ref.get_item(i), port.get_item(i)
            assert a.keys() == b.keys()
            for k in a:
                x, y = a[k], b[k]  # bit patterns (random floats include NaNs)
                assert (x.tobytes() == y.tobytes() and x.dtype == y.dtype and x.shape == y.shape
                        if isinstance(x, (np.ndarray, np.generic)) else x == y), (config, k)
        rr = timed_loop(ref, n, args.seconds)
        rp = timed_loop(port, n, args.seconds)
        print(json.dumps({'config': config, 'samples_per_shard': n, 'shard_bytes': len(data),
                          'reference_samples_per_s': round(rr), 'port_samples_per_s': round(rp),
                          'port_over_reference': round(rp / rr, 3),
                          'reference_mib_per_s': round(rr * len(data) / n / 2**20, 1)}),
              flush=True)


if __name__ == '__main__':
    main()
