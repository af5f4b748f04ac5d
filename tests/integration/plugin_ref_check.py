"""Build the REAL reference StreamingDataset on config A through the device stream plugin
(streams_registry name 'mdsx') and report, as one JSON line, what it holds. Run in its own
process by tests/test_plugin_reference.py (the offline boot of the reference patches sys.modules).

    python tests/integration/plugin_ref_check.py <reference dir> <scratch dir>
"""
import json
import os
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tests', 'golden'))


def main(ref: str, scratch: str) -> None:
    from make_golden import boot_reference
    boot_reference(ref)
    from streaming.base.batching import generate_work
    from streaming.base.dataset import StreamingDataset
    from streaming.base.util import clean_stale_shared_memory
    from streaming.base.world import World

    from streaming_amd.plugin import register_device_stream
    from streaming_amd.reader import MDSReader

    register_device_stream('mdsx')
    clean_stale_shared_memory()
    local = os.path.join(scratch, 'config_a')
    shutil.copytree(os.path.join(REPO, 'tests', 'golden', 'config_a'), local)
    ds = StreamingDataset(local=local, stream_name='mdsx', batch_size=16, shuffle=False,
                          num_canonical_nodes=1)
    ids = generate_work(ds.batching_method, ds, World(1, 1, 1, 0), 0, 0)
    want = np.load(os.path.join(REPO, 'tests', 'golden', 'order', 'config_a.npz'))['noshuffle_w1.start']
    out = {
        'stream_class': type(ds.streams[0]).__name__,
        'all_device_readers': all(isinstance(s, MDSReader) for s in ds.shards),
        'shards': len(ds.shards),
        'num_samples': int(ds.num_samples),
        'sizes': [int(s.samples) for s in ds.shards][:3],
        'ids_match_fixture': bool(np.array_equal(ids, want)),
    }
    try:  # reading a sample goes to the device reader: no GPU here, so it must fail loudly
        ds[0]
        out['get_item'] = 'returned'
    except Exception as e:  # noqa: BLE001
        out['get_item'] = f'{type(e).__name__}: {e}'
    del ds
    clean_stale_shared_memory()
    print(json.dumps(out))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
