"""device_iter under two ranks against the REAL reference (build container; one process per rank,
started by tests/test_plugin_reference.py under RANK / WORLD_SIZE / LOCAL_WORLD_SIZE with a gloo
rendezvous on 127.0.0.1).

Each rank builds StreamingDataset(stream_name='mdsx') on config A and iterates it with
streaming_amd.plugin.device_iter(num_workers=2), rows read by the CPU oracle (no GPU here). Phase
``start``: the samples in order against the digest of the reference's own
StreamingDataLoader(num_workers=2) on this rank (tests/golden/order/loader.json, setting
py1s_r2w2), then a checkpoint after the fixture's batch count through DeviceBatches.state_dict.
Phase ``resume``: a new dataset after load_state_dict of that state. Prints one JSON line.

    python tests/integration/device_iter_ranks_check.py <reference dir> <local dir> <setting>
        <phase> [state]

``<setting>``: a two-rank setting of tests/golden/order/loader.json; ``<local dir>`` holds the
copy of its streams' golden dirs (config_a itself for a one-stream setting).
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tests', 'golden'))


def main(ref: str, local: str, name: str, phase: str, state_json: str = '') -> None:
    from make_golden import boot_reference
    boot_reference(ref)
    from streaming.base.dataset import StreamingDataset
    from streaming.base.util import clean_stale_shared_memory

    from oracle.mds_oracle import OracleMDSReader
    from streaming_amd.order import DeviceSampleGather
    from streaming_amd.plugin import DeviceBatches, device_iter, register_device_stream

    rank = int(os.environ['RANK'])
    DeviceStream = register_device_stream('mdsx')
    with open(os.path.join(REPO, 'tests', 'golden', 'order', 'loader.json')) as f:
        st = {s['name']: s for s in json.load(f)['settings']}[name]
    pr = st['per_rank'][rank]
    bs, W = st['kwargs']['batch_size'], st['workers']
    dirs = [os.path.join(local, e['dir']) for e in st.get('streams', [])] or [local]
    readers = []
    for d in dirs:
        with open(os.path.join(d, 'index.json')) as f:
            readers += [OracleMDSReader(d, None, info) for info in json.load(f)['shards']]

    def dataset():
        if st.get('streams'):  # two streams, each a device stream (the plugin's Stream subclass)
            return StreamingDataset(streams=[
                DeviceStream(local=os.path.join(local, e['dir']), **e['kwargs'])
                for e in st['streams']], **st['kwargs'])
        return StreamingDataset(local=local, stream_name='mdsx', **st['kwargs'])

    class OracleGather(DeviceSampleGather):

        def gather(self, ids):
            shard, loc = self.locate(ids)
            return [readers[int(s)].get_item(int(i)) for s, i in zip(shard, loc)]

    def run(it):
        h, sizes = hashlib.sha256(), []
        for b in it:
            sizes.append(len(b))
            for r in b:
                h.update(np.int64(r['number']).tobytes())
                h.update(r['words'].encode('utf-8'))
        return h.hexdigest(), sizes

    # One process group for the whole run. Without it each StreamingDataset.__init__ creates one
    # and destroys it again (distributed.py:114-128 maybe_init_dist, dataset.py:431): a second
    # dataset in the same process then rendezvouses on the same MASTER_PORT while rank 0's store
    # of the first is being torn down, and rank 1 can connect to the dying one ("Failed to recv").
    import torch.distributed as dist
    dist.init_process_group('gloo')
    clean_stale_shared_memory()  # collective under WORLD_SIZE=2: every rank calls it
    res = {'rank': rank}
    if phase == 'start':
        ds = dataset()
        d, sizes = run(device_iter(ds, bs, num_workers=W, gather=OracleGather(ds.shards)))
        res['start'] = d == pr['iter_start_sha256']
        res['start_sizes'] = sizes == pr['start_batch_sizes']
        ds2 = dataset()
        batches = DeviceBatches(ds2, bs, num_workers=W, gather=OracleGather(ds2.shards))
        it = iter(batches)
        for _ in range(st['resume_batches']):
            next(it)
        state = batches.state_dict()
        res['state_dict'] = state == st['state_dict']
        res['state'] = state
        ds2._iterator.exit()
    else:
        ds = dataset()
        ds.load_state_dict(json.loads(state_json))
        d, sizes = run(device_iter(ds, bs, num_workers=W, gather=OracleGather(ds.shards)))
        res['resume'] = d == pr['iter_resume_sha256']
        res['resume_sizes'] = sizes == pr['resume_batch_sizes']
    dist.barrier()
    dist.destroy_process_group()
    print(json.dumps(res))


if __name__ == '__main__':
    main(*sys.argv[1:])
