"""device_iter against the REAL reference StreamingDataset (build container; run in its own
process by tests/test_plugin_reference.py, the offline boot of the reference patches sys.modules).

StreamingDataset(stream_name='mdsx') on config A, iterated by streaming_amd.plugin.DeviceBatches
/ device_iter -- the reference's own epoch / resumption / generate_work / prepare and ready
threads -- with the rows of each batch read by the CPU oracle (no GPU here; the GPU gather is
tests/test_device_plugin_iter.py). Reports, as one JSON line, whether the samples in order match
the digests the reference's own __iter__ recorded (tests/golden/order), from the epoch start and
after a mid-epoch state_dict -> load_state_dict taken from the samples the batches handed out.

    python tests/integration/device_iter_ref_check.py <reference dir> <scratch dir>
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
    from streaming.base.dataset import StreamingDataset
    from streaming.base.util import clean_stale_shared_memory

    from oracle.mds_oracle import OracleMDSReader
    from streaming_amd.order import DeviceSampleGather
    from streaming_amd.plugin import DeviceBatches, device_iter, register_device_stream

    def digest(numbers, words) -> str:  # tests/test_order.digest (the reference has a `tests`)
        import hashlib
        h = hashlib.sha256()
        for n, w in zip(numbers, words):
            h.update(np.int64(n).tobytes())
            h.update(w.encode('utf-8'))
        return h.hexdigest()

    DeviceStream = register_device_stream('mdsx')
    with open(os.path.join(REPO, 'tests', 'golden', 'order', 'config_a.json')) as f:
        settings = {s['name']: s for s in json.load(f)['settings']}
    out = {}
    for name in ('noshuffle_w1', 'py1e_w1'):
        st = settings[name]
        clean_stale_shared_memory()
        local = os.path.join(scratch, name)
        shutil.copytree(os.path.join(REPO, 'tests', 'golden', 'config_a'), local)
        with open(os.path.join(local, 'index.json')) as f:
            infos = json.load(f)['shards']

        class OracleGather(DeviceSampleGather):
            """The batch's rows read by the CPU oracle (the device gather's stand-in here)."""
            readers = [OracleMDSReader(local, None, info) for info in infos]

            def gather(self, ids):
                shard, loc = self.locate(ids)
                for s in np.unique(shard):
                    os.stat(self.shards[int(s)]._filename())  # FileNotFoundError, as on the GPU
                return [self.readers[int(s)].get_item(int(i)) for s, i in zip(shard, loc)]

        def run(it):
            numbers, words, sizes = [], [], []
            for b in it:
                sizes.append(len(b))
                numbers += [r['number'] for r in b]
                words += [r['words'] for r in b]
            return numbers, words, sizes

        res = {}
        ds = StreamingDataset(local=local, stream_name='mdsx', **st['kwargs'])
        numbers, words, sizes = run(device_iter(ds, 16, gather=OracleGather(ds.shards)))
        res['start'] = digest(numbers, words) == st['iter_start_sha256']
        res['start_count'] = len(numbers) == st['iter_start_count']
        res['full_batches'] = all(s == 16 for s in sizes[:-1]) and 0 < sizes[-1] <= 16
        # a mid-epoch checkpoint from the samples the batches handed out (a new epoch: 1)
        ds2 = StreamingDataset(local=local, stream_name='mdsx', **st['kwargs'])
        batches = DeviceBatches(ds2, 16, gather=OracleGather(ds2.shards))
        it = iter(batches)
        while batches.num_samples_yielded < st['resume_at']:
            next(it)
        state = batches.state_dict()
        res['state_dict'] = state == st['state_dict']
        ds2._iterator.exit()
        del it, batches, ds2, ds
        clean_stale_shared_memory()
        ds3 = StreamingDataset(local=local, stream_name='mdsx', **st['kwargs'])
        ds3.load_state_dict(state)
        numbers, words, _ = run(device_iter(ds3, 16, gather=OracleGather(ds3.shards)))
        res['resume'] = digest(numbers, words) == st['iter_resume_sha256']
        res['resume_count'] = len(numbers) == st['iter_resume_count']
        del ds3
        out[name] = res
    # multi-worker loaders (tests/golden/order/loader.json, one rank): device_iter(num_workers=W)
    # against the reference's StreamingDataLoader(num_workers=W), start, checkpoint and resume
    with open(os.path.join(REPO, 'tests', 'golden', 'order', 'loader.json')) as f:
        loaders = {s['name']: s for s in json.load(f)['settings']}
    one_rank = [n for n, st in loaders.items() if st['ranks'] == 1]
    for name in one_rank:
        st = loaders[name]
        pr = st['per_rank'][0]
        bs, W = st['kwargs']['batch_size'], st['workers']
        clean_stale_shared_memory()
        local = os.path.join(scratch, name)
        dirs = [e['dir'] for e in st.get('streams', [])]
        readers = []
        for d in dirs or ['config_a']:
            dst = os.path.join(local, d) if dirs else local
            shutil.copytree(os.path.join(REPO, 'tests', 'golden', d), dst)
            with open(os.path.join(dst, 'index.json')) as f:
                readers += [OracleMDSReader(dst, None, info) for info in json.load(f)['shards']]
        OracleGather.readers = readers

        def dataset():
            if dirs:  # two streams, each a device stream (the plugin's Stream subclass)
                return StreamingDataset(streams=[
                    DeviceStream(local=os.path.join(local, e['dir']), **e['kwargs'])
                    for e in st['streams']], **st['kwargs'])
            return StreamingDataset(local=local, stream_name='mdsx', **st['kwargs'])

        res = {}
        ds = dataset()
        res['device_readers'] = all(type(s).__module__ == 'streaming_amd.reader'
                                    for s in ds.shards)
        numbers, words, sizes = run(device_iter(ds, bs, num_workers=W,
                                                gather=OracleGather(ds.shards)))
        res['start'] = digest(numbers, words) == pr['iter_start_sha256']
        res['start_sizes'] = sizes == pr['start_batch_sizes']
        ds2 = dataset()
        batches = DeviceBatches(ds2, bs, num_workers=W, gather=OracleGather(ds2.shards))
        it = iter(batches)
        for _ in range(st['resume_batches']):
            next(it)
        state = batches.state_dict()
        res['state_dict'] = state == st['state_dict']
        ds2._iterator.exit()
        del it, batches, ds2, ds
        clean_stale_shared_memory()
        ds3 = dataset()
        ds3.load_state_dict(state)
        numbers, words, sizes = run(device_iter(ds3, bs, num_workers=W,
                                                gather=OracleGather(ds3.shards)))
        res['resume'] = digest(numbers, words) == pr['iter_resume_sha256']
        res['resume_sizes'] = sizes == pr['resume_batch_sizes']
        del ds3
        out[name] = res
    clean_stale_shared_memory()
    print(json.dumps(out))


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2])
