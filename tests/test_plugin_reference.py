"""The plugin against the REAL reference (build container only; skipped where /root/reference is
absent, e.g. on the GPU box): StreamingDataset(stream_name='mdsx') built by the reference's own
registry-based construction (dataset.py:447-468) holds device readers for every shard, its
control plane (generate_work) lays out the recorded reference order over them, and reading a sample
goes to the device reader (no silent CPU fallback: without a GPU it raises)."""

import json
import os
import subprocess
import sys
import tempfile

import pytest

REF = os.environ.get('MDSX_REFERENCE', '/root/reference')
HERE = os.path.dirname(os.path.abspath(__file__))

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, 'streaming')),
                                reason='the reference source tree is not present')


@pytest.fixture(autouse=True)
def _one_reference_run_at_a_time():
    """The reference keeps its state in /dev/shm under global names, and its
    clean_stale_shared_memory() removes every such segment: two of these tests running at once
    (pytest-xdist workers) would pull each other's state away. One at a time, across processes."""
    from filelock import FileLock
    with FileLock(os.path.join(tempfile.gettempdir(), 'mdsx_reference_tests.lock')):
        yield


def test_streaming_dataset_with_device_stream(tmp_path):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE='1', HIP_VISIBLE_DEVICES='')
    res = subprocess.run([sys.executable, os.path.join(HERE, 'integration', 'plugin_ref_check.py'),
                          REF, str(tmp_path)], capture_output=True, text=True, timeout=300,
                         env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    assert out['stream_class'] == 'DeviceStream'
    assert out['all_device_readers']
    assert out['shards'] == 64 and out['num_samples'] == 10_000
    assert out['ids_match_fixture']
    assert out['get_item'].startswith('RuntimeError') and 'GPU' in out['get_item']


def test_device_iter_follows_the_reference_iteration(tmp_path):
    """device_iter / DeviceBatches over the real StreamingDataset: the reference's order from the
    epoch start and resumed from a checkpoint of the samples handed out (rows read by the oracle
    here; on the GPU by the device gather, tests/test_device_plugin_iter.py)."""
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE='1', HIP_VISIBLE_DEVICES='')
    res = subprocess.run([sys.executable, os.path.join(HERE, 'integration',
                                                       'device_iter_ref_check.py'), REF,
                          str(tmp_path)], capture_output=True, text=True, timeout=600, env=env)
    assert res.returncode == 0, res.stderr[-3000:]
    out = json.loads(res.stdout.strip().splitlines()[-1])
    for name, r in out.items():
        assert all(r.values()), (name, r)


_PORT_BASE = 20000  # below the kernel's ephemeral range (32768+): no OS-assigned port lands here
_PORTS_PER_WORKER = 200


def _worker_port():
    """A free port from this pytest worker's own range (PYTEST_XDIST_WORKER gwN: ports
    20000 + 200 N ...): no other worker and no ephemeral socket picks from it, so the port rank 0
    binds for its TCP-store rendezvous cannot be taken between this check and that bind. (The
    ranks' hangs of earlier rounds had a second cause, fixed in the rank script: each
    StreamingDataset creating and destroying its own process group on the same port.)"""
    import socket
    w = os.environ.get('PYTEST_XDIST_WORKER', 'gw0')
    idx = int(w[2:]) if w[2:].isdigit() else 0
    lo = _PORT_BASE + _PORTS_PER_WORKER * (idx % 60)
    for port in range(lo, lo + _PORTS_PER_WORKER):
        with socket.socket() as s:
            try:
                s.bind(('127.0.0.1', port))
            except OSError:  # in TIME_WAIT after an earlier run of this worker
                continue
            return port
    raise RuntimeError(f'no free port in {lo}..{lo + _PORTS_PER_WORKER}')


def _ranks(script, args):
    return _ranks_once(script, args)


def _ranks_once(script, args):
    port = _worker_port()
    procs = []
    for rank in range(2):
        env = dict(os.environ, PYTHONDONTWRITEBYTECODE='1', HIP_VISIBLE_DEVICES='',
                   RANK=str(rank), WORLD_SIZE='2', LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE='2',
                   MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, script] + args, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = []
    try:
        for p in procs:
            out, err = p.communicate(timeout=150)
            assert p.returncode == 0, err[-3000:]
            outs.append(json.loads(out.strip().splitlines()[-1]))
    finally:
        for p in procs:  # a rank left waiting for the other at a barrier
            if p.poll() is None:
                p.kill()
                p.wait()
    return outs


def _two_rank_settings():
    with open(os.path.join(HERE, 'golden', 'order', 'loader.json')) as f:
        return [s['name'] for s in json.load(f)['settings'] if s['ranks'] == 2]


@pytest.mark.parametrize('name', _two_rank_settings())
def test_device_iter_two_ranks_two_workers(tmp_path, name):
    """Two ranks (RANK / WORLD_SIZE, gloo on 127.0.0.1), each device_iter(num_workers=2) over the
    real StreamingDataset: each rank's samples equal what the reference's
    StreamingDataLoader(num_workers=2) yielded on that rank, and DeviceBatches.state_dict (this
    rank's count times the ranks, // replication, dataloader.py:74-84) checkpoints and resumes as
    the reference -- one stream; two streams under device_per_stream / per_stream batching; and
    replication=2 (both ranks of the group the same samples)."""
    import shutil
    with open(os.path.join(HERE, 'golden', 'order', 'loader.json')) as f:
        st = {s['name']: s for s in json.load(f)['settings']}[name]
    local = tmp_path / 'a'
    for e in st.get('streams', []):
        shutil.copytree(os.path.join(HERE, 'golden', e['dir']), local / e['dir'])
    if not st.get('streams'):
        shutil.copytree(os.path.join(HERE, 'golden', 'config_a'), local)
    script = os.path.join(HERE, 'integration', 'device_iter_ranks_check.py')
    start = _ranks(script, [REF, str(local), name, 'start'])
    for r in start:
        assert r['start'] and r['start_sizes'] and r['state_dict'], r
    resumed = _ranks(script, [REF, str(local), name, 'resume', json.dumps(start[0]['state'])])
    for r in resumed:
        assert r['resume'] and r['resume_sizes'], r
