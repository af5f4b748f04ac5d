"""bench.py's N-GPU launcher, on CPU: ``python bench.py --gpus N --dry-run`` starts N child ranks
itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* as torch.distributed.run sets them), they join
a gloo process group and report the shards they own; a world size other than ``--gpus`` fails."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT')}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, env=env,
                          capture_output=True, text=True, timeout=timeout, cwd=ROOT)


@pytest.mark.parametrize('gpus', [2, 3])
def test_launcher_spawns_ranks_and_partitions_shards(gpus):
    p = _run(['--gpus', str(gpus), '--dry-run'])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith('{')]
    assert len(lines) == 1  # rank 0 only
    line = lines[0]
    assert line['n_gpus'] == gpus
    for config, per_gpu in (('B', 62), ('C', 64)):
        ranks = line['ownership'][config]
        assert [r['rank'] for r in ranks] == list(range(gpus))
        total = ranks[0]['total']
        assert total == per_gpu * gpus
        flat = sorted(s for r in ranks for s in r['shards'])
        assert flat == list(range(total))  # every global shard owned exactly once
        for r in ranks:
            assert all(s % gpus == r['rank'] for s in r['shards'])  # owned_shards: g -> g % N
            assert len(r['shards']) == per_gpu  # weak scaling: fixed work per GPU
    # the N-GPU line's per-rank report (gathered over the gloo group) and its aggregation
    per = line['per_rank']
    assert [p['rank'] for p in per] == list(range(gpus))
    for p in per:
        for k in ('ms_per_step', 'kernel_ms', 'frac', 'step_frac', 'copy_ceiling_GBps',
                  'frac_of_same_run_copy'):
            assert isinstance(p[k], float) and p[k] > 0, (k, p)
    summ = line['per_rank_summary']
    assert summ['ranks'] == gpus and summ['slowest_rank'] == gpus - 1
    for k in ('ms_per_step', 'kernel_ms', 'frac', 'copy_ceiling_GBps', 'frac_of_same_run_copy'):
        xs = [p[k] for p in per]
        assert summ[k]['min'] == min(xs) and summ[k]['max'] == max(xs), k


def test_world_mismatch_is_an_error():
    p = _run(['--gpus', '2', '--dry-run'], {'WORLD_SIZE': '3', 'RANK': '0'})
    assert p.returncode != 0
    assert 'WORLD_SIZE=3' in p.stderr


def test_single_rank_dry_run():
    p = _run(['--gpus', '1', '--dry-run', '--config', 'B'])
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    assert line['n_gpus'] == 1
    assert line['ownership']['B'][0]['shards'] == list(range(62))


def test_committed_traffic_is_keyed_on_workload_kernel_and_sources(tmp_path, monkeypatch):
    """bench.py reports a PMC traffic figure only from a summary taken on the same workload,
    kernel and library sources (the sha compiled into mdsx_version); else null."""
    import json

    import bench
    from streaming_amd import build
    sha = build.source_sha()
    assert bench.src_sha() == sha  # the loaded library names these sources
    prof = tmp_path / 'profiles' / 'r99'
    prof.mkdir(parents=True)
    entry = {'workload_key': 'B:k', 'kernel': 'decode_kernel<4, true>', 'src_sha': sha,
             'hbm_traffic_bytes_per_launch': 123.0}
    stale = dict(entry, src_sha='0' * 16, hbm_traffic_bytes_per_launch=7.0)
    (prof / 'pmc_x.json').write_text(json.dumps({'entries': [stale, entry]}))
    monkeypatch.setattr(bench, 'HERE', str(tmp_path))
    assert bench.committed_traffic('B:k', 'decode_kernel<4, true>') == (
        123.0, os.path.join('profiles', 'r99', 'pmc_x.json'))
    assert bench.committed_traffic('B:other', 'decode_kernel<4, true>') == (None, None)
    assert bench.committed_traffic('B:k', 'run_decode_kernel<4, false>') == (None, None)
    (prof / 'pmc_x.json').write_text(json.dumps({'entries': [stale]}))
    assert bench.committed_traffic('B:k', 'decode_kernel<4, true>') == (None, None)


def test_block_sizes():
    """bench.py splits each config's K timed steps into interleaved blocks."""
    import bench
    assert bench.block_sizes(20) == [7, 7, 6]
    assert bench.block_sizes(3) == [1, 1, 1]
    assert bench.block_sizes(2) == [1, 1]
    assert bench.block_sizes(1) == [1]
    assert sum(bench.block_sizes(101)) == 101
