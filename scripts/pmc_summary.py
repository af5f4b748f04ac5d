"""Summarise rocprofv3 runs of bench.py into per-(workload, kernel) traffic entries.

Usage: python scripts/pmc_summary.py <dir>   (the layout scripts/profile_bench.sh writes:
<dir>/trace (kernel-trace --stats), <dir>/fetch (--pmc FETCH_SIZE), <dir>/write (--pmc WRITE_SIZE),
and the bench JSON line in <dir>/trace.log).

For every config of the bench line (headline + ``config_c``) the entry holds the workload key
and the exact decode-kernel template name the bench reported, that kernel's rocprofv3 stats and
its per-launch HBM traffic: FETCH_SIZE / WRITE_SIZE are KiB per dispatch; per
MI355X_MICROARCH.md §HBM, FETCH_SIZE on gfx950 reads exactly half the bytes of a wide (16 B/lane)
coalesced streaming read, so the read side is doubled; WRITE_SIZE is exact for 16 B/lane
streaming stores. bench.py uses an entry only when both the workload key and the kernel match.
"""
import csv
import glob
import json
import os
import sys


def rows(out, pattern):
    res = []
    for f in glob.glob(os.path.join(out, pattern), recursive=True):
        with open(f) as fh:
            res.extend(csv.DictReader(fh))
    return res


def bench_lines(out):
    lines = []
    for log in ('trace.log', 'fetch.log', 'write.log'):
        p = os.path.join(out, log)
        if not os.path.exists(p):
            continue
        for x in open(p):
            if x.startswith('{') and '"metric"' in x:
                lines.append(json.loads(x))
    return lines


def configs(line):
    res = [line]
    if line.get('config_c'):
        res.append(line['config_c'])
    return res


def counter(out, sub, name, kernel):
    vals = []
    for r in rows(out, f'{sub}/**/*counter_collection.csv'):
        if kernel in r.get('Kernel_Name', '') and r.get('Counter_Name') == name:
            vals.append(float(r['Counter_Value']))
    return vals


def main(out):
    lines = bench_lines(out)
    if not lines:
        raise SystemExit(f'no bench line in {out}/*.log')
    stats = rows(out, 'trace/**/*kernel_stats.csv')
    entries = []
    for cfg in configs(lines[0]):
        kernel = cfg['roofline']['kernel']
        key = cfg['config']['workload_key']
        e = {
            'workload_key': key,
            'kernel': kernel,
            'lib_sha': cfg['roofline'].get('lib_sha'),
            'algorithmic_bytes_per_launch': cfg['roofline']['algorithmic_bytes_per_launch'],
            'kernel_stats': [r for r in stats if kernel in r['Name']],
        }
        fetch = counter(out, 'fetch', 'FETCH_SIZE', kernel)
        write = counter(out, 'write', 'WRITE_SIZE', kernel)
        if fetch and write:
            f = sum(fetch) / len(fetch) * 1024
            w = sum(write) / len(write) * 1024
            e.update({
                'fetch_size_bytes_per_launch_raw': f,
                'write_size_bytes_per_launch': w,
                'hbm_traffic_bytes_per_launch': 2 * f + w,
                'traffic_over_algorithmic': (2 * f + w) / e['algorithmic_bytes_per_launch'],
                'launches_counted': [len(fetch), len(write)],
            })
        entries.append(e)
    # every kernel of the trace, for context (scan passes, gather, copy probe)
    return {'entries': entries, 'all_kernel_stats': stats, 'bench_line': lines[0]}


if __name__ == '__main__':
    print(json.dumps(main(sys.argv[1]), indent=1))
