"""Summarise rocprofv3 runs of bench.py into per-(workload, kernel) traffic entries.

Usage: python scripts/pmc_summary.py <dir>   (the layout scripts/profile_bench.sh writes:
<dir>/trace (kernel-trace --stats), <dir>/read (--pmc TCC_EA0_RDREQ by request size),
<dir>/write (--pmc TCC_EA0_WRREQ, _64B), and the bench JSON line in <dir>/trace.log).

For every config of the bench line (headline + ``config_c``) the entry holds the workload key
and the exact decode-kernel template name the bench reported, that kernel's rocprofv3 stats and
its per-launch HBM traffic from the request counters by size: read bytes = 32 x RDREQ_32B +
64 x RDREQ_64B + 128 x RDREQ_128B, write bytes = 64 x WRREQ_64B + 32 x (WRREQ - WRREQ_64B).
Calibrated on the copy probe (profiles/r02/counters_calibration.txt): a copy of N bytes counts
exactly N / 128 128-byte reads and N / 64 64-byte writes (FETCH_SIZE, which tallies a 128-byte
request at 64 bytes, reads half of that on gfx950, MI355X_MICROARCH.md §HBM, and mis-weighs
narrower requests). bench.py uses an entry only when the workload key, the kernel and the library
build match.
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
    for log in ('trace.log', 'read.log', 'write.log'):
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


def named(kernel, name):
    """Whether the dispatch / stats name `name` is the bench's kernel: the bench reports the
    template arguments it chose (`seg_decode_kernel<7, true, 2>`), the symbol also carries the
    defaulted ones (`seg_decode_kernel<7, true, 2, false>`)."""
    name = name.replace('(anonymous namespace)::', '')
    if kernel in name:
        return True
    k = kernel[:-1] if kernel.endswith('>') else kernel
    return k + ', ' in name or k + ',' in name


def counter(out, sub, name, kernel):
    vals = []
    for r in rows(out, f'{sub}/**/*counter_collection.csv'):
        if named(kernel, r.get('Kernel_Name', '')) and r.get('Counter_Name') == name:
            vals.append(float(r['Counter_Value']))
    return vals


def mean(out, sub, name, kernel):
    vals = counter(out, sub, name, kernel)
    return sum(vals) / len(vals) if vals else None


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
            'src_sha': cfg['roofline'].get('src_sha'),
            'algorithmic_bytes_per_launch': cfg['roofline']['algorithmic_bytes_per_launch'],
            'kernel_stats': [r for r in stats if named(kernel, r['Name'])],
        }
        # the bench's timed launches: the kernel's last `steps` dispatches of this workload in
        # the trace (warm-up and verification launches come before them), against the bench
        # line's HIP-event timing of the same launches
        durs = [int(r['End_Timestamp']) - int(r['Start_Timestamp'])
                for r in sorted(rows(out, 'trace/**/*kernel_trace.csv'),
                                key=lambda r: int(r['Start_Timestamp']))
                if named(kernel, r['Kernel_Name'])]
        steps = int(lines[0].get('steps', 20))
        if len(durs) >= steps:
            # the config's own launches: B's come first in the trace, C's after them
            idx = configs(lines[0]).index(cfg)
            same = [c for c in configs(lines[0]) if c['roofline']['kernel'] == kernel]
            block = durs if len(same) == 1 else durs[idx * len(durs) // len(same):
                                                      (idx + 1) * len(durs) // len(same)]
            # the bench's blocks (bench.py timed_block): each block's timed launches follow its
            # `rewarm` untimed ones; walked back from the config's last launch
            sizes = [b['steps'] for b in cfg.get('blocks', [])] or [steps]
            rewarm = int(cfg.get('rewarm', 0))
            timed, pos = [], len(block)
            for nb in reversed(sizes):
                timed = block[max(pos - nb, 0):pos] + timed
                pos -= nb + rewarm
            avg = sum(timed) / len(timed)
            algo = e['algorithmic_bytes_per_launch']
            e['trace_timed'] = {
                'launches': len(timed), 'avg_ns': avg,
                'achieved_GBps': algo / avg, 'frac': algo / avg / 8000.0,
                'bench_line_frac': cfg['roofline']['frac'],
                'bench_line_kernel_ms': cfg['roofline']['kernel_ms'],
            }
        # memory-side requests by size (TCC_EA0_*: the L2's requests to HBM / fabric), exact
        # bytes: a copy of N bytes counts N / 128 128-byte reads and N / 64 64-byte writes
        n32, n64, n128, nrd = (mean(out, 'read', f'TCC_EA0_RDREQ{s}_sum', kernel)
                               for s in ('_32B', '_64B', '_128B', ''))
        nwr, nw64 = (mean(out, 'write', f'TCC_EA0_WRREQ{s}_sum', kernel) for s in ('', '_64B'))
        if None not in (n32, n64, n128, nwr, nw64):
            rd = 32 * n32 + 64 * n64 + 128 * n128
            wr = 64 * nw64 + 32 * (nwr - nw64)
            e.update({
                'read_requests': {'32B': n32, '64B': n64, '128B': n128, 'all': nrd},
                'write_requests': {'64B': nw64, 'all': nwr},
                'read_bytes_per_launch': rd,
                'write_bytes_per_launch': wr,
                'hbm_traffic_bytes_per_launch': rd + wr,
                'traffic_over_algorithmic': (rd + wr) / e['algorithmic_bytes_per_launch'],
                'read_over_R': rd / cfg['roofline']['algorithmic']['R'],
                'write_over_W': wr / cfg['roofline']['algorithmic']['W'],
            })
        entries.append(e)
    # every kernel of the trace, for context (scan passes, gather, copy probe)
    return {'entries': entries, 'all_kernel_stats': stats, 'bench_line': lines[0]}


if __name__ == '__main__':
    print(json.dumps(main(sys.argv[1]), indent=1))
