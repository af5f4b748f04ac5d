#!/bin/bash
# Raw memory-side request counters (read requests by size, write requests by size, DRAM-bound
# requests) of the decode kernels and the copy probe (a known byte count: the calibration), one
# --pmc pass per counter set and variant. RUNS: "config:variant" pairs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-counters}
mkdir -p "$OUT"
export TMPDIR=/tmp
RUNS="${RUNS:-C:tile=16 C:tile=32 B:tile=4}"
P1="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum"
P2="TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum"
if [ -n "$TIME_C" ]; then
  timeout -k 10 300 python3 scripts/tune_decode.py --config C --shards 16 --rounds 3 --variants $TIME_C > "$OUT/C.json" 2> "$OUT/C.err" || { tail -30 "$OUT/C.err"; exit 1; }
  python3 -c "
import json; d = json.load(open('$OUT/C.json'))
for k, v in d['results'].items(): print('C %-24s %8.3f ms %6d GB/s' % (k, v['median_ms'], v['GBps']))"
fi
i=0
for run in $RUNS; do
  cfg=${run%%:*}; var=${run#*:}
  for p in ${PASSES:-1 2}; do
    i=$((i + 1))
    if [ $p = 1 ]; then C=$P1; else C=$P2; fi
    timeout -s KILL 120 rocprofv3 --pmc $C -d "$OUT/p$i" -o run --output-format csv -- python3 scripts/tune_decode.py --config $cfg --shards 16 --samples 250000 --rounds 1 --iters 2 --variants $var > "$OUT/p$i.log" 2>&1 || { tail -20 "$OUT/p$i.log"; exit 1; }
    python3 - "$OUT/p$i" "$run" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0]
        if any(x in k for x in ('decode_kernel', 'scan_tiles', 'stage_totals', 'copy_probe',
                                'gather_ragged')):
            agg[(k[-48:], r['Counter_Name'])].append(float(r['Counter_Value']))
for (k, c), v in sorted(agg.items()):
    print(sys.argv[2], '%-48s %-26s n=%d %.4g' % (k, c, len(v), sum(v) / len(v)))
PY
  done
done
