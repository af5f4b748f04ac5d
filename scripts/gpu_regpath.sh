#!/bin/bash
# Register/ring decode on config C and short rows: timing per knob, FETCH_SIZE per variant (one
# --pmc pass each), the counters this box offers, and a kernel-trace of the short-row decode.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-regpath}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1 || true
grep -o "TCC_EA0_[A-Z0-9_]*\|TCC_[A-Z_]*RDREQ[A-Z0-9_]*" "$OUT/avail.txt" | sort -u | tr '\n' ' '; echo
VC="${VC:-tile=8 tile=16 tile=32 tile=64 ring=0 tile=16,ring=0}"
timeout -k 10 300 python3 scripts/tune_decode.py --config C --shards 16 --rounds 3 --variants $VC > "$OUT/C.json" 2> "$OUT/C.err" || { tail -30 "$OUT/C.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/C.json'))
for k, v in d['results'].items(): print('C %-24s %8.3f ms %6d GB/s' % (k, v['median_ms'], v['GBps']))
print('R', d['R'], 'W', d['W'])"
for v in $VC; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch_$v" -o run --output-format csv -- python3 scripts/tune_decode.py --config C --shards 16 --rounds 1 --iters 2 --variants $v > "$OUT/fetch_$v.log" 2>&1 || { tail -20 "$OUT/fetch_$v.log"; exit 1; }
  python3 - "$OUT/fetch_$v" "$v" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        agg[r['Kernel_Name'].split('(')[0][-60:]].append(float(r['Counter_Value']))
for k, v in agg.items():
    if 'decode' in k or 'scan' in k or 'gather' in k:
        print('fetch', sys.argv[2], k, 'n=%d' % len(v), 'raw MB/launch %.1f' % (sum(v) / len(v) * 1024 / 1e6))
PY
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/short_trace" -o run --output-format csv -- python3 scripts/tune_decode.py --config C --shards 16 --blob 32,256 --chars 8,64 --rounds 2 --variants tile=32 > "$OUT/short.log" 2>&1 || { tail -30 "$OUT/short.log"; exit 1; }
python3 - "$OUT/short_trace" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True):
    for r in list(csv.DictReader(open(f)))[:8]:
        print('short', r['Name'][:90], r['Calls'], '%.3f ms' % (float(r['AverageNs']) / 1e6))
PY
