#!/bin/bash
# Config D slice (765 shards = one GPU's share of 100M samples) vs config B (62 shards): decode
# rate and the address-translation counters of the decode kernel (TCP UTCL1 hits / misses per
# request), one --pmc pass each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-dslice}
mkdir -p "$OUT"
export TMPDIR=/tmp
for sh in 62 765; do
  timeout -k 10 600 python3 bench.py --config B --shards $sh --steps 10 --cpu-seconds 0 --no-copy-probe > "$OUT/bench_$sh.json" 2> "$OUT/bench_$sh.err" || { tail -20 "$OUT/bench_$sh.err"; exit 1; }
  python3 -c "
import json; l = json.load(open('$OUT/bench_$sh.json')); r = l['roofline']
print('shards $sh', r['kernel'], 'kern %.3f ms frac %.3f' % (r['kernel_ms'], r['frac']), 'samples/s %.3g' % l['value'])"
  timeout -s KILL 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum -d "$OUT/utcl_$sh" -o run --output-format csv -- python3 bench.py --config B --shards $sh --steps 3 --warmup 1 --cpu-seconds 0 --no-copy-probe --no-verify > "$OUT/utcl_$sh.log" 2>&1 || { tail -20 "$OUT/utcl_$sh.log"; exit 1; }
  python3 - "$OUT/utcl_$sh" $sh <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'decode_kernel' in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
m = {k: sum(v) / len(v) for k, v in agg.items()}
miss, hit = (m.get(f'TCP_UTCL1_TRANSLATION_{x}_sum') for x in ('MISS', 'HIT'))
req = m.get('TCP_UTCL1_REQUEST_sum')
print('shards', sys.argv[2], 'per launch: UTCL1 requests %.4g hits %.4g misses %.4g miss rate %.4f' % (req, hit, miss, miss / max(req, 1)))
PY
done
