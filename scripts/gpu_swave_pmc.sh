#!/bin/bash
# Memory-side request counters (reads by size, writes, 64-byte writes) of the config-C decodes
# from one tune process per pass (rocprofv3 --pmc, one pass per counter group), plus the A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-swave_pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
VARS=${VARS:-"swave=0 swave=1 swave=1,swx=64 swave=1,swx=32,nocheck swave=0#ctl swave=1#ctl"}
PVARS=${PVARS:-"swave=0 swave=1 swave=1,swx=64 swave=1,swx=32,nocheck"}
timeout -k 10 180 python3 scripts/swave_check.py "swave=1,swx=64" > "$OUT/checks.log" 2>&1 || { tail -20 "$OUT/checks.log"; exit 1; }
export MDSX_PROBES=5,10
timeout -k 10 500 python3 scripts/tune_decode.py --config C --shards 64 --rounds ${ROUNDS:-3} --variants $VARS > "$OUT/C.json" 2> "$OUT/C.err" || { tail -20 "$OUT/C.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/C.json'))
print('C', {k: (round(v['GBps']), round(v.get('decode_GBps', 0))) for k, v in d['results'].items()})"
unset MDSX_PROBES
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d "$OUT/read" -o run --output-format csv -- python3 scripts/tune_decode.py --config C --shards 64 --rounds 1 --iters 3 --variants $PVARS > "$OUT/read.log" 2>&1 || { tail -20 "$OUT/read.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d "$OUT/write" -o run --output-format csv -- python3 scripts/tune_decode.py --config C --shards 64 --rounds 1 --iters 3 --variants $PVARS > "$OUT/write.log" 2>&1 || { tail -20 "$OUT/write.log"; exit 1; }
python3 - "$OUT" <<'PY' > "$OUT/traffic.json"
import csv, glob, json, os, re, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(os.path.join(out, '*', '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.search(r'(seg_decode_kernel|swave_decode_kernel)<[^>]*>', r['Kernel_Name'])
        if k:
            acc[(k.group(0), r['Counter_Name'])].append(float(r['Counter_Value']))
m = lambda k, c: sum(acc[(k, c)]) / max(1, len(acc[(k, c)]))
ab = json.load(open(os.path.join(out, 'C.json')))
R, W = ab['R'], ab['W']
res = {}
for k in sorted({k for k, _ in acc}):
    rd = 32 * m(k, 'TCC_EA0_RDREQ_32B_sum') + 64 * m(k, 'TCC_EA0_RDREQ_64B_sum') + \
        128 * m(k, 'TCC_EA0_RDREQ_128B_sum')
    wr = 64 * m(k, 'TCC_EA0_WRREQ_64B_sum') + 32 * (m(k, 'TCC_EA0_WRREQ_sum') -
                                                    m(k, 'TCC_EA0_WRREQ_64B_sum'))
    res[k] = {'launches': len(acc[(k, 'TCC_EA0_WRREQ_sum')]), 'read_over_R': rd / R,
              'write_over_W': wr / W, 'traffic_over_RW': (rd + wr) / (R + W),
              'wrreq_sub64': m(k, 'TCC_EA0_WRREQ_sum') - m(k, 'TCC_EA0_WRREQ_64B_sum')}
print(json.dumps(res, indent=1))
PY
cat "$OUT/traffic.json"
