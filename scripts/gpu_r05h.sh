#!/bin/bash
# Config C lean path, the run-boundary lines with the default cache policy (MDSX_TUNE sv=128):
# parity of the mode, in-process A/B against the default, and the L2's memory-side request
# counters of both kernels from the same tune process (one --pmc pass per counter group).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r05h}
mkdir -p "$OUT"
export TMPDIR=/tmp
VARS=${VARS:-"run=7 run=7,sv=128 run=7,sv=256 run=7,sv=512 run=7,sv=1280 run=7#ctl"}
PVARS=${PVARS:-"run=7 run=7,sv=256 run=7,sv=512 run=7,sv=1280"}
timeout -k 10 600 python3 -u -m pytest tests/test_device_copy_modes.py tests/test_device_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-seg7_edge or seg7_v7}" > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 64 --rounds ${ROUNDS:-4} --variants $VARS > "$OUT/ab.json" 2> "$OUT/ab.err" || { tail -20 "$OUT/ab.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/ab.json'))
print('C', {k: round(v['GBps']) for k, v in d['results'].items()})"
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d "$OUT/read" -o run --output-format csv -- python3 scripts/tune_decode.py --config C --shards 64 --rounds 1 --variants $PVARS > "$OUT/read.log" 2>&1 || { tail -20 "$OUT/read.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d "$OUT/write" -o run --output-format csv -- python3 scripts/tune_decode.py --config C --shards 64 --rounds 1 --variants $PVARS > "$OUT/write.log" 2>&1 || { tail -20 "$OUT/write.log"; exit 1; }
python3 - "$OUT" <<'PY' > "$OUT/traffic.json"
import csv, glob, json, os, re, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(os.path.join(out, '*', '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.search(r'seg_decode_kernel<[^>]*>', r['Kernel_Name'])
        if k:
            acc[(k.group(0), r['Counter_Name'])].append(float(r['Counter_Value']))
m = lambda k, c: sum(acc[(k, c)]) / max(1, len(acc[(k, c)]))
ab = json.load(open(os.path.join(out, 'ab.json')))
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
print(json.dumps({'R': R, 'W': W, 'kernels': res}, indent=1))
PY
cat "$OUT/traffic.json"
