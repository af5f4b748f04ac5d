#!/bin/bash
# Round-5 steps: scan-ahead tests, short rows / config C with and without the scan ahead, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r05b}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_device_scan_ahead.py -x -q --timeout 120 \
  --timeout-method thread > "$OUT/pytest_scan_ahead.log" 2>&1 || { tail -40 "$OUT/pytest_scan_ahead.log"; exit 1; }
tail -1 "$OUT/pytest_scan_ahead.log"
timeout -k 10 300 python3 scripts/tune_decode.py --config C --shards 16 --blob 32,256 --chars 8,64 \
  --rounds 4 --variants "rows=-1" "rows=-1,ahead" "rows=-1#ctl" "rows=-1,ahead#ctl" > "$OUT/rows_ahead.json" \
  2> "$OUT/rows_ahead.err" || { tail -20 "$OUT/rows_ahead.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/rows_ahead.json'))
print('rows', {k: round(v['GBps']) for k, v in d['results'].items()})"
timeout -k 10 300 python3 scripts/tune_decode.py --config C --shards 64 --rounds 4 \
  --variants "run=7" "run=7,ahead" "run=7#ctl" "run=7,ahead#ctl" > "$OUT/c_ahead.json" \
  2> "$OUT/c_ahead.err" || { tail -20 "$OUT/c_ahead.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/c_ahead.json'))
print('C', {k: round(v['GBps']) for k, v in d['results'].items()})"
timeout -k 10 400 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for name, r in (('B', d), ('C', d['config_c'])):
    r.setdefault('ms_per_step_blocks', None)
    rf = r['roofline']
    print(name, 'value', round(r['value']), 'ms', round(r['ms_per_step'], 4), r['ms_per_step_blocks'],
          'frac', round(rf['frac'], 3), 'step', round(rf['step_frac'], 3), 'copy', round(rf['frac_of_same_run_copy'], 3),
          'blocks', [round(x, 3) for x in rf['frac_blocks']], [round(x, 3) for x in rf['step_frac_blocks']])
PY
