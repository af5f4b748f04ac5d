#!/bin/bash
# One sample per wave (mdsx_swave.hip): parity in its modes, a full-size check, then where the
# cost of the columns past the first goes on config C (ablations, in one process).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-swave6}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_device_copy_modes.py tests/test_device_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-swave}" > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 180 python3 scripts/swave_check.py "swave=1" > "$OUT/checks.log" 2>&1 || { tail -20 "$OUT/checks.log"; exit 1; }
grep swave_check "$OUT/checks.log"
export MDSX_PROBES=5,10
VARS=${VARS:-"swave=0 swave=1 swave=1,swx=1 swave=1,swx=2,nocheck swave=1,swx=3,nocheck swave=1,swx=4,nocheck swave=1,swx=16,nocheck swave=1,swx=32,nocheck swave=1,swx=48,nocheck swave=0#ctl swave=1#ctl"}
timeout -k 10 500 python3 scripts/tune_decode.py --config C --shards 64 --rounds ${ROUNDS:-3} --variants $VARS > "$OUT/C.json" 2> "$OUT/C.err" || { tail -20 "$OUT/C.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/C.json'))
print('C', {k: (round(v['GBps']), round(v.get('decode_GBps', 0))) for k, v in d['results'].items()})
print(json.dumps(d['phase_cycles_per_tile']))"
