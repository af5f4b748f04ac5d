#!/bin/bash
# Config C lean path, two runs per wave far apart (MDSX_TUNE sv=4096), with one- and two-sample
# runs: parity, then in-process A/B against the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-pair}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_device_copy_modes.py tests/test_device_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-seg7_pair}" > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 64 --rounds ${ROUNDS:-4} --variants ${VARS:-"run=7" "run=7,rkb=8" "run=7,rkb=8,sv=4096" "run=7,sv=4096" "run=7#ctl"} > "$OUT/C.json" 2> "$OUT/C.err" || { tail -20 "$OUT/C.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/C.json'))
print('C', {k: round(v['GBps']) for k, v in d['results'].items()})"
