#!/bin/bash
# The one-row-per-wave decode of all-fixed plans (MDSX_TUNE rw): parity (its tests, the fuzz
# modes), then config B in-process against decode_kernel, with occupancy (lpad) and the probes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-rowwave}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_device_rowwave.py tests/test_device_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
export MDSX_PROBES=1,5,7,8
timeout -k 10 400 python3 scripts/tune_decode.py --config B --rounds ${ROUNDS:-3} --variants ${VB:-"rw=0" "rw=1" "rw=1,lpad=10" "rw=1,lpad=13" "rw=1,lpad=16" "rw=2,lpad=20" "rw=2,lpad=26" "rw=4,lpad=40" "rw=0#ctl"} > "$OUT/B.json" 2> "$OUT/B.err" || { tail -20 "$OUT/B.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/B.json'))
print('B', {k: round(v['GBps']) for k, v in d['results'].items()})"
