#!/bin/bash
# Row-parallel decode variants read from L2: parity in their modes, then short rows A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r05f}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_device_copy_modes.py tests/test_device_fuzz.py -x -q \
  --timeout 120 --timeout-method thread -k "srows" > "$OUT/pytest_srows.log" 2>&1 \
  || { tail -40 "$OUT/pytest_srows.log"; exit 1; }
tail -1 "$OUT/pytest_srows.log"
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 16 --blob 32,256 --chars 8,64 \
  --rounds 3 --variants ${VARS:-"rows=-1" "rows=-1,srows=2" "rows=-1,srows=2,srlim=8" "rows=-1,srows=2,srlim=24,srtile=64" "rows=-1,srows=2,srtile=20" "rows=-1#ctl"} \
  > "$OUT/l2rows.json" 2> "$OUT/l2rows.err" || { tail -20 "$OUT/l2rows.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/l2rows.json'))
print('rows', {k: round(v['GBps']) for k, v in d['results'].items()})"
