#!/bin/bash
# Streaming row-parallel decode: parity in its modes, then short rows against the row-parallel kernel.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r05d}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_device_copy_modes.py tests/test_device_fuzz.py -x -q \
  --timeout 120 --timeout-method thread -k "${PYTEST_K:-srows}" > "$OUT/pytest_srows.log" 2>&1 \
  || { tail -40 "$OUT/pytest_srows.log"; exit 1; }
tail -1 "$OUT/pytest_srows.log"
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 16 --blob 32,256 --chars 8,64 \
  --rounds ${ROUNDS:-3} --variants ${VARS:-"rows=-1" "rows=-1,srows=1" "rows=-1,srows=1,srkb=6" "rows=-1,srows=1,srkb=12" "rows=-1,srows=1,srtile=80" "rows=-1#ctl"} \
  > "$OUT/srows.json" 2> "$OUT/srows.err" || { tail -20 "$OUT/srows.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/srows.json'))
print('rows', {k: round(v['GBps']) for k, v in d['results'].items()})"
