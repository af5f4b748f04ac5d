#!/bin/bash
# Config C: the touch-ahead lean-path variant; short rows: streaming row-parallel windows smaller than its ring.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r05e}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_device_copy_modes.py -x -q --timeout 120 \
  --timeout-method thread -k "seg" > "$OUT/pytest_seg.log" 2>&1 || { tail -30 "$OUT/pytest_seg.log"; exit 1; }
tail -1 "$OUT/pytest_seg.log"
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 64 --rounds 4 \
  --variants "run=7" "run=7,sv=32" "run=7,sv=33" "run=7#ctl" > "$OUT/c_touch.json" 2> "$OUT/c_touch.err" \
  || { tail -20 "$OUT/c_touch.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/c_touch.json'))
print('C', {k: round(v['GBps']) for k, v in d['results'].items()})"
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 16 --blob 32,256 --chars 8,64 \
  --rounds 3 --variants "rows=-1" "rows=-1,srows=1" "rows=-1,srows=1,srkb=12,srlim=4" \
  "rows=-1,srows=1,srkb=12,srlim=6" "rows=-1,srows=1,srlim=4" "rows=-1#ctl" > "$OUT/srows2.json" \
  2> "$OUT/srows2.err" || { tail -20 "$OUT/srows2.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/srows2.json'))
print('rows', {k: round(v['GBps']) for k, v in d['results'].items()})"
