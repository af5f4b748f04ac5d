#!/bin/bash
# Config C lean-path ablations in one process (measurement only; sv 8/16/24 leave outputs incomplete).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r05c}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 64 --rounds ${ROUNDS:-4} \
  --variants ${VARS:-"run=7" "run=7,sv=8,nocheck" "run=7,sv=16,nocheck" "run=7,sv=24,nocheck" "run=7#ctl" "run=7,rkb=32"} \
  > "$OUT/abl.json" 2> "$OUT/abl.err" || { tail -20 "$OUT/abl.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/abl.json'))
print('C', {k: round(v['GBps']) for k, v in d['results'].items()})"
