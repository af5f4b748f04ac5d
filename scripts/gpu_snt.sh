#!/bin/bash
# The scan pass's head loads, non-temporal or not (MDSX_TUNE snt), on short rows and config C,
# in-process A/B (scan + decode per step).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-snt}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 16 --blob 32,256 --chars 8,64 --rounds ${ROUNDS:-4} --variants "snt=0" "snt=1" "snt=0#ctl" "snt=1#ctl" > "$OUT/short.json" 2> "$OUT/short.err" || { tail -20 "$OUT/short.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/short.json'))
print('short', {k: round(v['GBps']) for k, v in d['results'].items()})"
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 64 --rounds ${ROUNDS:-4} --variants "snt=0" "snt=1" "snt=0#ctl" "snt=1#ctl" > "$OUT/C.json" 2> "$OUT/C.err" || { tail -20 "$OUT/C.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/C.json'))
print('C', {k: round(v['GBps']) for k, v in d['results'].items()})"
