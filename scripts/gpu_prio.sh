#!/bin/bash
# The next step's scan pass on a side stream (ScanAheadDecoder), normal and high priority,
# against the one-stream step, short rows and config C, in-process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-prio}
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -c "import torch; print('priority range', torch.cuda.Stream.priority_range())" > "$OUT/range.txt" 2>&1; cat "$OUT/range.txt"
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 16 --blob 32,256 --chars 8,64 --rounds ${ROUNDS:-4} --variants "snt=-1" "snt=-1,ahead" "snt=-1,ahead_hi" "snt=-1#ctl" > "$OUT/short.json" 2> "$OUT/short.err" || { tail -20 "$OUT/short.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/short.json'))
print('short', {k: round(v['GBps']) for k, v in d['results'].items()})"
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 64 --rounds ${ROUNDS:-4} --variants "snt=-1" "snt=-1,ahead" "snt=-1,ahead_hi" "snt=-1#ctl" > "$OUT/C.json" 2> "$OUT/C.err" || { tail -20 "$OUT/C.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/C.json'))
print('C', {k: round(v['GBps']) for k, v in d['results'].items()})"
