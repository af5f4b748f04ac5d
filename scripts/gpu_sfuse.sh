#!/bin/bash
# The chunk sums added by the totals pass (MDSX_TUNE sfuse=1, no scan_chunks / chunk_sums
# launches) against the three-kernel scan, short rows and config C, after the GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-sfuse}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 16 --blob 32,256 --chars 8,64 --rounds ${ROUNDS:-4} --variants "sfuse=1" "sfuse=0" "sfuse=1#ctl" "sfuse=0#ctl" > "$OUT/short.json" 2> "$OUT/short.err" || { tail -20 "$OUT/short.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/short.json'))
print('short', {k: round(v['GBps']) for k, v in d['results'].items()})"
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 64 --rounds ${ROUNDS:-4} --variants "sfuse=1" "sfuse=0" "sfuse=1#ctl" "sfuse=0#ctl" > "$OUT/C.json" 2> "$OUT/C.err" || { tail -20 "$OUT/C.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/C.json'))
print('C', {k: round(v['GBps']) for k, v in d['results'].items()})"
