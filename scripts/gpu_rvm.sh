#!/bin/bash
# Value-major writes in the row-parallel decode (MDSX_TUNE rvm=1): parity (copy modes, fuzz,
# golden), then short rows and 256-1024-byte rows in-process against the default.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-rvm}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_device_copy_modes.py tests/test_device_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-rows_vm}" > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 16 --blob 32,256 --chars 8,64 --rounds ${ROUNDS:-4} --variants "rvm=0" "rvm=1" "rvm=0#ctl" "rvm=1#ctl" > "$OUT/short.json" 2> "$OUT/short.err" || { tail -20 "$OUT/short.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/short.json'))
print('short', {k: round(v['GBps']) for k, v in d['results'].items()})"
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 16 --blob 256,1024 --chars 64,256 --rounds ${ROUNDS:-4} --variants "rvm=0" "rvm=1" > "$OUT/medium.json" 2> "$OUT/medium.err" || { tail -20 "$OUT/medium.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/medium.json'))
print('medium', {k: round(v['GBps']) for k, v in d['results'].items()})"
