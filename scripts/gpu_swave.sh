#!/bin/bash
# One sample per one-wave workgroup for ragged plans (MDSX_TUNE swave, mdsx_swave.hip): parity
# (the copy-mode and fuzz suites in its modes, the full-size oracle check), then config C in one
# process against the lean streaming path (seg_decode_kernel), by occupancy and register window.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-swave}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_device_copy_modes.py tests/test_device_fuzz.py tests/test_malformed.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-swave or malformed or reference_outcomes or decode_sample}" > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
export MDSX_PROBES=5,10
VARS=${VARS:-"swave=0 swave=1 swave=1,swocc=4 swave=1,swocc=6 swave=1,swkb=8 swave=1,swtile=256 swave=0#ctl"}
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 64 --rounds ${ROUNDS:-4} --variants $VARS > "$OUT/C.json" 2> "$OUT/C.err" || { tail -20 "$OUT/C.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/C.json'))
print('C', {k: round(v['GBps']) for k, v in d['results'].items()})"
