#!/bin/bash
# Streaming decode's lean path (seg_decode_kernel) on the GPU box: parity of its modes (copy-mode
# tests + fuzz), then A/B against the general streaming decode on config C.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-seg}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests/test_device_copy_modes.py tests/test_device_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread -k "${PYTEST_K:-seg or fuzz}" > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
VC="${VC:-run=4 run=8,seg=1 run=16,seg=1 run=8,seg=1,rkb=64 run=16,seg=1,rkb=64 run=16,seg=1,rkb=128 run=8,seg=1,rnt=1}"
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards ${SHARDS:-64} --rounds 3 --variants $VC > "$OUT/C.json" 2> "$OUT/C.err" || { tail -30 "$OUT/C.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/C.json'))
print('C', d['rows'], {k: (round(v['GBps']), round(v['median_ms'], 4)) for k, v in d['results'].items()})"
