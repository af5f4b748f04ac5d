#!/bin/bash
# Streaming decode on the GPU box: parity of its modes (copy-mode tests), then A/B against the
# register decode on config C, short and medium rows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-run}" > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
VC="${VC:-tile=16 run=8 run=8,rkb=32 run=8,rkb=128 run=4 run=16 run=16,rkb=256}"
timeout -k 10 300 python3 scripts/tune_decode.py --config C --shards 16 --rounds 3 --variants $VC > "$OUT/C.json" 2> "$OUT/C.err" || { tail -30 "$OUT/C.err"; exit 1; }
VS="${VS:-tile=32 run=8 run=8,rkb=16 run=8,rkb=256 run=4 run=16,rkb=256}"
timeout -k 10 300 python3 scripts/tune_decode.py --config C --shards 16 --blob 32,256 --chars 8,64 --rounds 3 --variants $VS > "$OUT/short.json" 2> "$OUT/short.err" || { tail -30 "$OUT/short.err"; exit 1; }
timeout -k 10 300 python3 scripts/tune_decode.py --config C --shards 16 --blob 256,1024 --chars 64,256 --rounds 3 --variants $VS > "$OUT/medium.json" 2> "$OUT/medium.err" || { tail -30 "$OUT/medium.err"; exit 1; }
for f in C short medium; do python3 -c "
import json; d = json.load(open('$OUT/$f.json'))
print('$f', d['rows'], {k: round(v['GBps']) for k, v in d['results'].items()})"; done
