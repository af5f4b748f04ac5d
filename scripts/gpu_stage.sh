#!/bin/bash
# Staged-decode check on the GPU box: full GPU parity suite, the bench line, then A/B of the
# staged decode against the register-copy decode on config C and on short rows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-stage}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
python3 -c "
import json; l = json.load(open('$OUT/bench.json'))
for x in (l, l['config_c']):
    r = x['roofline']; print(r['kernel'], 'kern %.3f scan %.3f frac %.3f step_frac %.3f' % (r['kernel_ms'], r['scan_ms'], r['frac'], r['step_frac']))"
timeout -k 10 300 python3 scripts/tune_decode.py --config C --shards 64 --rounds 3 --variants stage=0 stage=24,fill=70 stage=16,fill=70 stage=32,fill=70 stage=24,fill=90 stage=32,fill=55 stage=20,fill=85 stage=40,fill=45 > "$OUT/tune_C.json" 2> "$OUT/tune_C.err" || { tail -30 "$OUT/tune_C.err"; exit 1; }
timeout -k 10 300 python3 scripts/tune_decode.py --config C --shards 16 --blob 32,256 --chars 8,64 --rounds 3 --variants stage=0 stage=24,fill=70 stage=16,fill=70 stage=32,fill=70 stage=48,fill=70 > "$OUT/tune_short.json" 2> "$OUT/tune_short.err" || { tail -30 "$OUT/tune_short.err"; exit 1; }
timeout -k 10 300 python3 scripts/tune_decode.py --config C --shards 16 --blob 256,1024 --chars 64,256 --rounds 3 --variants stage=0 stage=24,fill=70 stage=32,fill=70 stage=16,fill=90 > "$OUT/tune_medium.json" 2> "$OUT/tune_medium.err" || { tail -30 "$OUT/tune_medium.err"; exit 1; }
for f in tune_C tune_short tune_medium; do python3 -c "
import json; d = json.load(open('$OUT/$f.json'))
print('$f', d['rows'], {k: round(v['GBps']) for k, v in d['results'].items()})"; done
