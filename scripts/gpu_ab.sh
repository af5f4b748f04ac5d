#!/bin/bash
# One GPU call: a pytest selection (PYTEST_ARGS), then tune_decode A/B runs (VC: config C
# variants, VB: config B variants; MDSX_PROBES=1 adds the copy-probe shapes). Output under
# gpurun_out/$TAG/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$PYTEST_ARGS" ]; then
  timeout -k 10 900 python3 -u -m pytest $PYTEST_ARGS ${PYTEST_K:+-k "$PYTEST_K"} -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
  tail -3 "$OUT/pytest_gpu.log"
fi
if [ -n "$VC" ]; then
  timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards ${SHARDS:-64} --rounds ${ROUNDS:-3} $CARGS --variants $VC > "$OUT/C.json" 2> "$OUT/C.err" || { tail -30 "$OUT/C.err"; exit 1; }
  python3 -c "
import json; d = json.load(open('$OUT/C.json'))
print('C', d['rows'], {k: (round(v['GBps']), round(v['median_ms'], 4)) for k, v in d['results'].items()})"
fi
for spec in "short:32,256:8,64:$VS" "medium:256,1024:64,256:$VM"; do
  IFS=: read -r nm blob chars vars <<< "$spec"
  [ -z "$vars" ] && continue
  timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards ${SHARDS_S:-16} --blob $blob --chars $chars --rounds ${ROUNDS:-3} --variants $vars > "$OUT/$nm.json" 2> "$OUT/$nm.err" || { tail -30 "$OUT/$nm.err"; exit 1; }
  python3 -c "
import json; d = json.load(open('$OUT/$nm.json'))
print('$nm', d['rows'], {k: (round(v['GBps']), round(v['median_ms'], 4)) for k, v in d['results'].items()})"
done
if [ -n "$VB" ]; then
  timeout -k 10 400 python3 scripts/tune_decode.py --config B --rounds ${ROUNDS:-3} --variants $VB > "$OUT/B.json" 2> "$OUT/B.err" || { tail -30 "$OUT/B.err"; exit 1; }
  python3 -c "
import json; d = json.load(open('$OUT/B.json'))
print('B', d['rows'], {k: (round(v['GBps']), round(v['median_ms'], 4)) for k, v in d['results'].items()})"
fi
