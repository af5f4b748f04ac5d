#!/bin/bash
# tune_decode A/B in one process on the GPU (after the parity tests KSEL picks, unless SKIP_TESTS):
# CARGS = tune_decode arguments, VARIANTS = its variants. Output under gpurun_out/$TAG/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-tune}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests/test_device_copy_modes.py} -m gpu -x -q --timeout 120 --timeout-method thread -k "${KSEL:-default}" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
fi
for i in $(seq 1 ${REPS:-2}); do
  timeout -k 10 300 python3 -u scripts/tune_decode.py ${CARGS:---config C --shards 64} --rounds ${ROUNDS:-4} --variants $VARIANTS > "$OUT/r$i.json" 2> "$OUT/r$i.err" || { tail -20 "$OUT/r$i.err"; exit 1; }
  python3 -c "
import json; d = json.load(open('$OUT/r$i.json'))
for k, v in d['results'].items(): print('r$i', k, round(v['GBps']), round(v['median_ms'], 4))
for k, v in d.get('phase_cycles_per_tile', {}).items(): print('r$i', k, 'phase medians', v.get('median'))"
done
