#!/bin/bash
# Short ragged rows through the row-parallel decode: optional GPU parity tests, then an
# in-process A/B (scripts/tune_decode.py) of MDSX_TUNE variants against the default. Round 6 ran
# it on the write-loop variants (MDSX_TUNE rv, mdsx_rows.hip kV, at the commit that held them)
# and on the UTF-8 ablations (profiles/r06/rows_var/). Output under gpurun_out/$TAG/.
# TESTS: pytest targets ('' skips); VARIANTS: tune_decode variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-rows_var}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
TESTS=${TESTS-}
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest $TESTS -m gpu -x -q --timeout 180 --timeout-method thread > "$OUT/pytest.log" 2>&1
  rc=$?
  tail -15 "$OUT/pytest.log"
  # a test failure (1) still measures; a fault, abort or time limit ends the call
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
for i in $(seq 1 ${REPS:-2}); do
  timeout -k 10 300 python3 -u scripts/tune_decode.py ${CARGS:---config C --shards 16 --blob 32,256 --chars 8,64} --rounds ${ROUNDS:-4} --variants $VARIANTS > "$OUT/r$i.json" 2> "$OUT/r$i.err" || { tail -20 "$OUT/r$i.err"; exit 1; }
  python3 -c "
import json; d = json.load(open('$OUT/r$i.json'))
for k, v in d['results'].items(): print('r$i', k, round(v['GBps']), round(v['median_ms'], 4), round(v.get('decode_ms', 0), 4))"
done
