#!/bin/bash
# A/B of two library builds on one box: parity tests on the new build, then tune_decode runs of
# each build alternated (MDSX_LIBRARY selects the build per process). BASE: the other build's path.
# NEWLIB: the build to test (default: the in-tree one). CARGS: tune_decode arguments; VARS: its
# variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p "$OUT"
export TMPDIR=/tmp
BASE=${BASE:?set BASE to the other build of libmdsx.so (e.g. one built from an earlier commit)}
if [ -z "$NOTEST" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
fi
for i in 1 2; do
  for lib in new base; do
    if [ $lib = base ]; then export MDSX_LIBRARY=$BASE
    elif [ -n "$NEWLIB" ]; then export MDSX_LIBRARY=$NEWLIB
    else unset MDSX_LIBRARY; fi
    timeout -k 10 300 python3 scripts/tune_decode.py ${CARGS:---config C --shards 64} --rounds 3 --variants ${VARS:-run=4} > "$OUT/$lib$i.json" 2> "$OUT/$lib$i.err" || { tail -20 "$OUT/$lib$i.err"; exit 1; }
    python3 -c "
import json; d = json.load(open('$OUT/$lib$i.json'))
print('$lib$i', d['rows'], {k: round(v['GBps']) for k, v in d['results'].items()})"
  done
done
