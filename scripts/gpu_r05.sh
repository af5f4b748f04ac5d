#!/bin/bash
# Round-5 measurement steps on one GPU box (each step under its own time limit; the first failure
# ends the call). STEPS: any of test, sv, rows (default: all). OUT: gpurun_out/<TAG>.
#   test -- the GPU parity suite at the in-tree library
#   sv   -- config C, the lean path's variants (MDSX_TUNE sv) in one process (scripts/tune_decode.py)
#   rows -- short ragged rows, the in-tree library against BASE (another build), alternated
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r05}
mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-test sv rows}
for step in $STEPS; do
  case $step in
    test)
      timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
        ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
      tail -2 "$OUT/pytest_gpu.log"
      ;;
    sv)
      timeout -k 10 600 python3 scripts/tune_decode.py --config C --shards 64 --rounds ${ROUNDS:-4} \
        --variants ${SV_VARS:-"run=7" "sv=1" "sv=2" "sv=3" "sv=4" "sv=6" "sv=7" "run=7#ctl"} \
        > "$OUT/sv.json" 2> "$OUT/sv.err" || { tail -20 "$OUT/sv.err"; exit 1; }
      python3 -c "
import json; d = json.load(open('$OUT/sv.json'))
print('sv', {k: round(v['GBps']) for k, v in d['results'].items()})"
      ;;
    rows)
      BASE=${BASE:-streaming_amd/lib/libmdsx_r04.so}
      for i in 1 2; do
        for lib in new base; do
          if [ $lib = base ]; then export MDSX_LIBRARY=$BASE; else unset MDSX_LIBRARY; fi
          timeout -k 10 300 python3 scripts/tune_decode.py --config C --shards 16 --blob 32,256 \
            --chars 8,64 --rounds 3 --variants ${ROWS_VARS:-"rows=-1"} > "$OUT/rows_$lib$i.json" \
            2> "$OUT/rows_$lib$i.err" || { tail -20 "$OUT/rows_$lib$i.err"; exit 1; }
          python3 -c "
import json; d = json.load(open('$OUT/rows_$lib$i.json'))
print('rows $lib$i', {k: round(v['GBps']) for k, v in d['results'].items()})"
        done
      done
      unset MDSX_LIBRARY
      ;;
  esac
done
