#!/bin/bash
# Row-parallel decode A/B on the GPU: its parity tests first (KSEL picks them), then
# scripts/tune_decode.py on short and medium rows with the variants in VARIANTS, then (E2E=1) the
# config E end-to-end run. Output under gpurun_out/$TAG/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-rows_ab}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests/test_device_copy_modes.py tests/test_device_fuzz.py tests/test_device_decode.py} -m gpu -x -q --timeout 120 --timeout-method thread -k "${KSEL:-rows or default or fuzz or decode}" > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
fi
V=${VARIANTS:-"rows=-1 rows=-1#b rows=-1,sdbg=1,nocheck"}
for shape in "short 32,256 8,64" "medium 256,1024 64,256"; do
  set -- $shape
  timeout -k 10 300 python3 -u scripts/tune_decode.py --config C --shards 16 --blob $2 --chars $3 --rounds ${ROUNDS:-4} --variants $V > "$OUT/$1.json" 2> "$OUT/$1.err" || { tail -20 "$OUT/$1.err"; exit 1; }
  python3 -c "
import json; d = json.load(open('$OUT/$1.json'))
for k, v in d['results'].items(): print('$1', k, round(v['GBps']), round(v['median_ms'], 4))"
done
if [ -n "$E2E" ]; then
  timeout -k 10 600 python3 -u scripts/e2e_bench.py --config E --depth 2 3 --validate xxh3_64 > "$OUT/e2e_E.json" 2> "$OUT/e2e_E.err" || { tail -20 "$OUT/e2e_E.err"; exit 1; }
  python3 -c "
import json; d = json.load(open('$OUT/e2e_E.json'))
for k, v in d.items(): print('e2e', k, v)"
fi
