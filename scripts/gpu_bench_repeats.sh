#!/bin/bash
# REPS default bench lines back to back on one box (box-to-box variance of the final sources).
# Output under gpurun_out/${TAG:-bench_repeats}/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-bench_repeats}
mkdir -p "$OUT"
for i in $(seq 1 ${REPS:-3}); do
  timeout -k 10 300 python3 bench.py > "$OUT/bench$i.json" 2> "$OUT/bench$i.err" || { tail -30 "$OUT/bench$i.err"; exit 1; }
  python3 - "$OUT/bench$i.json" "$i" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for name, r in (('B', d), ('C', d['config_c'])):
    rf = r['roofline']
    print(sys.argv[2], name, round(rf['frac'], 3), round(rf['step_frac'], 3),
          round(rf['frac_of_same_run_copy'], 3), round(rf['copy_ceiling_same_run']['GBps']))
PY
done
