#!/bin/bash
# Three default bench lines on one box (box-internal spread of the headline numbers); output under
# gpurun_out/${TAG:-rep}/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-rep}
mkdir -p "$OUT"
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --cpu-seconds 0 > "$OUT/b$i.json" 2> "$OUT/b$i.err" || { tail -20 "$OUT/b$i.err"; exit 1; }
done
python3 - "$OUT" <<'PY'
import json, sys
for i in (1, 2, 3):
    d = json.loads(open(f'{sys.argv[1]}/b{i}.json').read().strip().splitlines()[-1])
    r, c = d['roofline'], d['config_c']['roofline']
    print(i, round(d['value'] / 1e6, 1), 'B', round(r['frac'], 3), round(r['step_frac'], 3), 'C',
          round(c['frac'], 3), round(c['step_frac'], 3), 'copy', round(r['copy_ceiling_same_run']['GBps']))
PY
