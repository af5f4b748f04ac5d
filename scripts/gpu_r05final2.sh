#!/bin/bash
# Final bench evidence: two default bench lines, then the rocprofv3 trace + PMC passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r05final2}
mkdir -p "$OUT"
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 600 python3 bench.py > "$OUT/bench$i.json" 2> "$OUT/bench$i.err" || { tail -30 "$OUT/bench$i.err"; exit 1; }
  python3 - "$OUT/bench$i.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for name, r in (('B', d), ('C', d['config_c'])):
    rf = r['roofline']
    print(name, round(r['value']), round(r['ms_per_step'], 4), 'frac', round(rf['frac'], 3), 'step', round(rf['step_frac'], 3),
          'copy', round(rf['frac_of_same_run_copy'], 3), [round(x, 3) for x in rf['frac_blocks']], rf['traffic'])
PY
done
TAG=${TAG:-r05final2}/prof bash scripts/profile_bench.sh || exit 1
