#!/bin/bash
# Final round-6 evidence at the final library sources: the GPU suite and smoke, two default
# bench lines, then the rocprofv3 trace + PMC passes (profile_bench.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r06final}
mkdir -p "$OUT"
export TMPDIR=/tmp
# PART: all (default), tests (suite + smoke only) or bench (bench lines + profiles only)
PART=${PART:-all}
if [ "$PART" != bench ]; then
timeout -k 10 900 python3 -u -m pytest tests -m gpu --maxfail=20 -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -2 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -30 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
fi
[ "$PART" = tests ] && exit 0
for i in 1 2; do
  timeout -k 10 600 python3 bench.py > "$OUT/bench$i.json" 2> "$OUT/bench$i.err" || { tail -30 "$OUT/bench$i.err"; exit 1; }
  python3 - "$OUT/bench$i.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for name, r in (('B', d), ('C', d['config_c'])):
    rf = r['roofline']
    print(name, round(r['value']), round(r['ms_per_step'], 4), rf['kernel'], 'frac', round(rf['frac'], 3), 'step', round(rf['step_frac'], 3),
          'copy', round(rf['frac_of_same_run_copy'], 3), rf['copy_ceiling_same_run']['variant'], [round(x, 3) for x in rf['frac_blocks']], rf['traffic'])
PY
done
TAG=${TAG:-r06final}/prof bash scripts/profile_bench.sh || exit 1
# (gpurun returns at most 64 MiB: the per-launch trace and counter files compressed)
find "$OUT" -name '*.csv' -size +4M -exec gzip -9 {} \;
du -sh "$OUT"
