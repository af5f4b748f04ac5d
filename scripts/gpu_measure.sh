#!/bin/bash
# One GPU call for the round's evidence: the whole GPU suite, smoke(), the default bench line,
# then rocprofv3 (kernel-trace stats with the bench line printed under it, and the memory-side
# read / write request counters in separate passes: scripts/profile_bench.sh) and the SQ issue /
# wait counters of the config-C decode (scripts/gpu_sq.sh). Output under gpurun_out/$TAG/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
TAG=${TAG:-measure}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -20 "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "
import json; d = json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
r, c = d['roofline'], d['config_c']['roofline']
print('B', round(d['ms_per_step'], 4), 'frac', round(r['frac'], 3), 'step', round(r['step_frac'], 3), 'copy', r['copy_ceiling_same_run'] and round(r['copy_ceiling_same_run']['GBps']))
print('C', round(d['config_c']['ms_per_step'], 4), 'frac', round(c['frac'], 3), 'step', round(c['step_frac'], 3), c['kernel'])
print('cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value']))"
[ -n "$SKIP_PROF" ] && exit 0
TAG=$TAG/prof bash scripts/profile_bench.sh || exit 1
TAG=$TAG/sq SET1=1 RUNS="${SQ_RUNS:-C:run=8,seg=1,rnt=1 C:run=4,seg=0,rnt=0}" bash scripts/gpu_sq.sh > "$OUT/sq.txt" 2>&1 || { tail -20 "$OUT/sq.txt"; exit 1; }
cat "$OUT/sq.txt"
# gpurun copies back at most 64 MiB: list the largest files, then drop the per-dispatch counter
# dumps the summaries above were made from and compress the kernel traces
du -ak "$OUT" | sort -n | tail -8
find "$OUT" -name '*counter_collection.csv' -size +1M -delete
find "$OUT" -name '*kernel_trace.csv' -size +1M -exec gzip -9 {} \;
du -sk "$OUT"
