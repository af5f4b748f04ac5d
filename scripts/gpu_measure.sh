#!/bin/bash
# The round's evidence: the whole GPU suite and smoke() (SKIP_BENCH=1: only these), then
# rocprofv3 (kernel-trace stats with the bench line printed under it, and the memory-side read /
# write request counters in separate passes: scripts/profile_bench.sh; SKIP_TESTS=1: only these
# and what follows), the default bench line, the one-rank process-group bench (--dist) and the SQ
# issue / wait counters of the config-C and short-row decodes (scripts/gpu_sq.sh). Output under
# gpurun_out/$TAG/.
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
[ -n "$SKIP_BENCH" ] && exit 0
# the PMC summary first, put where bench.py looks for it (PROFDIR, e.g. profiles/r04/final), so
# the bench line below carries its traffic
if [ -z "$SKIP_PROF" ]; then
  TAG=$TAG/prof bash scripts/profile_bench.sh || exit 1
  if [ -n "$PROFDIR" ]; then mkdir -p "$PROFDIR" && cp "$OUT/prof/pmc_summary.json" "$PROFDIR/pmc_summary.json"; fi
fi
timeout -k 10 600 python3 bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
python3 -c "
import json; d = json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1])
r, c = d['roofline'], d['config_c']['roofline']
print('B', round(d['ms_per_step'], 4), 'frac', round(r['frac'], 3), 'step', round(r['step_frac'], 3), 'traffic', r['traffic'], 'copy', r['copy_ceiling_same_run'] and round(r['copy_ceiling_same_run']['GBps']))
print('C', round(d['config_c']['ms_per_step'], 4), 'frac', round(c['frac'], 3), 'step', round(c['step_frac'], 3), 'traffic', c['traffic'], c['kernel'])
print('cpu', d['cpu_baseline'] and round(d['cpu_baseline']['value']))"
timeout -k 10 300 python3 bench.py --dist --steps 5 --warmup 5 --cpu-seconds 0 > "$OUT/bench_dist.json" 2> "$OUT/bench_dist.err" || { tail -20 "$OUT/bench_dist.err"; exit 1; }
tail -c 300 "$OUT/bench_dist.json"; echo
[ -n "$SKIP_SQ" ] && exit 0
TAG=$TAG/sq SET1=1 RUNS="${SQ_RUNS:-C:run=7}" bash scripts/gpu_sq.sh > "$OUT/sq.txt" 2>&1 || { tail -20 "$OUT/sq.txt"; exit 1; }
TAG=$TAG/sq_rows SET1=1 RUNS="C:rows=-1" CARGS="--blob 32,256 --chars 8,64" bash scripts/gpu_sq.sh > "$OUT/sq_rows.txt" 2>&1 || { tail -20 "$OUT/sq_rows.txt"; exit 1; }
cat "$OUT/sq.txt" "$OUT/sq_rows.txt"
# gpurun copies back at most 64 MiB: list the largest files, then drop the per-dispatch counter
# dumps the summaries above were made from and compress the kernel traces
du -ak "$OUT" | sort -n | tail -8
find "$OUT" -name '*counter_collection.csv' -size +1M -delete
find "$OUT" -name '*kernel_trace.csv' -size +1M -exec gzip -9 {} \;
du -sk "$OUT"
