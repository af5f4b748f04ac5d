#!/bin/bash
# rocprofv3 evidence for the bench: kernel-trace stats, then FETCH_SIZE and WRITE_SIZE in separate
# --pmc passes (never combined with tracing domains). Output under gpurun_out/$TAG/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-prof}
mkdir -p "$OUT"
ARGS="${BENCH_ARGS:---steps 20 --warmup 3 --cpu-seconds 0}"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python bench.py $ARGS > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python bench.py $ARGS > "$OUT/fetch.log" 2>&1 || { tail -20 "$OUT/fetch.log"; exit 1; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python bench.py $ARGS > "$OUT/write.log" 2>&1 || { tail -20 "$OUT/write.log"; exit 1; }
python scripts/pmc_summary.py "$OUT" > "$OUT/summary.json" && cat "$OUT/summary.json"
