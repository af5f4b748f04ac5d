#!/bin/bash
# rocprofv3 evidence for the bench: kernel-trace stats, then the L2's memory-side read requests by
# size and write requests in separate --pmc passes (never combined with tracing domains). Output under gpurun_out/$TAG/; the summary
# (per workload + kernel entries, read by bench.py's committed_traffic) in $TAG/pmc_summary.json.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-prof}
mkdir -p "$OUT"
ARGS="${BENCH_ARGS:---steps 20 --warmup 20 --cpu-seconds 0}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/trace.log" 2>&1 || { tail -20 "$OUT/trace.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d "$OUT/read" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/read.log" 2>&1 || { tail -20 "$OUT/read.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d "$OUT/write" -o run --output-format csv -- python3 bench.py $ARGS > "$OUT/write.log" 2>&1 || { tail -20 "$OUT/write.log"; exit 1; }
python3 scripts/pmc_summary.py "$OUT" > "$OUT/pmc_summary.json" && python3 -c "
import json; s = json.load(open('$OUT/pmc_summary.json'))
for e in s['entries']:
    print(e['workload_key'], e['kernel'], e.get('traffic_over_algorithmic'))"
