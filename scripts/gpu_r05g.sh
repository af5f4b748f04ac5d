#!/bin/bash
# Short rows: per-kernel times of the row-parallel decode and the streaming / L2 forms (rocprofv3 stats).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-r05g}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 scripts/tune_decode.py --config C --shards 16 --blob 32,256 --chars 8,64 --rounds 2 \
  --variants "rows=-1" "rows=-1,srows=1" "rows=-1,srows=2" > "$OUT/stats_run.json" 2> "$OUT/stats_run.err" \
  || { tail -20 "$OUT/stats_run.err"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
out = sys.argv[1]
for p in glob.glob(f'{out}/trace/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(p)):
        print(f"{r['Name'][:90]:90s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
