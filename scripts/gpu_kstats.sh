#!/bin/bash
# Per-kernel times of decode variants on one synthetic batch (rocprofv3 kernel trace).
#   TAG=... CFG="C --blob 32,256 --chars 8,64" V="run=0 rows=48,rmin=1000000000" bash scripts/gpu_kstats.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-kstats}
mkdir -p "$OUT"
CFG="${CFG:-C --blob 32,256 --chars 8,64}"
i=0
for v in ${V:-run=0}; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/p$i" -o run --output-format csv -- python3 scripts/tune_decode.py --config $CFG --shards 16 --rounds 1 --iters 10 --variants "$v" > "$OUT/t$i.json" 2> "$OUT/t$i.err" || { tail -30 "$OUT/t$i.err"; exit 1; }
  echo "== $v"
  f=$(find "$OUT/p$i" -name '*kernel_stats.csv' | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
    name = r['Name'].replace('(anonymous namespace)::', '')[:60]
    print('%-60s %6s calls %9.1f us avg' % (name, r['Calls'], float(r['AverageNs']) / 1e3))
PY
done
