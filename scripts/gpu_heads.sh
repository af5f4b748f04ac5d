#!/bin/bash
# The sparse-heads microbenchmark: timing, then the L2's memory-side read requests by size per
# kernel (one --pmc pass).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-heads}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/microbench/sparse_heads > "$OUT/time.jsonl" 2> "$OUT/time.err" || { tail -20 "$OUT/time.err"; exit 1; }
cat "$OUT/time.jsonl"
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d "$OUT/read" -o run --output-format csv -- ./scripts/microbench/sparse_heads > "$OUT/read.log" 2>&1 || { tail -20 "$OUT/read.log"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, os, re, sys, collections
out = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(os.path.join(out, 'read', '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        k = re.search(r'heads<(\d+)>', r['Kernel_Name'])
        if k:
            acc[(int(k.group(1)), r['Counter_Name'])].append(float(r['Counter_Value']))
# launches in order: per stride 6 policies x 6 launches; report per policy the list of means
for (p, c), v in sorted(acc.items()):
    per = [round(sum(v[i:i + 6]) / 6) for i in range(0, len(v), 6)]
    print(p, c, per)
PY
