#!/bin/bash
# Is the streaming decode bound by the scalar unit? Per-kernel SALU / VALU instruction counts
# and busy cycles next to the GPU's elapsed cycles (one --pmc pass per counter set), config C.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-salu}
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/counters.txt" 2>&1 || true
SETS=("SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
      "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU SQ_WAVES")
i=0
for set in "${SETS[@]}"; do
  i=$((i + 1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv -- python3 scripts/tune_decode.py --config C --shards 16 --rounds 1 --iters 2 --variants ${VARS:-run=4} > "$OUT/p$i.log" 2>&1 || { tail -5 "$OUT/p$i.log"; echo "pass $i failed"; continue; }
  python3 - "$OUT/p$i" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0]
        if 'decode_kernel' in k:
            agg[(k[-36:], r['Counter_Name'])].append(float(r['Counter_Value']))
for (k, c), v in sorted(agg.items()):
    print('%-36s %-24s %.4g' % (k, c, sum(v) / len(v)))
PY
done
