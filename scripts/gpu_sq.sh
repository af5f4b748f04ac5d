#!/bin/bash
# SQ counters (issue, waits, memory-pipe back-pressure) of the decode kernels, one --pmc pass per
# counter set and variant (8 SQ counters at most per pass). RUNS: "config:variant" pairs;
# CARGS: extra tune_decode arguments (e.g. "--blob 32,256 --chars 8,64").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-sq}
mkdir -p "$OUT"
export TMPDIR=/tmp
RUNS="${RUNS:-C:run=4 C:tile=16}"
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS"
      "SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_WR"
      "SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS")
[ -n "$SET1" ] && SETS=("${SETS[0]}")  # SET1=1: the issue / wait set only
i=0
for run in $RUNS; do
  cfg=${run%%:*}; var=${run#*:}
  for set in "${SETS[@]}"; do
    i=$((i + 1))
    timeout -s KILL 120 rocprofv3 --pmc $set -d "$OUT/p$i" -o run --output-format csv -- python3 scripts/tune_decode.py --config $cfg $CARGS --shards 16 --rounds 1 --iters 2 --variants $var > "$OUT/p$i.log" 2>&1 || { tail -20 "$OUT/p$i.log"; exit 1; }
    python3 - "$OUT/p$i" "$run" <<'PY'
import csv, glob, sys, collections
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'].replace('(anonymous namespace)::', '').split('(')[0]
        if 'decode_kernel' in k:
            agg[(k[-40:], r['Counter_Name'])].append(float(r['Counter_Value']))
for (k, c), v in sorted(agg.items()):
    print(sys.argv[2], '%-40s %-30s %.4g' % (k, c, sum(v) / len(v)))
PY
  done
done
