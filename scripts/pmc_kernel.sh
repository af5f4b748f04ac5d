#!/bin/bash
# PMC counters for one kernel of a command: one rocprofv3 --pmc pass per counter group.
# usage: TAG=x KERNEL=gather_ragged bash scripts/pmc_kernel.sh python scripts/tune_decode.py ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-pmck}
mkdir -p "$OUT"
CGROUPS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
        "SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
        "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum")
i=0
for g in "${CGROUPS[@]}"; do
  timeout -k 10 300 rocprofv3 --pmc $g -d "$OUT/p$i" -o run --output-format csv -- "$@" > "$OUT/p$i.log" 2>&1 || { tail -20 "$OUT/p$i.log"; exit 1; }
  i=$((i+1))
done
python - "$OUT" "${KERNEL:-gather}" <<'PY'
import csv, glob, os, sys, collections
out, kern = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for f in glob.glob(os.path.join(out, 'p*', '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r['Kernel_Name']:
            acc[(r['Kernel_Name'][:60], r['Counter_Name'])].append(float(r['Counter_Value']))
for (k, c), v in sorted(acc.items()):
    print(f'{k:60s} {c:24s} n={len(v):3d} mean={sum(v)/len(v):.4g}')
PY
