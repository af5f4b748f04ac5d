#!/bin/bash
# Dissect the staged decode: parts skipped (measurement-only knob sdbg), tiles per workgroup, and
# one PMC pass of SQ counters on the default staged variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-stagedbg}
mkdir -p "$OUT"
export TMPDIR=/tmp
V="stage=0 stage=24 stage=24,sdbg=16 stage=64,fill=90,sdbg=16 stage=24,sdbg=1,nocheck stage=24,sdbg=2,nocheck stage=24,sdbg=4,nocheck stage=24,sdbg=6,nocheck stage=24,sdbg=8,nocheck stage=24,sdbg=15,nocheck stage=24,stiles=1 stage=24,stiles=8 stage=24,stiles=256"
timeout -k 10 300 python3 scripts/tune_decode.py --config C --shards 16 --rounds 3 --variants $V > "$OUT/dbg.json" 2> "$OUT/dbg.err" || { tail -30 "$OUT/dbg.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/dbg.json'))
for k, v in d['results'].items(): print('%-32s %8.3f ms %6d GB/s' % (k, v['median_ms'], v['GBps']))
for k, v in d['phase_cycles_per_tile'].items(): print(k, v)"
timeout -k 10 300 python3 scripts/tune_decode.py --config C --shards 16 --blob 32,256 --chars 8,64 --rounds 3 --variants stage=0 stage=24 stage=24,sdbg=16 stage=64,fill=90,sdbg=16 stage=24,sdbg=8,nocheck > "$OUT/short.json" 2> "$OUT/short.err" || { tail -30 "$OUT/short.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/short.json'))
for k, v in d['results'].items(): print('short %-32s %8.3f ms %6d GB/s' % (k, v['median_ms'], v['GBps']))
for k, v in d['phase_cycles_per_tile'].items(): print(k, v)"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS -d "$OUT/pmc" -o run --output-format csv -- python3 scripts/tune_decode.py --config C --shards 16 --rounds 1 --iters 2 --variants stage=24 > "$OUT/pmc.log" 2>&1 || { tail -20 "$OUT/pmc.log"; exit 1; }
python3 - <<PY
import csv, glob, collections
rows = []
for f in glob.glob('$OUT/pmc/**/*counter_collection.csv', recursive=True):
    rows += list(csv.DictReader(open(f)))
agg = collections.defaultdict(list)
for r in rows:
    if 'stage_decode' in r['Kernel_Name']:
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(agg.items()): print(k, sum(v) / len(v))
PY
