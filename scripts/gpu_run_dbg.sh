#!/bin/bash
# Streaming decode: parity of its modes, then timing with parts skipped (sdbg) on config C and short rows.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out/${TAG:-rundbg} && export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-rundbg}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "${PYTEST_K:-run}" > "$OUT/pytest_gpu.log" 2>&1 || { tail -60 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
V="${V:-tile=16 run=8 run=4 run=8,sdbg=16 run=8,sdbg=1,nocheck run=8,sdbg=2,nocheck run=8,sdbg=4,nocheck}"
IFS=';' read -r -a CFG_LIST <<< "${CFGS:-C;C --blob 32,256 --chars 8,64;C --blob 256,1024 --chars 64,256}"
for cfg in "${CFG_LIST[@]}"; do
timeout -k 10 300 python3 scripts/tune_decode.py --config $cfg --shards 16 --rounds 3 --variants $V > $OUT/t.json 2> $OUT/t.err || { tail -30 $OUT/t.err; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/t.json'))
print('$cfg', d['rows'])
for k, v in d['results'].items(): print('%-28s %8.3f ms %6d GB/s' % (k, v['median_ms'], v['GBps']))
print(d['phase_cycles_per_tile'])"
done
