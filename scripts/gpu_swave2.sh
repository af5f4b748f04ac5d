#!/bin/bash
# One sample per wave (mdsx_swave.hip): where its time goes on config C -- per-wave stamps (swx=8),
# ablations (1 no UTF-8 check, 2 no edge stores, 4 register-path column only), occupancy by LDS
# pad -- in one process against the lean streaming path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-swave2}
mkdir -p "$OUT"
export TMPDIR=/tmp
export MDSX_PROBES=5,10
VARS=${VARS:-"swave=0 swave=1 swave=1,swx=1 swave=1,swx=2,nocheck swave=1,swx=4,nocheck swave=1,swx=7,nocheck swave=1,lpad=4 swave=1,lpad=8 swave=1,swx=8,nocheck swave=0#ctl"}
timeout -k 10 500 python3 scripts/tune_decode.py --config C --shards 64 --rounds ${ROUNDS:-3} --variants $VARS > "$OUT/C.json" 2> "$OUT/C.err" || { tail -20 "$OUT/C.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/C.json'))
print('C', {k: (round(v['GBps']), round(v.get('decode_GBps', 0))) for k, v in d['results'].items()})
print(json.dumps(d['phase_cycles_per_tile']))"
