#!/bin/bash
# One sample per wave (mdsx_swave.hip) vs the lean streaming path on config C, in one process:
# cache policy, sample order (XCD-contiguous or launch order), scan tile size.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-swave7}
mkdir -p "$OUT"
export TMPDIR=/tmp
export MDSX_PROBES=5,10
VARS=${VARS:-"swave=0 swave=1 swave=1,rnt=0 swave=1,xcd=0 swave=1,swtile=256 swave=1,swtile=16 swave=0#ctl swave=1#ctl"}
timeout -k 10 500 python3 scripts/tune_decode.py --config C --shards 64 --rounds ${ROUNDS:-4} --variants $VARS > "$OUT/C.json" 2> "$OUT/C.err" || { tail -20 "$OUT/C.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/C.json'))
print('C', {k: (round(v['GBps']), round(v.get('decode_GBps', 0))) for k, v in d['results'].items()})"
