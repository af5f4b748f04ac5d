#!/bin/bash
# Occupancy (MDSX_TUNE lpad: unused LDS per workgroup) of the config-B register decode and the
# config-C lean path, in-process against the default, with the copy probe shapes incl. the
# occupancy-limited ones (7, 8).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-occ}
mkdir -p "$OUT"
export TMPDIR=/tmp
export MDSX_PROBES=1,5,7,8
timeout -k 10 400 python3 scripts/tune_decode.py --config B --rounds ${ROUNDS:-3} --variants ${VB:-"lpad=0" "lpad=22" "lpad=28" "lpad=36" "lpad=50" "lpad=72" "lpad=0#ctl"} > "$OUT/B.json" 2> "$OUT/B.err" || { tail -20 "$OUT/B.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/B.json'))
print('B', {k: round(v['GBps']) for k, v in d['results'].items()})"
timeout -k 10 400 python3 scripts/tune_decode.py --config C --shards 64 --rounds ${ROUNDS:-3} --variants ${VC:-"run=7" "run=7,lpad=5" "run=7,lpad=9" "run=7,lpad=13" "run=7#ctl"} > "$OUT/C.json" 2> "$OUT/C.err" || { tail -20 "$OUT/C.err"; exit 1; }
python3 -c "
import json; d = json.load(open('$OUT/C.json'))
print('C', {k: round(v['GBps']) for k, v in d['results'].items()})"
