set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/rsq
timeout -k 10 300 python3 scripts/tune_decode.py --config C --shards 16 --blob 32,256 --chars 8,64 --rounds 3 --variants rows=-1 rows=-1,sdbg=64 > gpurun_out/rsq/phase.json 2> gpurun_out/rsq/phase.err || { tail -20 gpurun_out/rsq/phase.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/rsq/phase.json')); print({k: round(v['GBps']) for k,v in d['results'].items()}); print(json.dumps(d['phase_cycles_per_tile']))"
TAG=rsq/sq RUNS="C:rows=-1" CARGS="--blob 32,256 --chars 8,64" bash scripts/gpu_sq.sh
