#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel stats. Stops at the first
# failing step (each step has its own time limit).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${TAG:-run}
mkdir -p "$OUT"
export TMPDIR=/tmp
python3 -c "import torch;print(torch.__version__, torch.cuda.get_device_name(0))" > "$OUT/env.txt" 2>&1 || exit 1
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { tail -30 "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
timeout -k 10 600 python3 bench.py ${BENCH_ARGS} > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -30 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
if [ -n "$PROFILE" ]; then
  TAG=${TAG:-run}/prof bash scripts/profile_bench.sh || exit 1
fi
