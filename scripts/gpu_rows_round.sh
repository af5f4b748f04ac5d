#!/bin/bash
# One box: the row-parallel decode's variants in one process (gpu_tune.sh), then the in-tree build
# against BASE on short rows, then RINGLIB against BASE on config C (gpu_ab_lib.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
T=${TAG:-rr}
TAG=$T/tune SKIP_TESTS=${SKIP_TESTS-1} REPS=1 ROUNDS=3 CARGS="--config C --shards 16 --blob 32,256 --chars 8,64" VARIANTS="$RVARS" bash scripts/gpu_tune.sh || exit 1
TAG=$T/ab NOTEST=1 CARGS="--config C --shards 16 --blob 32,256 --chars 8,64" VARS="rows=-1" bash scripts/gpu_ab_lib.sh || exit 1
if [ -n "$RINGLIB" ]; then
  TAG=$T/ring NOTEST=1 NEWLIB=$RINGLIB CARGS="--config C --shards 64" VARS="run=7" bash scripts/gpu_ab_lib.sh || exit 1
fi
