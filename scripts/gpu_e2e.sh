#!/bin/bash
# GPU box: the pipeline / plugin / stream GPU tests, then the end-to-end benches (configs E, B, C)
# with verified, repeated passes. Output under gpurun_out/e2e/.
set -o pipefail
mkdir -p gpurun_out/e2e
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_device_pipeline.py tests/test_device_plugin_iter.py tests/test_device_streams.py \
  > gpurun_out/e2e/pytest.txt 2>&1 || exit 1
for cfg in E B C; do
  extra=""
  [ "$cfg" = E ] && extra="--validate xxh3_64 --trace e2e_with_d2h_overlapped_depth2,e2e_with_d2h_depth2"
  timeout -k 10 300 python -u scripts/e2e_bench.py --config $cfg $extra \
    --out gpurun_out/e2e/e2e_$cfg.json > gpurun_out/e2e/e2e_$cfg.log 2>&1 || exit 1
done
