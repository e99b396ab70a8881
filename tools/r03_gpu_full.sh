#!/bin/bash
# Round-3 GPU pass: the GPU test suite (optionally -k), then the default bench line (the driver's
# command: realtime + churn + capacity ladder + CPU baseline).  Usage: tools/r03_gpu_full.sh TAG [K]
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r03}
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/${T}_pytest.log 2>&1 || exit 1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 1
fi
timeout -k 10 900 python -u bench.py > gpurun_out/${T}_bench_default.json 2> gpurun_out/${T}_bench_default.err
