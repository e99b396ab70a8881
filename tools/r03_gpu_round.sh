#!/bin/bash
# Round-3 GPU pass: the whole GPU test suite, then the C3 bench at 2^20 and 2^22 blocks.
# Usage (via gpurun, from the repo root): tools/r03_gpu_round.sh TAG [pytest -k expr]
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r03}
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > gpurun_out/${T}_pytest.log 2>&1 || exit 1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 1
fi
for cfg in "b20 --block 1048576" "b22 --block 4194304"; do
  set -- $cfg; t=$1; shift
  timeout -k 10 150 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --realtime-seconds 0 \
    --capacity-ladder "" "$@" > gpurun_out/${T}_bench_$t.json 2> gpurun_out/${T}_bench_$t.err || exit 1
done
