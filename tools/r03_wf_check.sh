#!/bin/bash
# Waterfall batching check (round 3): GPU tests of the waterfall / ring, then the C3 bench at
# 2^20-sample blocks with and without FFT batching and at 2^22.  Run via gpurun from the repo root.
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r03b}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "waterfall or ring" > gpurun_out/${T}_wf_tests.log 2>&1 || exit 1
for cfg in "b20 --block 1048576" "b20nb --block 1048576 --wf-batch 0" "b22 --block 4194304"; do
  set -- $cfg; t=$1; shift
  timeout -k 10 150 python -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --realtime-seconds 0 \
    --capacity-ladder "" "$@" > gpurun_out/${T}_bench_$t.json 2> gpurun_out/${T}_bench_$t.err || exit 1
done
