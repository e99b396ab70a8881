#!/bin/bash
# A/B of owrx_set_input_retention in the C3 bench at 2^20 (resident recording), alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-ab}
STEPS=${2:-200}
for rep in 1 2; do
  for r in 1 2 4 8; do
    OWRX_BENCH_RETENTION=$r timeout -k 10 200 python3 -u bench.py --steps $STEPS --warmup 5 --no-cpu-baseline \
      --realtime-seconds 0 --capacity-ladder "" > gpurun_out/${T}_r${r}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['kernels_ms_per_block'], d['host_ms_per_block'])" gpurun_out/${T}_r${r}_$rep.json r$r
  done
done
