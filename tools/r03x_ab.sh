#!/bin/bash
# A/B: waterfall row encoders on CUs of their own (default "4,4,4,4") vs sharing the gathers'
# CUs (round-2 layout "4,4,8"), C3 at the driver's 20/5 steps, alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
for rep in 1 2; do
  for cus in 4,4,4,4 4,4,8; do
    OWRX_SERIAL_CUS=$cus timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --realtime-seconds 0 \
      --capacity-ladder "" --churn-chains 0 > gpurun_out/r03x_$cus.$rep.json 2> gpurun_out/r03x_$cus.$rep.err || exit 1
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['kernels_ms_per_block'], d['host_ms_per_block'])" gpurun_out/r03x_$cus.$rep.json $cus >> gpurun_out/r03x_ab.txt
  done
done
