#!/bin/bash
# A/B of the blocks in flight (kSlots): the default library vs builds with OWRX_SLOTS=6 / 8
# (tools/ab_libs/, built by hand from engine.hip -DOWRX_SLOTS=N), C3 at 2^20, alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-ab}
for rep in 1 2; do
  for v in 4 6 8; do
    if [ $v = 4 ]; then lib=openwebrx_amd/libowrx_amd.so; else lib=tools/ab_libs/libowrx_amd_s$v.so; fi
    OWRX_AMD_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 80 --warmup 5 --no-cpu-baseline \
      --realtime-seconds 0 --capacity-ladder "" > gpurun_out/${T}_s${v}_$rep.json 2>/dev/null || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'], d['host_ms_per_block'])" gpurun_out/${T}_s${v}_$rep.json s$v
  done
done
