#!/bin/bash
# Round-3 PMC traffic passes (FETCH_SIZE, WRITE_SIZE; separate runs) and kernel-trace stats for
# the given configs.  Usage (via gpurun): tools/r03_pmc.sh TAG "c3 c4 c5"
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:?tag}
CFGS=${2:-c3 c4 c5}
mkdir -p gpurun_out
for CFG in $CFGS; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${T}_${CFG}_$c -o pmc \
      -- python3 -u bench.py --config $CFG --steps 5 --warmup 3 --no-cpu-baseline --no-timing \
      --realtime-seconds 0 --capacity-ladder "" > gpurun_out/${T}_pmc_${CFG}_$c.log 2>&1 || exit 1
  done
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T}_${CFG} -o bench \
    -- python3 -u bench.py --config $CFG --steps 40 --warmup 5 --no-cpu-baseline --realtime-seconds 0 \
    --capacity-ladder "" > gpurun_out/prof_${T}_${CFG}.json 2> gpurun_out/prof_${T}_${CFG}.err || exit 1
done
