#!/bin/bash
# rocprofv3 kernel trace + stats of the C3 bench (round 3).  Usage: tools/r03_prof.sh TAG [bench args]
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:?tag}; shift
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$T -o bench \
  -- python3 -u bench.py --steps 40 --warmup 5 --no-cpu-baseline --realtime-seconds 0 --capacity-ladder "" "$@" \
  > gpurun_out/prof_$T.json 2> gpurun_out/prof_$T.err
