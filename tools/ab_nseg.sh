#!/bin/bash
# Same-box A/B of the DDC segment count: automatic choice vs OWRX_DDC_NSEG=$2, per config,
# interleaved twice (run via gpurun from the repo root).  tools/ab_nseg.sh TAG NSEG [configs...]
R=${1:?tag}
N=${2:?nseg}
shift 2
CONFIGS=${*:-c2 c3 c4}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for rep in 1 2; do
  for c in $CONFIGS; do
    timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline --realtime-seconds 0 \
      >> gpurun_out/${R}_auto_$c.json 2>/dev/null || exit 1
    OWRX_DDC_NSEG=$N timeout -k 10 200 python -u bench.py --config $c --no-cpu-baseline \
      --realtime-seconds 0 >> gpurun_out/${R}_n${N}_$c.json 2>/dev/null || exit 1
  done
done
