#!/bin/bash
# DDC segment-count sweep on the default bench (diagnostic)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
OWRX_VERBOSE=1 timeout -k 10 120 python -u bench.py --no-cpu-baseline --realtime-seconds 0 > gpurun_out/sw_auto.json 2> gpurun_out/sw_auto.err || exit $?
for s in "$@"; do
  OWRX_DDC_NSEG=$s timeout -k 10 120 python -u bench.py --no-cpu-baseline --realtime-seconds 0 > gpurun_out/sw_$s.json 2> gpurun_out/sw_$s.err || exit $?
done
