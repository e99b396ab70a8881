#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for cus in 0 12 24 6; do
  OWRX_SERIAL_CUS=$cus timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r18_$cus.json 2> gpurun_out/r18_$cus.err || exit $?
done
OWRX_SERIAL_CUS=12 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r18 -o bench -- python bench.py --steps 20 --warmup 10 --no-cpu-baseline > gpurun_out/r18_prof.log 2>&1
