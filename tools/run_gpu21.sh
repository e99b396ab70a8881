#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/run_gpu16.sh r21 || exit $?
for cus in "16,4,4" "8,4,4" "0"; do
  OWRX_SERIAL_CUS=$cus timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/r21_$cus.json 2> gpurun_out/r21_$cus.err || exit $?
done
