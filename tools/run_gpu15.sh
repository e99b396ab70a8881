#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for v in "" "--no-timing" "--no-waterfall" "--no-timing --no-waterfall" "--warmup 10"; do
  echo "== $v" >> gpurun_out/r15.err
  timeout -k 10 300 python bench.py --steps 20 --no-cpu-baseline $v > gpurun_out/r15.json 2>> gpurun_out/r15.err || exit $?
  cat gpurun_out/r15.json >> gpurun_out/r15.all
done
