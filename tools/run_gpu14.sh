#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r14_bench.json 2> gpurun_out/r14_bench.err || exit $?
timeout -k 10 300 python bench.py --steps 60 --warmup 3 --no-cpu-baseline > gpurun_out/r14_bench60.json 2>> gpurun_out/r14_bench.err || exit $?
