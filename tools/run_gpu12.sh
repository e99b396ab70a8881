#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r12_bench_t.json 2> gpurun_out/r12_bench.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-timing > gpurun_out/r12_bench_nt.json 2>> gpurun_out/r12_bench.err || exit $?
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-timing --no-waterfall > gpurun_out/r12_bench_nwf.json 2>> gpurun_out/r12_bench.err || exit $?
