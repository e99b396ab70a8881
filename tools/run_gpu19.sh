#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 60 ./tools/micro/adpcm_bench > gpurun_out/r19_adpcmb.log 2>&1 || exit $?
bash tools/run_gpu16.sh r19
