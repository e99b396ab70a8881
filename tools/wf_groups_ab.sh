#!/bin/bash
# Waterfall FFT in isolation at 1, 2 and 4 groups per CU (OWRX_WF_GROUPS_PER_CU): per-block
# kernel time by FFT size (run via gpurun from the repo root).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for g in 1 2 4; do
  OWRX_WF_GROUPS_PER_CU=$g timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/wfg$g -o run \
    -- python3 tools/wf_micro.py 4096 8192 16384 > gpurun_out/wfg$g.log 2>&1 || exit 1
  echo "groups/CU $g" >> gpurun_out/wfg.txt
  python3 tools/prof_db_stats.py gpurun_out/wfg$g/run_results.db wf_ >> gpurun_out/wfg.txt
done
