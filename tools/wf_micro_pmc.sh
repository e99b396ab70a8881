#!/bin/bash
# Counter passes over the waterfall micro-benchmark (tools/micro/wf_bench, built beforehand):
# where the waves of each waterfall kernel spend their cycles.  Run via gpurun from the repo root.
# Usage: tools/wf_micro_pmc.sh TAG FRAMES
R=${1:?tag}
FT=${2:-366}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/${R}_counters_list.txt 2>&1 || true
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"
i=0
for grp in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${R}_pmc_$i -o pmc \
    -- ./tools/micro/wf_bench $FT > gpurun_out/${R}_pmc_$i.log 2>&1
  rc=$?; echo "pmc [$grp] rc=$rc" >> gpurun_out/${R}_pmc_$i.log; [ $rc -eq 0 ] || exit $rc
done
