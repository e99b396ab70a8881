#!/bin/bash
# PMC passes over tools/micro/fc_bench (fc_mac alone at C3's shape): MFMA busy vs wave cycles,
# and the L1 -> L2 request traffic (run via gpurun from the repo root).
cd "$GRAFT_REPO_ROOT/tools/micro" || exit 1
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD \
  --output-format csv -d $O/fcpmc1 -o p -- ./fc_bench 256 192 31 833 3 > $O/fcpmc1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum \
  --output-format csv -d $O/fcpmc2 -o p -- ./fc_bench 256 192 31 833 3 > $O/fcpmc2.log 2>&1 || exit 1
