#!/bin/bash
# SQ counter pass over the default bench (run via gpurun from the repo root): where the waves of
# each kernel spend their cycles.  Usage: tools/sq_counters.sh TAG [config] [counters...]
R=${1:?tag}
CFG=${2:-c3}
shift 2
CTRS=${*:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc $CTRS --output-format csv -d gpurun_out/sq_${R}_${CFG} -o sq \
  -- python -u bench.py --config $CFG --steps 5 --warmup 3 --no-cpu-baseline --no-timing \
  --realtime-seconds 0 --capacity-ladder "" > gpurun_out/sq_${R}_${CFG}.log 2>&1
