#!/bin/bash
# Same-box A/B of the DDC forms at one config (run via gpurun from the repo root):
#   direct polyphase FIR (ddc_lds) vs fast convolution (fc_fwd / fc_mac / fc_out)
# Usage: tools/ab_ddc.sh TAG [config]
R=${1:?tag}
CFG=${2:-c3}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for form in direct fast direct fast; do
  timeout -k 10 300 python -u bench.py --config $CFG --ddc $form --no-cpu-baseline --realtime-seconds 0 \
    --capacity-ladder "" >> gpurun_out/${R}_ab_${CFG}.jsonl 2>> gpurun_out/${R}_ab_${CFG}.err || exit $?
done
for form in direct fast; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${R}_${CFG}_$form -o bench \
    -- python -u bench.py --config $CFG --ddc $form --steps 20 --warmup 10 --no-cpu-baseline --realtime-seconds 0 \
    --capacity-ladder "" > /dev/null 2>> gpurun_out/${R}_ab_${CFG}.err || exit $?
done
