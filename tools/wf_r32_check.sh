#!/bin/bash
# radix-32 waterfall kernel: parity tests under OWRX_WF_KERNEL=r32, then a same-box A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
OWRX_WF_KERNEL=r32 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_full_configs.py -x -q \
  -k "waterfall or c4_gpu" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/wf_r32_tests.log 2>&1 || exit 1
bash tools/ab_env.sh wfr32 OWRX_WF_KERNEL "" r32
