#!/bin/bash
# Same-box A/B of fc_mac's operand path at C4's per-GPU share (128 chains, D = 5120: one
# workgroup per CU, so the ring runs 4 slots deep): registers (OWRX_FC_MAC=reg) vs the LDS-DMA
# ring (default); C4 / fast-convolution parity tests first; one summary line per run in
# gpurun_out/r03ap_ab.txt.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
run() {  # tag, args, env...
  local tag=$1 args=$2; shift 2
  env "$@" timeout -k 10 200 python3 -u bench.py $args --warmup 5 --no-cpu-baseline \
    --realtime-seconds 0 --capacity-ladder "" --churn-chains 0 --extra-block 0 \
    > gpurun_out/r03ap_$tag.json 2> gpurun_out/r03ap_$tag.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['bound'], r['frac'], r['achieved'], d['kernels_ms_per_block'])" \
    gpurun_out/r03ap_$tag.json $tag >> gpurun_out/r03ap_ab.txt
}
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_full_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "c4 or fast_convolution or large_groups" > gpurun_out/r03ap_pytest.log 2>&1 || exit 1
for rep in 1 2 3; do
  run c4_lds_$rep "--config c4 --steps 20" X=1
  run c4_reg_$rep "--config c4 --steps 20" OWRX_FC_MAC=reg
done
