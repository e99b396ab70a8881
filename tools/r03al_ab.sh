#!/bin/bash
# Same-box A/B of fc_mac's operand path: registers (default) vs the LDS-DMA ring
# (OWRX_FC_MAC=lds, fc_mac_lds<FTT, CTT, 2>): fast-convolution parity tests with the ring, then C3
# bench runs (40 steps x 4 blocks of 2^20) alternating, one summary line each in
# gpurun_out/r03al_ab.txt.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || OWRX_FC_MAC=lds timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "fast_convolution or large_groups or c3_256" > gpurun_out/r03al_pytest_lds.log 2>&1 || exit 1
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --steps 100 --warmup 5 --no-cpu-baseline \
    --realtime-seconds 0 --capacity-ladder "" --churn-chains 0 --extra-block 0 \
    > gpurun_out/r03al_$tag.json 2> gpurun_out/r03al_$tag.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], r['achieved'], r['frac'], d['kernels_ms_per_block'])" \
    gpurun_out/r03al_$tag.json $tag >> gpurun_out/r03al_ab.txt
}
for rep in 3 4 5 6; do
  run reg_$rep X=1
  run lds_$rep OWRX_FC_MAC=lds
done
