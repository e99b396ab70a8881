#!/bin/bash
# Same-box A/B of fc_mac's W tile (chains per tile T: 8 in-tree, 32 and 64 in tools/ab_libs):
# fast-convolution DDC parity tests on each build, then C3 bench runs (40 steps x 4 blocks of
# 2^20) alternating, one summary line per run in gpurun_out/r03aj_ab.txt.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for T in 8 32 64; do
  if [ $T = 8 ]; then L=openwebrx_amd/libowrx_amd.so; else L=tools/ab_libs/libowrx_amd_t$T.so; fi
  OWRX_AMD_LIB=$GRAFT_REPO_ROOT/$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider \
    -k "fast_convolution or large_groups or c3_256" > gpurun_out/r03aj_pytest_t$T.log 2>&1 || exit 1
done
run() {  # tag, lib
  OWRX_AMD_LIB=$GRAFT_REPO_ROOT/$2 timeout -k 10 200 python3 -u bench.py --steps 40 --warmup 5 --no-cpu-baseline \
    --realtime-seconds 0 --capacity-ladder "" --churn-chains 0 --extra-block 0 \
    > gpurun_out/r03aj_$1.json 2> gpurun_out/r03aj_$1.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], r['achieved'], r['frac'], d['kernels_ms_per_block'])" \
    gpurun_out/r03aj_$1.json $1 >> gpurun_out/r03aj_ab.txt
}
for rep in 1 2; do
  run t8_$rep openwebrx_amd/libowrx_amd.so
  run t32_$rep tools/ab_libs/libowrx_amd_t32.so
  run t64_$rep tools/ab_libs/libowrx_amd_t64.so
done
