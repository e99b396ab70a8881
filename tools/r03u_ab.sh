#!/bin/bash
# Round-3 A/B of the bench's blocks per step (1 vs 4 at the driver's 20 steps) and of 16 blocks
# in flight (OWRX_SLOTS=16 build in tools/ab_libs) with input retention 8, C3 at 2^20.
cd "$GRAFT_REPO_ROOT" || exit 1
run() {  # tag, env..., bench args
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --realtime-seconds 0 \
    --capacity-ladder "" --churn-chains 0 $BARGS > gpurun_out/r03u_$tag.json 2> gpurun_out/r03u_$tag.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['kernels_ms_per_block'], d['host_ms_per_block'])" gpurun_out/r03u_$tag.json $tag >> gpurun_out/r03u_ab.txt
}
for rep in 1 2; do
  BARGS="--blocks-per-step 1" run bps1_$rep X=1
  BARGS="--blocks-per-step 4" run bps4_$rep X=1
  BARGS="--blocks-per-step 4" run s16r8_$rep OWRX_AMD_LIB=tools/ab_libs/libowrx_amd_s16.so OWRX_BENCH_RETENTION=8
  BARGS="--blocks-per-step 4" run r8_$rep OWRX_BENCH_RETENTION=8
done
