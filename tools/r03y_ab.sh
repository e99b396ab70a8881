#!/bin/bash
# Long-run A/B (100 steps x 4 blocks of 2^20, C3): default; 16 slots + retention 8; row encoders
# sharing the gathers' CUs (round-2 layout), alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --steps 100 --warmup 5 --no-cpu-baseline --realtime-seconds 0 \
    --capacity-ladder "" --churn-chains 0 > gpurun_out/r03y_$tag.json 2> gpurun_out/r03y_$tag.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['kernels_ms_per_block'], d['host_ms_per_block'])" gpurun_out/r03y_$tag.json $tag >> gpurun_out/r03y_ab.txt
}
for rep in 1 2; do
  run def_$rep X=1
  run s16r8_$rep OWRX_AMD_LIB=tools/ab_libs/libowrx_amd_s16.so OWRX_BENCH_RETENTION=8
  run r448_$rep OWRX_SERIAL_CUS=4,4,8
  run s16r8w_$rep OWRX_AMD_LIB=tools/ab_libs/libowrx_amd_s16.so OWRX_BENCH_RETENTION=8 OWRX_SERIAL_CUS=4,4,8
done
