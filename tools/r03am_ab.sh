#!/bin/bash
# Same-box A/B of the flush's waterfall row encoders: whole chip (default) vs the row slot's
# own CUs (OWRX_FLUSH_ROWS=masked); waterfall parity tests first, then the driver's bench
# arguments (20 steps x 4 blocks: the final flush is inside the timed region) alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "waterfall or fft or adpcm or full_config or c4 or shim or spectrum" \
  > gpurun_out/r03am_pytest.log 2>&1 || exit 1
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline \
    --realtime-seconds 0 --capacity-ladder "" --churn-chains 0 --extra-block 0 \
    > gpurun_out/r03am_$tag.json 2> gpurun_out/r03am_$tag.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['frac'], d['kernels_ms_per_block'])" \
    gpurun_out/r03am_$tag.json $tag >> gpurun_out/r03am_ab.txt
}
for rep in 1 2 3; do
  run wide_$rep X=1
  run masked_$rep OWRX_FLUSH_ROWS=masked
done
