#!/bin/bash
# Same-box A/B of the intra-device ordering events (evA, evF, evC, row evWf): device scope
# (default) vs system scope (OWRX_EV_FENCE=system); the whole GPU suite first, then C3 bench
# runs (100 steps x 4 blocks of 2^20) alternating, one summary line each in gpurun_out/r03an_ab.txt.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 800 python3 -u -m pytest tests -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r03an_pytest.log 2>&1 || exit 1
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 -u bench.py --steps 100 --warmup 5 --no-cpu-baseline \
    --realtime-seconds 0 --capacity-ladder "" --churn-chains 0 --extra-block 0 \
    > gpurun_out/r03an_$tag.json 2> gpurun_out/r03an_$tag.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], r['frac'], d['kernels_ms_per_block'])" \
    gpurun_out/r03an_$tag.json $tag >> gpurun_out/r03an_ab.txt
}
for rep in 1 2 3; do
  run dev_$rep X=1
  run sys_$rep OWRX_EV_FENCE=system
done
