#!/bin/bash
# Check of the shape-selected fc_mac form (ring for multi-round grids, registers otherwise):
# fast-convolution / C4 parity tests, then one C3 and one C4 bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_full_configs.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "c4 or fast_convolution or large_groups or c3_256" > gpurun_out/r03aq_pytest.log 2>&1 || exit 1
for c in c3 c4; do
  timeout -k 10 200 python3 -u bench.py --config $c --steps 40 --warmup 5 --no-cpu-baseline --realtime-seconds 0 \
    --capacity-ladder "" --churn-chains 0 --extra-block 0 > gpurun_out/r03aq_$c.json 2> gpurun_out/r03aq_$c.err || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], r['frac'], r['traffic'], r['kernel'][:20])" gpurun_out/r03aq_$c.json $c >> gpurun_out/r03aq.txt
done
