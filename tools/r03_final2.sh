#!/bin/bash
# Round-3 final GPU pass, PMC first so the bench line carries this build's traffic: the GPU
# suite, smoke, FETCH_SIZE / WRITE_SIZE passes of C3 -> profiles/<TAG>_pmc_traffic_c3.json (copied
# to gpurun_out/), the driver's bench command, then rocprof kernel stats.  Usage: TAG
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
T=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${T}_c3_$c -o pmc \
    -- python3 -u bench.py --config c3 --steps 5 --warmup 3 --no-cpu-baseline --no-timing \
    --realtime-seconds 0 --capacity-ladder "" > gpurun_out/${T}_pmc_c3_$c.log 2>&1 || exit 1
done
python3 tools/pmc_traffic.py $T c3 gpurun_out/pmc_${T}_c3_FETCH_SIZE gpurun_out/pmc_${T}_c3_WRITE_SIZE || exit 1
cp profiles/${T}_pmc_traffic_c3.json gpurun_out/ || exit 1
timeout -k 10 800 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${T}_c3 -o bench \
  -- python3 -u bench.py --config c3 --steps 40 --warmup 5 --no-cpu-baseline --realtime-seconds 0 \
  --capacity-ladder "" --extra-block 0 > gpurun_out/prof_${T}_c3.json 2> gpurun_out/prof_${T}_c3.err || exit 1
