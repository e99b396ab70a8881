#!/bin/bash
# One GPU verification pass (run via gpurun from the repo root):
#   parity tests -> smoke -> default bench line -> kernel-trace profile (summary -> profiles/)
# Usage: tools/gpu_round.sh TAG [stages...]   stages: test smoke bench prof pmc (default: all)
R=${1:?tag}
shift
STAGES=${*:-test smoke bench prof}
CFG=${CONFIG:-c3}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for st in $STAGES; do
  case $st in
    test)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        -p no:cacheprovider > gpurun_out/${R}_pytest.log 2>&1
      rc=$?; echo "pytest rc=$rc" >> gpurun_out/${R}_pytest.log; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${R}_smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc" >> gpurun_out/${R}_smoke.log; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 600 python -u bench.py --config $CFG > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err
      rc=$?; echo "bench rc=$rc" >> gpurun_out/${R}_bench.err; [ $rc -eq 0 ] || exit $rc ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${R} -o bench \
        -- python -u bench.py --config $CFG --steps 20 --warmup 10 --no-cpu-baseline --realtime-seconds 0 --capacity-ladder "" > gpurun_out/${R}_prof.json 2> gpurun_out/${R}_prof.log
      rc=$?; echo "prof rc=$rc" >> gpurun_out/${R}_prof.log; [ $rc -eq 0 ] || exit $rc ;;
    pmc)
      # HBM traffic of the dominant kernel: FETCH_SIZE and WRITE_SIZE in separate passes
      for c in FETCH_SIZE WRITE_SIZE; do
        timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${R}_${CFG}_$c -o pmc \
          -- python -u bench.py --config $CFG --steps 5 --warmup 3 --no-cpu-baseline --no-timing --realtime-seconds 0 --capacity-ladder "" > gpurun_out/${R}_pmc_$c.log 2>&1
        rc=$?; echo "pmc $c rc=$rc" >> gpurun_out/${R}_pmc_$c.log; [ $rc -eq 0 ] || exit $rc
      done ;;
  esac
done
