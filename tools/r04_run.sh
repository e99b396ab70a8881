#!/bin/bash
# round-4 GPU steps (run via gpurun from the repo root): tools/r04_run.sh STEP...
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for st in "$@"; do
  case $st in
    micro) timeout -k 10 180 ./tools/micro/wf_r04 ${FT:-960} > gpurun_out/${TAG}_wf_micro.txt 2>&1 || exit $? ;;
    probe) timeout -k 10 120 ./tools/micro/cumask_probe > gpurun_out/${TAG}_cumask.txt 2>&1 || exit $? ;;
    stamps) timeout -k 10 180 ./tools/micro/wf_r04s ${FT:-960} > gpurun_out/${TAG}_wf_stamps.txt 2>&1 || exit $? ;;
    wftest) timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "waterfall" > gpurun_out/${TAG}_pytest_wf.log 2>&1 || exit $? ;;
    sel) timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "${SEL}" > gpurun_out/${TAG}_pytest_sel.log 2>&1 || exit $? ;;
    test) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1 || exit $? ;;
    bench) timeout -k 10 300 python -u bench.py --config ${CFG:-c3} --realtime-seconds 0 --capacity-ladder "" --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $? ;;
    full) timeout -k 10 1000 python -u bench.py --config ${CFG:-c3} ${BARGS} > gpurun_out/${TAG}_full.json 2> gpurun_out/${TAG}_full.err || exit $? ;;
    benchab)  # A/B of env settings (AB="NAME=VAL NAME2=VAL2 ..." one run each, plus the default)
      for v in default $AB; do
        if [ "$v" = default ]; then envs=""; else envs="$v"; fi
        env $envs timeout -k 10 300 python -u bench.py --config ${CFG:-c3} --realtime-seconds 0 --capacity-ladder "" --no-cpu-baseline --extra-block 0 > gpurun_out/${TAG}_ab_${v//[=,]/_}.json 2> gpurun_out/${TAG}_ab_${v//[=,]/_}.err || exit $?
      done ;;
    prof) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o bench \
        -- python -u bench.py --config ${CFG:-c3} --steps 20 --warmup 10 --no-cpu-baseline --realtime-seconds 0 --capacity-ladder "" > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.log || exit $? ;;
  esac
done
