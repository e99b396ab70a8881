#!/bin/bash
# GPU steps, run via gpurun from the repo root:  TAG=x [CFG=c3] [BARGS=...] tools/gpu_steps.sh STEP...
#   test     every -m gpu test                     -> gpurun_out/$TAG_pytest.log
#   sel      the -m gpu tests matching $SEL (-k)   -> gpurun_out/$TAG_pytest_sel.log
#   smoke    __graft_entry__.smoke()               -> gpurun_out/$TAG_smoke.log
#   bench    short bench line (no real-time/capacity/drop-in/CPU legs)  -> $TAG_bench.json
#   full     the default bench (every leg)          -> $TAG_full.json
#   benchab  the short bench per environment setting in $AB ("VAR=V VAR2=W"; plus the default)
#   prof     rocprofv3 --kernel-trace --stats of the short bench  -> gpurun_out/prof_$TAG/
#   pmc      rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs) of the short bench
#            (tools/pmc_traffic.py turns them into profiles/<tag>_pmc_traffic_<cfg>.json)
#   micro / stamps / probe   tools/micro/wf_r04, wf_r04s (-DOWRX_WF_STAMPS), cumask_probe
# Each step has its own time limit; the first failing step ends the call.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
CFG=${CFG:-c3}
SHORT="--config $CFG --realtime-seconds 0 --capacity-ladder \"\" --no-cpu-baseline --dropin-clients 0"
for st in "$@"; do
  case $st in
    micro) timeout -k 10 180 ./tools/micro/wf_r04 ${FT:-960} > gpurun_out/${TAG}_wf_micro.txt 2>&1 || exit $? ;;
    stamps) timeout -k 10 180 ./tools/micro/wf_r04s ${FT:-960} > gpurun_out/${TAG}_wf_stamps.txt 2>&1 || exit $? ;;
    probe) timeout -k 10 120 ./tools/micro/cumask_probe > gpurun_out/${TAG}_cumask.txt 2>&1 || exit $? ;;
    test) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_pytest.log 2>&1 || exit $? ;;
    sel) timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "${SEL}" > gpurun_out/${TAG}_pytest_sel.log 2>&1 || exit $? ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || exit $? ;;
    bench) eval timeout -k 10 300 python -u bench.py $SHORT ${BARGS} > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit $? ;;
    full) timeout -k 10 1000 python -u bench.py --config $CFG ${BARGS} > gpurun_out/${TAG}_full.json 2> gpurun_out/${TAG}_full.err || exit $? ;;
    benchab)
      for v in default $AB; do
        if [ "$v" = default ]; then envs=""; else envs="${v//+/ }"; fi
        eval env $envs timeout -k 10 300 python -u bench.py $SHORT --extra-block 0 ${BARGS} > gpurun_out/${TAG}_ab_${v//[=,+.\/]/_}.json 2> gpurun_out/${TAG}_ab_${v//[=,+.\/]/_}.err || exit $?
      done ;;
    prof) eval timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG} -o bench \
        -- python3 -u bench.py $SHORT --steps 20 --warmup 5 --extra-block 0 ${BARGS} > gpurun_out/${TAG}_prof.json 2> gpurun_out/${TAG}_prof.log || exit $? ;;
    pmc)
      for c in FETCH_SIZE WRITE_SIZE; do
        eval timeout -s KILL 150 rocprofv3 --pmc $c --output-format csv -d gpurun_out/pmc_${TAG}_${CFG}_$c -o pmc \
          -- python3 -u bench.py $SHORT --steps 20 --warmup 5 --no-timing --extra-block 0 ${BARGS} > gpurun_out/${TAG}_pmc_${CFG}_$c.log 2>&1 || exit $?
      done ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
