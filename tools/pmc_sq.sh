#!/bin/bash
# Counter passes over a short bench run (one --pmc group per pass, each its own process).
R=${1:?tag}
shift
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 -L > gpurun_out/${R}_counters.txt 2>&1 || true
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc_${R}_$i -o pmc \
    -- python -u bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-timing --realtime-seconds 0 > gpurun_out/${R}_pmc_$i.log 2>&1
  rc=$?; echo "pmc [$grp] rc=$rc" >> gpurun_out/${R}_pmc_$i.log; [ $rc -eq 0 ] || exit $rc
done
