#!/bin/bash
# Same-box A/B of an engine environment switch, in situ on the default bench under
# rocprofv3 --kernel-trace --stats, values alternating twice; each value first passes the tests
# matching PYTEST_K (its own process: the switches are read once per process).
# Usage (via gpurun from the repo root): tools/ab_env_prof.sh TAG VAR KERNEL_GREP V1 V2 ...
# (value "-" = unset)
R=${1:?tag}; VAR=${2:?var}; KG=${3:?kernel}; shift 3
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" != "-" ]; then export $VAR="$v"; else unset $VAR; fi
  if [ -n "$PYTEST_K" ]; then
    timeout -k 10 400 python -u -m pytest tests -m gpu -k "$PYTEST_K" -x -q --timeout 120 \
      --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_test_$v.log 2>&1 || exit 1
    echo "$VAR=$v tests: $(tail -1 gpurun_out/${R}_test_$v.log)" >> gpurun_out/${R}_ab.txt
  fi
done
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" != "-" ]; then export $VAR="$v"; else unset $VAR; fi
    d=gpurun_out/${R}_prof_${v}_$rep
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o bench \
      -- python3 -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --realtime-seconds 0 --capacity-ladder "" \
      > $d.json 2> $d.log || exit 1
    line=$(python3 -c "import json; d=json.load(open('$d.json')); print(d['value'], d['ms_per_step'])")
    k=$(grep -h "$KG" $(find $d -name '*kernel_stats.csv') | awk -F'",' '{print $2}' | cut -d, -f1,3 | head -3 | tr '\n' ' ')
    echo "$VAR=$v rep $rep: Msps ms/step $line | $KG calls,avg_ns $k" >> gpurun_out/${R}_ab.txt
  done
done
