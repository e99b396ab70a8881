#!/bin/bash
# Same-box A/B of an engine environment switch on the default bench (run via gpurun from the repo
# root).  Usage: tools/ab_env.sh TAG VAR VALUE_A VALUE_B   (empty value = unset)
R=${1:?tag}; VAR=${2:?var}; A=$3; B=$4
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in "$A" "$B" "$A" "$B"; do
  if [ -n "$v" ]; then export $VAR="$v"; else unset $VAR; fi
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --realtime-seconds 0 --capacity-ladder "" \
    > gpurun_out/${R}_ab.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/${R}_ab.json')); print('$VAR=$v', d['value'], d['ms_per_step'], d['kernels_ms_per_block'], d['roofline']['achieved'])" >> gpurun_out/${R}_ab.txt
done
