#!/bin/bash
# Same-box A/B of two builds of libowrx_amd.so (run via gpurun from the repo root):
#   tools/ab_lib.sh TAG OTHER_LIB [configs...]
# Runs the DDC parity tests on the in-tree library first, then alternates bench runs of the
# in-tree library ("new") and OTHER_LIB ("old") twice per config, appending one JSON line per run
# to gpurun_out/TAG_ab_{old,new}_CONFIG.json.
R=${1:?tag}
OTHER=${2:?other library}
shift 2
CONFIGS=${*:-c2 c3}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider -k "nfm_chain or large_groups or c3 or c4 or modes or retune or wfm" \
  > gpurun_out/${R}_pytest.log 2>&1 || exit 1
for v in old new old new; do
  if [ $v = old ]; then L=$GRAFT_REPO_ROOT/$OTHER; else L=$GRAFT_REPO_ROOT/openwebrx_amd/libowrx_amd.so; fi
  for c in $CONFIGS; do
    OWRX_AMD_LIB=$L timeout -k 10 200 python -u bench.py --config $c --steps 30 --warmup 5 \
      --no-cpu-baseline --realtime-seconds 0 >> gpurun_out/${R}_ab_${v}_$c.json 2>/dev/null || exit 1
  done
done
