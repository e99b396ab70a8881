#!/bin/bash
# Waterfall kernel A/B: production radix-16 Stockham vs the wave-local kernel (OWRX_WF_KERNEL=wl)
# at N = 16384: parity of the variant, then the kernel alone (tools/wf_micro.py) and in situ (the
# default C3 bench under rocprofv3 --kernel-trace --stats), alternating A B A B on one box.
# Usage (via gpurun from the repo root): tools/wf_wl_ab.sh TAG [VARIANT]
R=${1:?tag}; V=${2:-wl}
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "variants and $V" -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/${R}_parity.log 2>&1 || exit 1
for v in "" "$V" "" "$V"; do
  tag=${v:-r16}
  if [ -n "$v" ]; then export OWRX_WF_KERNEL="$v"; else unset OWRX_WF_KERNEL; fi
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${R}_micro_$tag -o run \
    -- python3 tools/wf_micro.py 16384 > gpurun_out/${R}_micro_$tag.log 2>&1 || exit 1
  echo "micro $tag" >> gpurun_out/${R}_ab.txt
  python3 tools/prof_db_stats.py gpurun_out/${R}_micro_$tag/run_results.db wf_ >> gpurun_out/${R}_ab.txt
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${R}_situ_$tag -o bench \
    -- python3 -u bench.py --steps 20 --warmup 10 --no-cpu-baseline --realtime-seconds 0 --capacity-ladder "" \
    > gpurun_out/${R}_situ_$tag.json 2> gpurun_out/${R}_situ_$tag.log || exit 1
  echo "situ $tag $(python3 -c "import json; d=json.load(open('gpurun_out/${R}_situ_$tag.json')); print(d['value'], d['ms_per_step'])")" >> gpurun_out/${R}_ab.txt
  grep -h 'wf_' $(find gpurun_out/${R}_situ_$tag -name '*kernel_stats.csv') | cut -c1-160 >> gpurun_out/${R}_ab.txt
done
