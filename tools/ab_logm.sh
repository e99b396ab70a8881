cd "$GRAFT_REPO_ROOT" || exit 1
for lm in 256 192 256 192; do
  OWRX_FC_M=$lm timeout -k 10 200 python -u bench.py --no-cpu-baseline --realtime-seconds 0 --capacity-ladder "" > gpurun_out/ab_logm_$lm.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/ab_logm_$lm.json')); print('logm $lm', d['value'], d['kernels_ms_per_block'], d['roofline']['achieved'])" >> gpurun_out/ab_logm.txt
done
