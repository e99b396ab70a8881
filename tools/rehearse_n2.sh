#!/bin/bash
# Rehearsal of bench.py's multi-GPU path on a one-GPU box (run via gpurun from the repo root):
# two ranks under torch.distributed.run share the card, the IQ broadcast goes over gloo (RCCL
# refuses two ranks on one device).  Checks that the N > 1 code path (chain sharding, rank-0
# stream + per-block broadcast into [history | block] windows, barrier + max-over-ranks timing,
# one JSON line from rank 0) runs end to end on real engines; the numbers are not a scaling
# measurement (both ranks share one GPU).  Usage: tools/rehearse_n2.sh TAG
R=${1:?tag}
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
OWRX_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 5 --capacity-ladder 256,4096 --capacity-seconds 1 \
  --capacity-hold-seconds 3 --no-cpu-baseline --dropin-clients 0 \
  > gpurun_out/${R}_n2.json 2> gpurun_out/${R}_n2.log
rc=$?; echo "n2 rc=$rc" >> gpurun_out/${R}_n2.log; exit $rc
