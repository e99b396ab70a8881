#!/bin/bash
# rehearsal of the N>1 bench path on a 1-GPU box: 2 ranks sharing the GPU, gloo broadcast
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OWRX_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/r24_n2.json 2> gpurun_out/r24_n2.err
echo "rc=$?" >> gpurun_out/r24_n2.err
