#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/ -m gpu -q -p no:cacheprovider > gpurun_out/r23_pytest.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r23_pytest.log
