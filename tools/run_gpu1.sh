#!/bin/bash
cd $GRAFT_REPO_ROOT
rocminfo | grep -m1 gfx > gpurun_out/r1_info.log 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r1_smoke.log 2>&1
rc=$?
echo "smoke rc=$rc" >> gpurun_out/r1_smoke.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q --maxfail=4 -p no:cacheprovider > gpurun_out/r1_pytest.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r1_pytest.log
