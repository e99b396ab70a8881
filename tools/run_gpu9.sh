#!/bin/bash
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider > gpurun_out/r9_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r9_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/r9_bench.json 2> gpurun_out/r9_bench.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/r9_bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r9 -o bench -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r9_prof.log 2>&1
echo "prof rc=$?" >> gpurun_out/r9_prof.log
