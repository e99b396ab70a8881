#!/bin/bash
# GPU round: parity tests, default bench line, kernel-trace profile (summary -> profiles/)
R=${1:-r16}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider > gpurun_out/${R}_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/${R}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py > gpurun_out/${R}_bench.json 2> gpurun_out/${R}_bench.err
rc=$?; echo "bench rc=$rc" >> gpurun_out/${R}_bench.err
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${R} -o bench -- python bench.py --steps 20 --warmup 10 --no-cpu-baseline > gpurun_out/${R}_prof.log 2>&1
echo "prof rc=$?" >> gpurun_out/${R}_prof.log
