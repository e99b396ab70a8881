#!/bin/bash
# Round-3 final GPU pass: the whole GPU suite, smoke, the driver's bench command, then the
# rocprof kernel stats and PMC traffic passes of C3 (tools/r03_pmc.sh).  Usage: TAG
cd "$GRAFT_REPO_ROOT" || exit 1
T=${1:-r03fin}
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || exit 1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || exit 1
timeout -k 10 800 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || exit 1
tools/r03_pmc.sh $T c3
