#!/usr/bin/env python3
"""Records tests/golden/dsp_graph.json: the reference's own ClientDemodulatorChain
(owrx/dsp.py) driven over the pycsdr shim through a demodulator / secondary demodulator / NR
sequence (tests/dsp_probe.py), step by step -- the planner's result and the module graph the
reference code built.  Needs the reference checkout (this container); the GPU tests replay the
recorded graphs with the shim's modules.

usage: python tests/golden/make_dsp_graph.py [/root/reference]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dsp_probe.py"), ROOT, REF],
                     capture_output=True, text=True, check=True, timeout=300)
steps = json.loads(out.stdout.strip().splitlines()[-1])
path = os.path.join(ROOT, "tests", "golden", "dsp_graph.json")
with open(path, "w") as f:
    json.dump(steps, f, indent=1, sort_keys=True)
print(path, len(steps), "steps")
