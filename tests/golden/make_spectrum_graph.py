#!/usr/bin/env python3
"""Records tests/golden/spectrum_graph.json: the reference's own SpectrumThread (owrx/fft.py)
driven over the pycsdr shim through start / compression "none" / fft_size 8192 (restart) /
compression "adpcm" / fps 20 / stop (tests/spectrum_probe.py) -- the planner's result and the
FftChain modules at each step.  Needs the reference checkout (this container).

usage: python tests/golden/make_spectrum_graph.py [/root/reference]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
out = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "spectrum_probe.py"), ROOT, REF],
                     capture_output=True, text=True, check=True, timeout=300)
steps = json.loads(out.stdout.strip().splitlines()[-1])
path = os.path.join(ROOT, "tests", "golden", "spectrum_graph.json")
with open(path, "w") as f:
    json.dump(steps, f, indent=1, sort_keys=True)
print(path, len(steps), "steps")
