"""Waterfall rows of the kernel OWRX_WF_KERNEL selects (run as a subprocess by
tests/test_gpu_parity.py::test_waterfall_kernel_variants: the selection is read once per
process).  For each FFT size it covers (1024 .. 16384; 32768 and 65536 for "fourstep") prints
the worst |dB| difference to the oracle's double-precision rows, one JSON object."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
import openwebrx_amd as amd  # noqa: E402
from openwebrx_amd import synth  # noqa: E402

out = {}
sizes = [(1024, 250000), (2048, 1000000), (4096, 2400000), (8192, 4800000), (16384, 10000000)]
if os.environ.get("OWRX_WF_KERNEL") == "fourstep":
    sizes = [(32768, 20000000), (65536, 61440000)]
for N, fs in sizes:
    avg, hop = amd.params.fft_parameters(fs, N, 9, 0.3)
    avg = min(avg, 4)
    n = hop * avg * 3 + N + 1000
    iq, _ = synth.make_iq(fs, n, ["nfm", "am", "usb"])
    eng = amd.Engine(fs, max_block=1 << 17)
    wf = eng.waterfall(N, hop, avg, adpcm=False)
    for i in range(0, iq.size, 1 << 17):
        eng.push(iq[i:i + (1 << 17)])
    eng.sync()
    g = wf.read_rows()
    eng.close()
    ref = np.stack([oracle.fftswap(r) for r in oracle.waterfall_rows(iq, N, hop, avg)])
    out[N] = float(np.max(np.abs(g - ref))) if g.shape == ref.shape else None
print(json.dumps(out))
