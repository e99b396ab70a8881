"""Bisect a host crash of the 256-chain SAm/RawAm engine test (diagnostic; one case per run)."""
import faulthandler
import os
import sys

if not os.environ.get("OWRX_SEGV_TRACE"):
    faulthandler.enable()
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import openwebrx_amd as amd  # noqa: E402
from openwebrx_amd import synth  # noqa: E402

case = sys.argv[1]
C = int(sys.argv[2])
debug = sys.argv[3] == "1"
fs = 2400000
kinds = {"sam": ("sam",), "rawam": ("rawam",), "rawsam": ("rawsam",), "mixed": ("sam", "rawam", "rawsam"),
         "am": ("am",), "amnfm": ("am", "nfm")}[case]
modes = [kinds[c % len(kinds)] for c in range(C)]
offs = synth.carrier_offsets(fs, C)
iq, _ = synth.make_iq(fs, 1 << 19, ["am"] * 8)
plist = [amd.params.chain_params(fs, o, m, output=amd._lib.OUT_S16) for o, m in zip(offs, modes)]
eng = amd.Engine(fs, max_block=1 << 17)
if debug:
    eng.set_debug(True)
chains = [eng.chain(p) for p in plist]
print("created", flush=True)
for i in range(0, iq.size, 1 << 17):
    eng.push(iq[i:i + (1 << 17)])
    print("pushed", i, flush=True)
eng.sync()
print("ok", case, C, debug, len(chains[0].read_audio()), flush=True)
