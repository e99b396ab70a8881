"""Chain audio of a stream whose chain count crosses OWRX_WIDE_SERIAL_CHAINS both ways (run as a
subprocess by tests/test_gpu_parity.py::test_wide_serial_streams_same_audio: the threshold is
read once per process).  Prints one JSON object: per chain handle the SHA-256 of its audio and
s-meter bytes."""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import openwebrx_amd as amd  # noqa: E402
from openwebrx_amd import synth  # noqa: E402

fs, block = 2400000, 1 << 17
modes = ["nfm", "am", "usb", "cw", "lsb", "nfm", "am", "usb"]
iq, offs = synth.make_iq(fs, 24 * block, modes)
eng = amd.Engine(fs, max_block=block)
outs = {}
chains = {}


def add(i):
    out = amd._lib.OUT_ADPCM if i % 2 else amd._lib.OUT_S16
    chains[i] = eng.chain(amd.params.chain_params(fs, offs[i], modes[i], output=out))
    outs[i] = [b"", b""]


def drain():
    for i, ch in chains.items():
        outs[i][0] += ch.read_audio()
        outs[i][1] += ch.read_smeter().tobytes()


for i in range(3):
    add(i)
for b in range(24):
    if b == 6:
        for i in range(3, 8):  # 8 chains: above a threshold of 4
            add(i)
    if b == 16:  # back to 3
        # the leaving chains' audio of the blocks still in flight is delivered before they close
        # (owrx_chain_destroy discards what a closed chain has not read), so their byte counts do
        # not depend on how far the pipeline got by the time of the drain
        eng.sync()
        drain()
        for i in range(3, 8):
            chains.pop(i).close()
    eng.push(iq[b * block:(b + 1) * block])
    if b % 4 == 3:
        drain()
eng.sync()
drain()
eng.close()
print(json.dumps({i: [hashlib.sha256(a).hexdigest(), hashlib.sha256(s).hexdigest(), len(a)]
                  for i, (a, s) in outs.items()}))
