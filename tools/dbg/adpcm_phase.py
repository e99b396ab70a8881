"""Diagnostic: chain_adpcm's cost when the chains' sync-frame phases differ (chains created at
different blocks, as clients join a live server) vs all chains created together (the bench).
usage: python3 tools/dbg/adpcm_phase.py together|spread   (run under rocprofv3 --kernel-trace --stats)"""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from openwebrx_amd import Engine, params  # noqa: E402

mode = sys.argv[1]
fs, block, C = 10_000_000, 1 << 20, 256
modes = [("nfm", "usb", "cw")[i % 3] for i in range(C)]
from openwebrx_amd.synth import carrier_offsets  # noqa: E402
offs = carrier_offsets(fs, C)
dev = torch.device("cuda:0")
nblk = 48
stream = bench.gen_stream_torch(torch, dev, fs, (nblk + 1) * block, modes, offs)
eng = Engine(fs, max_block=block)
plist = [params.chain_params(fs, o, m) for o, m in zip(offs, modes)]
chains = []
pos = 0
if mode == "together":
    chains = [eng.chain(p) for p in plist]
else:  # 8 batches of 32 chains, 1..3 blocks apart: their byte counters (and frame phases) differ
    for b in range(8):
        chains += [eng.chain(p) for p in plist[32 * b:32 * (b + 1)]]
        for _ in range(1 + b % 3):
            eng.process_device(stream.data_ptr() + 8 * pos * block, block)
            pos += 1
eng.sync()
eng.read_chains(chains)
torch.cuda.synchronize()
for i in range(pos, nblk):
    eng.process_device(stream.data_ptr() + 8 * i * block, block)
    eng.read_chains(chains)
eng.sync()
a, lens, _, _ = eng.read_chains(chains)
print(mode, "blocks", nblk - pos, "audio bytes", int(lens.sum()))
eng.close()
