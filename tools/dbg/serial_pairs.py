"""usage: serial_pairs.py [pairs] [chains] [modes, comma-separated]

Per-pair serial-stage time and per-chain audio bytes at C3 (diagnostic): the rocprof trace of
the C3 bench shows post_serial_front and chain_adpcm ~30 % slower on the same engine blocks
(about every third pair); this runs the bench's C3 chains (no waterfall) pair by pair, synced,
with the engine's HIP-event timing on, and prints each pair's serial GPU time next to the spread
of the chains' audio bytes per mode."""
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from bench import gen_stream_torch  # noqa: E402
from openwebrx_amd import Engine, params  # noqa: E402
from openwebrx_amd.synth import carrier_offsets  # noqa: E402

fs, block = 10000000, 1 << 20
pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 16
C = int(sys.argv[2]) if len(sys.argv) > 2 else 256
mset = tuple(sys.argv[3].split(",")) if len(sys.argv) > 3 else ("nfm", "usb", "cw")
modes = [mset[c % len(mset)] for c in range(C)]
offs = carrier_offsets(fs, C)
plist = [params.chain_params(fs, o, m) for o, m in zip(offs, modes)]
dev = torch.device("cuda", 0)
eng = Engine(fs, max_block=block)
eng.set_input_retention(8)
eng.set_block_pairing(True)
eng.set_timing(True, 1)
chains = [eng.chain(p) for p in plist]
hist = eng.history
stream = gen_stream_torch(torch, dev, fs, hist + 2 * pairs * block, modes, offs)
base = stream.data_ptr() + 8 * hist
torch.cuda.synchronize()
mi = {m: np.array([i for i, x in enumerate(modes) if x == m]) for m in mset}
last = eng.stats()
for p in range(pairs):
    for j in (2 * p, 2 * p + 1):
        eng.process_device(base + 8 * j * block, block)
    eng.sync()
    s = eng.stats()
    audio, alens, _, _ = eng.read_chains(chains)
    d = {k: s[k] - last[k] for k in ("gpu_ms_serial", "gpu_ms_post", "gpu_ms_ddc", "blocks")}
    last = s
    per = " ".join("%s %d..%d" % (m, alens[ix].min(), alens[ix].max()) for m, ix in mi.items())
    print("pair %2d  blocks %d  serial %.3f ms  post %.3f  ddc %.3f  | bytes %s"
          % (p, d["blocks"], d["gpu_ms_serial"], d["gpu_ms_post"], d["gpu_ms_ddc"], per), flush=True)
eng.close()
