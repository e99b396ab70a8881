"""Device memory before / after an engine that runs out of memory while creating chains
(diagnostic): is everything it allocated returned at close()?"""
import sys
import time

import torch

sys.path.insert(0, ".")
from openwebrx_amd import Engine, params  # noqa: E402
from openwebrx_amd.synth import carrier_offsets  # noqa: E402

fs = 10000000
free0, total = torch.cuda.mem_get_info()
print("free %.1f GB of %.1f" % (free0 / 1e9, total / 1e9), flush=True)
for C in (32768, 200000):
    plist = [params.chain_params(fs, o, ("nfm", "usb", "cw")[c % 3])
             for c, o in enumerate(carrier_offsets(fs, C))]
    eng = Engine(fs, max_block=1 << 20, history=22_000_000)
    n, t0 = 0, time.time()
    try:
        for p in plist:
            eng.chain(p)
            n += 1
            if n % 16384 == 0:
                print("  %d chains, free %.1f GB" % (n, torch.cuda.mem_get_info()[0] / 1e9), flush=True)
    except Exception as exc:
        print("  stopped at %d chains: %s" % (n, str(exc)[:120]), flush=True)
    free1 = torch.cuda.mem_get_info()[0]
    eng.close()
    free2 = torch.cuda.mem_get_info()[0]
    print("C=%d: %d created in %.1f s; free %.1f GB with them, %.1f GB after close (before: %.1f)"
          % (C, n, time.time() - t0, free1 / 1e9, free2 / 1e9, free0 / 1e9), flush=True)
