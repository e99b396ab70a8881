"""Device memory per chain for the capacity ladder's engine shape (diagnostic): a C3 engine with
the batched waterfall's history, chains added until `C` or out of memory, free memory printed
every 16 384 chains."""
import sys
import time

import torch

sys.path.insert(0, ".")
from openwebrx_amd import Engine, params  # noqa: E402
from openwebrx_amd.synth import carrier_offsets  # noqa: E402

fs, N = 10000000, 16384
avg, hop = params.fft_parameters(fs, N, 9, 0.3)
batch = int(sys.argv[1]) if len(sys.argv) > 1 else 3424
C = int(sys.argv[2]) if len(sys.argv) > 2 else 163840
hist = (batch + 16) * hop + 2 * N + (1 << 20)
free0, total = torch.cuda.mem_get_info()
print("free %.1f GB of %.1f; history %d samples" % (free0 / 1e9, total / 1e9, hist), flush=True)
plist = [params.chain_params(fs, o, ("nfm", "usb", "cw")[c % 3])
         for c, o in enumerate(carrier_offsets(fs, C))]
eng = Engine(fs, max_block=1 << 20, history=hist)
wf = eng.waterfall(N, hop, avg, adpcm=True)
wf.set_batch(batch)
print("engine + waterfall: free %.1f GB" % (torch.cuda.mem_get_info()[0] / 1e9), flush=True)
n, t0, last = 0, time.time(), torch.cuda.mem_get_info()[0]
try:
    for p in plist:
        eng.chain(p)
        n += 1
        if n % 16384 == 0:
            f = torch.cuda.mem_get_info()[0]
            print("  %d chains, free %.1f GB (%.0f KB per chain over the last 16384)"
                  % (n, f / 1e9, (last - f) / 16384 / 1e3), flush=True)
            last = f
except Exception as exc:
    print("  stopped at %d chains: %s" % (n, str(exc)[:160]), flush=True)
print("%d created in %.1f s (%.1f us per chain)" % (n, time.time() - t0, 1e6 * (time.time() - t0) / max(1, n)), flush=True)
eng.close()
