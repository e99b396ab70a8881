"""Waterfall FFT in isolation (diagnostic): one engine per FFT size at 10 Msps with only an
FftChain (C3's fps 9, overlap 0.3), 2^22-sample device blocks pushed back to back.  Run under
rocprofv3 --kernel-trace and read the wf_fft_* averages (tools/prof_db_stats.py)."""
import sys
import time

import os

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from openwebrx_amd import params  # noqa: E402
from openwebrx_amd.engine import Engine  # noqa: E402

fs, blk = 10000000, 1 << 22
sizes = [int(s) for s in sys.argv[1:]] or [8192, 16384]
# a contiguous recording of 4 blocks: owrx_process_device reads the stream history before the
# pointer it is handed (include/owrx_amd.h), so blocks start at offsets >= 1 block
x = (torch.randn(4 * blk, dtype=torch.complex64, device="cuda") * 0.1).contiguous()


def ptr(i):
    return x.data_ptr() + 8 * blk * (1 + i % 3)


for n in sizes:
    avg, hop = params.fft_parameters(fs, n, 9, 0.3)
    eng = Engine(fs, max_block=blk)
    wf = eng.waterfall(n, hop, avg, adpcm=False)
    for i in range(3):
        eng.process_device(ptr(i), blk)
    eng.sync()
    wf.read_rows()
    t0 = time.time()
    for i in range(30):
        eng.process_device(ptr(i), blk)
        if i % 8 == 7:
            eng.sync()
            wf.read_rows()
    eng.sync()
    dt = (time.time() - t0) / 30
    print("N=%d hop=%d avg=%d frames/block=%.1f wall %.1f us/block" % (n, hop, avg, blk / hop, dt * 1e6),
          flush=True)
    wf.close()
    eng.close()
