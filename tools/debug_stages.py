"""Stage-by-stage comparison of engine debug taps against the oracle (GPU diagnostic)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
import openwebrx_amd as amd  # noqa: E402
from openwebrx_amd import synth  # noqa: E402


def rel(a, b):
    m = min(a.size, b.size)
    if m == 0:
        return float("nan")
    a, b = a[:m], b[:m]
    return float(np.sqrt(np.mean(np.abs(a - b) ** 2) / max(np.mean(np.abs(b) ** 2), 1e-30)))


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "am"
    nch = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    fs = 2400000
    modes = ([mode, "nfm", mode, "am", mode] * 4)[:nch]
    n = 1 << 20
    iq, offs = synth.make_iq(fs, n, modes)
    plist = [amd.params.chain_params(fs, o, m, output=amd._lib.OUT_S16) for o, m in zip(offs, modes)]
    eng = amd.Engine(fs, max_block=1 << 18)
    eng.set_debug(True)
    chains = [eng.chain(p) for p in plist]
    i = 0
    while i < iq.size:
        eng.push(iq[i:i + (1 << 18)])
        i += 1 << 18
    eng.sync()
    keys = [(0, "ddc"), (1, "frac"), (2, "bandpass"), (3, "squelch"), (4, "demod"), (5, "agc")]
    for ci, (p, ch) in enumerate(zip(plist, chains)):
        ref = oracle.stages(iq, p)
        line = ["chain %d %s" % (ci, modes[ci])]
        for st, k in keys:
            g = ch.read_debug(st)
            line.append("%s n=%d/%d r=%.2e" % (k, g.size, ref[k].size, rel(g, ref[k])))
        s16 = np.frombuffer(ch.read_audio(), np.int16)
        m = min(s16.size, ref["s16"].size)
        d = np.abs(s16[:m].astype(np.int32) - ref["s16"][:m])
        line.append("s16 n=%d/%d ok=%.4f" % (s16.size, ref["s16"].size, np.mean(d <= 1) if m else -1))
        print(" | ".join(line), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
