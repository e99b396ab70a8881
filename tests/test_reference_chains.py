"""Drop-in check with the reference's own chain code: csdr/chain/{selector,analog,clientaudio,
fft}.py, imported over the pycsdr shim, build module graphs that the planner fuses with exactly
the engine parameters of openwebrx_amd.params (the golden-pinned restatement).

CPU only (no engine is created: nothing is written to the wideband buffer).  It runs where the
reference checkout is present (this container; the GPU box has none and skips it), in a
subprocess so the reference's modules never leak into the other tests' sys.modules.
"""
import json
import os
import subprocess
import sys

import pytest

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "csdr", "chain")),
                                reason="reference checkout absent")

PROBE = r'''
import json, sys
sys.path.insert(0, ROOT)
import openwebrx_amd.pycsdr as shim
shim.install()                      # sys.modules["pycsdr"] (INTEGRATION.md section 1)
sys.path.append(REF)
from csdr.chain import Chain
from csdr.chain.selector import Selector
from csdr.chain.analog import NFm, Am, Ssb, WFm
from csdr.chain.clientaudio import ClientAudioChain
from csdr.chain.fft import FftChain
from pycsdr.modules import Buffer
from pycsdr.types import Format, AgcProfile
from openwebrx_amd.pycsdr import _graph

out = {}
fs = 10000000
cases = [("nfm", -200000, (-5999, 5999), 12000, lambda: NFm(12000), False),
         ("am", 310000, (-4700, 4700), 12000, lambda: Am(), False),
         ("usb", -1234567, (150, 3000), 12000, lambda: Ssb(AgcProfile("Fast")), True),
         ("wfm", 2500000, (-124000, 124000), 250000, lambda: WFm(48000, 50e-6, False), False)]
for mode, off, (lo, hi), rate, demod, nr in cases:
    wide = Buffer(Format.COMPLEX_FLOAT)
    sel = Selector(fs, rate)
    dem = demod()
    audio_rate = 48000 if mode == "wfm" else 12000
    cac = ClientAudioChain(dem.getOutputFormat(), audio_rate, audio_rate, "adpcm", nr, 10)
    chain = Chain([sel, dem, cac])            # ClientDemodulatorChain's composition (owrx/dsp.py:72)
    chain.setReader(wide.getReader())
    chain.setWriter(Buffer(Format.CHAR))
    sel.setFrequencyOffset(off)
    sel.setBandpass(lo, hi)
    kind, p, used = _graph.plan_segment(sel.workers[0])
    out[mode] = {"kind": kind, "n_modules": len(used),
                 "params": {k: v for k, v in p.items()
                            if k not in ("power_writer", "secondary_modules", "secondary_writer")}}
    _graph.finish(wide)

wide = Buffer(Format.COMPLEX_FLOAT)
fc = FftChain(fs, 16384, 0.3, 9, "adpcm")
fc.setReader(wide.getReader())
fc.setWriter(Buffer(Format.CHAR))
kind, p, used = _graph.plan_segment(fc.workers[0])
out["fft"] = {"kind": kind, "params": p}
_graph.finish(wide)
print(json.dumps(out))
'''


@pytest.fixture(scope="module")
def planned():
    code = "ROOT = %r\nREF = %r\n" % (ROOT, REF) + PROBE
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("mode,off,nr", [("nfm", -200000, False), ("am", 310000, False),
                                         ("usb", -1234567, True), ("wfm", 2500000, False)])
def test_reference_client_chain_fuses(planned, mode, off, nr):
    from openwebrx_amd import _lib, params
    got = planned[mode]
    assert got["kind"] == "chain"
    want = params.chain_params(10000000, off, mode, output=_lib.OUT_ADPCM, nr_enabled=nr,
                               nr_threshold=10 if nr else 0)
    for name, _ in _lib.ChainParams._fields_:
        if mode == "wfm" and name in ("agc_profile", "agc_initial_gain", "agc_max_gain"):
            continue  # WFm has no Agc
        g = got["params"].get(name, 0.0 if name in ("if_rate", "deemph_tau") else None)
        assert g is not None, name
        assert g == pytest.approx(getattr(want, name), rel=1e-6, abs=1e-12), (mode, name)


def test_reference_fft_chain_fuses(planned):
    from openwebrx_amd import params
    avg, hop = params.fft_parameters(10000000, 16384, 9, 0.3)
    assert planned["fft"] == {"kind": "waterfall",
                              "params": dict(fft_size=16384, hop=hop, avg=avg, add_db=-70.0,
                                             adpcm=True)}
