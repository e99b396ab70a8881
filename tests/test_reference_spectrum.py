"""The reference's own SpectrumThread (owrx/fft.py:13-109) over the pycsdr shim (SURVEY §4 step 3,
round-2 verdict item 3): its FftChain fuses into one engine waterfall with the golden-pinned
FftChain parameters at every step -- start, `_setCompression("none")` (FftAdpcm swapped out, the
format-change ValueError caught, a fresh Buffer and pump thread wired, :61-73), `restart` on
fft_size (:50, :89-91), compression back to adpcm, fps changed on the fly -- and `stop` leaves no
live head or client.  The probe needs the reference checkout (this container) and runs in a
subprocess; the fixture checks need only tests/golden/spectrum_graph.json."""
import json
import os
import subprocess
import sys

import pytest

from openwebrx_amd import params

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "spectrum_graph.json")
HAVE_REF = os.path.isfile(os.path.join(REF, "owrx", "fft.py"))


def _fixture():
    with open(GOLDEN) as f:
        return {s["step"]: s for s in json.load(f)}


@pytest.mark.skipif(not HAVE_REF, reason="reference checkout absent")
def test_probe_equals_fixture():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "spectrum_probe.py"), ROOT, REF],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    got = {s["step"]: s for s in json.loads(r.stdout.strip().splitlines()[-1])}
    assert json.loads(json.dumps(got, sort_keys=True)) == _fixture()


@pytest.mark.parametrize("step,n,fps,adpcm", [("start_adpcm", 16384, 9, True),
                                              ("compression_none", 16384, 9, False),
                                              ("fft_size_8192", 8192, 9, False),
                                              ("compression_adpcm_again", 8192, 9, True),
                                              ("fps_20", 8192, 20, True)])
def test_every_step_is_one_fused_waterfall(step, n, fps, adpcm):
    s = _fixture()[step]
    assert s["fused"] and s["kind"] == "waterfall" and s["live_heads"] == 1 and s["clients"] == 1
    avg, hop = params.fft_parameters(10000000, n, fps, 0.3)
    assert s["params"] == dict(fft_size=n, hop=hop, avg=avg, add_db=-70.0, adpcm=adpcm)
    cls = [g["class"] for g in s["graph"]]
    assert cls == ["Fft", "LogAveragePower", "FftSwap"] + (["FftAdpcm"] if adpcm else [])
    # the writer SpectrumThread's pump reads has the chain's output format (CHAR rows / FLOAT)
    assert s["writer_format"] == ("CHAR" if adpcm else "FLOAT") == s["dsp_output_format"]
    assert s["pump_threads"] == 1  # the swapped-out pump ended with its reader


def test_stop_leaves_nothing_running():
    s = _fixture()["stopped"]
    assert s["clients"] == 0 and s["live_heads"] == 0
