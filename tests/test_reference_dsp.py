"""The reference's own ClientDemodulatorChain (owrx/dsp.py:39-225) over the pycsdr shim: every
step of a demodulator / secondary demodulator / secondary FFT / NoiseFilter sequence stays fused,
with the golden-pinned engine parameters, and publishes the Selector / audio taps its secondary
readers need (tests/dsp_probe.py).  The recorded graphs are the fixture the GPU replay uses.

The probe needs the reference checkout (this container) and runs in a subprocess; the replay
checks need only the fixture."""
import json
import os
import subprocess
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import dsp_replay  # noqa: E402

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HAVE_REF = os.path.isfile(os.path.join(REF, "owrx", "dsp.py"))

MODES = {"nfm": ("nfm", -200000), "am": ("am", -200000), "usb": ("usb", -200000),
         "wfm": ("wfm", -200000), "nfm_again": ("nfm", -200000),
         "nfm_secondary_selector": ("nfm", -200000), "nfm_secondary_fft_4096": ("nfm", -200000),
         "nfm_nr": ("nfm", -200000), "nfm_audio_secondary": ("nfm", -200000),
         "nfm_plain": ("nfm", -200000)}


@pytest.fixture(scope="module")
def probed():
    if not HAVE_REF:
        pytest.skip("reference checkout absent")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "dsp_probe.py"), ROOT, REF],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return {s["step"]: s for s in json.loads(r.stdout.strip().splitlines()[-1])}


def test_fixture_is_what_the_reference_builds(probed):
    golden = dsp_replay.steps()
    assert set(probed) == set(golden)
    for k in golden:
        assert json.loads(json.dumps(probed[k], sort_keys=True)) == \
            json.loads(json.dumps(golden[k], sort_keys=True)), k


@pytest.mark.parametrize("step", sorted(MODES))
def test_every_step_stays_fused_with_golden_params(step):
    from openwebrx_amd import _lib, params
    s = dsp_replay.steps()[step]
    assert s["fused"] and s["kind"] == "chain", step
    mode, off = MODES[step]
    nr = step in ("nfm_nr", "nfm_audio_secondary")
    want = params.chain_params(10000000, off, mode, output=_lib.OUT_ADPCM, nr_enabled=nr,
                               nr_threshold=5 if nr else 0)
    got = s["params"]
    for name, _ in _lib.ChainParams._fields_:
        if mode == "wfm" and name in ("agc_profile", "agc_initial_gain", "agc_max_gain"):
            continue
        g = got.get(name, 0.0 if name in ("if_rate", "deemph_tau") else None)
        if name == "sq_level":  # ClientDemodulatorChain's default squelch: -150 dB
            assert g == pytest.approx(1e-15, rel=1e-6)
            continue
        assert g == pytest.approx(getattr(want, name), rel=1e-6, abs=1e-12), (step, name)


def test_taps_and_secondary_fft_follow_the_secondary_readers():
    s = dsp_replay.steps()
    assert not s["nfm_again"]["tap_selector"] and not s["nfm_again"]["tap_audio"]
    # a SecondarySelector on selectorBuffer (owrx/dsp.py:188-202) + its secondary FFT
    assert s["nfm_secondary_selector"]["tap_selector"]
    assert s["nfm_secondary_selector"]["params"]["secondary_fft"]["fft_size"] == 2048
    assert s["nfm_secondary_fft_4096"]["params"]["secondary_fft"]["fft_size"] == 4096
    # a FLOAT secondary demodulator on audioBuffer (:205-206)
    assert s["nfm_audio_secondary"]["tap_audio"]
    assert s["nfm_nr"]["params"]["nr_enabled"] == 1


@pytest.mark.parametrize("step,output", [("service_iq", 4), ("service_audio", 2)])
def test_service_demodulator_chains_fuse(step, output):
    """ServiceDemodulatorChain (owrx/service/chain.py:7-23): Selector(withSquelch=False) at the
    service's 250 kHz IF into an IQ decoder (OWRX_OUT_SEL: the engine emits the Selector output)
    or through Ssb into an audio decoder (OWRX_OUT_F32); the Selector design is the reference's
    (decimation / FractionalDecimator / bandpass of csdr/chain/selector.py for 250 kHz -> 12 kHz)
    and no squelch gate (level 0)."""
    from openwebrx_amd import params
    s = dsp_replay.steps()[step]
    assert s["fused"] and s["kind"] == "chain"
    p = s["params"]
    d, frac, tbw, cutoff = params.decimation(250000, 12000)
    assert (p["output"], p["decimation"], p["demod"]) == (output, d, 2)
    assert p["frac_rate"] == pytest.approx(frac) and p["transition"] == pytest.approx(tbw)
    assert (p["bandpass"], p["bp_low"], p["bp_high"]) == (1, 0.0, pytest.approx(3000 / 12000))
    assert p["sq_level"] == 0.0 and not s["tap_selector"] and not s["tap_audio"]


def test_sam_fuses_whole():
    """SAm (csdr/chain/analog.py:141-154: Afc -> RealPart -> DcBlock -> Agc) set on the
    reference's ClientDemodulatorChain fuses whole into one engine chain: OWRX_DEMOD_SAM with
    Afc(10, 4) and Agc(Slow, initial gain 200), ADPCM audio (Afc runs in chain_afc, lane per
    chain, ahead of the serial front)."""
    s = dsp_replay.steps()["sam"]
    assert s["fused"] and s["kind"] == "chain" and s["params"]["output"] == 1
    p = s["params"]
    assert (p["demod"], p["afc_update"], p["afc_sample"], p["audio_gain"]) == (4, 10, 4, 0.0)
    assert (p["agc_profile"], p["agc_initial_gain"]) == (1, 200.0)
    cls = [d["class"] for _, d, _ in s["graph"]]
    assert cls.index("Squelch") < cls.index("Afc") < cls.index("RealPart") < cls.index("Agc")
    afc = [d for _, d, _ in s["graph"] if d["class"] == "Afc"][0]
    assert (afc["update_period"], afc["sample_period"]) == (10, 4)


def test_rawsam_runs_the_selector_at_the_hd_rate():
    """RawSAm (csdr/chain/analog.py:156-167) is HdAudio: ClientDemodulatorChain runs its
    Selector at the hd output rate (48 kHz, owrx/dsp.py:150-166); fused whole: Afc(50, 8) ->
    RealPart -> DcBlock -> Gain(100) (audio_gain in the Agc's place)."""
    s = dsp_replay.steps()["rawsam"]
    assert s["fused"] and s["params"]["output"] == 1 and s["params"]["decimation"] == 208
    p = s["params"]
    assert (p["demod"], p["afc_update"], p["afc_sample"], p["audio_gain"]) == (4, 50, 8, 100.0)
    cls = [d["class"] for _, d, _ in s["graph"]]
    assert cls.index("Squelch") < cls.index("Afc") < cls.index("RealPart") < cls.index("Gain")
    g = {d["class"]: d for _, d, _ in s["graph"]}
    assert (g["Afc"]["update_period"], g["Afc"]["sample_period"]) == (50, 8)
    assert g["Gain"]["gain"] == 100.0


def test_rawam_and_ssbdigital_plan():
    """RawAm (csdr/chain/analog.py:23-31: AmDemod -> DcBlock -> Gain(100), no Agc) fuses whole
    (OWRX_DEMOD_AM with audio_gain 100); SsbDigital (FixedAudioRateChain + HdAudio, :169-181)
    fuses whole as RealPart + Agc(Slow) with the Selector at its fixed 48 kHz rate (D = 208)."""
    s = dsp_replay.steps()["rawam"]
    assert s["fused"] and s["params"]["output"] == 1 and s["params"]["decimation"] == 208
    assert (s["params"]["demod"], s["params"]["audio_gain"]) == (1, 100.0)
    cls = [d["class"] for _, d, _ in s["graph"]]
    assert cls.index("Squelch") < cls.index("AmDemod") < cls.index("DcBlock") < cls.index("Gain")
    s = dsp_replay.steps()["ssbdigital"]
    assert s["fused"] and s["kind"] == "chain"
    assert s["params"]["demod"] == 2 and s["params"]["decimation"] == 208
    assert s["params"]["agc_profile"] == 1 and s["params"]["output"] == 1  # SLOW, ADPCM


@pytest.mark.parametrize("step", sorted(MODES) + ["service_iq", "service_audio", "sam", "rawsam",
                                  "rawam", "ssbdigital"])
def test_replayed_graph_plans_like_the_reference(step):
    """The shim-built replay of each recorded graph is planned exactly as the reference's."""
    from openwebrx_amd.pycsdr import _graph
    s = dsp_replay.steps()[step]
    wide, mods, outs, power = dsp_replay.build(s)
    seg = _graph.plan_segment(mods[0])
    assert seg is not None
    kind, p, used = seg
    assert kind == s["kind"] and len(used) == s["n_modules"]
    got = {k: v for k, v in p.items() if k not in ("power_writer", "secondary_modules",
                                                   "secondary_writer", "tap_selector",
                                                   "tap_audio")}
    assert json.loads(json.dumps(got)) == s["params"]
    assert (p["tap_selector"] is not None) == s["tap_selector"]
    assert (p["tap_audio"] is not None) == s["tap_audio"]
    _graph.finish(wide)
