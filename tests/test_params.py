"""openwebrx_amd.params reproduces the module arguments the reference's chain code builds
(tests/golden/chain_params.json, recorded from csdr/chain/*.py with a stub pycsdr)."""
import json
import os

import numpy as np
import pytest

from openwebrx_amd import params

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "chain_params.json")


@pytest.fixture(scope="module")
def gold():
    with open(GOLDEN) as f:
        return json.load(f)


def _calls(entries, module, method=None):
    out = []
    for e in entries:
        if e["module"] != module:
            continue
        if method is None and e["op"] == "new":
            out.append(e)
        elif method is not None and e["op"] == "call" and e["method"] == method:
            out.append(e)
    return out


@pytest.mark.parametrize("key", ["fft_c1", "fft_c2", "fft_c4", "fft_nooverlap_none",
                                 "fft_secondary"])
def test_fft_parameters(gold, key):
    g = gold[key]
    sr, size, ovl, fps, comp = g["ctor"]
    avg, hop = params.fft_parameters(sr, size, fps, ovl)
    assert _calls(g["calls"], "Fft", "setEveryNSamples")[-1]["args"] == [hop]
    lap = _calls(g["calls"], "LogAveragePower")
    if avg:
        assert lap[-1]["kwargs"]["avg_number"] == avg
    else:
        assert _calls(g["calls"], "LogPower")
    for fps2, ovl2, sub in ((25, ovl, "setFps25"), (25, 0.5, "setVOverlap05")):
        avg2, hop2 = params.fft_parameters(sr, size, fps2, ovl2)
        c = _calls(g[sub], "Fft", "setEveryNSamples")
        if c:
            assert c[-1]["args"] == [hop2]
        lap = _calls(g[sub], "LogAveragePower")
        if lap and avg2:
            assert lap[-1]["kwargs"]["avg_number"] == avg2


@pytest.mark.parametrize("sr", [2400000, 10000000, 61440000])
def test_selector_parameters(gold, sr):
    g = gold["selector_%d" % sr]
    d, frac, tbw, cutoff = params.decimation(sr, 12000)
    fd = _calls(g["calls"], "FirDecimate")[0]["args"]
    assert fd[0] == d and float(fd[1]) == tbw and float(fd[2]) == cutoff
    fr = _calls(g["calls"], "FractionalDecimator")
    if frac != 1.0:
        assert float(fr[0]["args"][1]) == frac
    else:
        assert not fr
    bp = _calls(g["calls"], "Bandpass")[0]["kwargs"]
    assert float(bp["transition"]) == 320.0 / 12000
    sq = _calls(g["calls"], "Squelch")[0]["kwargs"]
    assert sq == dict(zip(["length", "decimation", "hangLength", "flushLength", "reportInterval"],
                          [params.squelch_parameters(12000)[k] for k in
                           ["length", "decimation", "hangLength", "flushLength", "reportInterval"]]))
    assert float(g["offset100k"][0]["args"][0]) == params.shift_rate(100000, sr)
    for mode, (lo, hi) in params.MODE_BANDPASS.items():
        if mode == "wfm":  # its Selector runs at 250 kHz (test_wfm_chain_params)
            continue
        if "bandpass_" + mode not in g:  # sam / rawam / rawsam: not in the recorded fixture
            continue                     # (owrx/modes.py:130-133, read as text)
        a = g["bandpass_" + mode][0]["args"]
        assert [float(v) for v in a] == [lo / 12000, hi / 12000]
    assert float(g["squelch_m150"][0]["args"][0]) == params.squelch_level(-150)
    assert float(g["squelch_m80"][0]["args"][0]) == params.squelch_level(-80)


def test_chain_params_struct(gold):
    p = params.chain_params(10000000, 100000, "nfm")
    assert p.decimation == 833 and p.frac_rate == 1.0004001600640255
    assert p.shift_rate == np.float32(-0.01)
    assert p.bandpass == 1 and p.bp_low == np.float32(-5999 / 12000)
    assert p.sq_length == 750 and p.sq_report == 4 and p.sq_level == np.float32(1e-15)
    assert p.agc_max_gain == 3.0  # NFm: agc.setMaxGain(3) (csdr/chain/analog.py:40)
    am = params.chain_params(10000000, 100000, "am")
    assert am.agc_initial_gain == 200.0  # Am: agc.setInitialGain(200) (analog.py:15)
    nfm_mods = [e["module"] for e in gold["nfm"] if e["op"] == "new"]
    assert nfm_mods == ["Agc", "FmDemod", "Limit", "NfmDeemphasis"]
    assert [e["method"] for e in gold["nfm"] if e["op"] == "call"] == ["setProfile", "setMaxGain"]


def test_resampler_params_follow_reference_math():
    """owrx/source/resampler.py:11-26: shift = (sdr_cf - cf) / sdr_rate, decimation =
    int(sdr_rate / rate), if rate = sdr_rate / decimation, transition = 0.15 * if / sdr_rate,
    FirDecimate default cutoff 0.5."""
    from openwebrx_amd import _lib
    p, if_rate = params.resampler_params(2400000, 145000000, 145300000, 48000)
    assert p.decimation == 50 and if_rate == 48000.0
    assert p.shift_rate == np.float32(-300000 / 2400000)
    assert p.transition == np.float32(0.15 * 48000 / 2400000)
    assert p.cutoff == 0.5 and p.frac_rate == 1.0 and p.output == _lib.OUT_IQ
    p, if_rate = params.resampler_params(10000000, 14100000, 14074000, 300000)
    assert p.decimation == 33 and abs(if_rate - 10e6 / 33) < 1e-9


@pytest.mark.parametrize("sr", [2400000, 10000000, 61440000])
def test_wfm_chain_params(gold, sr):
    """WFM: Selector(sr, 250000) with the mode's bandpass and squelch (recorded from
    csdr/chain/selector.py) and WFm(48000, 50e-6) (csdr/chain/analog.py:55-116)."""
    from openwebrx_amd import _lib
    g = gold["selector_wfm_%d" % sr]
    offset = -600000 if sr > 2400000 else 300000
    p = params.chain_params(sr, offset, "wfm")
    fd = _calls(g["calls"], "FirDecimate")[0]["args"]
    assert fd[0] == p.decimation and np.float32(float(fd[1])) == p.transition
    assert np.float32(float(fd[2])) == p.cutoff
    fr = _calls(g["calls"], "FractionalDecimator")
    assert (float(fr[0]["args"][1]) if fr else 1.0) == p.frac_rate
    bp = _calls(g["calls"], "Bandpass")[0]["kwargs"]
    assert np.float32(float(bp["transition"])) == p.bp_transition
    lo, hi = (float(v) for v in g["bandpass_wfm"][0]["args"])
    assert (np.float32(lo), np.float32(hi)) == (p.bp_low, p.bp_high)
    sq = _calls(g["calls"], "Squelch")[0]["kwargs"]
    assert (sq["length"], sq["hangLength"], sq["flushLength"], sq["reportInterval"]) == \
        (p.sq_length, p.sq_hang, p.sq_flush, p.sq_report)
    assert np.float32(float(g["offset"][0]["args"][0])) == p.shift_rate
    assert p.demod == _lib.DEMOD_WFM and p.if_rate == 250000.0 and p.audio_rate == 48000
    wfm = {e["module"]: e for e in gold["wfm"] if e["op"] == "new"}
    assert float(wfm["FractionalDecimator"]["args"][1]) == p.if_rate / p.audio_rate
    assert wfm["FractionalDecimator"]["kwargs"] == {"prefilter": True}
    assert wfm["WfmDeemphasis"]["args"][0] == p.audio_rate
    assert np.float32(float(wfm["WfmDeemphasis"]["args"][1])) == p.deemph_tau
    assert [e["module"] for e in gold["clientaudio_hd_adpcm"]] == ["Convert", "AdpcmEncoder"]
