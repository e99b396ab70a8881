"""Chain parameter math, restated from the reference's chain code so the engine receives the
exact module arguments the reference would construct (pinned by tests/golden/chain_params.json):

* FftChain._updateParameters / _setBlockSize -- csdr/chain/fft.py:51-55, 75-85
* Decimator._getDecimation, transition, cutoff -- csdr/chain/selector.py:11-51
* Selector._buildBandpass / setBandpass / _buildSquelch / _updateShift / _convertToLinear
  -- csdr/chain/selector.py:115-147, 159-166
* NFm / Am / Ssb / ClientAudioChain module choices -- csdr/chain/analog.py, clientaudio.py
* mode bandpass table -- owrx/modes.py:124-129
* service Resampler (Shift + FirDecimate to a band) -- owrx/source/resampler.py:11-26
"""
import math

import numpy as np

from . import _lib

MODE_BANDPASS = {  # owrx/modes.py:124-129
    "nfm": (-5999, 5999),
    "am": (-4700, 4700),
    "lsb": (-3000, -150),
    "usb": (150, 3000),
    "cw": (700, 900),
    "wfm": (-124000, 124000),  # owrx/modes.py:125
    "sam": (-4700, 4700),      # owrx/modes.py:130
    "rawam": (-10000, 10000),  # owrx/modes.py:132
    "rawsam": (-10000, 10000),  # owrx/modes.py:133
}
MODE_DEMOD = {"nfm": _lib.DEMOD_NFM, "am": _lib.DEMOD_AM, "usb": _lib.DEMOD_SSB,
              "lsb": _lib.DEMOD_SSB, "cw": _lib.DEMOD_SSB, "wfm": _lib.DEMOD_WFM,
              "sam": _lib.DEMOD_SAM, "rawam": _lib.DEMOD_AM, "rawsam": _lib.DEMOD_SAM}
# HdAudio demodulators: the Selector runs at the hd output rate (owrx/dsp.py:150-166)
HD_MODES = ("rawam", "rawsam")
# SAm: Afc(10, 4), Agc(Slow, initial gain 200); RawSAm: Afc(50, 8), Gain(100); RawAm: Gain(100)
# (csdr/chain/analog.py:23-31, 141-167)
MODE_AFC = {"sam": (10, 4), "rawsam": (50, 8)}
MODE_GAIN = {"rawam": 100.0, "rawsam": 100.0}
WFM_IF_RATE = 250000  # WFm.getFixedIfSampleRate (csdr/chain/analog.py:81-82)


def f32(x):
    """pycsdr receives float arguments as C float."""
    return float(np.float32(x))


def fft_parameters(samp_rate, fft_size, fps, voverlap):
    """(avg_number, every_n_samples) exactly as FftChain._updateParameters computes them."""
    avg = 0
    if voverlap > 0:
        avg = int(round(1.0 * samp_rate / fft_size / fps / (1.0 - voverlap)))
    if avg == 0:
        block = samp_rate / fps
    else:
        block = samp_rate / fps / avg
    return avg, int(block)


def decimation(input_rate, output_rate):
    """Decimator._getDecimation + transition/cutoff (selector.py:22-27, 40-51)."""
    if output_rate > input_rate:
        output_rate = input_rate
    d = input_rate / output_rate
    d_int = int(d)
    frac = float(input_rate / d_int) / output_rate
    transition = 0.15 * (output_rate / float(input_rate))
    cutoff = 0.5 * d_int / (input_rate / output_rate)
    return d_int, frac, transition, cutoff


def shift_rate(offset, input_rate):
    return -offset / input_rate  # Selector._updateShift


def squelch_parameters(output_rate, measurements_per_sec=16, readings_per_sec=4):
    block = int(output_rate / measurements_per_sec)  # Selector._buildSquelch
    return dict(length=block, decimation=5, hangLength=2 * block, flushLength=5 * block,
                reportInterval=int(measurements_per_sec / readings_per_sec))


def squelch_level(db):
    return float(math.pow(10, db / 10))  # Selector._convertToLinear


def chain_params(input_rate, offset, mode="nfm", output_rate=12000, bandpass=None,
                 squelch_db=-150, output=_lib.OUT_ADPCM, agc_profile=None, hd_output_rate=48000,
                 wfm_deemphasis_tau=50e-6, nr_enabled=False, nr_threshold=0):
    """owrx_chain_params for ClientDemodulatorChain([Selector, demod, ClientAudioChain]).

    WFM (FixedIfSampleRateChain + HdAudio): the Selector runs at 250 kHz
    (ClientDemodulatorChain._getSelectorOutputRate, owrx/dsp.py:150-158) and the audio at
    hd_output_rate (owrx/dsp.py:494, :160-166)."""
    wfm = mode == "wfm"
    audio_rate = hd_output_rate if wfm or mode in HD_MODES else output_rate
    if wfm:
        output_rate = WFM_IF_RATE
    elif mode in HD_MODES:
        output_rate = hd_output_rate
    d, frac, tbw, cutoff = decimation(input_rate, output_rate)
    if bandpass is None:
        bandpass = MODE_BANDPASS.get(mode)
    sq = squelch_parameters(output_rate)
    p = _lib.ChainParams()
    p.shift_rate = f32(shift_rate(offset, input_rate))
    p.decimation = d
    p.transition = f32(tbw)
    p.cutoff = f32(cutoff)
    p.frac_rate = frac  # FractionalDecimator(rate) only when frac != 1.0 (selector.py:32)
    if bandpass is not None:
        p.bandpass = 1
        p.bp_low = f32(bandpass[0] / output_rate)
        p.bp_high = f32(bandpass[1] / output_rate)
    p.bp_transition = f32(320.0 / output_rate)
    p.sq_length = sq["length"]
    p.sq_decimation = sq["decimation"]
    p.sq_hang = sq["hangLength"]
    p.sq_flush = sq["flushLength"]
    p.sq_report = sq["reportInterval"]
    p.sq_level = f32(squelch_level(squelch_db))
    demod = MODE_DEMOD[mode]
    p.demod = demod
    if agc_profile is None:  # NFm/Am: SLOW (analog.py:35,12); Ssb: ssb_agc_profile "Fast"
        agc_profile = _lib.AGC_FAST if demod == _lib.DEMOD_SSB else _lib.AGC_SLOW
    p.agc_profile = agc_profile
    # Am, SAm: setInitialGain(200)
    p.agc_initial_gain = 200.0 if demod in (_lib.DEMOD_AM, _lib.DEMOD_SAM) else -1.0
    p.agc_max_gain = 3.0 if demod == _lib.DEMOD_NFM else -1.0        # NFm: setMaxGain(3)
    p.audio_rate = audio_rate
    p.output = output
    p.nr_enabled = 1 if nr_enabled else 0  # ClientAudioChain NoiseFilter (clientaudio.py:12-13)
    p.nr_threshold = f32(nr_threshold)
    if wfm:
        p.if_rate = float(WFM_IF_RATE)
        p.deemph_tau = f32(wfm_deemphasis_tau)
    p.afc_update, p.afc_sample = MODE_AFC.get(mode, (0, 0))
    p.audio_gain = MODE_GAIN.get(mode, 0.0)
    return p


def resampler_params(sdr_samp_rate, sdr_center_freq, center_freq, samp_rate):
    """(owrx_chain_params, if_samp_rate) for the service Resampler (owrx/source/resampler.py:11-26):
    Shift((sdr_cf - cf) / sdr_rate) -> FirDecimate(int(sdr_rate / rate), 0.15 * if_rate / sdr_rate)
    with FirDecimate's default cutoff 0.5; the output is the cf32 IF at sdr_rate / decimation."""
    shift = (sdr_center_freq - center_freq) / sdr_samp_rate
    d = int(float(sdr_samp_rate) / samp_rate)
    if_rate = sdr_samp_rate / d
    p = _lib.ChainParams()
    p.shift_rate = f32(shift)
    p.decimation = d
    p.transition = f32(0.15 * (if_rate / float(sdr_samp_rate)))
    p.cutoff = f32(0.5)
    p.frac_rate = 1.0
    p.output = _lib.OUT_IQ
    return p, if_rate
