"""ctypes wrapper of oracle/liboracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the csdr modules (oracle/csdr_oracle.c) used as the parity checker by
tests/, by __graft_entry__.smoke() and as the cpu_baseline leg of bench.py.  Never imported by
the product package (openwebrx_amd/, pycsdr/).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "liboracle.so")


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


class AgcParams(ctypes.Structure):
    _fields_ = [("reference", ctypes.c_float), ("attack_rate", ctypes.c_float),
                ("decay_rate", ctypes.c_float), ("max_gain", ctypes.c_float),
                ("initial_gain", ctypes.c_float), ("hang_time", ctypes.c_int)]


class ChainParams(ctypes.Structure):
    _fields_ = [("shift_rate", ctypes.c_float), ("decimation", ctypes.c_int),
                ("ntaps", ctypes.c_int), ("taps", ctypes.c_void_p),
                ("frac_rate", ctypes.c_double), ("bp_ntaps", ctypes.c_int),
                ("bp_taps", ctypes.c_void_p), ("sq_length", ctypes.c_int),
                ("sq_decimation", ctypes.c_int), ("sq_hang", ctypes.c_int),
                ("sq_flush", ctypes.c_int), ("sq_report", ctypes.c_int),
                ("sq_level", ctypes.c_float), ("mode", ctypes.c_int), ("agc", AgcParams),
                ("deemph_alpha", ctypes.c_float), ("compression", ctypes.c_int)]


_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_int64
_F = ctypes.c_float
_D = ctypes.c_double
PROTOS = {
    "orc_firdes_filter_len": (_I, [_F]),
    "orc_firdes_lowpass_f": (None, [_P, _I, _F]),
    "orc_firdes_bandpass_c": (None, [_P, _I, _F, _F]),
    "orc_hamming_window": (None, [_P, _I]),
    "orc_shift": (None, [_P, _P, _L, _F]),
    "orc_fir_decimate": (_L, [_P, _L, _P, _I, _I, _P]),
    "orc_fractional_decimator": (_L, [_P, _L, _D, _P]),
    "orc_fir_complex": (None, [_P, _L, _P, _I, _P]),
    "orc_fir_real": (None, [_P, _L, _P, _I, _P]),
    "orc_noise_filter": (_L, [_P, _L, _F, _P]),
    "orc_fractional_decimator_f": (_L, [_P, _L, _D, _P]),
    "orc_wfm_deemphasis_alpha": (_F, [_I, _F]),
    "orc_squelch": (_L, [_P, _L, _I, _I, _I, _I, _I, _F, _P, _P, _P]),
    "orc_fmdemod": (None, [_P, _L, _P]),
    "orc_amdemod": (None, [_P, _L, _P]),
    "orc_realpart": (None, [_P, _L, _P]),
    "orc_limit": (None, [_P, _L, _F, _P]),
    "orc_convert_s16_f": (None, [_P, _L, _P]),
    "orc_gain": (None, [_P, _L, _F, _P]),
    "orc_dcblock": (None, [_P, _L, _P]),
    "orc_deemphasis": (None, [_P, _L, _F, _P]),
    "orc_nfm_deemphasis_alpha": (_F, [_I]),
    "orc_agc_profile": (None, [_I, _P]),
    "orc_agc": (None, [_P, _L, _P, _P]),
    "orc_convert_f_s16": (None, [_P, _L, _P]),
    "orc_adpcm_encode": (_L, [_P, _L, _I, _P]),
    "orc_adpcm_decode": (_L, [_P, _L, _P]),
    "orc_waterfall_rows": (_L, [_P, _L, _I, _I, _I, _F, _P]),
    "orc_fftswap": (None, [_P, _I, _P]),
    "orc_fft_adpcm_row": (_L, [_P, _I, _P]),
    "orc_fft": (None, [_P, _I, _P]),
    "orc_run_chain": (_L, [_P, _L, _P, _P, _L, _P, _P]),
    "orc_run_chains_parallel": (_L, [_P, _L, _P, _I, _I]),
    "orc_run_workload": (_L, [_P, _L, _I, _I, _I, _F, _P, _I, _I]),
}

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        l = ctypes.CDLL(_SO)
        for k, (r, a) in PROTOS.items():
            f = getattr(l, k)
            f.restype = r
            f.argtypes = a
        _lib = l
    return _lib


def _c64(x):
    return np.ascontiguousarray(x, dtype=np.complex64)


def _f32(x):
    return np.ascontiguousarray(x, dtype=np.float32)


# ---- stage helpers (numpy in / numpy out) ---------------------------------------------------
def filter_len(tbw):
    return lib().orc_firdes_filter_len(tbw)


def lowpass(ntaps, cutoff):
    t = np.zeros(ntaps, np.float32)
    lib().orc_firdes_lowpass_f(t.ctypes.data, ntaps, cutoff)
    return t


def bandpass_taps(ntaps, lo, hi):
    t = np.zeros(ntaps, np.complex64)
    lib().orc_firdes_bandpass_c(t.ctypes.data, ntaps, lo, hi)
    return t


def hamming(n):
    w = np.zeros(n, np.float32)
    lib().orc_hamming_window(w.ctypes.data, n)
    return w


def shift(x, rate):
    x = _c64(x)
    y = np.empty_like(x)
    lib().orc_shift(x.ctypes.data, y.ctypes.data, x.size, rate)
    return y


def fir_decimate(x, taps, d):
    x = _c64(x)
    taps = _f32(taps)
    y = np.empty(max(1, x.size // d + 1), np.complex64)
    m = lib().orc_fir_decimate(x.ctypes.data, x.size, taps.ctypes.data, taps.size, d, y.ctypes.data)
    return y[:m]


def fractional_decimator(x, rate):
    x = _c64(x)
    y = np.empty(int(x.size / rate) + 4, np.complex64)
    m = lib().orc_fractional_decimator(x.ctypes.data, x.size, rate, y.ctypes.data)
    return y[:m]


def fir_real(x, taps):
    x = _f32(x)
    taps = _f32(taps)
    y = np.empty_like(x)
    lib().orc_fir_real(x.ctypes.data, x.size, taps.ctypes.data, taps.size, y.ctypes.data)
    return y


def fractional_decimator_f(x, rate):
    x = _f32(x)
    y = np.empty(int(x.size / rate) + 4, np.float32)
    m = lib().orc_fractional_decimator_f(x.ctypes.data, x.size, rate, y.ctypes.data)
    return y[:m]


def noise_filter(x, threshold_db):
    """NoiseFilter (documented choice, see orc_noise_filter)."""
    x = _f32(x)
    y = np.empty(x.size + 512, np.float32)
    m = lib().orc_noise_filter(x.ctypes.data, x.size, threshold_db, y.ctypes.data)
    return y[:m]


def wfm_audio(sq, if_rate, audio_rate, tau):
    """WFm (csdr/chain/analog.py:55-116) after the Selector: FmDemod, Limit,
    FractionalDecimator(FLOAT, if/audio, prefilter=True), WfmDeemphasis(audio, tau)."""
    r = float(if_rate) / float(audio_rate)
    pf = lowpass(filter_len(np.float32(0.03)), np.float32(0.5 / r))
    a = fractional_decimator_f(fir_real(limit(fmdemod(sq)), pf), r)
    return deemphasis(a, lib().orc_wfm_deemphasis_alpha(int(audio_rate), np.float32(tau or 50e-6)))


def fir_complex(x, taps):
    x = _c64(x)
    taps = _c64(taps)
    y = np.empty_like(x)
    lib().orc_fir_complex(x.ctypes.data, x.size, taps.ctypes.data, taps.size, y.ctypes.data)
    return y


def squelch(x, length, dec, hang, flush, report, level):
    x = _c64(x)
    y = np.empty_like(x)
    p = np.zeros(x.size // max(1, length) + 2, np.float32)
    npw = ctypes.c_int64()
    m = lib().orc_squelch(x.ctypes.data, x.size, length, dec, hang, flush, report, level,
                          y.ctypes.data, p.ctypes.data, ctypes.byref(npw))
    return y[:m], p[:npw.value]


def _unary(name, x, out_dtype=np.float32, inp=_f32):
    x = inp(x)
    y = np.empty(x.size, out_dtype)
    getattr(lib(), name)(x.ctypes.data, x.size, y.ctypes.data)
    return y


def fmdemod(x):
    return _unary("orc_fmdemod", x, inp=_c64)


def amdemod(x):
    return _unary("orc_amdemod", x, inp=_c64)


def realpart(x):
    return _unary("orc_realpart", x, inp=_c64)


def dcblock(x):
    return _unary("orc_dcblock", x)


def convert_s16_f(x):
    """Convert(COMPLEX_SHORT | SHORT, COMPLEX_FLOAT | FLOAT): int16 scalars -> float32."""
    x = np.ascontiguousarray(x, dtype=np.int16)
    y = np.empty(x.size, np.float32)
    lib().orc_convert_s16_f(x.ctypes.data, x.size, y.ctypes.data)
    return y


def gain(x, g):
    """Gain(FLOAT | COMPLEX_FLOAT, g) on float32 scalars."""
    x = _f32(x)
    y = np.empty_like(x)
    lib().orc_gain(x.ctypes.data, x.size, g, y.ctypes.data)
    return y


def limit(x, m=1.0):
    x = _f32(x)
    y = np.empty_like(x)
    lib().orc_limit(x.ctypes.data, x.size, m, y.ctypes.data)
    return y


def deemphasis(x, alpha):
    x = _f32(x)
    y = np.empty_like(x)
    lib().orc_deemphasis(x.ctypes.data, x.size, alpha, y.ctypes.data)
    return y


def nfm_alpha(rate):
    return lib().orc_nfm_deemphasis_alpha(rate)


def agc_params(profile, initial_gain=None, max_gain=None):
    p = AgcParams()
    lib().orc_agc_profile(profile, ctypes.byref(p))
    if initial_gain is not None:
        p.initial_gain = initial_gain
    if max_gain is not None:
        p.max_gain = max_gain
    return p


def agc(x, params):
    x = _f32(x)
    y = np.empty_like(x)
    lib().orc_agc(x.ctypes.data, x.size, ctypes.byref(params), y.ctypes.data)
    return y


def convert_s16(x):
    return _unary("orc_convert_f_s16", x, out_dtype=np.int16)


def adpcm_encode(s16, sync):
    s = np.ascontiguousarray(s16, dtype=np.int16)
    out = np.zeros(s.size // 2 + 8 * (s.size // 2002 + 2), np.uint8)
    n = lib().orc_adpcm_encode(s.ctypes.data, s.size, 1 if sync else 0, out.ctypes.data)
    return out[:n].tobytes()


def adpcm_decode(data):
    b = np.frombuffer(bytes(data), np.uint8).copy()
    out = np.zeros(2 * b.size, np.int16)
    lib().orc_adpcm_decode(b.ctypes.data, b.size, out.ctypes.data)
    return out


def waterfall_rows(x, n_fft, hop, avg, add_db=-70.0):
    x = _c64(x)
    nframes = (x.size - n_fft) // hop + 1 if x.size >= n_fft else 0
    rows = np.zeros((max(1, nframes // max(1, avg)), n_fft), np.float32)
    r = lib().orc_waterfall_rows(x.ctypes.data, x.size, n_fft, hop, max(1, avg), add_db,
                                 rows.ctypes.data)
    return rows[:r]


def fftswap(row):
    row = _f32(row)
    out = np.empty_like(row)
    lib().orc_fftswap(row.ctypes.data, row.size, out.ctypes.data)
    return out


def fft_adpcm_row(row_db):
    row_db = _f32(row_db)
    out = np.zeros((row_db.size + 10) // 2 + 1, np.uint8)
    n = lib().orc_fft_adpcm_row(row_db.ctypes.data, row_db.size, out.ctypes.data)
    return out[:n].tobytes()


# ---- whole chain -----------------------------------------------------------------------------
MODE_INDEX = {0: 0, 1: 1, 2: 2}


def chain_from_engine_params(p):
    """Oracle chain parameters equivalent to an openwebrx_amd ChainParams.  Filter taps are
    designed by the oracle's own restatement (not the product's)."""
    ntaps = filter_len(p.transition)
    taps = lowpass(ntaps, np.float32(p.cutoff) / np.float32(p.decimation))
    bp = None
    if p.bandpass:
        bp = bandpass_taps(filter_len(p.bp_transition), p.bp_low, p.bp_high)
    agcp = agc_params(p.agc_profile,
                      p.agc_initial_gain if p.agc_initial_gain >= 0 else None,
                      p.agc_max_gain if p.agc_max_gain >= 0 else None)
    c = ChainParams()
    c.shift_rate = p.shift_rate
    c.decimation = p.decimation
    c.ntaps = ntaps
    c.taps = taps.ctypes.data
    c.frac_rate = p.frac_rate
    c.bp_ntaps = 0 if bp is None else bp.size
    c.bp_taps = None if bp is None else bp.ctypes.data
    c.sq_length = p.sq_length
    c.sq_decimation = p.sq_decimation
    c.sq_hang = p.sq_hang
    c.sq_flush = p.sq_flush
    c.sq_report = p.sq_report
    c.sq_level = p.sq_level
    c.mode = p.demod
    c.agc = agcp
    c.deemph_alpha = nfm_alpha(p.audio_rate)
    c.compression = 1 if p.output == 1 else 0
    c._keep = (taps, bp)  # keep numpy buffers alive
    return c


def run_chain(iq, cparams):
    iq = _c64(iq)
    cap = iq.size // 4 + 65536
    out = np.zeros(cap, np.uint8)
    sm = np.zeros(iq.size // 64 + 16, np.float32)
    ns = ctypes.c_int64()
    n = lib().orc_run_chain(iq.ctypes.data, iq.size, ctypes.byref(cparams), out.ctypes.data, cap,
                            sm.ctypes.data, ctypes.byref(ns))
    if n < 0:
        raise RuntimeError("oracle output capacity")
    return out[:n].tobytes(), sm[:ns.value].copy()


def stages(iq, p):
    """Every intermediate stage of one chain (oracle), keyed like the engine's debug taps."""
    c = chain_from_engine_params(p)
    taps = c._keep[0]
    s = shift(iq, p.shift_rate)
    ddc = fir_decimate(s, taps, p.decimation)
    fd = fractional_decimator(ddc, p.frac_rate) if p.frac_rate != 1.0 else ddc
    bp = fir_complex(fd, c._keep[1]) if p.bandpass else fd
    sq, power = squelch(bp, p.sq_length, p.sq_decimation, p.sq_hang, p.sq_flush, p.sq_report,
                        p.sq_level)
    if p.demod == 3:  # WFM: no Agc
        dem = wfm_audio(sq, p.if_rate, p.audio_rate, p.deemph_tau)
        return dict(ddc=ddc, frac=fd, bandpass=bp, squelch=sq, smeter=power, demod=dem, agc=dem,
                    s16=convert_s16(dem))
    if p.demod == 0:
        dem = deemphasis(limit(fmdemod(sq)), c.deemph_alpha)
    elif p.demod == 1:
        dem = dcblock(amdemod(sq))
    elif p.demod == 4:  # SAm / RawSAm: Afc -> RealPart -> DcBlock (csdr/chain/analog.py:141-167)
        dem = dcblock(realpart(afc(sq, p.afc_update, p.afc_sample)))
    else:
        dem = realpart(sq)
    # RawAm / RawSAm: Gain(audio_gain) in the Agc's place (analog.py:29, :165)
    ag = gain(dem, p.audio_gain) if getattr(p, "audio_gain", 0) > 0 else agc(dem, c.agc)
    out = dict(ddc=ddc, frac=fd, bandpass=bp, squelch=sq, smeter=power, demod=dem, agc=ag)
    if getattr(p, "nr_enabled", 0):
        out["nr"] = noise_filter(ag, p.nr_threshold)
        out["s16"] = convert_s16(out["nr"])
    else:
        out["s16"] = convert_s16(ag)
    return out


def audio_resample(x, in_rate, out_rate):
    """AudioResampler(inputRate, clientRate) (csdr/chain/clientaudio.py:15-16), restated in
    float64: rational L/M with L = out/g, M = in/g; y[m] = L sum_j h[j] x_up[m M - j] with x_up
    the input upsampled by L (zeros between samples); h = lowpass at 0.5 / max(L, M) of the
    upsampled rate, transition a fifth of that (csdr's own design is not in the reference:
    parity unpinned, the build's documented choice)."""
    from math import gcd
    x = np.asarray(x, np.float64)
    g = gcd(int(in_rate), int(out_rate))
    L, M = int(out_rate) // g, int(in_rate) // g
    c = 0.5 / max(L, M)
    h = lowpass(filter_len(np.float32(0.2 * c)), c).astype(np.float64)
    n_out = ((x.size - 1) * L) // M + 1 if x.size else 0
    y = np.zeros(n_out)
    for m in range(n_out):
        up = m * M
        j = np.arange(up % L, h.size, L)
        i = (up - j) // L
        ok = i >= 0
        y[m] = L * np.dot(h[j[ok]], x[i[ok]])
    return y


def afc(x, update_period=10, sample_period=4):
    """Afc(updatePeriod, samplePeriod) of SAm / RawSAm (csdr/chain/analog.py:141-167).  csdr's
    algorithm is not in the reference (parity unpinned); this restates the build's documented
    choice: y = x e^{-j ph}, ph += w (ph wrapped to [-pi, pi]); every S samples the pair
    product y[n] conj(y[n - S]) is summed, and after U pairs w += arg(sum) / (2 S).  Phase and
    frequency in float64, the rotation of each sample in float32 without fused multiply-adds
    (as the kernel computes it)."""
    x = np.asarray(x, np.complex64)
    U, S = int(update_period), int(sample_period)
    out = np.empty(x.size, np.complex64)
    ph = w = acc_re = acc_im = 0.0
    prev = (np.float32(0), np.float32(0))
    pairs = 0
    for n in range(x.size):
        c, s = np.float32(np.cos(ph)), np.float32(np.sin(ph))
        xr, xi = np.float32(x[n].real), np.float32(x[n].imag)
        yr = np.float32(np.float32(xr * c) + np.float32(xi * s))
        yi = np.float32(np.float32(xi * c) - np.float32(xr * s))
        ph += w
        if ph > np.pi:
            ph -= 2.0 * np.pi
        elif ph < -np.pi:
            ph += 2.0 * np.pi
        if n % S == 0:
            if n >= S:
                pr, pi_ = float(prev[0]), float(prev[1])
                acc_re += float(yr) * pr + float(yi) * pi_
                acc_im += float(yi) * pr - float(yr) * pi_
                pairs += 1
                if pairs == U:
                    w += np.arctan2(acc_im, acc_re) / (2.0 * S)
                    acc_re = acc_im = 0.0
                    pairs = 0
            prev = (yr, yi)
        out[n] = np.complex64(complex(yr, yi))
    return out
