"""Synthetic wideband cf32 IQ for tests and the benchmark:
complex AWGN sigma=0.01 per component (numpy PCG64, seed 20251114) plus one modulated carrier
per chain at f_c = -0.45 fs + (c + 0.5) * 0.9 fs / C (rounded to 1 Hz, not bin aligned).
NFM: 1 kHz tone, 2.5 kHz deviation, amplitude 0.05; AM: 30 % 1 kHz; USB / CW: +1 kHz /
+800 Hz tones; WFM: 1 kHz tone, 75 kHz deviation, amplitude 0.2.  No datasets exist offline;
the data is labelled "synthetic" everywhere."""
import numpy as np

SEED = 20251114


def carrier_offsets(samp_rate, nchains):
    return [int(round(-0.45 * samp_rate + (c + 0.5) * 0.9 * samp_rate / nchains))
            for c in range(nchains)]


def make_iq(samp_rate, n, modes, seed=SEED, noise=0.01, amp=0.05, start=0):
    """modes: list of 'nfm' | 'am' | 'usb' | 'lsb' | 'cw' | 'wfm', one carrier per entry."""
    rng = np.random.Generator(np.random.PCG64(seed))
    x = (rng.standard_normal(n, dtype=np.float32) * noise
         + 1j * rng.standard_normal(n, dtype=np.float32) * noise).astype(np.complex64)
    t = (np.arange(n, dtype=np.float64) + start) / samp_rate
    offs = carrier_offsets(samp_rate, len(modes))
    for mode, f in zip(modes, offs):
        if mode == "nfm":
            ph = 2 * np.pi * f * t + (2500.0 / 1000.0) * np.sin(2 * np.pi * 1000.0 * t)
            x += (amp * np.exp(1j * ph)).astype(np.complex64)
        elif mode == "am":
            env = amp * (1.0 + 0.3 * np.sin(2 * np.pi * 1000.0 * t))
            x += (env * np.exp(2j * np.pi * f * t)).astype(np.complex64)
        elif mode == "wfm":
            ph = 2 * np.pi * f * t + (75000.0 / 1000.0) * np.sin(2 * np.pi * 1000.0 * t)
            x += (0.2 * np.exp(1j * ph)).astype(np.complex64)
        elif mode in ("usb", "cw", "lsb"):
            tone = {"usb": 1000.0, "cw": 800.0, "lsb": -1000.0}[mode]
            x += (amp * np.exp(2j * np.pi * (f + tone) * t)).astype(np.complex64)
        else:
            raise ValueError(mode)
    return x, offs
