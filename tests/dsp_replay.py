"""Rebuilds, with the shim's pycsdr modules, a module graph the reference's ClientDemodulatorChain
built (recorded in tests/golden/dsp_graph.json by tests/golden/make_dsp_graph.py): same classes,
constructor parameters, setters and wiring order.  Test infrastructure (no reference needed)."""
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "dsp_graph.json")


def steps():
    with open(GOLDEN) as f:
        return {s["step"]: s for s in json.load(f)}


def _make(d):
    from openwebrx_amd.pycsdr import modules as M
    from openwebrx_amd.pycsdr.types import AgcProfile, Format
    c = d["class"]
    if c == "Shift":
        return M.Shift(d["rate"])
    if c == "FirDecimate":
        return M.FirDecimate(d["decimation"], d["transition"], d["cutoff"])
    if c == "FractionalDecimator":
        return M.FractionalDecimator(Format[d["format"]], d["rate"], prefilter=d["prefilter"])
    if c == "Bandpass":
        return M.Bandpass(d["low_cut"], d["high_cut"], d["transition"], d["use_fft"])
    if c == "Squelch":
        m = M.Squelch(Format.COMPLEX_FLOAT, length=d["length"], decimation=d["decimation"],
                      hangLength=d["hang_length"], flushLength=d["flush_length"],
                      reportInterval=d["report_interval"])
        m.setSquelchLevel(d["level"])
        return m
    if c in ("FmDemod", "AmDemod", "RealPart", "DcBlock"):
        return getattr(M, c)()
    if c == "Limit":
        return M.Limit(d["max_amplitude"])
    if c == "Afc":
        return M.Afc(d["update_period"], d["sample_period"])
    if c == "Gain":
        return M.Gain(Format[d["format"]], d["gain"])
    if c == "NfmDeemphasis":
        return M.NfmDeemphasis(d["sample_rate"])
    if c == "WfmDeemphasis":
        return M.WfmDeemphasis(d["sample_rate"], d["tau"])
    if c == "Agc":
        m = M.Agc(Format.FLOAT)
        m.setProfile(AgcProfile(d["profile"]))
        if d.get("initial_gain") is not None:
            m.setInitialGain(d["initial_gain"])
        if d.get("max_gain") is not None:
            m.setMaxGain(d["max_gain"])
        return m
    if c == "NoiseFilter":
        return M.NoiseFilter(d["threshold"])
    if c == "Convert":
        return M.Convert(Format[d["format"]], Format[d["out_format"]])
    if c == "AdpcmEncoder":
        return M.AdpcmEncoder(sync=d["sync"])
    if c == "Fft":
        return M.Fft(d["size"], every_n_samples=d["every_n_samples"])
    if c == "LogAveragePower":
        return M.LogAveragePower(add_db=d["add_db"], fft_size=d["fft_size"],
                                 avg_number=d["avg_number"])
    if c == "LogPower":
        return M.LogPower(add_db=d["add_db"])
    if c == "FftSwap":
        return M.FftSwap(d["fft_size"])
    if c == "FftAdpcm":
        return M.FftAdpcm(d["fft_size"])
    raise ValueError("replay: no builder for %s" % c)


def build(step, wide=None):
    """(wideband Buffer, modules by graph index, output Buffer by graph index, squelch power
    Buffer).  Modules that feed nothing in the recorded graph write into a Buffer of their own
    (the client's audio / rows / secondary outputs).  `wide`: an existing wideband Buffer
    (several clients on one source)."""
    from openwebrx_amd.pycsdr import modules as M
    from openwebrx_amd.pycsdr.types import Format
    g = step["graph"]
    # the test writes faster than real time: room for the whole stream (a lagging reader of a
    # full ring loses the oldest data, like the reference's Buffer)
    if wide is None:
        wide = M.Buffer(Format.COMPLEX_FLOAT, size=1 << 23)
    mods = [None if d["class"] == "PythonReader" else _make(d) for _, d, _ in g]
    outs = {}

    def out_of(i):
        if i not in outs:
            outs[i] = M.Buffer(Format[g[i][1]["out_format"]])
            mods[i].setWriter(outs[i])
        return outs[i]

    power = None
    for i, d, src in g:
        if mods[i] is None:
            continue
        if d["class"] == "Squelch":
            power = M.Buffer(Format.FLOAT)
            mods[i].setPowerWriter(power)
        out_of(i)
    for i, d, src in g:
        r = (wide if src < 0 else outs[src]).getReader()
        if mods[i] is None:
            mods[i] = r  # a Python consumer (decoder stand-in): the test reads it directly
        else:
            mods[i].setReader(r)
    return wide, mods, outs, power
