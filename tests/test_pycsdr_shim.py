"""The pycsdr drop-in (openwebrx_amd.pycsdr): API surface and error behaviour of
pycsdr.modules / pycsdr.types as the reference calls them, the fusion planner
against the reference's chain parameters, and (GPU) byte-identical outputs of a module graph
wired like csdr.chain vs the engine driven directly."""
import threading
import time

import numpy as np
import pytest

from openwebrx_amd import _lib, params
from openwebrx_amd import pycsdr
from openwebrx_amd.pycsdr import _graph
from openwebrx_amd.pycsdr import modules as M
from openwebrx_amd.pycsdr.types import AgcProfile, Format


class Chain:
    """What csdr/chain/__init__.py:11-20 does with a worker list: one Buffer between
    consecutive workers, typed by the producer's output format."""

    def __init__(self, workers):
        self.workers = workers
        for a, b in zip(workers, workers[1:]):
            buf = M.Buffer(a.getOutputFormat())
            a.setWriter(buf)
            b.setReader(buf.getReader())

    def setReader(self, r):
        self.workers[0].setReader(r)

    def setWriter(self, w):
        self.workers[-1].setWriter(w)


def selector(fs, offset, mode, squelch=True):
    """Modules of Selector(fs, 12000) + setFrequencyOffset + setBandpass
    (csdr/chain/selector.py:89-166), parameters from openwebrx_amd.params."""
    d, frac, tbw, cutoff = params.decimation(fs, 12000)
    shift = M.Shift(0.0)
    shift.setRate(params.shift_rate(offset, fs))
    w = [shift, M.FirDecimate(d, tbw, cutoff)]
    if frac != 1.0:
        w.append(M.FractionalDecimator(Format.COMPLEX_FLOAT, frac))
    bp = M.Bandpass(transition=320.0 / 12000, use_fft=True)
    lo, hi = params.MODE_BANDPASS[mode]
    bp.setBandpass(lo / 12000, hi / 12000)
    w.append(bp)
    if squelch:
        sq = params.squelch_parameters(12000)
        w.append(M.Squelch(Format.COMPLEX_FLOAT, length=sq["length"],
                           decimation=sq["decimation"], hangLength=sq["hangLength"],
                           flushLength=sq["flushLength"], reportInterval=sq["reportInterval"]))
    return w


def demodulator(mode):
    """NFm / Am / Ssb (csdr/chain/analog.py:11-52, 119-127)."""
    agc = M.Agc(Format.FLOAT)
    if mode == "nfm":
        agc.setProfile(AgcProfile.SLOW)
        agc.setMaxGain(3)
        return [M.FmDemod(), M.Limit(), M.NfmDeemphasis(12000), agc]
    if mode == "am":
        agc.setProfile(AgcProfile.SLOW)
        agc.setInitialGain(200)
        return [M.AmDemod(), M.DcBlock(), agc]
    agc.setProfile(AgcProfile("Fast"))
    return [M.RealPart(), agc]


def client_audio(adpcm=True):
    """ClientAudioChain(FLOAT, 12000, 12000, "adpcm") (csdr/chain/clientaudio.py:6-35)."""
    w = [M.Convert(Format.FLOAT, Format.SHORT)]
    if adpcm:
        w.append(M.AdpcmEncoder(sync=True))
    return w


def fft_chain(n, hop, avg, adpcm=True):
    """FftChain workers (csdr/chain/fft.py:25-96)."""
    fft = M.Fft(size=n, every_n_samples=0)
    fft.setEveryNSamples(hop)
    w = [fft, M.LogAveragePower(add_db=-70, fft_size=n, avg_number=avg), M.FftSwap(fft_size=n)]
    if adpcm:
        w.append(M.FftAdpcm(fft_size=n))
    return w


# ---- API surface (CPU) ---------------------------------------------------------------------

def test_types_and_versions():
    assert AgcProfile("Fast") is AgcProfile.FAST
    assert [p.value for p in AgcProfile] == ["Fast", "Slow", "Mid", "Laggy"]
    assert {f.itemsize for f in Format} == {1, 2, 4, 8}
    assert tuple(int(x) for x in M.csdr_version.split(".")) >= (0, 18, 0)
    assert tuple(int(x) for x in M.version.split(".")) >= (0, 18, 0)


def test_imports_of_the_reference_resolve():
    """Every name the reference imports from pycsdr.modules exists."""
    names = ("AdpcmEncoder Afc Agc AmDemod AudioResampler Bandpass BaudotDecoder Buffer "
             "Ccir476Decoder Ccir493Decoder Convert CwDecoder DBPskDecoder DcBlock Downmix "
             "DscDecoder ExecModule FaxDecoder Fft FftAdpcm FftSwap FirDecimate FmDemod "
             "FractionalDecimator Gain Limit LogAveragePower LogPower Lowpass MFRttyDecoder "
             "Module NavtexDecoder NfmDeemphasis NoiseFilter Reader RealPart RttyDecoder Shift "
             "SitorBDecoder SnrSquelch Squelch SstvDecoder TcpSource Throttle TimingRecovery "
             "VaricodeDecoder WfmDeemphasis Writer csdr_version version").split()
    for n in names:
        assert hasattr(M, n), n
    with pytest.raises(NotImplementedError):
        M.SstvDecoder()


def test_install_registers_pycsdr():
    import sys
    pycsdr.install()
    from pycsdr.modules import Buffer  # noqa: F401  (the reference's import lines)
    from pycsdr.types import Format as F2
    assert F2 is Format and sys.modules["pycsdr.modules"] is M


def test_buffer_multireader_and_stop():
    b = M.Buffer(Format.FLOAT)
    r1, r2 = b.getReader(), b.getReader()
    b.write(np.arange(5, dtype=np.float32).tobytes() + b"\x01")  # a stray byte stays pending
    assert np.frombuffer(r1.read(), np.float32).tolist() == [0, 1, 2, 3, 4]
    assert len(r2.read()) == 20
    got = []
    t = threading.Thread(target=lambda: got.append(r1.read()))
    t.start()
    time.sleep(0.05)
    r1.stop()
    t.join(2)
    assert got == [None]


def test_buffer_ring_wraps_and_lagging_reader_loses_oldest():
    """The byte ring (owrx/dsp.py:846-863 pumps read what writers put in): writes of random
    sizes wrap the ring; readers at different paces see exactly the stream, item aligned, and
    one that falls more than the capacity behind resumes at the oldest byte still held."""
    rng = np.random.default_rng(3)
    b = M.Buffer(Format.COMPLEX_FLOAT, size=1000)  # 8000 bytes
    fast, slow = b.getReader(), b.getReader()
    stream = rng.standard_normal(2 * 30000).astype(np.float32).view(np.complex64)
    got_fast, pos = [], 0
    while pos < stream.size:
        m = min(int(rng.integers(1, 700)), stream.size - pos)
        b.write(stream[pos:pos + m].tobytes())
        pos += m
        got_fast.append(np.frombuffer(bytes(fast.read()), np.complex64))
    assert np.array_equal(np.concatenate(got_fast), stream[:pos])
    tail = np.frombuffer(bytes(slow.read()), np.complex64)   # fell far behind: the last 1000
    assert np.array_equal(tail, stream[pos - 1000:pos])
    b.write(stream[:3].tobytes())
    assert np.array_equal(np.frombuffer(bytes(slow.read()), np.complex64), stream[:3])


def test_buffer_write_cost_independent_of_history():
    """write() / read() do not scan earlier chunks or all readers: 20 000 small writes with a
    reader that never reads (it only loses the oldest data) cost about what 2 000 do, per write."""
    def run(nw):
        b = M.Buffer(Format.CHAR, size=1 << 16)
        idle = [b.getReader() for _ in range(8)]
        r = b.getReader()
        t0 = time.perf_counter()
        for i in range(nw):
            b.write(b"x" * 100)
            if i % 16 == 0:
                r.read()
        return (time.perf_counter() - t0) / nw
    run(500)
    small, large = run(2000), run(20000)
    assert large < 3 * small + 2e-5, (small, large)


def test_reader_stop_drops_unread_bytes():
    """Reader.stop() (csdr/module/__init__.py:36-53 pumps exit on None): read() returns None at
    once, whatever the buffer still holds for this reader -- unread bytes are dropped, which is
    the mechanism behind round 2's truncated collector (r02ag: a collector stopped right after
    the engine finished).  resume() re-arms it and the held bytes come back."""
    b = M.Buffer(Format.CHAR)
    r = b.getReader()
    b.write(b"abcdef")
    assert bytes(r.read()) == b"abcdef"
    b.write(b"ghij")
    r.stop()
    assert r.available() == 4
    assert r.read() is None  # stopped: the 4 pending bytes are not returned
    r.resume()
    assert bytes(r.read()) == b"ghij"


def test_collector_stopped_after_draining_sees_every_byte():
    """A collector thread behind a fast writer: stopped without draining it loses the tail (the
    r02ag symptom); stopped once available() is 0 (_stop_collector) it sees every byte, in order."""
    payload = [bytes([i % 251]) * (1 + (i * 7) % 300) for i in range(2000)]
    total = b"".join(payload)

    def run(drain):
        b = M.Buffer(Format.CHAR, size=1 << 22)
        r = b.getReader()
        out = []
        slow = threading.Event()

        def collect():
            for x in iter(r.read, None):
                out.append(bytes(x))
                if not slow.is_set():
                    time.sleep(0.1)  # behind the writer at first
                    slow.set()
        t = threading.Thread(target=collect)
        t.start()
        for p in payload:
            b.write(p)
        if drain:
            deadline = time.time() + 5
            while r.available() > 0 and time.time() < deadline:
                time.sleep(0.002)
        r.stop()
        t.join(5)
        return b"".join(out)

    assert run(True) == total
    got = run(False)
    assert total.startswith(got) and len(got) < len(total)


def test_tcp_source_feeds_the_wideband_buffer():
    """SdrSource.getBuffer (owrx/source/__init__.py:307-314, 325-329): TcpSource(port,
    COMPLEX_FLOAT) writes whatever the SDR's IQ socket delivers into the wideband Buffer.  A
    local server sends cf32 in odd-sized pieces (TCP splits samples anywhere): every read of the
    Buffer returns whole samples, and the bytes are the stream's, in order; stop() ends the pump
    and closes the socket."""
    import socket
    rng = np.random.default_rng(3)
    iq = (rng.standard_normal(50000) + 1j * rng.standard_normal(50000)).astype(np.complex64)
    raw = iq.tobytes()
    srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    srv.bind(("127.0.0.1", 0))
    srv.listen(1)
    port = srv.getsockname()[1]
    sizes = [1, 7, 13, 4099, 65537, 3]

    def serve():
        conn, _ = srv.accept()
        i, k = 0, 0
        while i < len(raw):
            n = sizes[k % len(sizes)]
            conn.sendall(raw[i:i + n])
            i += n
            k += 1
        time.sleep(0.2)
        conn.close()

    t = threading.Thread(target=serve, daemon=True)
    t.start()
    buf = M.Buffer(Format.COMPLEX_FLOAT)
    r = buf.getReader()
    src = M.TcpSource(port, Format.COMPLEX_FLOAT)
    src.setWriter(buf)
    got, t0 = [], time.time()
    while sum(len(g) for g in got) < len(raw) and time.time() - t0 < 20:
        d = r.read() if r.available() >= 8 else None
        if d:
            assert len(d) % 8 == 0
            got.append(bytes(d))
        else:
            time.sleep(0.01)
    assert b"".join(got) == raw
    src.stop()
    t.join(5)
    srv.close()
    src._worker.join(5)
    assert not src._worker.is_alive()


def test_format_mismatch_raises_valueerror():
    """setReader / setWriter raise ValueError (callers catch it, csdr/chain/__init__.py:60-84)."""
    with pytest.raises(ValueError):
        M.FmDemod().setReader(M.Buffer(Format.FLOAT).getReader())
    with pytest.raises(ValueError):
        M.FmDemod().setWriter(M.Buffer(Format.COMPLEX_FLOAT))
    M.FmDemod().setWriter(M.Buffer(Format.FLOAT))


@pytest.mark.parametrize("mode", ["nfm", "am", "usb"])
def test_planner_matches_reference_chain_params(mode):
    """A graph wired like ClientDemodulatorChain plans to exactly the engine parameters the
    reference chain code implies (openwebrx_amd.params, pinned by tests/golden)."""
    fs, off = 10000000, 123456
    wide = M.Buffer(Format.COMPLEX_FLOAT)
    mods = selector(fs, off, mode) + demodulator(mode) + client_audio()
    ch = Chain(mods)
    out = M.Buffer(Format.CHAR)
    ch.setWriter(out)
    ch.setReader(wide.getReader())
    seg = _graph.plan_segment(mods[0])
    assert seg is not None and seg[0] == "chain" and seg[2] == mods
    got = _graph.chain_params_struct(seg[1])
    want = params.chain_params(fs, off, mode, output=_lib.OUT_ADPCM)
    for name, _ in _lib.ChainParams._fields_:
        g, w = getattr(got, name), getattr(want, name)
        assert g == pytest.approx(w, rel=1e-6, abs=1e-12), name
    _graph.finish(wide)


def test_bench_c4_dropin_graphs_plan_like_the_reference():
    """bench.py's drop-in at C4's rate rebuilds the recorded NFM client graph and FftChain at
    61.44 Msps (_scaled_steps): the planner fuses them into exactly the chain parameters the
    reference chain code implies at that rate (params.chain_params: D = 5120, no
    FractionalDecimator) and the 65 536-bin FftChain's (avg 149, hop 45 816)."""
    import os
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    import bench
    import dsp_replay
    fs = 61440000
    s, sg = bench._scaled_steps(fs, 65536)
    wide, mods, outs, power = dsp_replay.build(s)
    mods[0].setRate(params.shift_rate(123456, fs))
    seg = _graph.plan_segment(mods[0])
    assert seg is not None and seg[0] == "chain"
    got = _graph.chain_params_struct(seg[1])
    want = params.chain_params(fs, 123456, "nfm", output=_lib.OUT_ADPCM)
    assert want.decimation == 5120
    for name, _ in _lib.ChainParams._fields_:
        g, w = getattr(got, name), getattr(want, name)
        assert g == pytest.approx(w, rel=1e-6, abs=1e-12), name
    fmods = [dsp_replay._make(d) for d in sg["graph"]]
    for a, b in zip(fmods, fmods[1:]):
        buf = M.Buffer(a.getOutputFormat())
        a.setWriter(buf)
        b.setReader(buf.getReader())
    fmods[-1].setWriter(M.Buffer(Format.CHAR))
    fmods[0].setReader(wide.getReader())
    kind, p, _ = _graph.plan_segment(fmods[0])
    avg, hop = params.fft_parameters(fs, 65536, 9, 0.3)
    assert kind == "waterfall" and p == dict(fft_size=65536, hop=hop, avg=avg, add_db=-70.0,
                                             adpcm=True) and (avg, hop) == (149, 45816)
    _graph.finish(wide)


def test_planner_waterfall_and_rewire():
    wide = M.Buffer(Format.COMPLEX_FLOAT)
    mods = fft_chain(4096, 2867, 93)
    ch = Chain(mods)
    ch.setWriter(M.Buffer(Format.CHAR))
    ch.setReader(wide.getReader())
    kind, p, used = _graph.plan_segment(mods[0])
    assert kind == "waterfall" and p == dict(fft_size=4096, hop=2867, avg=93, add_db=-70.0,
                                             adpcm=True)
    # FftAverager.setFftAverages replaces the averager (csdr/chain/fft.py:13-17)
    new = M.LogAveragePower(add_db=-70, fft_size=4096, avg_number=10)
    mods[1].stop()
    buf = M.Buffer(Format.FLOAT)
    new.setWriter(buf)
    mods[2].setReader(buf.getReader())
    b0 = M.Buffer(Format.COMPLEX_FLOAT)
    mods[0].setWriter(b0)
    new.setReader(b0.getReader())
    kind, p, used = _graph.plan_segment(mods[0])
    assert p["avg"] == 10 and used[1] is new
    _graph.finish(wide)


def test_planner_secondary_fft_tap():
    """ClientDemodulatorChain with a secondary FftChain on the Selector output buffer
    (owrx/dsp.py:220-225): the chain still fuses and carries the FftChain parameters."""
    fs, off = 2400000, 50000
    wide = M.Buffer(Format.COMPLEX_FLOAT)
    sel = selector(fs, off, "usb")
    mods = sel + demodulator("usb") + client_audio()
    ch = Chain(mods)
    ch.setWriter(M.Buffer(Format.CHAR))
    ch.setReader(wide.getReader())
    avg, hop = params.fft_parameters(12000, 2048, 9, 0.3)
    fmods = fft_chain(2048, hop, avg)
    Chain(fmods)
    fmods[-1].setWriter(M.Buffer(Format.CHAR))
    fmods[0].setReader(sel[-1].writer.getReader())
    kind, p, used = _graph.plan_segment(mods[0])
    assert kind == "chain" and used == mods
    assert p["secondary_fft"] == dict(fft_size=2048, hop=1333, avg=1, add_db=-70.0, adpcm=True)
    assert p["secondary_modules"] == fmods
    _graph.finish(wide)


@pytest.mark.parametrize("fs", [2400000, 10000000])
def test_planner_wfm_chain(fs):
    """Selector(fs, 250000) + WFm(48000, 50e-6) + ClientAudioChain(FLOAT, 48000, 48000) wired
    like ClientDemodulatorChain plans to params.chain_params(fs, off, "wfm") exactly."""
    off = 300000
    d, frac, tbw, cutoff = params.decimation(fs, 250000)
    shift = M.Shift(0.0)
    shift.setRate(params.shift_rate(off, fs))
    sel = [shift, M.FirDecimate(d, tbw, cutoff)]
    if frac != 1.0:
        sel.append(M.FractionalDecimator(Format.COMPLEX_FLOAT, frac))
    bp = M.Bandpass(transition=320.0 / 250000, use_fft=True)
    bp.setBandpass(-124000 / 250000, 124000 / 250000)
    sq = params.squelch_parameters(250000)
    sel += [bp, M.Squelch(Format.COMPLEX_FLOAT, length=sq["length"], decimation=sq["decimation"],
                          hangLength=sq["hangLength"], flushLength=sq["flushLength"],
                          reportInterval=sq["reportInterval"])]
    dem = [M.FmDemod(), M.Limit(),
           M.FractionalDecimator(Format.FLOAT, 250000.0 / 48000, prefilter=True),
           M.WfmDeemphasis(48000, 50e-6)]
    mods = sel + dem + client_audio()
    wide = M.Buffer(Format.COMPLEX_FLOAT)
    ch = Chain(mods)
    ch.setWriter(M.Buffer(Format.CHAR))
    ch.setReader(wide.getReader())
    kind, p, used = _graph.plan_segment(mods[0])
    assert kind == "chain" and used == mods
    got = _graph.chain_params_struct(p)
    want = params.chain_params(fs, off, "wfm", output=_lib.OUT_ADPCM)
    for name, _ in _lib.ChainParams._fields_:
        if name in ("agc_profile", "agc_initial_gain", "agc_max_gain"):
            continue  # WFm has no Agc
        g, w = getattr(got, name), getattr(want, name)
        assert g == pytest.approx(w, rel=1e-6, abs=1e-12), name
    _graph.finish(wide)


def test_planner_noise_filter(tmp_path):
    """ClientAudioChain(FLOAT, 12000, 12000, "adpcm", True, 10) = [NoiseFilter(10), Convert,
    AdpcmEncoder] (recorded in tests/golden/chain_params.json "clientaudio_nr") fuses with
    nr_enabled / nr_threshold (BASELINE config 5)."""
    import json
    import os
    with open(os.path.join(os.path.dirname(__file__), "golden", "chain_params.json")) as f:
        rec = json.load(f)["clientaudio_nr"]
    assert [e["module"] for e in rec if e["op"] == "new"] == ["NoiseFilter", "Convert",
                                                              "AdpcmEncoder"]
    thr = rec[0]["args"][0]
    fs, off = 10000000, -250000
    wide = M.Buffer(Format.COMPLEX_FLOAT)
    mods = selector(fs, off, "usb") + demodulator("usb") + [M.NoiseFilter(thr)] + client_audio()
    ch = Chain(mods)
    ch.setWriter(M.Buffer(Format.CHAR))
    ch.setReader(wide.getReader())
    kind, p, used = _graph.plan_segment(mods[0])
    assert kind == "chain" and used == mods
    got = _graph.chain_params_struct(p)
    want = params.chain_params(fs, off, "usb", output=_lib.OUT_ADPCM, nr_enabled=True,
                               nr_threshold=thr)
    for name, _ in _lib.ChainParams._fields_:
        assert getattr(got, name) == pytest.approx(getattr(want, name), rel=1e-6, abs=1e-12), name
    assert got.nr_enabled == 1 and got.nr_threshold == 10.0
    _graph.finish(wide)


def test_unrecognised_graph_is_not_fused():
    wide = M.Buffer(Format.COMPLEX_FLOAT)
    shift = M.Shift(0.1)
    fm = M.FmDemod()
    Chain([shift, fm])
    shift.setReader(wide.getReader())
    fm.setWriter(M.Buffer(Format.FLOAT))
    assert _graph.plan_segment(shift) is None
    _graph.finish(wide)


# ---- end to end on the GPU -------------------------------------------------------------

def _collect(buf):
    r = buf.getReader()
    out = []
    t = threading.Thread(target=lambda: [out.append(bytes(x)) for x in iter(r.read, None)])
    t.start()
    return r, t, out


def _stop_collector(col, timeout=5.0):
    """Let a collector read what its buffer holds, then stop it: Reader.stop() makes read()
    return None at once, dropping unread bytes (the reference's semantics), so stopping a
    collector that is still behind would truncate what it saw."""
    r, t, _ = col
    deadline = time.time() + timeout
    while r.available() > 0 and time.time() < deadline:
        time.sleep(0.005)
    r.stop()
    t.join(timeout)


@pytest.mark.gpu
def test_pycsdr_graph_equals_engine():
    """Wideband Buffer -> two ClientDemodulatorChain-shaped graphs + an FftChain graph, fed in
    odd-sized writes: audio, s-meter and waterfall bytes equal the engine driven directly."""
    from openwebrx_amd import Engine, synth
    fs = 2400000
    modes = ["nfm", "am"]
    iq, offs = synth.make_iq(fs, 1 << 20, modes)
    avg, hop = params.fft_parameters(fs, 4096, 9, 0.3)

    wide = M.Buffer(Format.COMPLEX_FLOAT, size=1 << 22)
    outs, smeters, graphs = [], [], []
    for off, mode in zip(offs, modes):
        mods = selector(fs, off, mode) + demodulator(mode) + client_audio()
        ch = Chain(mods)
        out, pw = M.Buffer(Format.CHAR, size=1 << 22), M.Buffer(Format.FLOAT, size=1 << 20)
        [m for m in mods if isinstance(m, M.Squelch)][0].setPowerWriter(pw)
        outs.append(_collect(out))
        smeters.append(_collect(pw))
        ch.setWriter(out)
        ch.setReader(wide.getReader())
        graphs.append(mods)
    # secondary FftChain on the first chain's Selector output (owrx/dsp.py:220-225)
    sel_out = [m for m in graphs[0] if isinstance(m, M.Squelch)][0].writer
    smods = fft_chain(2048, 1333, 1)
    Chain(smods)
    sfout = M.Buffer(Format.CHAR, size=1 << 22)
    sfcol = _collect(sfout)
    smods[-1].setWriter(sfout)
    smods[0].setReader(sel_out.getReader())
    wmods = fft_chain(4096, hop, avg)
    wch = Chain(wmods)
    wout = M.Buffer(Format.CHAR, size=1 << 22)
    wcol = _collect(wout)
    wch.setWriter(wout)
    wch.setReader(wide.getReader())

    i = 0
    for s in [100003, 77777, 300001] * 10:
        if i >= iq.size:
            break
        wide.write(iq[i:i + s].tobytes())
        i += s
    while _graph._drivers.get(id(wide)).reader.available() > 0:
        time.sleep(0.01)
    _graph.finish(wide)
    for col in outs + smeters + [wcol, sfcol]:
        _stop_collector(col)

    eng = Engine(1.0, max_block=_graph.BLOCK)
    ref_ch = [eng.chain(params.chain_params(fs, o, m, output=_lib.OUT_ADPCM))
              for o, m in zip(offs, modes)]
    wf = eng.waterfall(4096, hop, avg, -70.0, True)
    ref_ch[0].set_secondary_fft(2048, 1333, 1, -70.0, True)
    for j in range(0, iq.size, _graph.BLOCK):
        eng.push(iq[j:j + _graph.BLOCK])
    eng.sync()
    for k, c in enumerate(ref_ch):
        assert b"".join(outs[k][2]) == c.read_audio()
        sm = np.frombuffer(b"".join(smeters[k][2]), np.float32)
        np.testing.assert_array_equal(sm, c.read_smeter())
    assert b"".join(wcol[2]) == wf.read()
    sf = b"".join(sfcol[2])
    assert len(sf) >= 2 * 1029 and sf == ref_ch[0].read_secondary_fft().tobytes()
    eng.close()


@pytest.mark.gpu
def test_standalone_modules_match_oracle():
    """Modules outside a fused segment run alone on the GPU (one worker each), like csdr's
    one-thread-per-module: FmDemod -> Limit -> Convert -> AdpcmEncoder on a Buffer graph."""
    import oracle
    rng = np.random.default_rng(5)
    x = (rng.standard_normal(40000) + 1j * rng.standard_normal(40000)).astype(np.complex64)
    src = M.Buffer(Format.COMPLEX_FLOAT, size=1 << 20)
    mods = [M.FmDemod(), M.Limit(), M.Convert(Format.FLOAT, Format.SHORT),
            M.AdpcmEncoder(sync=True)]
    ch = Chain(mods)
    out = M.Buffer(Format.CHAR, size=1 << 20)
    r, t, got = _collect(out)
    ch.setWriter(out)
    ch.setReader(src.getReader())
    for i in range(0, x.size, 9999):
        src.write(x[i:i + 9999].tobytes())
    want = oracle.adpcm_encode(oracle.convert_s16(oracle.limit(oracle.fmdemod(x))), 1)
    deadline = time.time() + 30
    while sum(len(g) for g in got) < len(want) - 1 and time.time() < deadline:
        time.sleep(0.05)
    r.stop()
    t.join(5)
    for m in mods:
        m.stop()
    data = b"".join(got)
    assert data == want[:len(data)] and len(want) - len(data) <= 1


def test_ingest_modules_formats():
    """The ingest conversion Chain of owrx/source/direct.py:51-71 builds on the shim."""
    conv = M.Convert(Format.COMPLEX_SHORT, Format.COMPLEX_FLOAT)
    gain = M.Gain(Format.COMPLEX_FLOAT, 5.0)
    assert conv.getInputFormat() == Format.COMPLEX_SHORT
    assert conv.getOutputFormat() == Format.COMPLEX_FLOAT == gain.getInputFormat()
    with pytest.raises(ValueError):
        conv.setReader(M.Buffer(Format.COMPLEX_FLOAT).getReader())
    with pytest.raises(NotImplementedError):
        M.Convert(Format.COMPLEX_FLOAT, Format.COMPLEX_SHORT)


def test_planner_recognises_service_resampler():
    """Shift -> FirDecimate -> Buffer (owrx/source/resampler.py) plans as an OUT_IQ chain even
    with a (non-fusable) consumer on the IF buffer."""
    wide = M.Buffer(Format.COMPLEX_FLOAT)
    p, _ = params.resampler_params(2400000, 145000000, 145300000, 48000)
    shift = M.Shift(p.shift_rate)
    fir = M.FirDecimate(p.decimation, p.transition)
    Chain([shift, fir])
    shift.setReader(wide.getReader())
    out = M.Buffer(Format.COMPLEX_FLOAT)
    fir.setWriter(out)
    out.getReader()
    kind, q, used = _graph.plan_segment(shift)
    assert kind == "chain" and used == [shift, fir]
    assert q["output"] == _lib.OUT_IQ and q["decimation"] == 50 and q["cutoff"] == 0.5
    _graph.finish(wide)


# ---- multi-GPU placement and failure propagation ---------------------------------------------

def test_placement_balances_groups():
    """multi.Placement (the drop-in's chain -> engine assignment): balanced within each
    FirDecimate design, then by total load; released slots are reused."""
    from openwebrx_amd.multi import Placement
    pl = Placement(3)
    a = [pl.place(("chain", 833)) for _ in range(7)]
    assert a == [0, 1, 2, 0, 1, 2, 0]
    assert [pl.place(("chain", 200)) for _ in range(2)] == [1, 2]
    assert pl.place(("waterfall",)) == 0  # every engine holds 3: lowest index
    pl.release(1, ("chain", 833))
    assert pl.place(("chain", 833)) == 1


def _graph_with_outputs(fs, offs, modes, wf=None):
    wide = M.Buffer(Format.COMPLEX_FLOAT, size=1 << 22)
    cols = []
    for off, mode in zip(offs, modes):
        mods = selector(fs, off, mode) + demodulator(mode) + client_audio()
        ch = Chain(mods)
        out, pw = M.Buffer(Format.CHAR, size=1 << 22), M.Buffer(Format.FLOAT, size=1 << 20)
        [m for m in mods if isinstance(m, M.Squelch)][0].setPowerWriter(pw)
        cols.append((_collect(out), _collect(pw)))
        ch.setWriter(out)
        ch.setReader(wide.getReader())
    wcol = None
    if wf is not None:
        wmods = fft_chain(*wf)
        wch = Chain(wmods)
        wout = M.Buffer(Format.CHAR, size=1 << 22)
        wcol = _collect(wout)
        wch.setWriter(wout)
        wch.setReader(wide.getReader())
    return wide, cols, wcol


def test_engine_failure_ends_outputs(monkeypatch):
    """An engine that cannot run (here: a GPU index that does not exist) puts the driver in
    FAILED, calls the on_failure callbacks (an SdrSource's fail(), owrx/source/__init__.py:
    224-227) and ends the output buffers, so the DSP pumps' read() returns None instead of
    blocking forever (owrx/dsp.py:858-861)."""
    monkeypatch.setenv("OWRX_AMD_DEVICES", "97")
    fs = 2400000
    wide = M.Buffer(Format.COMPLEX_FLOAT)
    mods = selector(fs, 1000, "nfm") + demodulator("nfm") + client_audio()
    ch = Chain(mods)
    out = M.Buffer(Format.CHAR)
    ch.setWriter(out)
    ch.setReader(wide.getReader())
    r = out.getReader()
    failed = []
    _graph.on_failure(wide, failed.append)
    wide.write(np.zeros(1000, np.complex64).tobytes())
    got = []
    t = threading.Thread(target=lambda: got.append(r.read()), daemon=True)
    t.start()
    t.join(20)
    assert got == [None]
    assert len(failed) == 1 and _graph.state(wide) == "FAILED"
    _graph.finish(wide)


@pytest.mark.gpu
def test_stalled_gpu_fails_driver_and_ends_outputs():
    """A GPU that stops completing work must fail like a dead SDR source, not hang the server
    (owrx/source/__init__.py:432-448 fail() -> onFail; owrx/dsp.py:858-861 pumps end on None):
    a stream-A kernel that sleeps 3 s (owrx_debug_stall) against a 300 ms stall bound makes the
    engine's bounded wait expire -> TimeoutError -> the driver is FAILED, the on_failure callback
    runs once with that error and the client's audio reader returns None within seconds."""
    import time
    fs = 2400000
    wide = M.Buffer(Format.COMPLEX_FLOAT, size=1 << 23)
    mods = selector(fs, 1000, "nfm") + demodulator("nfm") + client_audio()
    ch = Chain(mods)
    out = M.Buffer(Format.CHAR, size=1 << 22)
    ch.setWriter(out)
    ch.setReader(wide.getReader())
    r = out.getReader()
    failed = []
    _graph.on_failure(wide, failed.append)
    blk = np.zeros(_graph.BLOCK, np.complex64).tobytes()
    wide.write(blk)  # the driver plans the chain, creates its engine and pushes
    drv, deadline = None, time.time() + 60
    while time.time() < deadline:
        drv = _graph._drivers.get(id(wide))
        if drv is not None and drv.engines:
            break
        time.sleep(0.05)
    assert drv is not None and drv.engines
    with _graph._lock:
        drv.engine.set_stall_timeout(300)
        drv.engine.debug_stall(0, 3000000)
        t_stall = time.time()
    for _ in range(8):
        wide.write(blk)
    got = []

    def pump():
        while r.read() is not None:
            pass
        got.append(time.time())

    t = threading.Thread(target=pump, daemon=True)
    t.start()
    t.join(20)
    assert got, "the audio reader did not end"
    assert got[0] - t_stall < 10.0
    assert _graph.state(wide) == "FAILED"
    assert len(failed) == 1 and isinstance(failed[0], TimeoutError), failed
    time.sleep(max(0.0, t_stall + 3.5 - time.time()))  # the injected kernel has exited
    _graph.finish(wide)


@pytest.mark.gpu
def test_pycsdr_sharded_engines_equal_single(monkeypatch):
    """The drop-in over several engines in one process (OWRX_AMD_DEVICES="0,0,0": three
    engines on the test box's one GPU -- the code path of one engine per GPU) writes
    byte-identical audio, s-meter and waterfall bytes to the single-engine run."""
    from openwebrx_amd import synth
    fs = 2400000
    modes = ["nfm", "am", "usb", "nfm", "cw", "am", "nfm"]
    iq, offs = synth.make_iq(fs, 1 << 20, modes)
    avg, hop = params.fft_parameters(fs, 4096, 9, 0.3)

    def run(devs):
        monkeypatch.setenv("OWRX_AMD_DEVICES", devs)
        wide, cols, wcol = _graph_with_outputs(fs, offs, modes, wf=(4096, hop, avg))
        i = 0
        for s in [100003, 77777, 300001] * 10:
            if i >= iq.size:
                break
            wide.write(iq[i:i + s].tobytes())
            i += s
        drv = _graph._drivers.get(id(wide))
        while drv.reader.available() > 0:
            time.sleep(0.01)
        _graph.finish(wide)  # the driver replans on its first read: count after it finished
        nengines = len(drv.engines)
        res = []
        for col in [c for pair in cols for c in pair] + [wcol]:
            _stop_collector(col)
            res.append(b"".join(col[2]))
        return nengines, res

    n1, single = run("0")
    n3, sharded = run("0,0,0")
    assert (n1, n3) == (1, 3)
    assert all(len(b) > 0 for b in single)
    for k, (a, b) in enumerate(zip(single, sharded)):
        assert a == b, k


class _Registry:
    """The part of owrx.metrics.Metrics (owrx/metrics.py:29-70) register() uses."""

    def __init__(self):
        self.metrics = {}

    def addMetric(self, name, metric):
        self.metrics[name] = metric

    def getFlatMetrics(self):
        return {k: m.getValue() for k, m in self.metrics.items()}


def test_engine_metrics_report_failed_driver(monkeypatch):
    """Engine counters as OpenWebRX metrics: a driver whose engine cannot start counts under
    gpu.failed, with no engines."""
    from openwebrx_amd.pycsdr import metrics
    monkeypatch.setenv("OWRX_AMD_DEVICES", "97")
    reg = _Registry()
    names = metrics.register(reg)
    assert "gpu.blocks" in names and "gpu.failed" in names
    fs = 2400000
    wide = M.Buffer(Format.COMPLEX_FLOAT)
    mods = selector(fs, 1000, "nfm") + demodulator("nfm") + client_audio()
    ch = Chain(mods)
    ch.setWriter(M.Buffer(Format.CHAR))
    ch.setReader(wide.getReader())
    failed = []
    _graph.on_failure(wide, failed.append)
    wide.write(np.zeros(1000, np.complex64).tobytes())
    t0 = time.time()
    while not failed and time.time() - t0 < 20:
        time.sleep(0.02)
    flat = reg.getFlatMetrics()
    assert flat["gpu.failed"] >= 1 and flat["gpu.engines"] == 0
    _graph.finish(wide)


@pytest.mark.gpu
def test_engine_metrics_count_blocks_and_audio():
    """After a fused graph ran, gpu.blocks / gpu.samples_in / gpu.audio_bytes count its work."""
    from openwebrx_amd import synth
    from openwebrx_amd.pycsdr import metrics
    reg = _Registry()
    metrics.register(reg)
    fs = 2400000
    iq, offs = synth.make_iq(fs, 1 << 20, ["nfm"])
    wide, cols, _ = _graph_with_outputs(fs, offs, ["nfm"])
    for i in range(0, iq.size, 200003):
        wide.write(iq[i:i + 200003].tobytes())
    drv = _graph._drivers.get(id(wide))
    while drv.reader.available() > 0:
        time.sleep(0.01)
    time.sleep(0.2)
    flat = reg.getFlatMetrics()
    _graph.finish(wide)
    for pair in cols:
        for col in pair:
            _stop_collector(col)
    assert flat["gpu.engines"] >= 1 and flat["gpu.segments"] >= 1
    assert flat["gpu.blocks"] >= 3 and flat["gpu.samples_in"] >= 3 * _graph.BLOCK
    assert flat["gpu.audio_bytes"] > 0 and flat["gpu.failed"] == 0
