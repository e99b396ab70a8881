"""HIP path vs the oracle (oracle/csdr_oracle.c) on the same seeded inputs, through the C ABI.

Bars (DESIGN.md "Parity"):
* per-sample fp32 stages (FmDemod, AmDemod, RealPart, Limit, DcBlock, NfmDeemphasis, Agc,
  Convert, AdpcmEncoder, FftSwap, FftAdpcm): bit-exact on identical inputs;
* filters (Shift+FirDecimate, FractionalDecimator, Bandpass) and the waterfall FFT: fp32 GPU vs
  the double-precision oracle, relative RMS error <= 1e-5 of the reference signal;
* end-to-end int16 audio within +-1 LSB on >= 99.9 % of samples (float rounding feeds the
  (short) truncation); waterfall int16 (dB*100) within +-1 on >= 99 % of bins.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

oracle = pytest.importorskip("oracle")


@pytest.fixture(scope="module")
def amd():
    import openwebrx_amd
    assert openwebrx_amd.device_count() > 0, "no GPU visible: the HIP path is the only path"
    return openwebrx_amd


def rel_rms(a, b):
    m = min(a.size, b.size)
    a, b = a[:m], b[:m]
    return float(np.sqrt(np.mean(np.abs(a - b) ** 2) / max(np.mean(np.abs(b) ** 2), 1e-30)))


RNG = np.random.Generator(np.random.PCG64(1234))


def cplx(n, scale=0.3):
    return (RNG.standard_normal(n) * scale + 1j * RNG.standard_normal(n) * scale).astype(np.complex64)


def run_module(amd, mtype, data, out_bytes, p0=0.0, p1=-1.0, p2=-1.0, pieces=3):
    m = amd.Module(mtype, p0, p1, p2)
    chunks = np.array_split(data, pieces)
    out = b"".join(m.process(c, out_bytes) for c in chunks)
    m.close()
    return out


# ---------------------------------------------------------------------------------------------
# single modules: bit exact
# ---------------------------------------------------------------------------------------------
def test_fmdemod_bit_exact(amd):
    x = cplx(20000)
    x[100:110] = 0  # zero denominator branch
    g = np.frombuffer(run_module(amd, amd._lib.MOD_FMDEMOD, x, 4 * x.size), np.float32)
    assert np.array_equal(g.view(np.uint32), oracle.fmdemod(x).view(np.uint32))


def test_am_real_limit_convert_bit_exact(amd):
    x = cplx(30001)
    g = np.frombuffer(run_module(amd, amd._lib.MOD_AMDEMOD, x, 4 * x.size), np.float32)
    assert np.array_equal(g, oracle.amdemod(x))
    g = np.frombuffer(run_module(amd, amd._lib.MOD_REALPART, x, 4 * x.size), np.float32)
    assert np.array_equal(g, oracle.realpart(x))
    f = (RNG.standard_normal(30001) * 1.5).astype(np.float32)
    f[:4] = [np.nan, np.inf, -np.inf, 0.0]
    g = np.frombuffer(run_module(amd, amd._lib.MOD_LIMIT, f[4:], 4 * f.size, 1.0), np.float32)
    assert np.array_equal(g, oracle.limit(f[4:]))
    g = np.frombuffer(run_module(amd, amd._lib.MOD_CONVERT_F_S16, f, 2 * f.size), np.int16)
    assert np.array_equal(g, oracle.convert_s16(f))


def test_ingest_convert_gain_bit_exact(amd):
    """Convert(COMPLEX_SHORT, COMPLEX_FLOAT) and Gain(FLOAT | COMPLEX_FLOAT, g) modules."""
    raw = RNG.integers(-32768, 32768, size=2 * 20001, dtype=np.int64).astype(np.int16)
    raw[:4] = [-32768, 32767, 0, -1]
    g = np.frombuffer(run_module(amd, amd._lib.MOD_CONVERT_CS16_CF32, raw.view(np.int32),
                                 8 * (raw.size // 2)), np.float32)
    ref = oracle.convert_s16_f(raw)
    assert np.array_equal(g, ref)
    x = ref.view(np.complex64)
    g = np.frombuffer(run_module(amd, amd._lib.MOD_GAIN, x, 8 * x.size, 5.0, 1.0), np.float32)
    assert np.array_equal(g, oracle.gain(ref, 5.0))
    f = ref[:30001]
    g = np.frombuffer(run_module(amd, amd._lib.MOD_GAIN, f, 4 * f.size, 100.0, 0.0), np.float32)
    assert np.array_equal(g, oracle.gain(f, 100.0))


def test_engine_cs16_ingest_equals_float_ingest(amd):
    """owrx_push_iq_cs16 (conversion fused into the engine window) gives byte-identical
    waterfall rows and chain audio to pushing the oracle-converted cf32 stream."""
    from openwebrx_amd import synth
    fs = 2400000
    n = 1 << 19
    iq, offs = synth.make_iq(fs, n, ["nfm", "am"], amp=0.02)
    raw = np.clip(np.round(np.stack([iq.real, iq.imag], 1).ravel() * 6000), -32768, 32767)
    raw = raw.astype(np.int16)
    conv = oracle.gain(oracle.convert_s16_f(raw), 5.0).view(np.complex64)
    avg, hop = amd.params.fft_parameters(fs, 4096, 9, 0.3)
    outs = []
    for mode in ("cs16", "cf32"):
        eng = amd.Engine(fs, max_block=1 << 17)
        wf = eng.waterfall(4096, hop, avg, adpcm=True)
        chs = [eng.chain(amd.params.chain_params(fs, o, m)) for o, m in zip(offs, ["nfm", "am"])]
        for i in range(0, n, 100000):
            if mode == "cs16":
                eng.push_cs16(raw[2 * i:2 * min(n, i + 100000)], 5.0)
            else:
                eng.push(conv[i:i + 100000])
        eng.sync()
        outs.append([wf.read()] + [c.read_audio() for c in chs])
        eng.close()
    assert len(outs[0][0]) > 0 and all(len(a) > 0 for a in outs[0][1:])
    assert outs[0] == outs[1]


def test_pipeline_depth_outputs_identical(amd):
    """owrx_set_pipeline_depth: 1, 8 (default) and 16 blocks in flight give byte-identical
    waterfall rows, chain audio and s-meter values; the depth is refused once a chain exists."""
    from openwebrx_amd import synth
    fs = 2400000
    n = 1 << 20
    iq, offs = synth.make_iq(fs, n, ["nfm", "usb", "am"], amp=0.02)
    avg, hop = amd.params.fft_parameters(fs, 4096, 9, 0.3)
    outs = []
    for depth in (1, None, 16):
        eng = amd.Engine(fs, max_block=1 << 16)
        if depth is not None:
            eng.set_pipeline_depth(depth)
        wf = eng.waterfall(4096, hop, avg, adpcm=True)
        chs = [eng.chain(amd.params.chain_params(fs, o, m))
               for o, m in zip(offs, ["nfm", "usb", "am"])]
        if depth == 16:
            with pytest.raises(Exception):
                eng.set_pipeline_depth(8)
        for i in range(0, n, 1 << 16):
            eng.push(iq[i:i + (1 << 16)])
        eng.sync()
        audio, _, sm, _ = eng.read_chains(chs)
        outs.append((wf.read(), audio.tobytes(), np.asarray(sm).tobytes()))
        eng.close()
    assert len(outs[0][0]) > 0 and len(outs[0][1]) > 0
    assert outs[0] == outs[1] == outs[2]


def test_dcblock_deemph_bit_exact(amd):
    f = (RNG.standard_normal(25000) * 0.2 + 0.1).astype(np.float32)
    g = np.frombuffer(run_module(amd, amd._lib.MOD_DCBLOCK, f, 4 * f.size), np.float32)
    assert np.array_equal(g.view(np.uint32), oracle.dcblock(f).view(np.uint32))
    a = oracle.nfm_alpha(12000)
    g = np.frombuffer(run_module(amd, amd._lib.MOD_DEEMPH, f, 4 * f.size, a), np.float32)
    assert np.array_equal(g.view(np.uint32), oracle.deemphasis(f, a).view(np.uint32))


@pytest.mark.parametrize("profile,init,maxg", [(0, -1, -1), (1, -1, 3.0), (1, 200.0, -1),
                                               (2, -1, -1), (3, -1, -1)])
def test_agc_bit_exact(amd, profile, init, maxg):
    t = np.arange(40000)
    f = (0.3 * np.sin(2 * np.pi * t / 37.0) * (1 + 0.9 * np.sin(2 * np.pi * t / 9000))).astype(np.float32)
    f[5000:7000] = 0.0
    f[20000:20500] *= 40
    g = np.frombuffer(run_module(amd, amd._lib.MOD_AGC, f, 4 * f.size, profile, init, maxg),
                      np.float32)
    ref = oracle.agc(f, oracle.agc_params(profile, None if init < 0 else init,
                                          None if maxg < 0 else maxg))
    assert np.array_equal(g.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("sync", [0, 1])
def test_adpcm_bit_exact(amd, sync):
    t = np.arange(9999)
    s = (9000 * np.sin(2 * np.pi * t / 55.0) + RNG.integers(-500, 500, t.size)).astype(np.int16)
    s[3000:3100] = 32767
    s[3100:3200] = -32768
    g = run_module(amd, amd._lib.MOD_ADPCM, s, s.size + 1024, sync, pieces=5)
    assert g == oracle.adpcm_encode(s, sync)


def test_fftswap_fftadpcm_bit_exact(amd):
    N = 2048
    rows = (RNG.standard_normal((5, N)) * 15 - 80).astype(np.float32)
    rows[0, 0] = -np.inf
    g = np.frombuffer(run_module(amd, amd._lib.MOD_FFTSWAP, rows.ravel(), 4 * rows.size, N, pieces=1),
                      np.float32).reshape(5, N)
    ref = np.stack([oracle.fftswap(r) for r in rows])
    assert np.array_equal(g, ref)
    g = run_module(amd, amd._lib.MOD_FFTADPCM, ref.ravel(), rows.size, N, pieces=1)
    assert g == b"".join(oracle.fft_adpcm_row(r) for r in ref)


# ---------------------------------------------------------------------------------------------
# waterfall (FftChain)
# ---------------------------------------------------------------------------------------------
def _wf(amd, iq, fs, N, hop, avg, adpcm, block):
    eng = amd.Engine(fs, max_block=block)
    wf = eng.waterfall(N, hop, avg, adpcm=adpcm)
    for i in range(0, iq.size, block):
        eng.push(iq[i:i + block])
    eng.sync()
    rows = wf.read_rows()
    eng.close()
    return rows


@pytest.mark.parametrize("N,fs", [(4096, 2400000), (16384, 10000000), (2048, 1000000), (512, 48000),
                                  (32768, 20000000), (65536, 61440000)])
def test_waterfall_float_rows(amd, N, fs):
    avg, hop = amd.params.fft_parameters(fs, N, 9, 0.3)
    avg = min(avg, 6)  # keep the double-precision oracle quick; avg semantics unchanged
    from openwebrx_amd import synth
    n = hop * avg * 3 + N + 1000
    iq, _ = synth.make_iq(fs, n, ["nfm", "am", "usb"])
    g = _wf(amd, iq, fs, N, hop, avg, False, 1 << 17)
    ref = np.stack([oracle.fftswap(r) for r in oracle.waterfall_rows(iq, N, hop, avg)])
    assert g.shape == ref.shape
    err = np.abs(g - ref)
    assert np.max(err) < 2e-3, np.max(err)   # dB; fp32 FFT vs double


@pytest.mark.parametrize("N,hop", [(16384, 200000), (65536, 150000)])
def test_waterfall_hop_near_the_history(amd, N, hop):
    """A waterfall whose every_n_samples is a large share of the engine's history (2^18 by
    default): a group still open at a block's end must keep its first frame inside the next
    block's window, so the frames per group are clamped to the history
    (wf_frames_per_group).  Rows equal the oracle's, with avg 3."""
    fs, avg = 10000000, 3
    from openwebrx_amd import synth
    n = hop * avg * 4 + N
    iq, _ = synth.make_iq(fs, n, ["nfm", "am"])
    g = _wf(amd, iq, fs, N, hop, avg, False, 1 << 17)
    ref = np.stack([oracle.fftswap(r) for r in oracle.waterfall_rows(iq, N, hop, avg)])
    assert g.shape == ref.shape
    assert np.max(np.abs(g - ref)) < 2e-3


def _wf_batched(amd, iq, fs, N, hop, avg, block, min_frames, history, ingest=False):
    eng = amd.Engine(fs, max_block=block, history=history)
    wf = eng.waterfall(N, hop, avg, adpcm=False)
    wf.set_batch(min_frames)
    for i in range(0, iq.size, block):
        piece = iq[i:i + block]
        if ingest:  # owrx_ingest_buffer / owrx_commit: the caller writes the ring slot
            import ctypes
            # the HIP runtime this process already loaded (torch may bring its own build)
            path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
            hip = ctypes.CDLL(path)
            ptr, cap = eng.ingest_buffer()
            assert cap >= piece.size
            piece = np.ascontiguousarray(piece)
            assert hip.hipMemcpy(ctypes.c_void_p(ptr), ctypes.c_void_p(piece.ctypes.data),
                                 ctypes.c_size_t(8 * piece.size), 1) == 0  # host to device
            eng.commit(piece.size)
        else:
            eng.push(piece)
    st = eng.stats()
    eng.sync()
    rows = wf.read_rows()
    st2 = eng.stats()
    eng.close()
    return rows, st, st2


def test_waterfall_batched_launches(amd):
    """owrx_waterfall_set_batch: frames of several blocks in one launch (rows out at the batch
    or at sync).  The rows match the oracle as per-block launches do, are bit-identical for any
    cut of the stream into blocks (the group size depends on the batch, not the blocks), the
    engine launched far fewer FFTs than it processed blocks, and the push-path ring wrapped
    (history 2^21 < the stream) without losing a sample."""
    fs, N = 10000000, 16384
    avg, hop = amd.params.fft_parameters(fs, N, 9, 0.3)
    avg = 6
    from openwebrx_amd import synth
    n = hop * avg * 7 + N
    iq, _ = synth.make_iq(fs, n, ["nfm", "am", "usb"])
    a, st, st2 = _wf_batched(amd, iq, fs, N, hop, avg, 1 << 16, 40, 1 << 21)
    b, _, _ = _wf_batched(amd, iq, fs, N, hop, avg, 99991, 40, 1 << 21)
    ref = np.stack([oracle.fftswap(r) for r in oracle.waterfall_rows(iq, N, hop, avg)])
    assert a.shape == ref.shape and b.shape == ref.shape
    assert np.max(np.abs(a - ref)) < 2e-3
    assert np.array_equal(a, b)
    blocks = (n + (1 << 16) - 1) >> 16
    # 42 frames: one launch once >= 40 are ready (the rest, if any, at sync); per-block: 7
    assert st["blocks"] == blocks and st["waterfall_launches"] == 1, st
    assert 1 <= st2["waterfall_launches"] <= 2, st2
    assert st2["waterfall_frames"] >= avg * ref.shape[0]
    assert st2["waterfall_samples"] == st2["waterfall_frames"] * hop


def test_waterfall_tail_split_rows_bit_identical(amd):
    """The tail split of the dealt N = 16384 kernels (wf_fft_q16, wf_fft_l32: a launch's last
    groups dealt frame by frame, their frames folded in order by wf_finalize): C3's waterfall (16384 bins, avg 97, hop 11454) over 1 100 frames,
    once batched into launches of ~1 000 frames (over 7/8 of a launch's groups per CU, so the
    split is on) and once per 2^20-sample block (~91 frames per launch: no split).  The rows
    are bit-identical, and equal the oracle's to 2e-3 dB on the first rows."""
    fs, N = 10000000, 16384
    avg, hop = amd.params.fft_parameters(fs, N, 9, 0.3)
    from openwebrx_amd import synth
    n = hop * 1100 + N
    iq, _ = synth.make_iq(fs, n, ["nfm", "am", "usb"])
    hist = 1000 * hop + 2 * N + (1 << 20)
    a, st, st2 = _wf_batched(amd, iq, fs, N, hop, avg, 1 << 20, 1000, hist)
    eng = amd.Engine(fs, max_block=1 << 20)
    wf = eng.waterfall(N, hop, avg, adpcm=False)
    for i in range(0, iq.size, 1 << 20):
        eng.push(iq[i:i + (1 << 20)])
    eng.sync()
    b = wf.read_rows()
    eng.close()
    assert a.shape == b.shape and a.shape[0] >= 10, (a.shape, b.shape)
    assert st2["waterfall_launches"] <= 3, st2
    assert np.array_equal(a, b)
    ref = np.stack([oracle.fftswap(r) for r in oracle.waterfall_rows(iq[:hop * avg * 2 + N], N,
                                                                      hop, avg)])
    assert np.max(np.abs(a[:ref.shape[0]] - ref)) < 2e-3


def test_waterfall_reconfigure_without_drain(amd):
    """SpectrumThread's live settings on a running engine (owrx/fft.py:49-56: fft_fps ->
    FftChain.setFps, fft_voverlap_factor -> setVOverlapFactor, both re-deriving the averaging
    and the block size, csdr/chain/fft.py:57-85) with a chain streaming beside the waterfall: an
    fps change and then an overlap change mid-row, mid-stream.  Rows before each switch row
    equal the oracle's under the old settings, rows after it the oracle's under the new ones
    from the switch frame on; a second FftChain is created and destroyed mid-stream; no call
    drains the pipeline (pipeline_drains unchanged until the final sync)."""
    from openwebrx_amd import synth
    fs, N, B = 2400000, 4096, 1 << 16
    fft = amd.params.fft_parameters
    settings = [fft(fs, N, 9, 0.3), fft(fs, N, 25, 0.3), fft(fs, N, 25, 0.6)]  # (avg, hop)
    rows_each = [4, 5, 4]
    n = sum(a * h * (r + 1) for (a, h), r in zip(settings, rows_each)) + N
    iq, offs = synth.make_iq(fs, n, ["nfm"])
    eng = amd.Engine(fs, max_block=B)
    ch = eng.chain(amd.params.chain_params(fs, offs[0], "nfm"))
    avg, hop = settings[0]
    wf = eng.waterfall(N, hop, avg, adpcm=False)
    d0 = None
    switches = []  # (frames before the switch row's end, settings index)
    frames_done, row_frames, cur = 0, 0, 0
    # push block by block; switch settings once the current setting has produced rows_each rows
    # plus half a row (mid-row), tracking the engine's frame schedule to know the switch row
    pos, extra = 0, None
    while pos < n:
        m = min(B, n - pos)
        eng.push(iq[pos:pos + m])
        pos += m
        if d0 is None:
            d0 = eng.stats()["pipeline_drains"]
        if pos > n // 3 and extra is None:
            extra = eng.waterfall(2048, 1000, 3, adpcm=True)  # a second FftChain joins ...
        if pos > n // 2 and extra is not None and extra is not False:
            extra.close()                                   # ... and leaves mid-stream
            extra = False
        if cur + 1 < len(settings):
            a, h = settings[cur]
            start = sum(s for s, _ in switches)  # sample where the current setting began
            launched = (pos - start - N) // h + 1 if pos - start >= N else 0
            if launched >= a * rows_each[cur] + a // 2:
                # applies at the end of the row in progress
                r_cur = launched // a + (1 if launched % a else 0)
                switches.append((start + r_cur * a * h - start, cur))
                cur += 1
                wf.set(settings[cur][1], settings[cur][0], False)
    assert eng.stats()["pipeline_drains"] == d0, "a waterfall change drained the pipeline"
    assert cur == len(settings) - 1
    eng.sync()
    rows = wf.read_rows()
    assert ch.read_audio()  # the chain streamed throughout
    eng.close()
    # oracle: each setting from its start sample
    refs, start = [], 0
    bounds = [s for s, _ in switches] + [None]
    for k, (a, h) in enumerate(settings):
        span = bounds[k]
        seg = iq[start:] if span is None else iq[start:start + span + N - h]
        r = oracle.waterfall_rows(seg, N, h, a)
        if span is not None:
            r = r[:span // (a * h)]
        refs.extend(oracle.fftswap(x) for x in r)
        if span is not None:
            start += span
    ref = np.stack(refs)
    assert rows.shape[0] >= ref.shape[0] - 1 and rows.shape[0] <= ref.shape[0], (rows.shape, ref.shape)
    k = rows.shape[0]
    per_row = np.max(np.abs(rows[:k] - ref[:k]), axis=1)
    err = np.max(per_row)
    assert err < 2e-3, (err, np.nonzero(per_row >= 2e-3)[0].tolist(), k, ref.shape[0], switches)


def test_waterfall_grow_with_row_copies_held(amd):
    """The round-4 race, forced: a live fps change (owrx_waterfall_set, FftChain.setFps,
    csdr/chain/fft.py:57-85) grows the row buffers while the row stream is held by a 300 ms
    kernel (owrx_debug_stall on stream 4), so the row slots staged before the change still have
    their copies in flight when their pinned destinations are replaced.  Every row equals the
    oracle's under its own settings (<= 2e-3 dB), before and after the switch."""
    import time
    from openwebrx_amd import synth
    fs, N, B = 2400000, 4096, 1 << 16
    fft = amd.params.fft_parameters
    (a0, h0), (a1, h1) = fft(fs, N, 9, 0.3), fft(fs, N, 30, 0.3)
    rows0 = 6
    switch = rows0 * a0 * h0            # the first setting's rows end here (whole blocks below)
    n = switch + 8 * a1 * h1 + N
    iq, _ = synth.make_iq(fs, n, ["nfm"])
    eng = amd.Engine(fs, max_block=B)
    wf = eng.waterfall(N, h0, a0, adpcm=False)
    pos, held, r_sw = 0, None, None
    while pos < n:
        m = min(B, n - pos)
        if held is None and pos + m > switch - 2 * a0 * h0:
            eng.debug_stall(4, 300000)   # the next row slots' copies wait behind this
            held = time.perf_counter()
        eng.push(iq[pos:pos + m])
        pos += m
        if held is not None and held is not False and pos >= switch:
            # applies at the end of the row in progress: the frames launched so far decide it
            launched = (pos - N) // h0 + 1
            r_sw = -(-launched // a0)
            wf.set(h1, a1, False)
            assert time.perf_counter() - held < 0.25, "the change waited for the held copies"
            held = False
    eng.sync()
    rows = wf.read_rows()
    eng.close()
    s0 = r_sw * a0 * h0
    ref = [oracle.fftswap(x) for x in oracle.waterfall_rows(iq[:s0 + N - h0], N, h0, a0)][:r_sw]
    ref += [oracle.fftswap(x) for x in oracle.waterfall_rows(iq[s0:], N, h1, a1)]
    ref = np.stack(ref)
    k = min(rows.shape[0], ref.shape[0])
    assert k >= r_sw + 4, (rows.shape, ref.shape, r_sw)
    assert np.max(np.abs(rows[:k] - ref[:k])) < 2e-3


def test_waterfall_recreate_without_chains_rows_identical(amd):
    """A waterfall destroyed and created again on an engine with no chains (blocks drain without
    waiting for any event, so the slot tail passes blocks whose stream-A copies of the pinned
    group descriptors may not have run: those pinned buffers go back to the pool only after
    stream A ran them): the new FftChain's rows equal a fresh engine's, bit for bit."""
    from openwebrx_amd import synth
    fs, N, B = 2400000, 4096, 1 << 16
    avg, hop = amd.params.fft_parameters(fs, N, 9, 0.3)
    n = 40 * B
    iq, _ = synth.make_iq(fs, n, ["nfm", "am"])
    eng = amd.Engine(fs, max_block=B)
    wf = eng.waterfall(N, hop, avg, adpcm=False)
    half = 20 * B
    for i in range(0, half, B):
        eng.push(iq[i:i + B])
        if i == 10 * B:               # destroy and recreate mid-stream, several times
            for _ in range(3):
                wf.close()
                wf = eng.waterfall(N, hop, avg, adpcm=False)
    start = 11 * B
    for i in range(half, n, B):
        eng.push(iq[i:i + B])
    eng.sync()
    got = wf.read_rows()
    eng.close()
    ref_eng = amd.Engine(fs, max_block=B)
    ref_wf = ref_eng.waterfall(N, hop, avg, adpcm=False)
    for i in range(start, n, B):
        ref_eng.push(iq[i:i + B])
    ref_eng.sync()
    want = ref_wf.read_rows()
    ref_eng.close()
    assert got.shape == want.shape and got.shape[0] > 5, (got.shape, want.shape)
    assert np.array_equal(got, want)


def test_read_chains_rejects_duplicate_handles(amd):
    """owrx_chains_read_audio / _smeter pop each listed chain's ring on host workers: a handle
    listed twice is refused (OWRX_EINVAL) and nothing is read."""
    from openwebrx_amd import synth
    fs = 2400000
    iq, offs = synth.make_iq(fs, 1 << 18, ["nfm", "am"])
    eng = amd.Engine(fs, max_block=1 << 16)
    a, b = (eng.chain(amd.params.chain_params(fs, o, m)) for o, m in zip(offs, ["nfm", "am"]))
    for i in range(0, iq.size, 1 << 16):
        eng.push(iq[i:i + (1 << 16)])
    eng.sync()
    with pytest.raises(Exception):
        eng.read_chains([a, b, a])
    with pytest.raises(Exception):
        eng.read_chains(eng.handles([a, b, a]))
    # half the stream read by chain objects, the rest by a handle array: same bytes as one read
    # of a twin engine
    audio, lens, sm, sc = eng.read_chains([a, b])
    audio = audio.copy()  # a view of the engine's read scratch, reused by the next read
    assert lens[0] > 0 and lens[1] > 0
    for i in range(0, iq.size, 1 << 16):
        eng.push(iq[i:i + (1 << 16)])
    eng.sync()
    audio2, lens2, sm2, sc2 = eng.read_chains(eng.handles([a, b]))
    audio2 = audio2.copy()
    eng.close()
    twin = amd.Engine(fs, max_block=1 << 16)
    a2, b2 = (twin.chain(amd.params.chain_params(fs, o, m)) for o, m in zip(offs, ["nfm", "am"]))
    for _ in range(2):
        for i in range(0, iq.size, 1 << 16):
            twin.push(iq[i:i + (1 << 16)])
    twin.sync()
    ta, tl, tsm, tsc = twin.read_chains([a2, b2])
    twin.close()
    for k in range(2):
        got = audio[lens[:k].sum():lens[:k + 1].sum()].tobytes() + \
            audio2[lens2[:k].sum():lens2[:k + 1].sum()].tobytes()
        assert got == ta[tl[:k].sum():tl[:k + 1].sum()].tobytes()
    assert np.array_equal(np.concatenate([sm[:sc[0]], sm2[:sc2[0]], sm[sc[0]:], sm2[sc2[0]:]]), tsm)


def test_input_retention_same_outputs(amd):
    """owrx_set_input_retention: with a resident recording the host runs up to r blocks ahead of
    stream A (no wait for block k - 1 before returning); audio, s-meter and waterfall rows are
    byte-identical to the default contract (r = 1)."""
    import torch
    from openwebrx_amd import synth
    fs, B = 2400000, 1 << 17
    modes = ["nfm", "usb", "am", "cw"] * 3
    iq, offs = synth.make_iq(fs, 12 * B, modes)
    plist = [amd.params.chain_params(fs, o, m) for o, m in zip(offs, modes)]
    N = 4096
    avg, hop = amd.params.fft_parameters(fs, N, 9, 0.3)

    def run(r):
        eng = amd.Engine(fs, max_block=B)
        eng.set_input_retention(r)
        wf = eng.waterfall(N, hop, avg, adpcm=True)
        chains = [eng.chain(p) for p in plist]
        h = eng.history
        buf = torch.zeros(h + iq.size, dtype=torch.complex64, device="cuda")
        buf[h:] = torch.from_numpy(iq).to("cuda")
        torch.cuda.synchronize()
        for k in range(12):
            eng.process_device(buf.data_ptr() + 8 * (h + k * B), B)
        eng.sync()
        out = ([c.read_audio() for c in chains], [c.read_smeter().tobytes() for c in chains],
               wf.read())
        eng.close()
        return out

    a, b = run(1), run(8)
    assert a[0] == b[0] and a[1] == b[1] and a[2] == b[2]
    assert all(len(x) > 0 for x in a[0]) and len(a[2]) > 0


@pytest.mark.parametrize("group", [2, 3, 4])
@pytest.mark.parametrize("fs,modes,B", [
    (2400000, ["nfm", "usb", "am", "cw"] * 3, 1 << 17),
    (10000000, ["nfm", "usb", "cw"] * 4, 1 << 18),  # C3's design: D = 833, fast convolution
])
def test_block_pairing_same_outputs(amd, fs, modes, B, group, monkeypatch):
    """owrx_set_block_pairing / owrx_set_block_group: contiguous blocks run two (three, four) at a
    time (one DDC GEMM over all their frames); audio, s-meter and waterfall rows byte-identical to
    unpaired processing at the same DDC frame length (a grouped engine may pick a longer one:
    test_block_quads_frame_length).  A block count that leaves blocks held (owrx_sync runs them), a block
    from another buffer (the held ones run alone) and a chain created mid-stream (the guard runs
    the held blocks first)."""
    import torch
    from openwebrx_amd import synth
    # blocks: 0+1 and 2+3 paired, 4 alone (chain created after it), 5 alone (6 is from another
    # buffer), 6 alone, 7+8, 9+10 paired, 11 held until owrx_sync
    nb = 12
    iq, offs = synth.make_iq(fs, nb * B, modes)
    plist = [amd.params.chain_params(fs, o, m) for o, m in zip(offs, modes)]
    N = 4096
    avg, hop = amd.params.fft_parameters(fs, N, 9, 0.3)

    def run(pair):
        eng = amd.Engine(fs, max_block=B)
        eng.set_input_retention(8)
        if pair and group == 2:
            eng.set_block_pairing(True)
        elif pair:
            eng.set_block_group(group)
        wf = eng.waterfall(N, hop, avg, adpcm=True)
        chains = [eng.chain(p) for p in plist[:-1]]
        h = eng.history
        buf = torch.zeros(h + iq.size, dtype=torch.complex64, device="cuda")
        buf[h:] = torch.from_numpy(iq).to("cuda")
        # block 6 from a copy of the stream (same samples and history, another address)
        alt = buf[6 * B:h + 7 * B].clone()
        torch.cuda.synchronize()
        for k in range(nb):
            if k == 5:
                chains.append(eng.chain(plist[-1]))
            ptr = alt.data_ptr() + 8 * h if k == 6 else buf.data_ptr() + 8 * (h + k * B)
            eng.process_device(ptr, B)
        eng.sync()
        st = eng.stats()
        out = ([c.read_audio() for c in chains], [c.read_smeter().tobytes() for c in chains],
               wf.read())
        eng.close()
        return out, st

    (a, sa) = run(False)
    monkeypatch.setenv("OWRX_FC_M", str(sa["ddc_frame_length"]))
    (b, sb) = run(True)
    assert sb["ddc_frame_length"] == sa["ddc_frame_length"]
    # engine blocks: the held blocks run when the group is complete, before the chain created at
    # block 5, and before the other buffer's block 6 and the block after it
    expect = {2: [(0, 1), (2, 3), (4,), (5,), (6,), (7, 8), (9, 10), (11,)],
              3: [(0, 1, 2), (3, 4), (5,), (6,), (7, 8, 9), (10, 11)],
              4: [(0, 1, 2, 3), (4,), (5,), (6,), (7, 8, 9, 10), (11,)]}[group]
    assert sa["blocks"] == nb and sb["blocks"] == len(expect)
    assert all(len(x) > 0 for x in a[0]) and len(a[2]) > 0
    for i in range(len(a[0])):
        assert a[0][i] == b[0][i] and a[1][i] == b[1][i], i
    assert a[2] == b[2]


def test_block_quads_tall_gemm_tiles_same_outputs(amd, monkeypatch):
    """BASELINE config 3 (10 Msps, 256 NFM/USB/CW chains, 2^20-sample blocks) grouped in fours
    (owrx_set_block_group(4)): one DDC GEMM over 52 frames, which takes the 64-frame GEMM tiles
    (fc_mac_lds<4, 4, 2>) and the frame-tile-fastest decode.  Audio and s-meter byte-identical to
    pairs and to one block at a time.  (The per-bin GEMM's K order is the same for every tile
    shape; the tile grids of all three stay unsliced at 256 chains -- fc_kslices -- which a grid
    with few chains would not, and K slices change the summation order.)"""
    import numpy as np
    import torch
    from openwebrx_amd import _lib, synth
    fs, B, nb = 10000000, 1 << 20, 4
    modes = (["nfm", "usb", "cw"] * 86)[:256]
    offs = synth.carrier_offsets(fs, len(modes))
    plist = [amd.params.chain_params(fs, o, m) for o, m in zip(offs, modes)]
    code = {"nfm": 0, "usb": 2, "cw": 3}

    def run(group):
        eng = amd.Engine(fs, max_block=B)
        eng.set_input_retention(8)
        if group > 1:
            eng.set_block_group(group)
        chains = [eng.chain(p) for p in plist]
        h = eng.history
        buf = torch.zeros(h + nb * B, dtype=torch.complex64, device="cuda")
        o64 = np.asarray(offs, np.float64)
        mds = np.asarray([code[m] for m in modes], np.int32)
        _lib.check(_lib.lib.owrx_synth_iq(0, buf.data_ptr() + 8 * h, nb * B, 0, float(fs), len(mds),
                                          o64.ctypes.data, mds.ctypes.data, 20251114, 0.01, 0.05),
                   "owrx_synth_iq")
        torch.cuda.synchronize()
        for k in range(nb):
            eng.process_device(buf.data_ptr() + 8 * (h + k * B), B)
        eng.sync()
        st = eng.stats()
        out = ([c.read_audio() for c in chains], [c.read_smeter().tobytes() for c in chains])
        eng.close()
        return out, st

    monkeypatch.setenv("OWRX_FC_M", "128")  # the default (pinned: the next test varies it)
    (a, sa), (b, sb), (c, sc) = run(1), run(4), run(2)
    assert sa["blocks"] == nb and sb["blocks"] == 1 and sc["blocks"] == 2
    assert sa["ddc_frame_length"] == sb["ddc_frame_length"] == sc["ddc_frame_length"] == 128
    assert all(len(x) > 0 for x in a[0])
    for i in range(len(plist)):
        assert a[0][i] == b[0][i] and a[1][i] == b[1][i], i
        assert a[0][i] == c[0][i] and a[1][i] == c[1][i], i


def test_block_quads_frame_length(amd, monkeypatch):
    """BASELINE config 3 in fours at the other DDC frame length the A/B tried (OWRX_FC_M=192: 32
    frames per grouped GEMM, no tile padding) against one block at a time at the default 128.
    The two frame lengths round the DDC differently (~1e-7), so the chains' int16 audio agrees to
    1 LSB on 99.9 % and their s-meter values to 1e-4 (relative), not byte for byte (at one frame
    length they are: the test above)."""
    import numpy as np
    import torch
    from openwebrx_amd import _lib, synth
    fs, B, nb = 10000000, 1 << 20, 4
    modes = (["nfm", "usb", "cw"] * 86)[:256]
    offs = synth.carrier_offsets(fs, len(modes))
    plist = [amd.params.chain_params(fs, o, m, output=_lib.OUT_S16) for o, m in zip(offs, modes)]
    code = {"nfm": 0, "usb": 2, "cw": 3}

    def run(group):
        eng = amd.Engine(fs, max_block=B)
        eng.set_input_retention(8)
        if group > 1:
            eng.set_block_group(group)
        chains = [eng.chain(p) for p in plist]
        h = eng.history
        buf = torch.zeros(h + nb * B, dtype=torch.complex64, device="cuda")
        o64 = np.asarray(offs, np.float64)
        mds = np.asarray([code[m] for m in modes], np.int32)
        _lib.check(_lib.lib.owrx_synth_iq(0, buf.data_ptr() + 8 * h, nb * B, 0, float(fs), len(mds),
                                          o64.ctypes.data, mds.ctypes.data, 20251114, 0.01, 0.05),
                   "owrx_synth_iq")
        torch.cuda.synchronize()
        for k in range(nb):
            eng.process_device(buf.data_ptr() + 8 * (h + k * B), B)
        eng.sync()
        st = eng.stats()
        out = ([np.frombuffer(c.read_audio(), np.int16) for c in chains], [c.read_smeter() for c in chains])
        eng.close()
        return out, st

    (a, sa) = run(1)
    monkeypatch.setenv("OWRX_FC_M", "192")
    (b, sb) = run(4)
    assert sa["ddc_frame_length"] == 128 and sb["ddc_frame_length"] == 192
    close = total = 0
    for i in range(len(plist)):
        x, y = a[0][i].astype(np.int32), b[0][i].astype(np.int32)
        assert x.size == y.size > 0, i
        close += int(np.sum(np.abs(x - y) <= 1))
        total += x.size
        assert a[1][i].size == b[1][i].size > 0, i
        assert np.allclose(a[1][i], b[1][i], rtol=1e-4, atol=1e-12), i
    assert close / total >= 0.999, close / total


def test_retention_floor_while_paired(amd):
    """Block pairing needs input retention >= 4 (owrx_set_block_pairing); lowering the retention
    below that afterwards is refused, and the paired engine keeps its retention."""
    eng = amd.Engine(2400000, max_block=1 << 16)
    eng.set_input_retention(4)
    eng.set_block_pairing(True)
    with pytest.raises(Exception):
        eng.set_input_retention(3)
    eng.set_input_retention(6)  # >= 4 stays allowed
    eng.close()
    eng = amd.Engine(2400000, max_block=1 << 16)
    eng.set_input_retention(7)
    with pytest.raises(Exception):
        eng.set_block_group(4)  # quads need retention >= 8
    eng.set_input_retention(8)
    eng.set_block_group(4)
    with pytest.raises(Exception):
        eng.set_input_retention(7)
    with pytest.raises(Exception):
        eng.set_block_group(5)
    eng.close()


def test_join_leave_join_before_first_block(amd):
    """A chain that joins and leaves before any block, then another chain that joins: the second
    one takes the first one's W slot and (from the pool) its buffers while both joins' spectra
    builds and initial-state uploads are still batched.  Its audio and s-meter equal an engine
    where only it ever existed, byte for byte."""
    import torch
    from openwebrx_amd import synth
    fs, B = 2400000, 1 << 17
    modes = ["nfm", "usb"]
    iq, offs = synth.make_iq(fs, 6 * B, modes)
    pa = amd.params.chain_params(fs, offs[0], "nfm")
    pb = amd.params.chain_params(fs, offs[1], "usb")

    def run(first):
        eng = amd.Engine(fs, max_block=B)
        if first:
            eng.chain(pa).close()
        c = eng.chain(pb)
        h = eng.history
        buf = torch.zeros(h + iq.size, dtype=torch.complex64, device="cuda")
        buf[h:] = torch.from_numpy(iq).to("cuda")
        torch.cuda.synchronize()
        for k in range(6):
            eng.process_device(buf.data_ptr() + 8 * (h + k * B), B)
        eng.sync()
        out = (c.read_audio(), c.read_smeter().tobytes())
        eng.close()
        return out

    a, b = run(False), run(True)
    assert len(a[0]) > 0 and a == b


def test_two_setbandpass_between_blocks_last_wins(amd):
    """Two setBandpass calls between blocks (a dragged passband) queue two uploads of the same
    taps buffer before the next block: the output equals an engine that got only the second."""
    import torch
    from openwebrx_amd import synth
    fs, B = 2400000, 1 << 17
    iq, offs = synth.make_iq(fs, 6 * B, ["usb"])
    p = amd.params.chain_params(fs, offs[0], "usb")

    def run(both):
        eng = amd.Engine(fs, max_block=B)
        c = eng.chain(p)
        h = eng.history
        buf = torch.zeros(h + iq.size, dtype=torch.complex64, device="cuda")
        buf[h:] = torch.from_numpy(iq).to("cuda")
        torch.cuda.synchronize()
        for k in range(6):
            if k == 3:
                if both:
                    c.set_bandpass(amd.params.f32(-0.15), amd.params.f32(0.05))
                c.set_bandpass(amd.params.f32(0.0), amd.params.f32(0.12))
            eng.process_device(buf.data_ptr() + 8 * (h + k * B), B)
        eng.sync()
        out = c.read_audio()
        eng.close()
        return out

    a, b = run(False), run(True)
    assert len(a) > 0 and a == b


def test_block_pairing_rejects_bad_state(amd):
    """Pairing needs input retention >= 4 and an engine with no chain, waterfall or block yet."""
    eng = amd.Engine(2400000, max_block=1 << 16)
    with pytest.raises(Exception):
        eng.set_block_pairing(True)  # retention 1
    eng.set_input_retention(4)
    eng.chain(amd.params.chain_params(2400000, 100000, "nfm"))
    with pytest.raises(Exception):
        eng.set_block_pairing(True)  # a chain exists
    eng.close()


def test_engine_ring_ingest_commit(amd):
    """The caller-written ring slot (owrx_ingest_buffer / owrx_commit, e.g. an RCCL broadcast)
    gives the same rows as owrx_push_iq through the ring's wraps."""
    fs, N = 2400000, 4096
    avg, hop = amd.params.fft_parameters(fs, N, 9, 0.3)
    from openwebrx_amd import synth
    n = hop * avg * 3 + N
    iq, _ = synth.make_iq(fs, n, ["nfm"])
    a, _, _ = _wf_batched(amd, iq, fs, N, hop, avg, 1 << 16, 0, 0)
    b, _, _ = _wf_batched(amd, iq, fs, N, hop, avg, 1 << 16, 0, 0, ingest=True)
    assert a.shape[0] == 3 and np.array_equal(a, b)


@pytest.mark.parametrize("variant,sizes", [("r16", 5), ("l32", 5), ("fourstep", 2)])
def test_waterfall_kernel_variants(variant, sizes):
    """The A/B waterfall kernels (OWRX_WF_KERNEL=r16: the radix-16 kernel at N = 16384 instead of
    wf_fft_q16; =l32: round 4's 512-thread radix-32 kernel; =fourstep: the four-step FFT at
    N = 32768 / 65536 instead of the DIF split onto wf_fft_l32) give the oracle's rows (<= 2e-3
    dB, as the production kernels); each runs in a child process since the selection is read
    once per process."""
    import json
    import os
    import subprocess
    import sys
    env = dict(os.environ, OWRX_WF_KERNEL=variant)
    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "wf_variant_rows.py")], env=env,
                       capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    errs = json.loads(r.stdout.strip().splitlines()[-1])
    assert len(errs) == sizes and all(e is not None and e < 2e-3 for e in errs.values()), errs


@pytest.mark.parametrize("N,fs", [(32768, 20000000), (65536, 61440000)])
def test_waterfall_fused_split_rows_bit_identical(amd, N, fs, monkeypatch):
    """N = 32768 / 65536: wf_fft_l32<true> forms the DIF split's sub-frames on load (no scratch)
    with the split kernel's operations in its order (OWRX_WF_FUSED=1, an A/B read at every launch),
    so its float and ADPCM rows are bit-identical to wf_dif_split + wf_fft_l32 (OWRX_WF_SUB=l32;
    the default transforms the sub-frames with wf_fft_q16)."""
    from openwebrx_amd import synth
    avg, hop = amd.params.fft_parameters(fs, N, 9, 0.3)
    avg = min(avg, 8)
    n = hop * avg * 4 + N + 1000
    iq, _ = synth.make_iq(fs, n, ["nfm", "am", "usb"])
    rows = {}
    monkeypatch.setenv("OWRX_WF_SUB", "l32")
    for fused in ("1", "0"):
        monkeypatch.setenv("OWRX_WF_FUSED", fused)
        rows[fused] = (_wf(amd, iq, fs, N, hop, avg, False, 1 << 17),
                       _wf(amd, iq, fs, N, hop, avg, True, 1 << 18))
    assert rows["1"][0].shape[0] >= 3 and rows["1"][0].shape == rows["0"][0].shape
    assert np.array_equal(rows["1"][0], rows["0"][0])
    assert rows["1"][1] == rows["0"][1] if isinstance(rows["1"][1], bytes) else np.array_equal(rows["1"][1], rows["0"][1])


def test_wide_serial_streams_same_audio():
    """Past OWRX_WIDE_SERIAL_CHAINS chains the serial kernels move from the CU-masked streams to
    unmasked ones (engine.hip process_block); a stream whose chain count crosses the threshold
    up and down (3 -> 8 -> 3 chains, threshold 4) gives every chain the same audio and s-meter
    bytes as with the masked streams only (threshold out of reach)."""
    import json
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    res = []
    for thr in ("1000000000", "4"):
        env = dict(os.environ, OWRX_WIDE_SERIAL_CHAINS=thr)
        r = subprocess.run([sys.executable, os.path.join(here, "serial_wide_run.py")], env=env,
                           capture_output=True, text=True, timeout=110)
        assert r.returncode == 0, r.stderr[-2000:]
        res.append(json.loads(r.stdout.strip().splitlines()[-1]))
    assert len(res[0]) == 8 and all(v[2] > 1000 for v in res[0].values()), res[0]
    assert res[0] == res[1]


def test_waterfall_adpcm_rows_and_block_invariance(amd):
    fs, N = 2400000, 4096
    avg, hop = amd.params.fft_parameters(fs, N, 9, 0.3)
    from openwebrx_amd import synth
    n = hop * avg * 2 + N
    iq, _ = synth.make_iq(fs, n, ["nfm"])
    a = _wf(amd, iq, fs, N, hop, avg, True, 1 << 16)
    b = _wf(amd, iq, fs, N, hop, avg, True, 99991)  # ragged blocks: rows identical bit for bit
    assert a.shape == (2, (N + 10) // 2)
    assert np.array_equal(a, b)
    ref_db = [oracle.fftswap(r) for r in oracle.waterfall_rows(iq, N, hop, avg)]
    for row_bytes, rdb in zip(a, ref_db):
        dec = oracle.adpcm_decode(row_bytes.tobytes())[10:]
        enc_ref = oracle.adpcm_decode(oracle.fft_adpcm_row(rdb))[10:]
        diff = np.abs(dec.astype(np.int32) - enc_ref)
        assert np.mean(diff == 0) > 0.95, np.mean(diff == 0)


# ---------------------------------------------------------------------------------------------
# client chains
# ---------------------------------------------------------------------------------------------
def _run_chains(amd, iq, fs, plist, block, debug=True, ddc_mode=None):
    eng = amd.Engine(fs, max_block=block)
    if debug:
        eng.set_debug(True)
    if ddc_mode:
        eng.set_ddc_mode(ddc_mode)
    chains = [eng.chain(p) for p in plist]
    i = 0
    sizes = [block, block // 3 + 17, block // 2 + 1]
    k = 0
    while i < iq.size:
        s = sizes[k % 3]
        eng.push(iq[i:i + s])
        i += s
        k += 1
    eng.sync()
    return eng, chains


def test_nfm_chain_10msps_stages(amd):
    """C2-style chain: 10 Msps, D=833, 22223 taps, fractional decimator, NFM bandpass."""
    from openwebrx_amd import synth
    fs = 10000000
    n = 3 * (1 << 20)
    iq, offs = synth.make_iq(fs, n, ["nfm", "am", "nfm", "usb"])
    p = amd.params.chain_params(fs, offs[2], "nfm", output=amd._lib.OUT_S16)
    eng, (ch,) = _run_chains(amd, iq, fs, [p], 1 << 20)
    ref = oracle.stages(iq, p)
    ddc = ch.read_debug(0)
    assert ddc.size == ref["ddc"].size, (ddc.size, ref["ddc"].size)
    assert rel_rms(ddc, ref["ddc"]) < 1e-5
    fd = ch.read_debug(1)
    assert abs(fd.size - ref["frac"].size) <= 1
    assert rel_rms(fd, ref["frac"]) < 1e-5
    bp = ch.read_debug(2)
    assert rel_rms(bp, ref["bandpass"]) < 1e-5
    dem = ch.read_debug(4)
    assert dem.size == ref["demod"].size
    assert rel_rms(dem, ref["demod"]) < 1e-5
    s16 = np.frombuffer(ch.read_audio(), np.int16)
    d = np.abs(s16.astype(np.int32) - ref["s16"][:s16.size])
    assert s16.size == ref["s16"].size
    assert np.mean(d <= 1) > 0.999, np.mean(d <= 1)
    sm = ch.read_smeter()
    assert sm.size == ref["smeter"].size
    assert rel_rms(sm, ref["smeter"]) < 1e-5
    eng.close()


@pytest.mark.parametrize("mode", ["am", "usb", "cw", "lsb"])
def test_modes_2400k_grouped(amd, mode):
    """Several chains share one DDC launch (same FirDecimate design) at 2.4 Msps."""
    from openwebrx_amd import synth
    fs = 2400000
    modes = [mode, "nfm", mode, "am", mode]
    n = 1 << 20
    iq, offs = synth.make_iq(fs, n, modes)
    plist = [amd.params.chain_params(fs, o, m, output=amd._lib.OUT_S16) for o, m in zip(offs, modes)]
    eng, chains = _run_chains(amd, iq, fs, plist, 1 << 18)
    for p, ch in zip(plist, chains):
        ref = oracle.stages(iq, p)
        assert rel_rms(ch.read_debug(0), ref["ddc"]) < 1e-5
        s16 = np.frombuffer(ch.read_audio(), np.int16)
        assert s16.size == ref["s16"].size
        d = np.abs(s16.astype(np.int32) - ref["s16"])
        assert np.mean(d <= 1) > 0.999, (p.demod, np.mean(d <= 1), np.max(d))
    eng.close()


@pytest.mark.parametrize("nch", [32, 40, 65])
def test_ddc_large_groups(amd, nch):
    """Groups of 32+ chains run the LDS-staged DDC kernel (two tiles per wave at 32 chains, one
    at 33-64, two chain groups per launch at 65): DDC stage of sampled chains vs the oracle,
    and their int16 audio within +-1 LSB."""
    from openwebrx_amd import synth
    fs = 2400000
    modes = [("nfm", "am", "usb", "cw")[c % 4] for c in range(nch)]
    n = 1 << 19
    iq, offs = synth.make_iq(fs, n, modes)
    plist = [amd.params.chain_params(fs, o, m, output=amd._lib.OUT_S16)
             for o, m in zip(offs, modes)]
    eng, chains = _run_chains(amd, iq, fs, plist, 1 << 17)
    for c in sorted({0, nch // 2, nch - 1}):
        ref = oracle.stages(iq, plist[c])
        ddc = chains[c].read_debug(0)
        assert ddc.size == ref["ddc"].size, (c, ddc.size, ref["ddc"].size)
        assert rel_rms(ddc, ref["ddc"]) < 1e-5, c
        s16 = np.frombuffer(chains[c].read_audio(), np.int16)
        assert s16.size == ref["s16"].size
        d = np.abs(s16.astype(np.int32) - ref["s16"])
        assert np.mean(d <= 1) > 0.999, (c, np.mean(d <= 1))
    eng.close()


@pytest.mark.parametrize("fs,bw", [(2400000, 48000), (10000000, 250000)])
def test_service_resampler_iq(amd, fs, bw):
    """Service Resampler (owrx/source/resampler.py:11-26): Shift + FirDecimate to a band, the cf32
    IF is the product (OWRX_OUT_IQ), next to a client chain on the same engine."""
    from openwebrx_amd import synth
    n = 1 << 20
    iq, offs = synth.make_iq(fs, n, ["nfm", "usb", "am"])
    sdr_cf = 145000000
    p, if_rate = amd.params.resampler_params(fs, sdr_cf, sdr_cf + offs[1] + 3000, bw)
    assert p.decimation == int(fs / bw) and abs(if_rate - fs / p.decimation) < 1e-6
    audio = amd.params.chain_params(fs, offs[0], "nfm", output=amd._lib.OUT_S16)
    eng, (rs, ch) = _run_chains(amd, iq, fs, [p, audio], 1 << 18, debug=False)
    got = np.frombuffer(rs.read_audio(), np.complex64)
    c = oracle.chain_from_engine_params(p)
    ref = oracle.fir_decimate(oracle.shift(iq, p.shift_rate), c._keep[0], p.decimation)
    assert got.size == ref.size, (got.size, ref.size)
    assert rel_rms(got, ref) < 1e-5
    s16 = np.frombuffer(ch.read_audio(), np.int16)
    ref_a = oracle.stages(iq, audio)["s16"]
    assert s16.size == ref_a.size
    assert np.mean(np.abs(s16.astype(np.int32) - ref_a) <= 1) > 0.999
    eng.close()


def test_adpcm_chain_output_decodes(amd):
    """AdpcmEncoder(sync=True) stream: SYNC frames every 1001 data bytes, decodable."""
    from openwebrx_amd import synth
    fs = 2400000
    iq, offs = synth.make_iq(fs, 1 << 20, ["nfm"])
    p = amd.params.chain_params(fs, offs[0], "nfm", output=amd._lib.OUT_ADPCM)
    eng, (ch,) = _run_chains(amd, iq, fs, [p], 1 << 18)
    data = ch.read_audio()
    agc = ch.read_debug(5)
    ref_bytes = oracle.adpcm_encode(oracle.convert_s16(agc), 1)
    assert data == ref_bytes[:len(data)] and len(ref_bytes) - len(data) <= 9
    eng.close()


def test_adpcm_chains_many_lanes_ragged_blocks(amd):
    """chain_adpcm across two workgroups (70 chains, mixed modes and so different audio
    lengths per block), blocks of ragged sizes (odd sample counts: bytes spanning blocks) and
    ~12 SYNC frames per chain: every chain's AdpcmEncoder(sync=True) bytes equal the oracle's
    encoding of its own AGC output (debug tap 5)."""
    from openwebrx_amd import synth
    fs = 2400000
    modes = [("nfm", "am", "usb", "cw", "lsb")[c % 5] for c in range(70)]
    n = 5 << 20
    iq, offs = synth.make_iq(fs, n, modes)
    plist = [amd.params.chain_params(fs, o, m, output=amd._lib.OUT_ADPCM)
             for o, m in zip(offs, modes)]
    eng, chains = _run_chains(amd, iq, fs, plist, 1 << 18)
    for c, ch in enumerate(chains):
        data = ch.read_audio()
        agc = ch.read_debug(5)
        ref = oracle.adpcm_encode(oracle.convert_s16(agc), 1)
        assert len(data) > 10000 and data == ref[:len(data)] and len(ref) - len(data) <= 9, c
    eng.close()


def test_adpcm_chains_staggered_sync_frames(amd):
    """Clients join a live server at different blocks, so the AdpcmEncoder byte counters -- and
    the places of the SYNC frames -- differ between the lanes of one chain_adpcm wave (frames on
    the encoder's group path, round 6): 70 chains created in seven batches, ragged blocks pushed
    between the batches; every chain's bytes equal the oracle's encoding of its own AGC output,
    and the batches' frame phases do differ."""
    from openwebrx_amd import synth
    fs, block = 2400000, 1 << 17
    modes = [("nfm", "am", "usb", "cw", "lsb")[c % 5] for c in range(70)]
    iq, offs = synth.make_iq(fs, 6 << 20, modes)
    plist = [amd.params.chain_params(fs, o, m, output=amd._lib.OUT_ADPCM)
             for o, m in zip(offs, modes)]
    eng = amd.Engine(fs, max_block=block)
    eng.set_debug(True)
    sizes = [block, block // 3 + 17, block // 2 + 1]
    chains, i, k = [], 0, 0

    def push():
        nonlocal i, k
        s = sizes[k % 3]
        eng.push(iq[i:i + s])
        i += s
        k += 1
    for b in range(7):
        chains += [eng.chain(p) for p in plist[10 * b:10 * (b + 1)]]
        for _ in range(1 + b % 3):
            push()
    while i < iq.size:
        push()
    eng.sync()
    starts = set()
    for c, ch in enumerate(chains):
        data = ch.read_audio()
        ref = oracle.adpcm_encode(oracle.convert_s16(ch.read_debug(5)), 1)
        assert len(data) > 10000 and data == ref[:len(data)] and len(ref) - len(data) <= 9, c
        starts.add(len(data) % 1009)  # byte counters of the batches at the end of the stream
    eng.close()
    assert len(starts) >= 5  # the batches' frame phases differ


@pytest.mark.parametrize("rates", [(48000, 12000), (12000, 48000), (24000, 12000)])
def test_audio_resampler_module(amd, rates):
    """AudioResampler(inputRate, clientRate) (csdr/chain/clientaudio.py:15-16), the standalone
    GPU module, fed in ragged pieces (history carried between calls): <=1e-5 rel-RMS against
    the oracle's float64 restatement of the same rational L/M design."""
    fin, fout = rates
    rng = np.random.default_rng(7)
    n = 40000
    t = np.arange(n) / fin
    x = (0.5 * np.sin(2 * np.pi * 700 * t) + 0.2 * np.sin(2 * np.pi * 2100 * t + 1)
         + 0.01 * rng.standard_normal(n)).astype(np.float32)
    mod = amd.Module(amd._lib.MOD_AUDIO_RESAMPLER, fin, fout)
    got = []
    i = 0
    for s in [1000, 3333, 12345, 7, 9000] * 4:
        if i >= n:
            break
        got.append(np.frombuffer(mod.process(x[i:i + s], 4 * (s * fout // fin + 64)),
                                 np.float32))
        i += s
    got = np.concatenate(got)
    ref = oracle.audio_resample(x[:i], fin, fout)
    assert got.size == ref.size, (got.size, ref.size)
    assert rel_rms(got, ref) < 1e-5, rel_rms(got, ref)
    mod.close()


@pytest.mark.parametrize("U,S", [(10, 4), (50, 8)])
def test_afc_module(amd, U, S):
    """Afc(updatePeriod, samplePeriod) of SAm (10, 4) and RawSAm (50, 8)
    (csdr/chain/analog.py:141-167), the standalone GPU module fed in ragged pieces (phase,
    frequency and the pair accumulator carried between calls): <=1e-5 rel-RMS against the
    oracle's restatement (parity unpinned: csdr's Afc is not in the reference).  A carrier
    150 Hz off at 12 kHz is pulled to DC: the last quarter of the output has a nearly
    constant phase."""
    rng = np.random.default_rng(11)
    n = 24000
    t = np.arange(n) / 12000.0
    env = 0.3 * (1 + 0.5 * np.sin(2 * np.pi * 800 * t))
    x = (env * np.exp(2j * np.pi * 150.0 * t + 0.7j)
         + 0.003 * (rng.standard_normal(n) + 1j * rng.standard_normal(n))).astype(np.complex64)
    mod = amd.Module(amd._lib.MOD_AFC, U, S)
    got, i = [], 0
    for s in [1000, 3333, 7, 4097, 9000, 1, 6000]:
        got.append(np.frombuffer(mod.process(x[i:i + s], 8 * s), np.complex64))
        i += s
    with pytest.raises(Exception):  # output capacity below 8 bytes per sample: OWRX_ENOSPC
        mod.process(x[i:i + 100], 8 * 99)
    mod.close()
    got = np.concatenate(got)
    ref = oracle.afc(x[:i], U, S)
    assert got.size == ref.size == i
    assert rel_rms(got, ref) < 1e-5, rel_rms(got, ref)
    tail = ref[3 * i // 4:]
    assert np.std(np.diff(np.unwrap(np.angle(tail)))) < 0.05


@pytest.mark.parametrize("N,fs", [(4096, 2400000), (16384, 10000000), (65536, 61440000)])
def test_waterfall_adpcm_rows_bit_exact(amd, N, fs):
    """The row-parallel speculative IMA-ADPCM encoder is bit-identical to the sequential
    FftAdpcm restatement: two FftChains on one engine (float and ADPCM output) see the same
    dB rows, and the ADPCM bytes equal oracle.fft_adpcm_row() of the float rows."""
    from openwebrx_amd import synth
    avg, hop = amd.params.fft_parameters(fs, N, 9, 0.3)
    avg = min(avg, 8)
    n = hop * avg * 5 + N
    iq, _ = synth.make_iq(fs, n, ["nfm", "am", "usb", "cw"])
    eng = amd.Engine(fs, max_block=1 << 18)
    wf_f = eng.waterfall(N, hop, avg, adpcm=False)
    wf_a = eng.waterfall(N, hop, avg, adpcm=True)
    for i in range(0, n, 1 << 18):
        eng.push(iq[i:i + (1 << 18)])
    eng.sync()
    rf = wf_f.read_rows()
    ra = wf_a.read_rows()
    assert rf.shape[0] == ra.shape[0] == 5
    for r in range(rf.shape[0]):
        assert ra[r].tobytes() == oracle.fft_adpcm_row(rf[r])
    eng.close()


@pytest.mark.parametrize("fs,modes,block", [
    (2400000, ["nfm"], 1 << 18),                                    # C1: D=200, 5333 taps
    (10000000, ["nfm", "am"] * 16, 1 << 20),                        # C2: D=833, 22223 taps
    (10000000, ["nfm", "usb", "cw", "am", "lsb"] * 8 + ["nfm"], 1 << 19),  # 41: ragged tiles
    (61440000, ["nfm", "usb", "am", "cw"] * 3, 1 << 21),            # C4: D=5120, 136533 taps
])
def test_ddc_fast_convolution_equals_direct(amd, fs, modes, block):
    """The fast-convolution DDC (kernels_fcddc.hip: branch DFTs, one f32-MFMA complex GEMM per
    bin, inverse DFT + exact rotator) against the direct polyphase FIR on the same input, and both
    against the oracle for sampled chains; blocks of ragged sizes (frames cut at block ends)."""
    from openwebrx_amd import synth
    n = 3 * block + 12345
    iq, offs = synth.make_iq(fs, n, modes)
    plist = [amd.params.chain_params(fs, o, m, output=amd._lib.OUT_S16)
             for o, m in zip(offs, modes)]
    eng_f, ch_f = _run_chains(amd, iq, fs, plist, block, ddc_mode="fast")
    eng_d, ch_d = _run_chains(amd, iq, fs, plist, block, ddc_mode="direct")
    assert eng_f.stats()["ddc_fast_launches"] == eng_f.stats()["ddc_launches"] > 0
    assert eng_d.stats()["ddc_fast_launches"] == 0
    fast = [ch.read_debug(0) for ch in ch_f]
    for c in range(len(plist)):
        a = fast[c]
        b = ch_d[c].read_debug(0)
        assert a.size == b.size > 0, (c, a.size, b.size)
        assert rel_rms(a, b) < 1e-5, (c, rel_rms(a, b))
    for c in sorted({0, len(plist) // 2, len(plist) - 1}):
        ref = oracle.stages(iq, plist[c])
        got = fast[c]
        assert got.size == ref["ddc"].size
        assert rel_rms(got, ref["ddc"]) < 1e-5, (c, rel_rms(got, ref["ddc"]))
    eng_f.close()
    eng_d.close()


@pytest.mark.parametrize("m", [64, 128, 192, 256, 384])
def test_ddc_fast_convolution_frame_lengths(amd, m, monkeypatch):
    """Every frame length the engine can pick -- powers of two and the radix-3 ones (192 = 3 x
    64, 384 = 3 x 128: a radix-3 pass then sub-row FFTs) -- forced on the C2 design (D = 833,
    22223 taps), ragged blocks: the DDC of sampled chains <= 1e-5 rel-RMS vs the oracle."""
    from openwebrx_amd import synth
    monkeypatch.setenv("OWRX_FC_M", str(m))
    fs = 10000000
    modes = ["nfm", "usb", "am", "cw"] * 5
    block = 1 << 19
    n = 2 * block + 54321
    iq, offs = synth.make_iq(fs, n, modes)
    plist = [amd.params.chain_params(fs, o, m_, output=amd._lib.OUT_S16)
             for o, m_ in zip(offs, modes)]
    eng, chains = _run_chains(amd, iq, fs, plist, block, ddc_mode="fast")
    assert eng.stats()["ddc_fast_launches"] == eng.stats()["ddc_launches"] > 0
    for c in (0, 7, 19):
        ref = oracle.stages(iq, plist[c])
        got = chains[c].read_debug(0)
        assert got.size == ref["ddc"].size, (c, got.size, ref["ddc"].size)
        assert rel_rms(got, ref["ddc"]) < 1e-5, (m, c, rel_rms(got, ref["ddc"]))
    eng.close()


def test_ddc_group_size_changes_rounding_only(amd):
    """The fast DDC splits K over workgroups when its tile grid would leave CUs idle
    (kernels_fcddc.hip fc_kslices), and the slice count follows the group's chain count: a
    chain alone gets K slices, the same chain among 200 none.  The slices are summed in a fixed
    order, so each output is deterministic for a given group size; across group sizes the
    association differs, i.e. a chain's DDC output may change at the rounding level when other
    clients join or leave (include/owrx_amd.h owrx_chain_create).  Pinned here: the same chain
    alone and in a 200-chain group agree to 1e-6 rel-RMS, both <= 1e-5 vs the oracle."""
    from openwebrx_amd import synth
    fs = 10000000
    modes = ["nfm", "usb", "am", "cw"] * 50
    n = 2 * (1 << 20)
    iq, offs = synth.make_iq(fs, n, modes)
    plist = [amd.params.chain_params(fs, o, m, output=amd._lib.OUT_S16) for o, m in zip(offs, modes)]
    eng1, (a,) = _run_chains(amd, iq, fs, plist[:1], 1 << 20, ddc_mode="fast")
    eng2, many = _run_chains(amd, iq, fs, plist, 1 << 20, ddc_mode="fast")
    ks1, ks2 = eng1.stats()["ddc_mac_kslices_max"], eng2.stats()["ddc_mac_kslices_max"]
    x, y = a.read_debug(0), many[0].read_debug(0)
    ref = oracle.stages(iq, plist[0])["ddc"]
    eng1.close()
    eng2.close()
    assert ks1 > ks2 >= 0, (ks1, ks2)  # the two group sizes do take different slice counts
    assert x.size == y.size == ref.size > 0
    assert rel_rms(x, y) < 1e-6, rel_rms(x, y)
    assert rel_rms(x, ref) < 1e-5 and rel_rms(y, ref) < 1e-5


def test_ddc_fast_convolution_membership_churn(amd):
    """Chains leaving a fast-convolution group mid-stream: the last member takes the freed slot
    of the group's filter-spectra matrix (swap-remove); the surviving chains' DDC output over the
    whole stream still equals the oracle's."""
    from openwebrx_amd import synth
    fs = 2400000
    modes = [("nfm", "am", "usb", "cw")[c % 4] for c in range(40)]
    n = 1 << 20
    iq, offs = synth.make_iq(fs, n, modes)
    plist = [amd.params.chain_params(fs, o, m, output=amd._lib.OUT_S16)
             for o, m in zip(offs, modes)]
    eng = amd.Engine(fs, max_block=1 << 17)
    eng.set_debug(True)
    chains = [eng.chain(p) for p in plist]
    blk = 1 << 17
    for i in range(0, n, blk):
        if i == 3 * blk:
            chains[3].close()
            chains[17].close()
        eng.push(iq[i:i + blk])
    eng.sync()
    for c in (0, 16, 18, 38, 39):
        ref = oracle.stages(iq, plist[c])
        got = chains[c].read_debug(0)
        assert got.size == ref["ddc"].size, (c, got.size, ref["ddc"].size)
        assert rel_rms(got, ref["ddc"]) < 1e-5, (c, rel_rms(got, ref["ddc"]))
    eng.close()


def test_retune_after_swap_remove(amd):
    """A chain that swap-remove moved into a freed slot of its group's filter-spectra matrix,
    then retuned (Shift.setRate): its spectra are rebuilt at that slot (fc_build_w after the
    move), and its DDC output follows the piecewise phase like test_retune_is_phase_continuous."""
    from openwebrx_amd import synth
    fs, B = 2400000, 1 << 17
    modes = [("nfm", "usb")[c % 2] for c in range(8)]
    iq, offs = synth.make_iq(fs, 6 * B, modes)
    plist = [amd.params.chain_params(fs, o, m, output=amd._lib.OUT_S16) for o, m in zip(offs, modes)]
    eng = amd.Engine(fs, max_block=B)
    eng.set_debug(True)
    chains = [eng.chain(p) for p in plist]
    eng.push(iq[:2 * B])
    chains[2].close()  # chain 7 (the last member) moves into slot 2
    eng.push(iq[2 * B:3 * B])
    new_rate = amd.params.f32(amd.params.shift_rate(offs[1] + 2500.0, fs))
    chains[7].set_shift_rate(new_rate)
    eng.push(iq[3 * B:])
    eng.sync()
    p = plist[7]
    got = chains[7].read_debug(0)
    c = oracle.chain_from_engine_params(p)
    T, D = c.ntaps, p.decimation
    nb = ((3 * B - T) // D + 1) * D  # first input sample of the first output after the retune
    n = np.arange(iq.size, dtype=np.uint64)
    f0, f1 = np.uint64(_rate_fx(p.shift_rate)), np.uint64(_rate_fx(new_rate))
    with np.errstate(over="ignore"):
        ph = np.where(n < nb, (n + np.uint64(1)) * f0,
                      np.uint64(nb) * f0 + (n - np.uint64(nb) + np.uint64(1)) * f1)
    turns = ph.astype(np.float64) / 18446744073709551616.0
    x = (iq.astype(np.complex128) * np.exp(2j * np.pi * turns)).astype(np.complex64)
    ref = oracle.fir_decimate(x, c._keep[0], D)
    k = nb // D
    old = oracle.fir_decimate(oracle.shift(iq, p.shift_rate), c._keep[0], D)
    assert got.size == ref.size, (got.size, ref.size)
    assert rel_rms(got[:k], old[:k]) < 1e-5
    assert rel_rms(got[k:], ref[k:]) < 1e-5
    for i in (0, 1, 3, 6):  # the other members are untouched
        r = oracle.stages(iq, plist[i])["ddc"]
        g = chains[i].read_debug(0)
        assert g.size == r.size and rel_rms(g, r) < 1e-5, i
    eng.close()


def _check_sampled_chains(iq, plist, chains, sample):
    for c in sample:
        ref = oracle.stages(iq, plist[c])
        ddc = chains[c].read_debug(0)
        assert ddc.size == ref["ddc"].size, (c, ddc.size, ref["ddc"].size)
        assert rel_rms(ddc, ref["ddc"]) < 1e-5, c
        s16 = np.frombuffer(chains[c].read_audio(), np.int16)
        assert s16.size == ref["s16"].size, (c, s16.size, ref["s16"].size)
        d = np.abs(s16.astype(np.int32) - ref["s16"])
        assert np.mean(d <= 1) > 0.999, (c, np.mean(d <= 1))


def test_sam_rawam_256_chains_one_engine(amd):
    """256 SAm / RawAm / RawSAm chains in one engine (csdr/chain/analog.py:23-31, 141-167):
    Afc in chain_afc (lane per chain), DcBlock -> Agc(Slow, 200) or Gain(100) in the serial
    front, the Raw* Selectors at the 48 kHz hd rate (D = 50 at 2.4 Msps) next to SAm's 12 kHz
    (D = 200).  Sampled chains of every mode vs the oracle: DDC and Selector output <= 1e-5
    rel-RMS; the int16 audio within 1 LSB on 99.9 % of the oracle's tail (Afc -> RealPart ->
    DcBlock -> Agc / Gain, or AmDemod -> DcBlock -> Gain) run on the engine's own Selector
    output -- the Afc's frequency loop turns a 1e-7 input difference into a slowly drifting
    phase, so end to end from the IQ only RawAm is held to that bar; every chain's audio length
    as the oracle's."""
    from openwebrx_amd import synth
    fs = 2400000
    kinds = ("sam", "rawam", "rawsam")
    C = 256
    modes = [kinds[c % 3] for c in range(C)]
    offs = synth.carrier_offsets(fs, C)
    n = 1 << 20
    iq, _ = synth.make_iq(fs, n, ["am"] * 24)  # AM carriers spread over the band
    plist = [amd.params.chain_params(fs, o, m, output=amd._lib.OUT_S16) for o, m in zip(offs, modes)]
    eng, chains = _run_chains(amd, iq, fs, plist, 1 << 17)
    for c in (0, 1, 2, 127, 128, 129, 253, 254, 255):
        ref = oracle.stages(iq, plist[c])
        ddc = chains[c].read_debug(0)
        assert ddc.size == ref["ddc"].size and rel_rms(ddc, ref["ddc"]) < 1e-5, (c, modes[c])
        sq = chains[c].read_debug(3)
        assert sq.size == ref["squelch"].size and rel_rms(sq, ref["squelch"]) < 1e-5, c
        p = plist[c]
        if p.demod == amd._lib.DEMOD_SAM:
            dem = oracle.dcblock(oracle.realpart(oracle.afc(sq, p.afc_update, p.afc_sample)))
        else:
            dem = oracle.dcblock(oracle.amdemod(sq))
        ag = (oracle.gain(dem, p.audio_gain) if p.audio_gain > 0 else
              oracle.agc(dem, oracle.agc_params(p.agc_profile, p.agc_initial_gain)))
        want = oracle.convert_s16(ag)
        s16 = np.frombuffer(chains[c].read_audio(), np.int16)
        assert s16.size == ref["s16"].size == want.size, (c, modes[c], s16.size, ref["s16"].size)
        d = np.abs(s16.astype(np.int32) - want)
        assert np.mean(d <= 1) > 0.999, (c, modes[c], np.mean(d <= 1), np.max(d))
        if modes[c] == "rawam":  # no Afc: end to end from the IQ as well
            d = np.abs(s16.astype(np.int32) - ref["s16"])
            assert np.mean(d <= 1) > 0.999, (c, modes[c], np.mean(d <= 1), np.max(d))
    # the rest: as much audio as the oracle's chain of the same shape produces
    sizes = {m: oracle.stages(iq, plist[kinds.index(m)])["s16"].size for m in kinds}
    for c in range(C):
        if c in (0, 1, 2, 127, 128, 129, 253, 254, 255):
            continue
        assert len(chains[c].read_audio()) == 2 * sizes[modes[c]], (c, modes[c])
    eng.close()


def test_c3_256_mixed_chains_10msps(amd):
    """BASELINE config 3 shape: 10 Msps, 256 chains (86 NFM + 85 USB + 85 CW), one
    (D=833, 22223-tap) design in one DDC group; sampled chains vs the oracle."""
    from openwebrx_amd import synth
    fs = 10000000
    modes = ["nfm"] * 86 + ["usb"] * 85 + ["cw"] * 85
    n = 1 << 20
    iq, offs = synth.make_iq(fs, n, modes)
    plist = [amd.params.chain_params(fs, o, m, output=amd._lib.OUT_S16)
             for o, m in zip(offs, modes)]
    eng, chains = _run_chains(amd, iq, fs, plist, 1 << 19)
    _check_sampled_chains(iq, plist, chains, [0, 100, 255])
    eng.close()


def test_batched_chain_reads_equal_per_chain_reads(amd):
    """owrx_chains_read_audio / owrx_chains_read_smeter (one native call for all chains) return,
    per chain, exactly what the per-chain reads return on an identical engine."""
    from openwebrx_amd import synth
    fs = 2400000
    modes = ["nfm", "am", "usb", "cw", "nfm", "am"]
    iq, offs = synth.make_iq(fs, 1 << 21, modes)  # 14 squelch blocks: 3 s-meter reports
    plist = [amd.params.chain_params(fs, o, m, output=amd._lib.OUT_ADPCM if i % 2 else amd._lib.OUT_S16)
             for i, (o, m) in enumerate(zip(offs, modes))]
    e1, c1 = _run_chains(amd, iq, fs, plist, 1 << 17, debug=False)
    e2, c2 = _run_chains(amd, iq, fs, plist, 1 << 17, debug=False)
    audio, alens, sm, scounts = e2.read_chains(c2)
    assert alens.sum() == audio.size > 0 and scounts.sum() == sm.size > 0
    ao = np.concatenate([[0], np.cumsum(alens)])
    so = np.concatenate([[0], np.cumsum(scounts)])
    for i, ch in enumerate(c1):
        assert ch.read_audio() == audio[ao[i]:ao[i + 1]].tobytes(), i
        assert np.array_equal(ch.read_smeter(), sm[so[i]:so[i + 1]]), i
    audio, sm, alens, scounts = audio.copy(), sm.copy(), alens.copy(), scounts.copy()
    again, alens2, _, _ = e2.read_chains(c2)
    assert again.size == 0 and not alens2.any()
    # capped reads: the chains in order until the cap, the rest stays in the rings for the next
    # (uncapped: size query + one read) call; each chain's pieces put together equal one read
    e3, c3 = _run_chains(amd, iq, fs, plist, 1 << 17, debug=False)
    a3, al3, sm3, sc3 = (x.copy() for x in e3.read_chains(c3, max_bytes=1000, max_values=5))
    assert al3.sum() == a3.size == 1000 and sc3.sum() == sm3.size == 5
    assert a3.tobytes() == audio[:1000].tobytes() and np.array_equal(sm3, sm[:5])
    a4, al4, sm4, sc4 = e3.read_chains(c3)
    assert np.array_equal(al3 + al4, alens) and np.array_equal(sc3 + sc4, scounts)
    o3, o4 = np.concatenate([[0], np.cumsum(al3)]), np.concatenate([[0], np.cumsum(al4)])
    for i in range(len(c3)):
        assert (a3[o3[i]:o3[i + 1]].tobytes() + a4[o4[i]:o4[i + 1]].tobytes()
                == audio[ao[i]:ao[i + 1]].tobytes()), i
    q3, q4 = np.concatenate([[0], np.cumsum(sc3)]), np.concatenate([[0], np.cumsum(sc4)])
    for i in range(len(c3)):
        assert np.array_equal(np.concatenate([sm3[q3[i]:q3[i + 1]], sm4[q4[i]:q4[i + 1]]]),
                              sm[so[i]:so[i + 1]]), i
    e1.close()
    e2.close()
    e3.close()


def test_c4_chains_61msps(amd):
    """BASELINE config 4 chain design at 61.44 Msps: D=5120, 136533 taps, no fractional
    decimator (61.44 MHz / 5120 = 12 kHz exactly); DDC and audio vs the oracle."""
    from openwebrx_amd import synth
    fs = 61440000
    modes = ["nfm", "usb", "am"]
    n = 1 << 23  # 1612 outputs per chain: two 750-sample squelch blocks of audio
    iq, offs = synth.make_iq(fs, n, modes)
    plist = [amd.params.chain_params(fs, o, m, output=amd._lib.OUT_S16)
             for o, m in zip(offs, modes)]
    assert plist[0].decimation == 5120 and plist[0].frac_rate == 1.0
    eng, chains = _run_chains(amd, iq, fs, plist, 1 << 19)
    _check_sampled_chains(iq, plist, chains, range(3))
    eng.close()


@pytest.mark.parametrize("avg", [1, 3])
def test_secondary_fft_rows(amd, avg):
    """Secondary FFT (owrx/dsp.py:220-225): FftChain(12000, 2048, ...) on the Selector output.
    Float rows vs the oracle's waterfall of the chain's own squelch output (debug tap 3), and the
    ADPCM rows of an identical chain bit-exact against oracle.fft_adpcm_row of those rows."""
    from openwebrx_amd import synth
    fs, N = 2400000, 2048
    a0, hop = amd.params.fft_parameters(12000, N, 9, 0.3)
    assert (a0, hop) == (1, 1333)  # the reference's digimodes defaults
    if avg != 1:
        hop = 444
    iq, offs = synth.make_iq(fs, (1 << 21) + 12345, ["usb"])
    p = amd.params.chain_params(fs, offs[0], "usb", output=amd._lib.OUT_S16)
    eng = amd.Engine(fs, max_block=1 << 18)
    eng.set_debug(True)
    cf, ca = eng.chain(p), eng.chain(p)
    cf.set_secondary_fft(N, hop, avg, -70.0, adpcm=False)
    ca.set_secondary_fft(N, hop, avg, -70.0, adpcm=True)
    for i, s in enumerate(range(0, iq.size, 77777)):
        eng.push(iq[s:s + 77777])
    eng.sync()
    rows = cf.read_secondary_fft()
    rows_a = ca.read_secondary_fft()
    sq = cf.read_debug(3)
    ref = np.stack([oracle.fftswap(r) for r in oracle.waterfall_rows(sq, N, hop, avg)])
    assert rows.shape[0] >= 5 and rows.shape == ref.shape, (rows.shape, ref.shape)
    # the Selector output is band-limited (USB 150..3000 Hz of 12 kHz): stop-band bins sit
    # ~80 dB under the peak, where fp32 FFT rounding (relative to the row's energy) shows in dB.
    # Bar: linear power rel-RMS <= 1e-5 per row, and <= 2e-3 dB on bins within 50 dB of the peak
    for g, r in zip(rows, ref):
        assert rel_rms(10.0 ** (g / 10.0), 10.0 ** (r / 10.0)) < 1e-5
        strong = r > r.max() - 50.0
        assert np.max(np.abs(g - r)[strong]) < 2e-3
    assert rows_a.shape == (rows.shape[0], (N + 10) // 2)
    for r in range(rows.shape[0]):
        assert rows_a[r].tobytes() == oracle.fft_adpcm_row(rows[r])
    # removing it stops the rows; the audio is untouched by the tap
    ca.set_secondary_fft(0)
    eng.push(iq[:1 << 18])
    eng.sync()
    assert cf.read_audio() == ca.read_audio()
    eng.close()


@pytest.mark.parametrize("fs", [2400000, 10000000])
def test_wfm_chain(amd, fs):
    """WFM: Selector at 250 kHz with the 3125-tap bandpass (bp_long kernel),
    15625-sample squelch blocks, FmDemod + Limit, FractionalDecimator(FLOAT, 250000/48000,
    prefilter) and WfmDeemphasis (no AGC) to 48 kHz HD audio; stages vs the oracle, next to an
    NFM chain on the same engine."""
    from openwebrx_amd import synth
    n = (1 << 21) + 4321
    iq, offs = synth.make_iq(fs, n, ["wfm", "nfm"])
    pw = amd.params.chain_params(fs, offs[0], "wfm", output=amd._lib.OUT_S16)
    pn = amd.params.chain_params(fs, offs[1], "nfm", output=amd._lib.OUT_S16)
    assert pw.sq_length == 15625 and pw.audio_rate == 48000
    eng, (cw, cn) = _run_chains(amd, iq, fs, [pw, pn], 1 << 18)
    ref = oracle.stages(iq, pw)
    assert rel_rms(cw.read_debug(0), ref["ddc"]) < 1e-5
    bp = cw.read_debug(2)
    assert bp.size == ref["bandpass"].size and rel_rms(bp, ref["bandpass"]) < 1e-5
    sq = cw.read_debug(3)
    assert sq.size == ref["squelch"].size and sq.size >= 2 * 15625
    dem = cw.read_debug(4)
    assert dem.size == ref["demod"].size and dem.size > 5000, (dem.size, ref["demod"].size)
    assert rel_rms(dem, ref["demod"]) < 1e-5
    s16 = np.frombuffer(cw.read_audio(), np.int16)
    assert s16.size == ref["s16"].size
    assert np.mean(np.abs(s16.astype(np.int32) - ref["s16"]) <= 1) > 0.999
    sn = np.frombuffer(cn.read_audio(), np.int16)
    ref_n = oracle.stages(iq, pn)["s16"]
    assert sn.size == ref_n.size and np.mean(np.abs(sn.astype(np.int32) - ref_n) <= 1) > 0.999
    eng.close()


def test_c5_ssb_noise_filter_chains(amd):
    """BASELINE config 5 shape: 10 Msps, 64 USB chains with NoiseFilter(10) (nr_enabled,
    ClientAudioChain, csdr/chain/clientaudio.py:12-13) and the 150..3000 Hz bandpass; sampled
    chains' audio (NoiseFilter output, int16) vs the oracle, one chain without NR alongside."""
    from openwebrx_amd import synth
    fs = 10000000
    modes = ["usb"] * 65
    n = 1 << 21
    iq, offs = synth.make_iq(fs, n, modes)
    plist = [amd.params.chain_params(fs, o, "usb", output=amd._lib.OUT_S16, nr_enabled=c < 64,
                                     nr_threshold=10) for c, o in enumerate(offs)]
    eng, chains = _run_chains(amd, iq, fs, plist, 1 << 19)
    for c in (0, 37, 63, 64):
        ref = oracle.stages(iq, plist[c])
        s16 = np.frombuffer(chains[c].read_audio(), np.int16)
        assert s16.size == ref["s16"].size and s16.size > 1000, (c, s16.size, ref["s16"].size)
        d = np.abs(s16.astype(np.int32) - ref["s16"])
        assert np.mean(d <= 1) > 0.999, (c, np.mean(d <= 1), d.max())
        if c < 64:
            assert "nr" in ref
    eng.close()


def test_noise_filter_float_and_reset(amd):
    """NoiseFilter float output (OUT_F32) within 1e-5 rel-RMS of the oracle; switching it off
    and on (a fresh NoiseFilter, clientaudio.py:80-90) restarts its state."""
    from openwebrx_amd import synth
    fs = 2400000
    iq, offs = synth.make_iq(fs, 1 << 20, ["nfm"])
    p = amd.params.chain_params(fs, offs[0], "nfm", output=amd._lib.OUT_F32, nr_enabled=True,
                                nr_threshold=5)
    eng, (ch,) = _run_chains(amd, iq, fs, [p], 1 << 18)
    got = np.frombuffer(ch.read_audio(), np.float32)
    ref = oracle.stages(iq, p)
    assert got.size == ref["nr"].size and got.size > 2000
    assert rel_rms(got, ref["nr"]) < 1e-5
    eng.close()


def _rate_fx(rate):
    """design.cpp rate_to_fx: a float rate in 2^-64 turns per sample."""
    r = float(np.float32(rate))
    r -= np.floor(r)
    s = r * 18446744073709551616.0
    return 0 if s >= 18446744073709551615.0 else int(s)


def test_retune_is_phase_continuous(amd):
    """Shift.setRate on a running chain (Selector.setFrequencyOffset -> Shift.setRate,
    csdr/chain/selector.py:132-140): the engine switches rate at the next output boundary with a
    continuous phase; DDC output vs float64 numpy of that piecewise phase."""
    from openwebrx_amd import synth
    fs, B = 2400000, 1 << 18
    iq, offs = synth.make_iq(fs, 3 * B, ["nfm", "usb"])
    p = amd.params.chain_params(fs, offs[0], "nfm", output=amd._lib.OUT_S16)
    eng = amd.Engine(fs, max_block=B)
    eng.set_debug(True)
    ch = eng.chain(p)
    eng.push(iq[:B])
    new_rate = amd.params.f32(amd.params.shift_rate(offs[1], fs))
    ch.set_shift_rate(new_rate)
    eng.push(iq[B:])
    eng.sync()
    got = ch.read_debug(0)
    c = oracle.chain_from_engine_params(p)
    T, D = c.ntaps, p.decimation
    nb = ((B - T) // D + 1) * D  # first input sample of the first output after the retune
    n = np.arange(iq.size, dtype=np.uint64)
    f0, f1 = np.uint64(_rate_fx(p.shift_rate)), np.uint64(_rate_fx(new_rate))
    with np.errstate(over="ignore"):
        ph = np.where(n < nb, (n + np.uint64(1)) * f0,
                      np.uint64(nb) * f0 + (n - np.uint64(nb) + np.uint64(1)) * f1)
    turns = ph.astype(np.float64) / 18446744073709551616.0
    x = (iq.astype(np.complex128) * np.exp(2j * np.pi * turns)).astype(np.complex64)
    ref = oracle.fir_decimate(x, c._keep[0], D)
    assert got.size == ref.size
    # the switch is per output: outputs before the boundary ran with the old rate over their whole
    # window (the csdr pipe's switch sample depends on its thread timing; this is the
    # deterministic choice), outputs from the boundary on follow the continuous piecewise phase
    k = nb // D
    old = oracle.fir_decimate(oracle.shift(iq, p.shift_rate), c._keep[0], D)
    assert rel_rms(got[:k], old[:k]) < 1e-5
    assert rel_rms(got[k:], ref[k:]) < 1e-5
    eng.close()


def test_live_changes_without_drain(amd):
    """Clients join, leave and drag the bandpass while others stream (owrx/dsp.py:538-562,
    Bandpass.setBandpass csdr/chain/selector.py:159-166) without draining the pipeline: the
    bandpass change applies from the next block, so chain 1's Bandpass output equals the oracle
    with the old taps up to the switch and with the new taps (same FIR history) after it; a
    chain leaving and one joining mid-stream leave the others untouched; the joiner's DDC follows
    its own origin; no call drained the block pipeline."""
    from openwebrx_amd import synth
    fs, B = 2400000, 1 << 17
    modes = ["nfm", "usb", "nfm", "am"]
    iq, offs = synth.make_iq(fs, 8 * B, modes + ["nfm"])
    plist = [amd.params.chain_params(fs, o, m, output=amd._lib.OUT_S16) for o, m in zip(offs, modes)]
    eng = amd.Engine(fs, max_block=B)
    eng.set_debug(True)
    chains = [eng.chain(p) for p in plist]
    d0 = eng.stats()["pipeline_drains"]
    eng.push(iq[:3 * B])
    lo, hi = amd.params.f32(300.0 / 12000), amd.params.f32(2400.0 / 12000)
    chains[1].set_bandpass(lo, hi)
    eng.push(iq[3 * B:4 * B])
    chains[3].close()
    pn = amd.params.chain_params(fs, offs[4], "nfm", output=amd._lib.OUT_S16)
    cn = eng.chain(pn)
    eng.push(iq[4 * B:])
    assert eng.stats()["pipeline_drains"] == d0  # join / leave / setBandpass: no drain
    eng.sync()
    # chain 1: Bandpass output piecewise (old taps, then new taps from the switch block on)
    p1 = plist[1]
    ref = oracle.stages(iq, p1)
    c1 = oracle.chain_from_engine_params(p1)
    T, D = c1.ntaps, p1.decimation
    k3 = (3 * B - T) // D + 1  # DDC outputs of the first three blocks
    fd = ref["frac"]
    s = (oracle.fractional_decimator(ref["ddc"][:k3], p1.frac_rate).size
         if p1.frac_rate != 1.0 else k3)
    new_taps = oracle.bandpass_taps(oracle.filter_len(p1.bp_transition), lo, hi)
    old = ref["bandpass"]
    new = oracle.fir_complex(fd, new_taps)
    got = chains[1].read_debug(2)
    assert got.size == fd.size, (got.size, fd.size)
    assert 0 < s < got.size
    assert rel_rms(got[:s], old[:s]) < 1e-5
    assert rel_rms(got[s:], new[s:]) < 1e-5
    assert rel_rms(got[s:], old[s:]) > 1e-2  # the change did take effect
    # untouched chains: whole stream vs the oracle
    _check_sampled_chains(iq, plist, chains, (0, 2))
    # the joiner: its shift phase starts at its origin (absolute sample index)
    org = cn.origin
    assert org > 0 and org % pn.decimation == 0
    cc = oracle.chain_from_engine_params(pn)
    n = np.arange(iq.size, dtype=np.uint64)
    with np.errstate(over="ignore"):
        ph = (n - np.uint64(org) + np.uint64(1)) * np.uint64(_rate_fx(pn.shift_rate))
    x = (iq.astype(np.complex128) * np.exp(2j * np.pi * ph.astype(np.float64) / 2.0 ** 64)).astype(np.complex64)
    refn = oracle.fir_decimate(x, cc._keep[0], pn.decimation)[org // pn.decimation:]
    gn = cn.read_debug(0)
    assert gn.size == refn.size, (gn.size, refn.size)
    assert rel_rms(gn, refn) < 1e-5
    assert len(cn.read_audio()) > 0
    eng.close()


def test_squelch_gating_and_chain_lifecycle(amd):
    """Squelch at -40 dB (setSquelchLevel(10^(dB/10)), selector.py:145-147): a chain on a carrier
    stays open, one on an empty channel closes to zeros -- both against the oracle; then an empty
    push, a chain removed and one added mid-stream (its output starts at its own origin)."""
    from openwebrx_amd import synth
    fs = 2400000
    iq, offs = synth.make_iq(fs, 1 << 20, ["nfm", "am"])
    empty = offs[0] + 60000
    pa = amd.params.chain_params(fs, offs[0], "nfm", squelch_db=-40, output=amd._lib.OUT_S16)
    pb = amd.params.chain_params(fs, empty, "nfm", squelch_db=-40, output=amd._lib.OUT_S16)
    eng, (ca, cb) = _run_chains(amd, iq, fs, [pa, pb], 1 << 18, debug=False)
    for ch, p in ((ca, pa), (cb, pb)):
        s16 = np.frombuffer(ch.read_audio(), np.int16)
        ref = oracle.stages(iq, p)
        assert s16.size == ref["s16"].size
        assert np.mean(np.abs(s16.astype(np.int32) - ref["s16"]) <= 1) > 0.999
    assert not np.any(oracle.stages(iq, pb)["squelch"])  # the empty channel is gated shut
    eng.push(iq[:0])
    cb.close()
    cc = eng.chain(amd.params.chain_params(fs, offs[1], "am", output=amd._lib.OUT_S16))
    more, _ = synth.make_iq(fs, 1 << 19, ["nfm", "am"], start=iq.size)
    eng.push(more)
    eng.sync()
    assert cc.origin >= iq.size - eng.history and len(cc.read_audio()) > 0
    assert len(ca.read_audio()) > 0
    eng.close()


def test_synthetic_source_model(amd):
    """owrx_synth_iq (the benchmark's stream): the SURVEY 8d model -- AWGN sigma 0.01 and one
    carrier of amplitude 0.05 per chain at its offset (+ the mode's tone); any sub-range of the
    stream generates identically on its own."""
    import torch
    fs, n = 2400000, 1 << 18
    offs = np.array([-600000.0, -100000.0, 250000.0, 700000.0])
    modes = np.array([2, 3, 4, 2], np.int32)  # usb, cw, lsb, usb: pure tones
    x = torch.empty(n, dtype=torch.complex64, device="cuda")
    assert amd._lib.lib.owrx_synth_iq(0, x.data_ptr(), n, 0, float(fs), 4, offs.ctypes.data,
                                      modes.ctypes.data, 7, 0.01, 0.05) == 0
    y = torch.empty(1000, dtype=torch.complex64, device="cuda")
    assert amd._lib.lib.owrx_synth_iq(0, y.data_ptr(), 1000, 5000, float(fs), 4, offs.ctypes.data,
                                      modes.ctypes.data, 7, 0.01, 0.05) == 0
    xs = x.cpu().numpy()
    assert np.array_equal(xs[5000:6000], y.cpu().numpy())
    spec = np.abs(np.fft.fft(xs)) / n
    tones = offs + np.array([1000.0, 800.0, -1000.0, 1000.0])
    for f in tones:  # tone energy within +-8 bins (the tones are not bin-centred)
        k = int(round(f / fs * n)) % n
        a = np.sqrt(np.sum(spec[k - 8:k + 9] ** 2))
        assert abs(a - 0.05) < 0.0025, (f, a)
    z = torch.empty(n, dtype=torch.complex64, device="cuda")  # noise alone: white, sigma 0.01
    assert amd._lib.lib.owrx_synth_iq(0, z.data_ptr(), n, 0, float(fs), 0, offs.ctypes.data,
                                      modes.ctypes.data, 7, 0.01, 0.05) == 0
    zs = z.cpu().numpy()
    assert abs(np.std(zs.real) - 0.01) < 2e-4 and abs(np.std(zs.imag) - 0.01) < 2e-4
    assert abs(np.mean(zs)) < 1e-4 and abs(np.corrcoef(zs.real[1:], zs.real[:-1])[0, 1]) < 0.01
