"""Fusion of pycsdr module graphs onto the GPU engine.

A *source* buffer is a COMPLEX_FLOAT Buffer whose writer is not a fusable module (the
wideband IQ buffer fed by TcpSource / the SDR source, owrx/source/__init__.py:307-330).
Every reader of a source buffer that belongs to a Shift (Selector, csdr/chain/selector.py:95)
or an Fft (FftChain, csdr/chain/fft.py:34) starts a *segment*: the modules linked through
single-reader Buffers downstream of it.  plan_segment() recognises the two hot-path shapes
and returns the engine parameters; one EngineDriver per source buffer owns one engine per GPU
(OWRX_AMD_DEVICES, default every visible device), places each recognised segment on one of
them (multi.Placement: balanced within FirDecimate designs, so each engine keeps one DDC
launch per design), feeds every engine the source's blocks and writes each segment's output
into the writer of its last module.

Failure (owrx/source/__init__.py:224-227 fail() -> clients' onFail()): an engine
error stops the driver, marks it FAILED, ends every output buffer it was writing (their
readers' read() returns None once drained, so the pumps of owrx/dsp.py:858-861 finish instead
of blocking forever) and calls the callbacks registered with on_failure(source).

The graph is re-planned at the next block boundary after any (re)wiring; setters that do not
change the shape (Shift.setRate, Bandpass.setBandpass, Squelch.setSquelchLevel,
Fft.setEveryNSamples) are applied to the live engine objects.
"""
import logging
import os
import threading
import weakref

import numpy as np

logger = logging.getLogger(__name__)

_drivers = weakref.WeakValueDictionary()  # id(source buffer) -> EngineDriver
_lock = threading.RLock()

BLOCK = 1 << 18  # IQ samples per engine block (26 ms at 10 Msps)
# Engine history (samples of the stream kept readable before each block): room for a waterfall
# batch of up to ~HISTORY / hop frames.  32 MiB of cf32 (two of them in the push ring).
HISTORY = 1 << 22
# Waterfall launch batching: frames per FFT launch (four per CU of a 256-CU MI355X) and the
# wall-clock bound on how long a ready frame may wait for its batch (OWRX_AMD_WF_LATENCY_MS).
# At the stream's real-time rate the bound launches every block or two (rows within ~50 ms);
# fed faster than real time (a recording, a backlog) the frame bound gives chip-filling launches.
WF_BATCH_FRAMES = 960


def wf_latency_ms():
    return float(os.environ.get("OWRX_AMD_WF_LATENCY_MS", "50"))

_failure_callbacks = {}  # id(source buffer) -> [callable(exception)]


def devices():
    """GPUs the drop-in spreads its engines over: OWRX_AMD_DEVICES ("0,1,2"; a repeated index
    runs several engines on one GPU), else every visible device."""
    env = os.environ.get("OWRX_AMD_DEVICES", "").strip()
    if env:
        return [int(v) for v in env.split(",") if v.strip()]
    from ..engine import device_count
    return list(range(max(1, device_count())))


def on_failure(source, callback):
    """Register callback(exception), called once if the engine driving `source` fails (an
    SdrSource would call its fail() here, owrx/source/__init__.py:224-227)."""
    with _lock:
        _failure_callbacks.setdefault(id(source), []).append(callback)


def state(source):
    """"RUNNING", "FAILED" or "STOPPED" for the driver of a source buffer (None: no driver)."""
    drv = _drivers.get(id(source))
    return None if drv is None else drv.state


def changed(module, structural=True):
    """A module was (re)wired or re-parameterised: find its source buffer's driver."""
    from . import modules as M
    with _lock:
        head = _find_head(module)
        if head is None:
            return
        src = head.reader._buffer
        if src.getFormat() != M.Format.COMPLEX_FLOAT:
            return
        drv = _drivers.get(id(src))
        if drv is None:
            drv = EngineDriver(src)
            _drivers[id(src)] = drv
        drv.mark_dirty(structural)


def _upstream(module):
    r = module.reader
    if r is None:
        return None
    w = r._buffer.writer_module
    return w if (w is not None and w.fusable) else None


def _find_head(module):
    """Walk upstream to the module that reads a source buffer."""
    seen = set()
    m = module
    while m is not None and id(m) not in seen:
        seen.add(id(m))
        up = _upstream(m)
        if up is None:
            return m if m.reader is not None else None
        m = up
    return None


def _readers_of(buf):
    return [r.module for r in buf._readers if r.module is not None and not r._stopped]


# Modules a client chain continues into, in the order a branch point prefers them
# (selectorBuffer: the demodulator; audioBuffer: ClientAudioChain's first module)
def _continuations():
    from . import modules as M
    return (M.FmDemod, M.AmDemod, M.Afc, M.RealPart, M.FractionalDecimator, M.Bandpass,
            M.Squelch, M.Limit, M.NfmDeemphasis, M.WfmDeemphasis, M.DcBlock, M.Agc, M.Gain,
            M.NoiseFilter,
            M.Convert, M.AdpcmEncoder, M.FirDecimate, M.LogAveragePower, M.LogPower, M.FftSwap,
            M.FftAdpcm)


def _downstream(module):
    """The module a segment continues into.  Other readers of the same buffer are taps, not the
    continuation: ClientDemodulatorChain hangs its secondary FftChain on the Selector output
    next to the demodulator (owrx/dsp.py:220-225), a SecondarySelector or a COMPLEX_FLOAT
    secondary demodulator on selectorBuffer and a FLOAT secondary demodulator on audioBuffer
    (:185-206).  The continuation is the first reader (in attachment order) of the most
    preferred class; a Shift or Fft is never one (they only start segments)."""
    from .modules import Buffer
    w = module.writer
    if not isinstance(w, Buffer):
        return None
    readers = [m for m in _readers_of(w) if m.fusable]
    for cls in _continuations():
        for m in readers:
            if type(m) is cls:
                return m
    return None


def _taps_of(module, continuation):
    """Live readers of `module`'s output buffer other than the chain's continuation and a fused
    secondary FFT: native modules, or Python modules (csdr.module, e.g. a decoder) whose readers
    carry no module -- they receive the tapped stream the engine driver writes there."""
    from . import modules as M
    w = module.writer
    if not isinstance(w, M.Buffer):
        return []
    with w._cond:
        rs = [r for r in w._readers if not (r._stopped or r._detached)]
    return [r for r in rs if r.module is not continuation and not isinstance(r.module, M.Fft)]


def _plan_fft(mods):
    """FftChain shape at the start of `mods`: (params, modules used) or None."""
    from . import modules as M
    if not mods or not isinstance(mods[0], M.Fft):
        return None
    fft, i = mods[0], 1

    def take(cls):
        nonlocal i
        if i < len(mods) and isinstance(mods[i], cls):
            i += 1
            return mods[i - 1]
        return None

    avg = take(M.LogAveragePower) or take(M.LogPower)
    swap = take(M.FftSwap)
    if avg is None or swap is None or fft.every_n_samples <= 0:
        return None
    if isinstance(avg, M.LogAveragePower) and avg.fft_size not in (0, fft.size):
        return None
    adp = take(M.FftAdpcm)
    used = mods[:i]
    if used[-1].writer is None:
        return None
    return (dict(fft_size=fft.size, hop=fft.every_n_samples,
                 avg=avg.avg_number if isinstance(avg, M.LogAveragePower) else 1,
                 add_db=avg.add_db, adpcm=adp is not None), used)


def _secondary_fft(selector_last):
    """An FftChain reading the Selector output buffer (the secondary FFT), or None."""
    from . import modules as M
    w = selector_last.writer
    if not isinstance(w, M.Buffer):
        return None
    for m in _readers_of(w):
        if isinstance(m, M.Fft) and not m._stopped:
            got = _plan_fft(_walk(m))
            if got is not None:
                return got
    return None


def _walk(head):
    mods = [head]
    while True:
        nxt = _downstream(mods[-1])
        if nxt is None or nxt in mods:
            return mods
        mods.append(nxt)


def plan_segment(head):
    """(kind, params, modules) for a recognised segment starting at `head`, else None.

    kind "chain": params = dict of owrx_chain_params fields (+ "power_writer");
    kind "waterfall": params = dict(fft_size, hop, avg, add_db, adpcm)."""
    from . import modules as M
    from .. import _lib
    mods = _walk(head)
    i = 0

    def take(cls):
        nonlocal i
        if i < len(mods) and isinstance(mods[i], cls):
            i += 1
            return mods[i - 1]
        return None

    if isinstance(head, M.Fft):
        got = _plan_fft(mods)
        return None if got is None else ("waterfall", got[0], got[1])

    if not isinstance(head, M.Shift):
        return None
    shift = take(M.Shift)
    fir = take(M.FirDecimate)
    if fir is None:
        return None
    chain_next = (M.FractionalDecimator, M.Bandpass, M.Squelch, M.FmDemod, M.AmDemod,
                  M.RealPart, M.Afc)
    if fir.writer is not None and (i == len(mods) or not isinstance(mods[i], chain_next)):
        # Shift -> FirDecimate -> Buffer(COMPLEX_FLOAT): the service Resampler
        # (owrx/source/resampler.py:11-26); the engine emits the cf32 DDC output itself
        p = dict(shift_rate=shift.rate, decimation=fir.decimation, transition=fir.transition,
                 cutoff=fir.cutoff, frac_rate=1.0, output=_lib.OUT_IQ, power_writer=None)
        return ("chain", p, mods[:i])
    frac = take(M.FractionalDecimator)
    bp = take(M.Bandpass)
    sq = take(M.Squelch)
    selector_last = mods[i - 1]
    sel_end = i

    def _selector_output():
        """Selector output read by something the engine does not fuse (an IQ-input decoder:
        ServiceDemodulatorChain with Selector(withSquelch=False), owrx/service/chain.py:7-23;
        a demodulator chain the engine does not know): the engine emits the cf32 Selector output
        itself and whatever reads it runs as standalone modules."""
        if selector_last.writer is None or selector_last is fir:
            return None
        p = dict(shift_rate=shift.rate, decimation=fir.decimation, transition=fir.transition,
                 cutoff=fir.cutoff, frac_rate=frac.rate if frac is not None else 1.0,
                 bandpass=0, bp_low=0.0, bp_high=0.0, bp_transition=0.0,
                 sq_length=750, sq_decimation=5, sq_hang=0, sq_flush=0, sq_report=0,
                 sq_level=0.0, demod=_lib.DEMOD_SSB, agc_profile=0, agc_initial_gain=-1.0,
                 agc_max_gain=-1.0, audio_rate=12000, output=_lib.OUT_SEL, power_writer=None,
                 tap_selector=None, tap_audio=None, secondary_fft=None, secondary_modules=[],
                 secondary_writer=None)
        if bp is not None and bp.low_cut is not None and bp.high_cut is not None:
            p.update(bandpass=1, bp_low=bp.low_cut, bp_high=bp.high_cut,
                     bp_transition=bp.transition)
        if sq is not None:
            p.update(sq_length=sq.length, sq_decimation=sq.decimation, sq_hang=sq.hang_length,
                     sq_flush=sq.flush_length, sq_report=sq.report_interval, sq_level=sq.level,
                     power_writer=sq.power_writer)
        return ("chain", p, mods[:sel_end])

    fm = take(M.FmDemod)
    wfm = None
    afc = None
    if fm is None:
        afc = take(M.Afc)
    if afc is not None:
        # SAm / RawSAm (csdr/chain/analog.py:141-167): Afc -> RealPart -> DcBlock -> Agc / Gain
        if take(M.RealPart) is None or take(M.DcBlock) is None:
            return _selector_output()
        demod, audio_rate = _lib.DEMOD_SAM, 12000
    elif fm is not None:
        lim = take(M.Limit)
        if lim is None or lim.max_amplitude != 1.0:
            return None
        de = take(M.NfmDeemphasis)
        if de is not None:
            demod, audio_rate = _lib.DEMOD_NFM, de.sample_rate
        else:  # WFm: FractionalDecimator(FLOAT, prefilter) -> WfmDeemphasis, no Agc
            fdf = take(M.FractionalDecimator)
            wde = take(M.WfmDeemphasis)
            if fdf is None or wde is None or not fdf.prefilter:
                return None
            demod, audio_rate = _lib.DEMOD_WFM, wde.sample_rate
            wfm = dict(if_rate=fdf.rate * wde.sample_rate, deemph_tau=wde.tau)
    elif take(M.AmDemod) is not None:
        if take(M.DcBlock) is None:
            return _selector_output()
        demod, audio_rate = _lib.DEMOD_AM, 12000
    elif take(M.RealPart) is not None:
        demod, audio_rate = _lib.DEMOD_SSB, 12000
    else:
        return _selector_output()
    agc = take(M.Agc) if wfm is None else None
    gain = None
    if agc is None and wfm is None:
        # no Agc: RawAm (AmDemod -> DcBlock -> Gain(100), csdr/chain/analog.py:23-31) and
        # RawSAm (:156-167) end in a FLOAT Gain, which the engine applies in the Agc's place
        gain = take(M.Gain) if demod in (_lib.DEMOD_AM, _lib.DEMOD_SAM) else None
        if gain is None or gain.input_format != M.Format.FLOAT or gain.gain <= 0:
            return _selector_output()
    demod_last = mods[i - 1]  # writes audioBuffer (ClientDemodulatorChain._connect, dsp.py:86-92)
    nr = take(M.NoiseFilter)
    output = _lib.OUT_F32
    if take(M.Convert) is not None:
        output = _lib.OUT_S16
        enc = take(M.AdpcmEncoder)
        if enc is not None:
            if not enc.sync:
                return None
            output = _lib.OUT_ADPCM
    used = mods[:i]
    if used[-1].writer is None:
        return None
    p = dict(shift_rate=shift.rate, decimation=fir.decimation, transition=fir.transition,
             cutoff=fir.cutoff, frac_rate=frac.rate if frac is not None else 1.0,
             bandpass=0, bp_low=0.0, bp_high=0.0, bp_transition=0.0,
             sq_length=750, sq_decimation=5, sq_hang=0, sq_flush=0, sq_report=0, sq_level=0.0,
             demod=demod, agc_profile=agc.profile.engine_id if agc is not None else 0,
             agc_initial_gain=-1.0 if agc is None or agc.initial_gain is None else agc.initial_gain,
             agc_max_gain=-1.0 if agc is None or agc.max_gain is None else agc.max_gain,
             audio_rate=audio_rate, output=output, power_writer=None,
             afc_update=afc.update_period if afc is not None else 0,
             afc_sample=afc.sample_period if afc is not None else 0,
             audio_gain=gain.gain if gain is not None else 0.0)
    if wfm is not None:
        p.update(wfm)
    p.update(nr_enabled=1 if nr is not None else 0,
             nr_threshold=nr.threshold if nr is not None else 0.0)
    if bp is not None and bp.low_cut is not None and bp.high_cut is not None:
        p.update(bandpass=1, bp_low=bp.low_cut, bp_high=bp.high_cut,
                 bp_transition=bp.transition)
    if sq is not None:
        p.update(sq_length=sq.length, sq_decimation=sq.decimation, sq_hang=sq.hang_length,
                 sq_flush=sq.flush_length, sq_report=sq.report_interval, sq_level=sq.level,
                 power_writer=sq.power_writer)
    sel_cont = mods[mods.index(selector_last) + 1]
    aud_cont = mods[mods.index(demod_last) + 1] if mods.index(demod_last) + 1 < len(mods) else None
    p["tap_selector"] = selector_last.writer if _taps_of(selector_last, sel_cont) else None
    p["tap_audio"] = demod_last.writer if aud_cont is not None and _taps_of(demod_last, aud_cont) \
        else None
    sec = _secondary_fft(selector_last)
    p["secondary_fft"] = sec[0] if sec is not None else None
    p["secondary_modules"] = sec[1] if sec is not None else []
    p["secondary_writer"] = sec[1][-1].writer if sec is not None else None
    return ("chain", p, used)


def chain_params_struct(p):
    from .. import _lib
    s = _lib.ChainParams()
    for k, v in p.items():
        if k not in ("power_writer", "secondary_fft", "secondary_modules", "secondary_writer",
                     "tap_selector", "tap_audio"):
            setattr(s, k, v)
    return s


class EngineDriver:
    """One driver per source buffer: reads it, runs every fused segment on one of its engines
    (one per entry of devices()), writes outputs."""

    def __init__(self, source):
        from ..multi import Placement
        self.source = source
        self.devices = devices()
        self.engines = {}   # slot (index into self.devices) -> Engine
        self.placement = Placement(len(self.devices))
        self.segments = {}  # head id -> (kind, params, modules, engine object, slot)
        self.state = "RUNNING"
        self.error = None
        self._dirty = True
        self._closing = False
        self._pool = None
        self.reader = source.getReader()  # before any further write: nothing is missed
        self._thread = threading.Thread(target=self._run, name="owrx-engine", daemon=True)
        self._thread.start()

    @property
    def engine(self):  # the first engine (single-GPU callers and tests)
        return self.engines.get(min(self.engines)) if self.engines else None

    def mark_dirty(self, structural=True):
        self._dirty = True

    def _heads(self):
        from . import modules as M
        with self.source._cond:
            rs = list(self.source._readers)
        return [r.module for r in rs if isinstance(r.module, (M.Shift, M.Fft))
                and not r.module._stopped]

    @staticmethod
    def _group_key(kind, p):
        if kind == "waterfall":
            return ("waterfall",)
        return ("chain", p["decimation"], p["transition"], p["cutoff"])

    def _engine(self, slot):
        from ..engine import Engine
        eng = self.engines.get(slot)
        if eng is None:
            eng = Engine(1.0, max_block=BLOCK, device=self.devices[slot], history=HISTORY)
            self.engines[slot] = eng
        return eng

    def _replan(self):
        plans = {}
        for h in self._heads():
            seg = plan_segment(h)
            if seg is not None:
                plans[id(h)] = seg
        self._planned = plans  # outputs to end should creating their engine objects fail
        # drop segments that vanished or changed shape / design parameters
        for hid in list(self.segments):
            kind, p, mods, obj, slot = self.segments[hid]
            new = plans.get(hid)
            if new is None or new[0] != kind or new[2] != mods or not _compatible(kind, p, new[1]):
                self._absorb(mods, False)
                self._absorb(p.get("secondary_modules", []), False)
                obj.close()
                self.placement.release(slot, self._group_key(kind, p))
                del self.segments[hid]
        for hid, (kind, p, mods) in plans.items():
            if hid in self.segments:
                self._update(hid, p)
                continue
            slot = self.placement.place(self._group_key(kind, p))
            eng = self._engine(slot)
            if kind == "waterfall":
                obj = eng.waterfall(p["fft_size"], p["hop"], max(1, p["avg"]), p["add_db"],
                                    p["adpcm"])
                lat = wf_latency_ms()
                if lat > 0:  # batched launches, bounded in wall-clock time
                    try:
                        obj.set_batch(WF_BATCH_FRAMES)
                        obj.set_latency(lat)
                    except ValueError:  # a hop the history cannot batch: per-block launches
                        pass
            else:
                obj = eng.chain(chain_params_struct(p))
                if p.get("secondary_fft") is not None:
                    _apply_secondary(obj, p["secondary_fft"])
                if p.get("tap_selector") is not None or p.get("tap_audio") is not None:
                    obj.set_taps(p.get("tap_selector") is not None, p.get("tap_audio") is not None)
            self.segments[hid] = (kind, p, mods, obj, slot)
            self._absorb(mods, True)
            self._absorb(p.get("secondary_modules", []), True)

    def _absorb(self, mods, on):
        for m in mods:
            m.absorbed = on
            if on and m is mods[0] and m.reader is not None:
                m.reader._detach()   # the engine reads the source through its own reader

    def _update(self, hid, p):
        kind, old, mods, obj, slot = self.segments[hid]
        if kind == "waterfall":
            if (old["hop"], old["avg"], old["adpcm"]) != (p["hop"], p["avg"], p["adpcm"]):
                obj.set(p["hop"], max(1, p["avg"]), p["adpcm"])
        else:
            if old["shift_rate"] != p["shift_rate"]:
                obj.set_shift_rate(p["shift_rate"])
            if (old.get("bandpass"), old.get("bp_low"), old.get("bp_high")) != \
                    (p.get("bandpass"), p.get("bp_low"), p.get("bp_high")):
                obj.set_bandpass(p["bp_low"], p["bp_high"]) if p["bandpass"] else \
                    obj.set_bandpass(None, None)
            if old.get("sq_level") != p.get("sq_level"):
                obj.set_squelch_level(p["sq_level"])
            if old.get("secondary_fft") != p.get("secondary_fft"):
                _apply_secondary(obj, p.get("secondary_fft"))
            if (old.get("tap_selector") is None, old.get("tap_audio") is None) != \
                    (p.get("tap_selector") is None, p.get("tap_audio") is None):
                obj.set_taps(p.get("tap_selector") is not None, p.get("tap_audio") is not None)
            olds, news = old.get("secondary_modules", []), p.get("secondary_modules", [])
            if olds != news:
                self._absorb([m for m in olds if m not in news], False)
                self._absorb(news, True)
        self.segments[hid] = (kind, p, mods, obj, slot)

    def _drain(self):
        """Every segment's new output into its writer: chain audio and s-meter values of each
        engine with two batched native calls (Engine.read_chains), waterfall rows, secondary
        FFT rows and taps per object."""
        by_slot = {}
        for kind, p, mods, obj, slot in list(self.segments.values()):
            out = mods[-1].writer
            if kind == "waterfall":
                data = obj.read()
                if data and out is not None:
                    out.write(data)
                continue
            by_slot.setdefault(slot, []).append((p, out, obj))
            sw = p.get("secondary_writer")
            if p.get("secondary_fft") and sw is not None:
                rows = obj.read_secondary_fft()
                if rows.size:
                    sw.write(rows.tobytes())
            # taps: the Selector output into selectorBuffer, the demodulator chain's audio
            # into audioBuffer, for their secondary readers
            for key, which in (("tap_selector", "selector"), ("tap_audio", "audio")):
                buf = p.get(key)
                if buf is not None:
                    t = obj.read_tap(which)
                    if t.size:
                        buf.write(t.tobytes())
        for slot, segs in by_slot.items():
            eng = self.engines[slot]
            audio, alens, sm, scounts = eng.read_chains([obj for _, _, obj in segs])
            ao = np.concatenate(([0], np.cumsum(alens)))
            so = np.concatenate(([0], np.cumsum(scounts)))
            for i, (p, out, obj) in enumerate(segs):
                if alens[i] and out is not None:
                    out.write(audio[ao[i]:ao[i + 1]].tobytes())
                pw = p.get("power_writer")
                if scounts[i] and pw is not None:
                    pw.write(sm[so[i]:so[i + 1]].tobytes())

    def _push(self, blk):
        # every engine gets the block from host memory over its own PCIe link (8 B per
        # sample: 0.5 GB/s per GPU at 61.44 Msps); with several engines the pushes run in
        # parallel threads (the native call releases the GIL), so the engines' host-side block
        # work overlaps instead of adding up
        engs = list(self.engines.values())
        if len(engs) == 1:
            engs[0].push(blk)
            return
        if self._pool is None:
            from concurrent.futures import ThreadPoolExecutor
            self._pool = ThreadPoolExecutor(max_workers=8, thread_name_prefix="owrx-push")
        for f in [self._pool.submit(e.push, blk) for e in engs]:
            f.result()  # re-raises an engine's error in the driver thread

    def close(self):
        """Stop reading the source; the thread pushes what it holds, syncs and drains."""
        self._closing = True
        if self.reader is not None:
            self.reader.stop()
        self._thread.join()

    def _outputs(self):
        segs = [(p, mods) for kind, p, mods, obj, slot in self.segments.values()]
        segs += [(p, mods) for kind, p, mods in getattr(self, "_planned", {}).values()]
        for p, mods in segs:
            for buf in (mods[-1].writer, p.get("power_writer"), p.get("secondary_writer"),
                        p.get("tap_selector"), p.get("tap_audio")):
                if buf is not None:
                    yield buf

    def _fail(self, exc):
        logger.error("GPU engine failed: %s", exc)
        self.state = "FAILED"
        self.error = exc
        self.reader.stop()
        for buf in list(self._outputs()):
            end = getattr(buf, "end", None)
            if end is not None:
                end()
        for cb in _failure_callbacks.get(id(self.source), []):
            try:
                cb(exc)
            except Exception:
                logger.exception("failure callback")

    def _run(self):
        try:
            self._loop()
        except Exception as exc:  # engine / HIP error: surface it, do not leave readers hanging
            with _lock:
                self._fail(exc)
            return
        if self.state == "RUNNING":
            self.state = "STOPPED"

    def _loop(self):
        pending = []
        npend = 0
        while True:
            data = self.reader.read()
            if data is None:
                if pending and self.engines:
                    with _lock:
                        self._push(np.concatenate(pending))
                if self.engines:
                    with _lock:
                        for eng in self.engines.values():
                            eng.sync()
                        self._drain()
                break
            with _lock:
                if self._dirty:
                    self._dirty = False
                    self._replan()
            if not self.engines:
                continue
            x = np.frombuffer(data, dtype=np.complex64)
            if not pending and x.size >= BLOCK:
                # a whole block in one read: pushed straight from the reader's buffer (valid
                # until its next read; the push copies it into the engine's staging)
                with _lock:
                    self._push(x)
                    self._drain()
                continue
            pending.append(x.copy())  # the reader's buffer is reused by the next read
            npend += x.size
            if npend < BLOCK:
                continue
            blk = np.concatenate(pending)
            pending, npend = [], 0
            with _lock:
                self._push(blk)
                self._drain()


def finish(source):
    """Flush and stop the engine driver of a source buffer (end of stream / tests)."""
    with _lock:
        drv = _drivers.pop(id(source), None)
    if drv is not None:
        drv.close()
    return drv


def _apply_secondary(obj, sf):
    if sf is None:
        obj.set_secondary_fft(0)
    else:
        obj.set_secondary_fft(sf["fft_size"], sf["hop"], sf["avg"], sf["add_db"], sf["adpcm"])


def _compatible(kind, old, new):
    """Parameters that can change on a live engine object (everything else re-creates it)."""
    if kind == "waterfall":
        keys = ("fft_size", "add_db")
    else:
        keys = ("decimation", "transition", "cutoff", "frac_rate", "bp_transition", "sq_length",
                "sq_decimation", "sq_hang", "sq_flush", "sq_report", "demod", "agc_profile",
                "agc_initial_gain", "agc_max_gain", "audio_rate", "output", "if_rate",
                "deemph_tau", "nr_enabled", "nr_threshold", "afc_update", "afc_sample",
                "audio_gain")
    return all(old.get(k) == new.get(k) for k in keys)
