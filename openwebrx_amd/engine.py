"""Python handles over the C ABI: one Engine per GPU / wideband stream, Waterfall
(FftChain) and Chain (ClientDemodulatorChain) objects attached to it.  Thin: every call goes
straight to libowrx_amd.so."""
import ctypes
import threading

import numpy as np

from . import _lib
from ._lib import check, lib

STAGE_DDC, STAGE_FRAC, STAGE_BANDPASS, STAGE_SQUELCH, STAGE_DEMOD, STAGE_AGC = range(6)
_STAGE_DTYPE = {0: np.complex64, 1: np.complex64, 2: np.complex64, 3: np.complex64,
                4: np.float32, 5: np.float32}


_TLS = threading.local()  # read buffers per thread: pump threads of several engines read at once


def _scratch_map():
    m = getattr(_TLS, "bufs", None)
    if m is None:
        m = _TLS.bufs = {}
    return m


def _scratch(nbytes):
    """Reusable host buffer for ring reads (avoids a fresh multi-MB allocation per call)."""
    m = _scratch_map()
    b = m.get(nbytes)
    if b is None:
        b = m[nbytes] = np.empty(nbytes, dtype=np.uint8)
    return b


def _grown(key, n, dtype):
    """A reusable buffer of at least n items for `key`, grown geometrically (read_chains)."""
    m = _scratch_map()
    b = m.get(key)
    if b is None or b.size < n:
        b = m[key] = np.empty(max(n, int(1.5 * (b.size if b is not None else 0)), 1 << 16),
                              dtype=dtype)
    return b


def nfm_deemphasis_alpha(sample_rate):
    """NfmDeemphasis(sampleRate) coefficient (same as design.cpp nfm_deemphasis_alpha)."""
    dt = 1.0 / float(sample_rate)
    tau = 1.0 / (2.0 * np.pi * 300.0)
    return float(np.float32(dt / (tau + dt)))


def device_count():
    n = lib.owrx_device_count()
    return n if n > 0 else 0


class Engine:
    def __init__(self, samp_rate, max_block=1 << 20, device=0, history=None):
        """history: samples of the stream kept readable before each block (None: the minimum,
        2^18).  A waterfall batches frames across blocks (Waterfall.set_batch) only as far as
        the history reaches; owrx_process_device callers must provide that much before each
        block pointer."""
        h = ctypes.c_void_p()
        check(lib.owrx_engine_create_ex(device, float(samp_rate), int(max_block),
                                        int(history or 0), ctypes.byref(h)),
              "owrx_engine_create_ex")
        self._h = h
        self.samp_rate = samp_rate
        self.device = device
        self.max_block = int(max_block)
        self.history = lib.owrx_engine_history(h)

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            lib.owrx_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def push(self, iq):
        """Host cf32 samples (complex64 array or interleaved float32)."""
        a = np.ascontiguousarray(iq)
        if a.dtype == np.complex64:
            n = a.size
        elif a.dtype == np.float32:
            n = a.size // 2
        else:
            raise ValueError("IQ must be complex64 / interleaved float32")
        check(lib.owrx_push_iq(self._h, a.ctypes.data, n), "owrx_push_iq")

    def push_cs16(self, iq, gain=1.0):
        """Host cs16 samples (interleaved int16 I,Q) through the ingest conversion
        Convert(COMPLEX_SHORT, COMPLEX_FLOAT) + Gain(COMPLEX_FLOAT, gain) on the GPU."""
        a = np.ascontiguousarray(iq)
        if a.dtype != np.int16 or a.size % 2:
            raise ValueError("cs16 IQ must be an even-length int16 array")
        check(lib.owrx_push_iq_cs16(self._h, a.ctypes.data, a.size // 2, float(gain)),
              "owrx_push_iq_cs16")

    def process_device(self, ptr, n):
        check(lib.owrx_process_device(self._h, ctypes.c_void_p(ptr), int(n)), "owrx_process_device")

    def ingest_buffer(self):
        p = ctypes.c_void_p()
        cap = ctypes.c_int64()
        check(lib.owrx_ingest_buffer(self._h, ctypes.byref(p), ctypes.byref(cap)), "ingest_buffer")
        return p.value, cap.value

    def commit(self, n):
        check(lib.owrx_commit(self._h, int(n)), "owrx_commit")

    def sync(self):
        check(lib.owrx_sync(self._h), "owrx_sync")

    def wait_stream(self, stream_handle):
        """The engine's next blocks wait on the GPU for the work enqueued so far on the given
        hipStream_t (e.g. torch.cuda.current_stream().cuda_stream after a broadcast)."""
        check(lib.owrx_wait_stream(self._h, ctypes.c_void_p(int(stream_handle or 0))),
              "owrx_wait_stream")

    def set_stall_timeout(self, ms):
        """Longest any call waits on the GPU before the engine fails with TimeoutError
        (owrx_set_stall_timeout; default 20 s)."""
        check(lib.owrx_set_stall_timeout(self._h, int(ms)), "owrx_set_stall_timeout")

    def debug_stall(self, stream, us):
        """Test hook: occupy stream 0 (A), 1 (B), 2 (C), 3 (R) or 4 (the next waterfall row
        slot's stream) for `us` microseconds."""
        check(lib.owrx_debug_stall(self._h, int(stream), int(us)), "owrx_debug_stall")

    def set_input_retention(self, blocks):
        """process_device callers whose blocks stay valid for `blocks` further calls (e.g. a
        resident recording): the host may then run that many blocks ahead of the GPU."""
        check(lib.owrx_set_input_retention(self._h, int(blocks)), "owrx_set_input_retention")

    def set_block_pairing(self, enable=True):
        """Run contiguous process_device blocks two at a time (owrx_set_block_pairing; input
        retention >= 4, before the first chain, waterfall and block): outputs byte-identical,
        one block more latency."""
        check(lib.owrx_set_block_pairing(self._h, 1 if enable else 0), "owrx_set_block_pairing")

    def set_block_group(self, blocks):
        """Run `blocks` (1..4) contiguous process_device blocks as one engine block
        (owrx_set_block_group; input retention >= 2 x blocks, before the first chain, waterfall
        and block): outputs byte-identical, blocks - 1 blocks more latency."""
        check(lib.owrx_set_block_group(self._h, int(blocks)), "owrx_set_block_group")

    def set_pipeline_depth(self, blocks):
        """Blocks of chain work in flight (1..16, default 8), before the first chain and block."""
        check(lib.owrx_set_pipeline_depth(self._h, int(blocks)), "owrx_set_pipeline_depth")

    def set_debug(self, on=True):
        check(lib.owrx_set_debug(self._h, 1 if on else 0), "owrx_set_debug")

    def set_ddc_mode(self, mode):
        """DDC form: "fast" (fast-convolution filter bank, default) or "direct" (polyphase FIR)."""
        check(lib.owrx_set_ddc_mode(self._h, {"fast": 0, "direct": 1}[mode]), "owrx_set_ddc_mode")

    def set_timing(self, on=True, every=1):
        """HIP-event timing of the kernel groups in every `every`-th block (off: on=False)."""
        check(lib.owrx_set_timing(self._h, int(every) if on else 0), "owrx_set_timing")

    def stats(self):
        s = _lib.Stats()
        check(lib.owrx_get_stats(self._h, ctypes.byref(s)), "owrx_get_stats")
        return {k: getattr(s, k) for k, _ in _lib.Stats._fields_}

    @staticmethod
    def handles(chains):
        """The chains' native handles as an int32 array (for read_chains)."""
        return np.fromiter((c.id for c in chains), dtype=np.int32, count=len(chains))

    def read_chains(self, chains, max_bytes=None, max_values=None):
        """Drains the audio and s-meter rings of many chains (owrx_chains_read_audio /
        owrx_chains_read_smeter) -- the one-thread pump for a server with many clients.  Returns
        (audio, alens, smeter, scounts): the concatenated bytes and float values as numpy arrays
        plus each chain's share, in the order of `chains`.  The arrays are views of reused read
        buffers: valid until the next read_chains call.

        max_bytes / max_values None (default): everything the rings hold -- a size query, then
        one read into a buffer of that size (at 131 072 C3 chains a block leaves ~80 MB of
        audio: a fixed 64 MiB buffer left the rest to pile up in the rings, whose growth then
        stalled the drains).  A number caps the call (the rest stays in the rings).

        `chains` may also be an int32 array of chain handles (`Engine.handles`): a server that
        keeps one pays no Python pass over its chain objects per read (~8 ms at 131 072 chains)."""
        n = len(chains)
        if isinstance(chains, np.ndarray):
            handles = np.ascontiguousarray(chains, dtype=np.int32)
        else:
            handles = self.handles(chains)
        ph = handles.ctypes.data_as(_lib._pi32)
        alens = np.zeros(n, np.int64)
        scounts = np.zeros(n, np.int64)
        pl, pc = alens.ctypes.data_as(_lib._pi64), scounts.ctypes.data_as(_lib._pi64)
        if max_bytes is None:
            max_bytes = check(lib.owrx_chains_read_audio(self._h, n, ph, None, 0, pl), "read_chains")
        if max_values is None:
            max_values = check(lib.owrx_chains_read_smeter(self._h, n, ph, None, 0, pc), "read_chains")
        abuf = _grown("read_audio", max_bytes, np.uint8)
        sbuf = _grown("read_smeter", max_values, np.float32)
        na = check(lib.owrx_chains_read_audio(self._h, n, ph, abuf.ctypes.data, max_bytes, pl),
                   "read_chains") if max_bytes > 0 else 0
        ns = check(lib.owrx_chains_read_smeter(self._h, n, ph, sbuf.ctypes.data, max_values, pc),
                   "read_chains") if max_values > 0 else 0
        if max_bytes == 0:
            alens[:] = 0
        if max_values == 0:
            scounts[:] = 0
        return abuf[:na], alens, sbuf[:ns], scounts

    def waterfall(self, fft_size, every_n_samples, avg_number, add_db=-70.0, adpcm=True):
        return Waterfall(self, fft_size, every_n_samples, avg_number, add_db, adpcm)

    def chain(self, params):
        return Chain(self, params)


class Waterfall:
    def __init__(self, engine, fft_size, every_n_samples, avg_number, add_db, adpcm):
        self.engine = engine
        h = ctypes.c_int()
        check(lib.owrx_waterfall_create(engine.handle, int(fft_size), int(every_n_samples),
                                        int(avg_number), float(add_db), 1 if adpcm else 0,
                                        ctypes.byref(h)), "owrx_waterfall_create")
        self.id = h.value
        self.fft_size = fft_size
        self.adpcm = adpcm

    def set(self, every_n_samples, avg_number, adpcm):
        check(lib.owrx_waterfall_set(self.engine.handle, self.id, int(every_n_samples),
                                     int(avg_number), 1 if adpcm else 0), "owrx_waterfall_set")
        self.adpcm = adpcm

    def set_batch(self, min_frames, max_lag=0):
        """Launch the FFT once `min_frames` frames are ready (or the oldest pending frame is
        `max_lag` samples behind the newest block, or at sync): chip-filling launches at the
        cost of row latency.  Call before streaming."""
        check(lib.owrx_waterfall_set_batch(self.engine.handle, self.id, int(min_frames),
                                           int(max_lag)), "owrx_waterfall_set_batch")

    def set_latency(self, max_wall_ms):
        """Wall-clock bound on the batching: pending frames launch before they would wait more
        than `max_wall_ms` (owrx_waterfall_set_latency; <= 0: none)."""
        check(lib.owrx_waterfall_set_latency(self.engine.handle, self.id, float(max_wall_ms)),
              "owrx_waterfall_set_latency")

    def row_bytes(self):
        return check(lib.owrx_waterfall_row_bytes(self.engine.handle, self.id), "row_bytes")

    def round_frames(self):
        """Frames one full round of the FFT launch deals (owrx_waterfall_round_frames; 0: n/a)."""
        return check(lib.owrx_waterfall_round_frames(self.engine.handle, self.id), "round_frames")

    def read(self, max_bytes=None):
        """Whole rows produced so far (or at most max_bytes worth of rows)."""
        rb = self.row_bytes()
        out = []
        left = max_bytes if max_bytes is not None else 1 << 62
        buf = _scratch(max(rb * 16, 1 << 20))
        while left >= rb:
            m = min(left, buf.size)
            n = check(lib.owrx_waterfall_read(self.engine.handle, self.id, buf.ctypes.data, m),
                      "owrx_waterfall_read")
            if n <= 0:
                break
            out.append(buf[:n].tobytes())
            left -= n
        return b"".join(out)

    def read_rows(self):
        rb = self.row_bytes()
        data = self.read()
        if self.adpcm:
            return np.frombuffer(data, dtype=np.uint8).reshape(-1, rb)
        return np.frombuffer(data, dtype=np.float32).reshape(-1, self.fft_size)

    def close(self):
        if self.id:
            lib.owrx_waterfall_destroy(self.engine.handle, self.id)
            self.id = 0


class Chain:
    def __init__(self, engine, params):
        self.engine = engine
        self.params = params
        h = ctypes.c_int()
        check(lib.owrx_chain_create(engine.handle, ctypes.byref(params), ctypes.byref(h)),
              "owrx_chain_create")
        self.id = h.value

    @property
    def origin(self):
        return check(lib.owrx_chain_origin(self.engine.handle, self.id), "origin")

    def set_shift_rate(self, rate):
        check(lib.owrx_chain_set_shift_rate(self.engine.handle, self.id, float(rate)), "shift")

    def set_bandpass(self, low, high):
        en = low is not None and high is not None
        check(lib.owrx_chain_set_bandpass(self.engine.handle, self.id, 1 if en else 0,
                                          float(low or 0), float(high or 0)), "bandpass")

    def set_squelch_level(self, level):
        check(lib.owrx_chain_set_squelch_level(self.engine.handle, self.id, float(level)),
              "squelch")

    def read_audio(self, max_bytes=None):
        """All audio bytes produced so far (or at most max_bytes)."""
        out = []
        left = max_bytes if max_bytes is not None else 1 << 62
        buf = _scratch(1 << 20)
        while left > 0:
            m = min(left, buf.size)
            n = check(lib.owrx_chain_read_audio(self.engine.handle, self.id, buf.ctypes.data, m),
                      "read_audio")
            if n <= 0:
                break
            out.append(buf[:n].tobytes())
            left -= n
            if n < m:
                break
        return b"".join(out)

    def read_smeter(self, max_values=1 << 16):
        buf = _scratch(4 * max_values).view(np.float32)[:max_values]
        n = check(lib.owrx_chain_read_smeter(self.engine.handle, self.id, buf.ctypes.data,
                                             max_values), "read_smeter")
        return buf[:n].copy()

    def set_taps(self, selector=False, audio=False):
        """Publish the Selector output (cf32) and / or the pre-ClientAudioChain audio (f32) for
        secondary readers (owrx/dsp.py:185-206)."""
        check(lib.owrx_chain_set_taps(self.engine.handle, self.id, 1 if selector else 0,
                                      1 if audio else 0), "owrx_chain_set_taps")

    def read_tap(self, which):
        """which: "selector" -> complex64 array, "audio" -> float32 array (all available)."""
        w = {"selector": 0, "audio": 1}[which]
        out = []
        buf = _scratch(1 << 20)
        while True:
            n = check(lib.owrx_chain_read_tap(self.engine.handle, self.id, w, buf.ctypes.data,
                                              buf.size), "read_tap")
            if n <= 0:
                break
            out.append(buf[:n].tobytes())
        return np.frombuffer(b"".join(out), np.complex64 if w == 0 else np.float32)

    def set_secondary_fft(self, fft_size, every_n_samples=0, avg_number=0, add_db=-70.0,
                          adpcm=True):
        """FftChain on this chain's Selector output (owrx/dsp.py:220-225); fft_size 0 removes
        it.  every_n_samples / avg_number as FftChain derives them (params.fft_parameters)."""
        check(lib.owrx_chain_set_secondary_fft(self.engine.handle, self.id, int(fft_size),
                                               int(every_n_samples), int(avg_number),
                                               float(add_db), 1 if adpcm else 0),
              "set_secondary_fft")
        self._sf = (int(fft_size), bool(adpcm))

    def read_secondary_fft(self):
        """Whole secondary FFT rows produced so far: uint8 [rows, (N+10)/2] (ADPCM) or
        float32 [rows, N] dB."""
        n_fft, adpcm = getattr(self, "_sf", (0, True))
        rb = check(lib.owrx_chain_secondary_fft_row_bytes(self.engine.handle, self.id),
                   "secondary_fft_row_bytes")
        buf = _scratch(max(rb, ((1 << 20) // rb) * rb))
        out = []
        while True:
            n = check(lib.owrx_chain_read_secondary_fft(self.engine.handle, self.id,
                                                        buf.ctypes.data, buf.size),
                      "read_secondary_fft")
            if n <= 0:
                break
            out.append(buf[:n].tobytes())
        data = b"".join(out)
        if adpcm:
            return np.frombuffer(data, np.uint8).reshape(-1, rb)
        return np.frombuffer(data, np.float32).reshape(-1, n_fft)

    def read_debug(self, stage, max_bytes=1 << 26):
        buf = np.empty(max_bytes, dtype=np.uint8)
        n = check(lib.owrx_chain_read_debug(self.engine.handle, self.id, stage, buf.ctypes.data,
                                            max_bytes), "read_debug")
        return np.frombuffer(buf[:n].tobytes(), dtype=_STAGE_DTYPE[stage])

    def close(self):
        if self.id:
            lib.owrx_chain_destroy(self.engine.handle, self.id)
            self.id = 0


class Module:
    """One csdr module on the GPU outside a fused chain (owrx_module_*)."""

    def __init__(self, mtype, p0=0.0, p1=-1.0, p2=-1.0, device=0):
        h = ctypes.c_void_p()
        check(lib.owrx_module_create(device, mtype, float(p0), float(p1), float(p2),
                                     ctypes.byref(h)), "owrx_module_create")
        self._h = h
        self.mtype = mtype

    def process(self, data, out_bytes):
        a = np.ascontiguousarray(data)
        if a.dtype == np.complex64:
            n = a.size
        else:
            n = a.size
        out = np.empty(max(int(out_bytes), 1), dtype=np.uint8)
        r = check(lib.owrx_module_process(self._h, a.ctypes.data, n, out.ctypes.data, out.size),
                  "owrx_module_process")
        return out[:r].tobytes()

    def set(self, p0, p1=0.0, p2=0.0):
        """Shift.setRate / Bandpass.setBandpass on a running standalone module."""
        check(lib.owrx_module_set(self._h, float(p0), float(p1), float(p2)), "owrx_module_set")

    def close(self):
        if self._h:
            lib.owrx_module_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
