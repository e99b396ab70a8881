"""pycsdr.modules mirror: Buffer / Reader / Writer, the Module base class and the
hot-path module classes with the reference's constructor signatures and setters.

Execution model.  csdr runs one native thread per module, connected by ring buffers.  Here
the modules are descriptors; the GPU engine (libowrx_amd.so) runs them:

* fused segments -- a wideband COMPLEX_FLOAT Buffer read by `Shift -> FirDecimate ->
  [FractionalDecimator] -> [Bandpass] -> [Squelch] -> FmDemod,Limit,NfmDeemphasis | AmDemod,
  DcBlock | RealPart -> Agc -> [Convert(FLOAT,SHORT) -> [AdpcmEncoder]]` (a Selector + demod +
  ClientAudioChain, csdr/chain/selector.py, analog.py, clientaudio.py) or by `Fft ->
  LogAveragePower | LogPower -> FftSwap -> [FftAdpcm]` (FftChain, csdr/chain/fft.py) becomes
  one engine chain / waterfall, all of them batched on one engine per wideband Buffer
  (_graph.EngineDriver).  The graph is re-planned whenever a module is (re)wired, so
  Chain.replace / insert / remove (csdr/chain/__init__.py:51-120) work as in the reference;
  setters (setRate, setBandpass, setSquelchLevel, setEveryNSamples) take effect at the next
  block.
* the post-demodulator modules also run alone (one worker thread each, owrx_module_* GPU
  runners): FmDemod, AmDemod, RealPart, Limit, DcBlock, NfmDeemphasis, Agc, Convert(FLOAT,
  SHORT), AdpcmEncoder, FftSwap, FftAdpcm.
* everything else the reference imports exists so imports succeed, and raises
  NotImplementedError when instantiated ("may raise when instantiated").

Error behaviour follows pycsdr: setReader / setWriter raise ValueError on a format mismatch
(callers catch it: csdr/chain/__init__.py:60-84, owrx/fft.py:64-68, owrx/dsp.py:100-105);
Reader.read() blocks, returns a memoryview (valid until the next read) and None once stopped.
"""
import socket
import threading

import numpy as np

from .types import AgcProfile, Format
from . import _graph

csdr_version = "0.18.99"   # owrx/feature.py:213-221 requires >= 0.18.0
version = "0.18.99"

_DEFAULT_BUFFER_BYTES = 1 << 24


class Writer:
    """Anything with write(bytes-like) (csdr/chain/__init__.py:24: a Buffer is a writer)."""

    def write(self, data):
        raise NotImplementedError


class Buffer(Writer):
    """Multi-reader ring buffer.  Buffer(format, size=None); size in items.

    A preallocated byte ring: write() copies the data in (at most two slices, no per-write
    allocation), each reader keeps its own stream offset, and a reader that falls more than
    the ring's capacity behind loses the oldest data (as csdr's ring buffer).  Every call is
    O(bytes moved), independent of the number of readers and of the chunks written so far."""

    def __init__(self, format, size=None):
        if not isinstance(format, Format):
            raise ValueError("Buffer format must be a pycsdr.types.Format")
        self._format = format
        item = format.itemsize
        cap = int(size) * item if size else _DEFAULT_BUFFER_BYTES
        self._cap = max(item, cap - cap % item)
        self._ring = np.empty(self._cap, dtype=np.uint8)
        self._cond = threading.Condition()
        self._end = 0            # stream offset past the last written byte
        self._readers = []
        self._ended = False
        self.writer_module = None  # native module that writes here (graph planning)

    def getFormat(self):
        return self._format

    def getReader(self):
        r = Reader(self)
        with self._cond:
            r._pos = self._end
            self._readers.append(r)
        return r

    def end(self):
        """No more data will come (the engine writing here failed): readers drain what is
        buffered, then read() returns None."""
        with self._cond:
            self._ended = True
            self._cond.notify_all()

    def write(self, data):
        src = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) \
            else data.reshape(-1).view(np.uint8)
        n = src.size
        if n == 0:
            return
        cap = self._cap
        with self._cond:
            if n > cap:  # only the newest `cap` bytes can be kept
                self._end += n - cap
                src = src[n - cap:]
                n = cap
            off = self._end % cap
            first = min(n, cap - off)
            self._ring[off:off + first] = src[:first]
            if first < n:
                self._ring[:n - first] = src[first:]
            self._end += n
            self._cond.notify_all()

    def _take(self, reader):
        """Called with the condition held: the bytes available to `reader` (item aligned),
        copied into the reader's own buffer; a memoryview of it (valid until its next read)."""
        cap = self._cap
        pos = max(reader._pos, self._end - cap)
        n = self._end - pos
        n -= n % self._format.itemsize
        if n <= 0:
            return None
        if reader._out.size < n:
            reader._out = np.empty(max(n, 2 * reader._out.size), dtype=np.uint8)
        off = pos % cap
        first = min(n, cap - off)
        reader._out[:first] = self._ring[off:off + first]
        if first < n:
            reader._out[first:n] = self._ring[:n - first]
        reader._pos = pos + n
        return memoryview(reader._out[:n])

    def _remove_reader(self, reader):
        with self._cond:
            if reader in self._readers:
                self._readers.remove(reader)


class Reader:
    def __init__(self, buffer):
        self._buffer = buffer
        self._pos = 0
        self._out = np.empty(0, dtype=np.uint8)  # read()'s memoryview points here
        self._stopped = False
        self._detached = False   # a fused engine reads this buffer instead of this reader
        self.module = None       # native module reading here (graph planning)

    def getFormat(self):
        return self._buffer.getFormat()

    def read(self):
        b = self._buffer
        with b._cond:
            while True:
                if self._stopped:
                    return None
                data = b._take(self)
                if data is not None:
                    return data
                if b._ended:
                    return None
                b._cond.wait(0.5)

    def available(self):
        b = self._buffer
        with b._cond:
            return b._end - max(self._pos, b._end - b._cap)

    def stop(self):
        self._stopped = True
        with self._buffer._cond:
            self._buffer._cond.notify_all()

    def resume(self):
        self._stopped = False

    def _detach(self):
        with self._buffer._cond:
            self._detached = True
            self._pos = self._buffer._end


class Module:
    """Base class (subclassed by csdr/module/__init__.py:16 with ABCMeta)."""

    def __init__(self):
        pass


class _NativeModule(Module):
    """Common plumbing of the GPU-backed modules."""

    input_format = None
    output_format = None
    fusable = True

    def __init__(self):
        super().__init__()
        self.reader = None
        self.writer = None
        self._lock = threading.Lock()
        self._stopped = False
        self._worker = None
        self.absorbed = False  # set by the engine driver while part of a fused segment

    def getInputFormat(self):
        return self.input_format

    def getOutputFormat(self):
        return self.output_format

    def setReader(self, reader):
        if reader is not None and self.input_format is not None \
                and reader.getFormat() != self.input_format:
            raise ValueError("%s: input format %s does not match reader format %s"
                             % (type(self).__name__, self.input_format, reader.getFormat()))
        old = self.reader
        if old is not None and old is not reader:
            old.module = None
            old.stop()
        self.reader = reader
        if reader is not None:
            reader.module = self
            # Chain.replace hands the stopped predecessor's reader to its replacement
            # (csdr/chain/__init__.py:54-64; the modules re-arm it, cf. csdr/module/__init__.py:188)
            reader.resume()
        _graph.changed(self)
        self._check_start()

    def setWriter(self, writer):
        if isinstance(writer, Buffer) and self.output_format is not None \
                and writer.getFormat() != self.output_format:
            raise ValueError("%s: output format %s does not match buffer format %s"
                             % (type(self).__name__, self.output_format, writer.getFormat()))
        old = self.writer
        if isinstance(old, Buffer) and old.writer_module is self:
            old.writer_module = None
        self.writer = writer
        if isinstance(writer, Buffer):
            writer.writer_module = self
        _graph.changed(self)
        self._check_start()

    def stop(self):
        self._stopped = True
        if self.reader is not None:
            self.reader.stop()
        _graph.changed(self)

    # -- standalone execution (outside a fused segment) -------------------------------------
    def _check_start(self):
        if self.reader is None or self.writer is None or self._worker is not None:
            return
        if not self._standalone_supported():
            return  # only meaningful inside a fused segment; idles otherwise
        self._worker = threading.Thread(target=self._run, name=type(self).__name__,
                                        daemon=True)
        self._worker.start()

    def _standalone_supported(self):
        return False

    def _run(self):
        # the runner is created on the first data: idle (fused) modules hold no GPU state
        self._runner = None
        try:
            while not self._stopped:
                reader = self.reader
                if reader is None:
                    break
                data = reader.read()
                if data is None:
                    break
                if self.absorbed:
                    continue
                with self._lock:
                    if self._runner is None:
                        self._runner = self._make_runner()
                    out = self._runner(np.frombuffer(data, dtype=np.uint8))
                if out and self.writer is not None:
                    self.writer.write(out)
        finally:
            with self._lock:
                close = getattr(self._runner, "close", None)
                self._runner = None
            if close:
                close()

    def _reads_module_output(self):
        """The input buffer is written by another module (a tap such as ClientDemodulatorChain's
        selectorBuffer, owrx/dsp.py:185-206), not by the wideband source a fused segment reads."""
        r = self.reader
        w = r._buffer.writer_module if r is not None else None
        return w is not None and getattr(w, "fusable", False)

    def _update_runner(self, *params):
        with self._lock:
            r = getattr(self, "_runner", None)
            if r is None:
                return
            if hasattr(r, "set"):
                r.set(*params)
            else:  # a stand-in (e.g. a pass-through): rebuilt from the new parameters
                self._runner = None

    def _make_runner(self):
        raise NotImplementedError


class _GpuModuleRunner:
    """owrx_module_* runner: one stateful GPU module, host buffers in and out."""

    def __init__(self, mtype, in_dtype, out_itemsize, out_per_in, p0=0.0, p1=-1.0, p2=-1.0):
        from ..engine import Module as _Mod
        self._m = _Mod(mtype, p0, p1, p2)
        self._in_dtype = in_dtype
        self._out_itemsize = out_itemsize
        self._out_per_in = out_per_in

    def __call__(self, raw):
        x = raw.view(self._in_dtype)
        cap = int(x.size * self._out_per_in * self._out_itemsize) + 64
        return self._m.process(x, cap)

    def set(self, *params):
        self._m.set(*params)

    def close(self):
        self._m.close()


# ---- waterfall (csdr/chain/fft.py) --------------------------------------------------------

class Fft(_NativeModule):
    input_format = Format.COMPLEX_FLOAT
    output_format = Format.COMPLEX_FLOAT

    def __init__(self, size, every_n_samples=0, window=None):
        super().__init__()
        self.size = int(size)
        self.every_n_samples = int(every_n_samples)

    def setEveryNSamples(self, every_n_samples):
        self.every_n_samples = int(every_n_samples)
        _graph.changed(self, structural=False)


class LogPower(_NativeModule):
    input_format = Format.COMPLEX_FLOAT
    output_format = Format.FLOAT

    def __init__(self, add_db=0.0):
        super().__init__()
        self.add_db = float(add_db)


class LogAveragePower(_NativeModule):
    input_format = Format.COMPLEX_FLOAT
    output_format = Format.FLOAT

    def __init__(self, add_db=0.0, fft_size=0, avg_number=1):
        super().__init__()
        self.add_db = float(add_db)
        self.fft_size = int(fft_size)
        self.avg_number = int(avg_number)

    def setAvgNumber(self, avg_number):
        self.avg_number = int(avg_number)
        _graph.changed(self, structural=False)


class FftSwap(_NativeModule):
    input_format = Format.FLOAT
    output_format = Format.FLOAT

    def __init__(self, fft_size):
        super().__init__()
        self.fft_size = int(fft_size)

    def _standalone_supported(self):
        return True

    def _make_runner(self):
        from .. import _lib
        return _GpuModuleRunner(_lib.MOD_FFTSWAP, np.float32, 4, 1.0, self.fft_size)


class FftAdpcm(_NativeModule):
    input_format = Format.FLOAT
    output_format = Format.CHAR

    def __init__(self, fft_size):
        super().__init__()
        self.fft_size = int(fft_size)

    def _standalone_supported(self):
        return True

    def _make_runner(self):
        from .. import _lib
        n = self.fft_size
        return _GpuModuleRunner(_lib.MOD_FFTADPCM, np.float32, 1, (n + 10) / (2.0 * n) + 1.0, n)


# ---- selector (csdr/chain/selector.py) -----------------------------------------------------

class Shift(_NativeModule):
    input_format = Format.COMPLEX_FLOAT
    output_format = Format.COMPLEX_FLOAT

    def __init__(self, rate):
        super().__init__()
        self.rate = float(rate)

    def setRate(self, rate):
        self.rate = float(rate)
        self._update_runner(self.rate)
        _graph.changed(self, structural=False)

    # standalone on a module's output (the SecondarySelector on selectorBuffer); at the head of
    # a chain on the wideband buffer it runs fused in the engine's DDC
    def _standalone_supported(self):
        return self._reads_module_output()

    def _make_runner(self):
        from .. import _lib
        return _GpuModuleRunner(_lib.MOD_SHIFT, np.complex64, 8, 1.0, self.rate)


class FirDecimate(_NativeModule):
    input_format = Format.COMPLEX_FLOAT
    output_format = Format.COMPLEX_FLOAT

    def __init__(self, decimation, transition, cutoff=0.5, window=None):
        super().__init__()
        self.decimation = int(decimation)
        self.transition = float(transition)
        self.cutoff = float(cutoff)


class FractionalDecimator(_NativeModule):
    """COMPLEX_FLOAT: the Selector's resampler (csdr/chain/selector.py:32-33).  FLOAT with
    prefilter=True: WFm's IF-to-audio decimator (csdr/chain/analog.py:69).  Both run fused in a
    chain segment on the engine."""

    def __init__(self, format, rate, num_poly_points=12, prefilter=False):
        super().__init__()
        if format not in (Format.COMPLEX_FLOAT, Format.FLOAT) or num_poly_points != 12:
            raise NotImplementedError("FractionalDecimator: COMPLEX_FLOAT or FLOAT, 12 points")
        if prefilter != (format == Format.FLOAT):
            raise NotImplementedError("FractionalDecimator: the GPU path has COMPLEX_FLOAT "
                                      "without and FLOAT with prefilter (the reference's uses)")
        self.input_format = self.output_format = format
        self.rate = float(rate)
        self.prefilter = bool(prefilter)


class Bandpass(_NativeModule):
    input_format = Format.COMPLEX_FLOAT
    output_format = Format.COMPLEX_FLOAT

    def __init__(self, low_cut=None, high_cut=None, transition=0.0, use_fft=False):
        super().__init__()
        self.low_cut = None if low_cut is None else float(low_cut)
        self.high_cut = None if high_cut is None else float(high_cut)
        self.transition = float(transition)
        self.use_fft = bool(use_fft)

    def setBandpass(self, low_cut, high_cut):
        self.low_cut = float(low_cut)
        self.high_cut = float(high_cut)
        self._update_runner(self.low_cut, self.high_cut, self.transition)
        _graph.changed(self, structural=False)

    # standalone outside a fused chain (the SecondarySelector's Bandpass, csdr/chain/
    # selector.py:212-224); inside a client chain it is part of the fused Selector
    def _standalone_supported(self):
        return self._reads_module_output() and self.transition > 0

    def _make_runner(self):
        from .. import _lib
        if self.low_cut is None or self.high_cut is None:
            return lambda raw: raw.tobytes()  # no cuts: Bandpass passes through
        return _GpuModuleRunner(_lib.MOD_BANDPASS, np.complex64, 8, 1.0, self.low_cut,
                                self.high_cut, self.transition)


class Squelch(_NativeModule):
    def __init__(self, format, length=1024, decimation=5, hangLength=0, flushLength=0,
                 reportInterval=0):
        super().__init__()
        if format != Format.COMPLEX_FLOAT:
            raise NotImplementedError("Squelch: only COMPLEX_FLOAT is on the GPU path")
        self.input_format = self.output_format = format
        self.length = int(length)
        self.decimation = int(decimation)
        self.hang_length = int(hangLength)
        self.flush_length = int(flushLength)
        self.report_interval = int(reportInterval)
        self.level = 0.0
        self.power_writer = None

    def setSquelchLevel(self, level):
        self.level = float(level)
        _graph.changed(self, structural=False)

    def setPowerWriter(self, writer):
        self.power_writer = writer


# ---- demodulators and audio (csdr/chain/analog.py, clientaudio.py) -------------------------

class _Unary(_NativeModule):
    _mod = None
    _in_dtype = np.float32
    _out_size = 4

    def _standalone_supported(self):
        return True

    def _params(self):
        return ()

    def _make_runner(self):
        from .. import _lib
        return _GpuModuleRunner(getattr(_lib, self._mod), self._in_dtype, self._out_size, 1.0,
                                *self._params())


class FmDemod(_Unary):
    input_format = Format.COMPLEX_FLOAT
    output_format = Format.FLOAT
    _mod = "MOD_FMDEMOD"
    _in_dtype = np.complex64


class AmDemod(_Unary):
    input_format = Format.COMPLEX_FLOAT
    output_format = Format.FLOAT
    _mod = "MOD_AMDEMOD"
    _in_dtype = np.complex64


class RealPart(_Unary):
    input_format = Format.COMPLEX_FLOAT
    output_format = Format.FLOAT
    _mod = "MOD_REALPART"
    _in_dtype = np.complex64


class DcBlock(_Unary):
    input_format = Format.FLOAT
    output_format = Format.FLOAT
    _mod = "MOD_DCBLOCK"


class Limit(_Unary):
    input_format = Format.FLOAT
    output_format = Format.FLOAT
    _mod = "MOD_LIMIT"

    def __init__(self, maxAmplitude=1.0):
        super().__init__()
        self.max_amplitude = float(maxAmplitude)

    def _params(self):
        return (self.max_amplitude,)


class NoiseFilter(_NativeModule):
    """NoiseFilter(threshold) of ClientAudioChain (csdr/chain/clientaudio.py:12-13): FLOAT ->
    FLOAT spectral subtraction; runs fused in a chain segment (kernels_nr.hip)."""
    input_format = Format.FLOAT
    output_format = Format.FLOAT

    def __init__(self, threshold=0):
        super().__init__()
        self.threshold = float(threshold)


class WfmDeemphasis(_Unary):
    """WfmDeemphasis(sampleRate, tau) (csdr/chain/analog.py:70): one-pole de-emphasis,
    alpha = dt / (tau + dt)."""
    input_format = Format.FLOAT
    output_format = Format.FLOAT
    _mod = "MOD_DEEMPH"

    def __init__(self, sampleRate, tau=50e-6):
        super().__init__()
        self.sample_rate = int(sampleRate)
        self.tau = float(tau)

    def _params(self):
        dt = 1.0 / float(self.sample_rate)
        return (float(np.float32(dt / (float(np.float32(self.tau)) + dt))),)


class NfmDeemphasis(_Unary):
    input_format = Format.FLOAT
    output_format = Format.FLOAT
    _mod = "MOD_DEEMPH"

    def __init__(self, sampleRate):
        super().__init__()
        self.sample_rate = int(sampleRate)

    def _params(self):
        from ..engine import nfm_deemphasis_alpha
        return (nfm_deemphasis_alpha(self.sample_rate),)


class Agc(_Unary):
    _mod = "MOD_AGC"

    def __init__(self, format):
        super().__init__()
        if format != Format.FLOAT:
            raise NotImplementedError("Agc: only FLOAT is on the GPU path")
        self.input_format = self.output_format = format
        self.profile = AgcProfile.FAST   # csdr's Agc default profile
        self.initial_gain = None
        self.max_gain = None

    def setProfile(self, profile):
        self.profile = AgcProfile(profile)
        _graph.changed(self)

    def setInitialGain(self, gain):
        self.initial_gain = float(gain)
        _graph.changed(self)

    def setMaxGain(self, gain):
        self.max_gain = float(gain)
        _graph.changed(self)

    def _params(self):
        return (self.profile.engine_id,
                -1.0 if self.initial_gain is None else self.initial_gain,
                -1.0 if self.max_gain is None else self.max_gain)


class Convert(_Unary):
    """Convert(FLOAT, SHORT) (csdr/chain/clientaudio.py:18) and Convert(COMPLEX_SHORT,
    COMPLEX_FLOAT), the SDR ingest conversion (owrx/source/direct.py:51-71)."""
    _mod = "MOD_CONVERT_F_S16"
    _out_size = 2

    def __init__(self, inFormat, outFormat):
        super().__init__()
        if (inFormat, outFormat) == (Format.COMPLEX_SHORT, Format.COMPLEX_FLOAT):
            self._mod = "MOD_CONVERT_CS16_CF32"
            self._in_dtype = np.int32      # one (I, Q) int16 pair per item
            self._out_size = 8
        elif (inFormat, outFormat) != (Format.FLOAT, Format.SHORT):
            raise NotImplementedError("Convert(%s, %s) is not on the GPU path yet"
                                      % (inFormat, outFormat))
        self.input_format = inFormat
        self.output_format = outFormat


class Gain(_Unary):
    """Gain(format, gain): FLOAT (csdr/chain/analog.py:29) or COMPLEX_FLOAT (the ingest
    conversion, owrx/source/direct.py:51-71, fifi_sdr.py:27-28)."""
    _mod = "MOD_GAIN"

    def __init__(self, format, gain):
        super().__init__()
        if format == Format.FLOAT:
            self._in_dtype, self._out_size, self._complex = np.float32, 4, 0.0
        elif format == Format.COMPLEX_FLOAT:
            self._in_dtype, self._out_size, self._complex = np.complex64, 8, 1.0
        else:
            raise NotImplementedError("Gain(%s) is not on the GPU path yet" % (format,))
        self.input_format = self.output_format = format
        self.gain = float(gain)

    def _params(self):
        return (self.gain, self._complex)


class AdpcmEncoder(_Unary):
    input_format = Format.SHORT
    output_format = Format.CHAR
    _mod = "MOD_ADPCM"
    _in_dtype = np.int16
    _out_size = 1

    def __init__(self, sync=False):
        super().__init__()
        self.sync = bool(sync)

    def _params(self):
        return (1.0 if self.sync else 0.0,)

    def _make_runner(self):
        from .. import _lib
        # one byte per two samples, plus an 8-byte frame every 1001 data bytes
        return _GpuModuleRunner(_lib.MOD_ADPCM, np.int16, 1, 0.51, *self._params())


# ---- ingest (owrx/source/__init__.py:307-330) ----------------------------------------------

class TcpSource(_NativeModule):
    """Connects to an SDR's IQ TCP port and writes what arrives (host-side ingest)."""
    input_format = None
    fusable = False

    def __init__(self, port, format):
        super().__init__()
        self.port = int(port)
        self.output_format = format
        self._sock = None

    def _check_start(self):
        if self.writer is None or self._worker is not None:
            return
        self._worker = threading.Thread(target=self._pump, name="TcpSource", daemon=True)
        self._worker.start()

    def _pump(self):
        try:
            self._sock = socket.create_connection(("127.0.0.1", self.port))
            while not self._stopped:
                data = self._sock.recv(1 << 16)
                if not data:
                    break
                self.writer.write(data)
        except OSError:
            pass
        finally:
            if self._sock is not None:
                self._sock.close()

    def stop(self):
        super().stop()
        if self._sock is not None:
            try:
                self._sock.shutdown(socket.SHUT_RDWR)
            except OSError:
                pass


class AudioResampler(_Unary):
    """AudioResampler(inputRate, outputRate) (csdr/chain/clientaudio.py:15-16): FLOAT, run
    standalone on the GPU behind a fused chain's F32 audio (ClientAudioChain inserts it when the
    demodulator's audio rate differs from the client rate, owrx/dsp.py:157-166).  Rational L/M
    polyphase lowpass; csdr's filter design is not in the reference (parity unpinned)."""
    input_format = Format.FLOAT
    output_format = Format.FLOAT
    _mod = "MOD_AUDIO_RESAMPLER"

    def __init__(self, inputRate, outputRate):
        super().__init__()
        self.input_rate = int(inputRate)
        self.output_rate = int(outputRate)

    def _params(self):
        return (self.input_rate, self.output_rate)

    def _make_runner(self):
        from .. import _lib
        return _GpuModuleRunner(_lib.MOD_AUDIO_RESAMPLER, np.float32, 4,
                                self.output_rate / self.input_rate + 0.01, *self._params())


class Afc(_Unary):
    """Afc(updatePeriod, samplePeriod) of SAm / RawSAm (csdr/chain/analog.py:141-167):
    COMPLEX_FLOAT carrier frequency tracking ahead of RealPart, standalone on the GPU behind a
    fused Selector (the planner then emits the Selector output, OWRX_OUT_SEL).  csdr's algorithm
    is not in the reference: the build's documented choice (OWRX_MOD_AFC; parity
    unpinned, pinned to oracle.afc)."""
    input_format = Format.COMPLEX_FLOAT
    output_format = Format.COMPLEX_FLOAT
    _mod = "MOD_AFC"
    _in_dtype = np.complex64
    _out_size = 8

    def __init__(self, updatePeriod=10, samplePeriod=4):
        super().__init__()
        self.update_period = int(updatePeriod)
        self.sample_period = int(samplePeriod)

    def _params(self):
        return (self.update_period, self.sample_period)


# ---- present for imports only (may raise when instantiated) -----------------

def _unsupported(name):
    def __init__(self, *args, **kwargs):
        raise NotImplementedError("pycsdr.modules.%s is outside the MI355X hot path "
                                  "(SURVEY.md 8a) and has no implementation here" % name)
    return type(name, (_NativeModule,), {"__init__": __init__, "fusable": False})


for _name in ("BaudotDecoder", "Ccir476Decoder", "Ccir493Decoder",
              "CwDecoder", "DBPskDecoder", "Downmix", "DscDecoder", "ExecModule", "FaxDecoder",
              "Lowpass", "MFRttyDecoder", "NavtexDecoder", "RttyDecoder",
              "SitorBDecoder", "SnrSquelch", "SstvDecoder", "Throttle", "TimingRecovery",
              "VaricodeDecoder"):
    globals()[_name] = _unsupported(_name)
del _name
