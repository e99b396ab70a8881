"""Drives the reference's own SpectrumThread (owrx/fft.py:13-109) over the pycsdr shim and records
what the planner makes of the FftChain it builds at each step: start (adpcm), the compression
switched to "none" (`_setCompression` swaps FftAdpcm out, catches the ValueError of the format
change and re-wires a fresh Buffer + pump thread, :61-73), the fft_size changed (`restart` on the
wired property, :50, :89-91) and the compression back to adpcm; also the module graph (classes,
parameters, wiring) so a GPU test can rebuild it without the reference
(tests/golden/spectrum_graph.json, made by tests/golden/make_spectrum_graph.py).

A stand-in SDR source supplies the properties, the wideband Buffer and writeSpectrumData (which
counts what the pump delivers); the shared Config is a plain PropertyLayer so nothing is read
from disk.  Run as a script with ROOT / REF (a subprocess: the reference's modules never enter
the test process).  No engine is created: nothing is written to the wideband buffer."""
import json
import sys
import threading
import time


def main(ROOT, REF):
    sys.path.insert(0, ROOT)
    import openwebrx_amd.pycsdr as shim
    shim.install()
    sys.path.append(REF)
    from owrx.property import PropertyLayer
    from owrx.config import Config
    Config.sharedConfig = PropertyLayer()  # the SDR layer carries every property used
    from owrx.fft import SpectrumThread
    from pycsdr.modules import Buffer
    from pycsdr.types import Format
    from openwebrx_amd.pycsdr import _graph

    class Source:
        """The parts of owrx.source.SdrSource SpectrumThread uses."""

        def __init__(self):
            self.props = PropertyLayer(samp_rate=10000000, fft_size=16384, fft_fps=9,
                                       fft_voverlap_factor=0.3, fft_compression="adpcm")
            self.buffer = Buffer(Format.COMPLEX_FLOAT)
            self.clients = []
            self.spectrum = []

        def isAvailable(self):
            return True

        def getBuffer(self):
            return self.buffer

        def addClient(self, c):
            self.clients.append(c)

        def removeClient(self, c):
            if c in self.clients:
                self.clients.remove(c)

        def writeSpectrumData(self, data):
            self.spectrum.append(len(data))

    def describe(m):
        d = {"class": type(m).__name__}
        for k in ("size", "every_n_samples", "add_db", "fft_size", "avg_number"):
            if hasattr(m, k):
                v = getattr(m, k)
                d[k] = v if isinstance(v, (int, float, bool, type(None))) else str(v)
        if getattr(m, "output_format", None) is not None:
            d["out_format"] = m.output_format.name
        return d

    def record(name, st, src):
        heads = [r.module for r in src.buffer._readers
                 if r.module is not None and not r._stopped and not r._detached]
        live = [h for h in heads if type(h).__name__ == "Fft"]
        entry = {"step": name, "live_heads": len(live), "clients": len(src.clients)}
        if live:
            seg = _graph.plan_segment(live[-1])
            entry["fused"] = seg is not None
            if seg is not None:
                kind, p, used = seg
                entry["kind"] = kind
                entry["params"] = p
                entry["graph"] = [describe(m) for m in used]
                # the chain writes into the Buffer SpectrumThread's pump reads
                entry["writer_format"] = used[-1].writer.getFormat().name
        def pumps():
            return sum(1 for t in threading.enumerate()
                       if t.is_alive() and "pump" in (t.name or "").lower()
                       or getattr(t, "_target", None) is not None and
                       "pump" in getattr(getattr(t, "_target"), "__qualname__", ""))
        # a swapped-out chain's pump ends asynchronously once its reader stops: give it a moment
        # (counting at once raced with that exit now and then)
        deadline = time.time() + 2.0
        n = pumps()
        while n > len(live) and time.time() < deadline:
            time.sleep(0.01)
            n = pumps()
        entry["pump_threads"] = n
        entry["dsp_output_format"] = st.dsp.getOutputFormat().name if st.dsp else None
        steps.append(entry)

    steps = []
    src = Source()
    st = SpectrumThread(src)
    st.start()
    record("start_adpcm", st, src)
    src.props["fft_compression"] = "none"
    record("compression_none", st, src)
    src.props["fft_size"] = 8192
    time.sleep(0.05)
    record("fft_size_8192", st, src)
    src.props["fft_compression"] = "adpcm"
    record("compression_adpcm_again", st, src)
    src.props["fft_fps"] = 20
    record("fps_20", st, src)
    st.stop()
    record_stop = {"step": "stopped", "clients": len(src.clients),
                   "live_heads": sum(1 for r in src.buffer._readers
                                     if r.module is not None and not r._stopped
                                     and not r._detached and type(r.module).__name__ == "Fft"),
                   "spectrum_writes": len(src.spectrum)}
    steps.append(record_stop)
    _graph.finish(src.buffer)
    print(json.dumps(steps))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
