"""Drives the reference's own ClientDemodulatorChain (owrx/dsp.py:39-225) over the pycsdr shim
and records, step by step, what the planner makes of the module graph it builds: the fused
chain's engine parameters, the taps it publishes for secondary readers and the module graph
itself (class names, constructor parameters and wiring), so a GPU test can rebuild the same
graph without the reference checkout (tests/golden/dsp_graph.json, made by
tests/golden/make_dsp_graph.py).

Run as a script with ROOT / REF set (a subprocess: the reference's modules never enter the test
process).  Prints one JSON document.  No engine is created: nothing is written to the
wideband buffer."""
import json
import sys


def main(ROOT, REF):
    sys.path.insert(0, ROOT)
    import openwebrx_amd.pycsdr as shim
    shim.install()
    sys.path.append(REF)
    from csdr.chain.analog import NFm, Am, Ssb, WFm, SAm, RawSAm, RawAm, SsbDigital
    from csdr.chain.demodulator import SecondaryDemodulator, SecondarySelectorChain, ServiceDemodulator
    from owrx.service.chain import ServiceDemodulatorChain
    from csdr.module import ThreadModule
    from owrx.dsp import ClientDemodulatorChain, ClientDemodulatorSecondaryDspEventClient
    from pycsdr.modules import Buffer
    from pycsdr.types import Format, AgcProfile
    from openwebrx_amd.pycsdr import _graph
    from openwebrx_amd.pycsdr import modules as M

    class Sink(ThreadModule):
        """Stand-in for a digital decoder (out of scope): consumes its input."""

        def __init__(self, fmt):
            self.fmt = fmt
            super().__init__()

        def getInputFormat(self):
            return self.fmt

        def getOutputFormat(self):
            return Format.CHAR

        def run(self):
            while self.doRun and self.reader is not None:
                if self.reader.read() is None:
                    break

        def stop(self):
            self.doRun = False
            if self.reader is not None:
                self.reader.stop()

    class SelectorSecondary(SecondaryDemodulator, SecondarySelectorChain):
        """A secondary demodulator behind a SecondarySelector (PSK31-like, owrx/dsp.py:188-202)."""

        def __init__(self):
            super().__init__([Sink(Format.COMPLEX_FLOAT)])

        def getBandwidth(self):
            return 100.0

    class AudioSecondary(SecondaryDemodulator):
        """A FLOAT secondary demodulator reading audioBuffer (owrx/dsp.py:205-206)."""

        def __init__(self):
            super().__init__([Sink(Format.FLOAT)])

    class IqService(ServiceDemodulator):
        """A service decoder that takes the Selector's IQ (getInputFormat COMPLEX_FLOAT):
        ServiceDemodulatorChain wires Selector(withSquelch=False) straight into it."""

        def __init__(self):
            super().__init__([Sink(Format.COMPLEX_FLOAT)])

        def getFixedAudioRate(self):
            return 12000

    class AudioService(ServiceDemodulator):
        """A service decoder on audio (FT8-like): ServiceDemodulatorChain puts the primary
        demodulator between the Selector and it."""

        def __init__(self):
            super().__init__([Sink(Format.FLOAT)])

        def getFixedAudioRate(self):
            return 12000

    class Events(ClientDemodulatorSecondaryDspEventClient):
        def onSecondaryDspRateChange(self, rate):
            pass

        def onSecondaryDspBandwidthChange(self, bw):
            pass

    def describe(mod):
        d = {"class": type(mod).__name__}
        for k in ("rate", "decimation", "transition", "cutoff", "low_cut", "high_cut", "use_fft",
                  "length", "decimation", "hang_length", "flush_length", "report_interval",
                  "level", "size", "every_n_samples", "avg_number", "add_db", "fft_size",
                  "max_amplitude", "sample_rate", "tau", "prefilter", "threshold", "sync",
                  "initial_gain", "max_gain", "update_period", "sample_period", "gain"):
            if hasattr(mod, k):
                v = getattr(mod, k)
                d[k] = v if isinstance(v, (int, float, bool, type(None))) else str(v)
        if hasattr(mod, "profile") and mod.profile is not None:
            d["profile"] = mod.profile.value
        if getattr(mod, "input_format", None) is not None:
            d["format"] = mod.input_format.name
        if getattr(mod, "output_format", None) is not None:
            d["out_format"] = mod.output_format.name
        return d

    def graph(wide):
        """Every native module reachable from the wideband buffer: [index, description,
        reads-from index (-1: wideband)]."""
        seen, order, edges = {}, [], []
        frontier = [(wide, -1)]
        while frontier:
            buf, src = frontier.pop(0)
            for r in list(buf._readers):
                m = r.module
                if r._stopped or r._detached:
                    continue
                if m is None:  # a Python module's reader (csdr.module, e.g. a decoder)
                    order.append(None)
                    edges.append(src)
                    continue
                if id(m) in seen:
                    continue
                seen[id(m)] = len(order)
                order.append(m)
                edges.append(src)
                if isinstance(m.writer, M.Buffer):
                    frontier.append((m.writer, seen[id(m)]))
        return [[i, describe(m) if m is not None else {"class": "PythonReader"}, edges[i]]
                for i, m in enumerate(order)]

    fs = 10000000
    steps = []

    def record(name, chain, wide):
        seg = _graph.plan_segment(chain.selector.workers[0] if hasattr(chain, "selector")
                                  else chain.workers[0].workers[0])
        entry = {"step": name, "fused": seg is not None}
        if seg is not None:
            kind, p, used = seg
            entry["kind"] = kind
            entry["params"] = {k: v for k, v in p.items()
                               if k not in ("power_writer", "secondary_modules", "secondary_writer",
                                            "tap_selector", "tap_audio")}
            entry["tap_selector"] = p.get("tap_selector") is not None
            entry["tap_audio"] = p.get("tap_audio") is not None
            entry["n_modules"] = len(used)
        entry["graph"] = graph(wide)
        steps.append(entry)

    wide = Buffer(Format.COMPLEX_FLOAT)
    chain = ClientDemodulatorChain(NFm(12000), fs, 12000, 48000, "adpcm", False, 0, False, Events())
    chain.setReader(wide.getReader())
    chain.setWriter(Buffer(Format.CHAR))
    chain.setPowerWriter(Buffer(Format.FLOAT))
    chain.setSecondaryFftWriter(Buffer(Format.CHAR))
    chain.setSecondaryWriter(Buffer(Format.CHAR))
    chain.setFrequencyOffset(-200000)
    chain.setBandpass(-5999, 5999)
    record("nfm", chain, wide)
    chain.setDemodulator(Am())
    chain.setBandpass(-4700, 4700)
    record("am", chain, wide)
    chain.setDemodulator(Ssb(AgcProfile("Fast")))
    chain.setBandpass(150, 3000)
    record("usb", chain, wide)
    chain.setDemodulator(WFm(48000, 50e-6, False))
    chain.setBandpass(-124000, 124000)
    record("wfm", chain, wide)
    chain.setDemodulator(NFm(12000))
    chain.setBandpass(-5999, 5999)
    record("nfm_again", chain, wide)
    chain.setSecondaryDemodulator(SelectorSecondary())
    chain.setSecondaryFrequencyOffset(1000)
    record("nfm_secondary_selector", chain, wide)
    chain.setSecondaryFftSize(4096)
    record("nfm_secondary_fft_4096", chain, wide)
    chain.setNrEnabled(True)
    chain.setNrThreshold(5)
    record("nfm_nr", chain, wide)
    chain.setSecondaryDemodulator(AudioSecondary())
    record("nfm_audio_secondary", chain, wide)
    chain.setSecondaryDemodulator(None)
    chain.setNrEnabled(False)
    record("nfm_plain", chain, wide)
    # synchronous AM: Afc -> RealPart -> DcBlock -> Agc (csdr/chain/analog.py:141-154); the
    # Selector stays fused (its output feeds the standalone Afc)
    chain.setDemodulator(SAm())
    chain.setBandpass(-4700, 4700)
    record("sam", chain, wide)
    # raw synchronous AM, HD audio (csdr/chain/analog.py:156-167): the Selector runs at the
    # client's hd rate (48 kHz here, owrx/dsp.py:150-166) into Afc(50, 8) -> RealPart ->
    # DcBlock -> Gain(100)
    chain.setDemodulator(RawSAm(48000))
    record("rawsam", chain, wide)
    # raw AM, HD audio (csdr/chain/analog.py:23-31): AmDemod -> DcBlock -> Gain(100), no Agc
    chain.setDemodulator(RawAm(48000))
    record("rawam", chain, wide)
    # SsbDigital (FixedAudioRateChain + HdAudio, csdr/chain/analog.py:169-181): RealPart ->
    # Agc(Slow) with the Selector at its fixed 48 kHz audio rate
    chain.setDemodulator(SsbDigital(48000))
    chain.setBandpass(150, 3000)
    record("ssbdigital", chain, wide)
    _graph.finish(wide)

    # background services (owrx/service/__init__.py): ServiceDemodulatorChain on a service
    # Resampler's buffer -- any COMPLEX_FLOAT source; offset / bandpass as a USB-family decoder
    for name, sec in (("service_iq", IqService()), ("service_audio", AudioService())):
        src = Buffer(Format.COMPLEX_FLOAT)
        svc = ServiceDemodulatorChain(Ssb(), sec, 250000, 31000)
        svc.setBandPass(0, 3000)
        svc.setReader(src.getReader())
        record(name, svc, src)
        _graph.finish(src)
    print(json.dumps(steps))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
