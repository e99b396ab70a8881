#!/usr/bin/env python3
"""Regenerates the golden fixtures in tests/golden/ from the reference tree.

Runs ONLY in the build container (needs /root/reference and node); the GPU box and the
test-suite only read the committed JSON outputs.  Nothing from the reference is copied:

* chain_params.json -- the csdr module constructor/setter calls that the reference's own
  chain code (csdr/chain/fft.py, selector.py, analog.py, clientaudio.py) makes for the
  BASELINE.json configs, recorded by importing it with a recording stub ``pycsdr``
  (SURVEY.md section 8c item 1).
* js_adpcm.json -- the browser IMA-ADPCM decoder (htdocs/lib/AudioEngine.js:410-509),
  executed under node, on random nibble streams and on sync-framed streams produced by the
  oracle encoder (oracle/liboracle.so).
* js_firdes.json -- the browser port of csdr firdes_lowpass_f
  (htdocs/lib/AudioEngine.js:540-565) evaluated at the tap counts / cutoffs the chains use.

Usage: python3 tests/golden/make_golden.py
"""
import ctypes
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

STUB_TYPES = '''
from enum import Enum
class Format(Enum):
    CHAR = "CHAR"; SHORT = "SHORT"; FLOAT = "FLOAT"; COMPLEX_FLOAT = "COMPLEX_FLOAT"
    COMPLEX_SHORT = "COMPLEX_SHORT"; COMPLEX_CHAR = "COMPLEX_CHAR"
class AgcProfile(Enum):
    FAST = "Fast"; SLOW = "Slow"; MID = "Mid"; LAGGY = "Laggy"
'''

STUB_MODULES = '''
import sys
LOG = []
WIRING = {"setReader", "setWriter", "getReader", "getOutputFormat", "getInputFormat",
          "stop", "getFormat"}
class Module:
    def __init__(self, *a, **k):
        pass
class _Rec:
    def __init__(self, *args, **kwargs):
        LOG.append(["new", type(self).__name__, id(self), args, kwargs])
    def __getattr__(self, name):
        if name.startswith("_"):
            raise AttributeError(name)
        def f(*a, **k):
            if name not in WIRING:
                LOG.append(["call", type(self).__name__, id(self), name, a, k])
            if name == "getReader":
                return _Rec.__new__(_Rec)
            return None
        return f
def __getattr__(name):
    cls = type(name, (_Rec,), {})
    setattr(sys.modules[__name__], name, cls)
    return cls
'''

PROBE = r'''
import json, sys
from enum import Enum
import csdr.chain.fft as fft
import csdr.chain.selector as selector
import csdr.chain.analog as analog
import csdr.chain.clientaudio as clientaudio
import pycsdr.modules as M
from pycsdr.types import Format, AgcProfile

IGNORED = {"Buffer", "_Rec"}

def enc(v):
    if isinstance(v, Enum):
        return v.name
    if isinstance(v, float):
        return repr(v)
    if isinstance(v, (list, tuple)):
        return [enc(x) for x in v]
    if isinstance(v, dict):
        return {k: enc(x) for k, x in v.items()}
    return v

def take():
    ids = {}
    out = []
    for e in M.LOG:
        if e[1] in IGNORED:
            continue
        oid = ids.setdefault(e[2], len(ids))
        if e[0] == "new":
            out.append({"op": "new", "module": e[1], "obj": oid, "args": enc(e[3]), "kwargs": enc(e[4])})
        else:
            out.append({"op": "call", "module": e[1], "obj": oid, "method": e[3], "args": enc(e[4]), "kwargs": enc(e[5])})
    M.LOG.clear()
    return out

res = {}
for name, (sr, size, ovl, fps, comp) in {
    "fft_c1": (2400000, 4096, 0.3, 9, "adpcm"),
    "fft_c2": (10000000, 16384, 0.3, 9, "adpcm"),
    "fft_c4": (61440000, 65536, 0.3, 9, "adpcm"),
    "fft_nooverlap_none": (10000000, 2048, 0.0, 9, "none"),
    "fft_secondary": (12000, 2048, 0.3, 9, "adpcm"),
}.items():
    c = fft.FftChain(sr, size, ovl, fps, comp)
    res[name] = {"ctor": [sr, size, ovl, fps, comp], "calls": take()}
    c.setFps(25)
    res[name]["setFps25"] = take()
    c.setVOverlapFactor(0.5)
    res[name]["setVOverlap05"] = take()

modes = {"nfm": (-5999, 5999), "am": (-4700, 4700), "usb": (150, 3000),
         "lsb": (-3000, -150), "cw": (700, 900)}
for sr in (2400000, 10000000, 61440000):
    s = selector.Selector(sr, 12000)
    entry = {"ctor": [sr, 12000], "calls": take()}
    s.setFrequencyOffset(100000)
    entry["offset100k"] = take()
    s.setFrequencyOffset(-1234567 if sr > 2400000 else -345678)
    entry["offset_neg"] = take()
    for m, (lo, hi) in modes.items():
        s.setBandpass(lo, hi)
        entry["bandpass_" + m] = take()
    s.setSquelchLevel(-150)
    entry["squelch_m150"] = take()
    s.setSquelchLevel(-80)
    entry["squelch_m80"] = take()
    res["selector_%d" % sr] = entry

# WFM: Selector(sr, 250000) (FixedIfSampleRateChain, csdr/chain/analog.py:81-82) with the
# mode's bandpass (owrx/modes.py:125) and WFm(hd_output_rate=48000, tau=50e-6)
for sr in (2400000, 10000000, 61440000):
    s = selector.Selector(sr, 250000)
    entry = {"ctor": [sr, 250000], "calls": take()}
    s.setFrequencyOffset(-600000 if sr > 2400000 else 300000)
    entry["offset"] = take()
    s.setBandpass(-124000, 124000)
    entry["bandpass_wfm"] = take()
    s.setSquelchLevel(-150)
    entry["squelch_m150"] = take()
    res["selector_wfm_%d" % sr] = entry
analog.WFm(48000, 50e-6, False)
res["wfm"] = take()
clientaudio.ClientAudioChain(Format.FLOAT, 48000, 48000, "adpcm", False, 0)
res["clientaudio_hd_adpcm"] = take()
analog.NFm(12000)
res["nfm"] = take()
analog.Am()
res["am"] = take()
analog.Ssb(AgcProfile.FAST)
res["ssb_fast"] = take()
analog.Ssb(AgcProfile("Slow"))
res["ssb_slow"] = take()
clientaudio.ClientAudioChain(Format.FLOAT, 12000, 12000, "adpcm", False, 0)
res["clientaudio_adpcm"] = take()
clientaudio.ClientAudioChain(Format.FLOAT, 12000, 12000, "none", False, 0)
res["clientaudio_none"] = take()
clientaudio.ClientAudioChain(Format.FLOAT, 12000, 12000, "adpcm", True, 10)
res["clientaudio_nr"] = take()
json.dump(res, sys.stdout, indent=1, sort_keys=True)
'''

JS = r'''
const fs = require("fs");
const vm = require("vm");
const ctx = {console: console, Math: Math, Float32Array, Int16Array, Uint8Array};
vm.createContext(ctx);
vm.runInContext(fs.readFileSync(process.argv[2], "utf8"), ctx);
const job = JSON.parse(fs.readFileSync(process.argv[3], "utf8"));
const out = {adpcm_plain: [], adpcm_sync: [], firdes: []};
for (const s of job.plain) {
  const c = new ctx.ImaAdpcmCodec();
  out.adpcm_plain.push({bytes: s, decoded: Array.from(c.decode(new Uint8Array(s)))});
}
for (const s of job.sync) {
  const c = new ctx.ImaAdpcmCodec();
  // deliver in uneven pieces like WebSocket frames would
  let dec = [];
  const cuts = [0, 3, 517, 1009, 2222, s.bytes.length];
  for (let i = 0; i + 1 < cuts.length; i++) {
    const a = Math.min(cuts[i], s.bytes.length), b = Math.min(cuts[i + 1], s.bytes.length);
    dec = dec.concat(Array.from(c.decodeWithSync(new Uint8Array(s.bytes.slice(a, b)))));
  }
  out.adpcm_sync.push({name: s.name, bytes: s.bytes, decoded: dec});
}
for (const f of job.firdes) {
  const lp = Object.create(ctx.Lowpass.prototype);
  lp.numtaps = f.ntaps;
  out.firdes.push({ntaps: f.ntaps, cutoff: f.cutoff, taps: lp.getCoefficients(f.cutoff)});
}
fs.writeFileSync(process.argv[4], JSON.stringify(out));
'''


def probe_chain_params():
    with tempfile.TemporaryDirectory() as d:
        os.makedirs(os.path.join(d, "pycsdr"))
        with open(os.path.join(d, "pycsdr", "__init__.py"), "w") as f:
            f.write('version = "0.18.99"\n')
        with open(os.path.join(d, "pycsdr", "types.py"), "w") as f:
            f.write(STUB_TYPES)
        with open(os.path.join(d, "pycsdr", "modules.py"), "w") as f:
            f.write(STUB_MODULES)
        env = dict(os.environ, PYTHONPATH=d + ":" + REF)
        out = subprocess.run([sys.executable, "-c", PROBE], env=env, check=True,
                             capture_output=True, text=True, cwd=d)
        return json.loads(out.stdout)


def oracle():
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "liboracle.so"))
    lib.orc_adpcm_encode.restype = ctypes.c_int64
    lib.orc_adpcm_encode.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_void_p]
    return lib


def adpcm_sync_streams(lib):
    rng = np.random.Generator(np.random.PCG64(20251114))
    t = np.arange(6000)
    sigs = {
        "tone": (8000 * np.sin(2 * np.pi * 1000 * t / 12000)).astype(np.int16),
        "noise": rng.integers(-3000, 3000, size=6000).astype(np.int16),
        "steps": np.repeat(rng.integers(-30000, 30000, size=60), 100).astype(np.int16),
    }
    streams = []
    for name, s in sigs.items():
        out = np.zeros(len(s), dtype=np.uint8)
        nb = lib.orc_adpcm_encode(s.ctypes.data, len(s), 1, out.ctypes.data)
        streams.append({"name": name, "input": s.tolist(), "bytes": out[:nb].tolist()})
    return streams


def main():
    params = probe_chain_params()
    with open(os.path.join(HERE, "chain_params.json"), "w") as f:
        json.dump(params, f, indent=1, sort_keys=True)

    lib = oracle()
    rng = np.random.Generator(np.random.PCG64(7))
    plain = [rng.integers(0, 256, size=n).tolist() for n in (1, 64, 4096)]
    sync = adpcm_sync_streams(lib)
    # tap counts and cutoffs: FirDecimate lowpass is cutoff/D in float
    # (csdr/chain/selector.py:22-29), Bandpass lowpass is (hi-lo)/2 (selector.py:159-166).
    f32 = lambda x: float(np.float32(x))
    firdes = [
        {"ntaps": 5333, "cutoff": f32(np.float32(0.5) / np.float32(200))},
        {"ntaps": 22223, "cutoff": f32(np.float32(0.5 * 833 / (10e6 / 12000)) / np.float32(833))},
        {"ntaps": 149, "cutoff": f32((np.float32(5999 / 12000) - np.float32(-5999 / 12000)) / 2)},
        {"ntaps": 149, "cutoff": f32((np.float32(3000 / 12000) - np.float32(150 / 12000)) / 2)},
        {"ntaps": 101, "cutoff": 0.1},
    ]
    job = {"plain": plain, "sync": [{"name": s["name"], "bytes": s["bytes"]} for s in sync],
           "firdes": firdes}
    with tempfile.TemporaryDirectory() as d:
        jp, js, op = (os.path.join(d, x) for x in ("job.json", "gen.js", "out.json"))
        with open(jp, "w") as f:
            json.dump(job, f)
        with open(js, "w") as f:
            f.write(JS)
        subprocess.run(["node", js, os.path.join(REF, "htdocs/lib/AudioEngine.js"), jp, op],
                       check=True)
        with open(op) as f:
            res = json.load(f)
    for s, r in zip(sync, res["adpcm_sync"]):
        r["input"] = s["input"]
    with open(os.path.join(HERE, "js_adpcm.json"), "w") as f:
        json.dump({"plain": res["adpcm_plain"], "sync": res["adpcm_sync"]}, f)
    with open(os.path.join(HERE, "js_firdes.json"), "w") as f:
        json.dump(res["firdes"], f)
    print("wrote chain_params.json, js_adpcm.json, js_firdes.json")


if __name__ == "__main__":
    main()
